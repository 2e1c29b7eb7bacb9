from .base import *  # noqa: F401,F403
from .conv import *  # noqa: F401,F403
from .diff import *  # noqa: F401,F403
from .sampling import *  # noqa: F401,F403

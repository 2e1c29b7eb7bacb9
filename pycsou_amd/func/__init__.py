from .base import *  # noqa: F401,F403
from .penalty import *  # noqa: F401,F403
from .loss import *  # noqa: F401,F403

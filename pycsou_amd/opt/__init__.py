from .proxalgs import *  # noqa: F401,F403

"""Proximal utilities (``pycsou/math/prox.py`` hot-path subset) on device arrays.

Accept NumPy or torch inputs and return the same kind.  Unlike the reference, the
projections do not modify their argument in place (``prox.py:253-256, 295-297,
340-343`` write into ``x``); the solvers only ever pass temporaries there, so results
are identical.
"""

import torch

from .. import _ops as O


def sign(x):
    """``prox.py:17-64`` (real inputs)."""
    t = O.to_dev(x)
    return O.like(torch.sign(t), x)


def soft(x, tau):
    """``prox.py:67-114``: ``clip(|x| - tau, 0) * sign(x)``."""
    t = O.to_dev(x)
    out = torch.clamp(t.abs() - tau, min=0) * torch.sign(t)
    return O.like(out, x)


def proj_l2_ball(x, radius):
    """``prox.py:167-210``."""
    t = O.to_dev(x)
    return O.like(O.axpby(t, O.prox_l2(t, radius), 1.0, -1.0), x)


def proj_linfty_ball(x, radius):
    """``prox.py:213-256``."""
    t = O.to_dev(x)
    return O.like(O.proj_segment(t, -radius, radius), x)


def proj_nonnegative_orthant(x):
    """``prox.py:259-297``."""
    t = O.to_dev(x)
    return O.like(O.proj_nonneg(t), x)


def proj_segment(x, a=0, b=1):
    """``prox.py:300-343``."""
    t = O.to_dev(x)
    return O.like(O.proj_segment(t, a, b), x)

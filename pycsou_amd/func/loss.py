"""Losses (``pycsou/func/loss.py`` hot-path subset).

``SquaredL2Loss(dim, data) = SquaredL2Norm(dim).shifter(-data)`` (``loss.py:165-219``,
through ``DifferentiableLoss``, ``loss.py:72-120``); ``(1/2) * SquaredL2Loss(...) * Op``
therefore has ``gradient(x) = Op^T((2*(Op x - y))*0.5)`` and ``diff_lipschitz_cst =
||Op||^2``, exactly as in the reference.
"""

import numpy as np
import torch

from ..core.functional import ProxFuncPreComp
from .penalty import L1Norm, L2Norm, SquaredL2Norm


def _neg(data):
    if isinstance(data, torch.Tensor):
        return -data
    return -np.asarray(data)


def ProximableLoss(func, data):
    """``loss.py:20-69``."""
    return ProxFuncPreComp(func, scale=1, shift=_neg(data))


def DifferentiableLoss(func, data):
    """``loss.py:72-120``."""
    return func.shifter(shift=_neg(data))


def L2Loss(dim, data):
    """``loss.py:123-162``."""
    return ProximableLoss(L2Norm(dim=dim), data=data)


def SquaredL2Loss(dim, data):
    """``loss.py:165-219``."""
    return DifferentiableLoss(SquaredL2Norm(dim=dim), data=data)


def L1Loss(dim, data):
    """``loss.py:222-268``."""
    return ProximableLoss(L1Norm(dim=dim), data=data)

"""Base functionals (``pycsou/func/base.py`` hot-path subset).

``IndicatorFunctional`` (``base.py:140-168``), ``NullDifferentiableFunctional`` /
``NullProximableFunctional`` (``base.py:171-212``, the PDS defaults for missing F / G)
and ``LpNorm`` (``base.py:215-240``: prox through the Moreau identity with a dual-ball
projection).  Stacked functionals (``ProxFuncHStack``/``DiffFuncHStack``) are out of scope.
"""

import numpy as np
import torch

from .. import _ops as O
from ..core.functional import DifferentiableFunctional, ProximableFunctional


class IndicatorFunctional(ProximableFunctional):
    """Indicator of a convex set; ``prox`` is the projection (``base.py:140-168``).

    ``projection_func`` / ``condition_func`` receive and return flat device tensors.
    """

    def __init__(self, dim, condition_func, projection_func, kind=None, params=()):
        super().__init__(dim=dim, data=None, is_differentiable=False, is_linear=False)
        self.condition_func = condition_func
        self.projection_func = projection_func
        self.kind = kind          # fused-engine tag: 'nonneg' / 'segment' / None
        self.params = params

    def _apply(self, t):
        return 0 if self.condition_func(t) else np.inf

    def _prox(self, t, tau, **kwargs):
        return self.projection_func(t, **kwargs)


class NullDifferentiableFunctional(DifferentiableFunctional):
    """``base.py:171-191``."""

    def __init__(self, dim):
        super().__init__(dim=dim, is_linear=True, lipschitz_cst=0, diff_lipschitz_cst=0)

    def _apply(self, t):
        return 0

    def _jacT(self, t):
        return torch.zeros(self.dim, dtype=t.dtype if isinstance(t, torch.Tensor) else torch.float64,
                           device=O.device())


class NullProximableFunctional(ProximableFunctional):
    """``base.py:194-212``: ``prox`` is the identity."""

    def __init__(self, dim):
        super().__init__(dim=dim, is_linear=True)

    def _apply(self, t):
        return 0

    def _prox(self, t, tau):
        return t


class LpNorm(ProximableFunctional):
    """``x - tau * proj_{q-ball}(x / tau, 1)`` (``base.py:215-240``); subclasses supply the
    fused kernel as ``_prox``."""

    def __init__(self, dim, proj_lq_ball=None):
        super().__init__(dim=dim, data=None, is_differentiable=False, is_linear=False)
        self.proj_lq_ball = proj_lq_ball

"""Base functionals (``pycsou/func/base.py`` hot-path subset).

``IndicatorFunctional`` (``base.py:140-168``), ``NullDifferentiableFunctional`` /
``NullProximableFunctional`` (``base.py:171-212``, the PDS defaults for missing F / G)
and ``LpNorm`` (``base.py:215-240``: prox through the Moreau identity with a dual-ball
projection), the horizontal stacks ``ProxFuncHStack`` / ``DiffFuncHStack`` (``base.py:21-137``;
notebook cell [62]: ``H = ProxFuncHStack(L1Loss(dim, data=y), mu * L1Norm(dim))``) and
``ExplicitLinearFunctional`` (``base.py:308-326``).
"""

import numpy as np
import torch

from .. import _ops as O
from ..core.functional import DifferentiableFunctional, LinearFunctional, ProximableFunctional
from ..core.map import DiffMapHStack, MapHStack, _cat


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


class ProxFuncHStack(ProximableFunctional, MapHStack):
    """``h(x_1, ..., x_k) = sum_i f_i(x_i)`` with the separable prox
    ``prox_{tau h}(x) = (prox_{tau f_1}(x_1), ..., prox_{tau f_k}(x_k))`` (``base.py:21-89``).
    ``fenchel_prox`` is the generic Moreau identity over the whole stack, as in the reference
    (``core/functional.py:176-207``)."""

    def __init__(self, *proxfuncs, n_jobs=1, joblib_backend='loky'):
        MapHStack.__init__(self, *proxfuncs, n_jobs=n_jobs, joblib_backend=joblib_backend)
        self.proxfuncs = self.maps
        ProximableFunctional.__init__(self, dim=self.shape[1], data=None, is_differentiable=self.is_differentiable,
                                      is_linear=self.is_linear)

    def _prox(self, t, tau):
        return _cat([f._prox(xi, tau) for f, xi in zip(self.proxfuncs, self._split(t))], t)


class DiffFuncHStack(DifferentiableFunctional, DiffMapHStack):
    """``h(x_1, ..., x_k) = sum_i f_i(x_i)`` with gradient ``(grad f_1(x_1), ..., grad f_k(x_k))``
    (``base.py:92-137``)."""

    def __init__(self, *difffuncs, n_jobs=1, joblib_backend='loky'):
        DiffMapHStack.__init__(self, *difffuncs, n_jobs=n_jobs, joblib_backend=joblib_backend)
        self.difffuncs = self.maps
        DifferentiableFunctional.__init__(self, dim=self.shape[1], data=None, is_linear=self.is_linear,
                                          lipschitz_cst=self.lipschitz_cst, diff_lipschitz_cst=self.diff_lipschitz_cst)

    def _jacT(self, t):
        return _cat([f._jacT(xi) for f, xi in zip(self.difffuncs, self._split(t))], t)


class ExplicitLinearFunctional(LinearFunctional):
    """``x -> <vec, x>`` (``base.py:308-326``); ``adjoint(y) = y * vec``."""

    def __init__(self, vec, dtype=np.float64):
        if isinstance(vec, torch.Tensor):
            self._vec_dev = vec.reshape(-1)
            dtype = np.float32 if vec.dtype == torch.float32 else np.float64
            self.vec = vec.reshape(-1)
        else:
            self.vec = np.asarray(vec).flatten().astype(dtype)
            self._vec_dev = None
        super().__init__(dim=int(self.vec.numel() if isinstance(self.vec, torch.Tensor) else self.vec.size),
                         dtype=dtype, is_explicit=True)

    def _v(self, like):
        if self._vec_dev is None or self._vec_dev.dtype != like.dtype:
            self._vec_dev = O.to_dev(self.vec if not isinstance(self.vec, torch.Tensor) else self.vec, like.dtype)
        return self._vec_dev

    def _apply(self, t):
        return torch.dot(self._v(t), t.reshape(-1)).reshape(1)

    def _adj(self, t):
        return O.scale(self._v(t), float(t.reshape(-1)[0].item()) if isinstance(t, torch.Tensor) else float(t))

"""Functionals and proximal calculus (mirrors ``pycsou/core/functional.py``).

* ``ProximableFunctional.prox(x, tau)`` and the Moreau identity
  ``fenchel_prox(z, sigma) = z - sigma * prox(z / sigma, 1 / sigma)`` (``functional.py:176-207``).
* ``lam * f`` (``lam > 0``) -> ``ProxFuncPostComp``: ``prox(x, tau) = f.prox(x, tau*lam)``
  (``functional.py:244-265``); ``f * a`` / ``f.shifter(s)`` -> ``ProxFuncPreComp``
  (``functional.py:286-299``).

Concrete functionals provide the device-level ``_prox(t, tau)``; the ones on the PDS hot
path (L1, L21) also provide ``_fenchel_scaled(w, sigma, lam)``, a single fused kernel for
``(lam*f).fenchel_prox`` that keeps the reference's operation order.
"""

from numbers import Number
import warnings

import numpy as np
import torch

from .. import _ops as O
from .linop import LinearOperator, UnitaryOperator
from .map import DifferentiableMap, Map, MapComp, MapSum


class Functional(Map):
    """``functional.py:20-45``."""

    def __init__(self, dim, data=None, is_differentiable=False, is_linear=False):
        Map.__init__(self, shape=(1, dim), is_differentiable=is_differentiable, is_linear=is_linear)
        self.data = data
        self.dim = dim


class DifferentiableFunctional(Functional, DifferentiableMap):
    """``functional.py:48-75``."""

    def __init__(self, dim, data=None, is_linear=False, lipschitz_cst=np.inf, diff_lipschitz_cst=np.inf):
        Functional.__init__(self, dim=dim, data=data, is_differentiable=True, is_linear=is_linear)
        DifferentiableMap.__init__(self, shape=self.shape, is_linear=self.is_linear, lipschitz_cst=lipschitz_cst,
                                   diff_lipschitz_cst=diff_lipschitz_cst)


class LinearFunctional(Functional, LinearOperator):
    """``functional.py:78-87``."""

    def __init__(self, dim, data=None, dtype=np.float64, is_explicit=False, is_dense=False, is_sparse=False,
                 is_dask=False):
        Functional.__init__(self, dim=dim, data=data, is_differentiable=True, is_linear=True)
        LinearOperator.__init__(self, shape=self.shape, dtype=dtype, is_explicit=is_explicit, is_dense=is_dense,
                                is_sparse=is_sparse, is_dask=is_dask, is_symmetric=False)


class ProximableFunctional(Functional):
    """Functional with a simple proximal operator (``functional.py:90-250``)."""

    def __init__(self, dim, data=None, is_differentiable=False, is_linear=False):
        if is_differentiable or is_linear:
            warnings.warn('For differentiable and/or linear maps, consider the dedicated classes DifferentiableMap '
                          'and LinearOperator.')
        super().__init__(dim=dim, data=data, is_differentiable=is_differentiable, is_linear=is_linear)

    # -- device layer
    def _prox(self, t, tau):
        raise NotImplementedError

    def _fenchel(self, w, sigma):
        # z - sigma * prox(z / sigma, 1 / sigma)
        v = O.scale(w, 1.0 / sigma)
        return O.axpby(w, self._prox(v, 1.0 / sigma), 1.0, -sigma)

    # -- public layer
    def prox(self, x, tau):
        return O.like(self._prox(O.to_dev(x), tau), x)

    def fenchel_prox(self, z, sigma):
        return O.like(self._fenchel(O.to_dev(z), sigma), z)

    def shifter(self, shift):
        return ProxFuncPreComp(prox_func=self, scale=1, shift=shift)

    def __add__(self, other):
        if isinstance(other, LinearFunctional):
            return ProxFuncAffineSum(self, linear_part=other, intercept=0)
        if isinstance(other, Map):
            return MapSum(self, other)
        raise NotImplementedError

    def __mul__(self, other):
        if isinstance(other, Number) or O.is_array(other):
            return ProxFuncPreComp(self, scale=other, shift=0)
        if isinstance(other, UnitaryOperator):
            return ProxFuncPreCompUnitOp(self, other)
        if isinstance(other, Map):
            return MapComp(self, other)
        raise NotImplementedError

    def __rmul__(self, other):
        if isinstance(other, Number) and other > 0:
            return ProxFuncPostComp(self, scale=other, shift=0)
        if isinstance(other, Map):
            return MapComp(other, self)
        raise NotImplementedError


class ProxFuncPostComp(ProximableFunctional):
    """``scale * f + shift`` (``functional.py:253-265``)."""

    def __init__(self, prox_func, scale, shift):
        super().__init__(dim=prox_func.dim, data=prox_func.data, is_differentiable=prox_func.is_differentiable)
        self.prox_func = prox_func
        self.scale = scale
        self.shift = shift

    def _apply(self, t):
        return self.scale * self.prox_func._apply(t) + self.shift

    def _prox(self, t, tau):
        return self.prox_func._prox(t, tau * self.scale)

    def _fenchel(self, w, sigma):
        fused = getattr(self.prox_func, '_fenchel_scaled', None)
        if fused is not None:
            return fused(w, sigma, self.scale)
        return ProximableFunctional._fenchel(self, w, sigma)


class ProxFuncAffineSum(ProximableFunctional):
    """``f + <a, .> + b`` (``functional.py:268-283``)."""

    def __init__(self, prox_func, linear_part, intercept):
        if not isinstance(linear_part, LinearFunctional) or linear_part.dim != prox_func.dim:
            raise TypeError('Invalid affine sum.')
        super().__init__(dim=prox_func.dim, data=prox_func.data, is_differentiable=prox_func.is_differentiable)
        self.prox_func, self.linear_part, self.intercept = prox_func, linear_part, intercept

    def _apply(self, t):
        return self.prox_func._apply(t) + self.linear_part._apply(t) + self.intercept

    def _prox(self, t, tau):
        a = self.linear_part._adj(torch.ones(1, dtype=t.dtype, device=t.device))
        return self.prox_func._prox(O.axpby(t, a, 1.0, -tau), tau)


class ProxFuncPreComp(ProximableFunctional):
    """``f(scale * x + shift)`` (``functional.py:286-299``)."""

    def __init__(self, prox_func, scale, shift):
        super().__init__(dim=prox_func.dim, data=prox_func.data, is_differentiable=prox_func.is_differentiable)
        self.prox_func, self.scale, self.shift = prox_func, scale, shift
        self._cache = {}

    def _affine(self, t, a, b):
        """a * t + b with scalar or array a, b."""
        key = (t.dtype, id(a), id(b))
        ab = self._cache.get(key)
        if ab is None:
            ab = tuple(v if isinstance(v, Number) else O.to_dev(v, t.dtype) for v in (a, b))
            self._cache[key] = ab
        a_, b_ = ab
        out = O.scale(t, a_) if isinstance(a_, Number) else t * a_
        if isinstance(b_, Number):
            return out if b_ == 0 else out + b_
        return O.add(out, b_)

    def _apply(self, t):
        return self.prox_func._apply(self._affine(t, self.scale, self.shift))

    def _prox(self, t, tau):
        s = self.scale
        s2 = s ** 2 if isinstance(s, Number) else None
        inner = self.prox_func._prox(self._affine(t, s, self.shift), tau * (s2 if s2 is not None else 1.0))
        if isinstance(self.shift, Number):
            num = inner if self.shift == 0 else inner - self.shift
        else:
            num = O.axpby(inner, O.to_dev(self.shift, t.dtype), 1.0, -1.0)
        return O.scale(num, 1.0 / s) if isinstance(s, Number) else num / O.to_dev(s, t.dtype)


class ProxFuncPreCompUnitOp(ProximableFunctional):
    """``f(U x)`` for unitary ``U`` (``functional.py:302-313``)."""

    def __init__(self, prox_func, unitary_op):
        super().__init__(dim=prox_func.dim, data=prox_func.data, is_differentiable=prox_func.is_differentiable)
        self.prox_func, self.unitary_op = prox_func, unitary_op

    def _apply(self, t):
        return self.prox_func._apply(self.unitary_op._apply(t))

    def _prox(self, t, tau):
        return self.unitary_op._adj(self.prox_func._prox(self.unitary_op._apply(t), tau))

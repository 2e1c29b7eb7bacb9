"""Basic linear operators (mirrors the hot-path part of ``pycsou/linop/base.py``).

``DiagonalOperator`` / ``IdentityOperator`` / ``NullOperator`` / ``HomothetyMap``
(``base.py:551-633``) are the defaults PDS inserts for missing K / F terms and the
scalar factors of the algebra; ``DenseLinearOperator`` (``base.py:102-118``) backs the
LASSO problem (C1).  Stacks, sparse / Dask / polynomial / Kronecker operators are out of
scope for this build.
"""

from numbers import Number

import numpy as np
import torch

from .. import _ops as O
from ..core.linop import LinearOperator


class ExplicitLinearOperator(LinearOperator):
    """Operator given by an explicit dense matrix, held in HBM (``base.py:57-99``)."""

    def __init__(self, array, is_symmetric=False):
        if isinstance(array, torch.Tensor):
            dt = np.float32 if array.dtype == torch.float32 else np.float64
        elif isinstance(array, np.ndarray):
            dt = array.dtype
        else:
            raise TypeError('Invalid input type.')
        super().__init__(shape=tuple(array.shape), dtype=dt, is_explicit=True, is_dask=False, is_dense=True,
                         is_sparse=False, is_symmetric=is_symmetric)
        self.mat = array
        self._dev = {}

    def _m(self, dtype):
        m = self._dev.get(dtype)
        if m is None:
            m = torch.as_tensor(np.asarray(self.mat) if not isinstance(self.mat, torch.Tensor) else self.mat)
            m = m.to(device=O.device(), dtype=dtype).contiguous()
            self._dev[dtype] = m
        return m

    def _apply(self, t):
        return torch.mv(self._m(t.dtype), t)

    def _adj(self, t):
        return torch.mv(self._m(t.dtype).T, t)


class DenseLinearOperator(ExplicitLinearOperator):
    """``base.py:102-118``."""

    def __init__(self, ndarray, is_symmetric=False):
        super().__init__(array=ndarray, is_symmetric=is_symmetric)


class DiagonalOperator(LinearOperator):
    """``base.py:551-579``."""

    def __init__(self, diag):
        self.diag = np.asarray(diag).reshape(-1)
        super().__init__(shape=(self.diag.size, self.diag.size), dtype=self.diag.dtype, is_explicit=False,
                         is_dense=False, is_sparse=False, is_dask=False,
                         is_symmetric=bool(np.all(np.isreal(self.diag))))
        self.lipschitz_cst = self.diff_lipschitz_cst = np.max(diag)
        self._dev = {}

    def _d(self, dtype):
        d = self._dev.get(dtype)
        if d is None:
            d = torch.as_tensor(self.diag).to(device=O.device(), dtype=dtype)
            self._dev[dtype] = d
        return d

    def _apply(self, t):
        if isinstance(t, Number):
            return float(self.diag[0]) * t
        if self.diag.size == 1:
            return O.scale(t, float(self.diag[0]))
        return t * self._d(t.dtype)

    def _adj(self, t):
        return self._apply(t)

    def __call__(self, x):
        if self.shape[1] == 1 and not O.is_array(x):
            return float(self.diag[0]) * x
        return LinearOperator.__call__(self, x)


class IdentityOperator(DiagonalOperator):
    """``base.py:582-598``."""

    def __init__(self, size, dtype=None):
        super().__init__(np.ones(shape=(size,), dtype=dtype))
        self.lipschitz_cst = self.diff_lipschitz_cst = 1

    def _apply(self, t):
        return t

    def _adj(self, t):
        return t


class NullOperator(LinearOperator):
    """``base.py:601-622``."""

    def __init__(self, shape, dtype=np.float64):
        super().__init__(shape=shape, dtype=dtype, is_explicit=False, is_dense=False, is_sparse=False,
                         is_dask=False, is_symmetric=shape[0] == shape[1])
        self.lipschitz_cst = self.diff_lipschitz_cst = 0

    def _apply(self, t):
        return torch.zeros(self.shape[0], dtype=t.dtype, device=t.device)

    def _adj(self, t):
        return torch.zeros(self.shape[1], dtype=t.dtype, device=t.device)

    def eigenvals(self, k, which='LM', **kwargs):
        return np.zeros(shape=(k,), dtype=self.dtype)

    def singularvals(self, k, which='LM', **kwargs):
        return np.zeros(shape=(k,), dtype=self.dtype)


class HomothetyMap(DiagonalOperator):
    """``x -> constant * x`` (``base.py:625-633``); ``jacobianT`` is the constant."""

    def __init__(self, size, constant):
        self.cst = constant
        super().__init__(diag=constant)
        self.shape = (size, size)
        self.lipschitz_cst = self.diff_lipschitz_cst = constant

    def _jacT(self, t=None):
        return self.cst

    def jacobianT(self, arg=None):
        return self.cst

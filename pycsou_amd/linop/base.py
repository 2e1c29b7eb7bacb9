"""Basic linear operators (mirrors the hot-path part of ``pycsou/linop/base.py``).

``DiagonalOperator`` / ``IdentityOperator`` / ``NullOperator`` / ``HomothetyMap``
(``base.py:551-633``) are the defaults PDS inserts for missing K / F terms and the
scalar factors of the algebra; ``DenseLinearOperator`` (``base.py:102-118``) backs the
LASSO problem (C1); ``LinOpStack`` / ``LinOpVStack`` / ``LinOpHStack`` (``base.py:159-302``)
build stacked K operators (notebook cell [62]: ``K = LinOpVStack(Gop, D)``);
``PolynomialLinearOperator`` (``base.py:636-700``) backs ``GeneralisedLaplacian``.
Sparse / Dask / Kronecker operators are out of scope for this build.
"""

from numbers import Number

import numpy as np
import torch

from .. import _ops as O
from ..core.linop import LinearOperator
from ..core.map import DiffMapStack


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
        return O.mul(t, self._d(t.dtype))

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


class LinOpStack(LinearOperator, DiffMapStack):
    """Vertical (``axis=0``) / horizontal (``axis=1``) stack of linear operators
    (``base.py:159-256``): ``V x = (L_1 x, ..., L_k x)``, ``V^* y = sum_i L_i^* y_i``;
    ``H (x_1, ..., x_k) = sum_i L_i x_i``, ``H^* y = (L_1^* y, ..., L_k^* y)``.  Sums are
    accumulated in block order (``result = 0; result += ...``) as the reference does."""

    def __init__(self, *linops, axis, n_jobs=1, joblib_backend='loky'):
        DiffMapStack.__init__(self, *linops, axis=axis, n_jobs=n_jobs, joblib_backend=joblib_backend)
        self.linops = self.maps
        self.is_explicit_list = [op.is_explicit for op in self.linops]
        self.is_dense_list = [op.is_dense for op in self.linops]
        self.is_sparse_list = [op.is_sparse for op in self.linops]
        self.is_dask_list = [op.is_dask for op in self.linops]
        self.is_symmetric_list = [op.is_symmetric for op in self.linops]
        LinearOperator.__init__(self, shape=self.shape, is_explicit=bool(np.prod(self.is_explicit_list).astype(bool)),
                                is_dense=bool(np.prod(self.is_dense_list).astype(bool)),
                                is_sparse=bool(np.prod(self.is_sparse_list).astype(bool)),
                                is_dask=bool(np.prod(self.is_dask_list).astype(bool)),
                                is_symmetric=bool(np.prod(self.is_symmetric_list).astype(bool)),
                                lipschitz_cst=self.lipschitz_cst)
        dts = {op.dtype for op in self.linops}
        self.dtype = dts.pop() if len(dts) == 1 else None

    def _adj(self, t):
        from ..core.map import _cat
        if self.axis == 0:
            o = _sections([op.shape[0] for op in self.linops])
            result = None
            for i, op in enumerate(self.linops):
                r = op._adj(t[o[i]:o[i + 1]])
                result = r if result is None else O.add(result, r)
            return result
        return _cat([op._adj(t) for op in self.linops], t)


def _sections(sizes):
    return [0] + [int(s) for s in np.cumsum(sizes)]


class LinOpVStack(LinOpStack):
    """``LinOpStack(*linops, axis=0)`` (``base.py:259-279``)."""

    def __init__(self, *linops, n_jobs=1, joblib_backend='loky'):
        super().__init__(*linops, axis=0, n_jobs=n_jobs, joblib_backend=joblib_backend)


class LinOpHStack(LinOpStack):
    """``LinOpStack(*linops, axis=1)`` (``base.py:282-302``)."""

    def __init__(self, *linops, n_jobs=1, joblib_backend='loky'):
        super().__init__(*linops, axis=1, n_jobs=n_jobs, joblib_backend=joblib_backend)


class PolynomialLinearOperator(LinearOperator):
    """``P(L) = a_0 I + a_1 L + ... + a_N L^N`` for a square ``L`` (``base.py:636-700``):
    ``y = a_0 x; z = x; y += a_i (z = L z)`` in the reference's order; the adjoint uses
    ``L^*`` (or ``P(L)`` itself when ``L`` is symmetric)."""

    def __init__(self, LinOp, coeffs):
        self.coeffs = np.asarray(coeffs).astype(LinOp.dtype if LinOp.dtype is not None else np.float64)
        if LinOp.shape[0] != LinOp.shape[1]:
            raise ValueError('Input linear operator must be square.')
        self.Linop = LinOp
        super().__init__(shape=LinOp.shape, dtype=LinOp.dtype, is_explicit=LinOp.is_explicit,
                         is_dense=LinOp.is_dense, is_sparse=LinOp.is_sparse, is_dask=LinOp.is_dask,
                         is_symmetric=LinOp.is_symmetric)

    def _poly(self, t, step):
        z = t
        y = O.scale(t, float(self.coeffs[0]))
        for c in self.coeffs[1:]:
            z = step(z)
            y = O.axpby(y, z, 1.0, float(c))
        return y

    def _apply(self, t):
        return self._poly(t, self.Linop._apply)

    def _adj(self, t):
        if self.is_symmetric:
            return self._apply(t)
        return self._poly(t, self.Linop._adj)

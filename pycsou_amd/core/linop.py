"""Linear operators (mirrors ``pycsou/core/linop.py``).

``LinearOperator`` keeps the reference contract: ``__call__``/``matvec`` and
``adjoint``, ``.H`` (``AdjointLinearOperator`` unless symmetric), ``jacobianT`` = the
adjoint operator, ``lipschitz_cst`` (= ``diff_lipschitz_cst``), sum / composition
algebra (``linop.py:442-553``).  Subclasses implement the device-level ``_apply`` and
``_adj`` on flat tensors.

``compute_lipschitz_cst`` replaces ARPACK ``svds``/``eigsh`` (``linop.py:279-321``,
host loop of tens to hundreds of operator applications) by a device Lanczos iteration
on ``K^T K`` with full re-orthogonalisation: every operator application stays on the
GPU, only the small tridiagonal eigenproblem runs on the host.
"""

from numbers import Number

import numpy as np
import torch

from .. import _ops as O
from .map import DifferentiableMap, DiffMapComp, DiffMapSum, Map, MapComp, MapSum


def _lanczos_sigma_max(apply_gram, n, dtype, sym=False, tol=1e-10, max_steps=300, seed=0):
    """Largest eigenvalue of the PSD Gram operator (or |eig| of a symmetric operator)
    by Lanczos with full re-orthogonalisation; returns the eigenvalue estimate."""
    g = torch.Generator(device='cpu').manual_seed(seed)
    q = torch.randn(n, generator=g, dtype=torch.float64).to(device=O.device(), dtype=dtype)
    q = q / torch.linalg.vector_norm(q)
    Q = torch.empty((min(max_steps, n) + 1, n), dtype=dtype, device=q.device)
    Q[0] = q
    alphas, betas = [], []
    prev = None
    theta = 0.0
    for j in range(min(max_steps, n)):
        w = apply_gram(Q[j])
        a = float(torch.dot(w.double(), Q[j].double()))
        alphas.append(a)
        # full re-orthogonalisation (twice is enough)
        for _ in range(2):
            c = Q[:j + 1] @ w
            w = w - Q[:j + 1].T @ c
        b = float(torch.linalg.vector_norm(w.double()))
        T = np.diag(alphas) + np.diag(betas, 1) + np.diag(betas, -1)
        ev = np.linalg.eigvalsh(T)
        theta = float(np.max(np.abs(ev))) if sym else float(ev[-1])
        if b <= 1e-300 or (prev is not None and abs(theta - prev) <= tol * abs(theta)):
            break
        prev = theta
        betas.append(b)
        Q[j + 1] = w / b
    return theta


class LinearOperator(DifferentiableMap):
    """Base class for linear operators (``pycsou/core/linop.py:21-485``)."""

    def __init__(self, shape, dtype=None, is_explicit=False, is_dense=False, is_sparse=False, is_dask=False,
                 is_symmetric=False, lipschitz_cst=np.inf):
        DifferentiableMap.__init__(self, shape=shape, is_linear=True, lipschitz_cst=lipschitz_cst,
                                   diff_lipschitz_cst=lipschitz_cst)
        self.dtype = dtype
        self.is_explicit = is_explicit
        self.is_dense = is_dense
        self.is_sparse = is_sparse
        self.is_dask = is_dask
        self.is_symmetric = is_symmetric
        self.is_square = shape[0] == shape[1]

    # -- device layer
    def _adj(self, t):
        raise NotImplementedError

    def _jacT(self, t=None):
        return self.get_adjointOp()

    # -- public layer
    def matvec(self, x):
        return self.__call__(x)

    def adjoint(self, y):
        if isinstance(y, Number):
            y = np.asarray([y], dtype=float)
        return O.like(self._adj(O.to_dev(y)), y)

    def transpose(self, y):
        return self.adjoint(y)  # real operators only

    def jacobianT(self, arg=None):
        return self.get_adjointOp()

    def get_adjointOp(self):
        return self if self.is_symmetric else AdjointLinearOperator(self)

    @property
    def H(self):
        return self.get_adjointOp()

    def get_transposeOp(self):
        return TransposeLinearOperator(self)

    @property
    def T(self):
        return self.get_transposeOp()

    @property
    def RangeGram(self):
        return SymmetricLinearOperator(self * self.H)

    @property
    def DomainGram(self):
        return SymmetricLinearOperator(self.H * self)

    # -- spectral helpers
    def _compute_dtype(self):
        return O.torch_dtype(self.dtype)

    def tosciop(self):
        import scipy.sparse.linalg as spls
        return spls.LinearOperator(dtype=np.float64, shape=self.shape, matvec=lambda v: self.matvec(v),
                                   rmatvec=lambda v: self.adjoint(v))

    @property
    def SciOp(self):
        return self.tosciop()

    def eigenvals(self, k, which='LM', **kwargs):
        import scipy.sparse.linalg as spls
        if self.is_symmetric:
            return spls.eigsh(A=self.SciOp, k=k, which=which, return_eigenvectors=False, **kwargs)
        if self.is_square:
            return spls.eigs(A=self.SciOp, k=k, which=which, return_eigenvectors=False, **kwargs)
        raise NotImplementedError('The function eigenvals is only for square linear operator. For non square linear '
                                  'operators, use the method singularvals.')

    def singularvals(self, k, which='LM', **kwargs):
        import scipy.sparse.linalg as spls
        return spls.svds(A=self.SciOp, k=k, which=which, return_singular_vectors=False, **kwargs)

    def compute_lipschitz_cst(self, tol=1e-10, max_steps=300, **kwargs):
        """Operator norm ``||K||_2`` by device Lanczos on ``K^T K`` (or ``|eig|`` if symmetric)."""
        dtype = torch.float64
        if self.is_symmetric:
            lam = _lanczos_sigma_max(lambda v: self._apply(v), self.shape[1], dtype, sym=True, tol=tol,
                                     max_steps=max_steps)
            self.lipschitz_cst = float(abs(lam))
        else:
            lam = _lanczos_sigma_max(lambda v: self._adj(self._apply(v)), self.shape[1], dtype, tol=tol,
                                     max_steps=max_steps)
            self.lipschitz_cst = float(np.sqrt(max(lam, 0.0)))
        self.diff_lipschitz_cst = self.lipschitz_cst

    # -- algebra (linop.py:442-485)
    def __add__(self, other):
        if isinstance(other, LinearOperator):
            return LinOpSum(self, other)
        if isinstance(other, DifferentiableMap):
            return DiffMapSum(self, other)
        if isinstance(other, Map):
            return MapSum(self, other)
        raise NotImplementedError

    def __mul__(self, other):
        if isinstance(other, Number):
            from ..linop.base import HomothetyMap
            other = HomothetyMap(constant=other, size=self.shape[1])
        if O.is_array(other):
            return self(other)
        if isinstance(other, LinearOperator):
            return LinOpComp(self, other)
        if isinstance(other, DifferentiableMap):
            return DiffMapComp(self, other)
        if isinstance(other, Map):
            return MapComp(self, other)
        raise NotImplementedError

    def __rmul__(self, other):
        if isinstance(other, Number):
            from ..linop.base import HomothetyMap
            other = HomothetyMap(constant=other, size=self.shape[0])
        if isinstance(other, LinearOperator):
            return LinOpComp(other, self)
        if isinstance(other, DifferentiableMap):
            return DiffMapComp(other, self)
        if isinstance(other, Map):
            return MapComp(other, self)
        raise NotImplementedError


class AdjointLinearOperator(LinearOperator):
    """``linop.py:488-506``."""

    def __init__(self, LinOp):
        super().__init__(shape=(LinOp.shape[1], LinOp.shape[0]), dtype=LinOp.dtype, is_explicit=LinOp.is_explicit,
                         is_dask=LinOp.is_dask, is_dense=LinOp.is_dense, is_sparse=LinOp.is_sparse,
                         is_symmetric=LinOp.is_symmetric)
        self.Linop = LinOp

    def _apply(self, t):
        return self.Linop._adj(t)

    def _adj(self, t):
        return self.Linop._apply(t)

    def compute_lipschitz_cst(self, **kwargs):
        if self.Linop.lipschitz_cst != np.inf:
            self.lipschitz_cst = self.Linop.lipschitz_cst
        else:
            LinearOperator.compute_lipschitz_cst(self, **kwargs)


class TransposeLinearOperator(AdjointLinearOperator):
    """``linop.py:509-521`` (real operators: transpose == adjoint)."""


class LinOpSum(LinearOperator, DiffMapSum):
    """``linop.py:524-537``."""

    def __init__(self, LinOp1, LinOp2, dtype=None):
        dtype = LinOp1.dtype if LinOp1.dtype is LinOp2.dtype else dtype
        DiffMapSum.__init__(self, map1=LinOp1, map2=LinOp2)
        LinearOperator.__init__(self, shape=self.shape, dtype=dtype, is_explicit=LinOp1.is_explicit & LinOp2.is_explicit,
                                is_dask=LinOp1.is_dask & LinOp2.is_dask, is_dense=LinOp1.is_dense & LinOp2.is_dense,
                                is_sparse=LinOp1.is_sparse & LinOp2.is_sparse,
                                is_symmetric=LinOp1.is_symmetric & LinOp2.is_symmetric,
                                lipschitz_cst=self.lipschitz_cst)
        self.LinOp1, self.LinOp2 = LinOp1, LinOp2

    def _apply(self, t):
        return O.add(self.LinOp1._apply(t), self.LinOp2._apply(t))

    def _adj(self, t):
        return O.add(self.LinOp1._adj(t), self.LinOp2._adj(t))


class LinOpComp(LinearOperator, DiffMapComp):
    """``linop.py:540-553``."""

    def __init__(self, LinOp1, LinOp2, dtype=None):
        dtype = LinOp1.dtype if LinOp1.dtype is LinOp2.dtype else dtype
        DiffMapComp.__init__(self, map1=LinOp1, map2=LinOp2)
        LinearOperator.__init__(self, shape=self.shape, dtype=dtype, is_explicit=LinOp1.is_explicit & LinOp2.is_explicit,
                                is_dask=LinOp1.is_dask & LinOp2.is_dask, is_dense=LinOp1.is_dense & LinOp2.is_dense,
                                is_sparse=LinOp1.is_sparse & LinOp2.is_sparse,
                                is_symmetric=LinOp1.is_symmetric & LinOp2.is_symmetric,
                                lipschitz_cst=self.lipschitz_cst)
        self.LinOp1, self.LinOp2 = LinOp1, LinOp2

    def _apply(self, t):
        return self.LinOp1._apply(self.LinOp2._apply(t))

    def _adj(self, t):
        return self.LinOp2._adj(self.LinOp1._adj(t))

    def _jacT(self, t=None):
        return self.get_adjointOp()


class SymmetricLinearOperator(LinearOperator):
    """``linop.py:556-571``."""

    def __init__(self, LinOp):
        if LinOp.shape[0] != LinOp.shape[1]:
            raise TypeError('The input linear operator is not symmetric.')
        super().__init__(shape=LinOp.shape, dtype=LinOp.dtype, is_explicit=LinOp.is_explicit, is_dask=LinOp.is_dask,
                         is_dense=LinOp.is_dense, is_sparse=LinOp.is_sparse, is_symmetric=True,
                         lipschitz_cst=LinOp.lipschitz_cst)
        self.LinOp = LinOp

    def _apply(self, t):
        return self.LinOp._apply(t)

    def _adj(self, t):
        return self.LinOp._apply(t)


class UnitaryOperator(LinearOperator):
    """``linop.py:574-615``."""

    def __init__(self, size, dtype=None, is_explicit=False, is_dense=False, is_sparse=False, is_dask=False,
                 is_symmetric=False):
        super().__init__(shape=(size, size), dtype=dtype, is_explicit=is_explicit, is_dense=is_dense,
                         is_sparse=is_sparse, is_dask=is_dask, is_symmetric=is_symmetric)
        self.size = size
        self.lipschitz_cst = self.diff_lipschitz_cst = 1

    def compute_lipschitz_cst(self, **kwargs):
        self.lipschitz_cst = self.diff_lipschitz_cst = 1

    def singularvals(self, k, which='LM', **kwargs):
        if k > min(self.shape):
            raise ValueError('The number of singular values must not exceed the smallest dimension size.')
        return np.ones(shape=(k,))

    def eigenvals(self, k, which='LM', **kwargs):
        return self.singularvals(k=k)

    def pinv(self, y, eps=0, **kwargs):
        return self.adjoint(y)

    @property
    def PinvOp(self):
        return self.H

    def cond(self, **kwargs):
        return 1

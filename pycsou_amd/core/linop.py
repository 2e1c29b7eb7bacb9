"""Linear operators (mirrors ``pycsou/core/linop.py``).

``LinearOperator`` keeps the reference contract: ``__call__``/``matvec`` and
``adjoint``, ``.H`` (``AdjointLinearOperator`` unless symmetric), ``jacobianT`` = the
adjoint operator, ``lipschitz_cst`` (= ``diff_lipschitz_cst``), sum / composition
algebra (``linop.py:442-553``).  Subclasses implement the device-level ``_apply`` and
``_adj`` on flat tensors.

``compute_lipschitz_cst`` replaces ARPACK ``svds``/``eigsh`` (``linop.py:279-321``,
host loop of tens to hundreds of operator applications) by a device Lanczos iteration
on ``K^T K`` in O(1) vectors: every operator application and the recurrence stay on the
GPU, only the small tridiagonal eigenproblem runs on the host every few steps.
"""

import warnings
from numbers import Number

import numpy as np
import torch

from .. import _ops as O
from .map import DifferentiableMap, DiffMapComp, DiffMapSum, Map, MapComp, MapSum


def _lanczos_extreme(apply, n, sym=False, tol=1e-9, max_steps=5000, check_every=10, seed=0, device=None):
    """Largest eigenvalue of a PSD Gram operator (or largest |eigenvalue| of a symmetric one) by
    plain Lanczos in fp64 with O(1) memory: three vectors of ``n`` (q_prev, q, w) plus what
    ``apply`` allocates, no re-orthogonalisation (the extreme Ritz value converges regardless;
    lost orthogonality only duplicates it).  The recurrence coefficients stay on the device
    (no host sync per step); every ``check_every`` steps the tridiagonal matrix T is copied to
    the host and its extreme eigenpair (theta, s) computed, with the residual of the Ritz pair
    r = beta_k |s_k| = ||A y - theta y|| (y the Ritz vector; no extra operator application).
    The run stops when r <= tol |theta|, when theta moved by at most ``tol`` (relative) since
    the previous check, or on an invariant subspace (beta ~ 0).

    Returns theta + r when the residual test or stagnation stopped the run (some eigenvalue lies
    within r of the Ritz value; a Ritz value never exceeds the extreme eigenvalue, so the value
    stays on the high side of theta, which keeps tau sigma ||K||^2 <= 1 on the safe side even
    without re-orthogonalisation), and theta itself on an invariant subspace (r = 0: theta is an
    eigenvalue of A).  A stagnated theta is accepted only while its residual is small too
    (r <= sqrt(tol) |theta|, so theta + r over-estimates by at most that much): otherwise the run
    goes on to the residual test or ``max_steps`` (ADVICE r5 -- a loose bound would shrink tau and
    sigma below the reference's svds-based step sizes); a run that ends with a residual above that
    warns.  The
    structured operators of the path (Gradient, derivatives, separable / 1-D convolutions) do not
    come here: their norms are exact (linop/_spectral.py).
    """
    from scipy.linalg import eigh_tridiagonal, eigvalsh_tridiagonal
    dev = O.device() if device is None else device
    g = torch.Generator(device='cpu').manual_seed(seed)
    q = torch.randn(n, generator=g, dtype=torch.float64).to(dev)
    q /= torch.linalg.vector_norm(q)
    q_prev = torch.zeros_like(q)
    steps = max(1, min(int(max_steps), 10 * n + 10))
    alphas = torch.zeros(steps, dtype=torch.float64, device=dev)
    betas = torch.zeros(steps, dtype=torch.float64, device=dev)
    b_prev = torch.zeros((), dtype=torch.float64, device=dev)
    theta, resid, prev = 0.0, 0.0, None
    for j in range(steps):
        w = apply(q).to(torch.float64)
        a = torch.dot(w, q)
        w -= a * q
        w -= b_prev * q_prev
        b = torch.linalg.vector_norm(w)
        alphas[j], betas[j] = a, b
        q_prev, q, b_prev = q, w / b, b
        if (j + 1) % check_every and j + 1 < steps:
            continue
        al = alphas[:j + 1].cpu().numpy()
        be = betas[:j + 1].cpu().numpy()
        scale = max(np.max(np.abs(al[np.isfinite(al)]), initial=0.0), 1e-300)
        bad = np.nonzero(~np.isfinite(be) | (be <= 1e-13 * scale))[0]
        k = int(bad[0]) + 1 if bad.size else j + 1  # T of size k: alphas[:k], betas[:k-1]
        if k > 1:
            # the extreme eigenvalue, then its eigenvector alone (O(k) per check, not the O(k^2)
            # of a full eigendecomposition of T)
            i = k - 1
            if sym:
                ends = eigvalsh_tridiagonal(al[:k], be[:k - 1], select='i', select_range=(0, 0)), \
                    eigvalsh_tridiagonal(al[:k], be[:k - 1], select='i', select_range=(k - 1, k - 1))
                i = 0 if abs(ends[0][0]) > abs(ends[1][0]) else k - 1
            ev, S = eigh_tridiagonal(al[:k], be[:k - 1], select='i', select_range=(i, i))
            theta = float(abs(ev[0])) if sym else float(ev[0])
            # residual of the Ritz pair: the next beta times the last component of its vector
            resid = 0.0 if bad.size else float(abs(be[k - 1] * S[-1, 0]))
        else:
            theta, resid = (float(abs(al[0])) if sym else float(al[0])), (0.0 if bad.size else float(abs(be[0])))
        if bad.size:
            return theta
        if resid <= tol * abs(theta):
            return theta + resid
        loose = resid > np.sqrt(tol) * abs(theta)
        if prev is not None and abs(theta - prev) <= tol * abs(theta) and not loose:
            return theta + resid
        prev = theta
    if resid > np.sqrt(tol) * abs(theta):
        warnings.warn(f'Lanczos: {steps} steps left the Ritz residual at {resid / max(abs(theta), 1e-300):.2e} of '
                      f'theta; the returned bound theta + r may over-estimate the norm by that much')
    return theta + resid


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

    def compute_lipschitz_cst(self, tol=1e-9, max_steps=5000, **kwargs):
        """Operator norm ``||K||_2`` (``pycsou/core/linop.py:279-321``: ARPACK ``svds`` / ``eigsh``
        with k=1) by device Lanczos on ``K^T K`` (or ``|eig|`` if symmetric) in bounded memory
        (a few vectors of the domain size, whatever the operator's size).  Other ARPACK keyword
        arguments are accepted and ignored; ``tol`` is the relative residual (or change of the
        estimate between checks) at which the iteration stops; the value is accurate to about
        ``tol`` relative (see _lanczos_extreme).  Structured operators override this with their
        exact norms (linop/_spectral.py)."""
        if self.is_symmetric:
            lam = _lanczos_extreme(lambda v: self._apply(v), self.shape[1], sym=True, tol=tol, max_steps=max_steps)
            self.lipschitz_cst = float(abs(lam))
        else:
            lam = _lanczos_extreme(lambda v: self._adj(self._apply(v)), self.shape[1], tol=tol, max_steps=max_steps)
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

    def _factors(self):
        out = []
        for op in (self.LinOp1, self.LinOp2):
            out.extend(op._factors() if isinstance(op, LinOpComp) else [op])
        return out

    def compute_lipschitz_cst(self, **kwargs):
        """A composition of Convolve1D along distinct axes of one shape (the reference's only 3-D
        blur, pycsou/linop/conv.py:20-164) is a Kronecker product: its norm is the product of the
        factors' exact norms.  Anything else: the device Lanczos."""
        from ..linop.conv import Convolve1DOp
        f = self._factors()
        if all(isinstance(o, Convolve1DOp) for o in f) and len({o.dims for o in f}) == 1 \
                and len({o.axis for o in f}) == len(f):
            self.lipschitz_cst = self.diff_lipschitz_cst = float(np.sqrt(np.prod([o.norm2() for o in f])))
            return
        LinearOperator.compute_lipschitz_cst(self, **kwargs)


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

"""Finite-difference operators on the GPU (``pycsou/linop/diff.py`` hot-path subset).

``FirstDerivative`` (``diff.py:24-130``), ``Gradient`` (``diff.py:777-882``) and
``Laplacian`` (``diff.py:885-957``) keep the reference signatures and defaults and the
PyLops 1.x arithmetic they delegate to (forward / backward / 3-point centred stencils,
one-sided ends with ``edge=True``, ``Gradient`` = stacked ``[D_0 x; D_1 x; ...]``,
adjoint = accumulated ``sum_k D_k^T z_k``).  Matvec and adjoint are the gfx950 kernels
``pcs_deriv1_*``, ``pcs_grad_*``, ``pcs_lap_*``.
"""

from numbers import Number

import numpy as np

from .. import _ops as O
from ..core.linop import LinearOperator
from . import _spectral as S


def _steps(step, nd):
    if isinstance(step, Number):
        return [float(step)] * nd
    step = [float(s) for s in step]
    if len(step) != nd:
        raise ValueError('step must be a float or one value per axis')
    return step


class _DiffOp(LinearOperator):
    def __init__(self, shape, size, dtype):
        super().__init__(shape=shape, dtype=np.dtype(dtype), is_explicit=False, lipschitz_cst=np.inf)
        self._size = size


class FirstDerivativeOp(_DiffOp):
    """``pylops.FirstDerivative`` restated on the GPU."""

    def __init__(self, size, shape=None, axis=0, step=1.0, edge=True, dtype='float64', kind='forward'):
        if kind not in ('forward', 'centered', 'backward'):
            raise NotImplementedError('kind must be forward, centered, or backward')
        dims = (size,) if shape is None else tuple(int(s) for s in shape)
        if int(np.prod(dims)) != size:
            raise ValueError('shape and size are not compatible')
        if not 1 <= len(dims) <= 32:
            raise NotImplementedError('FirstDerivative supports 1-D to 32-D arrays')
        super().__init__((size, size), size, dtype)
        self.dims, self.axis, self.step, self.edge, self.kind = dims, int(axis), float(step), bool(edge), kind

    def _apply(self, t):
        return O.deriv1(t, self.dims, self.axis, self.step, self.kind, self.edge)

    def _adj(self, t):
        return O.deriv1(t, self.dims, self.axis, self.step, self.kind, self.edge, adjoint=True)

    def compute_lipschitz_cst(self, **kwargs):
        """Exact ||D|| = sqrt(lambda_max(D_1^T D_1)) of the 1-D stencil along the axis (K = I (x) D_1 (x) I;
        linop/_spectral.py), in place of the reference's ARPACK svds (pycsou/core/linop.py:279-321)."""
        self.lipschitz_cst = self.diff_lipschitz_cst = float(
            np.sqrt(S.deriv1_norm2(self.dims[self.axis], self.kind, self.edge, self.step)))


def FirstDerivative(size, shape=None, axis=0, step=1.0, edge=True, dtype='float64', kind='forward'):
    """``pycsou/linop/diff.py:24-130``."""
    return FirstDerivativeOp(size, shape=shape, axis=axis, step=step, edge=edge, dtype=dtype, kind=kind)


class GradientOp(_DiffOp):
    """``pylops.Gradient`` = ``VStack([FirstDerivative(dir=k)])`` on the GPU."""

    def __init__(self, shape, step=1.0, edge=True, dtype='float64', kind='centered'):
        if kind not in ('forward', 'centered', 'backward'):
            raise NotImplementedError('kind must be forward, centered, or backward')
        dims = tuple(int(s) for s in shape)
        if not 1 <= len(dims) <= 32:
            raise NotImplementedError('Gradient supports 1-D to 32-D arrays')
        N = int(np.prod(dims))
        super().__init__((len(dims) * N, N), N, dtype)
        self.dims, self.steps, self.edge, self.kind = dims, _steps(step, len(dims)), bool(edge), kind

    def _apply(self, t):
        return O.grad_fwd(t, self.dims, self.steps, self.kind, self.edge)

    def _adj(self, t):
        return O.grad_adj(t, self.dims, self.steps, self.kind, self.edge)

    def compute_lipschitz_cst(self, **kwargs):
        """Exact ||K||: K^T K = sum_k I (x) D_k^T D_k (x) I is a Kronecker sum, so ||K||^2 = sum_k
        lambda_max(D_k^T D_k) over the 1-D stencils of the axes (linop/_spectral.py; forward /
        backward: 4 sin^2(pi (n-1) / 2n) / h^2 per axis), in place of the reference's ARPACK svds
        (pycsou/core/linop.py:279-321)."""
        self.lipschitz_cst = self.diff_lipschitz_cst = float(np.sqrt(sum(
            S.deriv1_norm2(n, self.kind, self.edge, h) for n, h in zip(self.dims, self.steps))))


def Gradient(shape, step=1., edge=True, dtype='float64', kind='centered'):
    """``pycsou/linop/diff.py:777-882``."""
    return GradientOp(shape, step=step, edge=edge, dtype=dtype, kind=kind)


class LaplacianOp(_DiffOp):
    """``pylops.Laplacian`` (2-D): ``w0 * D2_0 + w1 * D2_1`` on the GPU."""

    def __init__(self, shape, weights=(1, 1), step=1., edge=True, dtype='float64'):
        dims = tuple(int(s) for s in shape)
        if len(dims) != 2:
            raise NotImplementedError('Laplacian is 2-D in the reference (pycsou/linop/diff.py:885)')
        N = int(np.prod(dims))
        super().__init__((N, N), N, dtype)
        self.dims, self.weights, self.steps, self.edge = dims, tuple(float(w) for w in weights), _steps(step, 2), bool(edge)

    def _apply(self, t):
        return O.lap(t, self.dims, self.weights, self.steps, self.edge)

    def _adj(self, t):
        return O.lap(t, self.dims, self.weights, self.steps, self.edge, adjoint=True)


def Laplacian(shape, weights=(1, 1), step=1., edge=True, dtype='float64'):
    """``pycsou/linop/diff.py:885-957``."""
    return LaplacianOp(shape, weights=weights, step=step, edge=edge, dtype=dtype)


class SecondDerivativeOp(_DiffOp):
    """``pylops.SecondDerivative`` restated on the GPU (``pcs_deriv2_*``)."""

    def __init__(self, size, shape=None, axis=0, step=1.0, edge=True, dtype='float64'):
        dims = (size,) if shape is None else tuple(int(s) for s in shape)
        if int(np.prod(dims)) != size:
            raise ValueError('shape and size are not compatible')
        if not 1 <= len(dims) <= 32:
            raise NotImplementedError('SecondDerivative supports 1-D to 32-D arrays')
        super().__init__((size, size), size, dtype)
        self.dims, self.axis, self.step, self.edge = dims, int(axis), float(step), bool(edge)

    def _apply(self, t):
        return O.deriv2(t, self.dims, self.axis, self.step, self.edge)

    def _adj(self, t):
        return O.deriv2(t, self.dims, self.axis, self.step, self.edge, adjoint=True)

    def compute_lipschitz_cst(self, **kwargs):
        """Exact ||D2|| of the 1-D second-difference stencil along the axis (linop/_spectral.py)."""
        self.lipschitz_cst = self.diff_lipschitz_cst = float(
            np.sqrt(S.deriv2_norm2(self.dims[self.axis], self.edge, self.step)))


def SecondDerivative(size, shape=None, axis=0, step=1.0, edge=True, dtype='float64'):
    """``pycsou/linop/diff.py:133-219``."""
    return SecondDerivativeOp(size, shape=shape, axis=axis, step=step, edge=edge, dtype=dtype)


def _kill_edges(Dgen, shape, axis, order, kind):
    from .base import DiagonalOperator
    k = np.ones(shape=Dgen.shape[0]) if shape is None else np.ones(shape=shape)
    if axis > 0:
        k = np.swapaxes(k, axis, 0)
    if kind == 'forward':
        k[-order:] = 0
    elif kind == 'backward':
        k[:order] = 0
    elif kind == 'centered':
        k[-order:] = 0
        k[:order] = 0
    if axis > 0:
        k = np.swapaxes(k, 0, axis)
    return DiagonalOperator(k.reshape(-1)) * Dgen


def GeneralisedDerivative(size, shape=None, axis=0, step=1.0, edge=True, dtype='float64', kind_op='iterated',
                          kind_diff='centered', **kwargs):
    """``pycsou/linop/diff.py:222-377``: ``D^N`` ('iterated'), ``(a^2 I - D2)^N`` ('sobolev'),
    ``(a I + D)^N`` ('exponential') or ``P(D)`` ('polynomial'), with the unreliable edge samples
    zeroed by a diagonal mask."""
    from .base import IdentityOperator, PolynomialLinearOperator
    D = FirstDerivative(size=size, shape=shape, axis=axis, step=step, edge=edge, dtype=dtype, kind=kind_diff)
    D.is_symmetric = False
    D2 = SecondDerivative(size=size, shape=shape, axis=axis, step=step, edge=edge, dtype=dtype)
    if kind_op == 'iterated':
        N = kwargs['order']
        Dgen, order = D ** N, N
    elif kind_op == 'sobolev':
        I = IdentityOperator(size=size)
        N = kwargs['order']
        Dgen, order = ((kwargs['constant'] ** 2) * I - D2) ** N, 2 * N
    elif kind_op == 'exponential':
        I = IdentityOperator(size=size)
        N = kwargs['order']
        Dgen, order = (kwargs['constant'] * I + D) ** N, N
    elif kind_op == 'polynomial':
        coeffs = kwargs['coeffs']
        Dgen, order = PolynomialLinearOperator(LinOp=D, coeffs=coeffs), len(coeffs) - 1
    else:
        raise NotImplementedError(
            'Supported generalised derivative types are: iterated, sobolev, exponential, polynomial.')
    return _kill_edges(Dgen, shape, axis, order, kind_diff)


def GeneralisedLaplacian(shape=None, step=1., edge=True, dtype='float64', kind='iterated', **kwargs):
    """``pycsou/linop/diff.py:960-1068``: ``Delta^N`` ('iterated'), ``(a^2 I - Delta)^N``
    ('sobolev') or ``P(Delta)`` ('polynomial') of the 2-D ``Laplacian``, with ``order`` edge samples
    zeroed along every axis."""
    from .base import DiagonalOperator, IdentityOperator, PolynomialLinearOperator
    Delta = Laplacian(shape=shape, step=step, edge=edge, dtype=dtype)
    Delta.is_symmetric = True
    if kind == 'iterated':
        N = kwargs['order']
        Dgen, order = Delta ** N, 2 * N
    elif kind == 'sobolev':
        I = IdentityOperator(size=shape[0] * shape[1])
        N = kwargs['order']
        Dgen, order = ((kwargs['constant'] ** 2) * I - Delta) ** N, 2 * N
    elif kind == 'polynomial':
        coeffs = kwargs['coeffs']
        Dgen, order = PolynomialLinearOperator(LinOp=Delta, coeffs=coeffs), 2 * (len(coeffs) - 1)
    else:
        raise NotImplementedError('Supported generalised derivative types are: iterated, sobolev, polynomial.')
    k = np.ones(shape=shape)
    for ax in range(len(shape)):
        k = np.swapaxes(k, ax, 0)
        k[-order:] = 0
        k[:order] = 0
        k = np.swapaxes(k, 0, ax)
    return DiagonalOperator(k.reshape(-1)) * Dgen

"""NumPy/SciPy restatement of the PyLops 1.x operators wrapped by pycsou.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

PyLops (``pylops >= 1.9.2``, 1.x keyword API) is not vendored under
``/root/reference`` and not installed.  This module restates its published
1.x algorithms for the operators on the hot path, as called from:

* ``pycsou/linop/diff.py:128``  ``pylops.FirstDerivative(N, dims, dir, sampling, edge, dtype, kind)``
* ``pycsou/linop/diff.py:219``  ``pylops.SecondDerivative(N, dims, dir, sampling, edge, dtype)``
* ``pycsou/linop/diff.py:882``  ``pylops.Gradient(dims, sampling, edge, dtype, kind)``
* ``pycsou/linop/diff.py:957``  ``pylops.Laplacian(dims, weights, sampling, edge, dtype)``
* ``pycsou/linop/conv.py:163``  ``pylops.signalprocessing.Convolve1D(N, h, dims, dir, dtype, method, offset)``
* ``pycsou/linop/conv.py:294``  ``pylops.signalprocessing.Convolve2D(N, h, dims, nodir, dtype, method, offset)``
* ``pycsou/linop/conv.py:358``  ``pylops.Smoothing1D(nsmooth, dims, dir, dtype)``
* ``pycsou/linop/conv.py:417``  ``pylops.Smoothing2D(nsmooth, dims, nodir, dtype)``
* ``pycsou/linop/sampling.py:121``  ``pylops.Restriction(M, iava, dims, dir, dtype, inplace)``

Every object exposes ``shape``, ``dtype``, ``explicit``, ``matvec`` and
``rmatvec`` -- the attributes pycsou's ``PyLopLinearOperator``
(``pycsou/linop/base.py:24-54``) reads -- so the fixture generator can hand
them to the reference's own adapter.
"""

import numpy as np
from scipy import signal


class _Op:
    explicit = False

    def __init__(self, shape, dtype):
        self.shape = (int(shape[0]), int(shape[1]))
        self.dtype = np.dtype(dtype)

    def __mul__(self, x):
        return self.matvec(x)


def _swap_in(x, dims, axis):
    x = np.reshape(x, dims)
    return np.swapaxes(x, axis, 0) if axis > 0 else x


def _swap_out(y, axis):
    if axis > 0:
        y = np.swapaxes(y, 0, axis)
    return np.ascontiguousarray(y).ravel()


class FirstDerivative(_Op):
    """PyLops 1.x ``FirstDerivative`` (first-order forward/backward, 3-point centered).

    forward : y[i] = (x[i+1]-x[i])/h for i<n-1, y[n-1] = 0
    backward: y[i] = (x[i]-x[i-1])/h for i>0,   y[0] = 0
    centered: y[i] = (0.5x[i+1]-0.5x[i-1])/h for 0<i<n-1; ends 0, or one-sided
              first-order differences when ``edge`` (pycsou default ``edge=True``,
              ``pycsou/linop/diff.py:24``).
    """

    def __init__(self, N, dims=None, dir=0, sampling=1.0, edge=False, dtype='float64', kind='centered'):
        super().__init__((N, N), dtype)
        if kind not in ('forward', 'backward', 'centered'):
            raise NotImplementedError('kind must be forward, centered, or backward')
        self.dims = (N,) if dims is None else tuple(int(d) for d in dims)
        if int(np.prod(self.dims)) != N:
            raise ValueError('product of dims must equal N')
        self.dir, self.sampling, self.edge, self.kind = int(dir), sampling, edge, kind

    def matvec(self, x):
        x = _swap_in(x, self.dims, self.dir)
        y = np.zeros(x.shape, self.dtype)
        h = self.sampling
        if self.kind == 'forward':
            y[:-1] = (x[1:] - x[:-1]) / h
        elif self.kind == 'backward':
            y[1:] = (x[1:] - x[:-1]) / h
        else:
            y[1:-1] = (0.5 * x[2:] - 0.5 * x[:-2]) / h
            if self.edge:
                y[0] = (x[1] - x[0]) / h
                y[-1] = (x[-1] - x[-2]) / h
        return _swap_out(y, self.dir)

    def rmatvec(self, x):
        x = _swap_in(x, self.dims, self.dir)
        y = np.zeros(x.shape, self.dtype)
        h = self.sampling
        if self.kind == 'forward':
            y[:-1] -= x[:-1] / h
            y[1:] += x[:-1] / h
        elif self.kind == 'backward':
            y[:-1] -= x[1:] / h
            y[1:] += x[1:] / h
        else:
            y[:-2] -= (0.5 * x[1:-1]) / h
            y[2:] += (0.5 * x[1:-1]) / h
            if self.edge:
                y[0] -= x[0] / h
                y[1] += x[0] / h
                y[-2] -= x[-1] / h
                y[-1] += x[-1] / h
        return _swap_out(y, self.dir)


class SecondDerivative(_Op):
    """PyLops 1.x ``SecondDerivative``: y[i] = (x[i+1]-2x[i]+x[i-1])/h^2, ends 0
    or second-order one-sided stencils when ``edge``."""

    def __init__(self, N, dims=None, dir=0, sampling=1.0, edge=False, dtype='float64'):
        super().__init__((N, N), dtype)
        self.dims = (N,) if dims is None else tuple(int(d) for d in dims)
        self.dir, self.sampling, self.edge = int(dir), sampling, edge

    def matvec(self, x):
        x = _swap_in(x, self.dims, self.dir)
        y = np.zeros(x.shape, self.dtype)
        h2 = self.sampling ** 2
        y[1:-1] = (x[2:] - 2 * x[1:-1] + x[:-2]) / h2
        if self.edge:
            y[0] = (x[0] - 2 * x[1] + x[2]) / h2
            y[-1] = (x[-3] - 2 * x[-2] + x[-1]) / h2
        return _swap_out(y, self.dir)

    def rmatvec(self, x):
        x = _swap_in(x, self.dims, self.dir)
        y = np.zeros(x.shape, self.dtype)
        h2 = self.sampling ** 2
        y[:-2] += x[1:-1] / h2
        y[1:-1] -= (2 * x[1:-1]) / h2
        y[2:] += x[1:-1] / h2
        if self.edge:
            y[0] += x[0] / h2
            y[1] -= (2 * x[0]) / h2
            y[2] += x[0] / h2
            y[-3] += x[-1] / h2
            y[-2] -= (2 * x[-1]) / h2
            y[-1] += x[-1] / h2
        return _swap_out(y, self.dir)


class VStack(_Op):
    """PyLops 1.x ``VStack``: matvec concatenates, rmatvec accumulates
    ``y = 0; y += op_k.rmatvec(x_k)`` in operator order."""

    def __init__(self, ops, dtype='float64'):
        n = ops[0].shape[1]
        super().__init__((sum(o.shape[0] for o in ops), n), dtype)
        self.ops = ops
        self.cuts = np.cumsum([0] + [o.shape[0] for o in ops])

    def matvec(self, x):
        return np.concatenate([o.matvec(x) for o in self.ops])

    def rmatvec(self, x):
        y = np.zeros(self.shape[1], dtype=self.dtype)
        for i, o in enumerate(self.ops):
            y += o.rmatvec(x[self.cuts[i]:self.cuts[i + 1]])
        return y


def Gradient(dims, sampling=1, edge=False, dtype='float64', kind='centered'):
    """PyLops 1.x ``Gradient``: ``VStack([FirstDerivative(dir=k) for k])``."""
    ndims = len(dims)
    if np.isscalar(sampling):
        sampling = [sampling] * ndims
    N = int(np.prod(dims))
    return VStack([FirstDerivative(N, dims=dims, dir=k, sampling=sampling[k], edge=edge, dtype=dtype, kind=kind)
                   for k in range(ndims)], dtype=dtype)


class _WeightedSum(_Op):
    def __init__(self, ops, weights, dtype):
        super().__init__(ops[0].shape, dtype)
        self.ops, self.weights = ops, weights

    def matvec(self, x):
        y = self.weights[0] * self.ops[0].matvec(x)
        for w, o in zip(self.weights[1:], self.ops[1:]):
            y = y + w * o.matvec(x)
        return y

    def rmatvec(self, x):
        y = np.conj(self.weights[0]) * self.ops[0].rmatvec(x)
        for w, o in zip(self.weights[1:], self.ops[1:]):
            y = y + np.conj(w) * o.rmatvec(x)
        return y


def Laplacian(dims, dirs=(0, 1), weights=(1, 1), sampling=(1, 1), edge=False, dtype='float64'):
    """PyLops 1.x ``Laplacian``: ``w0*SecondDerivative(dir0) + w1*SecondDerivative(dir1)``."""
    N = int(np.prod(dims))
    ops = [SecondDerivative(N, dims=dims, dir=dirs[i], sampling=sampling[i], edge=edge, dtype=dtype)
           for i in range(2)]
    return _WeightedSum(ops, list(weights), dtype)


def _pad_filter(h, offsets):
    """PyLops 1.x offset rule: ``2*(nh//2 - offset)`` (minus 1 for even nh)
    zeros are padded in front (positive) or at the back (negative)."""
    pad = []
    for n, off in zip(h.shape, offsets):
        o = 2 * (n // 2 - int(off))
        if n % 2 == 0:
            o -= 1
        pad.append((o, 0) if o > 0 else (0, -o))
    return np.pad(h, pad, mode='constant')


class ConvolveND(_Op):
    """PyLops 1.x ``ConvolveND``: forward ``signal.convolve(x, h, 'same')``,
    adjoint ``signal.correlate(x, h, 'same')`` (zero boundary)."""

    def __init__(self, N, h, dims, offset, dirs=None, method='fft', dtype='float64'):
        super().__init__((N, N), dtype)
        self.dims = tuple(int(d) for d in dims)
        h = _pad_filter(np.asarray(h), offset)
        dirs = list(range(len(self.dims))) if dirs is None else list(dirs)
        if h.ndim != len(self.dims):
            shp = [1] * len(self.dims)
            for i, d in enumerate(dirs):
                shp[d] = h.shape[i]
            h = h.reshape(shp)
        self.h = h
        self.method = method

    def matvec(self, x):
        x = np.reshape(x, self.dims)
        return signal.convolve(x, self.h, mode='same', method=self.method).ravel().astype(self.dtype, copy=False)

    def rmatvec(self, x):
        x = np.reshape(x, self.dims)
        return signal.correlate(x, self.h, mode='same', method=self.method).ravel().astype(self.dtype, copy=False)


def Convolve2D(N, h, dims, offset=(0, 0), nodir=None, dtype='float64', method='fft'):
    """PyLops 1.x ``Convolve2D`` (``ConvolveND`` over the two axes != ``nodir``)."""
    if nodir is None:
        dirs = (0, 1)
    elif nodir == 0:
        dirs = (1, 2)
    elif nodir == 1:
        dirs = (0, 2)
    else:
        dirs = (0, 1)
    return ConvolveND(N, h, dims, offset, dirs=dirs, method=method, dtype=dtype)


def Convolve1D(N, h, offset=0, dims=None, dir=0, dtype='float64', method=None):
    """PyLops 1.x ``Convolve1D`` along axis ``dir`` of ``dims`` ('same', zero boundary)."""
    h = np.asarray(h)
    if offset > h.size - 1:
        raise ValueError('offset must be smaller than h.size - 1')
    dims = (N,) if dims is None else tuple(int(d) for d in dims)
    if method is None:
        method = 'direct'
    return ConvolveND(N, h, dims, (offset,), dirs=(dir,), method='fft' if method == 'overlapadd' else method,
                      dtype=dtype)


def pycsou_offset(n):
    """Offset pycsou passes to PyLops for a filter of length n
    (``pycsou/linop/conv.py:159-162, 285-292``)."""
    return n // 2 - 1 if n % 2 == 0 else n // 2


def Smoothing1D(nsmooth, dims, dir=0, dtype='float64'):
    """PyLops 1.x ``Smoothing1D``: an even ``nsmooth`` is raised by one; ``Convolve1D`` with
    ``ones(nsmooth) / nsmooth`` and offset ``(nsmooth - 1) / 2``."""
    dims = (int(dims),) if np.isscalar(dims) else tuple(int(d) for d in dims)
    if nsmooth % 2 == 0:
        nsmooth += 1
    return Convolve1D(int(np.prod(dims)), np.ones(nsmooth) / float(nsmooth), offset=(nsmooth - 1) // 2, dims=dims,
                      dir=dir, dtype=dtype)


def Smoothing2D(nsmooth, dims, nodir=None, dtype='float64'):
    """PyLops 1.x ``Smoothing2D``: box filter ``ones(n0, n1) / (n0 n1)`` (even sizes raised by
    one), centred, via ``Convolve2D``."""
    n = [int(v) for v in nsmooth]
    n = [v + 1 if v % 2 == 0 else v for v in n]
    h = np.ones((n[0], n[1])) / float(n[0] * n[1])
    dims = tuple(int(d) for d in dims)
    return Convolve2D(int(np.prod(dims)), h, dims, offset=((n[0] - 1) // 2, (n[1] - 1) // 2), nodir=nodir,
                      dtype=dtype)


class Restriction(_Op):
    """PyLops 1.x ``Restriction``: ``y = x.take(iava, axis=dir)``; adjoint ``x = 0;
    x[..., iava, ...] = y`` along ``dir``."""

    def __init__(self, M, iava, dims=None, dir=0, dtype='float64', inplace=True):
        self.iava = np.asarray(iava, dtype=np.int64).ravel()
        self.dims = (int(M),) if dims is None else tuple(int(d) for d in dims)
        self.dir = int(dir)
        out = list(self.dims)
        out[self.dir] = self.iava.size
        self.dimsd = tuple(out)
        super().__init__((int(np.prod(self.dimsd)), int(M)), dtype)

    def matvec(self, x):
        return np.take(np.reshape(x, self.dims), self.iava, axis=self.dir).ravel()

    def rmatvec(self, y):
        y = np.swapaxes(np.reshape(y, self.dimsd), self.dir, 0)
        x = np.zeros(np.swapaxes(np.zeros(self.dims, bool), self.dir, 0).shape, dtype=self.dtype)
        x[self.iava] = y
        return np.ascontiguousarray(np.swapaxes(x, 0, self.dir)).ravel()

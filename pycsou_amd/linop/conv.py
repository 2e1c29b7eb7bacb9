"""Convolution operators on the GPU (``pycsou/linop/conv.py`` hot-path subset).

``Convolve2D(size, filter, shape)`` (``conv.py:167-295``) and
``Convolve1D(size, filter, reshape_dims, axis)`` (``conv.py:20-164``) keep pycsou's
offset rule (``K//2`` for odd, ``K//2 - 1`` for even filters, ``conv.py:159-162,
285-292``) and PyLops 1.x semantics: forward = zero-boundary 'same' convolution,
adjoint = correlation.  The reference goes through ``scipy.signal.convolve(method='fft')``;
here both directions are direct gfx950 kernels, identical up to floating-point rounding:
``Convolve2D`` through a packed correlation plan (``pcs_conv2d_planned``, the register-blocked
row-marching kernel of ``csrc/corr2d.hip``, PSFs up to 31 x 31; ``pcs_conv2d`` beyond),
``Convolve1D`` through ``pcs_conv1d``.

``Convolve2D.separable()`` exposes a rank-1 factorisation ``h = c r^T`` when the PSF has
one (a Gaussian PSF does to ~1e-16): the fused PDS engine then applies the blur as two
1-D passes inside its tile kernel (60 instead of 450 flop/pixel per direction).
"""

import numpy as np
import torch

from .. import _ops as O
from ..core.linop import LinearOperator
from . import _spectral as S


def pycsou_offset(n):
    """``conv.py:159-162, 285-292``."""
    return n // 2 - 1 if n % 2 == 0 else n // 2


class _DevCache:
    def __init__(self, arr):
        self.arr = np.ascontiguousarray(arr)
        self._d = {}

    def get(self, dtype):
        t = self._d.get(dtype)
        if t is None:
            t = torch.as_tensor(self.arr.reshape(-1)).to(device=O.device(), dtype=dtype).contiguous()
            self._d[dtype] = t
        return t


class Convolve2DOp(LinearOperator):
    def __init__(self, size, filter, shape, dtype='float64', method='fft'):
        filt = np.asarray(filter, dtype=np.float64)
        if filt.ndim != 2:
            raise ValueError('filter must be a 2D array')
        dims = tuple(int(s) for s in shape)
        if len(dims) != 2 or dims[0] * dims[1] != size:
            raise ValueError('shape and size are not compatible')
        super().__init__(shape=(size, size), dtype=np.dtype(dtype), is_explicit=False, lipschitz_cst=np.inf)
        self.filter, self.dims, self.method = filt, dims, method
        self.kh, self.kw = filt.shape
        self.off = (pycsou_offset(self.kh), pycsou_offset(self.kw))
        self._h = _DevCache(filt)
        self._hf = _DevCache(filt[::-1, ::-1])
        self._plans = {}
        self._ffts = {}

    def plan(self, dtype, adjoint):
        """(tier, packed window) for pcs_conv2d_planned, or None (PSF wider than 31)."""
        key = (dtype, bool(adjoint))
        if key not in self._plans:
            self._plans[key] = O.conv2d_plan(self.filter, self.off[0], self.off[1], adjoint, dtype)
        return self._plans[key]

    def fft(self, dtype):
        """The FFT-domain plan (pcs_fftconv2d, rocFFT) used when the PSF is wider than the direct
        correlation's tiers (> 31 taps): cost independent of the PSF size, as the reference's
        default method='fft' (conv.py:209-217, 294)."""
        if dtype not in self._ffts:
            self._ffts[dtype] = O.FFTConv2D(self.filter, self.dims, self.off[0], self.off[1], dtype)
        return self._ffts[dtype]

    def _apply(self, t):
        p = self.plan(t.dtype, False)
        if p is not None:
            return O.conv2d_planned(t, self.dims, p)
        return self.fft(t.dtype).apply(t)

    def _apply_minus(self, t, y):
        """Conv x - y in one pass (residual of the data-fidelity term)."""
        p = self.plan(t.dtype, False)
        if p is not None:
            return O.conv2d_planned(t, self.dims, p, b=y, beta=-1.0)
        return self.fft(t.dtype).apply(t, b=y, beta=-1.0)

    def _adj(self, t):
        p = self.plan(t.dtype, True)
        if p is not None:
            return O.conv2d_planned(t, self.dims, p)
        return self.fft(t.dtype).apply(t, adjoint=True)

    def separable(self, rtol=1e-12):
        """(taps_axis0, taps_axis1, half) with centred taps of length 2*half+1 if the PSF is
        rank one to relative tolerance ``rtol``, else None."""
        u, s, vt = np.linalg.svd(self.filter)
        if s[0] == 0 or (s.size > 1 and s[1] > rtol * s[0]):
            return None
        c = u[:, 0] * np.sqrt(s[0])
        r = vt[0] * np.sqrt(s[0])
        if c.sum() < 0:
            c, r = -c, -r
        half = max(self.off[0], self.kh - 1 - self.off[0], self.off[1], self.kw - 1 - self.off[1])
        t0 = np.zeros(2 * half + 1)
        t1 = np.zeros(2 * half + 1)
        # out[i] = sum_j h[j] x[i + off - j] = sum_s w[s] x[i - s], s = j - off  ->  w[s + half] = h[s + off]
        t0[half - self.off[0]: half - self.off[0] + self.kh] = c
        t1[half - self.off[1]: half - self.off[1] + self.kw] = r
        return t0, t1, half

    def compute_lipschitz_cst(self, **kwargs):
        """||Conv||: a rank-1 PSF h = c r^T makes Conv = C_0 (x) C_1 (two 1-D 'same' convolutions at
        pycsou's offsets), so ||Conv|| = ||C_0|| ||C_1||, each exact from its banded Gram matrix
        (linop/_spectral.py); other PSFs keep the device Lanczos (core/linop.py).  Replaces the
        reference's ARPACK svds (pycsou/core/linop.py:279-321)."""
        u, s, vt = np.linalg.svd(self.filter)
        if s[0] > 0 and (s.size == 1 or s[1] <= 1e-13 * s[0]):
            c, r = u[:, 0] * np.sqrt(s[0]), vt[0] * np.sqrt(s[0])
            n0, n1 = self.dims
            # + the rank-1 remainder's bound ||Conv_e|| <= sum |e| <= sqrt(kh kw) ||e||_F (safe side)
            rest = float(np.sqrt(self.kh * self.kw * np.sum(s[1:] ** 2)))
            self.lipschitz_cst = self.diff_lipschitz_cst = float(
                np.sqrt(S.conv1d_norm2(n0, c, self.off[0]) * S.conv1d_norm2(n1, r, self.off[1]))) + rest
            return
        LinearOperator.compute_lipschitz_cst(self, **kwargs)


def Convolve2D(size, filter, shape, dtype='float64', method='fft'):
    """``pycsou/linop/conv.py:167-295``."""
    return Convolve2DOp(size, filter, shape, dtype=dtype, method=method)


class Convolve1DOp(LinearOperator):
    def __init__(self, size, filter, reshape_dims=None, axis=0, dtype='float64', method=None):
        h = np.asarray(filter, dtype=np.float64).reshape(-1)
        dims = (size,) if reshape_dims is None else tuple(int(s) for s in reshape_dims)
        if int(np.prod(dims)) != size:
            raise ValueError('reshape_dims and size are not compatible')
        if not 1 <= len(dims) <= 32:
            raise NotImplementedError('Convolve1D supports 1-D to 32-D arrays')
        super().__init__(shape=(size, size), dtype=np.dtype(dtype), is_explicit=False, lipschitz_cst=np.inf)
        self.filter, self.dims, self.axis, self.method = h, dims, int(axis), method
        self.k = h.size
        self.off = pycsou_offset(self.k)
        self._h = _DevCache(h)
        self._hf = _DevCache(h[::-1])

    def _apply(self, t):
        return O.conv1d(t, self.dims, self.axis, self._h.get(t.dtype), self.k, self.off)

    def _adj(self, t):
        return O.conv1d(t, self.dims, self.axis, self._hf.get(t.dtype), self.k, self.k - 1 - self.off)

    def norm2(self):
        """||Conv1D||^2 exactly: the 1-D banded Gram matrix along the axis (linop/_spectral.py)."""
        return S.conv1d_norm2(self.dims[self.axis], self.filter, self.off)

    def compute_lipschitz_cst(self, **kwargs):
        """Exact ||Conv1D|| (K = I (x) C (x) I), in place of the reference's ARPACK svds
        (pycsou/core/linop.py:279-321)."""
        self.lipschitz_cst = self.diff_lipschitz_cst = float(np.sqrt(self.norm2()))


def Convolve1D(size, filter, reshape_dims=None, axis=0, dtype='float64', method=None):
    """``pycsou/linop/conv.py:20-164``."""
    return Convolve1DOp(size, filter, reshape_dims=reshape_dims, axis=axis, dtype=dtype, method=method)


def _odd(n):
    n = int(n)
    return n + 1 if n % 2 == 0 else n


def MovingAverage1D(window_size, shape, axis=0, dtype='float64'):
    """``pycsou/linop/conv.py:298-359`` -> ``pylops.Smoothing1D(nsmooth, dims, dir)``: a box filter
    ``ones(n)/n`` (an even ``n`` is raised to ``n + 1``, PyLops 1.x) applied with ``Convolve1D``
    along ``axis``, centred (offset ``(n - 1) / 2``)."""
    n = _odd(window_size)
    dims = (int(shape),) if np.isscalar(shape) else tuple(int(s) for s in shape)
    return Convolve1DOp(int(np.prod(dims)), np.ones(n) / float(n), reshape_dims=dims, axis=axis, dtype=dtype)


def MovingAverage2D(window_shape, shape, dtype='float64'):
    """``pycsou/linop/conv.py:362-418`` -> ``pylops.Smoothing2D(nsmooth, dims)``: the 2-D box filter
    ``ones((n0, n1)) / (n0 n1)`` (even sizes raised to odd), centred, via ``Convolve2D``."""
    n0, n1 = _odd(window_shape[0]), _odd(window_shape[1])
    dims = tuple(int(s) for s in shape)
    return Convolve2DOp(int(np.prod(dims)), np.ones((n0, n1)) / float(n0 * n1), dims, dtype=dtype)

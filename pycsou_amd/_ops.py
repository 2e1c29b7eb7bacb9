"""Tensor-level wrappers over the C ABI + the array boundary of the public API.

Public pycsou-style methods accept NumPy arrays or torch tensors and return the same
kind they were given (NumPy in -> NumPy out, as in the reference; torch in -> device
tensor out).  Everything in between is a contiguous 1-D device tensor handled by the
gfx950 kernels.
"""

from numbers import Number

import ctypes

import numpy as np
import torch

from . import _lib as L

_ws_cache = {}


# ---------------------------------------------------------------- array boundary

def device():
    return torch.device('cuda', torch.cuda.current_device())


def torch_dtype(dtype, default=torch.float64):
    if dtype is None:
        return default
    if isinstance(dtype, torch.dtype):
        return dtype
    d = np.dtype(dtype)
    if d == np.float32:
        return torch.float32
    return torch.float64


def to_dev(x, dtype=None):
    """Contiguous flat device tensor (float32/float64) from NumPy / torch / scalar."""
    L.gpu()
    if isinstance(x, torch.Tensor):
        t = x
        if dtype is None and t.dtype not in (torch.float32, torch.float64):
            dtype = torch.float64
        if dtype is not None and t.dtype != dtype:
            t = t.to(dtype)
        if not t.is_cuda:
            t = t.to(device())
        return t.reshape(-1).contiguous()
    a = np.asarray(x)
    if dtype is None:
        dtype = torch.float32 if a.dtype == np.float32 else torch.float64
    return torch.as_tensor(np.ascontiguousarray(a).reshape(-1)).to(device=device(), dtype=dtype)


def like(out, ref):
    """Return `out` (device tensor) as the array kind of `ref`."""
    if isinstance(ref, torch.Tensor):
        return out
    return out.detach().cpu().numpy()


def numel(x):
    return int(x.numel()) if isinstance(x, torch.Tensor) else int(np.size(x))


def is_array(x):
    return isinstance(x, (np.ndarray, torch.Tensor))


def empty_like(t):
    return torch.empty_like(t)


# ---------------------------------------------------------------- elementwise / algebra

def axpby(x, y, a, b, out=None):
    """out = a*x + b*y  (y may be None)."""
    lib = L.gpu()
    out = torch.empty_like(x) if out is None else out
    L.check(lib.pcs_axpby(L.dtcode(x), L.ptr(x), L.ptr(y), L.ptr(out), x.numel(), float(a), float(b),
                          L.stream()), 'pcs_axpby')
    return out


def scale(x, a):
    return axpby(x, None, a, 0.0)


def add(x, y):
    return axpby(x, y, 1.0, 1.0)


def mul(x, d):
    """d * x elementwise (pcs_mul)."""
    lib = L.gpu()
    out = torch.empty_like(x)
    L.check(lib.pcs_mul(L.dtcode(x), L.ptr(x), L.ptr(d), L.ptr(out), x.numel(), L.stream()), 'pcs_mul')
    return out


def rel_sums(old, new, out):
    """out[0], out[1] = sum (old - new)^2, sum old^2 (fp64, fixed order) into a device slice."""
    lib = L.gpu()
    L.check(lib.pcs_rel_sums(L.dtcode(old), L.ptr(old), L.ptr(new), old.numel(), L.ptr(out), L.ptr(_ws(old)),
                             L.stream()), 'pcs_rel_sums')
    return out


def sub2(x, y, w, a, b):
    """(x - a*y) - b*w  (proxalgs.py:348)."""
    lib = L.gpu()
    out = torch.empty_like(x)
    L.check(lib.pcs_sub2(L.dtcode(x), L.ptr(x), L.ptr(y), L.ptr(w), L.ptr(out), x.numel(), float(a), float(b),
                         L.stream()), 'pcs_sub2')
    return out


def _ws(t):
    key = (t.device, 'reduce')
    ws = _ws_cache.get(key)
    if ws is None:
        lib = L.gpu()
        ws = torch.empty(int(lib.pcs_reduce_ws_bytes()) // 8 + 8, dtype=torch.float64, device=t.device)
        _ws_cache[key] = ws
    return ws


def reduce_dev(kind, x, y=None, out=None):
    """Deterministic fp64 reduction into a 1-element device tensor.
    kind: 0 sum x^2, 1 sum |x|, 2 sum (x-y)^2, 3 sum x*y."""
    lib = L.gpu()
    out = torch.empty(1, dtype=torch.float64, device=x.device) if out is None else out
    L.check(lib.pcs_reduce(L.dtcode(x), int(kind), L.ptr(x), L.ptr(y), x.numel(), L.ptr(out), L.ptr(_ws(x)),
                           L.stream()), 'pcs_reduce')
    return out


def apgd_step(x, g, aux, tau, a, gkind, lam=1.0, seg=(0.0, 1.0), sums=None):
    """Fused APGD update (``pcs_apgd_step``): returns (x', x_t, sums) with sums[0..1] =
    ||x - x'||^2, ||x||^2 on the device."""
    lib = L.gpu()
    xn, auxn = torch.empty_like(x), torch.empty_like(x)
    sums = torch.empty(2, dtype=torch.float64, device=x.device) if sums is None else sums
    L.check(lib.pcs_apgd_step(L.dtcode(x), L.ptr(x), L.ptr(g), L.ptr(aux), L.ptr(xn), L.ptr(auxn), x.numel(),
                              float(tau), float(a), int(gkind), float(lam), float(seg[0]), float(seg[1]), L.ptr(sums),
                              L.ptr(_ws(x)), L.stream()), 'pcs_apgd_step')
    return xn, auxn, sums


def sumsq(x):
    return float(reduce_dev(0, x).item())


def norm(x):
    return float(np.sqrt(sumsq(x)))


# ---------------------------------------------------------------- prox

def prox_l1(x, tau):
    lib = L.gpu()
    out = torch.empty_like(x)
    L.check(lib.pcs_prox_l1(L.dtcode(x), L.ptr(x), L.ptr(out), x.numel(), float(tau), L.stream()), 'pcs_prox_l1')
    return out


def fenchel_l1(w, sigma, lam):
    lib = L.gpu()
    out = torch.empty_like(w)
    L.check(lib.pcs_fenchel_l1(L.dtcode(w), L.ptr(w), L.ptr(out), w.numel(), float(sigma), float(lam), L.stream()),
            'pcs_fenchel_l1')
    return out


def prox_l21_pixel(x, tau, d):
    lib = L.gpu()
    out = torch.empty_like(x)
    L.check(lib.pcs_prox_l21_pixel(L.dtcode(x), L.ptr(x), L.ptr(out), x.numel() // d, int(d), float(tau),
                                   L.stream()), 'pcs_prox_l21_pixel')
    return out


def fenchel_l21_pixel(w, sigma, lam, d):
    lib = L.gpu()
    out = torch.empty_like(w)
    L.check(lib.pcs_fenchel_l21_pixel(L.dtcode(w), L.ptr(w), L.ptr(out), w.numel() // d, int(d), float(sigma),
                                      float(lam), L.stream()), 'pcs_fenchel_l21_pixel')
    return out


def prox_l21_labels(x, tau, gid, ngroups):
    lib = L.gpu()
    out = torch.empty_like(x)
    ws = torch.empty(int(ngroups), dtype=torch.float64, device=x.device)
    L.check(lib.pcs_prox_l21_labels(L.dtcode(x), L.ptr(x), L.ptr(out), x.numel(), L.ptr(gid), int(ngroups),
                                    float(tau), L.ptr(ws), L.stream()), 'pcs_prox_l21_labels')
    return out


def prox_l21_groups(x, tau, gid, ngroups, order, off, maxlen):
    """L21Norm.prox over general labels with deterministic group sums (pcs_prox_l21_groups)."""
    lib = L.gpu()
    out = torch.empty_like(x)
    ws = torch.empty(int(ngroups), dtype=torch.float64, device=x.device)
    L.check(lib.pcs_prox_l21_groups(L.dtcode(x), L.ptr(x), L.ptr(out), x.numel(), L.ptr(gid), int(ngroups),
                                    L.ptr(order), L.ptr(off), int(maxlen), float(tau), L.ptr(ws), L.stream()),
            'pcs_prox_l21_groups')
    return out


def prox_l2(x, tau):
    lib = L.gpu()
    ss = reduce_dev(0, x)
    out = torch.empty_like(x)
    L.check(lib.pcs_prox_l2(L.dtcode(x), L.ptr(x), L.ptr(out), x.numel(), float(tau), L.ptr(ss), L.stream()),
            'pcs_prox_l2')
    return out


def prox_sql2(x, tau):
    lib = L.gpu()
    out = torch.empty_like(x)
    L.check(lib.pcs_prox_sql2(L.dtcode(x), L.ptr(x), L.ptr(out), x.numel(), float(tau), L.stream()),
            'pcs_prox_sql2')
    return out


def proj_nonneg(x):
    lib = L.gpu()
    out = torch.empty_like(x)
    L.check(lib.pcs_proj_nonneg(L.dtcode(x), L.ptr(x), L.ptr(out), x.numel(), L.stream()), 'pcs_proj_nonneg')
    return out


def proj_segment(x, a, b):
    lib = L.gpu()
    out = torch.empty_like(x)
    L.check(lib.pcs_proj_segment(L.dtcode(x), L.ptr(x), L.ptr(out), x.numel(), float(a), float(b), L.stream()),
            'pcs_proj_segment')
    return out


# ---------------------------------------------------------------- operators

def grad_fwd(x, dims, steps, kind, edge):
    lib = L.gpu()
    out = torch.empty(len(dims) * x.numel(), dtype=x.dtype, device=x.device)
    L.check(lib.pcs_grad_fwd(L.dtcode(x), L.ptr(x), L.ptr(out), len(dims), L.i64s(dims), L.dbls(steps),
                             L.KINDS[kind], int(bool(edge)), L.stream()), 'pcs_grad_fwd')
    return out


def grad_adj(z, dims, steps, kind, edge):
    lib = L.gpu()
    out = torch.empty(z.numel() // len(dims), dtype=z.dtype, device=z.device)
    L.check(lib.pcs_grad_adj(L.dtcode(z), L.ptr(z), L.ptr(out), len(dims), L.i64s(dims), L.dbls(steps),
                             L.KINDS[kind], int(bool(edge)), L.stream()), 'pcs_grad_adj')
    return out


def deriv1(x, dims, axis, step, kind, edge, adjoint=False):
    lib = L.gpu()
    out = torch.empty_like(x)
    fn = lib.pcs_deriv1_adj if adjoint else lib.pcs_deriv1_fwd
    L.check(fn(L.dtcode(x), L.ptr(x), L.ptr(out), len(dims), L.i64s(dims), int(axis), float(step), L.KINDS[kind],
               int(bool(edge)), L.stream()), 'pcs_deriv1')
    return out


def deriv2(x, dims, axis, step, edge, adjoint=False):
    lib = L.gpu()
    out = torch.empty_like(x)
    fn = lib.pcs_deriv2_adj if adjoint else lib.pcs_deriv2_fwd
    L.check(fn(L.dtcode(x), L.ptr(x), L.ptr(out), len(dims), L.i64s(dims), int(axis), float(step), int(bool(edge)),
               L.stream()), 'pcs_deriv2')
    return out


def gather(x, idx):
    """x[idx] (idx: int32 device tensor)."""
    lib = L.gpu()
    out = torch.empty(idx.numel(), dtype=x.dtype, device=x.device)
    L.check(lib.pcs_gather(L.dtcode(x), L.ptr(x), L.ptr(idx), L.ptr(out), idx.numel(), L.stream()), 'pcs_gather')
    return out


def gather_or_zero(y, inv):
    """out[p] = y[inv[p]] if inv[p] >= 0 else 0 (inv: int32 device tensor)."""
    lib = L.gpu()
    out = torch.empty(inv.numel(), dtype=y.dtype, device=y.device)
    L.check(lib.pcs_gather_or_zero(L.dtcode(y), L.ptr(y), L.ptr(inv), L.ptr(out), inv.numel(), L.stream()),
            'pcs_gather_or_zero')
    return out


def lap(x, dims, weights, steps, edge, adjoint=False):
    lib = L.gpu()
    out = torch.empty_like(x)
    fn = lib.pcs_lap_adj if adjoint else lib.pcs_lap_fwd
    L.check(fn(L.dtcode(x), L.ptr(x), L.ptr(out), L.i64s(dims), L.dbls(weights), L.dbls(steps), int(bool(edge)),
               L.stream()), 'pcs_lap')
    return out


def conv2d(x, dims, psf_dev, kh, kw, off0, off1, b=None, beta=0.0):
    lib = L.gpu()
    out = torch.empty_like(x)
    L.check(lib.pcs_conv2d(L.dtcode(x), L.ptr(x), L.ptr(out), int(dims[0]), int(dims[1]), L.ptr(psf_dev), int(kh),
                           int(kw), int(off0), int(off1), L.ptr(b), float(beta), L.stream()), 'pcs_conv2d')
    return out


def conv2d_plan(psf, off0, off1, adjoint, dtype):
    """Packed correlation window of a PSF for pcs_conv2d_planned (host pack, one device copy):
    returns (tier, device tensor) or None if the PSF is larger than the kernel's tiers."""
    lib = L.load()
    h = np.ascontiguousarray(np.asarray(psf, dtype=np.float64))
    kh, kw = h.shape
    tier = int(lib.pcs_conv2d_plan_tier(kh, kw, int(off0), int(off1)))
    if tier < 0:
        return None
    code = L.PCS_F32 if dtype == torch.float32 else L.PCS_F64
    nbytes = int(lib.pcs_conv2d_plan_bytes(code, kh, kw, int(off0), int(off1)))
    host = np.empty(nbytes // (4 if code == L.PCS_F32 else 8), dtype=np.float32 if code == L.PCS_F32 else np.float64)
    L.check(lib.pcs_conv2d_plan_pack(code, h.ctypes.data_as(L._pdbl), kh, kw, int(off0), int(off1), int(adjoint),
                                     host.ctypes.data), 'pcs_conv2d_plan_pack')
    return tier, torch.as_tensor(host).to(device=device())


def conv2d_planned(x, dims, plan, b=None, beta=0.0, out=None):
    lib = L.gpu()
    tier, w = plan
    out = torch.empty_like(x) if out is None else out
    L.check(lib.pcs_conv2d_planned(L.dtcode(x), L.ptr(x), L.ptr(out), int(dims[0]), int(dims[1]), L.ptr(w), int(tier),
                                   L.ptr(b), float(beta), L.stream()), 'pcs_conv2d_planned')
    return out


class FFTConv2D:
    """An FFT-domain Convolve2D plan (pcs_fftconv2d_*: rocFFT R2C / C2R on the zero-padded grid,
    PSF spectrum formed once) for one (dtype, image shape, PSF); freed with the object."""

    def __init__(self, psf, dims, off0, off1, dtype):
        lib = L.gpu()
        self._lib = lib
        h = np.ascontiguousarray(np.asarray(psf, dtype=np.float64))
        kh, kw = h.shape
        code = L.PCS_F32 if dtype == torch.float32 else L.PCS_F64
        handle = ctypes.c_void_p()
        L.check(lib.pcs_fftconv2d_create(code, int(dims[0]), int(dims[1]), h.ctypes.data_as(L._pdbl), kh, kw,
                                         int(off0), int(off1), ctypes.byref(handle)), 'pcs_fftconv2d_create')
        self.handle, self.dims, self.dtype = handle, tuple(dims), dtype

    def apply(self, x, adjoint=False, b=None, beta=0.0, out=None):
        """Conv x (+ beta b) or Conv^T x into a new (or the given) device vector."""
        if x.dtype != self.dtype:
            raise ValueError('FFTConv2D: dtype mismatch')
        out = torch.empty_like(x) if out is None else out
        n = self.dims[0] * self.dims[1]
        dev = torch.device('cuda', torch.cuda.current_device())
        for name, t in (('x', x), ('out', out), ('b', b)):
            if t is None:
                continue
            # the kernels read / write n0*n1 elements through raw pointers: validate before the call
            if not isinstance(t, torch.Tensor) or t.dtype != self.dtype or t.numel() != n or not t.is_contiguous() \
                    or t.device != dev:
                raise ValueError(f'FFTConv2D.apply: {name} must be a contiguous {self.dtype} tensor of {n} elements '
                                 f'on {dev} (got {getattr(t, "dtype", type(t))}, '
                                 f'{getattr(t, "numel", lambda: "?")()} elements on {getattr(t, "device", "?")})')
        L.check(self._lib.pcs_fftconv2d_apply(self.handle, L.ptr(x), L.ptr(out), int(bool(adjoint)), L.ptr(b),
                                              float(beta), L.stream()), 'pcs_fftconv2d_apply')
        return out

    def __del__(self):
        if getattr(self, 'handle', None):
            self._lib.pcs_fftconv2d_destroy(self.handle)
            self.handle = None


def conv1d(x, dims, axis, taps_dev, k, off):
    lib = L.gpu()
    out = torch.empty_like(x)
    L.check(lib.pcs_conv1d(L.dtcode(x), L.ptr(x), L.ptr(out), len(dims), L.i64s(dims), int(axis), L.ptr(taps_dev),
                           int(k), int(off), L.stream()), 'pcs_conv1d')
    return out


def scalar(x):
    return isinstance(x, Number)

"""Fused, hipGraph-replayed PDS engine for 2-D TV problems (single GPU).

Pattern-matches the problem a user script builds with the reference API
(``F = (1/2)*SquaredL2Loss(dim, data=y) [* Convolve2D]``, ``K = Gradient(shape,
kind='forward')``, ``H = lam * L21Norm(groups=tile(arange(N), 2))`` or ``lam * L1Norm``,
``G = None / NonNegativeOrthant / Segment``) and runs ``PrimalDualSplitting.iterate``
(``pycsou/opt/proxalgs.py:343-394`` inside ``pycsou/core/solver.py:55-76``) as

    per iteration:  [GRADBUF only: r = h*x - y ; g = h^T r]   (pcs_conv2d_planned x2)
                    pcs_pds2d_step        x, z  ->  x', z', per-block norm partials
                    pcs_pds_reduce_finalize      -> relative improvements, iteration
                                                    counter, device stop flag

captured once into a hipGraph of ``chunk`` iterations (x/z ping-pong between two
buffers) and replayed.  The stop flag implements the reference loop condition on the
device, so a replay after convergence is a sequence of no-op launches and the
iteration count is exactly the reference's.
"""

import ctypes
import os

import numpy as np
import torch

from .. import _lib as L
from .. import _ops as O
from ..core.functional import ProxFuncPostComp
from ..core.map import DiffMapComp, DiffMapShifted
from ..func.base import IndicatorFunctional, NullDifferentiableFunctional, NullProximableFunctional
from ..func.penalty import L1Norm, L21Norm, SquaredL2Norm
from ..linop.base import HomothetyMap
from ..linop.conv import Convolve2DOp
from ..linop.diff import GradientOp, LaplacianOp

# images at least this large launch chunks from C instead of replaying a captured graph
NATIVE_MIN_PIXELS = int(os.environ.get('PCS_NATIVE_MIN_PIXELS', 1 << 20))


HIST_CHUNK = 4096  # iterations of device history allocated at first; doubled as the loop goes on

# deferred finalization (pcs_pds2d_args.fin_partials, csrc/pds_ctrl.hpp): each step launch finalizes the
# previous launch's partials in a workgroup of its own instead of reducing its own at its end.
# PCS_DEFER_FIN=0: diagnostics, the in-launch reduction.
DEFER_FIN = os.environ.get('PCS_DEFER_FIN', '1') != '0'


def grow_hist(hist, ctrl, need_iters, total):
    """Device history with room for `need_iters` iterations (at most `total`): `hist` itself, or a
    copy twice as long with the loop control's length updated (stream-ordered after every
    iteration already enqueued).  A max_iter of 1e9 with accuracy_threshold doing the stopping
    must not allocate 2 * max_iter doubles up front."""
    have = (hist.numel() - 2) // 2
    if need_iters + 1 <= have or have >= total:
        return hist
    cap = min(total, max(2 * have, need_iters + 1))
    new = torch.full((2 * cap + 2,), float('nan'), dtype=torch.float64, device=hist.device)
    new[:hist.numel()].copy_(hist)
    ctrl.view(torch.int32)[5].fill_(int(new.numel()))  # Ctrl.hist_len (csrc/pds_ctrl.hpp)
    return new


def _half_loss_data(F):
    """If F is (1/2) * SquaredL2Norm.shifter(s) return s (the shift = -data), else None."""
    if (isinstance(F, DiffMapComp) and isinstance(F.map1, HomothetyMap) and F.map1.cst == 0.5
            and isinstance(F.map2, DiffMapShifted) and isinstance(F.map2.map, SquaredL2Norm)
            and not np.isscalar(F.map2.shift)):
        return F.map2.shift
    return None


def _match_g(G, spec):
    """G = None / NullProximableFunctional / NonNegativeOrthant / Segment -> spec['gkind'], spec['seg']."""
    if G is None or isinstance(G, NullProximableFunctional):
        spec['gkind'], spec['seg'] = L.PCS_G_NULL, (0.0, 1.0)
    elif isinstance(G, IndicatorFunctional) and G.kind == 'nonneg':
        spec['gkind'], spec['seg'] = L.PCS_G_NONNEG, (0.0, 1.0)
    elif isinstance(G, IndicatorFunctional) and G.kind == 'segment':
        spec['gkind'], spec['seg'] = L.PCS_G_SEGMENT, G.params
    else:
        return False
    return True


def _match_h(H, ncomp, N):
    """H = lam * (L1Norm | L21Norm over the ncomp components of each pixel) -> (hkind, lam) or None."""
    base, lam = H, 1.0
    if isinstance(H, ProxFuncPostComp):
        if H.shift != 0:
            return None
        base, lam = H.prox_func, float(H.scale)
    if ncomp > 1 and isinstance(base, L21Norm) and base.pixel_d == ncomp and base.dim == ncomp * N:
        return L.PCS_H_L21, lam
    if isinstance(base, L1Norm) and base.dim == ncomp * N:
        return L.PCS_H_L1, lam
    return None


def nmarch_taps(t0, t1, half, dtype=np.float32):
    """The N = Conv^T Conv tables of the normal-operator march kernel (pds_nmarch.hpp) for a
    separable PSF with centred taps t0 (axis 0) and t1 (axis 1) of half width `half`, padded to
    the tier H (3 or 7): (Conv v)[i] = sum_d c[d] v[i - d], c[d] = t[H + d].  Away from the
    edges N is the autocorrelation a[e] = sum_m c[m] c[m + e] (window taps a[|q - 2H|],
    q = 0..4H); on the H samples nearest each edge the zero boundary removes the terms of the
    samples outside the image: N[j, k] = a[j - k] - E[j][k], E[j][k] = sum_{i < 0} c[i - j] c[i - k]
    (left / top, j, k < H) and the mirror sum over i >= n on the right / bottom.  Computed in fp64,
    returned in the layout the kernels read (64 + 32 H values) as `dtype` (the fp32 march: float32; the
    fp64 march, pds_nm64.hip: float64)."""
    H = 3 if half <= 3 else 7
    out = np.zeros(64 + 32 * H)

    def taps(t):
        w = np.zeros(2 * H + 1)
        w[H - half:H + half + 1] = np.asarray(t, dtype=np.float64)
        return lambda d: w[H + d] if -H <= d <= H else 0.0

    def window(c):
        a = [sum(c(m) * c(m + e) for m in range(-H, H + 1)) for e in range(2 * H + 1)]
        return [a[abs(q - 2 * H)] for q in range(4 * H + 1)]

    def e_lo(c):  # E[j][k], j, k < H: the rows i = -H..-1 above the image
        return [[sum(c(i - j) * c(i - k) for i in range(-H, 0)) for k in range(H)] for j in range(H)]

    def e_hi(c):  # the last H samples, j = n-H+jj, k = n-H+kk, rows i = n..n+H-1 (i - j = H + ii - jj)
        return [[sum(c(H + ii - jj) * c(H + ii - kk) for ii in range(H)) for kk in range(H)] for jj in range(H)]

    c0, c1 = taps(t0), taps(t1)
    out[0:4 * H + 1] = window(c0)
    out[32:32 + 4 * H + 1] = window(c1)
    ev_lo, ev_hi, eh_lo, eh_hi = e_lo(c0), e_hi(c0), e_lo(c1), e_hi(c1)
    base = 64
    for j in range(H):  # E_v rows: [j][k]
        out[base + 8 * j:base + 8 * j + H] = ev_lo[j]
        out[base + 8 * H + 8 * j:base + 8 * H + 8 * j + H] = ev_hi[j]
    for k in range(H):  # E_h transposed: ET[k][c] for the left band, ET[k][i] (column n1-8+i) right
        for cc in range(H):
            out[base + 16 * H + 8 * k + cc] = eh_lo[cc][k]
            out[base + 24 * H + 8 * k + (8 - H) + cc] = eh_hi[cc][k]
    return out.astype(dtype)


def match_stencil2d(F, G, H, K, has_H):
    """Engine spec for the general-stencil fused step (pcs_pds2d_stencil_step): K a 2-D Gradient of
    any kind (pycsou/linop/diff.py:777-882) or a 2-D Laplacian (diff.py:885-957), H = lam * L1 / L21,
    F = 0, (1/2) SquaredL2Loss(y), or (1/2) SquaredL2Loss(y) * Convolve2D (grad F through the
    correlation kernel into a buffer); None otherwise."""
    if not has_H:
        return None
    if isinstance(K, GradientOp) and len(K.dims) == 2:
        kk, ncomp, w = {'forward': L.PCS_K_GRAD_FORWARD, 'backward': L.PCS_K_GRAD_BACKWARD,
                        'centered': L.PCS_K_GRAD_CENTERED}[K.kind], 2, (1.0, 1.0)
    elif isinstance(K, LaplacianOp) and len(K.dims) == 2:
        kk, ncomp, w = L.PCS_K_LAPLACIAN, 1, tuple(K.weights)
    else:
        return None
    shape = tuple(K.dims)
    N = shape[0] * shape[1]
    hm = _match_h(H, ncomp, N)
    if hm is None:
        return None
    spec = {'stencil': True, 'shape': shape, 'steps': tuple(K.steps), 'kkind': kk, 'ncomp': ncomp,
            'weights': w, 'edge': bool(K.edge), 'hkind': hm[0], 'lam': hm[1]}
    if not _match_g(G, spec):
        return None
    if F is None or isinstance(F, NullDifferentiableFunctional):
        spec['fkind'] = L.PCS_F_NULL
        return spec
    s = _half_loss_data(F)
    if s is not None and O.numel(s) == N:
        spec['fkind'], spec['shift'] = L.PCS_F_DENOISE, s
        return spec
    if isinstance(F, DiffMapComp) and isinstance(F.map2, Convolve2DOp) and F.map2.dims == shape:
        s = _half_loss_data(F.map1)
        if s is not None and O.numel(s) == N:
            spec['fkind'], spec['shift'], spec['conv'] = L.PCS_F_GRADBUF, s, F.map2
            return spec
    return None


def match_pds2d(F, G, H, K, has_H):
    """Return an engine spec dict if (F, G, H, K) is a fused-engine problem, else None."""
    if not has_H or not isinstance(K, GradientOp) or len(K.dims) != 2 or K.kind != 'forward':
        return None
    shape = K.dims
    N = shape[0] * shape[1]
    spec = {'shape': shape, 'steps': tuple(K.steps)}
    # H = lam * (L1 | L21 pixel groups)
    base, lam = H, 1.0
    if isinstance(H, ProxFuncPostComp):
        if H.shift != 0:
            return None
        base, lam = H.prox_func, float(H.scale)
    if isinstance(base, L21Norm) and base.pixel_d == 2 and base.dim == 2 * N:
        spec['hkind'] = L.PCS_H_L21
    elif isinstance(base, L1Norm) and base.dim == 2 * N:
        spec['hkind'] = L.PCS_H_L1
    else:
        return None
    spec['lam'] = lam
    if not _match_g(G, spec):
        return None
    # F
    if F is None or isinstance(F, NullDifferentiableFunctional):
        spec['fkind'] = L.PCS_F_NULL
        return spec
    s = _half_loss_data(F)
    if s is not None and O.numel(s) == N:
        spec['fkind'], spec['shift'] = L.PCS_F_DENOISE, s
        return spec
    if isinstance(F, DiffMapComp) and isinstance(F.map2, Convolve2DOp) and F.map2.dims == shape:
        s = _half_loss_data(F.map1)
        if s is not None and O.numel(s) == N:
            spec['fkind'], spec['shift'], spec['conv'] = L.PCS_F_SEPCONV, s, F.map2
            return spec
    return None


class PDS2DEngine:
    """Device state + captured loop for one fused 2-D PDS problem."""

    def __init__(self, spec, dtype, tau, sigma, rho, x0, z0, chunk=32, use_graph=True):
        self.lib = L.gpu()
        self.spec = spec
        self.dtype = dtype
        n0, n1 = spec['shape']
        self.N = n0 * n1
        self.X = [x0.to(dtype).clone(), torch.empty(self.N, dtype=dtype, device=x0.device)]
        self.Z = [z0.to(dtype).clone(), torch.empty(2 * self.N, dtype=dtype, device=x0.device)]
        dev = self.X[0].device
        self.chunk = max(2, chunk + (chunk % 2))
        self.use_graph = use_graph
        a = L.PdsArgs()
        a.dtype = L.PCS_F32 if dtype == torch.float32 else L.PCS_F64
        a.hkind, a.gkind = spec['hkind'], spec['gkind']
        a.n0, a.n1, a.row0, a.rows = n0, n1, 0, n0
        a.halo_x = a.halo_z = a.halo_y = 0
        a.tau, a.sigma, a.rho, a.lam = float(tau), float(sigma), float(rho), spec['lam']
        a.step0, a.step1 = spec['steps']
        a.seg_a, a.seg_b = spec['seg']
        self.keep = []
        fk = spec['fkind']
        self.conv = None
        if fk in (L.PCS_F_DENOISE, L.PCS_F_SEPCONV):
            # y = -shift (exact), so x + shift == x - y bit for bit
            self.y = -O.to_dev(spec['shift'], dtype)
            a.y = self.y.data_ptr()
        if fk == L.PCS_F_SEPCONV:
            conv = spec['conv']
            sep = conv.separable(rtol=2e-7 if dtype == torch.float32 else 1e-13)
            if sep is not None:
                t0, t1, half = sep
                self.taps = [torch.as_tensor(t0).to(device=dev, dtype=dtype),
                             torch.as_tensor(t1).to(device=dev, dtype=dtype)]
                a.taps0, a.taps1 = self.taps[0].data_ptr(), self.taps[1].data_ptr()
                a.half = half
                # PCS_NMARCH=0: diagnostics, the four-pass march kernel (grad F = Conv^T (Conv x - y))
                if dtype == torch.float32 and half <= 7 and os.environ.get('PCS_NMARCH', '1') != '0':
                    # normal-operator march kernel: grad F = N x - Conv^T y (pds_nmarch.hpp),
                    # Conv^T y formed once here in fp64
                    self.ntaps = torch.as_tensor(nmarch_taps(t0, t1, half)).to(dev)
                    self.cty = conv._adj(-O.to_dev(spec['shift'], torch.float64)).to(dtype).contiguous()
                    a.cty, a.ntaps = self.cty.data_ptr(), self.ntaps.data_ptr()
            else:
                fk = L.PCS_F_GRADBUF
                self.conv = conv
                # device PSF copies / packed correlation plans / the FFT plan exist before capture
                conv._h.get(dtype), conv._hf.get(dtype)
                self.plans = (conv.plan(dtype, False), conv.plan(dtype, True))
                if self.plans[0] is None or self.plans[1] is None:
                    conv.fft(dtype)
                self.R = torch.empty(self.N, dtype=dtype, device=dev)
                self.Gb = torch.empty(self.N, dtype=dtype, device=dev)
                a.gbuf = self.Gb.data_ptr()
        a.fkind = fk
        self.fkind = fk
        self.args = a
        self.nblocks = int(self.lib.pcs_pds2d_nblocks(ctypes.byref(a)))
        self._alloc_partials(a, dev)
        self.ctrl = torch.zeros(int(self.lib.pcs_ctrl_bytes()) // 8, dtype=torch.float64, device=dev)
        a.ctrl = self.ctrl.data_ptr()
        # in-kernel reduce + finalize (one launch per iteration); counters must start at 0
        self.fused_finalize = True
        self.ws = torch.zeros(int(self.lib.pcs_pds2d_ws_bytes(ctypes.byref(a))) // 8 + 2, dtype=torch.float64,
                              device=dev)
        a.ws = self.ws.data_ptr()
        self.graph = None
        self.hist = None
        self.ctrl_host = torch.zeros(2, dtype=torch.int32).pin_memory()
        # large images: each chunk is launched back to back from C (pcs_pds2d_run) -- per-launch
        # host cost is far below the step, and back-to-back launches measured faster than
        # replaying a captured graph of the same launches; small images keep the graph
        self.native = fk != L.PCS_F_GRADBUF and self.N >= NATIVE_MIN_PIXELS

    def _alloc_partials(self, a, dev):
        """[nblocks][4] partials; with deferred finalization two such arrays, swapped with the
        iterate parity (the launch of parity p writes array p and finalizes array 1 - p)."""
        self.defer = DEFER_FIN and isinstance(a, L.PdsArgs)
        nb4 = self.nblocks * 4
        self.partials = torch.empty((2 if self.defer else 1) * nb4, dtype=torch.float64, device=dev)
        self.part_halves = [self.partials[:nb4], self.partials[nb4:]] if self.defer else [self.partials]
        a.partials = self.partials.data_ptr()
        if self.defer:
            a.fin_partials = self.part_halves[1].data_ptr()

    def _bind(self, a, p):
        """Point the step's iterate buffers at parity p (reads buffers p, writes 1 - p)."""
        a.x, a.xn = self.X[p].data_ptr(), self.X[1 - p].data_ptr()
        a.z, a.zn = self.Z[p].data_ptr(), self.Z[1 - p].data_ptr()
        if getattr(self, 'defer', False):
            a.partials, a.fin_partials = self.part_halves[p].data_ptr(), self.part_halves[1 - p].data_ptr()

    def _flush(self, next_p, hist):
        """Deferred finalization: finalize the last launch's partials (parity 1 - next_p) if they
        are pending (pcs_pds_finalize_pending; a no-op when the loop has stopped)."""
        if getattr(self, 'defer', False):
            L.check(self.lib.pcs_pds_finalize_pending(L.ptr(self.part_halves[1 - next_p]), self.nblocks,
                                                      L.ptr(self.ctrl), L.ptr(hist), L.stream()),
                    'pcs_pds_finalize_pending')

    # the fused step / the chunk of n steps launched back to back from C, on self.args
    def _step_call(self, st):
        L.check(self.lib.pcs_pds2d_step(ctypes.byref(self.args), st), 'pcs_pds2d_step')

    def _run_call(self, n):
        L.check(self.lib.pcs_pds2d_run(ctypes.byref(self.args), int(n), L.stream()), 'pcs_pds2d_run')

    # one iteration with parity p (reads buffers p, writes 1-p)
    def _iteration(self, p, hist):
        a, lib, st = self.args, self.lib, L.stream()
        if self.fkind == L.PCS_F_GRADBUF:
            self._grad_conv(p, st)
        self._bind(a, p)
        a.hist = hist.data_ptr() if self.fused_finalize else None
        self._step_call(st)
        if not self.fused_finalize:
            L.check(lib.pcs_pds_reduce_finalize(L.ptr(self.partials), self.nblocks, L.ptr(self.ctrl), L.ptr(hist),
                                                st), 'pcs_pds_reduce_finalize')

    def _grad_conv(self, p, st):
        """GRADBUF: r = h*x - y (residual fused into the forward pass), g = h^T r -- the
        packed-plan correlation kernel (pcs_conv2d_planned) when the PSF fits its tiers."""
        c, a, lib = self.conv, self.args, self.lib
        fwd, adj = self.plans
        n0, n1 = c.dims
        if fwd is not None and adj is not None:
            L.check(lib.pcs_conv2d_planned(a.dtype, L.ptr(self.X[p]), L.ptr(self.R), n0, n1, L.ptr(fwd[1]), fwd[0],
                                           L.ptr(self.y), -1.0, st), 'pcs_conv2d_planned')
            L.check(lib.pcs_conv2d_planned(a.dtype, L.ptr(self.R), L.ptr(self.Gb), n0, n1, L.ptr(adj[1]), adj[0],
                                           None, 0.0, st), 'pcs_conv2d_planned')
            return
        # wider PSFs: the FFT-domain plan (rocFFT; cost independent of the PSF size)
        f = c.fft(self.dtype)
        f.apply(self.X[p], b=self.y, beta=-1.0, out=self.R)
        f.apply(self.R, adjoint=True, out=self.Gb)

    def _chunk(self, hist):
        for i in range(self.chunk):
            self._iteration(i % 2, hist)

    def _chunk_native(self, hist):
        a = self.args
        self._bind(a, 0)
        a.hist = hist.data_ptr()
        self._run_call(self.chunk)

    # ---- fixed-count loop for benchmarking (bench.py): no early stop, optional per-step events
    def prepare_fixed(self, total_iters, chunk):
        """Device state for `total_iters` iterations that never stop early, captured in
        graphs of `chunk` (even) iterations."""
        self.chunk = chunk
        self._fixed_p = 0
        hist_len = 2 * (total_iters + 1) + 2
        self.hist = torch.empty(hist_len, dtype=torch.float64, device=self.X[0].device)
        L.check(self.lib.pcs_ctrl_init2(L.ptr(self.ctrl), int(total_iters), int(total_iters), -1.0, 1, hist_len,
                                        L.stream()), 'pcs_ctrl_init2')
        torch.cuda.synchronize()
        if not self.native:
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self._chunk(self.hist)
            torch.cuda.synchronize()

    def replay(self):
        if self.native:
            self._chunk_native(self.hist)
        else:
            self.graph.replay()

    def advance_fixed(self, n):
        """Enqueue exactly n iterations of a prepare_fixed() loop, continuing from the buffer
        parity the previous call left (odd counts allowed): native images as one
        pcs_pds2d_run of n launches, graph images as whole captured chunks while the parity
        allows plus eager single iterations."""
        p = getattr(self, '_fixed_p', 0)
        if self.native:
            a = self.args
            self._bind(a, p)
            a.hist = self.hist.data_ptr()
            self._run_call(int(n))
            self._fixed_p = p ^ (int(n) & 1)
            self._flush(self._fixed_p, self.hist)
            return
        while n >= self.chunk and p == 0:
            self.graph.replay()
            n -= self.chunk
        for _ in range(n):
            self._iteration(p, self.hist)
            p ^= 1
        self._fixed_p = p
        self._flush(p, self.hist)

    def time_iteration_kernels(self, n):
        """Median duration (ms) of each kernel of an iteration over n eager iterations, HIP
        events on the launching stream around every launch: {'step': ...} and, for a
        non-separable PSF, {'conv_fwd': ..., 'conv_adj': ...}.  (Median: a single launch
        delayed by an unrelated host or driver event does not move it.)"""
        a, lib = self.args, self.lib
        st = torch.cuda.current_stream()
        n = min(n, (self.hist.numel() - 2) // 2 - 1)
        L.check(lib.pcs_ctrl_init2(L.ptr(self.ctrl), n + 1, n + 1, -1.0, 1, int(self.hist.numel()), L.stream()),
                'pcs_ctrl_init2')
        names = ['conv_fwd', 'conv_adj', 'step'] if self.fkind == L.PCS_F_GRADBUF else ['step']
        ev = {k: [] for k in names}

        def timed(name, fn):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            fn()
            e1.record(st)
            ev[name].append((e0, e1))
        for i in range(n):
            p = i % 2
            if self.fkind == L.PCS_F_GRADBUF and (self.plans[0] is None or self.plans[1] is None):
                # PSF wider than the direct tiers: the FFT-domain plan's two passes
                f = self.conv.fft(self.dtype)
                timed('conv_fwd', lambda: f.apply(self.X[p], b=self.y, beta=-1.0, out=self.R))
                timed('conv_adj', lambda: f.apply(self.R, adjoint=True, out=self.Gb))
            elif self.fkind == L.PCS_F_GRADBUF:
                fwd, adj = self.plans
                n0, n1 = self.conv.dims
                timed('conv_fwd', lambda: L.check(lib.pcs_conv2d_planned(
                    a.dtype, L.ptr(self.X[p]), L.ptr(self.R), n0, n1, L.ptr(fwd[1]), fwd[0], L.ptr(self.y), -1.0,
                    L.stream()), 'pcs_conv2d_planned'))
                timed('conv_adj', lambda: L.check(lib.pcs_conv2d_planned(
                    a.dtype, L.ptr(self.R), L.ptr(self.Gb), n0, n1, L.ptr(adj[1]), adj[0], None, 0.0, L.stream()),
                    'pcs_conv2d_planned'))
            self._bind(a, p)
            a.hist = self.hist.data_ptr()
            timed('step', lambda: self._step_call(L.stream()))
        self._flush(n % 2, self.hist)
        torch.cuda.synchronize()
        return {k: float(np.median([s.elapsed_time(e) for s, e in v])) for k, v in ev.items()}

    def time_step_kernel(self, n, stream=None):
        """Average duration (ms) of the fused step kernel over `n` eager launches, measured
        with HIP events on the stream the kernel runs on."""
        a = self.args
        st = torch.cuda.current_stream() if stream is None else stream
        # fresh loop state that runs all n launches (the in-kernel reduce + finalize is timed too)
        n = min(n, (self.hist.numel() - 2) // 2 - 1)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        L.check(self.lib.pcs_ctrl_init2(L.ptr(self.ctrl), n + 1, n + 1, -1.0, 1, int(self.hist.numel()), L.stream()),
                'pcs_ctrl_init2')
        ctrl, hist = a.ctrl, a.hist
        a.hist = self.hist.data_ptr()
        if not self.fused_finalize:
            a.hist = None
        for i in range(n):
            p = i % 2
            self._bind(a, p)
            evs[i][0].record(st)
            self._step_call(L.stream())
            evs[i][1].record(st)
        self._flush(n % 2, self.hist)
        torch.cuda.synchronize()
        a.ctrl, a.hist = ctrl, hist
        return float(np.mean([s.elapsed_time(e) for s, e in evs]))

    def run(self, max_iter, min_iter, accuracy_threshold, has_dual=True):
        max_iter, min_iter = int(max_iter), int(min_iter)
        total = max(min_iter, max_iter) + 1
        hist_len = 2 * min(total, max(HIST_CHUNK, 2 * self.chunk)) + 2
        if self.hist is None or self.hist.numel() < hist_len:
            # the history buffer is captured by pointer: (re)capture when it grows
            self.hist = torch.empty(hist_len, dtype=torch.float64, device=self.X[0].device)
            self.graph = None
        self.hist.fill_(float('nan'))
        L.check(self.lib.pcs_ctrl_init2(L.ptr(self.ctrl), min_iter, max_iter, float(accuracy_threshold),
                                        int(has_dual), int(self.hist.numel()), L.stream()), 'pcs_ctrl_init2')
        n_chunks = -(-total // self.chunk)
        if self.use_graph or self.native:
            pending = []
            for k in range(n_chunks):
                grown = grow_hist(self.hist, self.ctrl, (k + 1) * self.chunk + 1, total)
                if grown is not self.hist:
                    self.hist, self.graph = grown, None
                hist = self.hist
                if self.graph is None and not self.native:
                    torch.cuda.synchronize()
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        self._chunk(hist)
                    self.graph = g
                if self.native:
                    self._chunk_native(hist)
                else:
                    self.graph.replay()
                ev = torch.cuda.Event()
                self.ctrl_host.copy_(self.ctrl.view(torch.int32)[:2], non_blocking=True)
                ev.record()
                pending.append(ev)
                if len(pending) >= 2:
                    pending.pop(0).synchronize()
                    if int(self.ctrl_host[1]) != 0:
                        break
        else:
            for k in range(n_chunks):
                self.hist = grow_hist(self.hist, self.ctrl, (k + 1) * self.chunk + 1, total)
                self._chunk(self.hist)
                if int(self.ctrl.view(torch.int32)[1].item()) != 0:
                    break
        hist = self.hist
        self._flush(0, hist)  # every chunk is an even number of launches
        torch.cuda.synchronize()
        c = self.ctrl.view(torch.int32)[:2].cpu().numpy()
        n = int(c[0])
        h = hist[:2 * n].cpu().numpy().reshape(n, 2) if n > 0 else np.zeros((0, 2))
        return n, self.X[n % 2], self.Z[n % 2], h


class PDS2DStencilEngine(PDS2DEngine):
    """Device state + loop of the general-stencil fused step (pcs_pds2d_stencil_step): the same
    loop machinery as PDS2DEngine (device stop flag, chunks launched from C for large images,
    hipGraph replay otherwise, GRADBUF convolutions before the step), another step kernel."""

    def __init__(self, spec, dtype, tau, sigma, rho, x0, z0, chunk=32, use_graph=True):
        self.lib = L.gpu()
        self.spec = spec
        self.dtype = dtype
        n0, n1 = spec['shape']
        self.N = N = n0 * n1
        nc = spec['ncomp']
        dev = x0.device
        self.X = [x0.to(dtype).clone(), torch.empty(N, dtype=dtype, device=dev)]
        self.Z = [z0.to(dtype).clone(), torch.empty(nc * N, dtype=dtype, device=dev)]
        self.chunk = max(2, chunk + (chunk % 2))
        self.use_graph = use_graph
        fk = spec['fkind']
        self.conv = None
        if fk in (L.PCS_F_DENOISE, L.PCS_F_GRADBUF):
            self.y = -O.to_dev(spec['shift'], dtype)  # y = -shift exactly
        if fk == L.PCS_F_GRADBUF:
            conv = self.conv = spec['conv']
            conv._h.get(dtype), conv._hf.get(dtype)
            self.plans = (conv.plan(dtype, False), conv.plan(dtype, True))
            if self.plans[0] is None or self.plans[1] is None:
                conv.fft(dtype)  # created before any capture
            self.R = torch.empty(N, dtype=dtype, device=dev)
            self.Gb = torch.empty(N, dtype=dtype, device=dev)
        gsrc = None if fk == L.PCS_F_NULL else (self.Gb if fk == L.PCS_F_GRADBUF else self.y)
        self.fkind = fk
        # images the general-stencil row-marching kernel covers (pds_smarch.hpp: 64-column strips,
        # 4-column groups; fp32 and fp64, every K kind in fp64) run through pcs_pds2d_step with K in
        # the args; the rest through the tile kernel (pcs_pds2d_stencil_step).  PCS_STENCIL_MARCH=0:
        # always the tile kernel.
        self.march = False
        a = None
        f64 = dtype == torch.float64
        if dtype in (torch.float32, torch.float64) and os.environ.get('PCS_STENCIL_MARCH', '1') != '0':
            a = L.PdsArgs()
            a.dtype, a.fkind, a.hkind, a.gkind = L.PCS_F64 if f64 else L.PCS_F32, fk, spec['hkind'], spec['gkind']
            a.n0, a.n1, a.row0, a.rows = n0, n1, 0, n0
            a.kkind, a.edge = spec['kkind'], int(spec['edge'])
            a.w0, a.w1 = spec['weights']
            a.tau, a.sigma, a.rho, a.lam = float(tau), float(sigma), float(rho), spec['lam']
            a.step0, a.step1 = spec['steps']
            a.seg_a, a.seg_b = spec['seg']
            a.x, a.xn = self.X[0].data_ptr(), self.X[1].data_ptr()
            a.z, a.zn = self.Z[0].data_ptr(), self.Z[1].data_ptr()
            a.partials = a.x  # placeholder for the support query (never written)
            if fk == L.PCS_F_DENOISE:
                a.y = gsrc.data_ptr()
            elif fk == L.PCS_F_GRADBUF:
                a.gbuf = gsrc.data_ptr()
                # separable PSF: grad F = N x - Conv^T y (the in-plane normal-operator kernel into the
                # gradient buffer, then the march step), Conv^T y formed once here in fp64
                sep = self.conv.separable(rtol=1e-13 if f64 else 2e-7)
                if sep is not None and sep[2] <= 7:
                    t0, t1, half = sep
                    self.taps = [torch.as_tensor(t).to(device=dev, dtype=dtype) for t in (t0, t1)]
                    self.cty = self.conv._adj(-O.to_dev(spec['shift'], torch.float64)).to(dtype).contiguous()
                    a.fkind, a.half, a.y = L.PCS_F_SEPCONV, half, self.y.data_ptr()
                    a.taps0, a.taps1 = self.taps[0].data_ptr(), self.taps[1].data_ptr()
                    a.cty = self.cty.data_ptr()
                    # the N tables: the fused normal-operator march (one launch: pds_nmarch.hpp for
                    # backward / centred K in fp32, pds_nm64.hip for every Gradient K in fp64) when the
                    # library takes the problem -- supported with no gradient buffer; otherwise the
                    # two-launch form (N x by the in-plane normal-operator kernel, then the march step)
                    self.ntaps = torch.as_tensor(nmarch_taps(t0, t1, half, np.float64 if f64 else np.float32)).to(dev)
                    a.ntaps = self.ntaps.data_ptr()
                    a.gbuf = None
                    self.nm_fused = self.lib.pcs_pds2d_path(ctypes.byref(a)) in L.PCS_PATH_FUSED_NORMAL
                    if not self.nm_fused:
                        a.ntaps = None
                    a.gbuf = gsrc.data_ptr()
                    if self.lib.pcs_pds2d_supported(ctypes.byref(a)) != 1:
                        a.fkind, a.cty, a.ntaps = fk, None, None
                        self.nm_fused = False
                    else:
                        fk = self.fkind = L.PCS_F_SEPCONV
            if self.lib.pcs_pds2d_supported(ctypes.byref(a)) == 1:
                self.march = True
            else:
                a = None
                fk = self.fkind = spec['fkind']
        if a is None:
            a = L.StencilArgs()
            a.dtype = L.PCS_F32 if dtype == torch.float32 else L.PCS_F64
            a.kkind, a.hkind, a.gkind, a.edge = spec['kkind'], spec['hkind'], spec['gkind'], int(spec['edge'])
            a.n0, a.n1 = n0, n1
            a.tau, a.sigma, a.rho, a.lam = float(tau), float(sigma), float(rho), spec['lam']
            a.step0, a.step1 = spec['steps']
            a.w0, a.w1 = spec['weights']
            a.seg_a, a.seg_b = spec['seg']
            a.fkind = fk
            if gsrc is not None:
                a.g = gsrc.data_ptr()
        self.args = a
        nb_fn = self.lib.pcs_pds2d_nblocks if self.march else self.lib.pcs_pds2d_stencil_nblocks
        ws_fn = self.lib.pcs_pds2d_ws_bytes if self.march else self.lib.pcs_pds2d_stencil_ws_bytes
        self.nblocks = int(nb_fn(ctypes.byref(a)))
        self._alloc_partials(a, dev)
        self.ctrl = torch.zeros(int(self.lib.pcs_ctrl_bytes()) // 8, dtype=torch.float64, device=dev)
        a.ctrl = self.ctrl.data_ptr()
        self.fused_finalize = True
        self.ws = torch.zeros(int(ws_fn(ctypes.byref(a))) // 8 + 2, dtype=torch.float64, device=dev)
        a.ws = self.ws.data_ptr()
        self.graph = None
        self.hist = None
        self.ctrl_host = torch.zeros(2, dtype=torch.int32).pin_memory()
        self.native = fk != L.PCS_F_GRADBUF and self.N >= NATIVE_MIN_PIXELS
        self.bar = None

    def time_iteration_kernels(self, n):
        """As PDS2DEngine's; with a separable PSF (SEPCONV here) either the fused normal-operator
        march (one launch, `nm_fused`) or one pcs_pds2d_step call holding two launches (N x into the
        gradient buffer, the step), timed as 'step' together and 'conv_nx' alone."""
        res = PDS2DEngine.time_iteration_kernels(self, n)
        if self.fkind == L.PCS_F_SEPCONV and not getattr(self, 'nm_fused', False):
            a, lib = self.args, self.lib
            ev = []
            for i in range(min(n, 50)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                L.check(lib.pcs_conv2d_sep_ata_planes(a.dtype, L.ptr(self.X[i % 2]), L.ptr(self.Gb), 1, a.n0, a.n1,
                                                      L.ptr(self.taps[0]), 2 * a.half + 1, a.half,
                                                      L.ptr(self.taps[1]), 2 * a.half + 1, a.half, L.stream()),
                        'pcs_conv2d_sep_ata_planes')
                e1.record()
                ev.append((e0, e1))
            torch.cuda.synchronize()
            res['conv_nx'] = float(np.median([s.elapsed_time(e) for s, e in ev]))
        return res

    def _step_call(self, st):
        if self.march:
            return PDS2DEngine._step_call(self, st)
        L.check(self.lib.pcs_pds2d_stencil_step(ctypes.byref(self.args), st), 'pcs_pds2d_stencil_step')

    def _run_call(self, n):
        if self.march:
            return PDS2DEngine._run_call(self, n)
        L.check(self.lib.pcs_pds2d_stencil_run(ctypes.byref(self.args), int(n), L.stream()), 'pcs_pds2d_stencil_run')


def match_masked_stencil2d(F, G, H, K, has_H):
    """Engine spec for the masked data-fidelity problem of the reference notebook (TV-LAD inpainting,
    solved by ChambollePockSplitting, pycsou/opt/proxalgs.py:628-716): F = 0,
    K = LinOpVStack(Masking(mask), K_s) (pycsou/linop/base.py:259-279, linop/sampling.py:125-196),
    H = ProxFuncHStack(L1Loss(dim=m, data=y), lam * L1Norm | lam * L21Norm) (func/base.py:21-89,
    func/loss.py:222-268) with K_s / the second block any problem match_stencil2d takes with F = 0;
    G = None / NonNegativeOrthant / Segment.  Only images the row march covers (n1 % 4 == 0, at
    least two 64-column strips); None otherwise (the generic per-operator path runs it)."""
    from ..core.functional import ProxFuncPreComp
    from ..func.base import ProxFuncHStack
    from ..linop.base import LinOpStack
    from ..linop.sampling import Masking
    if not has_H or not (F is None or isinstance(F, NullDifferentiableFunctional)):
        return None
    if not isinstance(K, LinOpStack) or K.axis != 0 or len(K.linops) != 2 or not isinstance(H, ProxFuncHStack) \
            or len(H.proxfuncs) != 2:
        return None
    M, Ks = K.linops
    h_loss, h_s = H.proxfuncs
    if not isinstance(M, Masking) or not hasattr(M, 'sampling_bool'):
        return None
    if not (isinstance(h_loss, ProxFuncPreComp) and isinstance(h_loss.prox_func, L1Norm)
            and isinstance(h_loss.scale, (int, float)) and h_loss.scale == 1 and not np.isscalar(h_loss.shift)):
        return None
    m = int(M.shape[0])
    if h_loss.dim != m or O.numel(h_loss.shift) != m:
        return None
    spec = match_stencil2d(None, G, h_s, Ks, True)
    if spec is None or spec['fkind'] != L.PCS_F_NULL:
        return None
    n0, n1 = spec['shape']
    if M.shape[1] != n0 * n1 or n1 % 4 or n1 <= 64:
        return None
    # the fused block marks unsampled pixels by a NaN in the expanded data: data that is not finite
    # itself would be read as unsampled there, so it takes the generic path (which propagates it, as
    # the reference's L1Loss prox does)
    sh = h_loss.shift
    finite = bool(torch.isfinite(sh).all().item()) if isinstance(sh, torch.Tensor) else bool(np.isfinite(sh).all())
    if not finite:
        return None
    spec['mask'] = M.sampling_bool
    spec['mask_shift'] = h_loss.shift  # = -y
    spec['m'] = m
    return spec


class PDS2DMaskEngine(PDS2DEngine):
    """The masked data-fidelity problem (match_masked_stencil2d) on the general-stencil row march with
    the masked block inside the step (pcs_pds2d_args.mkind = PCS_M_L1LOSS, pds_smarch.hpp SM_F_MASK):
    one launch per iteration.  The masked dual block z_m is held expanded to the image (ZM, 0 where the
    mask is False) and y expanded with NaN there; the solver's z = [z_m; z_s] is assembled on return."""

    def __init__(self, spec, dtype, tau, sigma, rho, x0, z0, chunk=32, use_graph=True):
        self.lib = L.gpu()
        self.spec = spec
        self.dtype = dtype
        n0, n1 = spec['shape']
        self.N = N = n0 * n1
        nc, m = spec['ncomp'], spec['m']
        dev = x0.device
        self.idx = torch.as_tensor(np.flatnonzero(spec['mask']).astype(np.int64)).to(dev)
        z0 = z0.to(dtype)
        self.X = [x0.to(dtype).clone(), torch.empty(N, dtype=dtype, device=dev)]
        self.Z = [z0[m:].clone(), torch.empty(nc * N, dtype=dtype, device=dev)]
        self.ZM = [torch.zeros(N, dtype=dtype, device=dev), torch.zeros(N, dtype=dtype, device=dev)]
        self.ZM[0][self.idx] = z0[:m]
        self.ym = torch.full((N,), float('nan'), dtype=dtype, device=dev)
        self.ym[self.idx] = -O.to_dev(spec['mask_shift'], dtype)  # y = -shift, exactly
        self.chunk = max(2, chunk + (chunk % 2))
        self.use_graph = use_graph
        self.fkind = L.PCS_F_NULL
        a = L.PdsArgs()
        a.dtype = L.PCS_F64 if dtype == torch.float64 else L.PCS_F32
        a.fkind, a.hkind, a.gkind = L.PCS_F_NULL, spec['hkind'], spec['gkind']
        a.n0, a.n1, a.row0, a.rows = n0, n1, 0, n0
        a.kkind, a.edge = spec['kkind'], int(spec['edge'])
        a.w0, a.w1 = spec['weights']
        a.tau, a.sigma, a.rho, a.lam = float(tau), float(sigma), float(rho), spec['lam']
        a.step0, a.step1 = spec['steps']
        a.seg_a, a.seg_b = spec['seg']
        a.mkind, a.ym = L.PCS_M_L1LOSS, self.ym.data_ptr()
        self.args = a
        self._bind(a, 0)
        a.partials = a.x  # placeholder for the support query (never written)
        if self.lib.pcs_pds2d_supported(ctypes.byref(a)) != 1:
            raise ValueError('masked data-fidelity problem not supported by the fused step')
        self.nblocks = int(self.lib.pcs_pds2d_nblocks(ctypes.byref(a)))
        self._alloc_partials(a, dev)
        self.ctrl = torch.zeros(int(self.lib.pcs_ctrl_bytes()) // 8, dtype=torch.float64, device=dev)
        a.ctrl = self.ctrl.data_ptr()
        self.fused_finalize = True
        self.ws = torch.zeros(int(self.lib.pcs_pds2d_ws_bytes(ctypes.byref(a))) // 8 + 2, dtype=torch.float64,
                              device=dev)
        a.ws = self.ws.data_ptr()
        self.graph = None
        self.hist = None
        self.ctrl_host = torch.zeros(2, dtype=torch.int32).pin_memory()
        self.native = self.N >= NATIVE_MIN_PIXELS
        self.bar = None

    def _bind(self, a, p):
        PDS2DEngine._bind(self, a, p)
        a.zm, a.zmn = self.ZM[p].data_ptr(), self.ZM[1 - p].data_ptr()

    def z_full(self, p):
        """The solver's dual variable [z_m; z_s] of buffer parity p (the reference layout)."""
        return torch.cat([self.ZM[p][self.idx], self.Z[p]])

    def run(self, max_iter, min_iter, accuracy_threshold, has_dual=True):
        n, x, _, h = PDS2DEngine.run(self, max_iter, min_iter, accuracy_threshold, has_dual)
        return n, x, self.z_full(n % 2), h


def engine_class(spec):
    """The engine class of a fused spec (proxalgs and bench.py build engines through this)."""
    from .engine3d import PDS3DEngine
    if spec.get('ndim', 2) == 3:
        return PDS3DEngine
    if 'mask' in spec:
        return PDS2DMaskEngine
    return PDS2DStencilEngine if spec.get('stencil') else PDS2DEngine

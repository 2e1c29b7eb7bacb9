"""Fused PDS engine for 3-D volumes.

Problem family (what a reference script builds for 3-D TV deconvolution / denoising):
``F = (1/2) * SquaredL2Loss(dim, data=y) [* C]`` with ``C`` a composition of
``Convolve1D(size, taps, reshape_dims=shape, axis=k)`` (the reference's only 3-D blur,
``pycsou/linop/conv.py:20-164``), ``K = Gradient(shape, kind=...)`` in 3-D (forward; backward / centred through k_pds3d_gen)
(``pycsou/linop/diff.py:777-882``), ``H = lam * L21Norm(groups=tile(arange(N), 3))`` or
``lam * L1Norm``, ``G = None / NonNegativeOrthant / Segment``.

One iteration of ``PrimalDualSplitting`` (``pycsou/opt/proxalgs.py:343-394``):

    g = C^T (C x - y)          in-plane pcs_conv1d passes, then pcs_conv0_residual_adjoint (the
                               axis-0 conv, the residual (C x) + (-y) and the axis-0 adjoint in
                               one plane-streaming pass), then the in-plane adjoint passes on the
                               planes the update reads (the reference's Conv^T((2 (Conv x - y)) 0.5)
                               with the separable passes regrouped); other chains: pcs_conv1d per
                               axis, pcs_axpby, the flipped chain
    pcs_pds3d_step             x, z, g -> x', z', norm partials, loop control

Volumes are split into slabs of planes (axis 0) across ranks exactly like the 2-D rows of
``pycsou_amd.parallel.slab``: a slab stores planes ``[plane0 - h, plane0 + planes + h)``; the
convolution chain runs on the slab's halo'd sub-volume (its axis-0 reach is covered by the
x halo of ``2 reach + 1`` planes), the update needs one plane of z halo.  Per iteration the
ranks all-gather the four norm sums and exchange the x' / z' halo planes.
"""

import ctypes
import os

import numpy as np
import torch

from .. import _lib as L
from .. import _ops as O
from ..core.functional import ProxFuncPostComp
from ..core.linop import LinOpComp
from ..core.map import DiffMapComp
from ..func.base import IndicatorFunctional, NullDifferentiableFunctional, NullProximableFunctional
from ..func.penalty import L1Norm, L21Norm
from ..linop.conv import Convolve1DOp
from ..linop.diff import GradientOp
from ..parallel.slab import SlabLayout
from .engine import HIST_CHUNK, _half_loss_data, grow_hist


def conv_chain(C, shape):
    """The Convolve1D operators of a composition in application order, or None."""
    if isinstance(C, Convolve1DOp):
        return [C] if tuple(C.dims) == tuple(shape) else None
    if isinstance(C, LinOpComp):
        first, then = conv_chain(C.LinOp2, shape), conv_chain(C.LinOp1, shape)
        return None if first is None or then is None else first + then
    return None


def match_pds3d(F, G, H, K, has_H):
    """Engine spec dict if (F, G, H, K) is a fused 3-D problem, else None."""
    if not has_H or not isinstance(K, GradientOp) or len(K.dims) != 3:
        return None
    kinds = {'forward': L.PCS_FORWARD, 'backward': L.PCS_BACKWARD, 'centered': L.PCS_CENTERED}
    if K.kind not in kinds:
        return None
    shape = tuple(K.dims)
    N = int(np.prod(shape))
    # kkind: forward -> k_pds3d; backward / centred (the reference's default) -> k_pds3d_gen
    spec = {'ndim': 3, 'shape': shape, 'steps': tuple(K.steps), 'kkind': kinds[K.kind], 'edge': int(K.edge)}
    base, lam = H, 1.0
    if isinstance(H, ProxFuncPostComp):
        if H.shift != 0:
            return None
        base, lam = H.prox_func, float(H.scale)
    if isinstance(base, L21Norm) and base.pixel_d == 3 and base.dim == 3 * N:
        spec['hkind'] = L.PCS_H_L21
    elif isinstance(base, L1Norm) and base.dim == 3 * N:
        spec['hkind'] = L.PCS_H_L1
    else:
        return None
    spec['lam'] = lam
    if G is None or isinstance(G, NullProximableFunctional):
        spec['gkind'], spec['seg'] = L.PCS_G_NULL, (0.0, 1.0)
    elif isinstance(G, IndicatorFunctional) and G.kind == 'nonneg':
        spec['gkind'], spec['seg'] = L.PCS_G_NONNEG, (0.0, 1.0)
    elif isinstance(G, IndicatorFunctional) and G.kind == 'segment':
        spec['gkind'], spec['seg'] = L.PCS_G_SEGMENT, G.params
    else:
        return None
    if F is None or isinstance(F, NullDifferentiableFunctional):
        spec['fkind'] = L.PCS_F_NULL
        return spec
    s = _half_loss_data(F)
    if s is not None and O.numel(s) == N:
        spec['fkind'], spec['shift'] = L.PCS_F_DENOISE, s
        return spec
    if isinstance(F, DiffMapComp):
        chain = conv_chain(F.map2, shape)
        s = _half_loss_data(F.map1)
        if chain and s is not None and O.numel(s) == N:
            spec['fkind'], spec['shift'], spec['chain'] = L.PCS_F_GRADBUF, s, chain
            return spec
    return None


class PDS3DEngine:
    """Device state + loop of one rank's slab (the whole volume when world == 1)."""

    def __init__(self, spec, dtype, tau, sigma, rho, x0, z0, comm=None, rank=0, world=1, chunk=8, use_graph=True,
                 overlap=True):
        self.lib = L.gpu()
        self.spec, self.dtype, self.comm = spec, dtype, comm
        self.rank, self.world = int(rank), int(world)
        # multi-GPU transport: the library's RCCL binding (pcs_halo_exchange / pcs_allgather_f64,
        # stream-ordered, so a chunk of iterations -- kernels and RCCL -- is captured into one
        # hipGraph) when the group offers it; PCS_3D_NATIVE=0 keeps the torch.distributed calls
        self.native_comm = False
        if (self.world > 1 and comm is not None and hasattr(comm, 'rccl')
                and os.environ.get('PCS_3D_NATIVE', '1') != '0'):
            rc = comm.rccl()
            if rc is not None:
                self.comm, self.native_comm = rc, True
        n0, n1, n2 = spec['shape']
        self.n0, self.n1, self.n2 = n0, n1, n2
        plane = n1 * n2
        self.plane = plane
        self.lay = lay = SlabLayout(n0, plane, rank, world)  # rows of the layout = planes
        self.row0, self.rows = lay.row0, lay.rows
        fk = spec['fkind']
        self.fkind = fk
        dev = torch.device('cuda', torch.cuda.current_device())
        self.chain = []
        self.ata = False
        reach = 0
        if fk == L.PCS_F_GRADBUF:
            for op in spec['chain']:
                k, off = op.k, op.off
                self.chain.append((op.axis, op._h.get(dtype), op._hf.get(dtype), k, off))
                if op.axis == 0:
                    reach += max(off, k - 1 - off)
        hx = 2 * reach + 1 if fk == L.PCS_F_GRADBUF else 1
        self.kkind = spec.get('kkind', L.PCS_FORWARD)
        # backward / centred K: K^T z at plane p reads z0(p + 1) and u is needed one plane below
        # the slab too (K u reaches back): z halo 2, and g on planes [-1, rows] (g_lo below)
        hz = 1 if self.kkind == L.PCS_FORWARD else 2
        hg = hx if fk == L.PCS_F_GRADBUF else 1
        if world > 1 and self.rows < max(hx, hz):
            raise ValueError(f'slab of {self.rows} planes is thinner than its halo ({hx} planes)')
        self.hx, self.hz, self.hg = hx, hz, hg
        self.g_lo = hx if self.kkind == L.PCS_FORWARD else hx - 1  # first sub-volume plane of g the update reads
        N = n0 * plane
        x0d, z0d = O.to_dev(x0, dtype), O.to_dev(z0, dtype)
        self.X = [lay.window(x0d, hx) for _ in range(2)]
        self.Z = [torch.cat([lay.window(z0d[c * N:(c + 1) * N], hz) for c in range(3)]) for _ in range(2)]
        self.gbuf = None
        if fk in (L.PCS_F_DENOISE, L.PCS_F_GRADBUF):
            self.yw = lay.window(-O.to_dev(spec['shift'], dtype), hg)  # y = -shift exactly
        if fk == L.PCS_F_GRADBUF:
            nloc = (self.rows + 2 * hx) * plane
            self.T = [torch.empty(nloc, dtype=dtype, device=dev) for _ in range(2)]
            self.sub_dims = (self.rows + 2 * hx, n1, n2)
            # planes of the sub-volume outside the image: the residual is 0 there
            self.zero_planes = [j for j in range(self.rows + 2 * hx)
                                if not 0 <= self.row0 - hx + j < n0]
            ax0 = [c for c in self.chain if c[0] == 0]
            # one axis-0 Convolve1D of <= 15 taps: in-plane passes, then the axis-0 forward conv,
            # residual and adjoint conv fused in one plane-streaming pass, then the in-plane
            # adjoint passes on the planes the update reads only
            self.fused0 = len(ax0) == 1 and ax0[0][3] <= 15
            if self.fused0:
                self.inplane = [c for c in self.chain if c[0] != 0]
                self.ax0 = ax0[0]
                nin = len(self.inplane)
                # forward passes alternate T0/T1 from x, the fused pass and the adjoint passes
                # continue the alternation: 2 nin + 1 passes end in T[(2 nin) % 2]
                self.gbuf = self.T[0]
                # one axis-1 and one axis-2 conv of <= 15 taps: both in-plane passes in one launch
                esz = torch.empty(0, dtype=dtype).element_size()
                self.sep2 = (sorted(c[0] for c in self.inplane) == [1, 2] and all(c[3] <= 15 for c in self.inplane)
                             and (plane * esz) % 16 == 0)
                # the in-plane normal operator in one launch (pcs_conv2d_sep_ata_planes: two
                # 29-tap passes).  The axis-0 pass commutes with the in-plane ones, so
                # g = C0^T (C0 (C12^T C12 x) - C12^T y) with C12^T y formed here once: two
                # sub-volume passes per iteration instead of three (15 words/voxel, not 17).
                # Default for fp32 (C4: 568-571 against 541-546 it/s) and, since the kernel's
                # one-task-per-workgroup grid (round 4: 5.6 against 7.2 ms for the two passes at
                # 1024^3), fp64 (C5 39.0 against 36.7-36.9 it/s with the three-pass chain,
                # profiles/r4_c5_ata_ab2.txt).  PCS_3D_ATA=0/1 overrides
                self.ata = False
                ata_default = '1'
                if self.sep2 and os.environ.get('PCS_3D_ATA', ata_default) == '1':
                    (ha, ka, oa), (hb, kb, ob) = self._inplane_ab(False)
                    rc = self.lib.pcs_conv2d_sep_ata_planes(L.dtcode(self.T[0]), L.ptr(self.T[0]), L.ptr(self.T[1]),
                                                            0, n1, n2, L.ptr(ha), ka, oa, L.ptr(hb), kb, ob,
                                                            L.stream())
                    self.ata = rc == 0
                if self.ata:
                    self.gbuf = self.T[1]
            else:
                # the chain's final buffer is fixed by its length: forward + adjoint passes
                self.gbuf = self.T[(2 * len(self.chain) - 1) % 2]
        # Banded schedule (multi-GPU): the update of the B = hx + 1 planes at each end of the slab
        # (the planes the neighbours' halos copy, and the only ones whose gradient reaches into
        # our halos) runs first, their halo exchange overlaps the interior update, and the
        # in-plane passes of our own planes run before the previous exchange is awaited.
        # Needs the fused axis-0 gradient with both in-plane passes in one launch (C4/C5).
        self.band = hx + 1
        self.banded = (fk == L.PCS_F_GRADBUF and self.fused0 and self.sep2 and world > 1
                       and self.rows > 2 * self.band) if fk == L.PCS_F_GRADBUF else False
        self.overlap = bool(overlap)
        # banded order: 'split' = g of the boundary bands before the exchange starts, the
        # interior's g after (the exchange overlaps the interior g + update); 'fullg' = g on
        # all planes before the exchange (one axis-0 launch: no extra 28-plane prologues per
        # band; the exchange overlaps the interior update only).  Same arithmetic either way.
        self.order = os.environ.get('PCS_3D_ORDER', 'split')
        # which order wins depends on the link speed (the halo bytes vs the overlap window):
        # with a real transport the first advance() of >= 7 iterations times both and the serial
        # schedule and keeps the fastest (max over ranks), unless PCS_3D_ORDER fixes it
        self._tuned = 'PCS_3D_ORDER' in os.environ or not getattr(comm, 'tunable', False)
        if fk == L.PCS_F_GRADBUF and self.fused0 and self.sep2 and not self.ata and self.rows > 2 * self.band:
            # g in a buffer of its own: the banded order writes g on the boundary planes while the
            # interior's axis-0 pass still reads the in-plane forward result around them
            self.T.append(torch.empty_like(self.T[0]))
            self.gbuf = self.T[2]
        a = L.Pds3Args()
        a.dtype = L.PCS_F32 if dtype == torch.float32 else L.PCS_F64
        a.fkind, a.hkind, a.gkind = fk, spec['hkind'], spec['gkind']
        a.n0, a.n1, a.n2, a.plane0, a.planes = n0, n1, n2, self.row0, self.rows
        a.halo_x, a.halo_z, a.halo_g = hx, hz, hg
        a.tau, a.sigma, a.rho, a.lam = float(tau), float(sigma), float(rho), spec['lam']
        a.step0, a.step1, a.step2 = spec['steps']
        a.seg_a, a.seg_b = spec['seg']
        a.kkind, a.edge = self.kkind, spec.get('edge', 0)
        if fk == L.PCS_F_DENOISE:
            a.g = self.yw.data_ptr()
        elif fk == L.PCS_F_GRADBUF:
            a.g = self.gbuf.data_ptr()
        self.nblocks = int(self.lib.pcs_pds3d_nblocks(ctypes.byref(a)))
        self.partials = torch.empty(self.nblocks * 4, dtype=torch.float64, device=dev)
        a.partials = self.partials.data_ptr()
        self.ctrl = torch.zeros(int(self.lib.pcs_ctrl_bytes()) // 8, dtype=torch.float64, device=dev)
        a.ctrl = self.ctrl.data_ptr()
        self.ws = torch.zeros(int(self.lib.pcs_pds3d_ws_bytes(ctypes.byref(a))) // 8 + 2, dtype=torch.float64,
                              device=dev)
        a.ws = self.ws.data_ptr()
        self.base_args = a
        if self.ata:  # C12^T y on every stored plane (setup, once)
            self.yb = torch.empty_like(self.yw)
            self._sep_planes(L.ptr(self.yw), L.ptr(self.yb), self.rows + 2 * hg, self.inplane[::-1], True, L.stream())
        # fp32 forward K: the axis-0 pass folded into the update (PCS_F_CONV0: g = C0^T (C0 t - C12^T y)
        # from t = C12^T C12 x inside k_pds3d, whose second set of 512 threads keeps two 15-plane
        # register rings per voxel): 13 words per voxel and iteration instead of 15, bitwise the same
        # iterates; C4 1.63-1.65 ms against 1.72-1.74 ms with the separate pass
        # (profiles/r3_ck30_fold_ab.txt).  PCS_3D_FOLD=0 keeps the separate pass.  (Backward / centred K:
        # the rings fit only beside 8-row k_pds3d_gen tiles, which cost more than the pass saves --
        # profiles/r5_c4cen_fold_ab.txt.)
        self.fold = False
        if self.ata and self.kkind == L.PCS_FORWARD and os.environ.get('PCS_3D_FOLD', '1') != '0':
            _, h0, _, k0, off0 = self.ax0
            b = L.Pds3Args()
            ctypes.pointer(b)[0] = a
            b.fkind, b.g, b.conv0_w, b.conv0_taps, b.conv0_k, b.conv0_off = (L.PCS_F_CONV0, self.T[0].data_ptr(),
                                                                            self.yb.data_ptr(), h0.data_ptr(),
                                                                            int(k0), int(off0))
            b.x = b.xn = b.z = b.zn = self.X[0].data_ptr()  # placeholders: the query launches nothing
            if int(self.lib.pcs_pds3d_nblocks_bands(ctypes.byref(b), 0, self.rows, self.rows, self.rows)) > 0:
                a.fkind, a.g, a.conv0_w, a.conv0_taps, a.conv0_k, a.conv0_off = (b.fkind, b.g, b.conv0_w,
                                                                                 b.conv0_taps, b.conv0_k, b.conv0_off)
                self.fold = True
                # the per-workgroup partials and the reduction workspace follow the folded launch's grid
                self.nblocks = int(self.lib.pcs_pds3d_nblocks(ctypes.byref(a)))
                self.partials = torch.empty(self.nblocks * 4, dtype=torch.float64, device=dev)
                a.partials = self.partials.data_ptr()
                self.ws = torch.zeros(int(self.lib.pcs_pds3d_ws_bytes(ctypes.byref(a))) // 8 + 2, dtype=torch.float64,
                                      device=dev)
                a.ws = self.ws.data_ptr()
        self.args = [self._args_for(p) for p in (0, 1)]
        self.sums = torch.zeros(4, dtype=torch.float64, device=dev)
        self.gathered = torch.zeros(4 * world, dtype=torch.float64, device=dev)
        # z halo planes the update reads (the exchange moved every component's full halo).
        # Backward / centred K: K^T z at plane p reads z0 of p - 1 .. p + 1 and the segments' one-plane-early
        # start / one-past end read z0 two planes out but z1 / z2 of one halo plane only (they are in-plane
        # derivatives): z1 / z2 send 1 of their 2 stored planes (C5/8: 19 planes per side instead of 21).
        # Forward K reads z0 one plane below and above, z1 / z2 one plane above (u on the plane past the slab),
        # all of its 1-plane halos (a one-directional z1 / z2 exchange would shorten the upward messages only,
        # and the downward ones, which carry them, set the exchange time)
        self.zdepth = (1, 1, 1) if self.kkind == L.PCS_FORWARD else (2, 1, 1)
        self.halos = [lay.halo_pairs([(self.X[q], hx, 0)] + [(self.Z[q], hz, c, self.zdepth[c]) for c in range(3)])
                      for q in (0, 1)] if world > 1 else [{}, {}]
        self.halo_planes = hx + sum(self.zdepth)  # planes one side sends per iteration
        self.hist = None
        self.graph = None
        self.chunk = max(2, chunk + chunk % 2)
        # graphs: one GPU, or the native RCCL transport (PCS_3D_GRAPH=0 launches eagerly)
        self.use_graph = use_graph and (world == 1 or (self.native_comm and os.environ.get('PCS_3D_GRAPH', '1') != '0'))

    def _args_for(self, p):
        b = L.Pds3Args()
        ctypes.pointer(b)[0] = self.base_args
        b.x, b.xn = self.X[p].data_ptr(), self.X[1 - p].data_ptr()
        b.z, b.zn = self.Z[p].data_ptr(), self.Z[1 - p].data_ptr()
        return b

    # ---- grad F = C^T (C x - y) on the slab's sub-volume
    def _conv_into(self, src, dst, axis, taps, k, off, st):
        L.check(self.lib.pcs_conv1d(self.base_args.dtype, L.ptr(src), L.ptr(dst), 3, L.i64s(self.sub_dims),
                                    int(axis), L.ptr(taps), int(k), int(off), st), 'pcs_conv1d')

    def _inplane_ab(self, flipped):
        """((taps, k, off) along axis 1, (taps, k, off) along axis 2) of the in-plane passes."""
        out = {}
        for axis, h, hf, k, off in self.inplane:
            out[axis] = (hf, k, k - 1 - off) if flipped else (h, k, off)
        return out[1], out[2]

    def _ata_planes(self, src, dst, np_, st):
        """dst = C12^T C12 src on np_ planes (both in-plane convolutions and their adjoints)."""
        (ha, ka, oa), (hb, kb, ob) = self._inplane_ab(False)
        L.check(self.lib.pcs_conv2d_sep_ata_planes(self.base_args.dtype, src, dst, np_, self.n1, self.n2, L.ptr(ha), ka,
                                                   oa, L.ptr(hb), kb, ob, st), 'pcs_conv2d_sep_ata_planes')

    def _sep_planes(self, src, dst, np_, ops, flipped, st):
        """Both in-plane passes of `ops` (one along axis 1, one along axis 2) in one launch.  The
        two convolutions commute; the axis-2 pass runs first (the faster kernel order,
        tools/sep2d_probe.py), which changes only the rounding order of the sums."""
        (a0, h0, hf0, k0, o0), (a1, h1, hf1, k1, o1) = ops
        first, second = (h0, k0, o0) if not flipped else (hf0, k0, k0 - 1 - o0), \
                        (h1, k1, o1) if not flipped else (hf1, k1, k1 - 1 - o1)
        (ha, ka, oa), (hb, kb, ob) = (first, second) if a0 == 1 else (second, first)
        L.check(self.lib.pcs_conv2d_sep_planes(self.base_args.dtype, src, dst, np_, self.n1, self.n2, L.ptr(ha), ka, oa,
                                               L.ptr(hb), kb, ob, 0, st), 'pcs_conv2d_sep_planes')

    def _gradient_fused0(self, p, st):
        nsub = self.rows + 2 * self.hx
        plane = self.plane
        if self.ata:
            self._ata_planes(L.ptr(self.X[p]), L.ptr(self.T[0]), nsub, st)
            self._g_range(self.g_lo, min(self.hx + self.rows + 1, nsub), st)
            return
        cur, j = self.X[p], 0
        if self.sep2:
            dst = self.T[0]
            self._sep_planes(L.ptr(cur), L.ptr(dst), nsub, self.inplane, False, st)
            cur, j = dst, 1
        else:
            for axis, h, _, k, off in self.inplane:
                dst = self.T[j % 2]
                self._conv_into(cur, dst, axis, h, k, off, st)
                cur, j = dst, j + 1
        # s on the planes the update reads: own planes + the next one (u on the slab's last plane + 1)
        # and, for backward / centred K, the one before
        q0, q1 = self.g_lo, min(self.hx + self.rows + 1, nsub)
        img_lo, img_hi = self.hx - self.row0, self.hx - self.row0 + self.n0
        _, h, _, k, off = self.ax0
        dst = self.T[j % 2]
        L.check(self.lib.pcs_conv0_residual_adjoint(self.base_args.dtype, L.ptr(cur), L.ptr(self.yw), L.ptr(dst), nsub,
                                                    plane, L.ptr(h), int(k), int(off), img_lo, img_hi, q0, q1, st),
                'pcs_conv0_residual_adjoint')
        cur, j = dst, j + 1
        dims = L.i64s((q1 - q0, self.n1, self.n2))
        esz = cur.element_size()
        if self.sep2:
            dst = self.gbuf
            self._sep_planes(ctypes.c_void_p(cur.data_ptr() + q0 * plane * esz),
                             ctypes.c_void_p(dst.data_ptr() + q0 * plane * esz), q1 - q0, self.inplane[::-1], True, st)
            return
        for axis, _, hf, k, off in reversed(self.inplane):
            dst = self.T[j % 2]
            L.check(self.lib.pcs_conv1d(self.base_args.dtype, ctypes.c_void_p(cur.data_ptr() + q0 * plane * esz),
                                        ctypes.c_void_p(dst.data_ptr() + q0 * plane * esz), 3, dims, int(axis),
                                        L.ptr(hf), int(k), int(k - 1 - off), st), 'pcs_conv1d')
            cur, j = dst, j + 1
        assert cur is self.gbuf

    # ---- banded order (sep2 + fused axis-0 pass): planes in sub-volume coordinates
    def _sep_range(self, src, dst, j0, j1, flipped, st):
        if j1 <= j0:
            return
        off = j0 * self.plane * src.element_size()
        if self.ata and not flipped:  # the forward in-plane stage is C12^T C12
            self._ata_planes(ctypes.c_void_p(src.data_ptr() + off), ctypes.c_void_p(dst.data_ptr() + off), j1 - j0, st)
            return
        ops = self.inplane[::-1] if flipped else self.inplane
        self._sep_planes(ctypes.c_void_p(src.data_ptr() + off), ctypes.c_void_p(dst.data_ptr() + off), j1 - j0, ops,
                         flipped, st)

    def _g_range(self, q0, q1, st):
        """g = C^T (C x - y) on sub-volume planes [q0, q1) from the in-plane result in T0 (nothing
        with the axis-0 pass folded into the update)."""
        if q1 <= q0 or self.fold:
            return
        nsub = self.rows + 2 * self.hx
        img_lo, img_hi = self.hx - self.row0, self.hx - self.row0 + self.n0
        _, h, _, k, off = self.ax0
        if self.ata:  # C0^T (C0 t - C12^T y) straight into g
            L.check(self.lib.pcs_conv0_residual_adjoint(self.base_args.dtype, L.ptr(self.T[0]), L.ptr(self.yb),
                                                        L.ptr(self.gbuf), nsub, self.plane, L.ptr(h), int(k), int(off),
                                                        img_lo, img_hi, q0, q1, st), 'pcs_conv0_residual_adjoint')
            return
        L.check(self.lib.pcs_conv0_residual_adjoint(self.base_args.dtype, L.ptr(self.T[0]), L.ptr(self.yw),
                                                    L.ptr(self.T[1]), nsub, self.plane, L.ptr(h), int(k), int(off),
                                                    img_lo, img_hi, q0, q1, st), 'pcs_conv0_residual_adjoint')
        self._sep_range(self.T[1], self.gbuf, q0, q1, True, st)

    def _band_pre(self, p, st):
        """In-plane forward passes of the own planes (no halo needed)."""
        self._sep_range(self.X[p], self.T[0], self.hx, self.hx + self.rows, False, st)

    def _band_boundary(self, p, st):
        """In-plane passes of the halo planes, g and the update on the two boundary bands."""
        hx, R, B = self.hx, self.rows, self.band
        nsub = R + 2 * hx
        self._sep_range(self.X[p], self.T[0], 0, hx, False, st)
        self._sep_range(self.X[p], self.T[0], hx + R, nsub, False, st)
        g0 = self.g_lo  # hx, or hx - 1 for backward / centred K (u one plane before each band)
        if self.order == 'fullg':  # g on every plane the update reads, one axis-0 launch
            self._g_range(g0, min(hx + R + 1, nsub), st)
        else:
            self._g_range(g0, hx + B + 1, st)
            self._g_range(hx + R - B - (hx - g0), min(hx + R + 1, nsub), st)
        a = self.args[p]
        a.hist = None
        a.partials = self.partials.data_ptr()
        L.check(self.lib.pcs_pds3d_step_bands(ctypes.byref(a), 0, B, R - B, R, st), 'pcs_pds3d_step_bands')

    def _band_interior(self, p, st):
        hx, R, B = self.hx, self.rows, self.band
        if self.order != 'fullg':
            self._g_range(hx + B + 1, hx + R - B, st)
        a = self.args[p]
        a.hist = None
        a.partials = self.partials.data_ptr() + 32 * self.nb_bands[0]
        L.check(self.lib.pcs_pds3d_step_bands(ctypes.byref(a), B, R - B, R - B, R - B, st), 'pcs_pds3d_step_bands')
        a.partials = self.partials.data_ptr()
        L.check(self.lib.pcs_reduce_partials(L.ptr(self.partials), sum(self.nb_bands), L.ptr(self.sums), st),
                'pcs_reduce_partials')

    def _init_bands(self):
        if getattr(self, 'nb_bands', None) is not None:
            return
        R, B = self.rows, self.band
        a = self.args[0]
        self.nb_bands = [int(self.lib.pcs_pds3d_nblocks_bands(ctypes.byref(a), 0, B, R - B, R)),
                         int(self.lib.pcs_pds3d_nblocks_bands(ctypes.byref(a), B, R - B, R - B, R - B))]
        if min(self.nb_bands) < 1:
            raise ValueError('banded 3-D step unavailable for this slab')
        need = 4 * sum(self.nb_bands)
        if self.partials.numel() < need:
            self.partials = torch.empty(need, dtype=torch.float64, device=self.partials.device)
            for q in (0, 1):
                self.args[q].partials = self.partials.data_ptr()

    def _gradient(self, p, st):
        if self.fused0:
            return self._gradient_fused0(p, st)
        cur, j = self.X[p], 0
        for axis, h, _, k, off in self.chain:
            dst = self.T[j % 2]
            self._conv_into(cur, dst, axis, h, k, off, st)
            cur, j = dst, j + 1
        # r = (C x) + (-y): the reference's residual, exact
        L.check(self.lib.pcs_axpby(self.base_args.dtype, L.ptr(cur), L.ptr(self.yw), L.ptr(cur), cur.numel(), 1.0,
                                   -1.0, st), 'pcs_axpby')
        if self.zero_planes:  # at most one run at each end of the sub-volume
            v = cur.view(-1, self.plane)
            lo = [j for j in self.zero_planes if j < self.hx]
            hi = [j for j in self.zero_planes if j >= self.hx]
            if lo:
                v[lo[0]:lo[-1] + 1].zero_()
            if hi:
                v[hi[0]:hi[-1] + 1].zero_()
        for axis, _, hf, k, off in reversed(self.chain):
            dst = self.T[j % 2]
            self._conv_into(cur, dst, axis, hf, k, k - 1 - off, st)
            cur, j = dst, j + 1
        assert cur is self.gbuf

    def _step(self, p, hist):
        st = L.stream()
        if self.fkind == L.PCS_F_GRADBUF:
            self._gradient(p, st)
        a = self.args[p]
        a.hist = None if hist is None else hist.data_ptr()
        L.check(self.lib.pcs_pds3d_step(ctypes.byref(a), st), 'pcs_pds3d_step')

    # phases of a multi-rank iteration (pycsou_amd.parallel.run_local interleaves them)
    def _compute(self, p, split=False):
        if split:  # the banded order, serialised (run_local)
            self._init_bands()
            st = L.stream()
            self._band_pre(p, st)
            self._band_boundary(p, st)
            self._band_interior(p, st)
            return
        self._step(p, None)
        L.check(self.lib.pcs_reduce_partials(L.ptr(self.partials), self.nblocks, L.ptr(self.sums), L.stream()),
                'pcs_reduce_partials')

    def _finalize(self):
        L.check(self.lib.pcs_pds_reduce_finalize(L.ptr(self.gathered), self.world, L.ptr(self.ctrl),
                                                 L.ptr(self.hist), L.stream()), 'pcs_pds_reduce_finalize')

    def iteration(self, p):
        if self.world == 1:
            self._step(p, self.hist)
            return
        if self.banded and self.overlap:
            # in-plane passes of our planes overlap the previous iteration's halo exchange and
            # sums all-gather; the boundary bands' exchange overlaps the interior update
            self._init_bands()
            st = L.stream()
            self._band_pre(p, st)
            self._drain()
            self._band_boundary(p, st)
            self._pending_ex = self.comm.exchange_start(self.halos[1 - p])
            self._band_interior(p, st)
            self._pending_ag = self.comm.allgather_start(self.sums, self.gathered)
            return
        self._compute(p)
        self.comm.allgather(self.sums, self.gathered)
        self._finalize()
        self.comm.exchange(self.halos[1 - p])

    def _drain(self):
        """Order the current stream after the in-flight exchange / all-gather and run the loop
        control of the iteration they belong to."""
        ex, ag = getattr(self, '_pending_ex', None), getattr(self, '_pending_ag', None)
        self._pending_ex = self._pending_ag = None
        if ex is not None:
            ex.wait()
        if ag is not None:
            ag.wait()
            self._finalize()

    # ---- loops
    def init_loop(self, max_iter, min_iter, accuracy_threshold, has_dual=True):
        max_iter, min_iter = int(max_iter), int(min_iter)
        total = max(min_iter, max_iter) + 1
        self._total, self._issued = total, 0
        hist_len = 2 * min(total, max(HIST_CHUNK, 2 * self.chunk)) + 2
        if self.hist is None or self.hist.numel() < hist_len:
            self.hist = torch.empty(hist_len, dtype=torch.float64, device=self.X[0].device)
            self.graph = None
        self.hist.fill_(float('nan'))
        L.check(self.lib.pcs_ctrl_init2(L.ptr(self.ctrl), int(min_iter), int(max_iter), float(accuracy_threshold),
                                        int(has_dual), int(self.hist.numel()), L.stream()), 'pcs_ctrl_init2')
        self._p = 0
        return total

    def _chunk(self):
        for i in range(self.chunk):
            self.iteration(i % 2)
        if self.world > 1:
            self._drain()  # the side stream rejoins before the chunk (and a capture) ends

    def _capture(self):
        """Capture one chunk into a hipGraph.  Multi-GPU: every rank must end up with a graph or
        none (the captured RCCL calls pair across ranks), so the outcome is agreed collectively and
        a failed capture anywhere falls back to eager launches everywhere."""
        torch.cuda.synchronize()
        g, ok = torch.cuda.CUDAGraph(), True
        try:
            with torch.cuda.graph(g):
                self._chunk()
        except Exception:  # noqa: BLE001 -- torch's capture errors and the ABI's HipError alike: the
            # flag all-gather below must run on every rank, or the others block in RCCL
            ok, g = False, None
            self._pending_ex = self._pending_ag = None  # handles of the aborted capture
            torch.cuda.synchronize()
        if self.world > 1:
            flag = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=self.sums.device)
            allf = torch.zeros(self.world, dtype=torch.float64, device=self.sums.device)
            self.comm.allgather(flag, allf)
            ok = bool(allf.min().item() > 0)
        if not ok:
            self.use_graph, g = False, None
        self.graph = g
        return ok

    def advance(self, k):
        """Enqueue exactly k iterations: the schedule trial's (the first call with k >= 7 on a
        banded multi-GPU engine), then whole captured chunks from buffer parity 0, then eager
        iterations (a parity fix before the replays, the remainder after them)."""
        grown = grow_hist(self.hist, self.ctrl, self._issued + k + 1, self._total)
        if grown is not self.hist:  # the captured chunk holds the history pointer: recapture
            self.hist, self.graph = grown, None
        self._issued += k
        if not self._tuned and self.banded and self.overlap and k >= 7:
            k -= self._autotune()  # eager, before any capture
            self._drain()
        if k > 0 and self.use_graph and (self.graph is not None or self._capture()):
            if self._p == 1:  # the captured chunk starts from buffers 0
                self.iteration(1)
                self._p = 0
                k -= 1
                self._drain()
            for _ in range(k // self.chunk):
                self.graph.replay()
            k %= self.chunk
        for _ in range(k):
            self.iteration(self._p)
            self._p ^= 1
        self._drain()

    def _autotune(self):
        """Time 2 iterations in each banded order and in the serial schedule (compute, then the
        blocking all-gather and exchange) after one untimed, and keep the fastest; every rank takes
        the same decision (max over ranks).  The three schedules compute bitwise the same iterates.
        Returns the iterations used."""
        self.iteration(self._p)
        self._p ^= 1
        cands = ('split', 'fullg', 'serial')
        times = []
        for cand in cands:
            self.overlap = cand != 'serial'
            if self.overlap:
                self.order = cand
            self._drain()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(2):
                self.iteration(self._p)
                self._p ^= 1
            self._drain()
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
        dev = self.sums.device
        mine = torch.tensor(times + [0.0], dtype=torch.float64, device=dev)
        allt = torch.zeros(4 * self.world, dtype=torch.float64, device=dev)
        self.comm.allgather(mine, allt)
        worst = allt.view(self.world, 4).max(dim=0).values[:3]
        best = int(torch.argmin(worst).item())
        self.overlap = cands[best] != 'serial'
        if self.overlap:
            self.order = cands[best]
        self.tune_ms = {c: float(worst[i]) / 2 for i, c in enumerate(cands)}
        self._tuned = True
        return 7

    def iterations(self):
        return int(self.ctrl.view(torch.int32)[0].item())

    def stopped(self):
        return int(self.ctrl.view(torch.int32)[1].item()) != 0

    def result(self):
        """(n_iter, own planes of x, own planes of z (3 components), hist [n, 2])."""
        torch.cuda.synchronize()
        n = self.iterations()
        q = n % 2
        x = self.lay.rows_view(self.X[q], self.hx, 0, self.rows).clone()
        z = torch.cat([self.lay.rows_view(self.Z[q], self.hz, 0, self.rows, c) for c in range(3)])
        h = self.hist[:2 * n].cpu().numpy().reshape(n, 2) if n > 0 else np.zeros((0, 2))
        return n, x, z, h

    def run(self, max_iter, min_iter, accuracy_threshold, has_dual=True):
        total = self.init_loop(max_iter, min_iter, accuracy_threshold, has_dual)
        step = self.chunk
        done = 0
        while done < total:
            self.advance(step)
            done += step
            if self.stopped():
                break
        return self.result()

    def time_parts(self, n):
        """Mean duration (ms) of each launch of one single-GPU iteration over n eager iterations (HIP
        events on the engine's stream): the in-plane normal operator (`nrm`), the axis-0 pass (`conv0`,
        absent when it is folded into the update) and the update (`step`).  Leaves the loop state as
        init_loop(n + 1, ...) set it; call init_loop again before a measured run."""
        if self.world != 1:
            raise ValueError('time_parts: single-GPU engines only')
        L.check(self.lib.pcs_ctrl_init2(L.ptr(self.ctrl), n + 1, n + 1, -1.0, 1, 2 * n + 6, L.stream()),
                'pcs_ctrl_init2')
        st = torch.cuda.current_stream()
        ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
        parts = {}
        for i in range(n):
            p = i % 2
            marks = [('start', ev())]
            marks[-1][1].record(st)
            if self.fkind == L.PCS_F_GRADBUF and self.fused0 and self.ata:
                nsub = self.rows + 2 * self.hx
                self._ata_planes(L.ptr(self.X[p]), L.ptr(self.T[0]), nsub, L.stream())
                marks.append(('nrm', ev()))
                marks[-1][1].record(st)
                if not self.fold:
                    self._g_range(self.g_lo, min(self.hx + self.rows + 1, nsub), L.stream())
                    marks.append(('conv0', ev()))
                    marks[-1][1].record(st)
            elif self.fkind == L.PCS_F_GRADBUF:
                self._gradient(p, L.stream())
                marks.append(('gradient', ev()))
                marks[-1][1].record(st)
            a = self.args[p]
            a.hist = None
            L.check(self.lib.pcs_pds3d_step(ctypes.byref(a), L.stream()), 'pcs_pds3d_step')
            marks.append(('step', ev()))
            marks[-1][1].record(st)
            parts.setdefault(i, marks)
        torch.cuda.synchronize()
        out = {}
        for marks in parts.values():
            for (_, e0), (name, e1) in zip(marks[:-1], marks[1:]):
                out.setdefault(name, []).append(e0.elapsed_time(e1))
        return {k: float(np.mean(v)) for k, v in out.items()}

    def time_step_kernel(self, n):
        """Mean duration (ms) of pcs_pds3d_step alone over n eager launches (HIP events)."""
        st = torch.cuda.current_stream()
        L.check(self.lib.pcs_ctrl_init2(L.ptr(self.ctrl), n + 1, n + 1, -1.0, 1, 2 * n + 6, L.stream()),
                'pcs_ctrl_init2')
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        for i in range(n):
            a = self.args[i % 2]
            a.hist = None
            evs[i][0].record(st)
            L.check(self.lib.pcs_pds3d_step(ctypes.byref(a), L.stream()), 'pcs_pds3d_step')
            evs[i][1].record(st)
        torch.cuda.synchronize()
        return float(np.mean([s.elapsed_time(e) for s, e in evs]))

"""Row-slab sharding of the fused 2-D PDS loop over GPUs.

The reference solves one image on one host (``PrimalDualSplitting`` in
``pycsou/opt/proxalgs.py:343-394``); here an ``n0 x n1`` image (C order) is split into
contiguous row slabs, one per rank (one process per GPU).  Rank ``r`` stores rows
``[row0 - h, row0 + rows + h)`` of every array the step reads at a row offset and computes
only its own rows.  One iteration is

    pcs_pds2d_step (slab mode)      x, z  ->  x', z' on own rows + per-block norm partials
    pcs_reduce_partials             -> 4 local sums, fixed order
    all-gather of the 4 sums        (RCCL, 32 B per rank)
    pcs_pds_reduce_finalize         -> the same global sums, history entry and stop flag
                                       on every rank (sums added in rank order)
    halo exchange                   x' (hx rows), z0'/z1' (hz rows) with the two
                                    neighbour ranks (RCCL point-to-point, one group call)

Halo depths follow the step's stencil reach: x' at row i reads x rows i-2H-1 .. i+2H+1
(conv^T conv of half-width H plus the forward difference of u = 2x' - x), y rows
i-H-1 .. i+H+1 and z rows i-1 .. i+1, hence hx = 2H+1, hy = H+1, hz = 1 (H = 0 without
a convolution).  y is static: its halo is sliced once from the global data.

Per-pixel arithmetic is the same as on one GPU, so x and z are bitwise identical to the
single-GPU engine; only the order in which the four diagnostic sums are added differs
(per-rank partial sums), which moves the relative improvements by a few ulps.

Transport: ``DistComm`` wraps a ``torch.distributed`` process group -- NCCL (= RCCL on
ROCm) with device buffers in production; any other backend (gloo) is host-staged, which
is what the multi-process tests on a single GPU use.  ``run_local`` drives several slabs
of one process (one GPU) with device-to-device halo copies for the parity tests.
"""

import ctypes
import os

import numpy as np
import torch
import torch.distributed as dist

from .. import _lib as L
from ..opt.engine import nmarch_taps
from .. import _ops as O


def row_split(n0, world, rank):
    """Balanced contiguous split of ``n0`` rows: (row0, rows) of ``rank``."""
    base, rem = divmod(int(n0), int(world))
    rows = base + (1 if rank < rem else 0)
    row0 = rank * base + min(rank, rem)
    return row0, rows


class DistComm:
    """Sum gathering and neighbour halo exchange over a torch.distributed group."""

    tunable = True  # a real transport: schedule choices may be timed through it

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.staged = dist.get_backend(group) != 'nccl'

        self._native = None

    def _peer(self, r):
        return r if self.group is None else dist.get_global_rank(self.group, r)

    def native(self):
        """An RCCL communicator over the same ranks for the native loop (pcs_slab2d_run), or
        None on a host-staged group or when RCCL could not be bound.  Collective: every
        rank of the group calls it (the unique id travels over the torch group)."""
        if self.staged or self.world == 1:
            return None
        if self._native is None:
            lib = L.gpu()
            ok = torch.tensor([int(lib.pcs_comm_available())], dtype=torch.int32, device='cuda')
            dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=self.group)
            if int(ok.item()) == 0:
                self._native = False
                return None
            nb = int(lib.pcs_comm_id_bytes())
            uid = (ctypes.c_ubyte * nb)()
            if self.rank == 0:
                L.check(lib.pcs_comm_unique_id(ctypes.cast(uid, ctypes.c_void_p)), 'pcs_comm_unique_id')
            t = torch.tensor(list(bytes(uid)), dtype=torch.uint8, device='cuda')
            dist.broadcast(t, src=self._peer(0), group=self.group)
            uid = (ctypes.c_ubyte * nb)(*t.cpu().tolist())
            h = ctypes.c_void_p()
            L.check(lib.pcs_comm_init(ctypes.cast(uid, ctypes.c_void_p), self.world, self.rank, ctypes.byref(h)),
                    'pcs_comm_init')
            self._native = h
        return self._native or None

    def rccl(self):
        """The in-library RCCL transport (RcclComm) over the same ranks, or None (host-staged
        group, one rank, or no RCCL).  Collective."""
        h = self.native()
        return RcclComm(h, self.rank, self.world, self) if h else None

    def close(self):
        if self._native:
            torch.cuda.synchronize()
            L.load().pcs_comm_destroy(self._native)
        self._native = None

    def allgather(self, src, dst):
        """dst[4 r : 4 r + 4] = src of rank r."""
        if self.world == 1:
            dst.copy_(src)
        elif self.staged:
            parts = [torch.empty_like(src, device='cpu') for _ in range(self.world)]
            dist.all_gather(parts, src.cpu(), group=self.group)
            dst.copy_(torch.cat(parts))
        else:
            dist.all_gather_into_tensor(dst, src, group=self.group)

    def allgather_start(self, src, dst):
        """allgather() without waiting: RCCL runs it on its own stream behind the work queued
        so far; the handle's wait() orders the current stream after it."""
        if self.world == 1 or self.staged:
            self.allgather(src, dst)
            return _Done()
        return _Works([dist.all_gather_into_tensor(dst, src, group=self.group, async_op=True)])

    def exchange_start(self, pairs):
        """exchange() without waiting (see allgather_start)."""
        if not pairs or self.staged:
            self.exchange(pairs)
            return _Done()
        ops = []
        for peer, lst in sorted(pairs.items()):
            for snd, rcv in lst:
                ops.append(dist.P2POp(dist.isend, snd, self._peer(peer), self.group))
                ops.append(dist.P2POp(dist.irecv, rcv, self._peer(peer), self.group))
        return _Works(dist.batch_isend_irecv(ops))

    def exchange(self, pairs):
        """pairs: {peer: [(send_view, recv_view), ...]}; the k-th send to a peer lands in the
        peer's k-th receive from us."""
        if not pairs:
            return
        if self.staged:
            if torch.cuda.is_available():
                torch.cuda.current_stream().synchronize()
            reqs, back = [], []
            for peer, lst in sorted(pairs.items()):
                for k, (s, r) in enumerate(lst):
                    sh = s.cpu()
                    rh = torch.empty_like(r, device='cpu')
                    reqs.append(dist.isend(sh, self._peer(peer), group=self.group, tag=k))
                    reqs.append(dist.irecv(rh, self._peer(peer), group=self.group, tag=k))
                    back.append((r, rh, sh))
            for q in reqs:
                q.wait()
            for r, rh, _ in back:
                r.copy_(rh)
            return
        ops = []
        for peer, lst in sorted(pairs.items()):
            for s, r in lst:
                ops.append(dist.P2POp(dist.isend, s, self._peer(peer), self.group))
                ops.append(dist.P2POp(dist.irecv, r, self._peer(peer), self.group))
        for q in dist.batch_isend_irecv(ops):
            q.wait()


class RcclComm:
    """Halo exchange and sums all-gather through the library's RCCL binding
    (pcs_halo_exchange / pcs_allgather_f64) instead of torch.distributed: plain
    stream-ordered launches, so a chunk of iterations (kernels + RCCL) can be captured into one
    hipGraph.  The *_start forms run on a side stream forked from the current one (event
    record / wait, capture-safe); the handle's wait() joins it back.  Same interface as
    DistComm for the engines."""

    tunable = True

    def __init__(self, handle, rank, world, owner=None):
        self.h, self.rank, self.world, self.owner = handle, int(rank), int(world), owner
        self.lib = L.gpu()
        self.side = torch.cuda.Stream()
        self._sets = {}

    def _halo_set(self, pairs):
        """pcs_halo_set of {peer: [(send, recv), ...]} (cached per pairs object: the engines
        build one per ping-pong parity)."""
        key = id(pairs)
        hs = self._sets.get(key)
        if hs is not None and hs[1] is pairs:
            return hs[0]
        lo, hi = pairs.get(self.rank - 1, []), pairs.get(self.rank + 1, [])
        n = max(len(lo), len(hi))
        if n > 4:
            raise ValueError('pcs_halo_exchange moves at most 4 buffers')
        h = L.HaloSet()
        h.nbuf = n
        for k in range(n):
            ref = (lo or hi)[k][0]
            h.bytes[k] = ref.numel() * ref.element_size()
            if lo:
                h.send_lo[k], h.recv_lo[k] = lo[k][0].data_ptr(), lo[k][1].data_ptr()
            if hi:
                h.send_hi[k], h.recv_hi[k] = hi[k][0].data_ptr(), hi[k][1].data_ptr()
        self._sets[key] = (h, pairs)
        return h

    def allgather(self, src, dst):
        L.check(self.lib.pcs_allgather_f64(self.h, self.world, L.ptr(src), L.ptr(dst), src.numel(), L.stream()),
                'pcs_allgather_f64')

    def exchange(self, pairs):
        if not pairs:
            return
        L.check(self.lib.pcs_halo_exchange(self.h, self.rank, self.world, ctypes.byref(self._halo_set(pairs)),
                                           L.stream()), 'pcs_halo_exchange')

    def _on_side(self, fn):
        cur = torch.cuda.current_stream()
        self.side.wait_stream(cur)
        with torch.cuda.stream(self.side):
            fn()
        return _SideJoin(self.side)

    def allgather_start(self, src, dst):
        return self._on_side(lambda: self.allgather(src, dst))

    def exchange_start(self, pairs):
        return self._on_side(lambda: self.exchange(pairs))

    def close(self):
        if self.owner is not None:
            self.owner.close()


class _SideJoin:
    """Handle of work queued on a side stream: wait() orders the current stream after it."""

    def __init__(self, side):
        self.side = side

    def wait(self):
        torch.cuda.current_stream().wait_stream(self.side)


class _Done:
    """Handle of a transfer that completed inside its start call (host-staged transport)."""

    def wait(self):
        pass


class _Works:
    """Handle of in-flight torch.distributed (NCCL = RCCL) operations: wait() makes the
    current stream wait for them (no host synchronisation)."""

    def __init__(self, works):
        self.works = works

    def wait(self):
        for w in self.works:
            w.wait()


class SlabLayout:
    """Row geometry of one rank's slab: arrays hold local rows [-h, rows + h) (C order,
    n1 columns); a buffer of `ncomp` components stacks them with stride (rows + 2h) n1."""

    def __init__(self, n0, n1, rank, world):
        self.n0, self.n1, self.rank, self.world = int(n0), int(n1), int(rank), int(world)
        self.row0, self.rows = row_split(n0, world, rank)

    def window(self, g, h):
        """Rows [row0 - h, row0 + rows + h) of a global n0*n1 array (zeros outside the image)."""
        n1 = self.n1
        out = torch.zeros((self.rows + 2 * h) * n1, dtype=g.dtype, device=g.device)
        lo, hi = max(0, self.row0 - h), min(self.n0, self.row0 + self.rows + h)
        d = lo - (self.row0 - h)
        out[d * n1:(d + hi - lo) * n1] = g[lo * n1:hi * n1]
        return out

    def rows_view(self, buf, h, r0, r1, comp=0):
        """Local rows [r0, r1) (own-row coordinates) of component `comp` of a halo'd buffer."""
        n1 = self.n1
        base = comp * (self.rows + 2 * h) * n1
        return buf[base + (r0 + h) * n1: base + (r1 + h) * n1]

    def halo_pairs(self, bufs):
        """bufs: [(buffer, h, comp[, d]), ...] -> {peer: [(send, recv), ...]}: own boundary rows go
        to the neighbour's halo, the neighbour's boundary rows fill ours -- the d <= h rows next to the
        own rows (default all h stored rows; d = 0 leaves the buffer out of the exchange)."""
        pairs = {}
        R = self.rows
        full = [(b[0], b[1], b[2], b[3] if len(b) > 3 else b[1]) for b in bufs]
        full = [(b, h, c, d) for b, h, c, d in full if d > 0]
        if self.rank > 0:
            pairs[self.rank - 1] = [(self.rows_view(b, h, 0, d, c), self.rows_view(b, h, -d, 0, c))
                                    for b, h, c, d in full]
        if self.rank < self.world - 1:
            pairs[self.rank + 1] = [(self.rows_view(b, h, R - d, R, c), self.rows_view(b, h, R, R + d, c))
                                    for b, h, c, d in full]
        return pairs


class SlabPDS2D:
    """One rank's slab of a fused 2-D PDS problem.

    ``spec`` is the global problem's engine spec (``PDS._fused_spec()``: shape, H/G kinds,
    data shift, convolution); ``x0`` / ``z0`` are the global starting points (z0 stacked
    as [D0 z; D1 z], each ``n0*n1``).  Only this rank's rows (+ halos) are kept.
    """

    def __init__(self, spec, dtype, tau, sigma, rho, x0, z0, rank, world, comm=None, chunk=16, native='auto',
                 overlap=True, depth=1):
        self.lib = L.gpu()
        self.comm = comm
        self.rank, self.world = int(rank), int(world)
        self.dtype = dtype
        n0, n1 = spec['shape']
        self.n0, self.n1 = n0, n1
        self.lay = lay = SlabLayout(n0, n1, rank, world)
        self.row0, self.rows = lay.row0, lay.rows
        fk = spec['fkind']
        kk = spec.get('kkind', L.PCS_K_GRAD_FORWARD)
        nc = spec.get('ncomp', 2)
        self.ncomp = nc
        a = L.PdsArgs()
        a.dtype = L.PCS_F32 if dtype == torch.float32 else L.PCS_F64
        a.hkind, a.gkind = spec['hkind'], spec['gkind']
        a.n0, a.n1, a.row0, a.rows = n0, n1, self.row0, self.rows
        a.tau, a.sigma, a.rho, a.lam = float(tau), float(sigma), float(rho), spec['lam']
        a.step0, a.step1 = spec['steps']
        a.seg_a, a.seg_b = spec['seg']
        a.kkind, a.edge = kk, int(spec.get('edge', True))
        a.w0, a.w1 = spec.get('weights', (1.0, 1.0))
        dev = torch.device('cuda', torch.cuda.current_device())
        fwd = kk == L.PCS_K_GRAD_FORWARD
        half, mode = 0, 'pointwise'
        conv = spec.get('conv')
        if fk in (L.PCS_F_SEPCONV, L.PCS_F_GRADBUF) and conv is not None:
            sep = conv.separable(rtol=2e-7 if dtype == torch.float32 else 1e-13)
            if sep is not None and (fwd or sep[2] <= 7):
                # forward K: the (normal-operator) march kernels; other K: the fused normal-operator
                # march (fp32 pds_nmarch.hpp, fp64 pds_nm64.hip) or N x by the in-plane normal-operator
                # pass into a buffer, then the general-stencil march step
                mode = 'sep' if fwd else 'sep_normal'
                t0, t1, half = sep
                self.taps = [torch.as_tensor(t0).to(device=dev, dtype=dtype),
                             torch.as_tensor(t1).to(device=dev, dtype=dtype)]
                a.taps0, a.taps1 = self.taps[0].data_ptr(), self.taps[1].data_ptr()
                a.half = half
                fk = L.PCS_F_SEPCONV
            else:
                # general (non-separable) PSF: grad F = Conv^T (Conv x - y) by two packed-plan
                # correlations over the stored rows inside the step call (PCS_F_CONV2D)
                mode = 'conv2d'
                plans = (conv.plan(dtype, False), conv.plan(dtype, True))
                if plans[0] is None or plans[1] is None:
                    raise ValueError('row-slab PDS: PSF wider than the direct correlation tiers (31 taps)')
                self.plans = plans
                a.conv_fwd, a.conv_adj, a.conv_tier = plans[0][1].data_ptr(), plans[1][1].data_ptr(), plans[0][0]
                fk = L.PCS_F_CONV2D
        elif fk not in (L.PCS_F_NULL, L.PCS_F_DENOISE):
            raise ValueError(f'row-slab PDS does not support fkind {fk}')
        a.fkind = fk
        self.fkind, self.mode = fk, mode
        # halo depths: the reach of the step (and of the gradient passes it runs on the stored rows)
        if mode == 'sep':
            hx = int(self.lib.pcs_pds2d_halo_x(half))
            hy = (hx - 1) // 2 + 1
        elif mode == 'sep_normal':
            hx = hy = 2 + 2 * (3 if half <= 3 else 7)
        elif mode == 'conv2d':
            hx = hy = max(a.conv_tier + 1, 1 if fwd else 2)
        else:
            hx, hy = (1, 1) if fwd else (2, 2)
        hz = 1 if fwd else 4
        # communication-avoiding depth (pcs_slab2d_deep_*): halos `depth` iterations deep, exchanged once per
        # chunk of `depth` iterations; iteration j of a chunk also computes (depth - j) * reach rows of each
        # halo, reach = the rows one iteration reads past its own (x and z), rounded up to even
        self.depth = int(depth)
        if not 1 <= self.depth <= L.DEEP_MAX:
            raise ValueError(f'depth must be in 1..{L.DEEP_MAX}')
        r = max(hx, hz)
        self.reach = r + r % 2
        if self.depth > 1:
            if mode not in ('pointwise', 'sep'):
                raise ValueError(f'deep halos need the banded row-marching step (F mode {mode!r} has none)')
            e = (self.depth - 1) * self.reach
            hx, hy, hz = hx + e, hy + e, hz + e
        if world > 1 and self.rows < max(hx, hy, hz):
            raise ValueError(f'slab of {self.rows} rows is thinner than its halo ({max(hx, hy, hz)} rows)')
        self.hx, self.hy, self.hz = hx, hy, hz
        self.nbuf = max(2, self.depth)
        a.halo_x, a.halo_y, a.halo_z = hx, hy, hz
        N = n0 * n1
        # deep halos: the virtual slab of an iteration whose extension is clipped on one side moves each
        # array's view by up to (depth - 1) reach / 2 rows (pcs_slab2d_deep_*), so the buffers carry that many
        # zero rows of padding before and after their stored rows: the view's surplus loads stay in memory
        self.pad = (self.depth - 1) * self.reach // 2
        self.X = [self._padded(lay.window(O.to_dev(x0, dtype), hx)) for _ in range(self.nbuf)]
        z0d = O.to_dev(z0, dtype)
        self.Z = [self._padded(torch.cat([lay.window(z0d[c * N:(c + 1) * N], hz) for c in range(nc)]))
                  for _ in range(self.nbuf)]
        if fk in (L.PCS_F_DENOISE, L.PCS_F_SEPCONV, L.PCS_F_CONV2D):
            self.y = self._padded(lay.window(-O.to_dev(spec['shift'], dtype), hy))  # y = -shift, exactly
            a.y = self.y.data_ptr()
        if mode in ('sep_normal', 'conv2d'):
            self.Gb = torch.zeros_like(self.X[0])  # grad F on the stored rows (x's layout)
            a.gbuf = self.Gb.data_ptr()
        if mode == 'conv2d':
            self.R = torch.zeros_like(self.X[0])
            a.rbuf = self.R.data_ptr()
        f64 = dtype == torch.float64
        if mode == 'sep_normal' or (mode == 'sep' and half <= 7 and os.environ.get('PCS_NMARCH', '1') != '0'):
            # Conv^T y in fp64 on this rank's window only (own rows + the y halo), from the y rows
            # within the PSF's reach of it -- exact, since the sub-image's zero boundary falls where
            # the image's does or beyond the reach
            if half <= 7:
                # 'sep_normal' too: backward / centred K run the fused normal-operator march when the
                # library takes it (no N x pass, no gradient buffer read); fp64 every Gradient K
                # (pds_nm64.hip, its N tables in fp64)
                self.ntaps = torch.as_tensor(nmarch_taps(t0, t1, half, np.float64 if f64 else np.float32)).to(dev)
                a.ntaps = self.ntaps.data_ptr()
            self.cty = self._padded(self._cty_window(spec, hy).to(dtype).contiguous())
            a.cty = self.cty.data_ptr()
        self.nm_fused = False
        if mode in ('sep_normal', 'sep') and getattr(self, 'ntaps', None) is not None:
            # the fused normal-operator march (one launch, no gradient buffer) when the library runs it
            # for these arguments (the iterate pointers are bound per parity later: placeholders for the
            # query, never written)
            saved = (a.gbuf, a.x, a.xn, a.z, a.zn, a.partials)
            ph = self.X[0].data_ptr()
            a.gbuf, a.x, a.xn, a.z, a.zn, a.partials = None, ph, ph, ph, ph, ph
            self.nm_fused = self.lib.pcs_pds2d_path(ctypes.byref(a)) in L.PCS_PATH_FUSED_NORMAL
            a.gbuf, a.x, a.xn, a.z, a.zn, a.partials = saved
        self.nblocks = int(self.lib.pcs_pds2d_nblocks(ctypes.byref(a)))
        if self.nblocks < 0:
            kname = {L.PCS_K_GRAD_FORWARD: 'forward Gradient', L.PCS_K_GRAD_BACKWARD: 'backward Gradient',
                     L.PCS_K_GRAD_CENTERED: 'centered Gradient', L.PCS_K_LAPLACIAN: 'Laplacian'}.get(kk, str(kk))
            raise ValueError(f'row-slab PDS: no fused slab kernel for K = {kname}, dtype {dtype}, image {n0}x{n1} '
                             f'(F mode {mode!r}); run this problem on one GPU (PDS.iterate)')
        self.partials = torch.empty(self.nblocks * 4, dtype=torch.float64, device=dev)
        a.partials = self.partials.data_ptr()
        a.hist, a.ws = None, None
        self.sums = torch.zeros(4, dtype=torch.float64, device=dev)
        self.gathered = torch.zeros(4 * world, dtype=torch.float64, device=dev)
        self.ctrl = torch.zeros(int(self.lib.pcs_ctrl_bytes()) // 8, dtype=torch.float64, device=dev)
        a.ctrl = self.ctrl.data_ptr()
        self.args = [self._args_for(a, p) for p in range(self.nbuf)]
        self.halos = [lay.halo_pairs([(self.X[q], hx, 0)] + [(self.Z[q], hz, c) for c in range(nc)])
                      for q in range(self.nbuf)]
        self.hist = None
        self.chunk = max(1, int(chunk))
        # native loop (pcs_slab2d_run): one C call per chunk instead of five Python-issued
        # operations per iteration; needs an RCCL communicator when world > 1
        # native='local' (depth > 1, tests): the deep plan without a communicator, driven with the other ranks'
        # plans of the same process by run_local_deep
        self.local = native == 'local'
        if self.local:
            native = True
        elif native == 'auto':
            native = world == 1 or (comm is not None and comm.native() is not None)
        elif native and world > 1 and (comm is None or comm.native() is None):
            raise ValueError('native slab loop needs an RCCL (nccl backend) process group')
        self.native = bool(native)
        if self.depth > 1 and not self.native:
            raise ValueError('deep halos run in the native loop only (pcs_slab2d_deep_run): an RCCL process group')
        self._deep = None
        self._b = 0
        # the gradient passes of 'conv2d' / 'sep_normal' run once per iteration over the whole slab:
        # no banded (overlapped) schedule for them
        self.overlap = bool(overlap) and (mode in ('pointwise', 'sep') or self.nm_fused)
        self._plan = None
        self._plan_key = None
        # multi-GPU native loop: chunks of 32 iterations replayed from a hipGraph (kernels, events
        # and RCCL calls; world-1 C3 probe: serial schedule equal, overlapped 0.164 -> 0.158 ms per
        # iteration, profiles/r2_slab_graph_probe.txt); PCS_SLAB_GRAPH=<even chunk> sets it, 0 = eager
        gc = int(os.environ.get('PCS_SLAB_GRAPH', '32' if world > 1 else '0') or 0)
        self.graph_chunk = (gc + gc % 2) if self.native and gc > 0 else 0
        self._graph = None

    def _padded(self, t):
        """t inside a buffer with self.pad zero rows before and after it (the view keeps the storage alive);
        t itself when there is no padding."""
        if self.pad == 0:
            return t
        p = self.pad * self.n1
        buf = torch.zeros(t.numel() + 2 * p, dtype=t.dtype, device=t.device)
        buf[p:p + t.numel()] = t
        return buf[p:p + t.numel()]

    def _cty_window(self, spec, h):
        """Rows [row0 - h, row0 + rows + h) of Conv^T y (fp64, zeros outside the image), computed on
        the sub-image of y rows within the PSF's reach of that window (never the global image)."""
        from ..linop.conv import Convolve2DOp
        conv, n0, n1 = spec['conv'], self.n0, self.n1
        reach = max(conv.kh, conv.kw)
        wlo, whi = max(0, self.row0 - h - reach), min(n0, self.row0 + self.rows + h + reach)
        shift = spec['shift']
        ys = shift.reshape(n0, n1)[wlo:whi] if isinstance(shift, torch.Tensor) else \
            np.asarray(shift).reshape(n0, n1)[wlo:whi]
        yw = -O.to_dev(ys, torch.float64)
        ctw = Convolve2DOp(n1 * (whi - wlo), conv.filter, (whi - wlo, n1))._adj(yw)
        out = torch.zeros((self.rows + 2 * h) * n1, dtype=torch.float64, device=ctw.device)
        lo, hi = max(0, self.row0 - h), min(n0, self.row0 + self.rows + h)
        d = lo - (self.row0 - h)
        out[d * n1:(d + hi - lo) * n1] = ctw[(lo - wlo) * n1:(hi - wlo) * n1]
        return out

    @classmethod
    def from_pds(cls, pds, comm, rank=None, world=None, chunk=16, native='auto', overlap=True, depth=1):
        """This rank's slab of a PDS problem built with the public API on the global image
        (every rank builds the same problem, as a single-host script would)."""
        spec = pds._fused_spec()
        if spec is None:
            raise ValueError('problem does not match the fused 2-D PDS engine (see opt/engine.match_pds2d)')
        rank = comm.rank if rank is None else rank
        world = comm.world if world is None else world
        return cls(spec, pds._compute_dtype(), pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, rank, world, comm, chunk,
                   native, overlap, depth)

    def _args_for(self, a, p):
        """The step from buffer set p to set p + 1 (mod nbuf; the ping-pong when nbuf == 2)."""
        b = L.PdsArgs()
        ctypes.pointer(b)[0] = a
        q = (p + 1) % self.nbuf
        b.x, b.xn = self.X[p].data_ptr(), self.X[q].data_ptr()
        b.z, b.zn = self.Z[p].data_ptr(), self.Z[q].data_ptr()
        return b

    # ---- native loop
    def _halo_set(self, q):
        """pcs_halo_set of the buffers X[q], Z[q] (written by the step of parity 1 - q)."""
        hs = L.HaloSet()
        pairs = self.halos[q]
        lst = pairs.get(self.rank - 1, []) or pairs.get(self.rank + 1, [])
        hs.nbuf = len(lst)
        for side, peer in (('lo', self.rank - 1), ('hi', self.rank + 1)):
            for k, (snd, rcv) in enumerate(pairs.get(peer, [])):
                getattr(hs, 'send_' + side)[k] = snd.data_ptr()
                getattr(hs, 'recv_' + side)[k] = rcv.data_ptr()
                hs.bytes[k] = snd.numel() * snd.element_size()
        return hs

    def _native_plan(self):
        if self.hist is None:
            self.hist = torch.full((2,), float('nan'), dtype=torch.float64, device=self.X[0].device)
        key = (self.hist.data_ptr(), self.overlap)
        if self._plan is not None and self._plan_key == key:
            return self._plan
        self._destroy_plan()
        d = L.Slab2DDesc()
        d.world, d.rank = self.world, self.rank
        for p in (0, 1):
            d.step[p] = self.args[p]
            d.halo[p] = self._halo_set(1 - p)
        d.ctrl, d.hist = self.ctrl.data_ptr(), self.hist.data_ptr()
        d.band = self.hx
        d.overlap = int(self.overlap)
        h = ctypes.c_void_p()
        comm = self.comm.native() if self.world > 1 else None
        L.check(self.lib.pcs_slab2d_create(ctypes.byref(d), comm, ctypes.byref(h)), 'pcs_slab2d_create')
        self._desc = d  # keeps the pointers' owners' layout alive with the plan
        self._plan, self._plan_key = h, key
        return h

    def _deep_plan(self):
        """The communication-avoiding plan (pcs_slab2d_deep_create) of a depth > 1 slab."""
        if self.hist is None:
            self.hist = torch.full((2,), float('nan'), dtype=torch.float64, device=self.X[0].device)
        key = (self.hist.data_ptr(),)
        if self._deep is not None and self._deep_key == key:
            return self._deep
        self._destroy_plan()
        d = L.SlabDeepDesc()
        d.world, d.rank, d.depth, d.nbuf, d.reach = self.world, self.rank, self.depth, self.nbuf, self.reach
        d.local = int(self.local)
        for b in range(self.nbuf):
            d.step[b] = self.args[b]
            d.halo[b] = self._halo_set(b)
        d.ctrl, d.hist = self.ctrl.data_ptr(), self.hist.data_ptr()
        h = ctypes.c_void_p()
        comm = self.comm.native() if self.world > 1 and not self.local else None
        L.check(self.lib.pcs_slab2d_deep_create(ctypes.byref(d), comm, ctypes.byref(h)), 'pcs_slab2d_deep_create')
        self._deep_desc = d
        self._deep, self._deep_key = h, key
        return h

    def _destroy_plan(self):
        self._graph = None  # captured against this plan's streams, events and buffers
        if self._plan is not None:
            torch.cuda.synchronize()
            L.load().pcs_slab2d_destroy(self._plan)
            self._plan = None
        if getattr(self, '_deep', None) is not None:
            torch.cuda.synchronize()
            L.load().pcs_slab2d_deep_destroy(self._deep)
            self._deep = None

    def overlapped(self):
        """True when the native loop overlaps the halo exchange with the interior band."""
        return self.native and bool(self.lib.pcs_slab2d_overlapped(self._native_plan()))

    def __del__(self):
        try:
            self._destroy_plan()
        except Exception:
            pass

    # ---- one iteration, split in phases (run_local interleaves them across slabs)
    def _compute(self, p, split=False):
        st = L.stream()
        if not split:
            L.check(self.lib.pcs_pds2d_step(ctypes.byref(self.args[p]), st), 'pcs_pds2d_step')
            L.check(self.lib.pcs_reduce_partials(L.ptr(self.partials), self.nblocks, L.ptr(self.sums), st),
                    'pcs_reduce_partials')
            return
        # the native loop's overlapped schedule, serialised: boundary bands, then the interior
        R, b = self.rows, self.hx
        bands = [(0, b, R - b, R), (b, R - b, R - b, R - b)]
        a = L.PdsArgs()
        ctypes.pointer(a)[0] = self.args[p]
        nbs = [int(self.lib.pcs_pds2d_nblocks_bands(ctypes.byref(a), *bd)) for bd in bands]
        if min(nbs) < 0:
            raise ValueError('banded step needs the row-marching kernels and rows > 2 * halo')
        if self.partials.numel() < 4 * sum(nbs):
            self.partials = torch.empty(4 * sum(nbs), dtype=torch.float64, device=self.partials.device)
        off = 0
        for bd, nb in zip(bands, nbs):
            a.partials = self.partials.data_ptr() + 8 * off
            L.check(self.lib.pcs_pds2d_step_bands(ctypes.byref(a), *bd, st), 'pcs_pds2d_step_bands')
            off += 4 * nb
        L.check(self.lib.pcs_reduce_partials(L.ptr(self.partials), sum(nbs), L.ptr(self.sums), st),
                'pcs_reduce_partials')

    def _finalize(self):
        L.check(self.lib.pcs_pds_reduce_finalize(L.ptr(self.gathered), self.world, L.ptr(self.ctrl), L.ptr(self.hist),
                                                 L.stream()), 'pcs_pds_reduce_finalize')

    def iteration(self, p):
        if self.world == 1:  # one slab = the whole image: no transport
            st = L.stream()
            L.check(self.lib.pcs_pds2d_step(ctypes.byref(self.args[p]), st), 'pcs_pds2d_step')
            L.check(self.lib.pcs_pds_reduce_finalize(L.ptr(self.partials), self.nblocks, L.ptr(self.ctrl),
                                                     L.ptr(self.hist), st), 'pcs_pds_reduce_finalize')
            return
        self._compute(p)
        self.comm.allgather(self.sums, self.gathered)
        self._finalize()
        self.comm.exchange(self.halos[1 - p])

    # ---- loops
    def init_loop(self, max_iter, min_iter, accuracy_threshold, has_dual=True):
        total = max(min_iter, max_iter) + 1
        hist_len = 2 * total + 2
        if self.hist is None or self.hist.numel() < hist_len:
            self.hist = torch.empty(hist_len, dtype=torch.float64, device=self.X[0].device)
        self.hist.fill_(float('nan'))
        L.check(self.lib.pcs_ctrl_init2(L.ptr(self.ctrl), int(min_iter), int(max_iter), float(accuracy_threshold),
                                        int(has_dual), int(self.hist.numel()), L.stream()), 'pcs_ctrl_init2')
        self._p = 0
        self._b = 0
        return total

    def advance(self, k):
        """Enqueue k iterations (no host synchronisation, except the one-off schedule trial)."""
        if self.depth > 1 or self.local:  # chunks of `depth` iterations per halo exchange
            if k:
                L.check(self.lib.pcs_slab2d_deep_run(self._deep_plan(), int(k), self._b, L.stream()),
                        'pcs_slab2d_deep_run')
                self._b = (self._b + int(k)) % self.nbuf
            return
        if self.native:
            if (not getattr(self, '_tuned', False) and self.world > 1 and self.overlap and k >= 8
                    and getattr(self.comm, 'tunable', False)):
                k -= self._autotune()
            if self.graph_chunk and k >= self.graph_chunk:
                k = self._replay_graph(k)
            if k:
                L.check(self.lib.pcs_slab2d_run(self._native_plan(), int(k), self._p, L.stream()), 'pcs_slab2d_run')
                self._p ^= int(k) & 1
            return
        for _ in range(k):
            self.iteration(self._p)
            self._p ^= 1

    def _replay_graph(self, k):
        """PCS_SLAB_GRAPH=<chunk>: the native loop's chunk (kernels, events, RCCL) captured into a
        hipGraph and replayed; returns the iterations left for eager launches.  Every rank must
        hold a graph or none (captured RCCL calls pair across ranks): agreed collectively, a
        failed capture anywhere leaves every rank on the eager native loop."""
        c = self.graph_chunk
        if self._p == 1:  # graphs start at parity 0
            L.check(self.lib.pcs_slab2d_run(self._native_plan(), 1, 1, L.stream()), 'pcs_slab2d_run')
            self._p, k = 0, k - 1
        if self._graph is None:
            plan = self._native_plan()
            torch.cuda.synchronize()
            g, ok = torch.cuda.CUDAGraph(), True
            try:
                with torch.cuda.graph(g):
                    L.check(self.lib.pcs_slab2d_run(plan, c, 0, L.stream()), 'pcs_slab2d_run')
            except Exception:  # noqa: BLE001 -- torch's capture errors and HipError alike: every rank
                # must reach the flag all-gather below, or the others block in RCCL
                ok, g = False, None
                torch.cuda.synchronize()
            if self.world > 1:
                flag = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=self.sums.device)
                allf = torch.zeros(self.world, dtype=torch.float64, device=self.sums.device)
                self.comm.allgather(flag, allf)
                ok = bool(allf.min().item() > 0)
            if not ok:
                self.graph_chunk = 0
                return k
            self._graph = g
        while k >= c:
            self._graph.replay()
            k -= c
        return k

    def _autotune(self):
        """Serial or overlapped native schedule: which is faster depends on the RCCL latency of
        the per-iteration exchange and all-gather (a few hundred KB: latency, not bytes) against
        the cross-stream synchronisation the overlap costs.  Time 3 iterations of
        each through the real transport (after 2 untimed) and keep the faster, max over ranks.
        Both schedules give bitwise the same iterates.  Returns the iterations used."""
        L.check(self.lib.pcs_slab2d_run(self._native_plan(), 2, self._p, L.stream()), 'pcs_slab2d_run')
        times = []
        for ov in (False, True):
            self.overlap = ov
            plan = self._native_plan()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            L.check(self.lib.pcs_slab2d_run(plan, 3, self._p, L.stream()), 'pcs_slab2d_run')
            e1.record()
            torch.cuda.synchronize()
            self._p ^= 1
            times.append(e0.elapsed_time(e1) / 3)
        dev = self.sums.device
        mine = torch.tensor(times + [0.0, 0.0], dtype=torch.float64, device=dev)
        allt = torch.zeros(4 * self.world, dtype=torch.float64, device=dev)
        self.comm.allgather(mine, allt)
        worst = allt.view(self.world, 4).max(dim=0).values
        self.overlap = float(worst[1]) < float(worst[0])
        self.tune_ms = [float(worst[0]), float(worst[1])]
        self._native_plan()
        self._tuned = True
        return 8

    def stopped(self):
        return int(self.ctrl.view(torch.int32)[1].item()) != 0

    def iterations(self):
        return int(self.ctrl.view(torch.int32)[0].item())

    def result(self):
        """(n_iter, own rows of x, own rows of z (2 components), hist [n, 2])."""
        torch.cuda.synchronize()
        n = self.iterations()
        q = n % self.nbuf
        x = self.lay.rows_view(self.X[q], self.hx, 0, self.rows).clone()
        z = torch.cat([self.lay.rows_view(self.Z[q], self.hz, 0, self.rows, c) for c in range(self.ncomp)])
        h = self.hist[:2 * n].cpu().numpy().reshape(n, 2) if n > 0 else np.zeros((0, 2))
        return n, x, z, h

    def run(self, max_iter, min_iter, accuracy_threshold, has_dual=True):
        """The reference loop (solver.py:65-76) across all ranks: every rank holds the
        same stop flag, so every rank leaves after the same iteration."""
        total = self.init_loop(max_iter, min_iter, accuracy_threshold, has_dual)
        done = 0
        while done < total:
            k = min(self.chunk, total - done)
            self.advance(k)
            done += k
            if self.stopped():
                break
        return self.result()

    def time_step_kernel(self, n):
        """Average duration (ms) of the slab step kernel over n eager launches (HIP events
        on the launching stream); leaves x/z advanced by n iterations of ping-pong."""
        st = torch.cuda.current_stream()
        L.check(self.lib.pcs_ctrl_init2(L.ptr(self.ctrl), n + 1, n + 1, -1.0, 1, 2 * n + 6, L.stream()),
                'pcs_ctrl_init2')
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        for i in range(n):
            evs[i][0].record(st)
            L.check(self.lib.pcs_pds2d_step(ctypes.byref(self.args[i % 2]), L.stream()), 'pcs_pds2d_step')
            evs[i][1].record(st)
        torch.cuda.synchronize()
        return float(np.mean([s.elapsed_time(e) for s, e in evs]))


def comm_probe(eng, reps=5):
    """Where one rank's multi-GPU iteration spends its time: the compute alone (the step +
    the partial-sum reduction on the whole slab), the sums all-gather alone and the halo
    exchange alone, each re-run `reps` times on the current iterate and timed by HIP events
    on the current stream (max over ranks).  Every phase is idempotent there: compute(p)
    rewrites the parity-(1 - p) buffers from the parity-p ones, the all-gather and the
    exchange re-send values already in place -- the iterate and the loop control are left as
    they were.  `eng`: a SlabPDS2D or a multi-rank PDS3DEngine (the loop being
    sharded is pycsou/core/solver.py:55-76).  Returns a dict of ms per phase, the halo bytes one
    side sends per iteration and the exchange's achieved GB/s per side."""
    if eng.world == 1 or eng.comm is None:
        return None
    comm = eng.comm
    if isinstance(comm, DistComm) and getattr(eng, 'native', False):
        comm = comm.rccl() or comm  # the 2-D native loop moves its halos through the library's RCCL binding
    p = eng._p
    pairs = eng.halos[p]
    side = next(iter(pairs.values()), [])
    halo = int(sum(s.numel() * s.element_size() for s, _ in side))
    phases = {
        'compute_ms': lambda: eng._compute(p),
        'allgather_ms': lambda: comm.allgather(eng.sums, eng.gathered),
        'exchange_ms': lambda: comm.exchange(pairs),
    }
    out = []
    for name, fn in phases.items():
        fn()  # untimed once
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) / reps)
    dev = eng.sums.device
    mine = torch.tensor(out + [0.0], dtype=torch.float64, device=dev)
    allt = torch.zeros(4 * eng.world, dtype=torch.float64, device=dev)
    comm.allgather(mine, allt)
    worst = allt.view(eng.world, 4).max(dim=0).values[:3].tolist()
    res = {k: round(v, 4) for k, v in zip(phases, worst)}
    res['halo_bytes_per_side'] = halo
    res['exchange_GBps_per_side'] = round(halo / (res['exchange_ms'] * 1e-3) / 1e9, 2) if res['exchange_ms'] > 0 else None
    res['reps'] = reps
    return res


def run_local(slabs, max_iter, min_iter, accuracy_threshold, split=False):
    """Drive all slabs of one image inside one process (device-to-device halo copies);
    the per-iteration phase order is the distributed one.  ``split``: each slab's step runs
    as the boundary-bands launch + the interior launch (pcs_pds2d_step_bands), as in the
    native loop's overlapped schedule."""
    total = None
    for s in slabs:
        total = s.init_loop(max_iter, min_iter, accuracy_threshold)
    by_rank = {s.rank: s for s in slabs}
    for i in range(total):
        p = i % 2
        for s in slabs:
            s._compute(p, split)
        g = torch.cat([s.sums for s in slabs])
        for s in slabs:
            s.gathered.copy_(g)
            s._finalize()
        for s in slabs:
            for peer, lst in s.halos[1 - p].items():
                back = by_rank[peer].halos[1 - p][s.rank]
                for (_, recv), (send, _) in zip(lst, back):
                    recv.copy_(send)
        if (i + 1) % 8 == 0 and slabs[0].stopped():
            break
    return [s.result() for s in slabs]


def run_local_deep(slabs, max_iter, min_iter, accuracy_threshold, chunk=None):
    """All deep-halo slabs of one image inside one process through the native chunk loop with a
    device-copy transport (pcs_slab2d_deep_run_local: the same launches, loop control and halo rows as
    pcs_slab2d_deep_run, the all-gather and the exchange as copies); the host checks the stop flag
    once per `chunk` iterations (default: 4 chunks of the depth)."""
    slabs = sorted(slabs, key=lambda s: s.rank)
    total = None
    for s in slabs:
        total = s.init_loop(max_iter, min_iter, accuracy_threshold)
    lib = slabs[0].lib
    plans = (ctypes.c_void_p * len(slabs))(*[s._deep_plan().value for s in slabs])
    step = chunk or 4 * slabs[0].depth
    done = 0
    while done < total:
        m = min(step, total - done)
        L.check(lib.pcs_slab2d_deep_run_local(plans, len(slabs), m, slabs[0]._b, L.stream()),
                'pcs_slab2d_deep_run_local')
        for s in slabs:
            s._b = (s._b + m) % s.nbuf
        done += m
        if slabs[0].stopped():
            break
    return [s.result() for s in slabs]


def gather_rows(local, n0, n1, world, rank, comm):
    """Assemble the global n0*n1 array from every rank's own rows (all ranks get it)."""
    if world == 1:
        return local
    counts = [row_split(n0, world, r)[1] * n1 for r in range(world)]
    mx = max(counts)
    buf = torch.zeros(mx, dtype=local.dtype, device=local.device)
    buf[:local.numel()] = local
    if comm.staged:
        parts = [torch.empty(mx, dtype=local.dtype) for _ in range(world)]
        dist.all_gather(parts, buf.cpu(), group=comm.group)
        parts = [t.to(local.device) for t in parts]
    else:
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf, group=comm.group)
    return torch.cat([t[:c] for t, c in zip(parts, counts)])

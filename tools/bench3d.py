"""3-D TV-deconvolution throughput on one GPU.

C4: 512^3 fp32, C5: 1024^3 fp64 -- a piecewise-constant phantom blurred by a 15-tap Gaussian
(sigma 2) along each axis (three Convolve1D, the reference's 3-D blur), y = h*x + 0.01 N(0,1),
PDS with K = Gradient(kind='forward') in 3-D and H = 0.05 * L21Norm (3 components), built
through the public API and run by PDS3DEngine (hipGraph chunks).  Prints one JSON line:
it/s, ms per iteration, the update kernel's mean duration and the algorithmic rates.

  python tools/bench3d.py --size 512 --dtype f32 --steps 20 --warmup 4

--rank-of W: time ONE rank's share of a W-GPU plane-slab run on this GPU (a middle rank:
both halos), with a transport that moves nothing (halo planes stay stale; per-iteration
compute is what is measured), in the serial order and in the banded order of the multi-GPU
loop.  The halo bytes per side per iteration are printed beside it.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pycsou_amd import _lib as L  # noqa: E402


def build(n, dtype, seed=0, kind='forward'):
    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L21Norm
    from pycsou_amd.linop.conv import Convolve1D
    from pycsou_amd.linop.diff import Gradient
    from pycsou_amd.opt.proxalgs import PDS
    shape = (n, n, n)
    N = n ** 3
    g = torch.Generator(device='cuda').manual_seed(seed)
    xs = torch.zeros(shape, dtype=dtype, device='cuda')
    rng = np.random.default_rng(seed)
    for _ in range(32):
        lo = rng.integers(0, n, 3)
        hi = np.minimum(n, lo + rng.integers(n // 16, n // 3, 3))
        xs[lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2]] = float(rng.uniform(0, 1))
    r = np.arange(15) - 7
    taps = np.exp(-0.5 * (r / 2.0) ** 2)
    taps /= taps.sum()
    C = None
    for ax in range(3):
        Ci = Convolve1D(N, taps, reshape_dims=shape, axis=ax)
        Ci.lipschitz_cst = Ci.diff_lipschitz_cst = 1.0
        C = Ci if C is None else Ci * C
    C.lipschitz_cst = C.diff_lipschitz_cst = 1.0
    y = C(xs.reshape(-1)) + 0.01 * torch.randn(N, generator=g, device='cuda', dtype=dtype)
    del xs
    print('  blurred data ready', flush=True)
    K = Gradient(shape=shape, kind=kind)
    K.lipschitz_cst = K.diff_lipschitz_cst = (float(np.sqrt(sum(4 * np.sin(np.pi * (n - 1) / (2 * n)) ** 2
                                                                for _ in range(3)))) if kind == 'forward' else 3.0)
    F = (1 / 2) * SquaredL2Loss(dim=N, data=y) * C
    H = 0.05 * L21Norm(dim=3 * N, groups=np.tile(np.arange(N), 3))
    print('  functionals ready', flush=True)
    return PDS(dim=N, F=F, H=H, K=K, x0=torch.zeros(N, dtype=dtype, device='cuda'),
               z0=torch.zeros(3 * N, dtype=dtype, device='cuda'), verbose=None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--size', type=int, default=512)
    ap.add_argument('--dtype', default='f32', choices=['f32', 'f64'])
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=4)
    ap.add_argument('--rank-of', type=int, default=0)
    ap.add_argument('--kind', default='forward', choices=['forward', 'backward', 'centered'])
    ap.add_argument('--one-gpu-ms', type=float, default=0.0,
                    help='--rank-of: the single-GPU ms per iteration of the same volume (the link-rate model '
                         'prints the speed-up it implies)')
    args = ap.parse_args()
    if args.rank_of > 1:
        return rank_share(args)
    torch.cuda.set_device(0)
    dtype = torch.float32 if args.dtype == 'f32' else torch.float64
    from pycsou_amd.opt.engine3d import PDS3DEngine
    t0 = time.time()
    pds = build(args.size, dtype, kind=args.kind)
    spec = pds._fused_spec()
    assert spec is not None and spec['ndim'] == 3
    chunk = 2
    eng = PDS3DEngine(spec, dtype, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, chunk=chunk)
    del pds
    K = args.steps + args.steps % 2
    W = args.warmup + args.warmup % 2
    eng.init_loop(W + K + 4, W + K + 4, -1.0)
    eng.advance(W)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    eng.advance(K)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / K
    assert eng.iterations() == W + K
    kms = eng.time_step_kernel(min(K, 10))
    N = args.size ** 3
    elem = 4 if dtype == torch.float32 else 8
    alg = 9 * N * elem  # (2d+3) N words, d = 3
    print(json.dumps({'workload': f'3-D TV-deconv {args.size}^3 {args.dtype}, 15-tap Gaussian per axis, '
                                  f'0.05*L21, PDS3DEngine', 'it_per_s': round(1e3 / ms, 3), 'ms_per_iter': round(ms, 4),
                      'update_kernel_ms': round(kms, 4), 'alg_bytes_per_iter': alg,
                      'iteration_GBps': round(alg / (ms * 1e-3) / 1e9, 1),
                      'update_kernel_GBps': round(alg / (kms * 1e-3) / 1e9, 1), 'setup_s': round(time.time() - t0, 1)}))


class NullComm:
    """Transport stand-in for timing one rank alone: no data moves."""
    staged = True

    def __init__(self, rank, world):
        self.rank, self.world = rank, world

    def allgather(self, src, dst):
        dst[:4].copy_(src)

    def exchange(self, pairs):
        pass

    def allgather_start(self, src, dst):
        self.allgather(src, dst)
        return self

    def exchange_start(self, pairs):
        return self

    def wait(self):
        pass


class NullGraphComm(NullComm):
    """NullComm shaped like the native RCCL transport: stream-ordered only, so the engine
    captures its chunks into hipGraphs (the multi-GPU path's launch structure)."""
    staged = False

    def rccl(self):
        return self


def rank_share(args):
    from pycsou_amd.opt.engine3d import PDS3DEngine
    torch.cuda.set_device(0)
    dtype = torch.float32 if args.dtype == 'f32' else torch.float64
    W = args.rank_of
    rank = W // 2 - 1 if W > 2 else 0
    t0 = time.time()
    print(f'building {args.size}^3 ...', flush=True)
    pds = build(args.size, dtype, kind=args.kind)
    spec = pds._fused_spec()
    print(f'built in {time.time() - t0:.1f} s', flush=True)
    K = -(-args.steps // 8) * 8  # whole chunks of 8 (the graph variants replay chunks)
    out = {'workload': f'one rank ({rank} of {W}) of 3-D TV-deconv {args.size}^3 {args.dtype}'}
    runs = [(name + ('_graph' if g else ''), ov, order, g) for g in (False, True)
            for name, ov, order in (('serial', False, 'split'), ('banded', True, 'split'),
                                    ('banded_fullg', True, 'fullg'))]
    for name, ov, order, graph in runs:
        comm = (NullGraphComm if graph else NullComm)(rank, W)
        eng = PDS3DEngine(spec, dtype, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, comm=comm,
                          rank=rank, world=W, overlap=ov, chunk=8)
        assert eng.use_graph == graph
        eng.order = order
        eng.init_loop(K + 16, K + 16, -1.0)
        eng.advance(8)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.advance(K)
        e1.record()
        torch.cuda.synchronize()
        out[f'{name}_ms_per_iter'] = round(e0.elapsed_time(e1) / K, 4)
        out['planes'], out['banded'] = eng.rows, bool(eng.banded)
        print(name, out[f'{name}_ms_per_iter'], 'ms/iter', flush=True)
        esz = eng.X[0].element_size()
        out['halo_bytes_per_side'] = eng.halo_planes * eng.plane * esz
        if ov and not graph and eng.banded:
            # the overlap window of this order: the exchange starts after the boundary bands and is awaited
            # after the next iteration's in-plane pass of the own planes -> window = interior + that pass
            ph = {'pre': [], 'boundary': [], 'interior': []}
            st = torch.cuda.current_stream()
            for i in range(4):
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
                ev[0].record(st)
                eng._band_pre(i % 2, L.stream())
                ev[1].record(st)
                eng._band_boundary(i % 2, L.stream())
                ev[2].record(st)
                eng._band_interior(i % 2, L.stream())
                ev[3].record(st)
                torch.cuda.synchronize()
                for k, (a, b) in zip(ph, zip(ev[:-1], ev[1:])):
                    ph[k].append(a.elapsed_time(b))
            ph = {k: float(np.median(v)) for k, v in ph.items()}
            out[f'{name}_phases_ms'] = {k: round(v, 4) for k, v in ph.items()}
            out[f'{name}_window_ms'] = round(ph['interior'] + ph['pre'], 4)
        del eng
        torch.cuda.empty_cache()
    # link-rate model: per direction and neighbour, the exchange takes halo / R; the banded
    # orders hide it behind their window, the serial schedule adds it.  Iteration = compute + exposed exchange
    hb = out['halo_bytes_per_side']
    model = {}
    for gbs in (50.0, 82.0, 120.0, 153.0):
        tx = hb / (gbs * 1e9) * 1e3
        est = {'serial': out['serial_ms_per_iter'] + tx}
        for name in ('banded', 'banded_fullg'):
            if f'{name}_window_ms' in out:
                est[name] = out[f'{name}_ms_per_iter'] + max(0.0, tx - out[f'{name}_window_ms'])
        best = min(est, key=est.get)
        m = {'exchange_ms': round(tx, 3), 'best_order': best, 'iteration_ms': round(est[best], 3)}
        if args.one_gpu_ms > 0:
            m['speedup'] = round(args.one_gpu_ms / est[best], 2)
        model[f'{gbs:.0f}GBps'] = m
    out['link_model'] = model
    if args.one_gpu_ms > 0:
        # the slowest link at which W GPUs still reach 6x: exchange <= T1 / 6 - compute + window, best order
        rates = {}
        for name in ('banded', 'banded_fullg'):
            if f'{name}_window_ms' in out:
                slack = args.one_gpu_ms / 6 - out[f'{name}_ms_per_iter'] + out[f'{name}_window_ms']
                if slack > 0:
                    rates[name] = round(hb / (slack * 1e-3) / 1e9, 1)
        out['min_GBps_for_6x'] = rates
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()

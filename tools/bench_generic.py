"""Throughput of problems that only the generic device path takes (no fused engine): one kernel per
operator per iteration, the stopping rule on the device (pycsou_amd/opt/proxalgs.py::_update_dev).
Prints one JSON line per problem: it/s from HIP events around iterate() at max_iter = min_iter = W + K
minus the same at W (steady state, host dispatch included -- that is this path's cost), launches per
iteration from torch.profiler's device activity.  Problems (2048^2, fp32 and fp64):
  l21_labels   TV denoising with a GENERAL-label L21Norm (groups of 2 horizontally adjacent pixels x both
               gradient components = 4 values; pycsou/func/penalty.py:525-560) -- the label kernel
  stack_h      TV denoising with H = ProxFuncHStack(0.1 L1Norm, 0.1 L1Norm) over the two gradient
               components (stacked H, pycsou/func/base.py:21-89)
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def problem(name, n, dtype):
    from pycsou_amd.func import L1Norm, ProxFuncHStack
    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L21Norm
    from pycsou_amd.linop import Gradient
    from pycsou_amd.opt import PDS
    N = n * n
    img = bench.phantom((n, n), 12, 5).ravel()
    rng = np.random.default_rng(3)
    y = torch.from_numpy((img + 0.1 * rng.standard_normal(N)).astype(np.float32 if dtype == torch.float32
                                                                         else np.float64)).cuda()
    K = Gradient(shape=(n, n), kind='forward')
    K.lipschitz_cst = K.diff_lipschitz_cst = float(np.sqrt(8.0))
    F = (1 / 2) * SquaredL2Loss(dim=N, data=y)
    if name == 'l21_labels':
        lab = np.arange(N) // 2
        H = 0.1 * L21Norm(dim=2 * N, groups=np.concatenate([lab, lab]))
    else:
        H = ProxFuncHStack(0.1 * L1Norm(dim=N), 0.1 * L1Norm(dim=N))
    return lambda it: PDS(dim=N, F=F, H=H, K=K, x0=torch.zeros(N, dtype=dtype, device='cuda'),
                          z0=torch.zeros(2 * N, dtype=dtype, device='cuda'), max_iter=it, min_iter=it, verbose=None)


def timed(mk, it):
    pds = mk(it)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    pds.iterate()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def launches(mk, it):
    from torch.profiler import ProfilerActivity, profile
    pds = mk(it)
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        pds.iterate()
        torch.cuda.synchronize()
    return sum(1 for e in prof.events() if e.device_type.name == 'CUDA')


def main():
    torch.cuda.set_device(0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048  # image side (256: the launch-bound regime)
    W, K = 20, 200
    for dtype in (torch.float32, torch.float64):
        for name in ('l21_labels', 'stack_h'):
            t0 = time.perf_counter()
            mk = problem(name, n, dtype)
            timed(mk, W)
            tw = min(timed(mk, W) for _ in range(2))
            tk = min(timed(mk, W + K) for _ in range(2))
            ms = (tk - tw) / K
            nl = (launches(mk, W + 10) - launches(mk, W)) / 10
            path = 'generic' if mk(1)._fused_spec() is None else 'fused'
            print(json.dumps({'problem': name, 'path': path, 'n': n, 'dtype': str(dtype).split('.')[-1], 'it_per_s': round(1e3 / ms, 1),
                              'ms_per_iter': round(ms, 4), 'launches_per_iter': nl,
                              'wall_s': round(time.perf_counter() - t0, 1)}), flush=True)


if __name__ == '__main__':
    main()

"""Round 6: the communication-avoiding slab loop's per-iteration cost, one GPU.

In-process W-slab run of a strong-scaled 4096^2 C3 image (run_local_deep: all W ranks' launches on one GPU, the all-gather / loop control /
    exchange as device copies once per chunk): per iteration, the W ranks' compute + the per-chunk sync
    work; with depth k the sync launches (W^2 sum copies, W finalize kernels, 6 (W - 1) halo copies) run once
    per k iterations.
Prints one JSON line per (W, depth); run it under rocprofv3 --kernel-trace --stats to split the time into
the step launches (k_pds2d_nmarch) and the per-chunk sync work (k_reduce_finalize_k, copies)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes  # noqa: E402

import torch  # noqa: E402

import bench  # noqa: E402
from pycsou_amd import _lib as L  # noqa: E402
from pycsou_amd.parallel import SlabPDS2D, run_local_deep  # noqa: E402


def main():
    n = int(os.environ.get('PCS_N', '4096'))
    world = int(os.environ.get('PCS_W', '8'))
    iters = int(os.environ.get('PCS_ITERS', '64'))
    pds = bench.build_problem(n, n, torch.float32, lipschitz='analytic')
    spec = pds._fused_spec()
    for depth in (1, 2, 4, 8):
        try:
            slabs = [SlabPDS2D(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, r, world,
                               native='local', depth=depth) for r in range(world)]
        except ValueError as e:
            print(json.dumps({'world': world, 'depth': depth, 'skipped': str(e)}), flush=True)
            continue
        total = iters + 2 * depth + 8
        run_local_deep(slabs, 2 * depth, 2 * depth, 0.0, chunk=2 * depth)  # warm (plans, kernels)
        torch.cuda.synchronize()
        for s in slabs:
            s.init_loop(total, total, -1.0)
        plans = (ctypes.c_void_p * world)(*[s._deep_plan().value for s in slabs])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        L.check(slabs[0].lib.pcs_slab2d_deep_run_local(plans, world, iters, 0, L.stream()), 'run_local')
        torch.cuda.synchronize()
        ms_all = (time.perf_counter() - t0) * 1e3 / iters
        r = slabs[world // 2]
        print(json.dumps({'world': world, 'depth': depth, 'rows_per_rank': r.rows, 'halo_rows_x': r.hx,
                          'reach': r.reach, 'ms_per_iter_all_ranks_one_gpu': round(ms_all, 4),
                          'ms_per_iter_per_rank': round(ms_all / world, 4),
                          'redundant_rows_per_iter_per_side': (depth - 1) * r.reach / 2}), flush=True)
        for s in slabs:
            s._destroy_plan()
        del slabs
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()

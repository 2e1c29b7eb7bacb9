"""Run the C3 fused PDS engine for a few iterations (eager launches) so rocprofv3 can
attribute time and counters per kernel.  Usage (GPU box):
  rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 tools/profile_step.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from pycsou_amd.opt.engine import PDS2DEngine  # noqa: E402


def main():
    n = int(os.environ.get('PCS_N', '4096'))
    iters = int(os.environ.get('PCS_ITERS', '20'))
    dtype = torch.float64 if os.environ.get('PCS_DTYPE', 'f32') == 'f64' else torch.float32
    torch.cuda.set_device(0)
    pds = bench.build_problem(n, n, dtype)
    spec = pds._fused_spec()
    eng = PDS2DEngine(spec, dtype, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, use_graph=False)
    eng.chunk = 2
    eng.run(iters - 1, iters - 1, 0.0)
    torch.cuda.synchronize()
    print('done', iters, 'iterations')


if __name__ == '__main__':
    main()

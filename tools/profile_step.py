"""Run one fused PDS problem for a few iterations (eager launches) so rocprofv3 can attribute
time and counters per kernel.  Usage (GPU box):
  PCS_PROBLEM=c3 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 tools/profile_step.py
PCS_PROBLEM: c3 (default: 4096^2 TV-deconvolution, forward K), c3_cen (default centred K), c3_nonsep,
c2 (2048^2 denoising), c2_lap / c2_cen (Laplacian / centred K).  Operator norms from the closed
forms (no Lanczos under the profiler).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from pycsou_amd.opt.engine import PDS2DEngine, PDS2DStencilEngine  # noqa: E402


def main():
    prob = os.environ.get('PCS_PROBLEM', 'c3')
    n = int(os.environ.get('PCS_N', '4096' if prob.startswith('c3') else '2048'))
    iters = int(os.environ.get('PCS_ITERS', '20'))
    dtype = torch.float64 if os.environ.get('PCS_DTYPE', 'f32') == 'f64' else torch.float32
    torch.cuda.set_device(0)
    if prob == 'c3':
        pds = bench.build_problem(n, n, dtype, lipschitz='analytic')
    elif prob == 'c3_cen':
        pds = bench.build_problem(n, n, dtype, lipschitz='analytic', kind='centered')
    elif prob == 'c3_nonsep':
        pds = bench.build_problem(n, n, dtype, psf=bench.aniso_psf(), lipschitz='analytic')
    elif prob == 'c2':
        pds = bench.build_denoise(n, dtype, lipschitz='analytic')
    else:
        pds = bench.build_denoise_k(n, dtype, 'lap' if prob == 'c2_lap' else 'centered', lipschitz='analytic')
    spec = pds._fused_spec()
    cls = PDS2DStencilEngine if spec.get('stencil') else PDS2DEngine
    eng = cls(spec, dtype, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, use_graph=False)
    eng.chunk = 2
    eng.run(iters - 1, iters - 1, 0.0)
    torch.cuda.synchronize()
    print('done', prob, iters, 'iterations')


if __name__ == '__main__':
    main()

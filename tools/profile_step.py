"""Run one fused PDS problem for a few iterations (eager launches) so rocprofv3 can attribute
time and counters per kernel.  Usage (GPU box):
  PCS_PROBLEM=c3 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 tools/profile_step.py
PCS_PROBLEM: c3 (default: 4096^2 TV-deconvolution, forward K), c3_cen (default centred K), c3_nonsep,
c2 (2048^2 denoising), c2_lap / c2_cen (Laplacian / centred K), cps (2048^2 CPS TV-LAD inpainting,
the masked fused step), c4 / c4_cen (512^3 3-D, forward / centred K); PCS_DTYPE=f64 for the fp64 forms.  Operator norms from the closed forms (no
Lanczos under the profiler).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from pycsou_amd import _ops as O  # noqa: E402
from pycsou_amd.opt.engine import engine_class  # noqa: E402


def cps_problem(n, dtype):
    """bench.py's cps_inpaint problem (analytic ||K||)."""
    import numpy as np
    from pycsou_amd.func import L1Loss, L1Norm, ProxFuncHStack, Segment
    from pycsou_amd.linop import Gradient, LinOpVStack, Masking
    from pycsou_amd.opt import CPS
    N = n * n
    mask = np.random.default_rng(5).random(N) < 0.5
    img = bench.phantom((n, n), 12, 5).ravel()
    y = torch.from_numpy(img[mask]).to('cuda', dtype)
    Kop = LinOpVStack(Masking(size=N, sampling_bool=mask), Gradient(shape=(n, n), kind='forward'))
    Kop.lipschitz_cst = Kop.diff_lipschitz_cst = 3.0
    H = ProxFuncHStack(L1Loss(dim=int(mask.sum()), data=y), 0.1 * L1Norm(dim=2 * N))
    return CPS(dim=N, G=Segment(dim=N, a=0, b=1), H=H, K=Kop, x0=torch.zeros(N, dtype=dtype, device='cuda'),
               z0=torch.zeros(int(mask.sum()) + 2 * N, dtype=dtype, device='cuda'), verbose=None)


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
    elif prob == 'cps':
        pds = cps_problem(n, dtype)
    elif prob in ('c4', 'c4_cen'):  # 3-D: tools/bench3d.py's problem (PCS_N = edge, default 512)
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
        from bench3d import build as build3d
        n = int(os.environ.get('PCS_N', '512'))
        pds = build3d(n, dtype, kind='centered' if prob == 'c4_cen' else 'forward')
    else:
        pds = bench.build_denoise_k(n, dtype, 'lap' if prob == 'c2_lap' else 'centered', lipschitz='analytic')
    spec = pds._fused_spec()
    eng = engine_class(spec)(spec, dtype, pds.tau, pds.sigma, pds.rho, O.to_dev(pds.x0, dtype),
                             O.to_dev(pds.z0, dtype), use_graph=False)
    eng.chunk = 2
    eng.run(iters - 1, iters - 1, 0.0)
    torch.cuda.synchronize()
    print('done', prob, iters, 'iterations')


if __name__ == '__main__':
    main()

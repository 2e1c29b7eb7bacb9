"""General-stencil march step (k_pds2d_smarch) launch-mode probe on 2048^2 denoising (Laplacian /
centred K): per iteration (a) back to back (pcs_pds2d_run chunks), (b) alone (a synchronize
between launches, HIP events around each launch).  Prints one JSON line per problem
(diagnostics; PCS_LIB_PATH selects a variant build)."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from pycsou_amd import _lib as L  # noqa: E402
from pycsou_amd.opt.engine import PDS2DStencilEngine  # noqa: E402


def main():
    torch.cuda.set_device(0)
    n = int(os.environ.get('PCS_N', '2048'))
    for kind in ('lap', 'centered'):
        pds = bench.build_denoise_k(n, torch.float32, kind, lipschitz='analytic')
        eng = PDS2DStencilEngine(pds._fused_spec(), torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0)
        assert eng.march
        K = 400
        eng.prepare_fixed(4 * K + 100, 50)
        bench.spin_up_fixed(eng)
        eng.prepare_fixed(4 * K + 100, 50)
        eng.advance_fixed(20)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.advance_fixed(K)
        e1.record()
        torch.cuda.synchronize()
        b2b = e0.elapsed_time(e1) * 1e3 / K
        alone = []
        for i in range(60):
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            eng.advance_fixed(1)
            s1.record()
            torch.cuda.synchronize()
            alone.append(s0.elapsed_time(s1) * 1e3)
        words = 5 if kind == 'lap' else 7
        print(json.dumps({'kind': kind, 'lib': os.environ.get('PCS_LIB_PATH', 'default'), 'b2b_us': round(b2b, 2),
                          'alone_us_median': round(float(np.median(alone)), 2),
                          'alone_frac': round(words * n * n * 4 / (np.median(alone) * 1e-6) / 8e12, 3),
                          'b2b_frac': round(words * n * n * 4 / (b2b * 1e-6) / 8e12, 3)}), flush=True)
        del eng, pds
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()

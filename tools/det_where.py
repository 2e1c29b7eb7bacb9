"""Where do two runs of the C3 centred fused march differ (round-5 determinism probe): column mod 64 / row
mod 32 histograms of the differing x pixels after 1 and 2 iterations."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import pycsou_amd.opt.engine as E  # noqa: E402
from pycsou_amd import _ops as O  # noqa: E402


def run(pds, iters):
    spec = pds._fused_spec()
    eng = E.engine_class(spec)(spec, torch.float32, pds.tau, pds.sigma, pds.rho, O.to_dev(pds.x0, torch.float32),
                               O.to_dev(pds.z0, torch.float32))
    n, x, z, h = eng.run(iters - 1, iters - 1, 0.0)
    torch.cuda.synchronize()
    return x.clone().view(4096, 4096), z.clone().view(2, 4096, 4096)


torch.cuda.set_device(0)
pds = bench.build_problem(4096, 4096, torch.float32, lipschitz='analytic', kind=os.environ.get('KIND', 'centered'))
for iters in (1, 2):
    ref = run(pds, iters)
    for rep in range(3):
        r = run(pds, iters)
        dx = (r[0] != ref[0]).nonzero().cpu().numpy()
        dz = (r[1] != ref[1]).nonzero().cpu().numpy()
        print('iters', iters, 'rep', rep, 'x diffs', len(dx), 'z diffs', len(dz), flush=True)
        if len(dx):
            print('  x cols mod 64:', np.bincount(dx[:, 1] % 64, minlength=64).tolist())
            print('  x rows mod 32:', np.bincount(dx[:, 0] % 32, minlength=32).tolist())
            print('  x rows range', dx[:, 0].min(), dx[:, 0].max(), 'cols range', dx[:, 1].min(), dx[:, 1].max())
            print('  first', dx[:8].tolist())
        if len(dz):
            print('  z comp', np.bincount(dz[:, 0], minlength=2).tolist(), 'cols mod 64:', np.bincount(dz[:, 2] % 64, minlength=64).tolist())
            print('  z rows mod 32:', np.bincount(dz[:, 1] % 32, minlength=32).tolist())

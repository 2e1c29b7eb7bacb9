"""Determinism probe (round 5): run a fused 2-D problem several times from the same state and compare the
iterates bitwise, with the deferred finalization on and off (PCS_DEFER_FIN read through engine.DEFER_FIN)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import pycsou_amd.opt.engine as E  # noqa: E402
from pycsou_amd import _ops as O  # noqa: E402


def run(pds, dtype, defer, iters):
    E.DEFER_FIN = defer
    spec = pds._fused_spec()
    eng = E.engine_class(spec)(spec, dtype, pds.tau, pds.sigma, pds.rho, O.to_dev(pds.x0, dtype), O.to_dev(pds.z0, dtype))
    n, x, z, h = eng.run(iters - 1, iters - 1, 0.0)
    torch.cuda.synchronize()
    return n, x.clone(), z.clone()


def main():
    torch.cuda.set_device(0)
    probs = {'c3_cen': lambda: bench.build_problem(4096, 4096, torch.float32, lipschitz='analytic', kind='centered'),
             'c3': lambda: bench.build_problem(4096, 4096, torch.float32, lipschitz='analytic'),
             'c2_lap': lambda: bench.build_denoise_k(2048, torch.float32, 'lap', lipschitz='analytic')}
    for name in os.environ.get('PROBS', 'c3_cen,c3,c2_lap').split(','):
        pds = probs[name]()
        for iters in (3, 10):
            for defer in (False, True):
                ref = run(pds, torch.float32, defer, iters)
                diffs = []
                for rep in range(4):
                    r = run(pds, torch.float32, defer, iters)
                    diffs.append((r[0] == ref[0], int((r[1] != ref[1]).sum()), int((r[2] != ref[2]).sum())))
                print(name, 'iters', iters, 'defer', defer, 'n', ref[0], 'reps (same n, x diffs, z diffs):', diffs, flush=True)


if __name__ == '__main__':
    main()

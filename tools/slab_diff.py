"""Where do the row slabs and the single-GPU engine differ (diagnostics for the bitwise slab tests):
per iteration count, the (row, col) of the first mismatching x / z elements."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pycsou_amd.parallel import SlabPDS2D, run_local  # noqa: E402
from tests.slab_worker import SYNTH, synth_problem  # noqa: E402


def main():
    torch.cuda.set_device(0)
    for name in sys.argv[1:]:
        shape = SYNTH[name][0]
        for niter in (1, 2, 3, 16):
            pds = synth_problem(name, niter=niter)
            pds.iterate()
            eng = pds._engine
            x1 = eng.X[pds.iter % 2].cpu().numpy().reshape(shape)
            z1 = eng.Z[pds.iter % 2].cpu().numpy().reshape(-1, *shape)
            pds2 = synth_problem(name, niter=niter)
            slabs = [SlabPDS2D.from_pds(pds2, None, rank=r, world=2) for r in range(2)]
            res = run_local(slabs, pds2.max_iter, pds2.min_iter, pds2.accuracy_threshold)
            x2 = torch.cat([r[1] for r in res]).cpu().numpy().reshape(shape)
            nc = slabs[0].ncomp
            z2 = torch.cat([torch.cat([r[2].view(nc, -1)[c] for r in res]) for c in range(nc)]).cpu().numpy()
            z2 = z2.reshape(-1, *shape)
            dx = np.argwhere(x1 != x2)
            dz = np.argwhere(z1 != z2)
            print(name, 'iters', niter, 'row0s', [s.row0 for s in slabs], 'x mism', len(dx), dx[:8].tolist(),
                  'z mism', len(dz), dz[:8].tolist(), flush=True)


if __name__ == '__main__':
    main()

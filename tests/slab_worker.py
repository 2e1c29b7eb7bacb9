"""One rank of the two-process slab test (tests/test_gpu_slab.py::test_two_process_gloo).

Run with RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the environment; both ranks use
cuda:0 and a gloo process group.  Rank 0 writes the gathered x, the history and the
iteration count to <outdir>.
"""

import os
import sys

import numpy as np
import torch
import torch.distributed as dist


def main(name, outdir):
    torch.cuda.set_device(0)
    dist.init_process_group('gloo')
    from pycsou_amd.parallel import DistComm, SlabPDS2D, gather_rows
    from tests.cases import pds_case
    from tests.test_gpu_pds import build
    comm = DistComm()
    if name == 'vol3d':  # banded, overlapped 3-D schedule (tests/test_gpu_slab.py::vol3d_case)
        from pycsou_amd.opt.engine3d import PDS3DEngine
        from tests.test_gpu_slab import vol3d_case
        pds = build(vol3d_case(), np.float64, engine='fused')
        spec = pds._fused_spec()
        eng = PDS3DEngine(spec, pds._compute_dtype(), pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, comm=comm,
                          rank=comm.rank, world=comm.world)
        assert eng.banded
        n, x, z, h = eng.run(pds.max_iter, pds.min_iter, pds.accuracy_threshold)
        xg = gather_rows(x, eng.n0, eng.plane, comm.world, comm.rank, comm)
    else:
        c = pds_case(name)
        pds = build(c, np.float64, engine='fused')
        eng = SlabPDS2D.from_pds(pds, comm, chunk=4)
        n, x, z, h = eng.run(pds.max_iter, pds.min_iter, pds.accuracy_threshold)
        xg = gather_rows(x, eng.n0, eng.n1, comm.world, comm.rank, comm)
    if comm.rank == 0:
        np.save(os.path.join(outdir, 'x.npy'), xg.cpu().numpy())
        np.save(os.path.join(outdir, 'hist.npy'), h)
        np.save(os.path.join(outdir, 'n.npy'), np.array(n))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])

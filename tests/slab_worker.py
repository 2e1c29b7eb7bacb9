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


# synthetic slab problems (no golden: the single-GPU fused engine is the reference):
# name -> (shape, K kind, H, PSF, dtype)
SYNTH = {
    'cen_denoise_f32': ((300, 200), 'centered', 'l21', None, np.float32),
    'lap_denoise_f32': ((260, 192), 'lap', 'l1', None, np.float32),
    'bwd_denoise_f32': ((150, 132), 'backward', 'l1', None, np.float32),
    'nonsep_fwd_f64': ((120, 96), 'forward', 'l21', 'nonsep9', np.float64),
    'nonsep_fwd_f32': ((140, 256), 'forward', 'l1', 'nonsep9', np.float32),
    'nonsep_cen_f32': ((200, 192), 'centered', 'l21', 'nonsep9', np.float32),
    'sep_cen_f32': ((240, 256), 'centered', 'l21', 'sep15', np.float32),
    'sep_cen_f64': ((240, 256), 'centered', 'l21', 'sep15', np.float64),
    'sep_fwd_f64': ((200, 320), 'forward', 'l1', 'sep15', np.float64),
}


def synth_problem(name, niter=16):
    """A PDS of the SYNTH table through the public API (fixed iteration count)."""
    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L1Norm, L21Norm
    from pycsou_amd.linop.conv import Convolve2D
    from pycsou_amd.linop.diff import Gradient, Laplacian
    from pycsou_amd.opt.proxalgs import PDS
    shape, kind, hname, psf, dtype = SYNTH[name]
    N = shape[0] * shape[1]
    rng = np.random.default_rng(11)
    y = rng.uniform(0, 1, N).astype(dtype)
    F = (1 / 2) * SquaredL2Loss(dim=N, data=y)
    if psf is not None:
        if psf == 'sep15':
            r = np.arange(15) - 7.0
            g = np.exp(-0.5 * (r / 2.0) ** 2)
            h = np.outer(g, g)
        else:  # 9 x 9, rank > 1
            h = rng.uniform(0, 1, (9, 9))
        C = Convolve2D(N, h / h.sum(), shape)
        C.lipschitz_cst = C.diff_lipschitz_cst = 1.0
        F = F * C
    if kind == 'lap':
        K, hdim = Laplacian(shape, edge=True), N
        K.lipschitz_cst = K.diff_lipschitz_cst = 8.0
    else:
        K, hdim = Gradient(shape, kind=kind), 2 * N
        K.lipschitz_cst = K.diff_lipschitz_cst = np.sqrt(8.0)
    H = 0.05 * (L21Norm(dim=hdim, groups=np.tile(np.arange(N), 2)) if hname == 'l21' else L1Norm(dim=hdim))
    return PDS(dim=N, F=F, H=H, K=K, x0=np.zeros(N, dtype), z0=np.zeros(hdim, dtype), max_iter=niter - 1,
               min_iter=niter - 1, accuracy_threshold=0.0, verbose=None, engine='fused')


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
        pds = synth_problem(name) if name in SYNTH else build(pds_case(name), np.float64, engine='fused')
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

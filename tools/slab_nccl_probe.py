"""Check: the row-slab engine over the NCCL (RCCL) transport, one rank per GPU (needs >= 2 GPUs:
RCCL refuses two ranks on one device, "Duplicate GPU detected").

Launch: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1
        --master-port P tools/slab_nccl_probe.py
Compares the gathered slab solution with the single-GPU fused engine on rank 0.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from pycsou_amd.opt.engine import PDS2DEngine
    from pycsou_amd.parallel import DistComm, SlabPDS2D, gather_rows
    n0, n1 = 512, 384
    pds = bench.build_problem(n0, n1, torch.float32)
    comm = DistComm()
    eng = SlabPDS2D.from_pds(pds, comm)
    t0 = time.perf_counter()
    n, x, z, h = eng.run(39, 39, 0.0)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    xg = gather_rows(x, n0, n1, comm.world, comm.rank, comm)
    if comm.rank == 0:
        spec = pds._fused_spec()
        ref = PDS2DEngine(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0)
        n1_, x1, _, h1 = ref.run(39, 39, 0.0)
        print(f'world={comm.world} n={n} ref_n={n1_} bitwise={torch.equal(xg, x1)} '
              f'maxdiff={(xg - x1).abs().max().item():.3e} time={dt:.3f}s', flush=True)
        assert n == n1_ and torch.equal(xg, x1)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()

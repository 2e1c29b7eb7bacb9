"""Per-iteration time of the row-slab loop at world 1 in each schedule (diagnostics, GPU box).

  python   : SlabPDS2D with the Python-issued per-iteration sequence (native=False)
  serial   : pcs_slab2d_run, step + reduce + finalize per iteration on one stream
  overlap  : pcs_slab2d_run, boundary bands + interior band + reduce, finalize on a side stream
Halo exchange / all-gather are no-ops at world 1: this isolates the launch-structure cost.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from pycsou_amd.parallel import SlabPDS2D  # noqa: E402


def main():
    torch.cuda.set_device(0)
    n = int(os.environ.get('PCS_N', '4096'))
    pds = bench.build_problem(n, n, torch.float32)
    spec = pds._fused_spec()
    N = 200
    for name, native, ov in (('python', False, False), ('serial', True, False), ('overlap', True, True)):
        s = SlabPDS2D(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, 0, 1, native=native,
                      overlap=ov)
        s.init_loop(3 * N, 3 * N, -1.0)
        s.advance(N)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        s.advance(N)
        e1.record()
        torch.cuda.synchronize()
        print(f'{name}: {e0.elapsed_time(e1) / N * 1e3:.1f} us/iter', flush=True)
        del s
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()

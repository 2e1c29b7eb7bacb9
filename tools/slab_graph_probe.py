"""World-1 native row-slab loop on the C3 problem (4096^2 fp32 TV-deconvolution): eager
pcs_slab2d_run chunks against the same chunks replayed from a hipGraph (PCS_SLAB_GRAPH), serial
and overlapped schedules.  ms per iteration over 400 iterations after 100 untimed."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from pycsou_amd.parallel import SlabPDS2D
    torch.cuda.set_device(0)
    pds = bench.build_problem(4096, 4096, torch.float32, lipschitz='analytic')
    spec = pds._fused_spec()
    for graph in ('0', '32'):
        os.environ['PCS_SLAB_GRAPH'] = graph
        for ov in (False, True):
            s = SlabPDS2D(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, 0, 1, native=True,
                          overlap=ov, chunk=64)
            s.init_loop(600, 600, -1.0)
            s.advance(128)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            s.advance(384)
            e1.record()
            torch.cuda.synchronize()
            print(f'graph={graph} overlap={ov}: {e0.elapsed_time(e1) / 384:.4f} ms/iter '
                  f'(captured: {s._graph is not None})', flush=True)
            del s
            torch.cuda.empty_cache()


if __name__ == '__main__':
    main()

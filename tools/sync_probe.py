"""Round 6 diagnostics: the 3-D update's plane lockstep (pcs_pds3d_args.sync) in the engine's loop forms --
isolated step launches (time_parts), eager back-to-back iterations, hipGraph-replayed chunks -- with the
lockstep on and off (PCS_3D_SYNC), C4 512^3 fp32 centred K.  One JSON line per configuration."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench3d import build  # noqa: E402


def main():
    from pycsou_amd.opt.engine3d import PDS3DEngine
    n = int(os.environ.get('PCS_N', '512'))
    kind = os.environ.get('PCS_KIND', 'centered')
    pds = build(n, torch.float32, kind=kind)
    spec = pds._fused_spec()
    for sync in ('0', '1'):
        os.environ['PCS_3D_SYNC'] = sync
        for graph in (False, True):
            eng = PDS3DEngine(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, chunk=2,
                              use_graph=graph)
            parts = eng.time_parts(3)
            eng.init_loop(60, 60, -1.0)
            eng.advance(6)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.advance(20)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / 20
            print(json.dumps({'sync': sync, 'graph': graph, 'iter_ms': round(ms, 4),
                              'parts_ms': {k: round(v, 4) for k, v in parts.items()}}), flush=True)
            del eng
            torch.cuda.empty_cache()


if __name__ == '__main__':
    main()

"""Diagnostics: iteration counter after K fused iterations, with and without the in-kernel finalize."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from pycsou_amd.opt.engine import PDS2DEngine  # noqa: E402

torch.cuda.set_device(0)
for n in [256, 1024, 4096]:
    pds = bench.build_problem(n, n, torch.float32)
    spec = pds._fused_spec()
    for fused in [True, False]:
        for graph in [True, False]:
            eng = PDS2DEngine(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, use_graph=graph)
            eng.fused_finalize = fused
            if graph:
                eng.prepare_fixed(64, 8)
                for _ in range(5):
                    eng.replay()
            else:
                eng.hist = torch.empty(2 * 65 + 2, dtype=torch.float64, device='cuda')
                eng.lib.pcs_ctrl_init2(eng.ctrl.data_ptr(), 64, 64, -1.0, 1, eng.hist.numel(), None)
                for i in range(40):
                    eng._iteration(i % 2, eng.hist)
            torch.cuda.synchronize()
            c = eng.ctrl.view(torch.int32)[:2].tolist()
            print(f'n={n} fused={fused} graph={graph} nblocks={eng.nblocks} it={c[0]} stopped={c[1]} '
                  f'hist[:6]={[round(v, 6) for v in eng.hist[:6].tolist()]}', flush=True)

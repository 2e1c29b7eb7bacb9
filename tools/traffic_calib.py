"""Calibrate PMC read-traffic counters against a plain copy, then run the 3-D C4 loop
(diagnostics for rocprofv3 --pmc passes).  PCS_N: volume edge (default 512)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tools.bench3d import build  # noqa: E402


def main():
    n = int(os.environ.get('PCS_N', '512'))
    torch.cuda.set_device(0)
    x = torch.randn(n, n, n, device='cuda')
    y = torch.empty_like(x)
    for _ in range(3):
        y.copy_(x)
    torch.cuda.synchronize()
    del x, y
    from pycsou_amd.opt.engine3d import PDS3DEngine
    pds = build(n, torch.float32)
    eng = PDS3DEngine(pds._fused_spec(), torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, chunk=2)
    eng.init_loop(12, 12, -1.0)
    eng.advance(6)
    torch.cuda.synchronize()
    print('done')


if __name__ == '__main__':
    main()

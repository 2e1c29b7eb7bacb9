"""C2 (2048^2 TV denoising) launch-mode probe: the same fixed-count loop timed as
(a) pcs_pds2d_run chunks, (b) eager pcs_pds2d_step launches, (c) eager launches with an event
recorded between launches.  Prints us per iteration for each (diagnostics)."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pycsou_amd import _lib as L  # noqa: E402
from pycsou_amd.opt.engine import PDS2DEngine  # noqa: E402
from tools.bench2d import c2  # noqa: E402


def main():
    n = int(os.environ.get('PCS_N', '2048'))
    torch.cuda.set_device(0)
    pds = c2(n)
    eng = PDS2DEngine(pds._fused_spec(), torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0)
    K = 400
    lib, a = eng.lib, eng.args
    out = {}

    def timed(fn):
        eng.prepare_fixed(4 * K + 8, 50)
        fn()  # warm
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / K

    def native():
        for _ in range(K // 50):
            eng.replay()

    def eager(ev):
        evs = [torch.cuda.Event() for _ in range(K)] if ev else None
        for i in range(K):
            p = i % 2
            a.x, a.xn = eng.X[p].data_ptr(), eng.X[1 - p].data_ptr()
            a.z, a.zn = eng.Z[p].data_ptr(), eng.Z[1 - p].data_ptr()
            a.hist = eng.hist.data_ptr()
            L.check(lib.pcs_pds2d_step(ctypes.byref(a), L.stream()), 'step')
            if ev:
                evs[i].record()

    out['native_us'] = round(timed(native), 2)
    out['eager_us'] = round(timed(lambda: eager(False)), 2)
    out['eager_events_us'] = round(timed(lambda: eager(True)), 2)
    out['alg_MB'] = 7 * n * n * 4 / 1e6
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()

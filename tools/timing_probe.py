"""How long does one fused C3 step take in each launch mode?  (diagnostics, GPU box)

  eager+events : one event pair per launch (bench.py's kernel_ms)
  eager        : N back-to-back launches, one event pair around all
  graph(c)     : hipGraph of c iterations replayed, one event pair around all replays
  native(c)    : pcs_pds2d_run launching c iterations back to back from C
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from pycsou_amd import _lib as L  # noqa: E402
from pycsou_amd.opt.engine import PDS2DEngine  # noqa: E402


def main():
    torch.cuda.set_device(0)
    n = int(os.environ.get('PCS_N', '4096'))
    pds = bench.build_problem(n, n, torch.float32)
    spec = pds._fused_spec()
    N = 100
    for native, c in ((False, 50), (False, 10), (True, 50), (True, 10), (True, 2)):
        eng = PDS2DEngine(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0)
        eng.native = native
        eng.prepare_fixed(4 * N + 10, c)
        for _ in range(20 // c if c < 20 else 1):
            eng.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(N // c):
            eng.replay()
        e1.record()
        torch.cuda.synchronize()
        print(f'{"native" if native else "graph"}({c}): {e0.elapsed_time(e1) / N * 1e3:.1f} us/iter', flush=True)
    print(f'eager+events: {eng.time_step_kernel(N) * 1e3:.1f} us/launch', flush=True)
    # eager back-to-back (fresh loop state, no events between launches)
    a = eng.args
    L.check(eng.lib.pcs_ctrl_init2(L.ptr(eng.ctrl), N + 1, N + 1, -1.0, 1, int(eng.hist.numel()), L.stream()), 'init')
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(N):
        p = i % 2
        a.x, a.xn = eng.X[p].data_ptr(), eng.X[1 - p].data_ptr()
        a.z, a.zn = eng.Z[p].data_ptr(), eng.Z[1 - p].data_ptr()
        L.check(eng.lib.pcs_pds2d_step(ctypes.byref(a), L.stream()), 'step')
    e1.record()
    torch.cuda.synchronize()
    print(f'eager: {e0.elapsed_time(e1) / N * 1e3:.1f} us/launch', flush=True)


if __name__ == '__main__':
    main()

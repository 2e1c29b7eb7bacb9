"""Round 5 probe: can the matrix-core and the VALU correlation kernels share the CUs?  4096^2 fp32, 15x15
(the planned path): the MFMA kernel alone, the VALU kernel alone, and both at once on two streams over
complementary row bands (fraction f to the MFMA kernel; the seam rows are wrong -- timing only).  Prints
JSON lines: microseconds per full-image pass."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pycsou_amd import _lib as L  # noqa: E402
from pycsou_amd.linop.conv import Convolve2D  # noqa: E402


def main():
    torch.cuda.set_device(0)
    lib = L.gpu()
    n = 4096
    h = np.random.default_rng(0).standard_normal((15, 15))
    op = Convolve2D(n * n, h, (n, n))
    tier, wpl = op.plan(torch.float32, False)
    x = torch.randn(n * n, device='cuda')
    out = torch.empty_like(x)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def launch(mf, r_lo, r_hi, st):
        os.environ['PCS_CORR_MFMA'] = '1' if mf else '0'
        off = r_lo * n * 4
        L.check(lib.pcs_conv2d_planned(L.PCS_F32, x.data_ptr() + off, out.data_ptr() + off, r_hi - r_lo, n,
                                       L.ptr(wpl), int(tier), None, 0.0, ctypes_stream(st)), 'conv')

    def ctypes_stream(st):
        import ctypes
        return ctypes.c_void_p(st.cuda_stream)

    def timed(fn, reps=50):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps

    cur = torch.cuda.current_stream()

    def both(f):
        cut = int(round(n * f / 16)) * 16

        def fn():
            ev = torch.cuda.Event()
            ev.record(cur)
            s1.wait_event(ev)
            s2.wait_event(ev)
            launch(True, 0, cut, s1)
            launch(False, cut, n, s2)
            e1, e2 = torch.cuda.Event(), torch.cuda.Event()
            e1.record(s1)
            e2.record(s2)
            cur.wait_event(e1)
            cur.wait_event(e2)
        return fn

    print(json.dumps({'mode': 'mfma', 'us': round(timed(lambda: launch(True, 0, n, cur)), 2)}), flush=True)
    print(json.dumps({'mode': 'valu', 'us': round(timed(lambda: launch(False, 0, n, cur)), 2)}), flush=True)
    for f in (0.5, 0.6, 0.7, 0.8):
        print(json.dumps({'mode': 'both', 'mfma_frac': f, 'us': round(timed(both(f)), 2)}), flush=True)
        print(json.dumps({'mode': 'mfma_band', 'mfma_frac': f,
                          'us': round(timed(lambda: launch(True, 0, int(round(n * f / 16)) * 16, cur)), 2)}), flush=True)


if __name__ == '__main__':
    main()

"""Can the in-plane normal operator run beside the 3-D update?  Times, on the C4 / C5 problem of
tools/bench3d.py, the update kernel (pcs_pds3d_step, no loop control) and one k_sep2d_nrm launch over a
volume of the same size (separate buffers) alone, back to back on one stream, and on two streams at once
(HIP events, median of 10).  Diagnostics for the two-stream 3-D schedule."""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pycsou_amd import _lib as L  # noqa: E402


def med(fn, n=10):
    for _ in range(2):
        fn()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--size', type=int, default=512)
    ap.add_argument('--dtype', default='f32', choices=['f32', 'f64'])
    args = ap.parse_args()
    torch.cuda.set_device(0)
    dtype = torch.float32 if args.dtype == 'f32' else torch.float64
    from bench3d import build
    from pycsou_amd.opt.engine3d import PDS3DEngine
    pds = build(args.size, dtype)
    spec = pds._fused_spec()
    eng = PDS3DEngine(spec, dtype, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, chunk=2, use_graph=False)
    del pds
    eng.init_loop(100, 100, -1.0)
    eng.advance(4)
    torch.cuda.synchronize()
    lib, n = eng.lib, args.size
    a = eng.args[0]
    a.hist = None
    xs = torch.randn(n, n, n, dtype=dtype, device='cuda')
    ts = torch.empty_like(xs)
    (ha, ka, oa), (hb, kb, ob) = eng._inplane_ab(False)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()

    def upd(st):
        L.check(lib.pcs_pds3d_step(ctypes.byref(a), ctypes.c_void_p(st.cuda_stream)), 'pcs_pds3d_step')

    def nrm(st):
        L.check(lib.pcs_conv2d_sep_ata_planes(L.dtcode(xs), L.ptr(xs), L.ptr(ts), n, n, n, L.ptr(ha), ka, oa, L.ptr(hb),
                                              kb, ob, ctypes.c_void_p(st.cuda_stream)), 'pcs_conv2d_sep_ata_planes')

    cur = torch.cuda.current_stream()

    def alone_upd():
        upd(cur)

    def alone_nrm():
        nrm(cur)

    def serial():
        upd(cur)
        nrm(cur)

    def both():
        sa.wait_stream(cur)
        sb.wait_stream(cur)
        upd(sa)
        nrm(sb)
        cur.wait_stream(sa)
        cur.wait_stream(sb)

    out = {'problem': f'{n}^3 {args.dtype}', 'fold': bool(getattr(eng, 'fold', False)),
           'update_ms': med(alone_upd), 'nrm_ms': med(alone_nrm), 'serial_ms': med(serial), 'two_streams_ms': med(both)}
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()

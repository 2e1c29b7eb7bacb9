"""Time the C3 fused step (k_pds2d_march) in several builds of the engine, alternating builds so
box drift hits all alike.  Diagnostics only (GPU box):

  python3 tools/march_ablate.py base=pycsou_amd/lib/libpycsou_hip.so v1=pycsou_amd/lib/var/v1/libpycsou_hip.so

Each build runs in its own process (the library is loaded at import): 300 ms spin-up, then the
isolated per-launch mean (HIP events around each of 100 launches) and the back-to-back rate
(200 launches, one event pair).  Variants with ablated phases compute wrong iterates; only
their timing is meaningful.
"""
import ctypes
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child():
    import torch
    import bench
    from pycsou_amd import _lib as L
    from pycsou_amd.opt.engine import PDS2DEngine
    torch.cuda.set_device(0)
    n = int(os.environ.get('PCS_N', '4096'))
    pds = bench.build_problem(n, n, torch.float32, kind=os.environ.get('PCS_KIND', 'forward'))
    if os.environ.get('PCS_KIND', 'forward') != 'forward':  # general-K engines: bench.py's timing
        r = bench.fused_2d(pds, torch.float32, 200, 20)
        print(f"RESULT {r['kernels_ms']['step'] * 1e3:.1f} {r['ms_per_step'] * 1e3:.1f} {r['nblocks']}", flush=True)
        return
    spec = pds._fused_spec()
    eng = PDS2DEngine(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, use_graph=False)
    N = 200
    eng.prepare_fixed(4 * N + 10, 2)
    a = eng.args
    a.hist = eng.hist.data_ptr() if eng.fused_finalize else None

    def b2b(k):
        L.check(eng.lib.pcs_ctrl_init2(L.ptr(eng.ctrl), k + 1, k + 1, -1.0, 1, int(eng.hist.numel()), L.stream()),
                'init')
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(k):
            p = i % 2
            a.x, a.xn = eng.X[p].data_ptr(), eng.X[1 - p].data_ptr()
            a.z, a.zn = eng.Z[p].data_ptr(), eng.Z[1 - p].data_ptr()
            L.check(eng.lib.pcs_pds2d_step(ctypes.byref(a), L.stream()), 'step')
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / k
    t0 = time.time()
    while time.time() - t0 < 0.3:
        b2b(50)
    iso = eng.time_step_kernel(100)
    bb = min(b2b(N) for _ in range(3))
    print(f'RESULT {iso * 1e3:.1f} {bb * 1e3:.1f} {eng.nblocks}', flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == '--child':
        return child()
    vs = [a.split('=', 1) for a in sys.argv[1:]]
    res = {k: [] for k, _ in vs}
    for rep in range(int(os.environ.get('PCS_REPS', '2'))):
        for k, path in (vs if rep % 2 == 0 else vs[::-1]):
            extra = {}
            if '@' in path:  # name=lib@VAR=value,VAR2=value: environment of that build's run
                path, ev = path.split('@', 1)
                extra = dict(kv.split('=', 1) for kv in ev.split(','))
            env = dict(os.environ, PCS_LIB_PATH=os.path.abspath(path), **extra)
            out = subprocess.run([sys.executable, __file__, '--child'], env=env, capture_output=True, text=True,
                                 timeout=240)
            line = [ln for ln in out.stdout.splitlines() if ln.startswith('RESULT')]
            if not line:
                print(k, 'FAILED', out.stderr[-2000:], flush=True)
                return 1
            iso, bb, nbk = map(float, line[0].split()[1:])
            res[k].append((iso, bb))
            print(f'{k:>10s} rep {rep}: isolated {iso:6.1f} us  back-to-back {bb:6.1f} us  ({nbk:.0f} workgroups)', flush=True)
    for k, r in res.items():
        print(f'{k:>10s} best: isolated {min(i for i, _ in r):6.1f} us  back-to-back {min(b for _, b in r):6.1f} us')
    return 0


if __name__ == '__main__':
    sys.exit(main())

"""Where a march-kernel step spends its cycles: loads the diagnostic build
(`make stamps` -> pycsou_amd/lib/diag/libpycsou_hip.so, s_memtime stamps around every
phase and barrier), runs a few eager C3 iterations and prints the per-step share of each
segment for wave 0 (busy in every phase) and wave 3 (idle in P1-P3).  Read the SHARES, not
the absolute time (the stamps' waits forbid some overlap)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ['PCS_LIB_PATH'] = os.path.join(ROOT, 'pycsou_amd', 'lib', 'diag', 'libpycsou_hip.so')
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from pycsou_amd import _lib as L  # noqa: E402
from pycsou_amd.opt.engine import PDS2DEngine  # noqa: E402

SEG = ['-', 'bar0', 'loads', 'P1', 'bar1', 'P2', 'bar2', 'P3', 'land', 'bar3', 'P45', 'bar4', 'P6']


def main():
    n = int(os.environ.get('PCS_N', '4096'))
    torch.cuda.set_device(0)
    pds = bench.build_problem(n, n, torch.float32)
    eng = PDS2DEngine(pds._fused_spec(), torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, use_graph=False)
    eng.chunk = 2
    eng.run(3, 3, 0.0)
    torch.cuda.synchronize()
    lib = ctypes.CDLL(L.LIB_PATH)
    buf = np.zeros((4096, 16), dtype=np.uint64)
    rc = lib.pcs_debug_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_int64(buf.nbytes))
    assert rc == 0, rc
    nb = eng.nblocks
    for w, name in ((0, 'wave0'), (1, 'wave3')):
        rows = buf[w:2 * nb:2]
        rows = rows[rows[:, 13] > 0]
        per = rows[:, :13].astype(np.float64) / rows[:, 13:14]
        m = per.mean(axis=0)
        tot = m.sum()
        print(f'{name}: blocks={len(rows)} cycles/step={tot:.0f}  ' +
              '  '.join(f'{s}={v:.0f}({100 * v / tot:.0f}%)' for s, v in zip(SEG, m)), flush=True)


if __name__ == '__main__':
    main()

"""Time the REAL reference's PDS beside the CPU restatement that bench.py's `cpu_baseline` runs
('Reference CPU path beside it'), in this container only (/root/reference does
not exist on the GPU box):  ``python tests/golden/time_reference_cpu.py``.

1. C3-shaped TV-deconvolution with the anisotropic 0.05*L1Norm (the isotropic L21Norm of the
   reference is an O(G*N) Python loop, infeasible at these sizes): reference PDS (shimmed
   import, PyLops arithmetic from oracle.pylops1 inside the reference's PyLopLinearOperator)
   vs the restatement, same op sequence, fixed 3 iterations, fp64, one core.
2. The reference's isotropic L21 PDS per-iteration time at 32^2..128^2 and its O(N^2)
   extrapolation to 2048^2 / 4096^2.

Writes tests/golden/cpu_baseline_check.json.
"""

import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from make_golden import import_reference  # noqa: E402


def problem(n, seed=0):
    from oracle.pycsou_ref import gaussian_psf, phantom
    from oracle import pylops1 as P
    N = n * n
    xs = phantom((n, n), 64, seed).ravel()
    h = gaussian_psf(15, 2.0)
    Cr = P.Convolve2D(N, h, (n, n), offset=(7, 7), method='fft')
    y = Cr.matvec(xs) + 0.01 * np.random.default_rng(1).standard_normal(N)
    return N, h, Cr, y


def time_reference(R, n, hname, iters):
    from oracle import pylops1 as P
    PyLop = R.lbase.PyLopLinearOperator
    N, h, Cr, y = problem(n)
    Conv = PyLop(Cr)
    Conv.lipschitz_cst = Conv.diff_lipschitz_cst = 1.0
    K = PyLop(P.Gradient((n, n), sampling=1., edge=True, kind='forward'))
    K.lipschitz_cst = K.diff_lipschitz_cst = float(np.sqrt(8 * np.sin(np.pi * (n - 1) / (2 * n)) ** 2))
    F = (1 / 2) * R.loss.SquaredL2Loss(dim=N, data=y) * Conv
    if hname == 'l1':
        H = 0.05 * R.penalty.L1Norm(dim=2 * N)
    else:
        H = 0.05 * R.penalty.L21Norm(dim=2 * N, groups=np.tile(np.arange(N), 2))
    pds = R.proxalgs.PDS(dim=N, F=F, H=H, K=K, max_iter=iters - 1, min_iter=iters - 1, accuracy_threshold=0.0,
                         verbose=None)
    t0 = time.perf_counter()
    est, _, _ = pds.iterate()
    dt = time.perf_counter() - t0
    return dt / iters, est['primal_variable']


def time_restatement(n, iters):
    """The op sequence of bench.py's cpu_baseline with H = 0.05 L1 (anisotropic)."""
    from oracle import pycsou_ref as OR
    from oracle import pylops1 as P
    N, h, Cr, y = problem(n)
    Kr = P.Gradient((n, n), edge=True, kind='forward')
    Klip = float(np.sqrt(8 * np.sin(np.pi * (n - 1) / (2 * n)) ** 2))
    tau, sigma = OR.pds_step_sizes(1.0, Klip)
    hprox = OR.postcomp(OR.prox_l1, 0.05)
    t0 = time.perf_counter()
    x, _, _ = OR.pds(lambda x: Cr.rmatvec((2 * (Cr.matvec(x) + (-y))) * 0.5), lambda v, t: v, Kr.matvec, Kr.rmatvec,
                     lambda w, s: OR.fenchel_prox(hprox, w, s), tau, sigma, 0.9, np.zeros(N), np.zeros(2 * N),
                     max_iter=iters - 1, min_iter=iters - 1, accuracy_threshold=0.0, pandas_diagnostics=True)
    dt = time.perf_counter() - t0
    return dt / iters, x


def main():
    R = import_reference()
    out = {'host': {'nproc': os.cpu_count(), 'OMP_NUM_THREADS': os.environ.get('OMP_NUM_THREADS')},
           'anisotropic_l1': [], 'isotropic_l21_reference': []}
    for n, iters in ((512, 3), (1024, 3), (2048, 3), (4096, 2)):
        tr, xr = time_reference(R, n, 'l1', iters)
        ts, xs = time_restatement(n, iters)
        rel = float(np.linalg.norm(xr - xs) / np.linalg.norm(xr))
        row = {'n': n, 'iters': iters, 'reference_s_per_iter': round(tr, 4), 'restatement_s_per_iter': round(ts, 4),
               'restatement_over_reference': round(ts / tr, 3), 'iterate_rel_diff': rel}
        print(row, flush=True)
        out['anisotropic_l1'].append(row)
    pts = []
    for n in (32, 64, 128):
        t, _ = time_reference(R, n, 'l21', 2)
        pts.append((n * n, t))
        out['isotropic_l21_reference'].append({'n': n, 's_per_iter': round(t, 4)})
        print('l21', n, t, flush=True)
    # O(N^2) fit through the largest point (the G x N group loop dominates)
    N0, t0 = pts[-1]
    out['isotropic_l21_extrapolated_s_per_iter'] = {str(n): round(t0 * (n * n / N0) ** 2, 1) for n in (2048, 4096)}
    json.dump(out, open(os.path.join(HERE, 'cpu_baseline_check.json'), 'w'), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()

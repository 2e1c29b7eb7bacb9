"""Golden trajectories of the thin PDS parameterisations and the operator defaults, from the
REAL reference (same import recipe as make_golden.py; run in the build container only):

  python tests/golden/make_golden_solvers.py   ->   tests/golden/solvers.npz

Cases (every array is an input or an expected output):
  * DRS (pycsou/opt/proxalgs.py:719-781): G = 0.3 L1Norm.shifter(-y), H = 0.2 L2Norm, K = I,
    sigma = 1/tau, rho = 1 -- a fixed 30-iteration run at tau = 0.7 and a natural stop at the
    default tau = 1 (accuracy_threshold 1e-3, min_iter 10).
  * FBS (proxalgs.py:784-862): F = 1/2 ||A x - y||^2 with a DenseLinearOperator, G = lam L1
    (default tau = 2/beta, rho = 1, no dual variable); and F = 1/2 ||h * x - y||^2 on a 40 x 36
    image with a 5 x 5 PSF, G = NonNegativeOrthant.
  * PDS with the default K (H given, K None -> IdentityOperator, linop/base.py:582-598).
  * PDS with a vector DiagonalOperator K (linop/base.py:551-579; lipschitz_cst = max(diag)).
  * GenericIterativeAlgorithm.iterates(4) (pycsou/core/solver.py:88-103) on the PDS above.
"""

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)


def main():
    from make_golden import import_reference
    R = import_reference()
    from oracle import pylops1 as P
    pen, loss, lbase, proxalgs = R.penalty, R.loss, R.lbase, R.proxalgs
    out = {}

    def put(tag, **arrays):
        for k, v in arrays.items():
            out[f'{tag}_{k}'] = np.asarray(v)

    def diag_cols(d):
        cols = {'diag_primal': d['Relative Improvement (primal variable)'].to_numpy(float)}
        if 'Relative Improvement (dual variable)' in d:
            cols['diag_dual'] = d['Relative Improvement (dual variable)'].to_numpy(float)
        return cols

    rng = np.random.default_rng(11)
    # ---------------- DRS ----------------
    N = 200
    y = rng.standard_normal(N)
    put('drs', y=y)
    for tag, tau, niter, thr, mi in [('drs_fixed', 0.7, 30, 0.0, 29), ('drs_stop', None, 500, 1e-3, 10)]:
        G = 0.3 * pen.L1Norm(dim=N).shifter(-y)
        H = 0.2 * pen.L2Norm(dim=N)
        kw = {} if tau is None else {'tau': tau}
        drs = proxalgs.DRS(dim=N, G=G, H=H, x0=np.zeros(N), z0=np.zeros(N), max_iter=niter - 1, min_iter=mi,
                           accuracy_threshold=thr, verbose=None, **kw)
        est, conv, d = drs.iterate()
        put(tag, x=est['primal_variable'], z=est['dual_variable'], n_iter=drs.iter, tau=drs.tau, sigma=drs.sigma,
            rho=drs.rho, max_iter=niter - 1, min_iter=mi, thr=thr, **diag_cols(d))
        print(tag, 'iters', drs.iter)

    # ---------------- FBS, dense LASSO ----------------
    A = rng.standard_normal((64, 128))
    xs = np.zeros(128)
    xs[rng.choice(128, 8, replace=False)] = 1.0
    yA = A @ xs
    Gop = lbase.DenseLinearOperator(A)
    Gop.lipschitz_cst = Gop.diff_lipschitz_cst = float(np.linalg.norm(A, 2))
    F = (1 / 2) * loss.SquaredL2Loss(dim=64, data=yA) * Gop
    lam = 0.1 * float(np.max(np.abs(F.gradient(np.zeros(128)))))
    fbs = proxalgs.FBS(dim=128, F=F, G=lam * pen.L1Norm(dim=128), x0=np.zeros(128), max_iter=39, min_iter=39,
                       accuracy_threshold=0.0, verbose=None)
    est, conv, d = fbs.iterate()
    put('fbs_dense', A=A, y=yA, lam=lam, Alip=Gop.lipschitz_cst, x=est['primal_variable'], n_iter=fbs.iter,
        tau=fbs.tau, beta=fbs.beta, dual_is_none=est['dual_variable'] is None, **diag_cols(d))
    print('fbs_dense iters', fbs.iter, 'tau', fbs.tau)

    # ---------------- FBS, 2-D deconvolution, nonnegativity ----------------
    shape = (40, 36)
    Nc = shape[0] * shape[1]
    psf = rng.uniform(0.0, 1.0, (5, 5))
    psf /= psf.sum()
    off = tuple(P.pycsou_offset(n) for n in psf.shape)
    Conv = lbase.PyLopLinearOperator(P.Convolve2D(Nc, psf, shape, offset=off))
    Conv.lipschitz_cst = Conv.diff_lipschitz_cst = 1.0
    img = np.zeros(shape)
    img[8:20, 5:25] = 1.0
    img[25:35, 10:30] = 0.5
    yc = Conv(img.ravel()) + 0.01 * rng.standard_normal(Nc)
    F = (1 / 2) * loss.SquaredL2Loss(dim=Nc, data=yc) * Conv
    fbs = proxalgs.FBS(dim=Nc, F=F, G=pen.NonNegativeOrthant(dim=Nc), x0=np.zeros(Nc), max_iter=24, min_iter=24,
                       accuracy_threshold=0.0, verbose=None)
    est, conv, d = fbs.iterate()
    put('fbs_deconv', shape=shape, psf=psf, y=yc, x=est['primal_variable'], n_iter=fbs.iter, tau=fbs.tau,
        **diag_cols(d))
    print('fbs_deconv iters', fbs.iter)

    # ---------------- PDS with K = None (IdentityOperator) and a vector DiagonalOperator ----------------
    Nd = 300
    yd = np.cumsum(rng.standard_normal(Nd)) * 0.1
    dvec = rng.uniform(0.5, 2.0, Nd)
    put('pds_k', y=yd, dvec=dvec)
    for tag, K in [('pds_kid', None), ('pds_kdiag', lbase.DiagonalOperator(dvec))]:
        F = (1 / 2) * loss.SquaredL2Loss(dim=Nd, data=yd)
        H = 0.1 * pen.L1Norm(dim=Nd)
        pds = proxalgs.PDS(dim=Nd, F=F, H=H, K=K, x0=np.zeros(Nd), z0=np.zeros(Nd), max_iter=24, min_iter=24,
                           accuracy_threshold=0.0, verbose=None)
        est, conv, d = pds.iterate()
        put(tag, x=est['primal_variable'], z=est['dual_variable'], n_iter=pds.iter, tau=pds.tau, sigma=pds.sigma,
            rho=pds.rho, Klip=pds.K.lipschitz_cst, **diag_cols(d))
        print(tag, 'iters', pds.iter, 'tau', pds.tau)

    # ---------------- iterates(4) on the K = I problem ----------------
    pds = proxalgs.PDS(dim=Nd, F=(1 / 2) * loss.SquaredL2Loss(dim=Nd, data=yd), H=0.1 * pen.L1Norm(dim=Nd),
                       x0=np.zeros(Nd), z0=np.zeros(Nd), verbose=None)
    xs_it, zs_it = [], []
    for it in pds.iterates(4):
        xs_it.append(np.array(it['primal_variable']))
        zs_it.append(np.array(it['dual_variable']))
    put('iterates', x=np.stack(xs_it), z=np.stack(zs_it), iter_after=pds.iter)

    np.savez_compressed(os.path.join(HERE, 'solvers.npz'), **out)
    print('solvers.npz', len(out), 'arrays')


if __name__ == '__main__':
    main()

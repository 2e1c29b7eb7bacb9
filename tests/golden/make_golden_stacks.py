"""Golden fixtures for the widened operator set, from the REAL
reference code imported as in ``make_golden.py`` (same stand-in modules, nothing copied).

Build container only:  ``python tests/golden/make_golden_stacks.py``  ->  ``tests/golden/stacks.npz``,
``tests/golden/cps_inpaint.npz``, ``tests/golden/apgd_tikhonov.npz``.

The reference's own ``LinOpStack`` / ``LinOpVStack`` / ``LinOpHStack`` (``pycsou/linop/base.py:159-302``),
``ProxFuncHStack`` / ``DiffFuncHStack`` (``pycsou/func/base.py:21-137``), ``Masking`` / ``DownSampling``
(``pycsou/linop/sampling.py:125-391``), ``PolynomialLinearOperator`` (``linop/base.py:636-700``),
``GeneralisedLaplacian`` / ``GeneralisedDerivative`` / ``SecondDerivative`` / ``MovingAverage1D/2D`` /
``SubSampling`` (``linop/diff.py``, ``linop/conv.py``, ``linop/sampling.py``) and ``CPS`` / ``APGD``
(``pycsou/opt/proxalgs.py``) produce the vectors.  The reference's wrappers call the absent
third-party PyLops 1.x; its arithmetic is supplied from ``oracle.pylops1`` by attaching the
restated operators to the stand-in ``pylops`` module (parity at that boundary is pinned only
by the restatement -- see DESIGN.md).  The notebook workflows reproduced: cell [55] (APGD, Tikhonov
+ Segment), cell [62] (CPS, ``K = LinOpVStack(Masking, Gradient)``,
``H = ProxFuncHStack(L1Loss, mu L1Norm)``, ``G = Segment``).
"""

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)


def main():
    from make_golden import import_reference
    from oracle import pylops1 as P
    from oracle.pycsou_ref import phantom
    R = import_reference()
    pylops = sys.modules['pylops']
    pylops.FirstDerivative = lambda N, dims=None, dir=0, sampling=1., edge=False, dtype='float64', kind='centered': \
        P.FirstDerivative(N, dims=dims, dir=dir, sampling=sampling, edge=edge, dtype=dtype, kind=kind)
    pylops.SecondDerivative = lambda N, dims=None, dir=0, sampling=1., edge=False, dtype='float64': \
        P.SecondDerivative(N, dims=dims, dir=dir, sampling=sampling, edge=edge, dtype=dtype)
    pylops.Gradient = lambda dims, sampling=1, edge=False, dtype='float64', kind='centered': \
        P.Gradient(dims, sampling=sampling, edge=edge, dtype=dtype, kind=kind)
    pylops.Laplacian = lambda dims, weights=(1, 1), sampling=(1, 1), edge=False, dtype='float64': \
        P.Laplacian(dims, weights=weights, sampling=sampling if np.ndim(sampling) else (sampling, sampling),
                    edge=edge, dtype=dtype)
    pylops.Smoothing1D = P.Smoothing1D
    pylops.Smoothing2D = P.Smoothing2D
    pylops.Restriction = P.Restriction
    from pycsou.linop import diff as rdiff, conv as rconv, sampling as rsamp
    lb, fb, pen, loss = R.lbase, R.fbase, R.penalty, R.loss

    out = {}
    rng = np.random.default_rng(11)
    shape = (12, 9)
    N = int(np.prod(shape))
    x = rng.standard_normal(N)
    out['x'] = x
    # ---- stacks of linear operators (doctest of linop/base.py:205-229 at a small size)
    D1 = rdiff.FirstDerivative(size=N, shape=shape, axis=0, kind='centered')
    D2 = rdiff.FirstDerivative(size=N, shape=shape, axis=1, kind='forward')
    V = lb.LinOpStack(D1, D2, axis=0)
    out['vstack_fwd'] = V(x)
    w = rng.standard_normal(2 * N)
    out['w'] = w
    out['vstack_adj'] = V.adjoint(w)
    Hs = lb.LinOpHStack(D1.H, D2.H)
    out['hstack_fwd'] = Hs(w)
    out['hstack_adj'] = Hs.adjoint(x)
    A = rng.standard_normal((5, N))
    Dn = lb.DenseLinearOperator(A)
    Dn.compute_lipschitz_cst()
    V2 = lb.LinOpVStack(Dn, D2)
    out['A'] = A
    out['vstack2_fwd'] = V2(x)
    out['vstack2_adj'] = V2.adjoint(np.concatenate([w[:5], w[:N]]))
    # ---- functional stacks (func/base.py:21-137)
    z = rng.standard_normal(2 * N)
    out['z'] = z
    f1, f2 = pen.L1Norm(dim=N), pen.L2Norm(dim=N)
    hs = fb.ProxFuncHStack(f1, 0.7 * f2)
    out['phs_value'] = np.array(hs(z))
    out['phs_prox_03'] = hs.prox(z.copy(), 0.3)
    out['phs_fenchel_05'] = hs.fenchel_prox(z.copy(), 0.5)
    yd = rng.standard_normal(N)
    out['yd'] = yd
    hs2 = fb.ProxFuncHStack(loss.L1Loss(dim=N, data=yd), 0.6 * pen.L1Norm(dim=N))
    out['phs2_prox_04'] = hs2.prox(z.copy(), 0.4)
    out['phs2_fenchel_07'] = hs2.fenchel_prox(z.copy(), 0.7)
    dh = fb.DiffFuncHStack(pen.SquaredL2Norm(dim=N), loss.SquaredL2Loss(dim=N, data=yd))
    out['dhs_value'] = np.array(dh(z))
    out['dhs_grad'] = dh.gradient(z)
    # ---- sampling (sampling.py) -- pure NumPy in the reference
    mask = rng.uniform(size=N) < 0.3
    M = rsamp.Masking(size=N, sampling_bool=mask)
    out['mask'] = mask
    out['mask_fwd'] = M(x)
    out['mask_adj'] = M.adjoint(M(x))
    Ds = rsamp.DownSampling(size=N, shape=shape, downsampling_factor=(3, 2))
    out['down_fwd'] = Ds(x)
    out['down_adj'] = Ds.adjoint(Ds(x))
    out['down_shape'] = np.array(Ds.output_shape)
    Da = rsamp.DownSampling(size=N, shape=shape, downsampling_factor=2, axis=1)
    out['downax_fwd'] = Da(x)
    out['downax_shape'] = np.array(Da.output_shape)
    iava = np.array([0, 3, 4, 8])
    Ss = rsamp.SubSampling(size=N, sampling_indices=iava, shape=shape, axis=0)
    out['iava'] = iava
    out['sub_fwd'] = Ss(x)
    out['sub_adj'] = Ss.adjoint(Ss(x))
    # ---- derivatives / generalised operators / moving averages
    sd = rdiff.SecondDerivative(size=N, shape=shape, axis=1, step=0.5, edge=True)
    out['d2_fwd'] = sd(x)
    out['d2_adj'] = sd.adjoint(x)
    sd0 = rdiff.SecondDerivative(size=N, shape=shape, axis=0, edge=False)
    out['d2ax0_fwd'] = sd0(x)
    out['d2ax0_adj'] = sd0.adjoint(x)
    gl = rdiff.GeneralisedLaplacian(shape=shape, kind='sobolev', order=2, constant=0.5)
    out['glap_sob_fwd'] = gl(x)
    out['glap_sob_adj'] = gl.adjoint(x)
    gl2 = rdiff.GeneralisedLaplacian(shape=shape, kind='polynomial', coeffs=[0.5, -1.0, 0.25])
    out['glap_pol_fwd'] = gl2(x)
    gd = rdiff.GeneralisedDerivative(size=N, shape=shape, axis=1, kind_op='exponential', order=2, constant=-0.1,
                                     kind_diff='forward')
    out['gder_exp_fwd'] = gd(x)
    out['gder_exp_adj'] = gd.adjoint(x)
    Dsq = lb.DenseLinearOperator(rng.standard_normal((N, N)) / N)
    out['Asq'] = Dsq.mat
    pl = lb.PolynomialLinearOperator(LinOp=Dsq, coeffs=[1.0, -0.5, 2.0])
    out['poly_fwd'] = pl(x)
    out['poly_adj'] = pl.adjoint(x)
    ma1 = rconv.MovingAverage1D(window_size=4, shape=shape, axis=0)
    out['ma1_fwd'] = ma1(x)
    out['ma1_adj'] = ma1.adjoint(x)
    ma2 = rconv.MovingAverage2D(window_shape=(3, 6), shape=shape)
    out['ma2_fwd'] = ma2(x)
    out['ma2_adj'] = ma2.adjoint(x)
    np.savez(os.path.join(HERE, 'stacks.npz'), **out)
    print('stacks.npz', len(out), 'arrays')

    # ---- notebook cell [62]: TV-LAD inpainting with CPS and stacked K / H
    img = phantom((40, 36), n_rect=12, seed=5)
    n = img.size
    r2 = np.random.default_rng(6)
    bmask = r2.binomial(1, p=0.25, size=n).astype(bool)
    Gop = rsamp.Masking(size=n, sampling_bool=bmask)
    Gop.lipschitz_cst = Gop.diff_lipschitz_cst = 1.0
    yv = Gop(img.ravel())
    yv[r2.binomial(n=1, p=0.02, size=yv.size).astype(bool)] = 1.0
    D = rdiff.Gradient(shape=img.shape, kind='forward')
    D.lipschitz_cst = D.diff_lipschitz_cst = np.sqrt(8.0)
    mu = 0.6
    res = {'mask': bmask, 'y': yv, 'shape': np.array(img.shape), 'mu': np.array(mu)}
    for tag, niter, thr, mi in [('fixed', 40, 0.0, 39), ('stop', 500, 1e-2, 10)]:
        H = fb.ProxFuncHStack(loss.L1Loss(dim=yv.size, data=yv), mu * pen.L1Norm(dim=D.shape[0]))
        K = lb.LinOpVStack(Gop, D)
        G = pen.Segment(dim=n, a=0, b=1)
        cps = R.proxalgs.CPS(dim=n, G=G, H=H, K=K, max_iter=niter - 1, min_iter=mi, accuracy_threshold=thr,
                             verbose=None)
        est, conv, diag = cps.iterate()
        for k, v in dict(x=est['primal_variable'], z=est['dual_variable'], n_iter=cps.iter, tau=cps.tau,
                         sigma=cps.sigma, rho=cps.rho, Klip=K.lipschitz_cst,
                         diag_primal=diag['Relative Improvement (primal variable)'].to_numpy(float),
                         diag_dual=diag['Relative Improvement (dual variable)'].to_numpy(float),
                         max_iter=niter - 1, min_iter=mi, thr=thr).items():
            res[f'{tag}_{k}'] = np.asarray(v)
        print('cps', tag, 'iters', cps.iter)
    np.savez_compressed(os.path.join(HERE, 'cps_inpaint.npz'), **res)

    # ---- notebook cell [55]: APGD, F = 1/2 ||Gop x - y||^2 + mu/2 ||D x||^2, G = Segment
    F = ((1 / 2) * loss.SquaredL2Loss(dim=yv.size, data=yv) * Gop) + \
        ((0.1 * (1.0 / 8.0) / 2) * pen.SquaredL2Norm(dim=D.shape[0]) * D)
    G = pen.Segment(dim=n, a=0, b=1)
    res = {'mask': bmask, 'y': yv, 'shape': np.array(img.shape), 'mu': np.array(0.1 / 8.0)}
    apgd = R.proxalgs.APGD(dim=n, F=F, G=G, max_iter=59, min_iter=59, accuracy_threshold=0.0, verbose=None)
    est, conv, diag = apgd.iterate()
    for k, v in dict(x=est['iterand'], n_iter=apgd.iter, tau=apgd.tau, beta=apgd.beta,
                     diag=diag['Relative Improvement'].to_numpy(float)).items():
        res[k] = np.asarray(v)
    print('apgd tikhonov iters', apgd.iter, 'beta', apgd.beta)
    np.savez_compressed(os.path.join(HERE, 'apgd_tikhonov.npz'), **res)


if __name__ == '__main__':
    main()

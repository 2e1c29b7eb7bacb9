"""Generate the golden fixtures in ``tests/golden/`` from the REAL reference code.

Run in the build container only (``/root/reference`` does not exist on the GPU
box):  ``python tests/golden/make_golden.py``.

How the reference is run
------------------------
``import pycsou`` fails here for ordinary reasons: numba /
dask / pylops are not installed and NumPy 2 removed ``np.infty``/``np.float``/
``np.alltrue``/``np.asscalar``.  We therefore pre-register small in-memory
stand-in *modules* for the three absent packages (``numba.njit`` = identity,
``dask.array.core.Array`` = placeholder type, ``pylops`` = empty namespaces:
none of them is on the hot path except PyLops' arithmetic, see below), alias
the four removed NumPy names, and import the reference read-only with
``sys.dont_write_bytecode``.  Nothing from ``/root/reference`` is copied.

With that, the reference's OWN ``PrimalDualSplitting``, ``APGD``,
``L1Norm``/``L2Norm``/``L21Norm``/``SquaredL2Norm``/``SquaredL2Loss``,
``fenchel_prox``, operator algebra, ``DenseLinearOperator`` and
``PyLopLinearOperator`` produce the vectors below.  The PyLops arithmetic
(derivatives, convolutions) that the reference delegates to the absent
third-party package is supplied by ``oracle.pylops1`` objects wrapped in the
reference's own ``PyLopLinearOperator`` (``pycsou/linop/base.py:24-54``).

Outputs: ``tests/golden/*.npz`` (inputs and expected outputs; plain arrays,
loadable with ``np.load(allow_pickle=False)``).
"""

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'
sys.path.insert(0, REPO)


def import_reference():
    sys.dont_write_bytecode = True
    np.infty = np.inf
    np.float = float
    np.alltrue = np.all
    np.asscalar = lambda a: np.asarray(a).item()

    numba = types.ModuleType('numba')
    numba.njit = lambda *a, **k: (a[0] if a and callable(a[0]) else (lambda f: f))
    dask = types.ModuleType('dask')
    dask_array = types.ModuleType('dask.array')
    dask_core = types.ModuleType('dask.array.core')

    class _DaskArray:  # placeholder type for isinstance checks only
        pass

    dask_core.Array = _DaskArray
    dask_array.core = dask_core
    dask.array = dask_array
    pylops = types.ModuleType('pylops')
    pylops_opt = types.ModuleType('pylops.optimization')
    pylops_ls = types.ModuleType('pylops.optimization.leastsquares')
    pylops_ls.NormalEquationsInversion = None
    pylops_sp = types.ModuleType('pylops.signalprocessing')
    pylops.LinearOperator = object
    pylops.optimization = pylops_opt
    pylops_opt.leastsquares = pylops_ls
    pylops.signalprocessing = pylops_sp
    skimage = types.ModuleType('skimage')
    skimage_measure = types.ModuleType('skimage.measure')
    skimage_measure.block_reduce = None
    skimage.measure = skimage_measure
    for name, mod in [('numba', numba), ('dask', dask), ('dask.array', dask_array),
                      ('dask.array.core', dask_core), ('pylops', pylops),
                      ('pylops.optimization', pylops_opt), ('pylops.optimization.leastsquares', pylops_ls),
                      ('pylops.signalprocessing', pylops_sp), ('skimage', skimage),
                      ('skimage.measure', skimage_measure)]:
        sys.modules.setdefault(name, mod)
    sys.path.insert(0, REF)
    import pycsou.core  # noqa: F401
    from pycsou.opt import proxalgs
    from pycsou.func import penalty, loss, base as fbase
    from pycsou.linop import base as lbase
    from pycsou.math import prox as mprox
    return types.SimpleNamespace(proxalgs=proxalgs, penalty=penalty, loss=loss, fbase=fbase, lbase=lbase,
                                 mprox=mprox)


def main():
    R = import_reference()
    from oracle import pylops1 as P
    from oracle.pycsou_ref import gaussian_psf, gaussian_taps, phantom

    PyLop = R.lbase.PyLopLinearOperator
    out = {}
    only = [c for c in os.environ.get('GOLDEN_ONLY', '').split(',') if c]  # regenerate just these PDS cases

    # ---------------- prox / functional known answers ----------------
    pen, loss = R.penalty, R.loss
    x10 = np.arange(10, dtype=np.float64)
    rng = np.random.default_rng(1)
    v = rng.standard_normal(200)
    groups = np.repeat(np.arange(40), 5)
    rng.shuffle(groups)
    l21 = pen.L21Norm(dim=200, groups=groups)
    pix = np.tile(np.arange(100), 2)
    l21pix = pen.L21Norm(dim=200, groups=pix)
    vz = v.copy()
    vz[[3, 103]] = 0.0  # a zero-norm pixel group (pixel 3 in both components)
    f = {
        'x': v, 'groups': groups, 'vz': vz,
        'l1_prox_07': pen.L1Norm(200).prox(v.copy(), 0.7),
        'l1_value': np.array(pen.L1Norm(200)(v)),
        'l2_prox_3': pen.L2Norm(200).prox(v.copy(), 3.0),
        'l2_prox_30': pen.L2Norm(200).prox(v.copy(), 30.0),
        'l21_prox_05': l21.prox(v.copy(), 0.5),
        'l21_value': np.array(l21(v)),
        'l21pix_prox_05': l21pix.prox(vz.copy(), 0.5),
        'l21pix_value': np.array(l21pix(vz)),
        'fenchel_l1_lam03_s07': (0.3 * pen.L1Norm(200)).fenchel_prox(v.copy(), 0.7),
        'fenchel_l21pix_lam03_s07': (0.3 * l21pix).fenchel_prox(vz.copy(), 0.7),
        'sql2_value': np.array(pen.SquaredL2Norm(200)(v)),
        'sql2_grad': pen.SquaredL2Norm(200).gradient(v),
        'nonneg': pen.NonNegativeOrthant(200).prox(v.copy(), 1.0),
        'segment': pen.Segment(200, a=-0.5, b=0.25).prox(v.copy(), 1.0),
        # doctest values (pycsou/func/penalty.py:35-46, 88-103, 207-218, 494-509)
        'doc_l1_arange': np.array(pen.L1Norm(10)(x10)),
        'doc_l2_arange': np.array(pen.L2Norm(10)(x10)),
        'doc_l21_arange': np.array(pen.L21Norm(10, groups=np.concatenate((np.ones(5), 2 * np.ones(5))))(x10)),
        'doc_sql2_arange': np.array(pen.SquaredL2Norm(10)(x10)),
        'doc_soft': R.mprox.soft(np.linspace(-1, 1, 5), 0.5),
    }
    if not only:
        np.savez(os.path.join(HERE, 'prox.npz'), **f)
    print('prox.npz', {k: np.shape(a) for k, a in f.items()})

    # ---------------- operator goldens (PyLops boundary) ----------------
    from scipy import signal
    ops = {}
    sig = np.zeros((100, 100))
    sig[48:53, 48:53] = 1
    filt = signal.windows.hann(25)
    filt[filt.size // 2:] = 0
    filt = filt[None, :] * filt[:, None]
    ops['doc_conv2d_x'] = sig.ravel()
    ops['doc_conv2d_h'] = filt
    ops['doc_conv2d_y'] = signal.convolve(sig, filt, mode='same', method='fft').ravel()  # conv.py:209-217
    s1 = np.repeat([0., 1., 0.], 10)
    f1 = signal.windows.hann(5)
    f1[f1.size // 2:] = 0
    ops['doc_conv1d_x'], ops['doc_conv1d_h'] = s1, f1
    ops['doc_conv1d_y'] = signal.convolve(s1, f1, mode='same', method='direct')  # conv.py:67-73
    xd = np.repeat([0, 2, 1, 3, 0, 2, 0], 10).astype(np.float64)
    ops['doc_d1_x'] = xd
    ops['doc_d1_y'] = np.diff(xd, append=0)  # diff.py:72-78
    if not only:
        np.savez(os.path.join(HERE, 'ops.npz'), **ops)

    # ---------------- solver trajectories from the reference PDS / APGD ----------------
    PDS, APGD = R.proxalgs.PDS, R.proxalgs.APGD

    def run_pds(shape, psf, lam, kind, hname, niter, gname=None, seed=0, thr=0.0, min_iter=None, conv1d=None):
        N = int(np.prod(shape))
        d = len(shape)
        xs = phantom(shape, n_rect=16, seed=seed)
        rng = np.random.default_rng(seed + 7)
        if psf is not None:
            off = tuple(P.pycsou_offset(n) for n in psf.shape)
            Conv = PyLop(P.Convolve2D(N, psf, shape, offset=off))
            Conv.lipschitz_cst = Conv.diff_lipschitz_cst = 1.0
            y = Conv(xs.ravel()) + 0.01 * rng.standard_normal(N)
        elif conv1d is not None:
            Conv = None
            for ax in range(d):
                C = PyLop(P.Convolve1D(N, conv1d, offset=P.pycsou_offset(conv1d.size), dims=shape, dir=ax))
                C.lipschitz_cst = C.diff_lipschitz_cst = 1.0
                Conv = C if Conv is None else C * Conv
            Conv.lipschitz_cst = Conv.diff_lipschitz_cst = 1.0
            y = Conv(xs.ravel()) + 0.01 * rng.standard_normal(N)
        else:
            Conv = None
            y = xs.ravel() + 0.1 * rng.standard_normal(N)
        if kind == 'lap':
            K = PyLop(P.Laplacian(shape, weights=(1, 1), sampling=(1., 1.), edge=True))
            Klip = 8.0
            Hdim = N
        else:
            K = PyLop(P.Gradient(shape, sampling=1., edge=True, kind=kind))
            Klip = np.sqrt(4.0 * d)
            Hdim = d * N
        K.lipschitz_cst = K.diff_lipschitz_cst = Klip
        F = (1 / 2) * loss.SquaredL2Loss(dim=N, data=y)
        if Conv is not None:
            F = F * Conv
        if hname == 'l21':
            H = lam * pen.L21Norm(dim=Hdim, groups=np.tile(np.arange(N), Hdim // N))
        else:
            H = lam * pen.L1Norm(dim=Hdim)
        G = None
        if gname == 'nonneg':
            G = pen.NonNegativeOrthant(dim=N)
        elif gname == 'segment':
            G = pen.Segment(dim=N, a=0.0, b=1.0)
        pds = PDS(dim=N, F=F, G=G, H=H, K=K, x0=np.zeros(N), z0=np.zeros(Hdim), max_iter=niter - 1,
                  min_iter=(niter - 1 if min_iter is None else min_iter), accuracy_threshold=thr, verbose=None)
        est, conv, diag = pds.iterate()
        res = {'y': y, 'x': est['primal_variable'], 'z': est['dual_variable'], 'tau': pds.tau,
               'sigma': pds.sigma, 'rho': pds.rho, 'beta': pds.beta, 'n_iter': pds.iter,
               'converged': conv, 'diag_primal': diag['Relative Improvement (primal variable)'].to_numpy(float),
               'diag_dual': diag['Relative Improvement (dual variable)'].to_numpy(float),
               'diag_iter': diag['Iter'].to_numpy(float)}
        return res

    cases = {
        'denoise2d_l21_fwd_64': dict(shape=(64, 64), psf=None, lam=0.1, kind='forward', hname='l21', niter=30),
        'denoise2d_l1_fwd_63x65': dict(shape=(63, 65), psf=None, lam=0.1, kind='forward', hname='l1', niter=30),
        'denoise2d_l21_cen_48': dict(shape=(48, 48), psf=None, lam=0.1, kind='centered', hname='l21', niter=20),
        'denoise2d_l1_bwd_40x33': dict(shape=(40, 33), psf=None, lam=0.1, kind='backward', hname='l1', niter=20),
        'deconv2d_l21_fwd_64_psf15': dict(shape=(64, 64), psf=gaussian_psf(15, 2.0), lam=0.05, kind='forward',
                                          hname='l21', niter=30),
        'deconv2d_l1_fwd_57x70_psf7x4': dict(shape=(57, 70), psf=np.random.default_rng(3).uniform(0, 1, (7, 4)) / 14,
                                             lam=0.05, kind='forward', hname='l1', niter=20, gname='nonneg'),
        'deconv2d_l21_fwd_64_seg': dict(shape=(64, 64), psf=gaussian_psf(9, 1.5), lam=0.05, kind='forward',
                                        hname='l21', niter=20, gname='segment'),
        'lap2d_l1_50': dict(shape=(50, 50), psf=None, lam=0.05, kind='lap', hname='l1', niter=20),
        'deconv3d_l21_fwd_24_sep15': dict(shape=(24, 20, 22), psf=None, conv1d=gaussian_taps(15, 2.0), lam=0.05,
                                          kind='forward', hname='l21', niter=20),
        'denoise3d_l1_fwd_16': dict(shape=(16, 17, 18), psf=None, lam=0.1, kind='forward', hname='l1', niter=15),
        # 3-D with the reference's default centred Gradient and the backward kind (k_pds3d_gen)
        'denoise3d_l21_cen_16': dict(shape=(16, 17, 20), psf=None, lam=0.1, kind='centered', hname='l21', niter=15),
        'deconv3d_l1_bwd_20_sep7': dict(shape=(20, 18, 24), psf=None, conv1d=gaussian_taps(7, 1.2), lam=0.05,
                                        kind='backward', hname='l1', niter=15),
        'deconv3d_l21_cen_24_sep15': dict(shape=(24, 20, 24), psf=None, conv1d=gaussian_taps(15, 2.0), lam=0.05,
                                          kind='centered', hname='l21', niter=15),
        # natural termination (accuracy_threshold=1e-3, min_iter=10): pins the iteration-count semantics
        'denoise2d_l21_fwd_32_stop': dict(shape=(32, 32), psf=None, lam=0.1, kind='forward', hname='l21',
                                          niter=500, thr=1e-3, min_iter=10),
    }
    for name, kw in cases.items():
        if only and name not in only:
            continue
        res = run_pds(**kw)
        meta = dict(kw)
        psf = meta.pop('psf')
        c1 = meta.pop('conv1d', None)
        arrays = {k: np.asarray(v) for k, v in res.items()}
        arrays['shape'] = np.array(meta.pop('shape'))
        if psf is not None:
            arrays['psf'] = psf
        if c1 is not None:
            arrays['taps'] = c1
        for k, v in meta.items():
            arrays['meta_' + k] = np.array(v if v is not None else '')
        np.savez_compressed(os.path.join(HERE, f'pds_{name}.npz'), **arrays)
        print(name, 'iters', res['n_iter'], 'last rel', res['diag_primal'][-1])

    if only:
        return
    # ---------------- APGD LASSO (C1), CD and BT ----------------
    rng = np.random.default_rng(0)
    A = rng.standard_normal((256, 512))
    xs = np.zeros(512)
    idx = rng.choice(512, 20, replace=False)
    xs[idx] = rng.choice([-1.0, 1.0], 20)
    y = A @ xs
    lasso = {'A': A, 'y': y}
    for acc in ['CD', 'BT', None]:
        Gop = R.lbase.DenseLinearOperator(A)
        Gop.lipschitz_cst = Gop.diff_lipschitz_cst = float(np.linalg.norm(A, 2))
        F = (1 / 2) * loss.SquaredL2Loss(dim=256, data=y) * Gop
        lam = 0.1 * np.max(np.abs(F.gradient(0 * xs)))
        Gf = lam * pen.L1Norm(dim=512)
        lasso['lam'], lasso['Glip'] = lam, Gop.lipschitz_cst
        for niter, thr, mi in [(50, 0.0, 49), (500, 1e-3, 10)]:
            apgd = APGD(dim=512, F=F, G=Gf, acceleration=acc, max_iter=niter - 1, min_iter=mi,
                        accuracy_threshold=thr, verbose=None)
            est, conv, diag = apgd.iterate()
            tag = f"{acc or 'none'}_{'fixed' if thr == 0 else 'stop'}"
            for k, val in dict(tau=apgd.tau, beta=apgd.beta, x=est['iterand'], past_aux=est['past_aux'],
                               past_t=float(est['past_t']), n_iter=apgd.iter,
                               diag=diag['Relative Improvement'].to_numpy(float), max_iter=niter - 1,
                               min_iter=mi, thr=thr).items():
                lasso[f'{tag}_{k}'] = np.asarray(val)
            print('apgd', tag, 'iters', apgd.iter)
    np.savez_compressed(os.path.join(HERE, 'apgd_lasso.npz'), **lasso)


if __name__ == '__main__':
    main()

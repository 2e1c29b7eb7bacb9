"""Shared loaders for the golden PDS/APGD cases (used by CPU and GPU tests)."""

import glob
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def load(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


def pds_case_names():
    return sorted(os.path.basename(p)[4:-4] for p in glob.glob(os.path.join(GOLDEN, 'pds_*.npz')))


def pds_case(name):
    c = load(f'pds_{name}.npz')
    meta = {k[5:]: c[k].item() for k in list(c) if k.startswith('meta_')}
    c['meta'] = meta
    c['shape'] = tuple(int(s) for s in c['shape'])
    return c


def oracle_pds(c, callback=None, dtype=np.float64, conv_method=None):
    """Run the oracle restatement on a golden case (same construction as make_golden.run_pds).
    conv_method='fft': the separable-PSF cases' Convolve1D by the FFT path of the restatement (the
    same operator to ~1e-15, 20x faster: the long-horizon 3-D tests)."""
    from oracle import pylops1 as P
    from oracle import pycsou_ref as O
    shape = c['shape']
    meta = c['meta']
    N = int(np.prod(shape))
    d = len(shape)
    y = c['y'].astype(dtype)
    if 'psf' in c:
        off = tuple(P.pycsou_offset(n) for n in c['psf'].shape)
        C = P.Convolve2D(N, c['psf'].astype(dtype), shape, offset=off)
        conv, convT = C.matvec, C.rmatvec
    elif 'taps' in c:
        Cs = [P.Convolve1D(N, c['taps'].astype(dtype), offset=P.pycsou_offset(c['taps'].size), dims=shape, dir=a,
                           method=conv_method) for a in range(d)]

        def conv(v):
            for C in Cs:
                v = C.matvec(v)
            return v

        def convT(v):
            for C in reversed(Cs):
                v = C.rmatvec(v)
            return v
    else:
        conv = convT = None
    if meta['kind'] == 'lap':
        K = P.Laplacian(shape, weights=(1, 1), sampling=(1., 1.), edge=True, dtype=dtype)
        Hdim = N
    else:
        K = P.Gradient(shape, sampling=1., edge=True, kind=meta['kind'], dtype=dtype)
        Hdim = d * N
    if conv is None:
        grad_F = lambda x: (2 * (x + (-y))) * 0.5  # noqa: E731  (pycsou/core/map.py:609-610, penalty.py:131)
    else:
        grad_F = lambda x: convT((2 * (conv(x) + (-y))) * 0.5)  # noqa: E731
    lam = meta['lam']
    if meta['hname'] == 'l21':
        hprox = O.postcomp(lambda v, t: O.prox_l21_pixel(v, t, Hdim // N), lam)
    else:
        hprox = O.postcomp(O.prox_l1, lam)
    fen = lambda w, s: O.fenchel_prox(hprox, w, s)  # noqa: E731
    g = meta.get('gname', '')
    if g == 'nonneg':
        gprox = lambda v, t: O.proj_nonnegative_orthant(v)  # noqa: E731
    elif g == 'segment':
        gprox = lambda v, t: O.proj_segment(v, 0.0, 1.0)  # noqa: E731
    else:
        gprox = lambda v, t: v  # noqa: E731
    tau, sigma, rho = float(c['tau']), float(c['sigma']), float(c['rho'])
    niter = int(meta['niter'])
    thr = float(meta.get('thr', 0.0))
    mi = meta.get('min_iter', '')
    min_iter = niter - 1 if mi in ('', None) else int(mi)
    x, z, diag = O.pds(grad_F, gprox, K.matvec, K.rmatvec, fen, tau, sigma, rho, np.zeros(N, dtype),
                       np.zeros(Hdim, dtype), max_iter=niter - 1, min_iter=min_iter, accuracy_threshold=thr,
                       callback=callback)
    return x, z, diag


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)


def oracle_cps_inpaint(f, tag, dtype=np.float64):
    """Oracle run of the notebook cell [62] golden (CPS, K = [Masking; Gradient],
    H = L1Loss(y) (+) mu L1Norm, G = Segment(0, 1))."""
    from oracle import pylops1 as P
    from oracle import pycsou_ref as O
    shape = tuple(int(s) for s in f['shape'])
    mask, y, mu = f['mask'], f['y'].astype(dtype), float(f['mu'])
    n = int(np.prod(shape))
    m = int(mask.sum())
    D = P.Gradient(shape, sampling=1., edge=True, kind='forward', dtype=dtype)

    def K(x):
        return np.concatenate([x[mask], D.matvec(x)])

    def KT(z):
        xa = np.zeros(n, dtype=dtype)
        xa[mask] = z[:m]
        return 0 + xa + D.rmatvec(z[m:])  # LinOpStack.adjoint: result = 0; result += ...

    def hprox(v, t):  # ProxFuncHStack.prox: L1Loss = L1Norm shifted by -y (ProxFuncPreComp), mu*L1Norm
        return np.concatenate([O.prox_l1(v[:m] + (-y), t) - (-y), O.postcomp(O.prox_l1, mu)(v[m:], t)])

    p = tag + '_'
    return O.pds(lambda x: np.zeros_like(x), lambda v, t: O.proj_segment(v, 0.0, 1.0), K, KT,
                 lambda w, s: O.fenchel_prox(hprox, w, s), float(f[p + 'tau']), float(f[p + 'sigma']),
                 float(f[p + 'rho']), np.zeros(n, dtype=dtype), np.zeros(m + 2 * n, dtype=dtype),
                 max_iter=int(f[p + 'max_iter']), min_iter=int(f[p + 'min_iter']),
                 accuracy_threshold=float(f[p + 'thr']))

"""The row-marching fused steps against the fp64 oracle: pds_march.hpp (fp32, separable PSF of
half-width <= 7) and pds_pt.hpp (fp32 denoising, grad F = x - y, and non-separable PSFs through
the gradient buffer), n1 >= 128, n1 % 4 == 0, on shapes that exercise their edges: partial
last strip, several row segments with a short last one, both tap tiers (3, 7) and PSFs narrower
than their tier, L1 / L21, every prox_G kind, non-unit gradient steps.

Tolerance: relative L2 of x and z <= 5e-5 after 12 iterations (fp32 against fp64, as the golden
fp32 cases), diagnostics to 1e-3 relative, iteration counts exact.
"""

import numpy as np
import pytest

from oracle import pycsou_ref as OR
from tests.cases import rel

pytestmark = pytest.mark.gpu

NITER = 12


def _problem(shape, psf_len, hname, gname, steps, seed):
    rng = np.random.default_rng(seed)
    n0, n1 = shape
    N = n0 * n1
    xs = OR.phantom(shape, seed=seed)
    if np.isscalar(psf_len) and psf_len == 0:  # denoising: no operator in F
        psf = None
    elif np.isscalar(psf_len) and psf_len < 0:  # non-separable (rank 2) -|psf_len| x -|psf_len| PSF: gradient-buffer path
        q = -psf_len
        psf = rng.uniform(0.0, 1.0, (q, q))
        psf /= psf.sum()
    else:  # separable: one length for both axes, or (l0, l1) (even lengths: the reference's K//2 - 1 offset)
        l0, l1 = (psf_len, psf_len) if np.isscalar(psf_len) else psf_len
        r0, r1 = np.arange(l0) - l0 // 2, np.arange(l1) - l1 // 2
        t0 = np.exp(-0.5 * (r0 / 1.7) ** 2)
        t1 = np.exp(-0.5 * (r1 / 2.3) ** 2)
        psf = np.outer(t0 / t0.sum(), t1 / t1.sum())
    return dict(shape=shape, N=N, psf=psf, y=xs.ravel() + 0.05 * rng.standard_normal(N), hname=hname, gname=gname,
                steps=steps, lam=0.05)


def _oracle(p):
    from oracle import pylops1 as P
    shape, N, psf, y = p['shape'], p['N'], p['psf'], p['y']
    if psf is None:
        grad = lambda v: (2 * (v + (-y))) * 0.5  # noqa: E731
    else:
        off = tuple(P.pycsou_offset(n) for n in psf.shape)
        C = P.Convolve2D(N, psf, shape, offset=off)
        grad = lambda v: C.rmatvec((2 * (C.matvec(v) + (-y))) * 0.5)  # noqa: E731
    K = P.Gradient(shape, sampling=p['steps'], edge=True, kind='forward')
    if p['hname'] == 'l21':
        hprox = OR.postcomp(lambda v, t: OR.prox_l21_pixel(v, t, 2), p['lam'])
    else:
        hprox = OR.postcomp(OR.prox_l1, p['lam'])
    gprox = {'nonneg': lambda v, t: OR.proj_nonnegative_orthant(v),
             'segment': lambda v, t: OR.proj_segment(v, 0.0, 1.0)}.get(p['gname'], lambda v, t: v)
    beta = 1.0
    lip = np.sqrt(sum(4.0 / s ** 2 for s in p['steps']))
    tau, sigma = OR.pds_step_sizes(beta, lip)[:2]
    x, z, d = OR.pds(grad, gprox, K.matvec, K.rmatvec,
                     lambda w, s: OR.fenchel_prox(hprox, w, s), tau, sigma, 0.9, np.zeros(N), np.zeros(2 * N),
                     max_iter=NITER - 1, min_iter=NITER - 1, accuracy_threshold=0.0)
    return x, z, d, lip


def _fused(p, lip):
    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L1Norm, L21Norm, NonNegativeOrthant, Segment
    from pycsou_amd.linop.conv import Convolve2D
    from pycsou_amd.linop.diff import Gradient
    from pycsou_amd.opt.proxalgs import PDS
    shape, N = p['shape'], p['N']
    F = (1 / 2) * SquaredL2Loss(dim=N, data=p['y'].astype(np.float32))
    if p['psf'] is not None:
        C = Convolve2D(N, p['psf'], shape)
        C.lipschitz_cst = C.diff_lipschitz_cst = 1.0
        F = F * C
    K = Gradient(shape, step=p['steps'], kind='forward')
    K.lipschitz_cst = K.diff_lipschitz_cst = lip
    H = p['lam'] * (L21Norm(dim=2 * N, groups=np.tile(np.arange(N), 2)) if p['hname'] == 'l21' else L1Norm(dim=2 * N))
    G = {'nonneg': NonNegativeOrthant(N), 'segment': Segment(N, 0.0, 1.0)}.get(p['gname'], None)
    pds = PDS(dim=N, F=F, G=G, H=H, K=K,
              x0=np.zeros(N, np.float32), z0=np.zeros(2 * N, np.float32), max_iter=NITER - 1, min_iter=NITER - 1,
              accuracy_threshold=0.0, verbose=None, engine='fused')
    est, _, diag = pds.iterate()
    assert pds._engine is not None and pds.iter == NITER
    return est['primal_variable'], est['dual_variable'], diag


CASES = [
    # shape, psf length, H, G, steps
    ((300, 200), 15, 'l21', '', (1.0, 1.0)),       # tier 7, partial last strip (200 = 3*64 + 8)
    ((300, 200), 7, 'l1', 'nonneg', (1.0, 1.0)),   # tier 3, L1
    ((261, 132), 11, 'l21', 'segment', (1.0, 1.0)),  # psf half 5 in tier 7, 4-column last strip
    ((190, 256), 5, 'l1', '', (2.0, 0.5)),          # psf half 2 in tier 3, non-unit steps
    ((1000, 128), 15, 'l1', 'segment', (0.5, 1.0)),  # tall: many row segments, short last one
    ((1000, 4096), 15, 'l21', 'nonneg', (1.0, 1.0)),  # C3 width: 6-step tasks, 3-step last segment
    ((300, 200), (4, 6), 'l21', '', (1.0, 1.0)),       # even lengths (offset K//2 - 1), tier 3, 4x6
    ((261, 260), (14, 14), 'l1', 'nonneg', (1.0, 1.0)),  # even 14x14, tier 7 (N-table edge rows)
    # pds_pt.hpp
    ((300, 200), 0, 'l21', '', (1.0, 1.0)),            # denoising, partial last strip
    ((1030, 2048), 0, 'l1', 'segment', (2.0, 0.5)),    # denoising, C2 width, short last segment
    ((261, 132), -5, 'l21', 'nonneg', (1.0, 1.0)),     # non-separable 5x5 PSF (gradient buffer)
    # non-separable PSFs through the packed-plan correlation kernel (corr2d.hip) + GRADBUF update
    ((1000, 4096), -15, 'l21', 'nonneg', (1.0, 1.0)),  # C3 width, 15x15, several strip segments
    ((517, 1000), -9, 'l1', '', (2.0, 0.5)),           # 9x9 (tier 9), ragged rows, non-unit steps
]


@pytest.mark.parametrize('case', range(len(CASES)))
def test_march_vs_oracle(case):
    shape, L, hname, gname, steps = CASES[case]
    p = _problem(shape, L, hname, gname, steps, seed=case)
    xr, zr, dr, lip = _oracle(p)
    x, z, diag = _fused(p, lip)
    assert x.dtype == np.float32
    assert rel(x, xr) < 5e-5, rel(x, xr)
    assert rel(z, zr) < 5e-5, rel(z, zr)
    np.testing.assert_allclose(diag['Relative Improvement (primal variable)'].to_numpy(float), dr['primal'],
                               rtol=1e-3)
    np.testing.assert_allclose(diag['Relative Improvement (dual variable)'].to_numpy(float), dr['dual'], rtol=1e-3)


def test_march_is_the_kernel_in_use():
    """The shapes above take the march kernel: one block per (64-column strip, row segment of
    16-row steps) -- 4 x 19 for 300 x 200 (the tile kernel would launch 4 x 10 tiles of 31 rows)."""
    import ctypes

    from pycsou_amd import _lib as L
    a = L.PdsArgs()
    a.dtype, a.fkind, a.hkind, a.gkind = L.PCS_F32, L.PCS_F_SEPCONV, L.PCS_H_L21, L.PCS_G_NULL
    a.n0, a.n1, a.row0, a.rows = 300, 200, 0, 300
    a.half, a.halo_x, a.halo_y, a.halo_z = 7, 0, 0, 0
    a.step0 = a.step1 = 1.0
    nb = L.load().pcs_pds2d_nblocks(ctypes.byref(a))
    assert nb == 4 * 19


def test_c2_full_size_fused_vs_generic():
    """C2 exactly (BASELINE configs[1]): 2048^2 fp32 isotropic-TV denoising, 0.1 * L21Norm,
    Gradient(kind='forward'), 12 iterations -- the fused row-marching engine against the
    per-operator generic path (separate Gradient / L21 / axpby kernels, device loop control):
    same iteration count, x and z to 1e-5 relative (fp32 rounding of two different op
    orders), diagnostics to 1e-3 relative."""
    import torch

    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L21Norm
    from pycsou_amd.linop.diff import Gradient
    from pycsou_amd.opt.proxalgs import PDS
    n = 2048
    N = n * n
    y = torch.as_tensor((OR.phantom((n, n), seed=3) + 0.1 * np.random.default_rng(3).standard_normal((n, n)))
                        .astype(np.float32).ravel()).cuda()
    out = {}
    for mode in ('fused', 'generic'):
        K = Gradient((n, n), kind='forward')
        K.lipschitz_cst = K.diff_lipschitz_cst = float(np.sqrt(8 * np.sin(np.pi * (n - 1) / (2 * n)) ** 2))
        pds = PDS(dim=N, F=(1 / 2) * SquaredL2Loss(dim=N, data=y), H=0.1 * L21Norm(dim=2 * N,
                  groups=np.tile(np.arange(N), 2)), K=K, x0=torch.zeros(N, device='cuda'),
                  z0=torch.zeros(2 * N, device='cuda'), max_iter=NITER - 1, min_iter=NITER - 1,
                  accuracy_threshold=0.0, verbose=None, engine=mode)
        est, _, diag = pds.iterate()
        assert (pds._engine is not None) == (mode == 'fused') and pds.iter == NITER
        out[mode] = (est['primal_variable'].cpu().numpy(), est['dual_variable'].cpu().numpy(), diag)
    (xf, zf, df), (xg, zg, dg) = out['fused'], out['generic']
    assert rel(xf, xg) < 1e-5 and rel(zf, zg) < 1e-5
    for col in ('Relative Improvement (primal variable)', 'Relative Improvement (dual variable)'):
        np.testing.assert_allclose(df[col].to_numpy(float)[1:], dg[col].to_numpy(float)[1:], rtol=1e-3)


SEP_CASES = [i for i, c in enumerate(CASES) if not np.isscalar(c[1]) or c[1] > 0]


@pytest.mark.parametrize('case', SEP_CASES)
def test_fourpass_march_vs_oracle(case, monkeypatch):
    """The separable cases again with PCS_NMARCH=0: grad F = Conv^T (Conv x - y) as four
    15-tap passes (pds_march.hpp) instead of N x - Conv^T y (pds_nmarch.hpp, the default
    above) -- both kernels stay parity-green against the oracle."""
    monkeypatch.setenv('PCS_NMARCH', '0')
    shape, L, hname, gname, steps = CASES[case]
    p = _problem(shape, L, hname, gname, steps, seed=case)
    xr, zr, dr, lip = _oracle(p)
    x, z, diag = _fused(p, lip)
    assert rel(x, xr) < 5e-5, rel(x, xr)
    assert rel(z, zr) < 5e-5, rel(z, zr)


def test_c3_full_size_normal_vs_fourpass(monkeypatch):
    """C3 exactly (BASELINE north_star: 4096^2 fp32, 15x15 Gaussian PSF, K = forward
    Gradient, 0.05 * L21Norm), 12 iterations, through the normal-operator kernel (the bench's)
    and the four-pass kernel: the two gradient factorisations agree to fp32 rounding (x and z
    to 1e-5 relative), the same iteration count, diagnostics to 1e-3."""
    import torch

    import bench
    out = {}
    for nm in ('1', '0'):
        monkeypatch.setenv('PCS_NMARCH', nm)
        pds = bench.build_problem(4096, 4096, torch.float32, lipschitz='analytic')
        pds.max_iter = pds.min_iter = NITER - 1
        pds.accuracy_threshold = 0.0
        est, _, diag = pds.iterate()
        eng = pds._engine
        assert eng is not None and pds.iter == NITER
        assert (eng.args.cty is not None and eng.args.cty != 0) == (nm == '1')
        out[nm] = (est['primal_variable'].cpu().numpy(), est['dual_variable'].cpu().numpy(), diag)
    (xn, zn, dn), (xf, zf, df) = out['1'], out['0']
    assert np.isfinite(xn).all() and np.abs(xn).max() > 0
    assert rel(xn, xf) < 1e-5, rel(xn, xf)
    assert rel(zn, zf) < 1e-5, rel(zn, zf)
    for col in ('Relative Improvement (primal variable)', 'Relative Improvement (dual variable)'):
        np.testing.assert_allclose(dn[col].to_numpy(float)[1:], df[col].to_numpy(float)[1:], rtol=1e-3)

"""Full-size parity against the oracle (not only HIP path against HIP path): the bench legs' own
problems at BASELINE sizes -- C3 4096^2 (separable 15x15 Gaussian: the headline fused kernel, the
reference's default centred K, fp64 through the fused fp64 march; the non-separable PSF) and the C2
2048^2 denoising family -- run 3 iterations through the public API and are checked against the fp64
oracle restatement of pycsou/core/solver.py:55-76 + opt/proxalgs.py:343-394 on the same y, tau, sigma,
rho (SciPy FFT convolutions on the oracle side: the same operator to ~1e-15).

Bars (the suite's): fp32 x and z to 5e-5 relative L2, fp64 to 1e-10; the two diagnostics columns to
1e-3 (fp32) / 1e-8 (fp64) relative.  The 512^3 / 1024^3 volumes stay at 48^3-128^3 for the oracle
(tests/test_gpu_long2.py, test_gpu_pds.py): the oracle's FFT convolution alone takes ~40 s per gradient
at 512^3.
"""

import numpy as np
import pytest
import torch

from tests.cases import oracle_pds, rel

pytestmark = pytest.mark.gpu

NITER = 3


def _c3(dtype, kind='forward', psf=None):
    import bench
    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L21Norm
    from pycsou_amd.linop.conv import Convolve2D
    from pycsou_amd.linop.diff import Gradient
    from pycsou_amd.opt.proxalgs import PDS
    n = 4096
    N = n * n
    h = bench.gaussian_psf(15, 2.0) if psf is None else psf
    xs = torch.as_tensor(bench.phantom((n, n), 64, 0).ravel()).to('cuda', dtype)
    C = Convolve2D(size=N, filter=h, shape=(n, n))
    K = Gradient(shape=(n, n), kind=kind)
    C.compute_lipschitz_cst()
    K.compute_lipschitz_cst()
    g = torch.Generator(device='cuda').manual_seed(1)
    y = C(xs) + 0.01 * torch.randn(N, generator=g, device='cuda', dtype=dtype)
    pds = PDS(dim=N, F=(1 / 2) * SquaredL2Loss(dim=N, data=y) * C,
              H=0.05 * L21Norm(dim=2 * N, groups=np.tile(np.arange(N), 2)), K=K,
              x0=torch.zeros(N, dtype=dtype, device='cuda'), z0=torch.zeros(2 * N, dtype=dtype, device='cuda'),
              max_iter=NITER - 1, min_iter=NITER - 1, accuracy_threshold=0.0, verbose=None)
    case = {'shape': (n, n), 'y': y.double().cpu().numpy(),
            'meta': {'kind': kind, 'hname': 'l21', 'lam': 0.05, 'niter': NITER}}
    if psf is None:  # the separable Gaussian as its 1-D factor along both axes
        t = np.exp(-0.5 * ((np.arange(15) - 7) / 2.0) ** 2)
        case['taps'] = t / t.sum()
    else:
        case['psf'] = psf
    return pds, case


def _check(pds, case, dtype, conv_method='fft'):
    est, conv, diag = pds.iterate()
    assert pds.iter == NITER
    assert pds._engine is not None, 'the fused engine must take the full-size problem'
    case['tau'], case['sigma'], case['rho'] = pds.tau, pds.sigma, pds.rho
    xr, zr, dr = oracle_pds(case, conv_method=conv_method)
    x = est['primal_variable']
    z = est['dual_variable']
    x = x.double().cpu().numpy() if torch.is_tensor(x) else np.asarray(x, np.float64)
    z = z.double().cpu().numpy() if torch.is_tensor(z) else np.asarray(z, np.float64)
    tol = 1e-10 if dtype == torch.float64 else 5e-5
    assert rel(x, xr) < tol, rel(x, xr)
    assert rel(z, zr) < tol, rel(z, zr)
    dtol = 1e-8 if dtype == torch.float64 else 1e-3
    np.testing.assert_allclose(diag['Relative Improvement (primal variable)'].to_numpy(float)[1:],
                               np.asarray(dr['primal'])[1:], rtol=dtol)
    np.testing.assert_allclose(diag['Relative Improvement (dual variable)'].to_numpy(float)[1:],
                               np.asarray(dr['dual'])[1:], rtol=dtol)


@pytest.mark.parametrize('dtype,kind', [(torch.float32, 'forward'), (torch.float32, 'centered'),
                                        (torch.float64, 'forward'), (torch.float64, 'centered')])
def test_c3_fullsize_vs_oracle(dtype, kind):
    """C3 4096^2 (the headline problem; fp64: the reference's default dtype through k_pds2d_nmarch64)."""
    pds, case = _c3(dtype, kind)
    _check(pds, case, dtype)
    if dtype == torch.float64:
        assert pds._engine.nm_fused, 'fp64 C3 must take the fused fp64 normal-operator march'


def test_c3_nonsep_fullsize_vs_oracle():
    """C3 4096^2 with the bench's rank > 1 15x15 PSF (two k_corr2d passes + the GRADBUF update)."""
    import bench
    pds, case = _c3(torch.float32, psf=bench.aniso_psf())
    _check(pds, case, torch.float32)


@pytest.mark.parametrize('kind', ['forward', 'centered', 'lap'])
def test_c2_fullsize_vs_oracle(kind):
    """C2 2048^2 TV denoising (forward K: k_pds2d_pt; centred / Laplacian: k_pds2d_smarch)."""
    import bench
    n = 2048
    if kind == 'forward':
        pds = bench.build_denoise(n, torch.float32)
        meta = {'kind': 'forward', 'hname': 'l21', 'lam': 0.1}
    else:
        pds = bench.build_denoise_k(n, torch.float32, kind)
        meta = {'kind': kind, 'hname': 'l1' if kind == 'lap' else 'l21', 'lam': 0.1}
    pds.max_iter, pds.min_iter, pds.accuracy_threshold = NITER - 1, NITER - 1, 0.0
    from pycsou_amd.opt.engine import _half_loss_data
    s = _half_loss_data(pds.F)  # F = (1/2) ||x - y||^2 carries y as the shift -y
    assert s is not None
    y = -(s.double().cpu().numpy() if torch.is_tensor(s) else np.asarray(s, np.float64))
    case = {'shape': (n, n), 'y': y, 'meta': dict(meta, niter=NITER)}
    _check(pds, case, torch.float32)


def test_cps_fullsize_vs_oracle():
    """The cps_inpaint bench leg's problem at its size (2048^2, 50 % mask, K = [Masking; Gradient(forward)],
    H = L1Loss (+) 0.1 L1Norm, G = Segment(0, 1): the masked march, one launch per iteration) against the
    fp64 oracle's op sequence (pycsou/opt/proxalgs.py:628-716 through the PDS update of :343-394)."""
    import bench
    from oracle import pycsou_ref as O
    from oracle import pylops1 as P
    from pycsou_amd.func import L1Loss, L1Norm, ProxFuncHStack, Segment
    from pycsou_amd.linop import Gradient, LinOpVStack, Masking
    from pycsou_amd.opt import CPS
    from pycsou_amd.opt.engine import PDS2DMaskEngine
    n = 2048
    N = n * n
    mask = np.random.default_rng(5).random(N) < 0.5
    m = int(mask.sum())
    y = bench.phantom((n, n), 12, 5).ravel()[mask].astype(np.float32)
    Kop = LinOpVStack(Masking(size=N, sampling_bool=mask), Gradient(shape=(n, n), kind='forward'))
    Kop.lipschitz_cst = Kop.diff_lipschitz_cst = 3.0
    cps = CPS(dim=N, G=Segment(dim=N, a=0, b=1), H=ProxFuncHStack(L1Loss(dim=m, data=y), 0.1 * L1Norm(dim=2 * N)),
              K=Kop, x0=np.zeros(N, np.float32), z0=np.zeros(m + 2 * N, np.float32), max_iter=NITER - 1,
              min_iter=NITER - 1, accuracy_threshold=0.0, verbose=None)
    est, _, diag = cps.iterate()
    assert isinstance(cps._engine, PDS2DMaskEngine) and cps.iter == NITER
    D = P.Gradient((n, n), sampling=1., edge=True, kind='forward')
    yd = y.astype(np.float64)

    def Kf(x):
        return np.concatenate([x[mask], D.matvec(x)])

    def KT(z):
        xa = np.zeros(N)
        xa[mask] = z[:m]
        return 0 + xa + D.rmatvec(z[m:])

    hs = O.postcomp(O.prox_l1, 0.1)

    def hprox(v, t):
        return np.concatenate([O.prox_l1(v[:m] + (-yd), t) - (-yd), hs(v[m:], t)])

    xr, zr, dr = O.pds(lambda x: np.zeros_like(x), lambda v, t: O.proj_segment(v, 0.0, 1.0), Kf, KT,
                       lambda w, s: O.fenchel_prox(hprox, w, s), cps.tau, cps.sigma, cps.rho, np.zeros(N),
                       np.zeros(m + 2 * N), max_iter=NITER - 1, min_iter=NITER - 1, accuracy_threshold=0.0)
    x = np.asarray(est['primal_variable'], np.float64)
    z = np.asarray(est['dual_variable'], np.float64)
    assert rel(x, xr) < 5e-5, rel(x, xr)
    assert rel(z, zr) < 5e-5, rel(z, zr)
    np.testing.assert_allclose(diag['Relative Improvement (primal variable)'].to_numpy(float)[1:],
                               np.asarray(dr['primal'])[1:], rtol=1e-3)
    np.testing.assert_allclose(diag['Relative Improvement (dual variable)'].to_numpy(float)[1:],
                               np.asarray(dr['dual'])[1:], rtol=1e-3)


@pytest.mark.parametrize('kind', ['forward', 'centered'])
def test_c5_fullsize_fused_vs_generic(kind):
    """C5 at its real size (BASELINE configs[4]: 1024^3 fp64, 15-tap Gaussian along every axis, 0.05 L21; the
    reference's default centred K and the forward K): the fused 3-D engine (k_sep2d_nrmm + k_conv0_rta +
    k_pds3d / k_pds3d_gen) against the operator-by-operator path for 3 iterations -- the only run of the
    > 2^31-element indexing (z holds 3 * 1024^3 = 3.2e9 elements) outside the bench.  The oracle cannot run
    at this size (its FFT convolution alone takes minutes per gradient); the generic path is the HIP
    operators one call at a time, checked against the oracle at 48^3-128^3 elsewhere.  Bars: 1e-12 relative
    on x and z (the two paths round the normal operator differently), finite, exact count, diagnostics 1e-9."""
    import bench
    from pycsou_amd.opt.engine3d import PDS3DEngine
    n = 1024
    out = []
    for eng in ('fused', 'generic'):
        pds = bench.build_volume(n, torch.float64, kind=kind)
        pds.max_iter, pds.min_iter, pds.accuracy_threshold = NITER - 1, NITER - 1, 0.0
        pds.engine_mode = eng
        est, _, diag = pds.iterate()
        assert pds.iter == NITER
        if eng == 'fused':
            assert isinstance(pds._engine, PDS3DEngine)
        else:
            assert pds._engine is None
        out.append((est['primal_variable'], est['dual_variable'],
                    diag['Relative Improvement (primal variable)'].to_numpy(float),
                    diag['Relative Improvement (dual variable)'].to_numpy(float)))
        del pds, est
        torch.cuda.empty_cache()
    assert out[0][1].numel() == 3 * n ** 3
    for k in range(2):
        assert torch.isfinite(out[0][k]).all()
        d = float(torch.linalg.vector_norm(out[0][k] - out[1][k]) / torch.linalg.vector_norm(out[1][k]))
        assert d < 1e-12, (k, d)
    for k in (2, 3):
        np.testing.assert_allclose(out[0][k][1:], out[1][k][1:], rtol=1e-9)

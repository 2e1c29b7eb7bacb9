"""Solver parity on the GPU: PDS (fused hipGraph engine and generic operator path) and
APGD against the golden trajectories of the real reference (tests/golden/).

Tolerances (relative L2 over the whole iterate): fp64 <= 1e-9 after 15-30 iterations
(direct vs FFT convolution and FMA rounding, amplified mildly by the iteration); fp32 <=
5e-5 (fp32 arithmetic against the fp64 reference).  Iteration counts must be identical
(the stopping rule runs on the device for the fused engine).
"""

import numpy as np
import pytest
import torch

from oracle import pycsou_ref as OR
from tests.cases import load, oracle_pds, pds_case, pds_case_names, rel

pytestmark = pytest.mark.gpu

FUSED_2D = [n for n in pds_case_names() if '3d' not in n and 'lap' not in n and '_cen_' not in n
            and '_bwd_' not in n]


def build(c, dtype=np.float64, engine='auto', torch_io=False):
    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L1Norm, L21Norm, NonNegativeOrthant, Segment
    from pycsou_amd.linop.conv import Convolve1D, Convolve2D
    from pycsou_amd.linop.diff import Gradient, Laplacian
    from pycsou_amd.opt.proxalgs import PDS
    shape, meta = c['shape'], c['meta']
    N, d = int(np.prod(shape)), len(shape)
    y = c['y'].astype(dtype)
    if torch_io:
        y = torch.as_tensor(y).cuda()
    F = (1 / 2) * SquaredL2Loss(dim=N, data=y)
    if 'psf' in c:
        C = Convolve2D(N, c['psf'], shape)
        C.lipschitz_cst = C.diff_lipschitz_cst = 1.0
        F = F * C
    elif 'taps' in c:
        C = None
        for ax in range(d):
            Ci = Convolve1D(N, c['taps'], reshape_dims=shape, axis=ax)
            Ci.lipschitz_cst = Ci.diff_lipschitz_cst = 1.0
            C = Ci if C is None else Ci * C
        C.lipschitz_cst = C.diff_lipschitz_cst = 1.0
        F = F * C
    if meta['kind'] == 'lap':
        K = Laplacian(shape, weights=(1, 1), step=1., edge=True)
        K.lipschitz_cst = K.diff_lipschitz_cst = 8.0
        Hdim = N
    else:
        K = Gradient(shape, step=1., edge=True, kind=meta['kind'])
        K.lipschitz_cst = K.diff_lipschitz_cst = np.sqrt(4.0 * d)
        Hdim = d * N
    lam = meta['lam']
    H = lam * (L21Norm(dim=Hdim, groups=np.tile(np.arange(N), Hdim // N)) if meta['hname'] == 'l21'
               else L1Norm(dim=Hdim))
    G = {'nonneg': NonNegativeOrthant(N), 'segment': Segment(N, 0.0, 1.0)}.get(meta.get('gname', ''), None)
    niter = int(meta['niter'])
    mi = meta.get('min_iter', '')
    x0, z0 = np.zeros(N, dtype), np.zeros(Hdim, dtype)
    if torch_io:
        x0, z0 = torch.as_tensor(x0).cuda(), torch.as_tensor(z0).cuda()
    return PDS(dim=N, F=F, G=G, H=H, K=K, x0=x0, z0=z0, max_iter=niter - 1,
               min_iter=niter - 1 if mi in ('', None) else int(mi), accuracy_threshold=float(meta.get('thr', 0.0)),
               verbose=None, engine=engine)


def _check(pds, c, dtype):
    est, conv, diag = pds.iterate()
    assert conv is True
    assert pds.iter == int(c['n_iter'])
    tol = 1e-9 if dtype == np.float64 else 5e-5
    x, z = est['primal_variable'], est['dual_variable']
    if isinstance(x, torch.Tensor):
        x, z = x.cpu().numpy(), z.cpu().numpy()
    assert x.dtype == dtype
    assert rel(x, c['x']) < tol, rel(x, c['x'])
    assert rel(z, c['z']) < tol, rel(z, c['z'])
    # fp32: 1e-3 relative, plus 1e-5 absolute for the late rows whose improvements (differences of
    # iterates that agree to 5e-5) approach the fp32 rounding of the iterates themselves
    dtol, atol = (1e-6, 0.0) if dtype == np.float64 else (1e-3, 1e-5)
    np.testing.assert_allclose(diag['Relative Improvement (primal variable)'].to_numpy(float), c['diag_primal'],
                               rtol=dtol, atol=atol)
    np.testing.assert_allclose(diag['Relative Improvement (dual variable)'].to_numpy(float), c['diag_dual'],
                               rtol=dtol, atol=atol)
    np.testing.assert_array_equal(diag['Iter'].to_numpy(), np.arange(pds.iter))


@pytest.mark.parametrize('name', FUSED_2D)
@pytest.mark.parametrize('dtype', [np.float64, np.float32])
def test_pds_fused_matches_reference(name, dtype):
    c = pds_case(name)
    pds = build(c, dtype, engine='fused')
    _check(pds, c, dtype)
    assert pds._engine is not None


@pytest.mark.parametrize('name', pds_case_names())
def test_pds_generic_matches_reference(name):
    c = pds_case(name)
    pds = build(c, np.float64, engine='generic')
    _check(pds, c, np.float64)
    assert pds._engine is None


def test_pds_torch_io_stays_on_device():
    c = pds_case('deconv2d_l21_fwd_64_psf15')
    pds = build(c, np.float32, torch_io=True)
    est, _, _ = pds.iterate()
    assert isinstance(est['primal_variable'], torch.Tensor) and est['primal_variable'].is_cuda
    assert rel(est['primal_variable'].cpu().numpy(), c['x']) < 5e-5


def test_pds_fused_vs_generic_nonseparable_psf():
    """A non-separable PSF takes the GRADBUF engine mode (pcs_conv2d + fused step)."""
    c = pds_case('deconv2d_l1_fwd_57x70_psf7x4')
    a = build(c, np.float64, engine='fused')
    ea, _, _ = a.iterate()
    assert a._engine.fkind == 3
    assert rel(ea['primal_variable'], c['x']) < 1e-9


@pytest.mark.parametrize('acc', ['CD', 'BT', 'none'])
@pytest.mark.parametrize('mode', ['fixed', 'stop'])
def test_apgd_lasso_matches_reference(acc, mode):
    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L1Norm
    from pycsou_amd.linop.base import DenseLinearOperator
    from pycsou_amd.opt.proxalgs import APGD
    f = load('apgd_lasso.npz')
    p = f'{acc}_{mode}_'
    Gop = DenseLinearOperator(f['A'])
    Gop.lipschitz_cst = Gop.diff_lipschitz_cst = float(f['Glip'])
    F = (1 / 2) * SquaredL2Loss(dim=256, data=f['y']) * Gop
    lam = 0.1 * np.max(np.abs(F.gradient(np.zeros(512))))
    assert abs(lam - float(f['lam'])) < 1e-12 * lam
    apgd = APGD(dim=512, F=F, G=lam * L1Norm(dim=512), acceleration=None if acc == 'none' else acc,
                max_iter=int(f[p + 'max_iter']), min_iter=int(f[p + 'min_iter']), accuracy_threshold=float(f[p + 'thr']),
                verbose=None)
    assert apgd.tau == float(f[p + 'tau'])
    est, conv, diag = apgd.iterate()
    assert apgd.iter == int(f[p + 'n_iter'])
    assert rel(est['iterand'], f[p + 'x']) < 1e-9
    assert rel(est['past_aux'], f[p + 'past_aux']) < 1e-9
    np.testing.assert_allclose(diag['Relative Improvement'].to_numpy(float), f[p + 'diag'], rtol=1e-6)


@pytest.mark.parametrize('dtype', [np.float32, np.float64])
def test_pds_fused_4096_properties(dtype):
    """Full C3 size (4096^2, 15x15 Gaussian PSF): parity of the fused engine with the
    oracle on a 512^2 crop is covered above; at full size check size-independent
    properties: fused == generic path to rounding after 3 iterations, monotone decrease
    of the relative improvement is not required, but finiteness and the exact count are."""
    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L21Norm
    from pycsou_amd.linop.conv import Convolve2D
    from pycsou_amd.linop.diff import Gradient
    from pycsou_amd.opt.proxalgs import PDS
    n = 4096 if dtype == np.float32 else 2048
    N = n * n
    xs = OR.phantom((n, n), n_rect=64, seed=0, dtype=dtype)
    h = OR.gaussian_psf(15, 2.0)
    C = Convolve2D(N, h, (n, n))
    C.lipschitz_cst = C.diff_lipschitz_cst = 1.0
    y = torch.as_tensor(xs.ravel()).cuda()
    y = C(y) + 0.01 * torch.randn(N, generator=torch.Generator('cuda').manual_seed(1), device='cuda', dtype=y.dtype)
    K = Gradient((n, n), kind='forward')
    K.lipschitz_cst = K.diff_lipschitz_cst = np.sqrt(8.0)
    H = 0.05 * L21Norm(dim=2 * N, groups=np.tile(np.arange(N), 2))
    F = (1 / 2) * SquaredL2Loss(dim=N, data=y) * C
    out = []
    for eng in ['fused', 'generic']:
        pds = PDS(dim=N, F=F, H=H, K=K, x0=torch.zeros(N, dtype=y.dtype, device='cuda'),
                  z0=torch.zeros(2 * N, dtype=y.dtype, device='cuda'), max_iter=2, min_iter=2,
                  accuracy_threshold=0.0, verbose=None, engine=eng)
        est, _, diag = pds.iterate()
        assert pds.iter == 3
        out.append((est['primal_variable'], est['dual_variable'], diag))
    # fused = separable 15+15-tap passes, generic = direct 225-tap conv: fp32 summation-order rounding
    tol = 1e-12 if dtype == np.float64 else 3e-5
    assert float(torch.linalg.vector_norm(out[0][0] - out[1][0]) / torch.linalg.vector_norm(out[1][0])) < tol
    assert float(torch.linalg.vector_norm(out[0][1] - out[1][1]) / torch.linalg.vector_norm(out[1][1])) < tol
    assert torch.isfinite(out[0][0]).all()


def test_pds_fused_crop_vs_oracle_fp32_512():
    """fp32 fused engine vs the fp64 oracle on a 512^2 TV-deconvolution, 20 iterations."""
    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L21Norm
    from pycsou_amd.linop.conv import Convolve2D
    from pycsou_amd.linop.diff import Gradient
    from pycsou_amd.opt.proxalgs import PDS
    from oracle import pylops1 as P
    n, N = 512, 512 * 512
    xs = OR.phantom((n, n), seed=3)
    h = OR.gaussian_psf(15, 2.0)
    Cr = P.Convolve2D(N, h, (n, n), offset=(7, 7))
    y = Cr.matvec(xs.ravel()) + 0.01 * np.random.default_rng(0).standard_normal(N)
    tau = sigma = OR.pds_step_sizes(1.0, np.sqrt(8.0))[0]
    Kr = P.Gradient((n, n), edge=True, kind='forward')
    hprox = OR.postcomp(lambda v, t: OR.prox_l21_pixel(v, t, 2), 0.05)
    xr, zr, dr = OR.pds(lambda x: Cr.rmatvec((2 * (Cr.matvec(x) + (-y))) * 0.5), lambda v, t: v, Kr.matvec,
                        Kr.rmatvec, lambda w, s: OR.fenchel_prox(hprox, w, s), tau, sigma, 0.9, np.zeros(N),
                        np.zeros(2 * N), max_iter=19, min_iter=19, accuracy_threshold=0.0)
    C = Convolve2D(N, h, (n, n))
    C.lipschitz_cst = C.diff_lipschitz_cst = 1.0
    K = Gradient((n, n), kind='forward')
    K.lipschitz_cst = K.diff_lipschitz_cst = np.sqrt(8.0)
    pds = PDS(dim=N, F=(1 / 2) * SquaredL2Loss(dim=N, data=y.astype(np.float32)) * C,
              H=0.05 * L21Norm(dim=2 * N, groups=np.tile(np.arange(N), 2)), K=K, x0=np.zeros(N, np.float32),
              z0=np.zeros(2 * N, np.float32), max_iter=19, min_iter=19, accuracy_threshold=0.0, verbose=None)
    est, _, diag = pds.iterate()
    assert pds._engine is not None and pds.iter == 20
    assert rel(est['primal_variable'], xr) < 5e-5
    assert rel(est['dual_variable'], zr) < 5e-5


@pytest.mark.parametrize('kind', ['centered', 'forward'])
def test_pds_4d_gradient_generic_vs_oracle(kind):
    """TV denoising of a 4-D array (volume x time) through the generic device path: a 4-axis
    Gradient (one derivative launch per axis) with L21 over the 4 components, 30 iterations,
    fp64 against the oracle (PyLops 1.x Gradient takes any ndim)."""
    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L21Norm
    from pycsou_amd.linop.diff import Gradient
    from pycsou_amd.opt.proxalgs import PDS
    from oracle import pylops1 as P
    shape = (6, 7, 8, 9)
    N = int(np.prod(shape))
    rng = np.random.default_rng(11)
    y = np.repeat(rng.standard_normal((6, 7, 1, 1)), 72, axis=2).reshape(-1) + 0.1 * rng.standard_normal(N)
    steps = [1.0, 0.5, 1.5, 2.0]
    lip = np.sqrt(sum(4.0 / s ** 2 for s in steps))
    tau, sigma = OR.pds_step_sizes(1.0, lip)[:2]
    Kr = P.Gradient(shape, sampling=steps, edge=True, kind=kind)
    hprox = OR.postcomp(lambda v, t: OR.prox_l21_pixel(v, t, 4), 0.1)
    xr, zr, _ = OR.pds(lambda x: x - y, lambda v, t: v, Kr.matvec, Kr.rmatvec,
                       lambda w, s: OR.fenchel_prox(hprox, w, s), tau, sigma, 0.9, np.zeros(N), np.zeros(4 * N),
                       max_iter=29, min_iter=29, accuracy_threshold=0.0)
    K = Gradient(shape, step=steps, kind=kind)
    K.lipschitz_cst = K.diff_lipschitz_cst = lip
    pds = PDS(dim=N, F=(1 / 2) * SquaredL2Loss(dim=N, data=y), H=0.1 * L21Norm(dim=4 * N, groups=np.tile(np.arange(N), 4)),
              K=K, x0=np.zeros(N), z0=np.zeros(4 * N), max_iter=29, min_iter=29, accuracy_threshold=0.0, verbose=None)
    est, _, _ = pds.iterate()
    assert pds.iter == 30
    assert rel(est['primal_variable'], xr) < 1e-9
    assert rel(est['dual_variable'], zr) < 1e-9


FUSED_3D = [n for n in pds_case_names() if '3d' in n]


@pytest.mark.parametrize('name', FUSED_3D)
@pytest.mark.parametrize('dtype', [np.float64, np.float32])
def test_pds3d_fused_matches_reference(name, dtype):
    """3-D volumes: Convolve1D chain + 3-D Gradient + L21/L1 through PDS3DEngine."""
    from pycsou_amd.opt.engine3d import PDS3DEngine
    c = pds_case(name)
    pds = build(c, dtype, engine='fused')
    _check(pds, c, dtype)
    assert isinstance(pds._engine, PDS3DEngine)


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
def test_pds3d_ata_opt_in_matches_reference(monkeypatch, dtype):
    """The two-pass gradient (PCS_3D_ATA=1, the default: pcs_conv2d_sep_ata_planes + the
    axis-0 pass against C12^T y).  The golden volume's last axis (22) is not a multiple of 4,
    which the in-plane kernels need: there the engine keeps the three-pass chain (same
    trajectory); on a 24 x 20 x 24 volume the two-pass gradient runs and matches the oracle."""
    from pycsou_amd.opt.engine3d import PDS3DEngine
    monkeypatch.setenv('PCS_3D_ATA', '1')
    c = pds_case('deconv3d_l21_fwd_24_sep15')
    pds = build(c, dtype, engine='fused')
    _check(pds, c, dtype)
    assert isinstance(pds._engine, PDS3DEngine) and not pds._engine.ata
    c = _vol_problem(24, dtype, seed=5, niter=20, shape=(24, 20, 24))
    pds = build(c, dtype, engine='fused')
    c['tau'], c['sigma'], c['rho'] = pds.tau, pds.sigma, pds.rho
    est, _, _ = pds.iterate()
    assert isinstance(pds._engine, PDS3DEngine) and pds._engine.ata
    x_ref, z_ref, _ = oracle_pds(c)
    tol = 1e-10 if dtype == np.float64 else 5e-5
    assert rel(est['primal_variable'], x_ref) < tol
    assert rel(est['dual_variable'], z_ref) < tol


def _vol_problem(n, dtype, seed=0, lam=0.05, niter=10, shape=None, kind='forward'):
    """A 3-D TV deconvolution case (separable 15-tap Gaussian along every axis), built like
    the golden cases so tests/cases.oracle_pds can run it."""
    rng = np.random.default_rng(seed)
    shape = (n, n, n) if shape is None else tuple(shape)
    xs = np.zeros(shape)
    for _ in range(12):
        lo = np.array([rng.integers(0, m) for m in shape])
        hi = np.minimum(shape, lo + np.array([rng.integers(max(1, m // 8), max(2, m // 2)) for m in shape]))
        xs[lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2]] = rng.uniform(0, 1)
    r = np.arange(15) - 7
    taps = np.exp(-0.5 * (r / 2.0) ** 2)
    taps /= taps.sum()
    from oracle import pylops1 as P
    N = int(np.prod(shape))
    v = xs.ravel()
    for a in range(3):
        v = P.Convolve1D(N, taps, offset=7, dims=shape, dir=a).matvec(v)
    y = v + 0.01 * rng.standard_normal(N)
    c = {'shape': shape, 'taps': taps, 'y': y,
         'meta': {'kind': kind, 'hname': 'l21', 'lam': lam, 'niter': niter}}
    return c


def test_pds3d_128_fp64_vs_oracle():
    """C5 parity size (BASELINE configs[4]): 128^3 fp64, 20 iterations vs the CPU
    oracle."""
    c = _vol_problem(128, np.float64, niter=20)
    pds = build(c, np.float64, engine='fused')
    c['tau'], c['sigma'], c['rho'] = pds.tau, pds.sigma, pds.rho
    est, _, diag = pds.iterate()
    assert pds.iter == 20
    x_ref, z_ref, d_ref = oracle_pds(c)
    assert rel(est['primal_variable'], x_ref) < 1e-10
    assert rel(est['dual_variable'], z_ref) < 1e-10
    np.testing.assert_allclose(diag['Relative Improvement (primal variable)'].to_numpy(float)[1:],
                               np.asarray(d_ref['primal'])[1:], rtol=1e-8)


@pytest.mark.parametrize('verbose', [1, 7])
def test_verbose_lines_fused_match_generic(capsys, verbose):
    """``verbose`` prints ``dict(diagnostics row)`` every ``verbose`` iterations
    (solver.py:69-71, proxalgs.py:357-358): the fused engine prints the same lines, from its
    device history, as the per-iteration generic path."""
    c = pds_case('deconv2d_l21_fwd_64_psf15')
    lines = {}
    for eng in ('fused', 'generic'):
        pds = build(c, np.float64, engine=eng)
        pds.verbose = verbose
        capsys.readouterr()
        pds.iterate()
        out = capsys.readouterr().out.strip().splitlines()
        assert len(out) == len(range(0, pds.iter, verbose))
        lines[eng] = [eval(s, {'inf': np.inf, 'np': np}) for s in out]
    for a, b in zip(lines['fused'], lines['generic']):
        assert list(a) == ['Iter', 'Relative Improvement (primal variable)', 'Relative Improvement (dual variable)']
        assert a['Iter'] == b['Iter']
        for k in list(a)[1:]:
            assert a[k] == b[k] or abs(a[k] - b[k]) <= 1e-9 * abs(b[k]), (k, a, b)


def test_pds3d_c4_full_size_fused_vs_generic():
    """Full C4 size (512^3 fp32, 15-tap Gaussian along every axis, 0.05 L21): the fused 3-D
    engine (sep2d march + conv0 residual-adjoint + k_pds3d) against the operator-by-operator
    path for 3 iterations -- same iterates to fp32 rounding, finite, exact count."""
    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L21Norm
    from pycsou_amd.linop.conv import Convolve1D
    from pycsou_amd.linop.diff import Gradient
    from pycsou_amd.opt.engine3d import PDS3DEngine
    from pycsou_amd.opt.proxalgs import PDS
    n = 512
    shape, N = (n, n, n), n ** 3
    g = torch.Generator(device='cuda').manual_seed(3)
    xs = (torch.rand(shape, generator=g, device='cuda') > 0.5).float()
    r = np.arange(15) - 7
    taps = np.exp(-0.5 * (r / 2.0) ** 2)
    taps /= taps.sum()
    C = None
    for ax in range(3):
        Ci = Convolve1D(N, taps, reshape_dims=shape, axis=ax)
        Ci.lipschitz_cst = Ci.diff_lipschitz_cst = 1.0
        C = Ci if C is None else Ci * C
    C.lipschitz_cst = C.diff_lipschitz_cst = 1.0
    y = C(xs.reshape(-1)) + 0.01 * torch.randn(N, generator=g, device='cuda')
    del xs
    K = Gradient(shape=shape, kind='forward')
    K.lipschitz_cst = K.diff_lipschitz_cst = np.sqrt(12.0)
    H = 0.05 * L21Norm(dim=3 * N, groups=np.tile(np.arange(N), 3))
    F = (1 / 2) * SquaredL2Loss(dim=N, data=y) * C
    out = []
    for eng in ['fused', 'generic']:
        pds = PDS(dim=N, F=F, H=H, K=K, x0=torch.zeros(N, device='cuda'), z0=torch.zeros(3 * N, device='cuda'),
                  max_iter=2, min_iter=2, accuracy_threshold=0.0, verbose=None, engine=eng)
        est, _, diag = pds.iterate()
        assert pds.iter == 3
        if eng == 'fused':
            assert isinstance(pds._engine, PDS3DEngine)
        out.append((est['primal_variable'], est['dual_variable'],
                    diag['Relative Improvement (primal variable)'].to_numpy(float)))
        del pds, est
        torch.cuda.empty_cache()
    for k in range(2):
        d = float(torch.linalg.vector_norm(out[0][k] - out[1][k]) / torch.linalg.vector_norm(out[1][k]))
        assert d < 3e-5, (k, d)
    assert torch.isfinite(out[0][0]).all() and torch.isfinite(out[0][1]).all()
    np.testing.assert_allclose(out[0][2][1:], out[1][2][1:], rtol=1e-3)


@pytest.mark.parametrize('shape,dtype', [((20, 36, 260), np.float64), ((17, 9, 132), np.float32),
                                         ((12, 33, 130), np.float64)])
def test_pds3d_ragged_tiles_vs_oracle(shape, dtype):
    """Ragged 3-D shapes for the 8 x 128 update tiles and the 128-column sep2d strips: a last
    column tile of 4 (260, 132: vector path) or 2 columns (130: scalar path), rows not a
    multiple of 8, against the CPU oracle (8 iterations)."""
    c = _vol_problem(0, dtype, seed=5, niter=8, shape=shape)
    pds = build(c, dtype, engine='fused')
    c['tau'], c['sigma'], c['rho'] = pds.tau, pds.sigma, pds.rho
    est, _, diag = pds.iterate()
    assert pds.iter == 8
    x_ref, z_ref, d_ref = oracle_pds(c)
    tol = 1e-10 if dtype == np.float64 else 5e-5
    assert rel(est['primal_variable'], x_ref) < tol
    assert rel(est['dual_variable'], z_ref) < tol


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
@pytest.mark.parametrize('ata', ['', '0'])
def test_pds3d_gradient_order_default(monkeypatch, dtype, ata):
    """Which 3-D gradient runs: by default the two-pass one (C12^T C12, then the axis-0 pass) for
    fp32 and fp64 (since round 4); PCS_3D_ATA=0 pins the three-pass chain.  Either way the iterates
    match the oracle."""
    from pycsou_amd.opt.engine3d import PDS3DEngine
    if ata:
        monkeypatch.setenv('PCS_3D_ATA', ata)
    else:
        monkeypatch.delenv('PCS_3D_ATA', raising=False)
    c = _vol_problem(24, dtype, seed=7, niter=12, shape=(20, 24, 32))
    pds = build(c, dtype, engine='fused')
    c['tau'], c['sigma'], c['rho'] = pds.tau, pds.sigma, pds.rho
    est, _, _ = pds.iterate()
    assert isinstance(pds._engine, PDS3DEngine)
    assert pds._engine.ata == (not ata)
    x_ref, z_ref, _ = oracle_pds(c)
    tol = 1e-10 if dtype == np.float64 else 5e-5
    assert rel(est['primal_variable'], x_ref) < tol
    assert rel(est['dual_variable'], z_ref) < tol


@pytest.mark.parametrize('shape', [(24, 20, 24), (40, 24, 136), (17, 9, 132), (23, 37, 260)])
def test_pds3d_folded_axis0_bitwise(monkeypatch, shape):
    """fp32 forward K: the axis-0 pass folded into k_pds3d (PCS_F_CONV0, register rings of t and
    the residual) computes k_conv0_rta's sums in its order, so the iterates equal the separate
    axis-0 pass (PCS_3D_FOLD=0) bit for bit; and they match the oracle."""
    from pycsou_amd.opt.engine3d import PDS3DEngine
    c = _vol_problem(0, np.float32, seed=9, niter=10, shape=shape)
    out = []
    for fold in ('1', '0'):
        monkeypatch.setenv('PCS_3D_FOLD', fold)
        pds = build(c, np.float32, engine='fused')
        est, _, diag = pds.iterate()
        assert isinstance(pds._engine, PDS3DEngine) and pds._engine.ata
        assert pds._engine.fold == (fold == '1')
        out.append((est['primal_variable'], est['dual_variable'],
                    diag['Relative Improvement (primal variable)'].to_numpy(float)))
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
    np.testing.assert_array_equal(out[0][2], out[1][2])
    c['tau'], c['sigma'], c['rho'] = pds.tau, pds.sigma, pds.rho
    x_ref, z_ref, _ = oracle_pds(c)
    assert rel(out[0][0], x_ref) < 5e-5 and rel(out[0][1], z_ref) < 5e-5


@pytest.mark.parametrize('shape,dtype,kind', [((20, 36, 260), np.float64, 'centered'), ((17, 9, 132), np.float32, 'centered'),
                                              ((12, 33, 130), np.float64, 'backward'), ((24, 20, 24), np.float32, 'backward'),
                                              ((12, 40, 136), np.float32, 'centered'), ((10, 30, 260), np.float32, 'centered'),
                                              ((9, 26, 258), np.float32, 'backward'), ((8, 30, 66), np.float64, 'centered')])
def test_pds3d_general_k_vs_oracle(shape, dtype, kind):
    """Backward / centred 3-D Gradient (the reference's default kind) through the general-K plane
    march (k_pds3d_gen): ragged tiles (last column tile of 4 or 2 columns, rows not a multiple of
    8), 15-tap blur along every axis, against the CPU oracle (8 iterations)."""
    from pycsou_amd.opt.engine3d import PDS3DEngine
    c = _vol_problem(0, dtype, seed=5, niter=8, shape=shape, kind=kind)
    pds = build(c, dtype, engine='fused')
    c['tau'], c['sigma'], c['rho'] = pds.tau, pds.sigma, pds.rho
    est, _, diag = pds.iterate()
    assert isinstance(pds._engine, PDS3DEngine) and pds._engine.kkind != 0
    assert pds.iter == 8
    x_ref, z_ref, d_ref = oracle_pds(c)
    tol = 1e-10 if dtype == np.float64 else 5e-5
    assert rel(est['primal_variable'], x_ref) < tol
    assert rel(est['dual_variable'], z_ref) < tol
    np.testing.assert_allclose(diag['Relative Improvement (primal variable)'].to_numpy(float)[1:],
                               np.asarray(d_ref['primal'])[1:], rtol=1e-8 if dtype == np.float64 else 1e-3)

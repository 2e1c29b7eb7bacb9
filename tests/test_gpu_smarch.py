"""The general-stencil row-marching fused step (pds_smarch.hpp: fp32, K = backward / centered /
forward Gradient or Laplacian, pointwise grad F) against the fp64 oracle.

Shapes exercise the kernel's edges: a partial last 64-column strip, a 4-column last strip,
several row segments with a short last one, images only a few rows tall (every edge rule of
both axes inside one 16-row step), edge=True / False, non-unit sampling, Laplacian weights, every
prox_G kind, L1 / L21, F = 0, (1/2)||x - y||^2, a non-separable PSF through the gradient buffer and
separable PSFs (odd and even lengths) through the normal operator (grad F = N x - Conv^T y).

Tolerance: relative L2 of x and z <= 5e-5 after 12 iterations (fp32 against fp64, as the golden
fp32 cases), diagnostics to 1e-3 relative, iteration counts exact.  The oracle restates
PrimalDualSplitting (pycsou/opt/proxalgs.py:343-394) over the PyLops 1.x stencils
(pycsou/linop/diff.py:777-957); edge rows are PARITY UNPINNED (PyLops is absent), see DESIGN.md.
"""

import numpy as np
import pytest

from oracle import pycsou_ref as OR
from tests.cases import rel

pytestmark = pytest.mark.gpu

NITER = 12


def _problem(shape, kind, hname, fk, gname, edge, steps, weights, seed):
    rng = np.random.default_rng(seed)
    n0, n1 = shape
    N = n0 * n1
    xs = OR.phantom(shape, seed=seed)
    psf = None
    if fk == 'conv':  # non-separable 5x5: the correlation kernel into the gradient buffer
        psf = rng.uniform(0.0, 1.0, (5, 5))
        psf /= psf.sum()
    elif fk.startswith('sep'):  # 'sep15', 'sep4x6': separable, grad F = N x - Conv^T y
        l0, l1 = (int(v) for v in (fk[3:].split('x') * 2)[:2])
        r0, r1 = np.arange(l0) - l0 // 2, np.arange(l1) - l1 // 2
        t0, t1 = np.exp(-0.5 * (r0 / 1.9) ** 2), np.exp(-0.5 * (r1 / 2.3) ** 2)
        psf = np.outer(t0 / t0.sum(), t1 / t1.sum())
    return dict(shape=shape, N=N, kind=kind, hname=hname, fk=fk, gname=gname, edge=edge, steps=steps,
                weights=weights, psf=psf, y=xs.ravel() + 0.05 * rng.standard_normal(N), lam=0.05)


def _lip(p):
    if p['kind'] == 'lap':
        return float(4.0 * sum(abs(w) / s ** 2 for w, s in zip(p['weights'], p['steps'])))
    return float(np.sqrt(sum(4.0 / s ** 2 for s in p['steps'])))


def _oracle(p):
    from oracle import pylops1 as P
    shape, N, y = p['shape'], p['N'], p['y']
    if p['fk'] == 'null':
        grad = lambda v: np.zeros_like(v)  # noqa: E731
    elif p['fk'] == 'denoise':
        grad = lambda v: (2 * (v + (-y))) * 0.5  # noqa: E731
    else:  # any PSF
        off = tuple(P.pycsou_offset(n) for n in p['psf'].shape)
        C = P.Convolve2D(N, p['psf'], shape, offset=off)
        grad = lambda v: C.rmatvec((2 * (C.matvec(v) + (-y))) * 0.5)  # noqa: E731
    if p['kind'] == 'lap':
        K = P.Laplacian(shape, weights=p['weights'], sampling=p['steps'], edge=p['edge'])
        Hdim = N
    else:
        K = P.Gradient(shape, sampling=p['steps'], edge=p['edge'], kind=p['kind'])
        Hdim = 2 * N
    if p['hname'] == 'l21':
        hprox = OR.postcomp(lambda v, t: OR.prox_l21_pixel(v, t, 2), p['lam'])
    else:
        hprox = OR.postcomp(OR.prox_l1, p['lam'])
    gprox = {'nonneg': lambda v, t: OR.proj_nonnegative_orthant(v),
             'segment': lambda v, t: OR.proj_segment(v, 0.0, 1.0)}.get(p['gname'], lambda v, t: v)
    beta = 0.0 if p['fk'] == 'null' else 1.0
    tau, sigma = OR.pds_step_sizes(beta, _lip(p))[:2]
    rho = 1.0 if beta == 0 else 0.9
    x, z, d = OR.pds(grad, gprox, K.matvec, K.rmatvec, lambda w, s: OR.fenchel_prox(hprox, w, s), tau, sigma, rho,
                     np.zeros(N), np.zeros(Hdim), max_iter=NITER - 1, min_iter=NITER - 1, accuracy_threshold=0.0)
    return x, z, d


def _fused(p, dtype=np.float32):
    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L1Norm, L21Norm, NonNegativeOrthant, Segment
    from pycsou_amd.linop.conv import Convolve2D
    from pycsou_amd.linop.diff import Gradient, Laplacian
    from pycsou_amd.opt.engine import PDS2DStencilEngine
    from pycsou_amd.opt.proxalgs import PDS
    shape, N = p['shape'], p['N']
    F = None
    if p['fk'] != 'null':
        F = (1 / 2) * SquaredL2Loss(dim=N, data=p['y'].astype(dtype))
    if p['psf'] is not None:
        C = Convolve2D(N, p['psf'], shape)
        C.lipschitz_cst = C.diff_lipschitz_cst = 1.0
        F = F * C
    if p['kind'] == 'lap':
        K = Laplacian(shape, weights=p['weights'], step=p['steps'], edge=p['edge'])
        Hdim = N
    else:
        K = Gradient(shape, step=p['steps'], edge=p['edge'], kind=p['kind'])
        Hdim = 2 * N
    K.lipschitz_cst = K.diff_lipschitz_cst = _lip(p)
    H = p['lam'] * (L21Norm(dim=Hdim, groups=np.tile(np.arange(N), 2)) if p['hname'] == 'l21' else L1Norm(dim=Hdim))
    G = {'nonneg': NonNegativeOrthant(N), 'segment': Segment(N, 0.0, 1.0)}.get(p['gname'], None)
    pds = PDS(dim=N, F=F, G=G, H=H, K=K, x0=np.zeros(N, dtype), z0=np.zeros(Hdim, dtype),
              max_iter=NITER - 1, min_iter=NITER - 1, accuracy_threshold=0.0, verbose=None, engine='stencil')
    est, _, diag = pds.iterate()
    eng = pds._engine
    assert isinstance(eng, PDS2DStencilEngine) and pds.iter == NITER
    return est['primal_variable'], est['dual_variable'], diag, eng


CASES = [
    # shape, K kind, H, F, G, edge, steps, Laplacian weights
    ((300, 200), 'centered', 'l21', 'denoise', '', True, (1.0, 1.0), (1, 1)),      # partial last strip (200 = 3*64 + 8)
    ((261, 132), 'backward', 'l1', 'denoise', 'segment', True, (2.0, 0.5), (1, 1)),  # 4-column last strip, non-unit
    ((190, 256), 'lap', 'l1', 'denoise', 'nonneg', True, (0.7, 1.3), (2.0, 0.5)),    # weights, sampling
    ((1030, 2048), 'centered', 'l21', 'denoise', '', False, (1.0, 1.0), (1, 1)),     # C2 width, short last segment
    ((517, 1000), 'lap', 'l1', 'denoise', 'segment', False, (1.0, 1.0), (1.0, 1.0)),  # ragged rows, edge=False
    ((1000, 128), 'centered', 'l1', 'conv', 'nonneg', True, (1.0, 1.0), (1, 1)),     # tall, gradient buffer
    ((3, 260), 'lap', 'l1', 'denoise', '', True, (1.0, 1.0), (1.0, 1.0)),            # 3 rows: both edge rules, one step
    ((5, 132), 'centered', 'l21', 'denoise', '', True, (1.0, 1.0), (1, 1)),          # 5 rows
    ((17, 68), 'centered', 'l21', 'null', '', True, (1.0, 1.0), (1, 1)),             # F = 0, strips of 64 + 4
    ((129, 192), 'forward', 'l21', 'denoise', 'segment', True, (1.0, 1.0), (1, 1)),  # forward through PCS_SM_FWD
    ((64, 4096), 'backward', 'l21', 'denoise', '', True, (1.0, 1.0), (1, 1)),        # C3 width, 4 steps
    ((48, 128), 'lap', 'l1', 'null', 'nonneg', True, (1.0, 2.0), (0.5, 1.5)),        # F = 0 Laplacian
    # separable PSFs: grad F = N x - Conv^T y (normal-operator kernel + march step, SEPCONV)
    ((1000, 4096), 'centered', 'l21', 'sep15', 'nonneg', True, (1.0, 1.0), (1, 1)),  # C3 width, default K
    ((300, 200), 'lap', 'l1', 'sep4x6', '', True, (1.0, 1.0), (1.0, 1.0)),            # even lengths, partial strip
    ((261, 132), 'backward', 'l21', 'sep9', 'segment', True, (2.0, 0.5), (1, 1)),     # tier 7 half 4, 4-col strip
    ((130, 256), 'centered', 'l1', 'sep14x14', '', False, (1.0, 1.0), (1, 1)),        # even 14x14
    # fused normal-operator march for backward / centred K (pds_nmarch.hpp GEN): one launch
    ((200, 320), 'backward', 'l1', 'sep15', 'segment', True, (2.0, 0.5), (1, 1)),     # non-unit steps
    ((96, 200), 'centered', 'l21', 'sep9', '', False, (1.0, 1.0), (1, 1)),            # 8-column last strip
    ((150, 196), 'centered', 'l21', 'sep7', 'nonneg', True, (1.0, 1.0), (1, 1)),      # tier 3, 4-column strip
    ((64, 4160), 'centered', 'l1', 'sep6x10', '', True, (1.0, 1.0), (1, 1)),         # 64 rows, even taps
]

# (shape, K kind, PSF) -> the fused march must take it (last strip wider than the tier)
FUSED = {('centered', 'sep15'), ('centered', 'sep14x14'), ('backward', 'sep15'), ('centered', 'sep9'),
         ('centered', 'sep7'), ('centered', 'sep6x10')}


@pytest.mark.parametrize('case', range(len(CASES)), ids=lambda i: f'{CASES[i][1]}-{CASES[i][0][0]}x{CASES[i][0][1]}')
def test_smarch_vs_oracle(case, monkeypatch):
    shape, kind, hname, fk, gname, edge, steps, weights = CASES[case]
    if kind == 'forward':
        monkeypatch.setenv('PCS_SM_FWD', '1')  # read once per process: the forward case checks routing below
    p = _problem(shape, kind, hname, fk, gname, edge, steps, weights, seed=case)
    xr, zr, dr = _oracle(p)
    x, z, diag, eng = _fused(p)
    assert eng.march or kind == 'forward', 'the row-marching kernel must take this problem'
    if fk.startswith('sep'):
        from pycsou_amd import _lib as L
        assert eng.fkind == L.PCS_F_SEPCONV and eng.cty is not None, 'separable PSF: normal-operator gradient'
        assert eng.nm_fused == ((kind, fk) in FUSED), ('fused normal-operator march', kind, fk, eng.nm_fused)
    assert x.dtype == np.float32
    assert rel(x, xr) < 5e-5, rel(x, xr)
    assert rel(z, zr) < 5e-5, rel(z, zr)
    np.testing.assert_allclose(diag['Relative Improvement (primal variable)'].to_numpy(float)[1:], dr['primal'][1:],
                               rtol=1e-3)
    np.testing.assert_allclose(diag['Relative Improvement (dual variable)'].to_numpy(float)[1:], dr['dual'][1:],
                               rtol=1e-3)


@pytest.mark.parametrize('kind', ['centered', 'lap'])
def test_smarch_matches_tile_kernel(kind, monkeypatch):
    """The march kernel and the 32 x 64 tile kernel (PCS_STENCIL_MARCH=0) on the same fp32 problem:
    same iteration count, x and z to 2e-6 relative (fp32 rounding of two operation orders)."""
    args = ((530, 388), kind, 'l1' if kind == 'lap' else 'l21', 'denoise', 'nonneg', True, (1.0, 1.0), (1.0, 1.0))
    p = _problem(*args, seed=7)
    x1, z1, d1, e1 = _fused(p)
    monkeypatch.setenv('PCS_STENCIL_MARCH', '0')
    x0, z0, d0, e0 = _fused(p)
    assert e1.march and not e0.march
    assert rel(x1, x0) < 2e-6 and rel(z1, z0) < 2e-6


@pytest.mark.parametrize('kind', ['centered', 'backward'])
def test_fused_normal_march_matches_two_launch(kind, monkeypatch):
    """Backward / centred K with a separable PSF: the fused normal-operator march (N x inside the
    step) against the two-launch path (PCS_NMARCH_GEN=0: k_sep2d_nrm into a buffer + the stencil
    march) on a 520 x 1024 problem -- the same iterates to fp32 rounding of two operation orders."""
    args = ((520, 1024), kind, 'l21', 'sep15', 'nonneg', True, (1.0, 1.0), (1, 1))
    p = _problem(*args, seed=11)
    x1, z1, d1, e1 = _fused(p)
    monkeypatch.setenv('PCS_NMARCH_GEN', '0')
    x0, z0, d0, e0 = _fused(p)
    assert e1.nm_fused and not e0.nm_fused
    assert rel(x1, x0) < 2e-6 and rel(z1, z0) < 2e-6, (rel(x1, x0), rel(z1, z0))


@pytest.mark.parametrize('case', range(len(CASES)), ids=lambda i: f'f64-{CASES[i][1]}-{CASES[i][0][0]}x{CASES[i][0][1]}')
def test_smarch_fp64_vs_oracle(case):
    """The same cases in fp64 (the reference's default dtype: pycsou/opt/proxalgs.py:327,341,
    linop/diff.py:777): the fp64 form of the row march for every K kind, the forward Gradient included;
    separable PSFs through the fused fp64 normal-operator march (Gradient K) or N x by k_sep2d_nrmm + the
    march step (Laplacian).  Bar: x and z to 1e-10 relative,
    both diagnostics columns to 1e-9 relative (fp64 against fp64: operation order only)."""
    from pycsou_amd import _lib as L
    shape, kind, hname, fk, gname, edge, steps, weights = CASES[case]
    p = _problem(shape, kind, hname, fk, gname, edge, steps, weights, seed=case)
    xr, zr, dr = _oracle(p)
    x, z, diag, eng = _fused(p, np.float64)
    assert eng.march, 'the fp64 row-marching kernel must take this problem'
    assert eng.args.dtype == L.PCS_F64
    if fk.startswith('sep'):  # Gradient K: the fused fp64 march (pds_nm64.hip); Laplacian: N x + the march step
        assert eng.fkind == L.PCS_F_SEPCONV and eng.cty is not None and eng.nm_fused == (kind != 'lap')
    assert x.dtype == np.float64
    assert rel(x, xr) < 1e-10, rel(x, xr)
    assert rel(z, zr) < 1e-10, rel(z, zr)
    np.testing.assert_allclose(diag['Relative Improvement (primal variable)'].to_numpy(float)[1:], dr['primal'][1:],
                               rtol=1e-9)
    np.testing.assert_allclose(diag['Relative Improvement (dual variable)'].to_numpy(float)[1:], dr['dual'][1:],
                               rtol=1e-9)


def test_fp64_default_routing_takes_the_march():
    """A reference-default fp64 script (NumPy float64 arrays, K = Gradient(shape) centred, and the forward
    K) on a C3-shaped image strip goes to the fp64 march through engine='fused' (auto)."""
    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L21Norm
    from pycsou_amd.linop.conv import Convolve2D
    from pycsou_amd.linop.diff import Gradient
    from pycsou_amd.opt.engine import PDS2DStencilEngine
    from pycsou_amd.opt.proxalgs import PDS
    shape = (96, 512)
    N = shape[0] * shape[1]
    y = np.random.default_rng(0).uniform(0, 1, N)
    for kind in ('centered', 'forward'):
        C = Convolve2D(N, OR.gaussian_psf(15, 2.0), shape)
        C.compute_lipschitz_cst()
        K = Gradient(shape, kind=kind)
        K.compute_lipschitz_cst()
        pds = PDS(dim=N, F=(1 / 2) * SquaredL2Loss(dim=N, data=y) * C,
                  H=0.05 * L21Norm(dim=2 * N, groups=np.tile(np.arange(N), 2)), K=K, max_iter=5, min_iter=5,
                  accuracy_threshold=0.0, verbose=None)
        pds.iterate()
        assert isinstance(pds._engine, PDS2DStencilEngine) and pds._engine.march, kind
        assert pds._engine.nm_fused, kind  # one launch per iteration (pds_nm64.hip)

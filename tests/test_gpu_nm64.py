"""The fused fp64 normal-operator march (pds_nm64.hip, k_pds2d_nmarch64): the reference's default dtype
(x0 / z0 np.float, pycsou/opt/proxalgs.py:327,341; Gradient / Convolve2D dtype='float64', linop/diff.py:777,
linop/conv.py:167) with a separable PSF in ONE launch per iteration.  Its per-element operations are the
split form's (k_sep2d_nrmm's N x minus Conv^T y into a buffer, then k_pds2d_smarch<double>, PCS_NM64=0),
so the two agree to the last bits; against the fp64 oracle the bar is the fp64 one (1e-10)."""

import numpy as np
import pytest

from tests.cases import rel
from tests.test_gpu_smarch import _fused, _oracle, _problem

pytestmark = pytest.mark.gpu

NM64_CASES = [
    # shape, K kind, H, F, G, edge, steps, Laplacian weights
    ((1000, 4096), 'centered', 'l21', 'sep15', 'nonneg', True, (1.0, 1.0), (1, 1)),   # C3 width, default K
    ((517, 1000), 'forward', 'l21', 'sep15', '', True, (1.0, 1.0), (1, 1)),          # ragged rows, partial strip
    ((261, 132), 'backward', 'l1', 'sep9', 'segment', True, (2.0, 0.5), (1, 1)),     # non-unit steps, 3 strips
    ((150, 196), 'centered', 'l21', 'sep7', 'nonneg', True, (1.0, 1.0), (1, 1)),     # tier 3
    ((130, 256), 'centered', 'l1', 'sep14x14', '', False, (1.0, 1.0), (1, 1)),       # even taps, edge=False
    ((64, 4160), 'centered', 'l1', 'sep6x10', '', True, (1.0, 1.0), (1, 1)),         # 64 rows: one segment
    ((333, 512), 'backward', 'l21', 'sep15', '', True, (1.0, 1.0), (1, 1)),          # 512 = 8 strips + 32 columns
]


def _ids(i):
    s = NM64_CASES[i]
    return f'{s[1]}-{s[3]}-{s[0][0]}x{s[0][1]}'


@pytest.mark.parametrize('case', range(len(NM64_CASES)), ids=_ids)
def test_nm64_vs_oracle(case):
    """x and z to 1e-10, both diagnostics columns to 1e-9 relative against the fp64 oracle; the fused
    march (not the split form) ran."""
    p = _problem(*NM64_CASES[case], seed=30 + case)
    xr, zr, dr = _oracle(p)
    x, z, diag, eng = _fused(p, np.float64)
    assert eng.march and eng.nm_fused, 'the fused fp64 normal-operator march must take this problem'
    assert x.dtype == np.float64
    assert rel(x, xr) < 1e-10, rel(x, xr)
    assert rel(z, zr) < 1e-10, rel(z, zr)
    np.testing.assert_allclose(diag['Relative Improvement (primal variable)'].to_numpy(float)[1:], dr['primal'][1:],
                               rtol=1e-9)
    np.testing.assert_allclose(diag['Relative Improvement (dual variable)'].to_numpy(float)[1:], dr['dual'][1:],
                               rtol=1e-9)


@pytest.mark.parametrize('case', [0, 1, 2, 3, 6], ids=lambda i: _ids(i))
def test_nm64_matches_split_form(case, monkeypatch):
    """The fused march against the split form on the same problem: the same per-element operations,
    so x and z agree to 1e-14 relative (operation order of the norms only differs)."""
    p = _problem(*NM64_CASES[case], seed=50 + case)
    x1, z1, d1, e1 = _fused(p, np.float64)
    monkeypatch.setenv('PCS_NM64', '0')
    x0, z0, d0, e0 = _fused(p, np.float64)
    assert e1.nm_fused and not e0.nm_fused
    assert rel(x1, x0) < 1e-14, rel(x1, x0)
    assert rel(z1, z0) < 1e-14, rel(z1, z0)
    np.testing.assert_allclose(d1['Relative Improvement (primal variable)'].to_numpy(float)[1:],
                               d0['Relative Improvement (primal variable)'].to_numpy(float)[1:], rtol=1e-12)


@pytest.mark.parametrize('kind', ['centered', 'forward'])
@pytest.mark.parametrize('thr', [1e-3, 1e-4])
def test_nm64_natural_stop(kind, thr):
    """A reference-default fp64 script with a natural stop (accuracy_threshold 1e-3 / 1e-4): the same
    stopping iteration as the fp64 oracle, x and z to 1e-10."""
    from oracle import pycsou_ref as OR
    from oracle import pylops1 as P
    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L21Norm
    from pycsou_amd.linop.conv import Convolve2D
    from pycsou_amd.linop.diff import Gradient
    from pycsou_amd.opt.proxalgs import PDS
    n0, n1 = 384, 512
    N = n0 * n1
    rng = np.random.default_rng(7)
    h = OR.gaussian_psf(15, 2.0)
    Cr = P.Convolve2D(N, h, (n0, n1), offset=(7, 7))
    y = Cr.matvec(OR.phantom((n0, n1), seed=7).ravel()) + 0.01 * rng.standard_normal(N)
    C = Convolve2D(N, h, (n0, n1))
    C.lipschitz_cst = C.diff_lipschitz_cst = 1.0
    K = Gradient((n0, n1), kind=kind)
    K.compute_lipschitz_cst()
    pds = PDS(dim=N, F=(1 / 2) * SquaredL2Loss(dim=N, data=y) * C,
              H=0.05 * L21Norm(dim=2 * N, groups=np.tile(np.arange(N), 2)), K=K, max_iter=499, min_iter=10,
              accuracy_threshold=thr, verbose=None)
    est, _, _ = pds.iterate()
    assert pds._engine is not None and pds._engine.nm_fused
    Kr = P.Gradient((n0, n1), edge=True, kind=kind)
    hprox = OR.postcomp(lambda v, t: OR.prox_l21_pixel(v, t, 2), 0.05)
    xr, zr, dr = OR.pds(lambda v: Cr.rmatvec((2 * (Cr.matvec(v) + (-y))) * 0.5), lambda v, t: v, Kr.matvec,
                        Kr.rmatvec, lambda w, s: OR.fenchel_prox(hprox, w, s), pds.tau, pds.sigma, pds.rho,
                        np.zeros(N), np.zeros(2 * N), max_iter=499, min_iter=10, accuracy_threshold=thr)
    assert pds.iter == len(dr['primal']), (pds.iter, len(dr['primal']))
    assert 10 < pds.iter < 500
    assert rel(est['primal_variable'], xr) < 1e-10
    assert rel(est['dual_variable'], zr) < 1e-10

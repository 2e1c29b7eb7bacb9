"""Long-horizon fp32 parity: the C3 kernels (k_pds2d_nmarch for forward K, k_pds2d_nmarch_gen for
the reference's default centred K) over the hundreds of iterations a max_iter=500 script runs,
against the fp64 oracle (pycsou/core/solver.py:55-76 loop, stopping rule
pycsou/opt/proxalgs.py:360-394).  512^2, 15x15 Gaussian PSF (sigma 2), 0.05 * L21Norm.

Bars (stated here, the fp32-vs-fp64 tolerance of north_star over long runs):
* natural stop (accuracy_threshold 1e-3, the default, and 1e-4): the SAME stopping iteration as
  fp64 (45 / 303 iterations for forward K; the metric falls ~0.4 % per iteration at the crossing,
  far above the fp32 error of the relative improvement), x and z to 1e-4 relative L2;
* fixed 500 iterations (accuracy_threshold 0): x and z to 1e-4 relative L2, both diagnostics
  columns to 5e-3 relative.
"""

import numpy as np
import pytest

from oracle import pycsou_ref as OR
from tests.cases import rel

pytestmark = pytest.mark.gpu

N0 = 512


def _setup(kind):
    from oracle import pylops1 as P
    from pycsou_amd.linop.diff import Gradient
    n = N0
    N = n * n
    rng = np.random.default_rng(11)
    xs = OR.phantom((n, n), seed=11)
    h = OR.gaussian_psf(15, 2.0)
    C = P.Convolve2D(N, h, (n, n), offset=(7, 7))
    y = C.matvec(xs.ravel()) + 0.01 * rng.standard_normal(N)
    Kd = Gradient((n, n), kind=kind)
    Kd.compute_lipschitz_cst()  # exact (linop/_spectral.py), the same value for both runs
    return dict(n=n, N=N, h=h, C=C, y=y, kind=kind, lip=float(Kd.lipschitz_cst))


def _oracle(p, max_iter, thr):
    from oracle import pylops1 as P
    C, y, N = p['C'], p['y'], p['N']
    K = P.Gradient((p['n'], p['n']), edge=True, kind=p['kind'])
    tau, sigma = OR.pds_step_sizes(1.0, p['lip'])[:2]
    hprox = OR.postcomp(lambda v, t: OR.prox_l21_pixel(v, t, 2), 0.05)
    return OR.pds(lambda v: C.rmatvec((2 * (C.matvec(v) + (-y))) * 0.5), lambda v, t: v, K.matvec, K.rmatvec,
                  lambda w, s: OR.fenchel_prox(hprox, w, s), tau, sigma, 0.9, np.zeros(N), np.zeros(2 * N),
                  max_iter=max_iter, min_iter=10 if thr > 0 else max_iter, accuracy_threshold=thr)


def _fused(p, max_iter, thr):
    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L21Norm
    from pycsou_amd.linop.conv import Convolve2D
    from pycsou_amd.linop.diff import Gradient
    from pycsou_amd.opt.proxalgs import PDS
    n, N = p['n'], p['N']
    C = Convolve2D(N, p['h'], (n, n))
    C.lipschitz_cst = C.diff_lipschitz_cst = 1.0  # as the oracle's beta = 1
    K = Gradient((n, n), kind=p['kind'])
    K.lipschitz_cst = K.diff_lipschitz_cst = p['lip']
    F = (1 / 2) * SquaredL2Loss(dim=N, data=p['y'].astype(np.float32)) * C
    H = 0.05 * L21Norm(dim=2 * N, groups=np.tile(np.arange(N), 2))
    pds = PDS(dim=N, F=F, H=H, K=K, x0=np.zeros(N, np.float32), z0=np.zeros(2 * N, np.float32),
              max_iter=max_iter, min_iter=10 if thr > 0 else max_iter, accuracy_threshold=thr, verbose=None,
              engine='fused')
    est, _, diag = pds.iterate()
    assert pds._engine is not None
    assert getattr(pds._engine, 'cty', None) is not None  # the normal-operator march (the C3 kernels)
    return pds.iter, est['primal_variable'], est['dual_variable'], diag


@pytest.mark.parametrize('kind', ['forward', 'centered'])
@pytest.mark.parametrize('thr', [1e-3, 1e-4])
def test_long_horizon_natural_stop(kind, thr):
    p = _setup(kind)
    xr, zr, dr = _oracle(p, 499, thr)
    it, x, z, diag = _fused(p, 499, thr)
    assert x.dtype == np.float32
    assert it == len(dr['primal']), (it, len(dr['primal']))
    assert 10 < it < 500
    assert rel(x, xr) < 1e-4, rel(x, xr)
    assert rel(z, zr) < 1e-4, rel(z, zr)


@pytest.mark.parametrize('kind', ['forward', 'centered'])
def test_long_horizon_fixed_500(kind):
    p = _setup(kind)
    xr, zr, dr = _oracle(p, 499, 0.0)
    it, x, z, diag = _fused(p, 499, 0.0)
    assert it == 500 == len(dr['primal'])
    assert rel(x, xr) < 1e-4, rel(x, xr)
    assert rel(z, zr) < 1e-4, rel(z, zr)
    np.testing.assert_allclose(diag['Relative Improvement (primal variable)'].to_numpy(float)[1:],
                               np.asarray(dr['primal'])[1:], rtol=5e-3)
    np.testing.assert_allclose(diag['Relative Improvement (dual variable)'].to_numpy(float)[1:],
                               np.asarray(dr['dual'])[1:], rtol=5e-3)

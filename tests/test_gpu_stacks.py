"""Widened operator set on the GPU against the real reference's
golden vectors (tests/golden/make_golden_stacks.py): operator / functional stacks, sampling,
second and generalised derivatives, moving averages, and the notebook workflows built from
them -- CPS TV-LAD inpainting (cell [62]) and APGD Tikhonov (cell [55]).

Tolerances: operators fp64 <= 1e-12 relative (gathers bitwise); solver iterates fp64 <= 1e-9
relative with identical iteration counts.
"""

import numpy as np
import pytest

from oracle import pycsou_ref as OR
from tests.cases import load, rel

pytestmark = pytest.mark.gpu

SHAPE = (12, 9)
N = 108


@pytest.fixture(scope='module')
def f():
    return load('stacks.npz')


def test_linop_stacks(f):
    from pycsou_amd.linop import DenseLinearOperator, FirstDerivative, LinOpHStack, LinOpStack, LinOpVStack
    x, w = f['x'], f['w']
    D1 = FirstDerivative(size=N, shape=SHAPE, axis=0, kind='centered')
    D2 = FirstDerivative(size=N, shape=SHAPE, axis=1, kind='forward')
    V = LinOpStack(D1, D2, axis=0)
    assert V.shape == (2 * N, N)
    assert rel(V(x), f['vstack_fwd']) < 1e-13
    assert rel(V.adjoint(w), f['vstack_adj']) < 1e-13
    Hs = LinOpHStack(D1.H, D2.H)
    assert Hs.shape == (N, 2 * N)
    assert rel(Hs(w), f['hstack_fwd']) < 1e-13
    assert rel(Hs.adjoint(x), f['hstack_adj']) < 1e-13
    Dn = DenseLinearOperator(f['A'])
    V2 = LinOpVStack(Dn, D2)
    assert rel(V2(x), f['vstack2_fwd']) < 1e-13
    assert rel(V2.adjoint(np.concatenate([w[:5], w[:N]])), f['vstack2_adj']) < 1e-13
    # Lipschitz bound of a vertical stack: sqrt(sum L_i^2) (core/map.py:916-918)
    D1.lipschitz_cst, D2.lipschitz_cst = 2.0, 3.0
    assert LinOpVStack(D1, D2).lipschitz_cst == pytest.approx(np.sqrt(13.0))
    assert LinOpHStack(D1, D2).lipschitz_cst == 3.0
    with pytest.raises(ValueError):
        LinOpVStack(D1, DenseLinearOperator(np.ones((3, 5))))


def test_functional_stacks(f):
    from pycsou_amd.func import DiffFuncHStack, L1Loss, L1Norm, L2Norm, ProxFuncHStack, SquaredL2Loss, SquaredL2Norm
    z, yd = f['z'], f['yd']
    hs = ProxFuncHStack(L1Norm(dim=N), 0.7 * L2Norm(dim=N))
    assert hs.dim == 2 * N
    assert float(hs(z)) == pytest.approx(float(f['phs_value']), rel=1e-13)
    assert rel(hs.prox(z, 0.3), f['phs_prox_03']) < 1e-13
    assert rel(hs.fenchel_prox(z, 0.5), f['phs_fenchel_05']) < 1e-13
    hs2 = ProxFuncHStack(L1Loss(dim=N, data=yd), 0.6 * L1Norm(dim=N))
    assert rel(hs2.prox(z, 0.4), f['phs2_prox_04']) < 1e-13
    assert rel(hs2.fenchel_prox(z, 0.7), f['phs2_fenchel_07']) < 1e-13
    dh = DiffFuncHStack(SquaredL2Norm(dim=N), SquaredL2Loss(dim=N, data=yd))
    assert float(dh(z)) == pytest.approx(float(f['dhs_value']), rel=1e-13)
    assert rel(dh.gradient(z), f['dhs_grad']) < 1e-14


def test_sampling(f):
    from pycsou_amd.linop import DownSampling, Masking, SubSampling
    x, mask = f['x'], f['mask']
    M = Masking(size=N, sampling_bool=mask)
    assert M.shape == (int(mask.sum()), N)
    np.testing.assert_array_equal(M(x), f['mask_fwd'])
    np.testing.assert_array_equal(M.adjoint(M(x)), f['mask_adj'])
    Ds = DownSampling(size=N, shape=SHAPE, downsampling_factor=(3, 2))
    assert Ds.output_shape == tuple(f['down_shape'])
    np.testing.assert_array_equal(Ds(x), f['down_fwd'])
    np.testing.assert_array_equal(Ds.adjoint(Ds(x)), f['down_adj'])
    Da = DownSampling(size=N, shape=SHAPE, downsampling_factor=2, axis=1)
    assert Da.output_shape == tuple(f['downax_shape'])
    np.testing.assert_array_equal(Da(x), f['downax_fwd'])
    Ss = SubSampling(size=N, sampling_indices=f['iava'], shape=SHAPE, axis=0)
    np.testing.assert_array_equal(Ss(x), f['sub_fwd'])
    np.testing.assert_array_equal(Ss.adjoint(Ss(x)), f['sub_adj'])
    with pytest.raises(ValueError):
        Masking(size=N + 1, sampling_bool=mask)
    with pytest.raises(ValueError):
        DownSampling(size=N, shape=SHAPE, downsampling_factor=(2, 2, 2))
    # empty selection
    E = Masking(size=N, sampling_bool=np.zeros(N, bool))
    assert E(x).size == 0 and np.all(E.adjoint(np.zeros(0)) == 0)


def test_derivatives_and_generalised(f):
    from pycsou_amd.linop import (DenseLinearOperator, GeneralisedDerivative, GeneralisedLaplacian,
                                  PolynomialLinearOperator, SecondDerivative)
    x = f['x']
    sd = SecondDerivative(size=N, shape=SHAPE, axis=1, step=0.5, edge=True)
    assert rel(sd(x), f['d2_fwd']) < 1e-14 and rel(sd.adjoint(x), f['d2_adj']) < 1e-14
    sd0 = SecondDerivative(size=N, shape=SHAPE, axis=0, edge=False)
    assert rel(sd0(x), f['d2ax0_fwd']) < 1e-14 and rel(sd0.adjoint(x), f['d2ax0_adj']) < 1e-14
    gl = GeneralisedLaplacian(shape=SHAPE, kind='sobolev', order=2, constant=0.5)
    assert rel(gl(x), f['glap_sob_fwd']) < 1e-13 and rel(gl.adjoint(x), f['glap_sob_adj']) < 1e-13
    gl2 = GeneralisedLaplacian(shape=SHAPE, kind='polynomial', coeffs=[0.5, -1.0, 0.25])
    assert rel(gl2(x), f['glap_pol_fwd']) < 1e-13
    gd = GeneralisedDerivative(size=N, shape=SHAPE, axis=1, kind_op='exponential', order=2, constant=-0.1,
                               kind_diff='forward')
    assert rel(gd(x), f['gder_exp_fwd']) < 1e-13 and rel(gd.adjoint(x), f['gder_exp_adj']) < 1e-13
    pl = PolynomialLinearOperator(LinOp=DenseLinearOperator(f['Asq']), coeffs=[1.0, -0.5, 2.0])
    assert rel(pl(x), f['poly_fwd']) < 1e-13 and rel(pl.adjoint(x), f['poly_adj']) < 1e-13


def test_moving_averages(f):
    from pycsou_amd.linop import MovingAverage1D, MovingAverage2D
    x = f['x']
    ma1 = MovingAverage1D(window_size=4, shape=SHAPE, axis=0)
    assert rel(ma1(x), f['ma1_fwd']) < 1e-13 and rel(ma1.adjoint(x), f['ma1_adj']) < 1e-13
    ma2 = MovingAverage2D(window_shape=(3, 6), shape=SHAPE)
    assert rel(ma2(x), f['ma2_fwd']) < 1e-13 and rel(ma2.adjoint(x), f['ma2_adj']) < 1e-13


def _inpaint_ops(g):
    from pycsou_amd.linop import Gradient, Masking
    shape = tuple(int(s) for s in g['shape'])
    n = int(np.prod(shape))
    Gop = Masking(size=n, sampling_bool=g['mask'])
    Gop.lipschitz_cst = Gop.diff_lipschitz_cst = 1.0
    D = Gradient(shape=shape, kind='forward')
    D.lipschitz_cst = D.diff_lipschitz_cst = np.sqrt(8.0)
    return n, Gop, D


@pytest.mark.parametrize('tag', ['fixed', 'stop'])
def test_cps_inpainting_notebook(tag):
    """Notebook cell [62]: K = LinOpVStack(Masking, Gradient), H = ProxFuncHStack(L1Loss, mu L1Norm),
    G = Segment, CPS (generic device path: one kernel per operator)."""
    from pycsou_amd.func import L1Loss, L1Norm, ProxFuncHStack, Segment
    from pycsou_amd.linop import LinOpVStack
    from pycsou_amd.opt import CPS
    g = load('cps_inpaint.npz')
    n, Gop, D = _inpaint_ops(g)
    y, mu = g['y'], float(g['mu'])
    H = ProxFuncHStack(L1Loss(dim=y.size, data=y), mu * L1Norm(dim=D.shape[0]))
    K = LinOpVStack(Gop, D)
    p = tag + '_'
    assert K.lipschitz_cst == pytest.approx(float(g[p + 'Klip']), rel=1e-15)
    cps = CPS(dim=n, G=Segment(dim=n, a=0, b=1), H=H, K=K, max_iter=int(g[p + 'max_iter']),
              min_iter=int(g[p + 'min_iter']), accuracy_threshold=float(g[p + 'thr']), verbose=None)
    assert (cps.tau, cps.sigma, cps.rho) == (float(g[p + 'tau']), float(g[p + 'sigma']), float(g[p + 'rho']))
    est, _, diag = cps.iterate()
    assert cps.iter == int(g[p + 'n_iter'])
    assert rel(est['primal_variable'], g[p + 'x']) < 1e-9
    assert rel(est['dual_variable'], g[p + 'z']) < 1e-9
    np.testing.assert_allclose(diag['Relative Improvement (primal variable)'].to_numpy(float)[1:],
                               g[p + 'diag_primal'][1:], rtol=1e-7)


def test_apgd_tikhonov_notebook():
    """Notebook cell [55]: F = 1/2 ||Masking x - y||^2 + mu/2 ||D x||^2 (a DiffMapSum), G = Segment."""
    from pycsou_amd.func import Segment, SquaredL2Loss, SquaredL2Norm
    from pycsou_amd.opt import APGD
    g = load('apgd_tikhonov.npz')
    n, Gop, D = _inpaint_ops(g)
    y, mu = g['y'], float(g['mu'])
    F = ((1 / 2) * SquaredL2Loss(dim=y.size, data=y) * Gop) + ((mu / 2) * SquaredL2Norm(dim=D.shape[0]) * D)
    apgd = APGD(dim=n, F=F, G=Segment(dim=n, a=0, b=1), max_iter=59, min_iter=59, accuracy_threshold=0.0,
                verbose=None)
    assert apgd.beta == pytest.approx(float(g['beta']), rel=1e-15)
    est, _, diag = apgd.iterate()
    assert apgd.iter == int(g['n_iter'])
    assert rel(est['iterand'], g['x']) < 1e-9


def _inpaint_problem(shape, seed, dtype, kind='forward', hname='l1'):
    from pycsou_amd.func import L1Loss, L1Norm, L21Norm, ProxFuncHStack, Segment
    from pycsou_amd.linop import Gradient, LinOpVStack, Masking
    rng = np.random.default_rng(seed)
    n = int(np.prod(shape))
    mask = rng.random(n) < 0.4
    img = np.clip(OR.phantom(shape, seed=seed).ravel() + 0.05 * rng.standard_normal(n), 0, 1)
    y = img[mask].astype(dtype)
    Gop = Masking(size=n, sampling_bool=mask)
    D = Gradient(shape=shape, kind=kind)
    mu = 0.6
    Hs = mu * (L21Norm(dim=2 * n, groups=np.tile(np.arange(n), 2)) if hname == 'l21' else L1Norm(dim=2 * n))
    H = ProxFuncHStack(L1Loss(dim=int(mask.sum()), data=y), Hs)
    K = LinOpVStack(Gop, D)
    K.lipschitz_cst = K.diff_lipschitz_cst = float(np.sqrt(1.0 + 8.0))
    return n, mask, y, mu, K, H, Segment(dim=n, a=0, b=1)


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
@pytest.mark.parametrize('shape,thr,kind,hname', [((130, 200), 0.0, 'forward', 'l1'), ((257, 388), 1e-3, 'forward', 'l1'),
                                                  ((96, 132), 0.0, 'centered', 'l21')])
def test_cps_inpainting_fused_vs_oracle(dtype, shape, thr, kind, hname):
    """The notebook's CPS TV-LAD inpainting (K = [Masking; Gradient], H = L1Loss (+) mu L1Norm, G =
    Segment) on images the row march covers: ONE launch per iteration (the masked block inside the
    general-stencil march, PCS_M_L1LOSS) against the oracle -- fp64 to 1e-9, fp32 to 5e-5, the same
    iteration count (a natural stop included), the dual variable in the reference's [z_m; z_s] layout."""
    from oracle import pycsou_ref as O
    from pycsou_amd.opt import CPS
    from pycsou_amd.opt.engine import PDS2DMaskEngine
    n, mask, y, mu, K, H, G = _inpaint_problem(shape, 3, dtype, kind, hname)
    max_iter = 30
    m = int(mask.sum())
    cps = CPS(dim=n, G=G, H=H, K=K, x0=np.zeros(n, dtype), z0=np.zeros(m + 2 * n, dtype), max_iter=max_iter,
              min_iter=5 if thr > 0 else max_iter, accuracy_threshold=thr, verbose=None)
    est, _, diag = cps.iterate()
    assert isinstance(cps._engine, PDS2DMaskEngine), 'the masked fused step must take this problem'
    assert est['primal_variable'].dtype == dtype
    # oracle (tests/cases.py oracle_cps_inpaint semantics; the reference's op sequence)
    from oracle import pylops1 as P
    D = P.Gradient(shape, sampling=1., edge=True, kind=kind)
    m = int(mask.sum())
    yd = y.astype(np.float64)

    def Kf(x):
        return np.concatenate([x[mask], D.matvec(x)])

    def KT(z):
        xa = np.zeros(n)
        xa[mask] = z[:m]
        return 0 + xa + D.rmatvec(z[m:])

    if hname == 'l21':
        hs = O.postcomp(lambda v, t: O.prox_l21_pixel(v, t, 2), mu)
    else:
        hs = O.postcomp(O.prox_l1, mu)

    def hprox(v, t):
        return np.concatenate([O.prox_l1(v[:m] + (-yd), t) - (-yd), hs(v[m:], t)])

    xr, zr, dr = O.pds(lambda x: np.zeros_like(x), lambda v, t: O.proj_segment(v, 0.0, 1.0), Kf, KT,
                       lambda w, s: O.fenchel_prox(hprox, w, s), cps.tau, cps.sigma, cps.rho, np.zeros(n),
                       np.zeros(m + 2 * n), max_iter=max_iter, min_iter=5 if thr > 0 else max_iter,
                       accuracy_threshold=thr)
    tol = 1e-9 if dtype == np.float64 else 5e-5
    assert cps.iter == len(dr['primal']), (cps.iter, len(dr['primal']))
    assert est['dual_variable'].shape == (m + 2 * n,)
    assert rel(est['primal_variable'], xr) < tol, rel(est['primal_variable'], xr)
    assert rel(est['dual_variable'], zr) < tol, rel(est['dual_variable'], zr)
    np.testing.assert_allclose(diag['Relative Improvement (primal variable)'].to_numpy(float)[1:], dr['primal'][1:],
                               rtol=1e-7 if dtype == np.float64 else 1e-3)
    np.testing.assert_allclose(diag['Relative Improvement (dual variable)'].to_numpy(float)[1:], dr['dual'][1:],
                               rtol=1e-7 if dtype == np.float64 else 1e-3)


def test_cps_inpainting_fused_vs_generic():
    """The fused masked step against the generic per-operator path on the same fp64 problem:
    iterates to 1e-12 (operation order only)."""
    from pycsou_amd.opt import CPS
    out = {}
    for mode in ('fused', 'generic'):
        n, mask, y, mu, K, H, G = _inpaint_problem((200, 256), 8, np.float64)
        cps = CPS(dim=n, G=G, H=H, K=K, max_iter=19, min_iter=19, accuracy_threshold=0.0, verbose=None)
        cps.engine_mode = mode
        est, _, _ = cps.iterate()
        assert (cps._engine is not None) == (mode == 'fused')
        out[mode] = est
    assert rel(out['fused']['primal_variable'], out['generic']['primal_variable']) < 1e-12
    assert rel(out['fused']['dual_variable'], out['generic']['dual_variable']) < 1e-12

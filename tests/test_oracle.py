"""Pin the CPU oracle (oracle/) against the golden vectors of the real reference.

CPU only.  These tests are what makes the oracle trustworthy as the checker of
the HIP path (tests/test_gpu_*.py).
"""

import numpy as np
import pytest
from scipy import signal

from oracle import pylops1 as P
from oracle import pycsou_ref as O
from tests.cases import load, oracle_pds, pds_case, pds_case_names, rel


# ---------------------------------------------------------------- prox / functionals

def test_prox_against_reference():
    f = load('prox.npz')
    x, vz, groups = f['x'], f['vz'], f['groups']
    np.testing.assert_allclose(O.prox_l1(x.copy(), 0.7), f['l1_prox_07'], rtol=0, atol=1e-15)
    np.testing.assert_allclose(O.prox_l2(x.copy(), 3.0), f['l2_prox_3'], rtol=1e-14, atol=1e-15)
    np.testing.assert_allclose(O.prox_l2(x.copy(), 30.0), f['l2_prox_30'], rtol=0, atol=1e-15)
    np.testing.assert_allclose(O.prox_l21(x.copy(), 0.5, groups), f['l21_prox_05'], rtol=1e-14, atol=1e-15)
    np.testing.assert_allclose(O.prox_l21_pixel(vz.copy(), 0.5, 2), f['l21pix_prox_05'], rtol=1e-14, atol=1e-15)
    np.testing.assert_allclose(O.l21_value_pixel(vz, 2), f['l21pix_value'], rtol=1e-14)
    fen1 = O.fenchel_prox(O.postcomp(O.prox_l1, 0.3), x.copy(), 0.7)
    np.testing.assert_allclose(fen1, f['fenchel_l1_lam03_s07'], rtol=0, atol=1e-15)
    fen21 = O.fenchel_prox(O.postcomp(lambda v, t: O.prox_l21_pixel(v, t, 2), 0.3), vz.copy(), 0.7)
    np.testing.assert_allclose(fen21, f['fenchel_l21pix_lam03_s07'], rtol=1e-14, atol=1e-15)
    np.testing.assert_allclose(2 * x, f['sql2_grad'], rtol=0, atol=0)
    np.testing.assert_allclose(O.proj_nonnegative_orthant(x.copy()), f['nonneg'], rtol=0, atol=0)
    np.testing.assert_allclose(O.proj_segment(x.copy(), -0.5, 0.25), f['segment'], rtol=0, atol=0)
    # exact-arithmetic identity: fenchel of lam*L1 is the clip to [-lam, lam]
    np.testing.assert_allclose(fen1, np.clip(x, -0.3, 0.3), rtol=0, atol=1e-15)


def test_reference_doctest_values():
    f = load('prox.npz')
    assert float(f['doc_l1_arange']) == 45.0                      # penalty.py:207-218
    assert float(f['doc_l2_arange']) == 16.881943016134134        # penalty.py:35-46
    assert float(f['doc_l21_arange']) == 21.44594499772297        # penalty.py:494-509
    assert float(f['doc_sql2_arange']) == 285.00000000000006      # penalty.py:88-103
    np.testing.assert_array_equal(f['doc_soft'], [-0.5, -0., 0., 0., 0.5])  # prox.py:51-58
    np.testing.assert_array_equal(O.soft(np.linspace(-1, 1, 5), 0.5), f['doc_soft'])


# ---------------------------------------------------------------- PyLops-boundary operators

def test_convolve2d_doctest():
    f = load('ops.npz')
    h = f['doc_conv2d_h']
    op = P.Convolve2D(10000, h, (100, 100), offset=(P.pycsou_offset(25), P.pycsou_offset(25)))
    np.testing.assert_allclose(op.matvec(f['doc_conv2d_x']), f['doc_conv2d_y'], atol=1e-12)  # conv.py:209-217


def test_convolve1d_doctest():
    f = load('ops.npz')
    h = f['doc_conv1d_h']
    op = P.Convolve1D(30, h, offset=P.pycsou_offset(h.size))
    np.testing.assert_allclose(op.matvec(f['doc_conv1d_x']), f['doc_conv1d_y'], atol=1e-14)  # conv.py:67-73


def test_first_derivative_doctest():
    f = load('ops.npz')
    x = f['doc_d1_x']
    y = P.FirstDerivative(x.size, kind='forward', edge=True).matvec(x)
    assert np.sum(np.abs(y) > 0) == 6                                # diff.py:72-78
    np.testing.assert_allclose(y, f['doc_d1_y'])


def test_gradient_consistency_doctest():
    g = np.linspace(-2.5, 2.5, 37)
    X, Y = np.meshgrid(g, g[:31])
    Z = np.sin(X) * np.cos(2 * Y) + X * Y
    G = P.Gradient(Z.shape, kind='forward', edge=True)
    D = P.FirstDerivative(Z.size, dims=Z.shape, dir=0, kind='forward', edge=True)
    np.testing.assert_allclose(G.matvec(Z.ravel())[:Z.size], D.matvec(Z.ravel()))  # diff.py:814-820


def _dot_test(op, n, m, rng, dtype=np.float64):
    u = rng.standard_normal(n).astype(dtype)
    v = rng.standard_normal(m).astype(dtype)
    a = np.dot(op.matvec(u), v)
    b = np.dot(u, op.rmatvec(v))
    assert abs(a - b) <= 1e-10 * max(abs(a), abs(b), 1.0)


@pytest.mark.parametrize('shape', [(17,), (8, 9), (5, 6, 7), (3, 4, 5, 6)])
@pytest.mark.parametrize('kind', ['forward', 'backward', 'centered'])
@pytest.mark.parametrize('edge', [True, False])
def test_gradient_adjoint(shape, kind, edge):
    rng = np.random.default_rng(0)
    G = P.Gradient(shape, sampling=[0.5 + i for i in range(len(shape))], edge=edge, kind=kind)
    _dot_test(G, G.shape[1], G.shape[0], rng)


@pytest.mark.parametrize('edge', [True, False])
def test_laplacian_adjoint(edge):
    rng = np.random.default_rng(1)
    L = P.Laplacian((11, 13), weights=(1.0, 0.5), sampling=(1.0, 2.0), edge=edge)
    _dot_test(L, L.shape[1], L.shape[0], rng)


@pytest.mark.parametrize('kshape', [(15, 15), (4, 6), (7, 4), (1, 5), (9, 1)])
def test_convolve2d_adjoint_and_same(kshape):
    rng = np.random.default_rng(2)
    shape = (23, 31)
    h = rng.standard_normal(kshape)
    off = tuple(P.pycsou_offset(n) for n in kshape)
    C = P.Convolve2D(int(np.prod(shape)), h, shape, offset=off)
    _dot_test(C, C.shape[1], C.shape[0], rng)
    x = rng.standard_normal(shape)
    # direct definition: y[i] = sum_j h[j] x[i + off - j]
    y = np.zeros(shape)
    for j0 in range(kshape[0]):
        for j1 in range(kshape[1]):
            s0, s1 = off[0] - j0, off[1] - j1
            src = np.zeros(shape)
            a0, b0 = max(0, -s0), min(shape[0], shape[0] - s0)
            a1, b1 = max(0, -s1), min(shape[1], shape[1] - s1)
            src[a0:b0, a1:b1] = x[a0 + s0:b0 + s0, a1 + s1:b1 + s1]
            y += h[j0, j1] * src
    np.testing.assert_allclose(C.matvec(x.ravel()), y.ravel(), atol=1e-12)
    if kshape[0] % 2 and kshape[1] % 2:
        np.testing.assert_allclose(C.matvec(x.ravel()), signal.convolve(x, h, mode='same').ravel(), atol=1e-12)


@pytest.mark.parametrize('axis', [0, 1, 2])
def test_convolve1d_axis_adjoint(axis):
    rng = np.random.default_rng(3)
    dims = (6, 7, 8)
    h = rng.standard_normal(5)
    C = P.Convolve1D(int(np.prod(dims)), h, offset=2, dims=dims, dir=axis)
    _dot_test(C, C.shape[1], C.shape[0], rng)


# ---------------------------------------------------------------- solver loops

@pytest.mark.parametrize('name', pds_case_names())
def test_oracle_pds_matches_reference(name):
    c = pds_case(name)
    x, z, diag = oracle_pds(c)
    assert diag['n_iter'] == int(c['n_iter'])
    assert rel(x, c['x']) < 1e-11
    assert rel(z, c['z']) < 1e-11
    np.testing.assert_allclose(diag['primal'], c['diag_primal'], rtol=1e-9)
    np.testing.assert_allclose(diag['dual'], c['diag_dual'], rtol=1e-9)
    assert bool(c['converged'])


def test_step_sizes_against_reference():
    for name in pds_case_names():
        c = pds_case(name)
        d = len(c['shape'])
        Klip = 8.0 if c['meta']['kind'] == 'lap' else np.sqrt(4.0 * d)
        tau, sigma = O.pds_step_sizes(float(c['beta']), Klip)
        assert tau == float(c['tau']) and sigma == float(c['sigma'])
        assert O.pds_momentum(float(c['beta'])) == float(c['rho'])


@pytest.mark.parametrize('acc', ['CD', 'BT', 'none'])
@pytest.mark.parametrize('mode', ['fixed', 'stop'])
def test_oracle_apgd_matches_reference(acc, mode):
    f = load('apgd_lasso.npz')
    A, y, lam = f['A'], f['y'], float(f['lam'])
    p = f'{acc}_{mode}_'
    tau = float(f[p + 'tau'])
    assert tau == 1 / float(f[p + 'beta'])
    grad = lambda x: A.T.dot((2 * (A.dot(x) + (-y))) * 0.5)  # noqa: E731
    x, it, diag = O.apgd(grad, O.postcomp(O.prox_l1, lam), tau, np.zeros(512),
                         acceleration=None if acc == 'none' else acc, max_iter=int(f[p + 'max_iter']),
                         min_iter=int(f[p + 'min_iter']), accuracy_threshold=float(f[p + 'thr']))
    assert diag['n_iter'] == int(f[p + 'n_iter'])
    assert rel(x, f[p + 'x']) < 1e-11
    assert rel(it['past_aux'], f[p + 'past_aux']) < 1e-11
    np.testing.assert_allclose(diag['hist'], f[p + 'diag'], rtol=1e-8)

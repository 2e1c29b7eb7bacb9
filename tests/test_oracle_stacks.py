"""Pin the oracle restatements of the widened operator set against
the golden vectors of the real reference (tests/golden/make_golden_stacks.py).  CPU only."""

import numpy as np

from oracle import pylops1 as P
from oracle import pycsou_ref as O
from tests.cases import load, oracle_cps_inpaint, rel

SHAPE = (12, 9)
N = 108


def test_stacks_restated():
    f = load('stacks.npz')
    x, w = f['x'], f['w']
    D1 = P.FirstDerivative(N, dims=SHAPE, dir=0, sampling=1., edge=True, kind='centered')
    D2 = P.FirstDerivative(N, dims=SHAPE, dir=1, sampling=1., edge=True, kind='forward')
    np.testing.assert_array_equal(np.concatenate([D1.matvec(x), D2.matvec(x)]), f['vstack_fwd'])
    np.testing.assert_allclose(0 + D1.rmatvec(w[:N]) + D2.rmatvec(w[N:]), f['vstack_adj'], rtol=0, atol=1e-14)
    np.testing.assert_allclose(0 + D1.rmatvec(w[:N]) + D2.rmatvec(w[N:]), f['hstack_fwd'], rtol=0, atol=1e-14)
    np.testing.assert_array_equal(np.concatenate([D1.matvec(x), D2.matvec(x)]), f['hstack_adj'])
    A = f['A']
    np.testing.assert_allclose(np.concatenate([A @ x, D2.matvec(x)]), f['vstack2_fwd'], rtol=1e-14)


def test_functional_stacks_restated():
    f = load('stacks.npz')
    z, yd = f['z'], f['yd']
    a, b = z[:N], z[N:]
    assert abs(float(f['phs_value']) - (np.abs(a).sum() + 0.7 * np.linalg.norm(b))) < 1e-12
    np.testing.assert_allclose(np.concatenate([O.prox_l1(a, 0.3), O.prox_l2(b, 0.3 * 0.7)]), f['phs_prox_03'],
                               rtol=1e-14, atol=1e-15)

    def hprox(v, t):
        return np.concatenate([O.prox_l1(v[:N], t), O.prox_l2(v[N:], t * 0.7)])

    np.testing.assert_allclose(O.fenchel_prox(hprox, z, 0.5), f['phs_fenchel_05'], rtol=1e-14, atol=1e-15)

    def hprox2(v, t):
        return np.concatenate([O.prox_l1(v[:N] + (-yd), t) - (-yd), O.prox_l1(v[N:], t * 0.6)])

    np.testing.assert_allclose(hprox2(z, 0.4), f['phs2_prox_04'], rtol=0, atol=1e-15)
    np.testing.assert_allclose(O.fenchel_prox(hprox2, z, 0.7), f['phs2_fenchel_07'], rtol=0, atol=1e-14)
    np.testing.assert_allclose(np.concatenate([2 * a, (2 * (b + (-yd)))]), f['dhs_grad'], rtol=1e-15)


def test_sampling_restated():
    f = load('stacks.npz')
    x, mask = f['x'], f['mask']
    np.testing.assert_array_equal(x[mask], f['mask_fwd'])
    back = np.zeros(N)
    back[mask] = x[mask]
    np.testing.assert_array_equal(back, f['mask_adj'])
    np.testing.assert_array_equal(x.reshape(SHAPE)[::3, ::2].ravel(), f['down_fwd'])
    assert tuple(f['down_shape']) == (4, 5)
    np.testing.assert_array_equal(x.reshape(SHAPE)[:, ::2].ravel(), f['downax_fwd'])
    R = P.Restriction(N, f['iava'], dims=SHAPE, dir=0)
    np.testing.assert_array_equal(R.matvec(x), f['sub_fwd'])
    np.testing.assert_array_equal(R.rmatvec(R.matvec(x)), f['sub_adj'])


def test_cps_inpaint_oracle():
    f = load('cps_inpaint.npz')
    for tag in ('fixed', 'stop'):
        x, z, diag = oracle_cps_inpaint(f, tag)
        assert diag['n_iter'] == int(f[tag + '_n_iter'])
        assert rel(x, f[tag + '_x']) < 1e-11
        assert rel(z, f[tag + '_z']) < 1e-11
        np.testing.assert_allclose(diag['primal'], f[tag + '_diag_primal'], rtol=1e-8)
    assert int(f['stop_n_iter']) < 500  # the stopping rule fired


def test_apgd_tikhonov_oracle():
    f = load('apgd_tikhonov.npz')
    shape = tuple(int(s) for s in f['shape'])
    mask, y, mu = f['mask'], f['y'], float(f['mu'])
    n = int(np.prod(shape))
    D = P.Gradient(shape, sampling=1., edge=True, kind='forward')

    def grad(x):
        g1 = np.zeros(n)
        g1[mask] = (2 * (x[mask] + (-y))) * 0.5
        return g1 + D.rmatvec((2 * D.matvec(x)) * (mu / 2))

    assert abs(float(f['beta']) - 1.1) < 1e-12
    x, _, diag = O.apgd(grad, lambda v, t: O.proj_segment(v, 0.0, 1.0), float(f['tau']), np.zeros(n),
                        acceleration='CD', max_iter=59, min_iter=59, accuracy_threshold=0.0)
    assert diag['n_iter'] == int(f['n_iter'])
    assert rel(x, f['x']) < 1e-11
    np.testing.assert_allclose(diag['hist'], f['diag'], rtol=1e-8)

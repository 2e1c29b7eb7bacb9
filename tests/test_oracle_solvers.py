"""The oracle restatement (oracle/pycsou_ref.py, oracle/pylops1.py) against the real
reference's DRS / FBS / default-K / diagonal-K trajectories (tests/golden/solvers.npz): pins
the oracle for these parameterisations (proxalgs.py:719-862, linop/base.py:551-622).  CPU only."""

import numpy as np

from oracle import pycsou_ref as OR
from tests.cases import load, rel


def _g():
    return load('solvers.npz')


def test_oracle_drs():
    g = _g()
    y = g['drs_y']
    N = y.size
    # G = 0.3 L1(. - y): prox(v, t) = y + prox_{0.3 t L1}(v - y);  H = 0.2 L2, K = I
    prox_g = OR.postcomp(lambda v, t: y + OR.prox_l1(v - y, t), 0.3)
    h = OR.postcomp(OR.prox_l2, 0.2)
    for tag in ('drs_fixed', 'drs_stop'):
        tau = float(g[f'{tag}_tau'])
        x, z, d = OR.pds(lambda v: np.zeros_like(v), prox_g, lambda v: v, lambda v: v,
                         lambda w, s: OR.fenchel_prox(h, w, s), tau, 1 / tau, 1, np.zeros(N), np.zeros(N),
                         max_iter=int(g[f'{tag}_max_iter']), min_iter=int(g[f'{tag}_min_iter']),
                         accuracy_threshold=float(g[f'{tag}_thr']))
        assert len(d['primal']) == int(g[f'{tag}_n_iter'])
        assert rel(x, g[f'{tag}_x']) < 1e-12 and rel(z, g[f'{tag}_z']) < 1e-12
        np.testing.assert_allclose(d['primal'], g[f'{tag}_diag_primal'], rtol=1e-10)


def test_oracle_fbs_dense():
    g = _g()
    A, y, lam = g['fbs_dense_A'], g['fbs_dense_y'], float(g['fbs_dense_lam'])
    beta = float(g['fbs_dense_Alip']) ** 2
    tau, _ = OR.pds_step_sizes(beta, 0.0, has_H=False)
    assert tau == float(g['fbs_dense_tau'])
    n = A.shape[1]  # H = None: K = NullOperator, K^T z = 0 (linop/base.py:601-622), z stays None
    x, z, d = OR.pds(lambda v: A.T @ ((2 * (A @ v + (-y))) * 0.5), OR.postcomp(OR.prox_l1, lam), None,
                     lambda zz: np.zeros(n), None,
                     tau, 0, 1, np.zeros(A.shape[1]), None, max_iter=39, min_iter=39, accuracy_threshold=0.0,
                     has_H=False)
    assert rel(x, g['fbs_dense_x']) < 1e-12
    np.testing.assert_allclose(d['primal'], g['fbs_dense_diag_primal'], rtol=1e-10)


def test_oracle_pds_identity_and_diagonal():
    g = _g()
    y, dvec = g['pds_k_y'], g['pds_k_dvec']
    N = y.size
    h = OR.postcomp(OR.prox_l1, 0.1)
    for tag, dk in (('pds_kid', np.ones(N)), ('pds_kdiag', dvec)):
        klip = float(g[f'{tag}_Klip'])
        assert klip == (1 if tag == 'pds_kid' else np.max(dvec))
        tau, sigma = OR.pds_step_sizes(1.0, klip)
        assert (tau, sigma) == (float(g[f'{tag}_tau']), float(g[f'{tag}_sigma']))
        x, z, d = OR.pds(lambda v: (2 * (v + (-y))) * 0.5, lambda v, t: v, lambda v: dk * v, lambda v: dk * v,
                         lambda w, s: OR.fenchel_prox(h, w, s), tau, sigma, OR.pds_momentum(1.0), np.zeros(N),
                         np.zeros(N), max_iter=24, min_iter=24, accuracy_threshold=0.0)
        assert rel(x, g[f'{tag}_x']) < 1e-12 and rel(z, g[f'{tag}_z']) < 1e-12

"""The generic (operator-by-operator) PDS loop as hipGraph chunks against the same loop launched
eagerly (PCS_GENERIC_GRAPH=0): the captured chunks issue the same kernels in the same order, so
x, z, the iteration count and every diagnostics row are bitwise equal -- for fixed counts that end
inside a chunk, natural stops, both dtypes, a general-label L21Norm, a ProxFuncHStack H and a
primal-only problem; the verbose lines match too.

Reference: the loop of pycsou/core/solver.py:55-76 with PrimalDualSplitting.update_iterand,
pycsou/opt/proxalgs.py:343-355; L21Norm labels pycsou/func/penalty.py:525-560, ProxFuncHStack
pycsou/func/base.py:21-89.
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _problem(name, n, dtype, max_iter, min_iter, thr, verbose=None):
    from pycsou_amd.func import L1Norm, ProxFuncHStack
    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L21Norm
    from pycsou_amd.linop import Gradient
    from pycsou_amd.opt import PDS
    N = n * n
    rng = np.random.default_rng(11)
    img = np.zeros((n, n))
    img[n // 4:3 * n // 4, n // 3:2 * n // 3] = 1.0
    npdt = np.float32 if dtype == torch.float32 else np.float64
    y = torch.from_numpy((img.ravel() + 0.1 * rng.standard_normal(N)).astype(npdt)).cuda()
    F = (1 / 2) * SquaredL2Loss(dim=N, data=y)
    if name == 'primal_only':
        return PDS(dim=N, F=F, G=0.05 * L1Norm(dim=N), x0=torch.zeros(N, dtype=dtype, device='cuda'),
                   max_iter=max_iter, min_iter=min_iter, accuracy_threshold=thr, verbose=verbose, engine='generic')
    K = Gradient(shape=(n, n), kind='forward')
    K.lipschitz_cst = K.diff_lipschitz_cst = float(np.sqrt(8.0))
    if name == 'l21_labels':
        lab = np.arange(N) // 2
        H = 0.1 * L21Norm(dim=2 * N, groups=np.concatenate([lab, lab]))
    else:
        H = ProxFuncHStack(0.1 * L1Norm(dim=N), 0.1 * L1Norm(dim=N))
    return PDS(dim=N, F=F, H=H, K=K, x0=torch.zeros(N, dtype=dtype, device='cuda'),
               z0=torch.zeros(2 * N, dtype=dtype, device='cuda'), max_iter=max_iter, min_iter=min_iter,
               accuracy_threshold=thr, verbose=verbose, engine='generic')


def _run(monkeypatch, graph, *args, **kw):
    monkeypatch.setenv('PCS_GENERIC_GRAPH', '1' if graph else '0')
    pds = _problem(*args, **kw)
    est, _, diag = pds.iterate()
    return pds, est, diag


def _same(a, b):
    (pa, ea, da), (pb, eb, db) = a, b
    assert pa.iter == pb.iter
    for k in ea:
        if ea[k] is None:
            assert eb[k] is None
        else:
            assert torch.equal(ea[k], eb[k]), k
    assert list(da.columns) == list(db.columns)
    for c in da.columns:
        np.testing.assert_array_equal(da[c].to_numpy(float), db[c].to_numpy(float))


@pytest.mark.parametrize('name,dtype', [('l21_labels', torch.float32), ('l21_labels', torch.float64),
                                        ('stack_h', torch.float32), ('primal_only', torch.float64)])
@pytest.mark.parametrize('stop', ['fixed_11', 'fixed_16', 'natural'])
def test_generic_graph_bitwise_eager(monkeypatch, name, dtype, stop):
    if stop == 'natural':
        args = (name, 64, dtype, 500, 3, 2e-3)
    else:  # max_iter = min_iter = m runs m + 1 iterations (solver.py:65-66): 11 ends inside a chunk of 4
        m = int(stop.split('_')[1]) - 1
        args = (name, 64, dtype, m, m, 1e-3)
    g = _run(monkeypatch, True, *args)
    e = _run(monkeypatch, False, *args)
    assert getattr(g[0], '_graph_used', False) and not getattr(e[0], '_graph_used', False)
    _same(g, e)
    if stop == 'natural':
        assert 3 < g[0].iter < 500
    else:
        assert g[0].iter == int(stop.split('_')[1])


def test_generic_graph_verbose_lines(monkeypatch, capsys):
    _run(monkeypatch, True, 'l21_labels', 32, torch.float64, 500, 3, 1e-3, verbose=5)
    out_g = capsys.readouterr().out
    _run(monkeypatch, False, 'l21_labels', 32, torch.float64, 500, 3, 1e-3, verbose=5)
    out_e = capsys.readouterr().out
    assert out_g == out_e and out_g.count('\n') >= 2

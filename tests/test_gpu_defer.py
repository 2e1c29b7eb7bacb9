"""Deferred finalization (pcs_pds2d_args.fin_partials, csrc/pds_ctrl.hpp) against the in-launch
reduction (PCS_DEFER_FIN=0) on every 2-D step-kernel family: the same iteration count, bitwise the same
primal and dual iterates, the diagnostics to 1e-12 relative (the two sum the fp64 partials in different
orders).  Loop endings covered: a fixed count ending on a chunk boundary (the last launch's partials are
finalized by pcs_pds_finalize_pending after the loop), and natural stops at an accuracy threshold on the
last launch of a chunk, on the first of the next and in between (the stopping rule of
pycsou/core/solver.py:65-66 then acts one launch later: the extra iterate must never be selected);
hipGraph-replayed images and images launched back to back from C (pcs_pds2d_run)."""

import numpy as np
import pytest
import torch

import pycsou_amd.opt.engine as E

pytestmark = pytest.mark.gpu


def _cps(n, dtype):
    from bench import phantom
    from pycsou_amd.func import L1Loss, L1Norm, ProxFuncHStack, Segment
    from pycsou_amd.linop import Gradient, LinOpVStack, Masking
    from pycsou_amd.opt import CPS
    N = n * n
    rng = np.random.default_rng(5)
    mask = rng.random(N) < 0.5
    img = phantom((n, n), 12, 5).ravel()
    y = torch.from_numpy(img[mask]).to('cuda', dtype)
    m = int(mask.sum())
    M = Masking(size=N, sampling_bool=mask)
    M.lipschitz_cst = M.diff_lipschitz_cst = 1.0
    D = Gradient(shape=(n, n), kind='forward')
    D.lipschitz_cst = D.diff_lipschitz_cst = float(np.sqrt(8.0))
    return CPS(dim=N, G=Segment(dim=N, a=0, b=1), H=ProxFuncHStack(L1Loss(dim=m, data=y), 0.1 * L1Norm(dim=2 * N)),
               K=LinOpVStack(M, D), x0=torch.zeros(N, dtype=dtype, device='cuda'),
               z0=torch.zeros(m + 2 * N, dtype=dtype, device='cuda'), verbose=None)


def _problem(name):
    import bench
    f32, f64 = torch.float32, torch.float64
    table = {
        'pt': lambda: (bench.build_denoise(256, f32, lipschitz='analytic'), f32),
        'pt_native': lambda: (bench.build_denoise(1024, f32, lipschitz='analytic'), f32),
        'tile_f64': lambda: (bench.build_denoise(192, f64, lipschitz='analytic'), f64),
        'nmarch': lambda: (bench.build_problem(200, 256, f32, lipschitz='analytic'), f32),
        'nmarch_cen': lambda: (bench.build_problem(200, 256, f32, lipschitz='analytic', kind='centered'), f32),
        'nm64': lambda: (bench.build_problem(200, 256, f64, lipschitz='analytic'), f64),
        'gradbuf': lambda: (bench.build_problem(160, 192, f32, lipschitz='analytic', psf=bench.aniso_psf()), f32),
        'smarch_lap': lambda: (bench.build_denoise_k(256, f32, 'lap', lipschitz='analytic'), f32),
        'smarch_cen_f64': lambda: (bench.build_denoise_k(256, f64, 'centered', lipschitz='analytic'), f64),
        'mask': lambda: (_cps(256, f32), f32),
    }
    return table[name]()


def _run(pds, dtype, defer, max_iter, min_iter, thr, monkeypatch):
    from pycsou_amd import _ops as O
    monkeypatch.setattr(E, 'DEFER_FIN', defer)
    spec = pds._fused_spec()
    assert spec is not None
    eng = E.engine_class(spec)(spec, dtype, pds.tau, pds.sigma, pds.rho, O.to_dev(pds.x0, dtype),
                               O.to_dev(pds.z0, dtype))
    assert eng.defer == defer, 'every 2-D step-kernel family takes the deferred finalization'
    n, x, z, h = eng.run(max_iter, min_iter, thr)
    torch.cuda.synchronize()
    return n, x.clone(), z.clone(), np.asarray(h), eng


NAMES = ['pt', 'pt_native', 'tile_f64', 'nmarch', 'nmarch_cen', 'nm64', 'gradbuf', 'smarch_lap', 'smarch_cen_f64',
         'mask']


@pytest.mark.parametrize('name', NAMES)
def test_deferred_finalization_matches_inlaunch(name, monkeypatch):
    pds, dtype = _problem(name)
    # fixed count: 64 iterations = two whole chunks of 32 -- no launch after the last iteration
    n0, x0, z0, h0, _ = _run(pds, dtype, False, 63, 63, 0.0, monkeypatch)
    n1, x1, z1, h1, eng = _run(pds, dtype, True, 63, 63, 0.0, monkeypatch)
    assert n0 == n1 == 64
    assert torch.equal(x0, x1) and torch.equal(z0, z1)
    np.testing.assert_allclose(h1, h0, rtol=1e-12)
    assert not np.isnan(h1).any()
    # natural stops: the threshold just above the primal improvement of iteration k0
    rp = h0[:, 0]
    for k0 in (31, 32, 45):
        thr = float(rp[k0]) * (1 + 1e-9)
        k_ref = int(np.argmax(rp <= thr))  # the first iteration the rule stops at (<= k0)
        n0, x0, z0, g0, _ = _run(pds, dtype, False, 500, 0, thr, monkeypatch)
        n1, x1, z1, g1, _ = _run(pds, dtype, True, 500, 0, thr, monkeypatch)
        assert n0 == n1 == k_ref + 1, (k0, k_ref, n0, n1)
        assert torch.equal(x0, x1) and torch.equal(z0, z1), k0
        np.testing.assert_allclose(g1, g0, rtol=1e-12)
    if name == 'pt_native':
        assert eng.native


def test_deferred_fixed_count_advance(monkeypatch):
    """bench.py's fixed-count form (prepare_fixed / advance_fixed with odd counts): every launch is
    finalized by the end of each advance_fixed call, in both modes, with the same diagnostics."""
    pds, dtype = _problem('smarch_lap')
    from pycsou_amd import _ops as O
    out = {}
    for defer in (False, True):
        monkeypatch.setattr(E, 'DEFER_FIN', defer)
        spec = pds._fused_spec()
        eng = E.engine_class(spec)(spec, dtype, pds.tau, pds.sigma, pds.rho, O.to_dev(pds.x0, dtype),
                                   O.to_dev(pds.z0, dtype))
        eng.prepare_fixed(80, 8)
        done = 0
        for n in (5, 16, 1, 30):
            eng.advance_fixed(n)
            done += n
            torch.cuda.synchronize()
            assert int(eng.ctrl.view(torch.int32)[0].item()) == done
        out[defer] = (eng.X[done % 2].clone(), eng.hist[:2 * done].cpu().numpy())
    assert torch.equal(out[False][0], out[True][0])
    np.testing.assert_allclose(out[True][1], out[False][1], rtol=1e-12)

"""Row-slab (multi-GPU) PDS against the single-GPU fused engine and the reference.

Slabs of one image are driven (a) inside one process on one GPU (`run_local`,
device-to-device halos) and (b) by two processes sharing the GPU over a gloo process
group (host-staged halos; the same DistComm code the RCCL path uses, minus the NCCL
calls).  The per-pixel arithmetic does not depend on the slab split, so x and z must be
bitwise identical to the single-GPU engine; the diagnostic sums are added per rank, so
the history agrees to 1e-12 relative and the iteration count exactly.
"""

import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from tests.cases import pds_case, rel
from tests.test_gpu_pds import build

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SLAB_CASES = ['denoise2d_l21_fwd_64', 'denoise2d_l1_fwd_63x65', 'deconv2d_l21_fwd_64_psf15', 'deconv2d_l21_fwd_64_seg',
              'denoise2d_l21_fwd_32_stop']


def _single(c, dtype):
    pds = build(c, dtype, engine='fused')
    est, _, diag = pds.iterate()
    h = pds._engine.hist[:2 * pds.iter].cpu().numpy().reshape(-1, 2)
    return pds.iter, pds._engine.X[pds.iter % 2].clone(), pds._engine.Z[pds.iter % 2].clone(), h


def _slabs(c, dtype, world):
    from pycsou_amd.parallel import SlabPDS2D, run_local
    pds = build(c, dtype, engine='fused')
    slabs = [SlabPDS2D.from_pds(pds, None, rank=r, world=world) for r in range(world)]
    res = run_local(slabs, pds.max_iter, pds.min_iter, pds.accuracy_threshold)
    N = int(np.prod(c['shape']))
    x = torch.cat([r[1] for r in res])
    z = torch.cat([torch.cat([r[2][:r[2].numel() // 2] for r in res]),
                   torch.cat([r[2][r[2].numel() // 2:] for r in res])])
    assert x.numel() == N and z.numel() == 2 * N
    ns = {r[0] for r in res}
    assert len(ns) == 1
    for r in res[1:]:
        np.testing.assert_array_equal(r[3], res[0][3])  # every rank holds the same history
    return res[0][0], x, z, res[0][3]


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
@pytest.mark.parametrize('world', [2, 3])
@pytest.mark.parametrize('name', SLAB_CASES)
def test_slabs_match_single_gpu(name, world, dtype):
    c = pds_case(name)
    n1, x1, z1, h1 = _single(c, dtype)
    n2, x2, z2, h2 = _slabs(c, dtype, world)
    assert n2 == n1 == int(c['n_iter'])
    assert torch.equal(x2, x1), (x2 - x1).abs().max().item()
    assert torch.equal(z2, z1), (z2 - z1).abs().max().item()
    fin = np.isfinite(h1)
    assert np.array_equal(fin, np.isfinite(h2))
    assert np.allclose(h2[fin], h1[fin], rtol=1e-12 if dtype == np.float64 else 1e-5, atol=0)
    tol = 1e-9 if dtype == np.float64 else 5e-5
    assert rel(x2.cpu().numpy(), c['x']) < tol


def test_slab_rejects_thin():
    from pycsou_amd.parallel import SlabPDS2D
    c = pds_case('deconv2d_l21_fwd_64_psf15')
    pds = build(c, np.float64, engine='fused')
    with pytest.raises(ValueError):
        SlabPDS2D.from_pds(pds, None, rank=0, world=8)  # 8 rows < 15-row halo


@pytest.mark.parametrize('shape', [(64, 66), (96, 60)])
def test_slab_rejects_unsupported_kernel(shape):
    """A problem no fused slab kernel takes (centred K on an fp32 image whose rows are not 16-B
    groups, or narrower than two 64-column strips) is a ValueError naming K, dtype and shape --
    not a negative-size allocation."""
    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L21Norm
    from pycsou_amd.linop.diff import Gradient
    from pycsou_amd.opt.proxalgs import PDS
    from pycsou_amd.parallel import SlabPDS2D
    N = shape[0] * shape[1]
    K = Gradient(shape, kind='centered')
    K.lipschitz_cst = K.diff_lipschitz_cst = 2.0
    y = np.random.default_rng(0).uniform(0, 1, N).astype(np.float32)
    pds = PDS(dim=N, F=(1 / 2) * SquaredL2Loss(dim=N, data=y), H=0.1 * L21Norm(dim=2 * N, groups=np.tile(np.arange(N), 2)),
              K=K, x0=np.zeros(N, np.float32), z0=np.zeros(2 * N, np.float32), max_iter=4, min_iter=4,
              accuracy_threshold=0.0, verbose=None)
    with pytest.raises(ValueError, match=r'centered Gradient.*float32'):
        SlabPDS2D.from_pds(pds, None, rank=0, world=2)


def _synth_single_and_slabs(name, world):
    """(single-GPU fused engine result, run_local slabs result) of a slab_worker.SYNTH problem."""
    from pycsou_amd.parallel import SlabPDS2D, run_local
    from tests.slab_worker import synth_problem
    pds = synth_problem(name)
    est, _, _ = pds.iterate()
    eng = pds._engine
    n1 = pds.iter
    x1, z1 = eng.X[n1 % 2].clone(), eng.Z[n1 % 2].clone()
    h1 = eng.hist[:2 * n1].cpu().numpy().reshape(-1, 2)
    pds2 = synth_problem(name)
    slabs = [SlabPDS2D.from_pds(pds2, None, rank=r, world=world) for r in range(world)]
    res = run_local(slabs, pds2.max_iter, pds2.min_iter, pds2.accuracy_threshold)
    nc = slabs[0].ncomp
    x2 = torch.cat([r[1] for r in res])
    z2 = torch.cat([torch.cat([r[2].view(nc, -1)[c] for r in res]) for c in range(nc)])
    return (n1, x1, z1, h1), (res[0][0], x2, z2, res[0][3]), slabs


@pytest.mark.parametrize('world', [2, 3])
@pytest.mark.parametrize('name', ['cen_denoise_f32', 'lap_denoise_f32', 'bwd_denoise_f32', 'nonsep_fwd_f64',
                                  'nonsep_fwd_f32', 'nonsep_cen_f32', 'sep_cen_f32', 'sep_cen_f64', 'sep_fwd_f64'])
def test_slabs_general_k_and_conv_bitwise(name, world):
    """Row slabs of the general-stencil K (backward / centred Gradient, Laplacian: pds_smarch.hpp),
    of a non-separable PSF (grad F by two correlation passes over the stored rows inside the step,
    PCS_F_CONV2D) and of a separable PSF with a centred K (N x over the stored rows, then the
    march step): x and z bitwise equal to the single-GPU engine, same iteration count."""
    (n1, x1, z1, h1), (n2, x2, z2, h2), slabs = _synth_single_and_slabs(name, world)
    assert n2 == n1 == 16
    assert {s.mode for s in slabs} == {'conv2d' if 'nonsep' in name else 'sep' if name == 'sep_fwd_f64'
                                        else 'sep_normal' if 'sep_' in name else 'pointwise'}
    assert torch.equal(x2, x1), (x2 - x1).abs().max().item()
    assert torch.equal(z2, z1), (z2 - z1).abs().max().item()
    assert np.allclose(h2[1:], h1[1:], rtol=1e-5)
    if name in ('sep_cen_f32', 'sep_cen_f64', 'sep_fwd_f64'):  # the fused normal-operator march on the slabs too
        assert all(s.nm_fused for s in slabs)


@pytest.mark.parametrize('name', ['sep_cen_f32', 'sep_cen_f64', 'sep_fwd_f64'])
def test_slab_fused_normal_march_banded_bitwise(name):
    """Separable PSF on the fused normal-operator march (fp32 centred K: pds_nmarch.hpp; fp64 centred /
    forward K: pds_nm64.hip): the banded (boundary bands, then interior) order on two slabs, bitwise the
    single-GPU engine."""
    from pycsou_amd.parallel import SlabPDS2D, run_local
    from tests.slab_worker import synth_problem
    pds = synth_problem(name)
    pds.iterate()
    eng = pds._engine
    assert eng.nm_fused
    n1 = pds.iter
    x1, z1 = eng.X[n1 % 2].clone(), eng.Z[n1 % 2].clone()
    pds2 = synth_problem(name)
    slabs = [SlabPDS2D.from_pds(pds2, None, rank=r, world=2) for r in range(2)]
    assert all(s.nm_fused and s.overlap for s in slabs)
    res = run_local(slabs, pds2.max_iter, pds2.min_iter, pds2.accuracy_threshold, split=True)
    assert all(r[0] == n1 for r in res)
    x2 = torch.cat([r[1] for r in res])
    z2 = torch.cat([torch.cat([r[2].view(2, -1)[c] for r in res]) for c in range(2)])
    assert torch.equal(x2, x1), (x2 - x1).abs().max().item()
    assert torch.equal(z2, z1), (z2 - z1).abs().max().item()


def _c3(n0, n1, dtype):
    sys.path.insert(0, ROOT)
    import bench
    return bench.build_problem(n0, n1, dtype)


@pytest.mark.parametrize('world', [4, 7])
def test_c3_slabs_bitwise(world):
    """C3 workload shape (15x15 Gaussian, TV, fp32) at 700 x 512 split 4 and 7 ways
    (uneven slabs), 30 fixed iterations."""
    from pycsou_amd.opt.engine import PDS2DEngine
    from pycsou_amd.parallel import SlabPDS2D, run_local
    pds = _c3(700, 512, torch.float32)
    spec = pds._fused_spec()
    eng = PDS2DEngine(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0)
    n, x1, z1, h1 = eng.run(29, 29, 0.0)
    slabs = [SlabPDS2D(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, r, world)
             for r in range(world)]
    res = run_local(slabs, 29, 29, 0.0)
    assert all(r[0] == n == 30 for r in res)
    x2 = torch.cat([r[1] for r in res])
    assert torch.equal(x2, x1)
    assert np.allclose(res[0][3][1:], h1[1:], rtol=1e-5)


@pytest.mark.parametrize('world', [3, 5])
def test_denoise_slabs_bitwise(world):
    """fp32 TV denoising 700 x 256 (the pointwise-F march kernel, pds_pt.hpp) split into uneven
    row slabs: bitwise equal to the single-GPU engine, 20 fixed iterations."""
    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L21Norm
    from pycsou_amd.linop.diff import Gradient
    from pycsou_amd.opt.engine import PDS2DEngine
    from pycsou_amd.opt.proxalgs import PDS
    from pycsou_amd.parallel import SlabPDS2D, run_local
    n0, n1 = 700, 256
    N = n0 * n1
    y = torch.as_tensor(np.random.default_rng(2).uniform(0, 1, N).astype(np.float32)).cuda()
    K = Gradient((n0, n1), kind='forward')
    K.lipschitz_cst = K.diff_lipschitz_cst = np.sqrt(8.0)
    pds = PDS(dim=N, F=(1 / 2) * SquaredL2Loss(dim=N, data=y), H=0.1 * L21Norm(dim=2 * N, groups=np.tile(np.arange(N), 2)),
              K=K, x0=torch.zeros(N, device='cuda'), z0=torch.zeros(2 * N, device='cuda'), verbose=None)
    spec = pds._fused_spec()
    eng = PDS2DEngine(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0)
    n, x1, z1, h1 = eng.run(19, 19, 0.0)
    slabs = [SlabPDS2D(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, r, world)
             for r in range(world)]
    res = run_local(slabs, 19, 19, 0.0)
    assert all(r[0] == n == 20 for r in res)
    assert torch.equal(torch.cat([r[1] for r in res]), x1)
    assert np.allclose(res[0][3][1:], h1[1:], rtol=1e-5)


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.parametrize('name', ['deconv2d_l21_fwd_64_psf15', 'nonsep_cen_f32', 'cen_denoise_f32', 'sep_cen_f32'])
def test_two_process_gloo(tmp_path, name):
    """Two ranks in two processes on the one GPU, gloo transport (host-staged): the golden
    separable deconvolution, a non-separable PSF with the reference's default centred K, and
    centred-K denoising; x bitwise equal to the single-GPU engine."""
    from tests.slab_worker import SYNTH, synth_problem
    if name in SYNTH:
        pds = synth_problem(name)
        pds.iterate()
        n1 = pds.iter
        x1 = pds._engine.X[n1 % 2].clone()
        h1 = pds._engine.hist[:2 * n1].cpu().numpy().reshape(-1, 2)
    else:
        n1, x1, z1, h1 = _single(pds_case(name), np.float64)
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE='2',
                   LOCAL_RANK='0', PYTHONPATH=ROOT)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, 'tests', 'slab_worker.py'), name,
                                       str(tmp_path)], env=env, cwd=ROOT))
    rcs = [p.wait(timeout=300) for p in procs]
    assert rcs == [0, 0]
    x = np.load(tmp_path / 'x.npy')
    h = np.load(tmp_path / 'hist.npy')
    assert int(np.load(tmp_path / 'n.npy')) == n1
    np.testing.assert_array_equal(x, x1.cpu().numpy())
    fin = np.isfinite(h1)
    assert np.allclose(h[fin], h1[fin], rtol=1e-12 if name not in SYNTH or SYNTH[name][4] == np.float64 else 1e-5)


def _pds3d_single_and_slabs(pds, world):
    from pycsou_amd.opt.engine3d import PDS3DEngine
    from pycsou_amd.parallel import run_local
    spec = pds._fused_spec()
    assert spec is not None and spec.get('ndim') == 3
    dt = pds._compute_dtype()
    one = PDS3DEngine(spec, dt, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0)
    n1, x1, z1, h1 = one.run(pds.max_iter, pds.min_iter, pds.accuracy_threshold)
    slabs = [PDS3DEngine(spec, dt, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, rank=r, world=world)
             for r in range(world)]
    res = run_local(slabs, pds.max_iter, pds.min_iter, pds.accuracy_threshold)
    x2 = torch.cat([r[1] for r in res])
    z2 = torch.cat([torch.cat([r[2].view(3, -1)[c] for r in res]) for c in range(3)])
    assert all(r[0] == n1 for r in res)
    return (n1, x1, z1, h1), (res[0][0], x2, z2, res[0][3])


@pytest.mark.parametrize('world', [2, 3])
def test_slab3d_denoise_bitwise(world):
    c = pds_case('denoise3d_l1_fwd_16')
    pds = build(c, np.float64, engine='fused')
    (n1, x1, z1, h1), (n2, x2, z2, h2) = _pds3d_single_and_slabs(pds, world)
    assert n1 == int(c['n_iter'])
    assert torch.equal(x2, x1) and torch.equal(z2, z1)
    fin = np.isfinite(h1)
    assert np.allclose(h2[fin], h1[fin], rtol=1e-12)


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
def test_slab3d_deconv_bitwise(dtype):
    """40 x 24 x 20 volume, 15-tap blur along every axis (x halo 15 planes), 2 slabs."""
    from tests.test_gpu_pds import _vol_problem
    c = _vol_problem(24, np.float64, seed=3, niter=6)
    rng = np.random.default_rng(4)
    c['shape'] = (40, 24, 20)
    c['y'] = rng.uniform(0, 1, 40 * 24 * 20)
    pds = build(c, dtype, engine='fused')
    (n1, x1, z1, h1), (n2, x2, z2, h2) = _pds3d_single_and_slabs(pds, 2)
    assert n1 == 6
    assert torch.equal(x2, x1), (x2 - x1).abs().max().item()
    assert torch.equal(z2, z1)


def _denoise_problem(n0, n1, thr=1e-3, max_iter=19, min_iter=19):
    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L21Norm
    from pycsou_amd.linop.diff import Gradient
    from pycsou_amd.opt.proxalgs import PDS
    N = n0 * n1
    y = torch.as_tensor(np.random.default_rng(2).uniform(0, 1, N).astype(np.float32)).cuda()
    K = Gradient((n0, n1), kind='forward')
    K.lipschitz_cst = K.diff_lipschitz_cst = np.sqrt(8.0)
    return PDS(dim=N, F=(1 / 2) * SquaredL2Loss(dim=N, data=y), H=0.1 * L21Norm(dim=2 * N, groups=np.tile(np.arange(N), 2)),
               K=K, x0=torch.zeros(N, device='cuda'), z0=torch.zeros(2 * N, device='cuda'), verbose=None,
               max_iter=max_iter, min_iter=min_iter, accuracy_threshold=thr)


def _problem(kind):
    return _c3(700, 512, torch.float32) if kind == 'deconv' else _denoise_problem(700, 256)


@pytest.mark.parametrize('world', [2, 3])
@pytest.mark.parametrize('kind', ['deconv', 'denoise'])
def test_banded_slabs_bitwise(kind, world):
    """The native loop's overlapped schedule (boundary bands, then interior, pcs_pds2d_step_bands)
    on uneven row slabs in one process: x, z bitwise equal to the single-GPU engine."""
    from pycsou_amd.opt.engine import PDS2DEngine
    from pycsou_amd.parallel import SlabPDS2D, run_local
    pds = _problem(kind)
    spec = pds._fused_spec()
    eng = PDS2DEngine(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0)
    n, x1, z1, h1 = eng.run(19, 19, 0.0)
    slabs = [SlabPDS2D(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, r, world)
             for r in range(world)]
    res = run_local(slabs, 19, 19, 0.0, split=True)
    assert all(r[0] == n == 20 for r in res)
    assert torch.equal(torch.cat([r[1] for r in res]), x1)
    z2 = torch.cat([torch.cat([r[2][:r[2].numel() // 2] for r in res]),
                    torch.cat([r[2][r[2].numel() // 2:] for r in res])])
    assert torch.equal(z2, z1)
    assert np.allclose(res[0][3][1:], h1[1:], rtol=1e-5)


@pytest.mark.parametrize('overlap', [True, False])
@pytest.mark.parametrize('kind', ['deconv', 'denoise'])
def test_native_loop_world1(kind, overlap):
    """pcs_slab2d_run at world 1 (no transport): serial schedule and overlapped schedule
    (side stream for the loop control) against the single-GPU engine, fixed 30 iterations."""
    from pycsou_amd.opt.engine import PDS2DEngine
    from pycsou_amd.parallel import SlabPDS2D
    pds = _problem(kind)
    spec = pds._fused_spec()
    eng = PDS2DEngine(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0)
    n, x1, z1, h1 = eng.run(29, 29, 0.0)
    s = SlabPDS2D(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, 0, 1, native=True,
                  overlap=overlap, chunk=7)
    assert s.native and s.overlapped() == overlap
    n2, x2, z2, h2 = s.run(29, 29, 0.0)
    assert n2 == n == 30
    assert torch.equal(x2, x1) and torch.equal(z2, z1)
    assert np.allclose(h2[1:], h1[1:], rtol=1e-5)


@pytest.mark.parametrize('overlap', [True, False])
def test_native_loop_graph_world1(monkeypatch, overlap):
    """PCS_SLAB_GRAPH: the native loop's chunks captured into a hipGraph (kernels, the side
    stream's events) and replayed, with an eager remainder and an odd start parity: bitwise the
    eager native loop."""
    from pycsou_amd.parallel import SlabPDS2D
    pds = _problem('deconv')
    spec = pds._fused_spec()
    s1 = SlabPDS2D(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, 0, 1, native=True,
                   overlap=overlap, chunk=7)
    n1, x1, z1, h1 = s1.run(40, 40, 0.0)
    monkeypatch.setenv('PCS_SLAB_GRAPH', '6')
    s2 = SlabPDS2D(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, 0, 1, native=True,
                   overlap=overlap, chunk=7)
    assert s2.graph_chunk == 6
    n2, x2, z2, h2 = s2.run(40, 40, 0.0)
    assert s2._graph is not None
    assert n1 == n2 == 41
    assert torch.equal(x2, x1) and torch.equal(z2, z1)
    np.testing.assert_array_equal(h2, h1)


@pytest.mark.parametrize('overlap', [True, False])
def test_native_loop_early_stop(overlap):
    """Stopping rule inside the native loop: the reference exit iteration and iterate, even
    though the overlapped schedule launches the next iteration before the stop decision."""
    from pycsou_amd.opt.engine import PDS2DEngine
    from pycsou_amd.parallel import SlabPDS2D
    pds = _denoise_problem(700, 256, thr=2e-3, max_iter=400, min_iter=5)
    spec = pds._fused_spec()
    eng = PDS2DEngine(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0)
    n, x1, z1, h1 = eng.run(400, 5, 2e-3)
    assert 6 < n < 400
    s = SlabPDS2D(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, 0, 1, native=True,
                  overlap=overlap, chunk=16)
    n2, x2, z2, h2 = s.run(400, 5, 2e-3)
    assert n2 == n
    assert torch.equal(x2, x1) and torch.equal(z2, z1)
    # the plan runs again after a stop: the step kernels' in-kernel reduction counters (every
    # workgroup still arrives once the flag is set) are consistent for the next run
    n, x1, z1, h1 = eng.run(9, 9, 0.0)
    n2, x2, z2, h2 = s.run(9, 9, 0.0)
    assert n2 == n == 10
    assert torch.equal(x2, x1) and torch.equal(z2, z1)
    assert np.isfinite(h2[:2 * n]).all()
    assert np.allclose(h2[1:2 * n], h1[1:2 * n], rtol=1e-5)


def vol3d_case(n0=80, seed=3, niter=8, kind='forward'):
    """n0 x 24 x 20 TV deconvolution (15-tap blur along every axis): slabs of >= 33 planes
    take the banded 3-D schedule (boundary bands of hx + 1 = 16 planes)."""
    from tests.test_gpu_pds import _vol_problem
    c = _vol_problem(24, np.float64, seed=seed, niter=niter, kind=kind)
    rng = np.random.default_rng(seed + 1)
    c['shape'] = (n0, 24, 20)
    c['y'] = rng.uniform(0, 1, n0 * 24 * 20)
    return c


@pytest.mark.parametrize('name,world', [('denoise3d_l21_cen_16', 2), ('denoise3d_l21_cen_16', 3),
                                        ('deconv3d_l1_bwd_20_sep7', 2)])
def test_slab3d_general_k_bitwise(name, world):
    """Backward / centred 3-D K (k_pds3d_gen: z halo 2, g on planes [-1, rows]) on 2-3 plane
    slabs in one process: x, z bitwise equal to the single-GPU engine, iteration count of the
    reference golden."""
    for dtype in (np.float64, np.float32):
        c = pds_case(name)
        pds = build(c, dtype, engine='fused')
        (n1, x1, z1, h1), (n2, x2, z2, h2) = _pds3d_single_and_slabs(pds, world)
        assert n1 == int(c['n_iter'])
        assert torch.equal(x2, x1), (dtype, (x2 - x1).abs().max().item())
        assert torch.equal(z2, z1), (dtype, (z2 - z1).abs().max().item())


@pytest.mark.parametrize('kind', ['centered', 'backward'])
def test_slab3d_banded_general_k_bitwise(kind):
    """The banded 3-D order with a backward / centred K (g of the plane before each band too):
    3 slabs of 100 planes, fp32, bitwise the single-GPU engine."""
    from pycsou_amd.opt.engine3d import PDS3DEngine
    from pycsou_amd.parallel import run_local
    pds = build(vol3d_case(100, kind=kind), np.float32, engine='fused')
    spec = pds._fused_spec()
    dt = pds._compute_dtype()
    one = PDS3DEngine(spec, dt, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0)
    n1, x1, z1, h1 = one.run(pds.max_iter, pds.min_iter, pds.accuracy_threshold)
    slabs = [PDS3DEngine(spec, dt, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, rank=r, world=3) for r in range(3)]
    assert all(s.banded and s.hz == 2 for s in slabs)
    res = run_local(slabs, pds.max_iter, pds.min_iter, pds.accuracy_threshold, split=True)
    assert all(r[0] == n1 == 8 for r in res)
    x2 = torch.cat([r[1] for r in res])
    z2 = torch.cat([torch.cat([r[2].view(3, -1)[c] for r in res]) for c in range(3)])
    assert torch.equal(x2, x1), (x2 - x1).abs().max().item()
    assert torch.equal(z2, z1)


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
@pytest.mark.parametrize('world,n0', [(2, 80), (3, 100)])
def test_slab3d_banded_bitwise(world, n0, dtype):
    """Banded 3-D order (own-plane in-plane passes, halo-plane passes, boundary-band g + update,
    interior g + update; pcs_pds3d_step_bands) on 2-3 slabs in one process: x, z bitwise equal
    to the single-GPU engine."""
    from pycsou_amd.opt.engine3d import PDS3DEngine
    from pycsou_amd.parallel import run_local
    pds = build(vol3d_case(n0), dtype, engine='fused')
    spec = pds._fused_spec()
    dt = pds._compute_dtype()
    one = PDS3DEngine(spec, dt, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0)
    n1, x1, z1, h1 = one.run(pds.max_iter, pds.min_iter, pds.accuracy_threshold)
    slabs = [PDS3DEngine(spec, dt, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, rank=r, world=world)
             for r in range(world)]
    assert all(s.banded for s in slabs)
    res = run_local(slabs, pds.max_iter, pds.min_iter, pds.accuracy_threshold, split=True)
    assert all(r[0] == n1 == 8 for r in res)
    x2 = torch.cat([r[1] for r in res])
    z2 = torch.cat([torch.cat([r[2].view(3, -1)[c] for r in res]) for c in range(3)])
    assert torch.equal(x2, x1), (x2 - x1).abs().max().item()
    assert torch.equal(z2, z1)
    fin = np.isfinite(h1)
    assert np.allclose(res[0][3][fin], h1[fin], rtol=1e-12 if dtype == np.float64 else 1e-5)


@pytest.mark.parametrize('world,dtype,n0', [(4, np.float32, 124), (4, np.float32, 160),
                                             (8, np.float64, 264), (8, np.float64, 320)])
@pytest.mark.parametrize('kind', ['forward', 'centered'])
def test_slab3d_many_ranks_bitwise(world, dtype, n0, kind):
    """The rank counts BASELINE names (C4 on 4 GPUs in fp32, C5 on 8 in fp64), in one
    process: slabs of 31 planes (2 x the 15-plane x halo + 1: the serial schedule, too thin for the bands) and
    of 33 / 40 planes (the banded schedule, boundary bands of hx + 1 = 16 planes), forward and the default
    centred K, every schedule -- serial, and the banded 'split' and 'fullg' orders -- bitwise equal to the
    single-GPU engine, with the reference's iteration count."""
    from pycsou_amd.opt.engine3d import PDS3DEngine
    from pycsou_amd.parallel import run_local
    pds = build(vol3d_case(n0, kind=kind), dtype, engine='fused')
    spec = pds._fused_spec()
    dt = pds._compute_dtype()
    one = PDS3DEngine(spec, dt, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0)
    n1, x1, z1, h1 = one.run(pds.max_iter, pds.min_iter, pds.accuracy_threshold)
    assert n1 == 8
    ran = []
    for order in ('serial', 'split', 'fullg'):
        slabs = [PDS3DEngine(spec, dt, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, rank=r, world=world)
                 for r in range(world)]
        rows = [s.rows for s in slabs]
        assert sum(rows) == n0 and min(rows) >= 2 * slabs[0].hx + 1, rows
        banded = all(s.banded for s in slabs)
        assert banded == (min(rows) > 2 * slabs[0].band), (rows, banded)
        if order != 'serial':
            if not banded:
                continue
            for s in slabs:
                s.order = order
        res = run_local(slabs, pds.max_iter, pds.min_iter, pds.accuracy_threshold, split=order != 'serial')
        assert all(r[0] == n1 for r in res)
        x2 = torch.cat([r[1] for r in res])
        z2 = torch.cat([torch.cat([r[2].view(3, -1)[c] for r in res]) for c in range(3)])
        assert torch.equal(x2, x1), (order, (x2 - x1).abs().max().item())
        assert torch.equal(z2, z1), (order, (z2 - z1).abs().max().item())
        fin = np.isfinite(h1)
        assert np.allclose(res[0][3][fin], h1[fin], rtol=1e-12 if dtype == np.float64 else 1e-5)
        ran.append(order)
        del slabs, res
    assert ran == (['serial', 'split', 'fullg'] if n0 // world > 32 else ['serial'])


def test_slab3d_two_process_overlap(tmp_path):
    """Two ranks (gloo, one GPU): the overlapped 3-D iteration (exchange started after the
    boundary bands, all-gather + loop control drained at the next iteration) against one GPU."""
    from pycsou_amd.opt.engine3d import PDS3DEngine
    pds = build(vol3d_case(), np.float64, engine='fused')
    spec = pds._fused_spec()
    one = PDS3DEngine(spec, pds._compute_dtype(), pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0)
    n1, x1, z1, h1 = one.run(pds.max_iter, pds.min_iter, pds.accuracy_threshold)
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE='2',
                   LOCAL_RANK='0', PYTHONPATH=ROOT)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, 'tests', 'slab_worker.py'), 'vol3d',
                                       str(tmp_path)], env=env, cwd=ROOT))
    rcs = [p.wait(timeout=300) for p in procs]
    assert rcs == [0, 0]
    assert int(np.load(tmp_path / 'n.npy')) == n1
    np.testing.assert_array_equal(np.load(tmp_path / 'x.npy'), x1.cpu().numpy())
    h = np.load(tmp_path / 'hist.npy')
    fin = np.isfinite(h1)
    assert np.allclose(h[fin], h1[fin], rtol=1e-12)


class _CopyComm:
    """One-rank stand-in transport for exercising the schedule trial (allgather = copy)."""
    tunable = True

    def allgather(self, src, dst):
        dst[:src.numel()].copy_(src)


@pytest.mark.parametrize('kind', ['deconv', 'denoise'])
def test_native_schedule_trial_bitwise(kind):
    """SlabPDS2D._autotune (serial vs overlapped native schedule, timed, plan switched in the
    middle of the loop) keeps the iteration count and gives bitwise the single-GPU iterates."""
    from pycsou_amd.opt.engine import PDS2DEngine
    from pycsou_amd.parallel import SlabPDS2D
    pds = _problem(kind)
    spec = pds._fused_spec()
    eng = PDS2DEngine(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0)
    n, x1, z1, _ = eng.run(29, 29, 0.0)
    s = SlabPDS2D(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, 0, 1, native=True,
                  overlap=True, chunk=7)
    s.comm = _CopyComm()
    total = s.init_loop(29, 29, 0.0)
    used = s._autotune()
    assert used == 8 and s._tuned and len(s.tune_ms) == 2
    s.advance(total - used)
    n2, x2, z2, _ = s.result()
    assert n2 == n == 30
    assert torch.equal(x2, x1) and torch.equal(z2, z1)


def test_rccl_binding_world1():
    """The run-time RCCL binding behind the native multi-GPU loops (dlopen of librccl, unique
    id, communicator init/destroy) on a one-rank communicator, plus pcs_halo_exchange and a
    native slab plan on it: the path the driver's multi-GPU bench takes first."""
    import ctypes
    from pycsou_amd import _lib as L
    from pycsou_amd.parallel import SlabPDS2D
    lib = L.gpu()
    assert lib.pcs_comm_available() == 1
    nb = int(lib.pcs_comm_id_bytes())
    assert nb == 128  # sizeof(ncclUniqueId)
    uid = (ctypes.c_ubyte * nb)()
    assert lib.pcs_comm_unique_id(ctypes.cast(uid, ctypes.c_void_p)) == 0
    assert any(uid)
    h = ctypes.c_void_p()
    assert lib.pcs_comm_init(ctypes.cast(uid, ctypes.c_void_p), 1, 0, ctypes.byref(h)) == 0 and h.value
    hs = L.HaloSet()
    assert lib.pcs_halo_exchange(h, 0, 1, ctypes.byref(hs), L.stream()) == 0
    pds = _problem('denoise')
    spec = pds._fused_spec()
    s = SlabPDS2D(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, 0, 1, native=True)
    n, x, z, _ = s.run(9, 9, 0.0)
    assert n == 10 and torch.isfinite(x).all()
    torch.cuda.synchronize()
    assert lib.pcs_comm_destroy(h) == 0


def test_rccl_transport_graph_capture_world1():
    """RcclComm (the 3-D engine's multi-GPU transport): the RCCL all-gather of the norm sums
    through pcs_allgather_f64 on a one-rank communicator, eager, on the side stream
    (allgather_start / wait) and captured into a hipGraph and replayed -- the capture the
    multi-GPU 3-D loop relies on."""
    import ctypes
    from pycsou_amd import _lib as L
    from pycsou_amd.parallel.slab import RcclComm
    lib = L.gpu()
    nb = int(lib.pcs_comm_id_bytes())
    uid = (ctypes.c_ubyte * nb)()
    assert lib.pcs_comm_unique_id(ctypes.cast(uid, ctypes.c_void_p)) == 0
    h = ctypes.c_void_p()
    assert lib.pcs_comm_init(ctypes.cast(uid, ctypes.c_void_p), 1, 0, ctypes.byref(h)) == 0
    rc = RcclComm(h, 0, 1)
    src = torch.arange(4, dtype=torch.float64, device='cuda') + 1.0
    dst = torch.zeros(4, dtype=torch.float64, device='cuda')
    rc.allgather(src, dst)
    torch.cuda.synchronize()
    assert torch.equal(dst, src)
    dst.zero_()
    rc.allgather_start(src, dst).wait()
    torch.cuda.synchronize()
    assert torch.equal(dst, src)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        src.mul_(2.0)
        rc.allgather_start(src, dst).wait()
        dst.add_(1.0)
    src.copy_(torch.arange(4, dtype=torch.float64, device='cuda'))
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(dst, torch.arange(4, dtype=torch.float64, device='cuda') * 8.0 + 1.0)
    rc.exchange({})  # no neighbours: nothing to move
    del g
    torch.cuda.synchronize()
    assert lib.pcs_comm_destroy(h) == 0


def test_pds3d_capture_failure_falls_back_to_eager(monkeypatch):
    """A library error (HipError) raised while a chunk is being captured leaves the 3-D engine on
    eager launches (the capture outcome is agreed collectively, so every rank must get past the
    failure): the run completes with the same iterates as an engine that never captured."""
    from pycsou_amd import _lib as L
    from pycsou_amd.opt.engine3d import PDS3DEngine
    pds = build(vol3d_case(), np.float64, engine='fused')
    spec = pds._fused_spec()
    dt = pds._compute_dtype()
    ref = PDS3DEngine(spec, dt, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0)
    ref.use_graph = False
    n0, x0, z0, _ = ref.run(pds.max_iter, pds.min_iter, pds.accuracy_threshold)
    eng = PDS3DEngine(spec, dt, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0)
    orig = eng.iteration

    def failing(p):
        if torch.cuda.is_current_stream_capturing():
            raise L.HipError('pcs_pds3d_step returned status -2 (injected)')
        return orig(p)
    monkeypatch.setattr(eng, 'iteration', failing)
    n1, x1, z1, _ = eng.run(pds.max_iter, pds.min_iter, pds.accuracy_threshold)
    assert not eng.use_graph and eng.graph is None
    assert n1 == n0
    assert torch.equal(x1, x0) and torch.equal(z1, z0)


@pytest.mark.parametrize('k', [1, 5, 8, 13])
def test_pds3d_advance_issues_exactly_k(k):
    """advance(k) issues exactly k iterations whatever the chunk and buffer parity (graph replays
    of whole chunks from parity 0, eager iterations for the parity fix and the remainder)."""
    from pycsou_amd.opt.engine3d import PDS3DEngine
    pds = build(vol3d_case(), np.float64, engine='fused')
    spec = pds._fused_spec()
    eng = PDS3DEngine(spec, pds._compute_dtype(), pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, chunk=4)
    eng.init_loop(100, 100, -1.0)
    eng.advance(3)
    eng.advance(k)
    torch.cuda.synchronize()
    assert eng.iterations() == 3 + k


def _stop_threshold(pds, kind, niter, j):
    """A primal relative-improvement threshold under which the single-GPU run stops after iteration j of
    a `niter` fixed run (between the metric of iterations j - 1 and j)."""
    from pycsou_amd.opt.engine import PDS2DEngine
    spec = pds._fused_spec()
    eng = PDS2DEngine(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0)
    _, _, _, h = eng.run(niter - 1, niter - 1, 0.0)
    m = h[:, 0]
    assert np.all(m[:j] > m[j]), m[:j + 1]  # the first iteration whose metric falls below the threshold
    return float(0.5 * (min(m[:j]) + m[j]))


@pytest.mark.parametrize('kind,world,depth', [('deconv', 2, 2), ('deconv', 3, 4), ('deconv', 8, 4),
                                              ('denoise', 3, 4), ('denoise', 5, 8)])
def test_deep_halo_slabs_bitwise(kind, world, depth):
    """The communication-avoiding slab loop (pcs_slab2d_deep_*: halos `depth` iterations deep, exchanged once
    per chunk; each iteration also computes the shrinking redundant halo rows) in one process with the
    device-copy transport: x, z bitwise the single-GPU engine and the same iteration count, for a fixed
    count that ends mid-chunk and for a natural stop landing inside a chunk."""
    from pycsou_amd.opt.engine import PDS2DEngine
    from pycsou_amd.parallel import SlabPDS2D, run_local_deep
    pds = _problem(kind)
    spec = pds._fused_spec()
    thr = _stop_threshold(pds, kind, 40, 2 * depth)
    for max_iter, min_iter, acc in ((21, 21, 0.0), (200, 2, thr)):
        eng = PDS2DEngine(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0)
        n, x1, z1, h1 = eng.run(max_iter, min_iter, acc)
        if acc > 0:
            assert n == 2 * depth + 1, (n, depth)  # the stop lands inside a chunk
        slabs = [SlabPDS2D(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, r, world,
                           native='local', depth=depth) for r in range(world)]
        assert all(s.depth == depth and s.nbuf == max(2, depth) for s in slabs)
        res = run_local_deep(slabs, max_iter, min_iter, acc, chunk=depth)
        assert all(r[0] == n for r in res), ([r[0] for r in res], n)
        x2 = torch.cat([r[1] for r in res])
        z2 = torch.cat([torch.cat([r[2][:r[2].numel() // 2] for r in res]),
                        torch.cat([r[2][r[2].numel() // 2:] for r in res])])
        assert torch.equal(x2, x1), (x2 - x1).abs().max().item()
        assert torch.equal(z2, z1), (z2 - z1).abs().max().item()
        assert np.allclose(res[0][3][1:], h1[1:], rtol=1e-5)


def test_deep_halo_world1_native_run():
    """depth > 1 on one rank (no neighbours: no redundant rows, the loop control once per chunk): the
    native pcs_slab2d_deep_run loop against the single-GPU engine, fixed count and natural stop."""
    from pycsou_amd.opt.engine import PDS2DEngine
    from pycsou_amd.parallel import SlabPDS2D
    pds = _problem('deconv')
    spec = pds._fused_spec()
    thr = _stop_threshold(pds, 'deconv', 40, 10)
    for max_iter, min_iter, acc in ((21, 21, 0.0), (200, 2, thr)):
        eng = PDS2DEngine(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0)
        n, x1, z1, h1 = eng.run(max_iter, min_iter, acc)
        s = SlabPDS2D(spec, torch.float32, pds.tau, pds.sigma, pds.rho, pds.x0, pds.z0, 0, 1, native=True, depth=4,
                      chunk=8)
        n2, x2, z2, h2 = s.run(max_iter, min_iter, acc)
        assert n2 == n
        assert torch.equal(x2, x1) and torch.equal(z2, z1)
        assert np.allclose(h2[1:], h1[1:], rtol=1e-5)

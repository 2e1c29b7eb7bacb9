"""Run-to-run determinism of the fused 2-D marches: the same problem from the same state gives bitwise the
same iterate, dual and diagnostics every run (every reduction is fixed-order; an LDS tile read before its
loads land -- the round-5 race of the centred normal-operator march -- shows up here as differing pixels
from the second iteration on).  tests/test_host.py::test_lds_dma_waits_cover_the_tiles checks the wait
counts statically."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _problem(name):
    import bench
    f32, f64 = torch.float32, torch.float64
    return {
        'c3_cen': lambda: (bench.build_problem(2048, 2048, f32, lipschitz='analytic', kind='centered'), f32),
        'c3': lambda: (bench.build_problem(2048, 2048, f32, lipschitz='analytic'), f32),
        'c3_cen_f64': lambda: (bench.build_problem(1024, 1024, f64, lipschitz='analytic', kind='centered'), f64),
        'lap': lambda: (bench.build_denoise_k(2048, f32, 'lap', lipschitz='analytic'), f32),
        'cen': lambda: (bench.build_denoise_k(2048, f32, 'centered', lipschitz='analytic'), f32),
        'pt': lambda: (bench.build_denoise(2048, f32, lipschitz='analytic'), f32),
    }[name]()


@pytest.mark.parametrize('name', ['c3_cen', 'c3', 'c3_cen_f64', 'lap', 'cen', 'pt'])
def test_fused_march_is_deterministic(name):
    import pycsou_amd.opt.engine as E
    from pycsou_amd import _ops as O
    pds, dtype = _problem(name)
    spec = pds._fused_spec()
    runs = []
    for _ in range(3):
        eng = E.engine_class(spec)(spec, dtype, pds.tau, pds.sigma, pds.rho, O.to_dev(pds.x0, dtype),
                                   O.to_dev(pds.z0, dtype))
        n, x, z, h = eng.run(7, 7, 0.0)
        torch.cuda.synchronize()
        runs.append((n, x.clone(), z.clone(), np.asarray(h).copy()))
    for n, x, z, h in runs[1:]:
        assert n == runs[0][0] == 8
        assert torch.equal(x, runs[0][1]), int((x != runs[0][1]).sum())
        assert torch.equal(z, runs[0][2]), int((z != runs[0][2]).sum())
        assert np.array_equal(h, runs[0][3])


@pytest.mark.parametrize('kind', ['forward', 'centered'])
def test_fused_3d_step_is_deterministic(kind):
    """The 3-D engine (k_pds3d with the folded axis-0 pass / k_pds3d_gen + the in-plane normal operator)
    through the public API, three runs of 8 iterations at 96^3: bitwise the same iterate and dual."""
    import bench
    outs = []
    for _ in range(3):
        pds = bench.build_volume(96, torch.float32, kind=kind)
        pds.max_iter, pds.min_iter, pds.accuracy_threshold = 7, 7, 0.0
        est, _, diag = pds.iterate()
        assert pds._engine is not None and pds.iter == 8
        outs.append((est['primal_variable'].clone(), est['dual_variable'].clone()))
    for x, z in outs[1:]:
        assert torch.equal(x, outs[0][0]), int((x != outs[0][0]).sum())
        assert torch.equal(z, outs[0][1]), int((z != outs[0][1]).sum())

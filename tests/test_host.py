"""CPU-side tests: the C-ABI library loads and exports the declared symbols, and the host
logic (algebra, Lipschitz propagation, step sizes, dispatch, validation) matches the
reference.  No compute calls (no GPU here)."""

import os
import re

import numpy as np
import pytest

from tests.cases import pds_case, pds_case_names

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    from pycsou_amd import _lib
    lib = _lib.load()
    hdr = open(os.path.join(REPO, 'include', 'pycsou_hip.h')).read()
    declared = set(re.findall(r'^\s*(?:int|int64_t)\s+(pcs_\w+)\(', hdr, flags=re.M))
    assert len(declared) >= 25
    for name in declared:
        assert hasattr(lib, name), name
    assert declared <= set(_lib.EXPORTS), declared - set(_lib.EXPORTS)
    assert lib.pcs_abi_version() == 10
    assert lib.pcs_ctrl_bytes() == 64
    assert lib.pcs_pds2d_halo_x(7) == 15


def test_compute_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    from pycsou_amd.func.penalty import L1Norm
    with pytest.raises(RuntimeError, match='no ROCm GPU'):
        L1Norm(4).prox(np.ones(4), 0.1)


def test_lipschitz_propagation_and_types():
    from pycsou_amd.core.map import DiffMapComp
    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L1Norm, L21Norm, L2Norm, SquaredL2Norm
    from pycsou_amd.linop.conv import Convolve2D
    from pycsou_amd.linop.base import HomothetyMap
    N = 16
    half = (1 / 2) * SquaredL2Loss(dim=N, data=np.ones(N))
    assert isinstance(half, DiffMapComp) and isinstance(half.map1, HomothetyMap)
    assert half.diff_lipschitz_cst == 1.0
    C = Convolve2D(N, np.ones((3, 3)) / 9, (4, 4))
    C.lipschitz_cst = C.diff_lipschitz_cst = 0.5
    F = half * C
    assert F.diff_lipschitz_cst == 0.25 and F.shape == (1, N)
    assert SquaredL2Loss(dim=N, data=np.ones(N)).diff_lipschitz_cst == 2
    assert (3 * L1Norm(N)).scale == 3
    # L21Norm.__new__ dispatch (penalty.py:525-530)
    assert isinstance(L21Norm(10, groups=None), L1Norm)
    assert isinstance(L21Norm(10, groups=np.arange(10)), L1Norm)
    assert isinstance(L21Norm(10, groups=np.zeros(10)), L2Norm)
    l21 = L21Norm(10, groups=np.tile(np.arange(5), 2))
    assert isinstance(l21, L21Norm) and l21.pixel_d == 2
    assert L21Norm(10, groups=np.repeat(np.arange(5), 2)).pixel_d == 0
    assert SquaredL2Norm(3).diff_lipschitz_cst == 2


@pytest.mark.parametrize('name', pds_case_names())
def test_pds_construction_matches_reference(name):
    """Step sizes, momentum and beta from our PDS constructor equal the reference's."""
    from tests.test_gpu_pds import build
    c = pds_case(name)
    pds = build(c, np.float64)
    assert pds.tau == float(c['tau']) and pds.sigma == float(c['sigma'])
    assert pds.rho == float(c['rho']) and pds.beta == float(c['beta'])
    from pycsou_amd.opt.engine import match_pds2d
    spec = match_pds2d(pds.F, pds.G, pds.H, pds.K, True)
    fused_expected = ('3d' not in name and 'lap' not in name and '_cen_' not in name and '_bwd_' not in name)
    assert (spec is not None) == fused_expected


def test_pds_validation_errors():
    from pycsou_amd.func.penalty import L1Norm
    from pycsou_amd.linop.diff import Gradient
    from pycsou_amd.opt.proxalgs import PDS, APGD
    from pycsou_amd.func.loss import SquaredL2Loss
    K = Gradient((4, 4), kind='forward')
    with pytest.raises(ValueError):
        PDS(dim=16, H=L1Norm(32), K=K)  # K.lipschitz_cst is inf (proxalgs.py:289-290)
    with pytest.raises(ValueError):
        PDS(dim=16, H=L1Norm(31), K=K)
    with pytest.raises(TypeError):
        PDS(dim=16, F=3.0)
    with pytest.raises(ValueError):
        PDS(dim=15, F=SquaredL2Loss(16, np.zeros(16)))
    with pytest.raises(TypeError):
        APGD(dim=16, G='x')
    K.lipschitz_cst = 2.0
    p = PDS(dim=16, H=L1Norm(32), K=K, verbose=None)
    assert p.tau == p.sigma == 0.5 and p.rho == 1
    p = PDS(dim=16, F=SquaredL2Loss(16, np.zeros(16)), verbose=None)
    assert p.tau == 1.0 and p.sigma == 0 and p.rho == 0.9 and p.K.lipschitz_cst == 0


def test_graft_entry_importable():
    import importlib
    m = importlib.import_module('__graft_entry__')
    assert callable(m.build) and callable(m.smoke)


def test_halo_exchange_argument_checks():
    """pcs_halo_exchange validates on the host before touching RCCL: bad rank/world or missing
    neighbour buffers -> PCS_EINVAL; world 1 -> no-op."""
    import ctypes
    from pycsou_amd import _lib
    lib = _lib.load()
    h = _lib.HaloSet()
    h.nbuf = 1
    h.bytes[0] = 16
    assert lib.pcs_halo_exchange(None, 0, 1, ctypes.byref(h), None) == 0
    assert lib.pcs_halo_exchange(None, 1, 1, ctypes.byref(h), None) == -1
    assert lib.pcs_halo_exchange(None, 0, 2, ctypes.byref(h), None) == -1  # rank 0 of 2 needs send_hi/recv_hi
    h.nbuf = 5
    assert lib.pcs_halo_exchange(None, 0, 1, ctypes.byref(h), None) == -1


def test_pds2d_reduce_only_argument_checks():
    """Slab reduce-only mode of pcs_pds2d_step (sums_out): the host checks reject a missing or
    misaligned workspace, a negative pre-partials count and pre partials without a pointer,
    before anything is launched (fake device addresses are never dereferenced)."""
    import ctypes
    from pycsou_amd import _lib
    lib = _lib.load()
    a = _lib.PdsArgs()
    a.dtype, a.fkind, a.hkind, a.gkind = _lib.PCS_F32, _lib.PCS_F_DENOISE, _lib.PCS_H_L21, _lib.PCS_G_NULL
    a.n0 = a.n1 = a.rows = 64
    a.sigma = a.step0 = a.step1 = 1.0
    for f in ('x', 'xn', 'z', 'zn', 'y', 'partials'):
        setattr(a, f, 0x10000)
    a.sums_out = 0x20000
    a.hist = None
    a.ws = None
    assert lib.pcs_pds2d_step(ctypes.byref(a), None) == -1  # no workspace
    a.ws = 0x30008
    assert lib.pcs_pds2d_step(ctypes.byref(a), None) == -1  # misaligned workspace
    a.ws = 0x30000
    a.n_pre = -1
    assert lib.pcs_pds2d_step(ctypes.byref(a), None) == -1
    a.n_pre = 4
    a.pre_partials = None
    assert lib.pcs_pds2d_step(ctypes.byref(a), None) == -1
    assert lib.pcs_pds2d_step_bands(ctypes.byref(a), 0, 8, 56, 64, None) == -1


def test_pds3d_general_k_argument_checks():
    """pcs_pds3d_* with backward / centred K: an unknown K kind is rejected, and a multi-plane slab
    needs z halos of two planes (K^T z reads z one plane past u's planes on both sides); the host
    checks run before anything is launched (fake device addresses are never dereferenced)."""
    import ctypes
    from pycsou_amd import _lib
    lib = _lib.load()
    a = _lib.Pds3Args()
    a.dtype, a.fkind, a.hkind, a.gkind = _lib.PCS_F32, _lib.PCS_F_NULL, _lib.PCS_H_L21, _lib.PCS_G_NULL
    a.n0, a.n1, a.n2, a.plane0, a.planes = 64, 64, 64, 16, 32
    a.sigma = a.step0 = a.step1 = a.step2 = 1.0
    for f in ('x', 'xn', 'z', 'zn', 'partials'):
        setattr(a, f, 0x10000)
    a.halo_x = a.halo_z = 1
    a.kkind = _lib.PCS_FORWARD
    assert lib.pcs_pds3d_nblocks_bands(ctypes.byref(a), 0, 32, 32, 32) > 0
    for kind in (_lib.PCS_BACKWARD, _lib.PCS_CENTERED):
        a.kkind, a.halo_z = kind, 1
        assert lib.pcs_pds3d_step(ctypes.byref(a), None) == -1
        assert lib.pcs_pds3d_nblocks_bands(ctypes.byref(a), 0, 32, 32, 32) == -1
        a.halo_z = 2
        assert lib.pcs_pds3d_nblocks_bands(ctypes.byref(a), 0, 32, 32, 32) > 0
    a.kkind = 7
    assert lib.pcs_pds3d_step(ctypes.byref(a), None) == -1


def test_pds2d_sepconv_general_k_dispatch():
    """Separable-PSF PDS with backward / centred K: the fused normal-operator march (no G buffer)
    covers the shape when the last 64-column strip is wider than the tap tier; otherwise the step
    needs the caller's G buffer (two-launch form) and is unsupported without one. A multi-row slab
    needs halos of 2 + 2*tier rows. Host-side queries only (fake device addresses)."""
    import ctypes
    from pycsou_amd import _lib
    lib = _lib.load()
    a = _lib.PdsArgs()
    a.dtype, a.fkind, a.hkind, a.gkind = _lib.PCS_F32, _lib.PCS_F_SEPCONV, _lib.PCS_H_L21, _lib.PCS_G_NULL
    a.kkind = _lib.PCS_K_GRAD_CENTERED
    a.half = 7
    a.n0 = a.rows = 256
    a.sigma = a.step0 = a.step1 = 1.0
    a.w0 = a.w1 = 0.5
    for f in ('x', 'xn', 'z', 'zn', 'y', 'partials', 'taps0', 'taps1', 'cty', 'ntaps'):
        setattr(a, f, 0x10000)
    a.gbuf = None
    a.n1 = 4096                      # last strip 64 wide: fused march
    assert lib.pcs_pds2d_supported(ctypes.byref(a)) == 1
    a.n1 = 4096 + 4                  # last strip 4 wide (<= tier 7): two-launch form, needs G
    assert lib.pcs_pds2d_supported(ctypes.byref(a)) == 0
    a.gbuf = 0x40000
    assert lib.pcs_pds2d_supported(ctypes.byref(a)) == 1
    a.n1, a.gbuf = 4096, None
    a.row0, a.rows = 64, 128         # slab: halos must cover 2 + 2*tier rows of x and y
    a.halo_x = a.halo_y = 15
    a.halo_z = 4
    assert lib.pcs_pds2d_supported(ctypes.byref(a)) == 0
    a.halo_x = a.halo_y = 16
    assert lib.pcs_pds2d_supported(ctypes.byref(a)) == 1


@pytest.mark.parametrize('half', [7, 5, 3, 2])
def test_nmarch_tables_equal_dense_normal_operator(half):
    """The normal-operator march kernel's tables (pycsou_amd.opt.engine.nmarch_taps) rebuild
    N = C^T C of the zero-boundary 'same' 1-D convolution along each axis exactly (fp32 table
    rounding): window taps away from the edges, window - E on the H samples nearest each edge,
    zero outside the 4H+1 band."""
    from pycsou_amd.opt.engine import nmarch_taps
    H = 3 if half <= 3 else 7
    r = np.arange(2 * half + 1) - half
    t0 = np.exp(-0.5 * (r / 2.0) ** 2)
    t0 /= t0.sum()
    t1 = np.exp(-0.5 * (r / 1.3) ** 2) * (1 + 0.1 * r)
    t1 /= t1.sum()
    tab = nmarch_taps(t0, t1, half).astype(np.float64)
    assert tab.size == 64 + 32 * H
    n = 40
    for t, axis in ((t0, 0), (t1, 1)):
        C = np.zeros((n, n))
        for i in range(n):
            for j in range(max(0, i - half), min(n, i + half + 1)):
                C[i, j] = t[half + i - j]
        N = C.T @ C
        win = tab[32 * axis:32 * axis + 4 * H + 1]
        M = np.zeros((n, n))
        for j in range(n):
            for k in range(max(0, j - 2 * H), min(n, j + 2 * H + 1)):
                v = win[k - j + 2 * H]
                if axis == 0:
                    if j < H and k < H:
                        v -= tab[64 + 8 * j + k]
                    if j >= n - H and k >= n - H:
                        v -= tab[64 + 8 * H + 8 * (j - (n - H)) + (k - (n - H))]
                else:  # transposed right/left tables, as the kernel indexes them
                    if j < H and k < H:
                        v -= tab[64 + 16 * H + 8 * k + j]
                    if j >= n - H and k >= n - H:
                        v -= tab[64 + 24 * H + 8 * (k - (n - H)) + (8 - H) + (j - (n - H))]
                M[j, k] = v
        np.testing.assert_allclose(M, N, atol=2e-8)


@pytest.mark.parametrize('k,off', [(15, 7), (6, 2), (3, 0), (5, 1), (1, 0), (2, 1), (8, 0), (8, 7)])
@pytest.mark.parametrize('n', [16, 17, 40])
def test_sep2d_nrm_tables_equal_dense_normal_operator(k, off, n):
    """The tables k_sep2d_nrm (csrc/sep_ata.hip) builds per workgroup: for taps reaching <= 7
    samples either side, C^T C of a zero-boundary Convolve1D (out[j] = sum_t h[t] in[j + off - t])
    is a[j - k] (a the taps' autocorrelation, c(d) = h[d + off]) minus the 7x7 blocks of the
    terms outside the line at each end -- equal to the dense C^T C, planes down to 16 samples."""
    rng = np.random.default_rng(k * 100 + off * 10 + n)
    h = rng.standard_normal(k)
    C = np.zeros((n, n))
    for j in range(n):
        for i in range(n):
            if 0 <= j + off - i < k:
                C[j, i] = h[j + off - i]

    def c(d):
        return h[d + off] if 0 <= d + off < k else 0.0
    a = [sum(c(m) * c(m + e) for m in range(-7, 8)) for e in range(-14, 15)]
    N = np.zeros((n, n))
    for j in range(n):
        for q in range(29):
            if 0 <= j - 14 + q < n:
                N[j, j - 14 + q] = a[q]
    for j in range(7):
        for cc in range(7):
            N[j, cc] -= sum(c(i - j) * c(i - cc) for i in range(-7, 0))
            N[n - 7 + j, n - 7 + cc] -= sum(c(7 + ii - j) * c(7 + ii - cc) for ii in range(7))
    np.testing.assert_allclose(N, C.T @ C, atol=1e-12)


def test_pds2d_masked_block_and_fp64_dispatch():
    """ABI 6 masked data-fidelity block (mkind = PCS_M_L1LOSS, the CPS inpainting step) and the fp64
    general-stencil march: host-side support queries only (fake device addresses, nothing launched).
    The masked block needs F = 0, whole images, its three buffers and the row march's geometry; fp64
    runs every K kind, the forward Gradient included, and separable PSFs only with N x's buffer."""
    import ctypes
    from pycsou_amd import _lib
    lib = _lib.load()
    assert ctypes.sizeof(_lib.PdsArgs) % 8 == 0
    for dt in (_lib.PCS_F32, _lib.PCS_F64):
        for kk in (_lib.PCS_K_GRAD_FORWARD, _lib.PCS_K_GRAD_CENTERED, _lib.PCS_K_LAPLACIAN):
            a = _lib.PdsArgs()
            a.dtype, a.fkind, a.gkind = dt, _lib.PCS_F_NULL, _lib.PCS_G_SEGMENT
            a.hkind = _lib.PCS_H_L1 if kk == _lib.PCS_K_LAPLACIAN else _lib.PCS_H_L21
            a.kkind, a.edge = kk, 1
            a.n0 = a.rows = 256
            a.n1 = 512
            a.sigma = a.step0 = a.step1 = 1.0
            a.seg_b = 1.0
            for f in ('x', 'xn', 'z', 'zn', 'partials', 'ym', 'zm', 'zmn'):
                setattr(a, f, 0x10000)
            a.mkind = _lib.PCS_M_L1LOSS
            assert lib.pcs_pds2d_supported(ctypes.byref(a)) == 1, (dt, kk)
            assert lib.pcs_pds2d_nblocks(ctypes.byref(a)) > 0
            a.zmn = None
            assert lib.pcs_pds2d_supported(ctypes.byref(a)) == 0  # missing buffer
            a.zmn = 0x10000
            a.fkind, a.y = _lib.PCS_F_DENOISE, 0x10000
            assert lib.pcs_pds2d_supported(ctypes.byref(a)) == 0  # F must be 0
            a.fkind = _lib.PCS_F_NULL
            a.row0, a.rows, a.halo_x, a.halo_y, a.halo_z = 64, 128, 4, 4, 4
            assert lib.pcs_pds2d_supported(ctypes.byref(a)) == 0  # slabs: no
            a.row0, a.rows = 0, 256
            a.n1 = 60
            assert lib.pcs_pds2d_supported(ctypes.byref(a)) == 0  # one strip: no march
    # fp64 separable PSF, forward K: the march with N x into gbuf (two launches); without gbuf the
    # tile kernel keeps it
    a = _lib.PdsArgs()
    a.dtype, a.fkind, a.hkind, a.gkind = _lib.PCS_F64, _lib.PCS_F_SEPCONV, _lib.PCS_H_L21, _lib.PCS_G_NULL
    a.kkind, a.half = _lib.PCS_K_GRAD_FORWARD, 7
    a.n0 = a.rows = 256
    a.n1 = 512
    a.sigma = a.step0 = a.step1 = 1.0
    for f in ('x', 'xn', 'z', 'zn', 'y', 'partials', 'taps0', 'taps1', 'cty'):
        setattr(a, f, 0x10000)
    assert lib.pcs_pds2d_supported(ctypes.byref(a)) == 1  # tile kernel
    nb_tile = lib.pcs_pds2d_nblocks(ctypes.byref(a))
    a.gbuf = 0x20000
    assert lib.pcs_pds2d_supported(ctypes.byref(a)) == 1
    assert lib.pcs_pds2d_nblocks(ctypes.byref(a)) != nb_tile  # the march's task count


def test_lds_dma_waits_cover_the_tiles(tmp_path):
    """The row marches land their z tiles with LDS-DMA loads and wait, before the barrier that precedes the
    tiles' first read, until only the loads issued after them are outstanding.  A load the compiler sinks
    past that wait breaks the count (round 5: the centred normal-operator march read a tile still in
    flight, and its iterate differed between runs).  Compile the two march units to gfx950 assembly and
    check every march kernel's loop: the wait's count never exceeds the loads issued after the last tile
    load (tools/vmcnt_check.py)."""
    import shutil
    import subprocess
    import sys
    hipcc = shutil.which('hipcc') or '/opt/rocm/bin/hipcc'
    if not os.path.exists(hipcc):
        pytest.skip('hipcc not available')
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    csrc = os.path.join(root, 'pycsou_amd', 'csrc')
    # every source that issues LDS-DMA loads, and the unit that instantiates its kernels: a new DMA kernel
    # elsewhere fails here until it is added to the check
    dma_units = {'pds_nmarch.hpp': 'pds_nm', 'pds_nm64.hip': 'pds_nm64'}
    dma_files = sorted(f for f in os.listdir(csrc) if f.endswith(('.hip', '.hpp'))
                       and 'buffer_load_lds' in open(os.path.join(csrc, f)).read())
    assert dma_files == sorted(dma_units), f'LDS-DMA sources {dma_files}: add their units to this check'
    units = sorted(set(dma_units.values()))
    outs = []
    for unit in units:
        out = str(tmp_path / f'{unit}.s')
        subprocess.run([hipcc, '--offload-arch=gfx950', '-O3', '-fno-slp-vectorize', '-std=c++17',
                        '-I' + os.path.join(root, 'include'), '--cuda-device-only', '-S',
                        os.path.join(root, 'pycsou_amd', 'csrc', unit + '.hip'), '-o', out],
                       check=True, capture_output=True, timeout=600)
        outs.append(out)
    r = subprocess.run([sys.executable, os.path.join(root, 'tools', 'vmcnt_check.py')] + outs, capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stdout
    assert r.stdout.count('ok ') >= 12, r.stdout


def test_vmcnt_check_sees_every_dma_site():
    """A kernel whose loop body the compiler emitted twice: the first copy's wait lets the tile load stay in
    flight (vmcnt(3) with 2 loads after it), the second copy is fine.  The checker must flag the first copy
    (the round-5 form inspected only the textually last DMA load)."""
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location('vmcnt_check', os.path.join(root, 'tools', 'vmcnt_check.py'))
    vc = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(vc)
    copy_bad = ['buffer_load_dwordx4 v0, s[0:3], 0 offen lds', 'buffer_load_dwordx4 v1, s[0:3], 0 offen lds',
                'buffer_load_dwordx4 v[4:7], v2, s[4:7], 0 offen', 'buffer_load_dwordx4 v[8:11], v3, s[4:7], 0 offen',
                'v_fma_f32 v12, v13, v14, v15', 's_waitcnt vmcnt(3)', 's_barrier', 'ds_read_b128 v[16:19], v20']
    copy_ok = [l.replace('vmcnt(3)', 'vmcnt(2)') for l in copy_bad]
    sites = vc.check_body(copy_bad + ['s_branch .LBB0_1'] + copy_ok)
    assert [ok for _, ok, _, _ in sites] == [False, True]
    # the round-5 single-site rule (last DMA load only) passes the same body
    assert vc.check_body(copy_ok)[0][1]
    # a wait split in two before the barrier: the later, tighter one covers the group
    split = copy_bad[:6] + ['s_waitcnt vmcnt(0)'] + copy_bad[6:]
    assert vc.check_body(split)[0][1]
    # the control-flow form used by check(): the same verdicts per copy ...
    cfg = vc.check_body_cfg(copy_bad + ['s_branch .LBB0_1'] + copy_ok)
    assert [ok for _, ok, _, _ in cfg] == [True, False, True, True]  # per DMA load: the first of a group defers
    # ... and a DMA loop laid out after the block it exits to (round 6, k_pds2d_nmarch64's tile loop), which
    # the linear scan misreads: the path from the DMA load runs through the branch to the loads and the wait
    ool = ['s_cbranch_vccz .LBB0_2', '.LBB0_1:', 'buffer_load_dwordx4 v[4:7], v2, s[4:7], 0 offen',
           's_waitcnt vmcnt(1)', 's_barrier', 's_endpgm', '.LBB0_2:', 'buffer_load_dwordx4 v0, s[0:3], 0 offen lds',
           's_cbranch_scc0 .LBB0_1', 's_branch .LBB0_2']
    assert vc.check_body_cfg(ool)[0][1]
    assert not vc.check_body_cfg([l.replace('vmcnt(1)', 'vmcnt(2)') for l in ool])[0][1]


@pytest.mark.parametrize('spectrum', ['cluster', 'gap'])
def test_lanczos_bound_is_tight_and_safe(spectrum):
    """Host logic of the device Lanczos (run here on CPU tensors): the returned norm bound lies in
    [lambda_max, lambda_max (1 + sqrt(tol))] -- never below the true value (the PDS step rule's safe
    side) and, with the stagnation exit guarded by the residual, never loose.  The 'cluster'
    spectrum (1500 eigenvalues in [0.999, 1]) converges slowly, so its theta stagnates long before the
    residual test passes."""
    import torch
    from pycsou_amd.core.linop import _lanczos_extreme
    rng = np.random.default_rng(3)
    if spectrum == 'cluster':
        ev = np.concatenate([rng.uniform(0.999, 1.0, 1500), rng.uniform(0, 0.5, 500)])
    else:
        ev = np.concatenate([[4.0], rng.uniform(0, 1.0, 1999)])
    d = torch.from_numpy(ev)
    tol = 1e-9
    lam = _lanczos_extreme(lambda q: d * q, d.numel(), tol=tol, device='cpu')
    top = float(ev.max())
    assert top * (1 - 1e-12) <= lam <= top * (1 + np.sqrt(tol)), (lam, top)


def test_graft_build_entry():
    """__graft_entry__.build() (the driver's build check, run on CPU) compiles and loads the library whose
    ABI the bindings expect -- a stale constant there failed it silently for part of round 6."""
    import __graft_entry__ as g
    g.build()


def test_l21_label_groups_csr():
    """The host side of pcs_prox_l21_groups: every group's members in ascending element order, the
    offsets of the groups in that list and the largest group (penalty.py:525-560 groups by np.unique)."""
    import numpy as np
    from pycsou_amd.func.penalty import L21Norm
    rng = np.random.default_rng(0)
    labels = rng.integers(0, 40, 1000) * 7 + 3  # arbitrary label values, some unused
    uniq, inv = np.unique(labels, return_inverse=True)
    order, off, maxlen = L21Norm._csr_host(inv, uniq.size)
    assert off[0] == 0 and off[-1] == labels.size and maxlen == np.bincount(inv).max()
    for g in range(uniq.size):
        members = order[off[g]:off[g + 1]]
        np.testing.assert_array_equal(members, np.flatnonzero(inv == g))  # ascending element order

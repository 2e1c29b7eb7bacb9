"""HIP kernels vs the oracle, operator by operator (through the C ABI).

Tolerances: fp64 kernels agree with the NumPy/SciPy oracle to <= 1e-12 relative (direct
convolution vs the reference's FFT path, FMA contraction); fp32 kernels to <= 2e-6
relative (single rounding per op).  Prox / projection kernels are compared
element-wise.
"""

import numpy as np
import pytest
import torch

from oracle import pylops1 as P
from oracle import pycsou_ref as OR
from tests.cases import load, rel

pytestmark = pytest.mark.gpu

TOL = {np.float64: 1e-12, np.float32: 2e-6}


def dev(a):
    return torch.as_tensor(np.ascontiguousarray(a)).cuda()


def host(t):
    return t.detach().cpu().numpy()


@pytest.fixture(scope='module')
def A():
    import pycsou_amd as pa
    from pycsou_amd import _ops
    return pa, _ops


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
@pytest.mark.parametrize('shape', [(64, 64), (63, 65), (2, 17), (5, 6, 7), (16, 17, 18), (129,), (3, 4, 5, 6),
                                   (2, 3, 3, 4, 5), (4, 3, 2, 3, 2, 3)])
@pytest.mark.parametrize('kind', ['forward', 'backward', 'centered'])
@pytest.mark.parametrize('edge', [True, False])
def test_gradient(A, dtype, shape, kind, edge):
    from pycsou_amd.linop.diff import Gradient
    rng = np.random.default_rng(0)
    steps = [1.0 + 0.25 * i for i in range(len(shape))]
    x = rng.standard_normal(int(np.prod(shape))).astype(dtype)
    ref = P.Gradient(shape, sampling=steps, edge=edge, kind=kind, dtype=np.float64)
    op = Gradient(shape, step=steps, edge=edge, kind=kind)
    y = op(x)
    assert y.dtype == dtype
    assert rel(y, ref.matvec(x.astype(np.float64))) < TOL[dtype]
    z = rng.standard_normal(op.shape[0]).astype(dtype)
    assert rel(op.adjoint(z), ref.rmatvec(z.astype(np.float64))) < TOL[dtype]


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
@pytest.mark.parametrize('axis', [0, 1, 2])
def test_first_derivative(A, dtype, axis):
    from pycsou_amd.linop.diff import FirstDerivative
    shape = (9, 10, 11)
    rng = np.random.default_rng(1)
    x = rng.standard_normal(990).astype(dtype)
    for kind in ['forward', 'backward', 'centered']:
        ref = P.FirstDerivative(990, dims=shape, dir=axis, sampling=0.5, edge=True, kind=kind)
        op = FirstDerivative(990, shape=shape, axis=axis, step=0.5, kind=kind)
        assert rel(op(x), ref.matvec(x.astype(np.float64))) < TOL[dtype]
        assert rel(op.adjoint(x), ref.rmatvec(x.astype(np.float64))) < TOL[dtype]


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
@pytest.mark.parametrize('axis', [0, 1, 2, 3])
def test_derivatives_4d(A, dtype, axis):
    """FirstDerivative / SecondDerivative of a 4-D array along each axis (PyLops 1.x takes any
    ndim; the kernels see the axis as the middle one of (outer, n, inner))."""
    from pycsou_amd.linop.diff import FirstDerivative, SecondDerivative
    shape = (5, 6, 7, 8)
    N = int(np.prod(shape))
    rng = np.random.default_rng(4 + axis)
    x = rng.standard_normal(N).astype(dtype)
    for kind in ['forward', 'backward', 'centered']:
        for edge in (True, False):
            ref = P.FirstDerivative(N, dims=shape, dir=axis, sampling=0.5, edge=edge, kind=kind)
            op = FirstDerivative(N, shape=shape, axis=axis, step=0.5, kind=kind, edge=edge)
            assert rel(op(x), ref.matvec(x.astype(np.float64))) < TOL[dtype]
            assert rel(op.adjoint(x), ref.rmatvec(x.astype(np.float64))) < TOL[dtype]
    for edge in (True, False):
        ref = P.SecondDerivative(N, dims=shape, dir=axis, sampling=1.5, edge=edge)
        op = SecondDerivative(N, shape=shape, axis=axis, step=1.5, edge=edge)
        assert rel(op(x), ref.matvec(x.astype(np.float64))) < TOL[dtype]
        assert rel(op.adjoint(x), ref.rmatvec(x.astype(np.float64))) < TOL[dtype]


def test_first_derivative_doctest(A):
    from pycsou_amd.linop.diff import FirstDerivative
    f = load('ops.npz')
    x = f['doc_d1_x']
    y = FirstDerivative(size=x.size) * x
    assert np.sum(np.abs(y) > 0) == 6
    np.testing.assert_allclose(y, f['doc_d1_y'])


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
@pytest.mark.parametrize('edge', [True, False])
def test_laplacian(A, dtype, edge):
    from pycsou_amd.linop.diff import Laplacian
    shape = (37, 45)
    rng = np.random.default_rng(2)
    x = rng.standard_normal(37 * 45).astype(dtype)
    ref = P.Laplacian(shape, weights=(1.0, 0.5), sampling=(1.0, 2.0), edge=edge)
    op = Laplacian(shape, weights=(1.0, 0.5), step=(1.0, 2.0), edge=edge)
    assert rel(op(x), ref.matvec(x.astype(np.float64))) < TOL[dtype]
    assert rel(op.adjoint(x), ref.rmatvec(x.astype(np.float64))) < TOL[dtype]


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
@pytest.mark.parametrize('kshape', [(15, 15), (4, 6), (7, 4), (1, 5), (9, 1), (31, 31), (40, 3)])
@pytest.mark.parametrize('shape', [(64, 64), (70, 33), (5, 200)])
def test_convolve2d(A, dtype, kshape, shape):
    from pycsou_amd.linop.conv import Convolve2D
    rng = np.random.default_rng(3)
    h = rng.standard_normal(kshape)
    N = shape[0] * shape[1]
    x = rng.standard_normal(N).astype(dtype)
    off = tuple(P.pycsou_offset(n) for n in kshape)
    ref = P.Convolve2D(N, h, shape, offset=off, method='direct')
    op = Convolve2D(N, h, shape)
    assert rel(op(x), ref.matvec(x.astype(np.float64))) < 10 * TOL[dtype]
    assert rel(op.adjoint(x), ref.rmatvec(x.astype(np.float64))) < 10 * TOL[dtype]


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
@pytest.mark.parametrize('k', [3, 5, 7, 9, 11, 13, 15, 31])
@pytest.mark.parametrize('shape', [(64, 64), (37, 130), (300, 7), (1, 1)])
def test_conv2d_raw_tiers(A, dtype, k, shape):
    """pcs_conv2d with an odd square centred PSF runs the marching correlation kernel with the
    PSF read flipped (forward) -- and its adjoint call (flipped PSF, mirrored offset); with the
    fused residual out = h*x - y."""
    from pycsou_amd import _lib as L
    lib = L.gpu()
    rng = np.random.default_rng(k)
    h = rng.standard_normal((k, k))
    N = shape[0] * shape[1]
    x = rng.standard_normal(N).astype(dtype)
    y = rng.standard_normal(N).astype(dtype)
    ref = P.Convolve2D(N, h, shape, offset=(k // 2, k // 2), method='direct')
    xd, yd, hd, hfd = dev(x), dev(y), dev(h.astype(dtype)), dev(h[::-1, ::-1].astype(dtype))
    out = torch.empty_like(xd)
    code = L.dtcode(xd)
    assert lib.pcs_conv2d(code, L.ptr(xd), L.ptr(out), shape[0], shape[1], L.ptr(hd), k, k, k // 2, k // 2, L.ptr(yd),
                          -1.0, L.stream()) == 0
    assert rel(host(out), ref.matvec(x.astype(np.float64)) - y) < 10 * TOL[dtype]
    assert lib.pcs_conv2d(code, L.ptr(xd), L.ptr(out), shape[0], shape[1], L.ptr(hfd), k, k, k // 2, k // 2, None,
                          0.0, L.stream()) == 0
    assert rel(host(out), ref.rmatvec(x.astype(np.float64))) < 10 * TOL[dtype]


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
@pytest.mark.parametrize('kshape', [(15, 15), (6, 11), (1, 30)])
@pytest.mark.parametrize('shape', [(1000, 4096), (517, 1023), (130, 64)])
def test_conv2d_planned_large(A, dtype, kshape, shape):
    """Packed-plan Convolve2D (pcs_conv2d_planned) at ragged and large sizes (many strip
    segments, partial last marching blocks, widths that are not 16-B multiples), forward,
    adjoint and the fused residual h*x - y, against the direct oracle."""
    from pycsou_amd.linop.conv import Convolve2D
    rng = np.random.default_rng(7)
    h = rng.standard_normal(kshape)
    N = shape[0] * shape[1]
    x = rng.standard_normal(N).astype(dtype)
    y = rng.standard_normal(N).astype(dtype)
    off = tuple(P.pycsou_offset(n) for n in kshape)
    ref = P.Convolve2D(N, h, shape, offset=off, method='fft')
    op = Convolve2D(N, h, shape)
    assert op.plan(torch.float32 if dtype == np.float32 else torch.float64, False) is not None
    xd, yd = dev(x), dev(y)
    x64 = x.astype(np.float64)
    tol = 10 * TOL[dtype] if dtype == np.float32 else 1e-11  # the oracle is SciPy FFT here
    assert rel(host(op._apply(xd)), ref.matvec(x64)) < tol
    assert rel(host(op._adj(xd)), ref.rmatvec(x64)) < tol
    assert rel(host(op._apply_minus(xd, yd)), ref.matvec(x64) - y) < tol


def test_conv2d_plan_pack(A):
    """Host packing: forward window = flipped zero-padded PSF centred at K/2, adjoint window =
    the padded PSF; tier choice and rejection of PSFs wider than 31."""
    from pycsou_amd import _lib as L
    lib = L.load()
    h = np.arange(1, 7, dtype=np.float64).reshape(2, 3)  # off = (0, 1)
    assert lib.pcs_conv2d_plan_tier(2, 3, 0, 1) == 3
    assert lib.pcs_conv2d_plan_tier(40, 3, 19, 1) == -3
    assert lib.pcs_conv2d_plan_tier(2, 3, 2, 1) == -1
    nb = lib.pcs_conv2d_plan_bytes(1, 2, 3, 0, 1)
    assert nb == 3 * 16 * 8
    for adj in (0, 1):
        buf = np.full(nb // 8, np.nan)
        assert lib.pcs_conv2d_plan_pack(1, h.ctypes.data_as(L._pdbl), 2, 3, 0, 1, adj, buf.ctypes.data) == 0
        wmat = buf.reshape(3, 16)
        assert np.all(wmat[:, 3:] == 0)
        hp = np.zeros((3, 3))
        hp[1:3, 0:3] = h  # h'[i + s0][j + s1], s0 = 1 - 0, s1 = 1 - 1
        np.testing.assert_array_equal(wmat[:, :3], hp if adj else hp[::-1, ::-1])


def test_convolve2d_doctest(A):
    from pycsou_amd.linop.conv import Convolve2D
    f = load('ops.npz')
    op = Convolve2D(size=10000, filter=f['doc_conv2d_h'], shape=(100, 100))
    np.testing.assert_allclose(op * f['doc_conv2d_x'], f['doc_conv2d_y'], atol=1e-12)


def test_convolve1d_doctest(A):
    from pycsou_amd.linop.conv import Convolve1D
    f = load('ops.npz')
    op = Convolve1D(size=30, filter=f['doc_conv1d_h'])
    np.testing.assert_allclose(op * f['doc_conv1d_x'], f['doc_conv1d_y'], atol=1e-14)


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
@pytest.mark.parametrize('axis', [0, 1, 2])
@pytest.mark.parametrize('k', [15, 4, 1, 20])
@pytest.mark.parametrize('dims', [(12, 13, 14), (20, 12, 24), (5, 3, 1100)])
def test_convolve1d_axis(A, dtype, axis, k, dims):
    """Odd shapes take the generic kernel; 16-B-aligned ones the strided / LDS-row kernels
    (k <= 15), including multi-segment rows (1100 columns)."""
    from pycsou_amd.linop.conv import Convolve1D
    N = int(np.prod(dims))
    rng = np.random.default_rng(4)
    h = rng.standard_normal(k)
    x = rng.standard_normal(N).astype(dtype)
    ref = P.Convolve1D(N, h, offset=P.pycsou_offset(k), dims=dims, dir=axis)
    op = Convolve1D(N, h, reshape_dims=dims, axis=axis)
    assert rel(op(x), ref.matvec(x.astype(np.float64))) < 10 * TOL[dtype]
    assert rel(op.adjoint(x), ref.rmatvec(x.astype(np.float64))) < 10 * TOL[dtype]


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
@pytest.mark.parametrize('axis', [0, 1, 2, 3])
@pytest.mark.parametrize('k', [5, 20])
def test_convolve1d_4d(A, dtype, axis, k):
    """Convolve1D along each axis of a 4-D array (16-B-aligned inner extent: the strided / LDS-row
    kernels for k <= 15, the generic kernel for k = 20)."""
    from pycsou_amd.linop.conv import Convolve1D
    dims = (3, 5, 6, 8)
    N = int(np.prod(dims))
    rng = np.random.default_rng(40 + axis)
    h = rng.standard_normal(k)
    x = rng.standard_normal(N).astype(dtype)
    ref = P.Convolve1D(N, h, offset=P.pycsou_offset(k), dims=dims, dir=axis)
    op = Convolve1D(N, h, reshape_dims=dims, axis=axis)
    assert rel(op(x), ref.matvec(x.astype(np.float64))) < 10 * TOL[dtype]
    assert rel(op.adjoint(x), ref.rmatvec(x.astype(np.float64))) < 10 * TOL[dtype]


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
@pytest.mark.parametrize('k,off', [(15, 7), (7, 3), (4, 1), (1, 0), (12, 9)])
@pytest.mark.parametrize('nsub,img,q', [(40, (5, 33), (5, 34)), (30, (0, 30), (0, 30)), (26, (-3, 40), (2, 25))])
def test_conv0_residual_adjoint(A, dtype, k, off, nsub, img, q):
    """pcs_conv0_residual_adjoint == axis-0 conv, residual on image planes, flipped-tap
    adjoint conv (NumPy restatement of the three pcs_conv1d/pcs_axpby passes)."""
    from pycsou_amd import _lib as L
    n1, n2 = 9, 12
    plane = n1 * n2
    rng = np.random.default_rng(k + nsub)
    h = rng.standard_normal(k)
    t = rng.standard_normal((nsub, plane))
    y = rng.standard_normal((nsub, plane))

    def conv0(v, taps, o):  # out[i] = sum_j taps[j] v[i + o - j], zero outside
        out = np.zeros_like(v)
        for i in range(nsub):
            for j in range(len(taps)):
                src = i + o - j
                if 0 <= src < nsub:
                    out[i] += taps[j] * v[src]
        return out
    r = conv0(t, h, off) - y
    lo, hi = max(img[0], 0), min(img[1], nsub)
    r[:lo] = 0
    r[hi:] = 0
    s_ref = conv0(r, h[::-1], k - 1 - off)
    td, yd, hd = dev(t.astype(dtype)), dev(y.astype(dtype)), dev(h.astype(dtype))
    sd = torch.full((nsub, plane), float('nan'), dtype=td.dtype, device='cuda')
    rc = L.load().pcs_conv0_residual_adjoint(L.dtcode(td), L.ptr(td), L.ptr(yd), L.ptr(sd), nsub, plane, L.ptr(hd), k,
                                             off, img[0], img[1], q[0], q[1], L.stream())
    assert rc == 0
    got = host(sd)
    assert np.isnan(got[:q[0]]).all() and np.isnan(got[q[1]:]).all()  # only [q0, q1) written
    assert rel(got[q[0]:q[1]], s_ref[q[0]:q[1]]) < 10 * TOL[dtype]


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
@pytest.mark.parametrize('ka,offa,kb,offb', [(15, 7, 15, 7), (7, 3, 5, 2), (4, 1, 12, 9), (1, 0, 15, 14)])
@pytest.mark.parametrize('dims', [(3, 40, 72), (2, 33, 130), (1, 5, 7)])
@pytest.mark.parametrize('vfirst', [1, 0])
def test_conv2d_sep_planes(A, dtype, ka, offa, kb, offb, dims, vfirst):
    """pcs_conv2d_sep_planes == the two pcs_conv1d passes (axis 1, axis 2) in the same order,
    bit for bit (same per-output sums); odd widths take the scalar staging path."""
    from pycsou_amd import _lib as L
    rng = np.random.default_rng(ka * 31 + kb)
    x = dev(rng.standard_normal(dims).astype(dtype))
    ha, hb = dev(rng.standard_normal(ka).astype(dtype)), dev(rng.standard_normal(kb).astype(dtype))
    lib, st = L.load(), L.stream()
    t1, ref, out = torch.empty_like(x), torch.empty_like(x), torch.empty_like(x)
    d = L.i64s(dims)
    order = [(1, ha, ka, offa), (2, hb, kb, offb)] if vfirst else [(2, hb, kb, offb), (1, ha, ka, offa)]
    (a0, h0, k0, o0), (a1, h1, k1, o1) = order
    assert lib.pcs_conv1d(L.dtcode(x), L.ptr(x), L.ptr(t1), 3, d, a0, L.ptr(h0), k0, o0, st) == 0
    assert lib.pcs_conv1d(L.dtcode(x), L.ptr(t1), L.ptr(ref), 3, d, a1, L.ptr(h1), k1, o1, st) == 0
    assert lib.pcs_conv2d_sep_planes(L.dtcode(x), L.ptr(x), L.ptr(out), dims[0], dims[1], dims[2], L.ptr(ha), ka,
                                     offa, L.ptr(hb), kb, offb, vfirst, st) == 0
    torch.cuda.synchronize()
    assert rel(host(out), host(ref)) < TOL[dtype]


def test_separable_factorisation(A):
    from pycsou_amd.linop.conv import Convolve2D
    for (kh, kw) in [(15, 15), (4, 6), (7, 3)]:
        c = np.exp(-np.linspace(-2, 2, kh) ** 2)
        r = np.exp(-np.linspace(-1, 1.5, kw) ** 2)
        op = Convolve2D(64 * 64, np.outer(c, r), (64, 64))
        t0, t1, half = op.separable()
        # rebuild the centred filter and compare to the PSF placed by its offsets
        full = np.outer(t0, t1)
        o0, o1 = op.off
        np.testing.assert_allclose(full[half - o0:half - o0 + kh, half - o1:half - o1 + kw], op.filter, atol=1e-14)
        assert abs(full.sum() - op.filter.sum()) < 1e-12
    assert Convolve2D(64 * 64, np.random.default_rng(0).standard_normal((5, 5)), (64, 64)).separable() is None


# ---------------------------------------------------------------- prox / functionals vs reference fixtures

def test_prox_vs_reference_fixtures(A):
    from pycsou_amd.func.penalty import L1Norm, L2Norm, L21Norm, SquaredL2Norm, NonNegativeOrthant, Segment
    f = load('prox.npz')
    x, vz, groups = f['x'], f['vz'], f['groups']
    np.testing.assert_allclose(L1Norm(200).prox(x, 0.7), f['l1_prox_07'], atol=1e-15)
    np.testing.assert_allclose(L1Norm(200)(x), f['l1_value'], rtol=1e-14)
    np.testing.assert_allclose(L2Norm(200).prox(x, 3.0), f['l2_prox_3'], rtol=1e-13, atol=1e-15)
    np.testing.assert_allclose(L2Norm(200).prox(x, 30.0), f['l2_prox_30'], atol=1e-15)
    l21 = L21Norm(dim=200, groups=groups)
    np.testing.assert_allclose(l21.prox(x, 0.5), f['l21_prox_05'], rtol=1e-13, atol=1e-15)
    np.testing.assert_allclose(l21(x), f['l21_value'], rtol=1e-13)
    l21p = L21Norm(dim=200, groups=np.tile(np.arange(100), 2))
    assert l21p.pixel_d == 2
    np.testing.assert_allclose(l21p.prox(vz, 0.5), f['l21pix_prox_05'], rtol=1e-13, atol=1e-15)
    np.testing.assert_allclose(l21p(vz), f['l21pix_value'], rtol=1e-13)
    np.testing.assert_allclose((0.3 * L1Norm(200)).fenchel_prox(x, 0.7), f['fenchel_l1_lam03_s07'], atol=1e-15)
    np.testing.assert_allclose((0.3 * l21p).fenchel_prox(vz, 0.7), f['fenchel_l21pix_lam03_s07'], rtol=1e-13,
                               atol=1e-15)
    np.testing.assert_allclose(SquaredL2Norm(200)(x), f['sql2_value'], rtol=1e-13)
    np.testing.assert_array_equal(SquaredL2Norm(200).gradient(x), f['sql2_grad'])
    np.testing.assert_array_equal(NonNegativeOrthant(200).prox(x, 1.0), f['nonneg'])
    np.testing.assert_array_equal(Segment(200, a=-0.5, b=0.25).prox(x, 1.0), f['segment'])
    np.testing.assert_allclose(SquaredL2Norm(200).prox(x, 0.25), x / 1.5, rtol=1e-15)


def test_reference_doctests(A):
    from pycsou_amd.func.penalty import L1Norm, L2Norm, L21Norm, SquaredL2Norm
    from pycsou_amd.math.prox import soft
    x = np.arange(10, dtype=np.float64)
    assert L1Norm(10)(x) == 45.0
    assert abs(L2Norm(10)(x) - 16.881943016134134) < 1e-14
    assert abs(L21Norm(10, groups=np.concatenate((np.ones(5), 2 * np.ones(5))))(x) - 21.44594499772297) < 1e-13
    assert abs(SquaredL2Norm(10)(x) - 285.00000000000006) < 1e-12
    np.testing.assert_array_equal(soft(np.linspace(-1, 1, 5), 0.5), [-0.5, -0., 0., 0., 0.5])
    # prox calculus identities (pycsou/core/functional.py:122-132)
    f = L1Norm(10)
    np.testing.assert_allclose((2 * f).prox(x, 0.1), f.prox(x, 0.2))
    np.testing.assert_allclose((f * 2).prox(x, 0.1), f.prox(2 * x, 0.4) / 2)
    np.testing.assert_allclose(f.shifter(x).prox(x, 0.1), f.prox(x + x, 0.1) - x)


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
def test_prox_large_fp32(A, dtype):
    from pycsou_amd import _ops
    rng = np.random.default_rng(5)
    n = 1 << 20
    x = rng.standard_normal(2 * n).astype(dtype)
    t = dev(x)
    np.testing.assert_allclose(host(_ops.prox_l1(t, 0.3)), OR.prox_l1(x.copy(), dtype(0.3)), rtol=0,
                               atol=4 * np.finfo(dtype).eps)
    got = host(_ops.fenchel_l21_pixel(t, 0.7, 0.2, 2))
    want = OR.fenchel_prox(OR.postcomp(lambda v, s: OR.prox_l21_pixel(v, s, 2), 0.2), x.astype(np.float64), 0.7)
    assert rel(got, want) < TOL[dtype]


def test_reductions(A):
    from pycsou_amd import _ops
    rng = np.random.default_rng(6)
    x = rng.standard_normal(3_000_001)
    y = rng.standard_normal(3_000_001)
    tx, ty = dev(x), dev(y)
    assert abs(_ops.reduce_dev(0, tx).item() - np.dot(x, x)) < 1e-9 * np.dot(x, x)
    assert abs(_ops.reduce_dev(1, tx).item() - np.abs(x).sum()) < 1e-9 * np.abs(x).sum()
    assert abs(_ops.reduce_dev(2, tx, ty).item() - np.sum((x - y) ** 2)) < 1e-9 * np.sum((x - y) ** 2)
    assert abs(_ops.reduce_dev(3, tx, ty).item() - np.dot(x, y)) < 1e-8 * np.sqrt(np.dot(x, x) * np.dot(y, y))
    # deterministic: same bits twice
    assert _ops.reduce_dev(0, tx).item() == _ops.reduce_dev(0, tx).item()
    assert _ops.reduce_dev(0, dev(np.zeros(0))).item() == 0.0


def test_abi_errors(A):
    from pycsou_amd import _lib as L
    lib = L.gpu()
    t = torch.zeros(16, device='cuda')
    assert lib.pcs_grad_fwd(7, L.ptr(t), L.ptr(t), 2, L.i64s([4, 4]), L.dbls([1, 1]), 0, 1, L.stream()) == -1
    # any ndim up to 32 (no launch for these: 33 axes, or an empty axis)
    assert lib.pcs_grad_fwd(0, L.ptr(t), L.ptr(t), 33, L.i64s([1] * 33), L.dbls([1] * 33), 0, 1, L.stream()) == -1
    assert lib.pcs_grad_fwd(0, L.ptr(t), L.ptr(t), 4, L.i64s([1, 0, 4, 4]), L.dbls([1] * 4), 0, 1, L.stream()) == -1
    assert lib.pcs_deriv1_fwd(0, L.ptr(t), L.ptr(t), 4, L.i64s([1, 1, 4, 4]), 4, 1.0, 0, 1, L.stream()) == -1
    assert lib.pcs_conv2d(0, L.ptr(t), L.ptr(t), 4, 4, L.ptr(t), 3, 3, 3, 1, None, 0.0, L.stream()) == -1
    with pytest.raises(L.HipError):
        L.check(lib.pcs_prox_l1(0, None, L.ptr(t), 16, 1.0, L.stream()), 'pcs_prox_l1')


def test_lipschitz_lanczos(A):
    from pycsou_amd.linop.diff import Gradient
    from pycsou_amd.linop.conv import Convolve2D
    G = Gradient((32, 40), kind='forward')
    G.compute_lipschitz_cst()
    # ||grad_fwd||^2 on a grid = 4 sin^2(pi (n0-1)/(2 n0)) + 4 sin^2(pi (n1-1)/(2 n1))
    exact = np.sqrt(4 * np.sin(np.pi * 31 / 64) ** 2 + 4 * np.sin(np.pi * 39 / 80) ** 2)
    assert abs(G.lipschitz_cst - exact) < 1e-6 * exact
    assert G.lipschitz_cst >= exact * (1 - 1e-12)
    h = OR.gaussian_psf(7, 1.5)
    C = Convolve2D(64 * 64, h, (64, 64))
    C.compute_lipschitz_cst()
    dense = np.stack([P.Convolve2D(4096, h, (64, 64), offset=(3, 3)).matvec(e) for e in np.eye(4096)[:: 1]]).T
    assert abs(C.lipschitz_cst - np.linalg.norm(dense, 2)) < 1e-6
    assert C.lipschitz_cst >= np.linalg.norm(dense, 2) * (1 - 1e-12)


@pytest.mark.parametrize('case', ['grad2d_4096', 'conv2d_4096', 'grad3d_512'])
def test_lipschitz_scalable(A, case):
    """compute_lipschitz_cst at the benchmark sizes (f1): bounded memory (a few vectors of the
    domain, however large the operator) and the analytic constants bench.py used to hard-code:
    never below them (Ritz value + residual bound), at most 1e-5 above.  For the blur: nonnegative PSF of unit sum, so ||C|| <= 1 and the top
    singular vector is smooth -- ||C|| = 1 up to the O((pi sigma / n)^2) boundary loss."""
    from pycsou_amd.linop.conv import Convolve2D
    from pycsou_amd.linop.diff import Gradient
    if case == 'grad3d_512':
        n = 512
        op = Gradient((n, n, n), kind='forward')
        exact = np.sqrt(3 * 4 * np.sin(np.pi * (n - 1) / (2 * n)) ** 2)
        N, tol = n ** 3, 1e-5
    elif case == 'grad2d_4096':
        n = 4096
        op = Gradient((n, n), kind='forward')
        exact = np.sqrt(2 * 4 * np.sin(np.pi * (n - 1) / (2 * n)) ** 2)
        N, tol = n * n, 1e-5
    else:
        n = 4096
        op = Convolve2D(n * n, OR.gaussian_psf(15, 2.0), (n, n))
        exact, N, tol = 1.0, n * n, 1e-5
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    op.compute_lipschitz_cst()
    torch.cuda.synchronize()
    extra = torch.cuda.max_memory_allocated() - base
    # an upper estimate (Ritz value + residual bound): step sizes from it respect tau sigma ||K||^2 <= 1
    # (the closed forms of the gradients are exact; the blur's 1.0 is itself an upper bound)
    if case != 'conv2d_4096':
        assert op.lipschitz_cst >= exact * (1 - 1e-12), (op.lipschitz_cst, exact)
    assert abs(op.lipschitz_cst - exact) <= tol * exact, (op.lipschitz_cst, exact)
    d = op.shape[0] // N
    assert extra <= (4 + d + 1) * N * 8, extra / (N * 8)


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
@pytest.mark.parametrize('ka,offa,kb,offb', [(15, 7, 15, 7), (15, 14, 15, 0), (6, 2, 9, 8)])
@pytest.mark.parametrize('dims', [(4, 200, 264), (2, 1100, 128), (9, 17, 36), (3, 150, 131), (40, 64, 256)])
def test_conv2d_sep_planes_march(A, dtype, ka, offa, kb, offb, dims):
    """The row-marching H-first kernel (ranges crossing planes and strips, ragged last strip,
    odd widths) == pcs_conv1d along axis 2 then axis 1 (same tap order; the rounding of the
    contiguous-axis kernel differs by an ulp here and there)."""
    from pycsou_amd import _lib as L
    rng = np.random.default_rng(ka * 7 + kb + dims[2])
    x = dev(rng.standard_normal(dims).astype(dtype))
    ha, hb = dev(rng.standard_normal(ka).astype(dtype)), dev(rng.standard_normal(kb).astype(dtype))
    lib, st = L.load(), L.stream()
    t1, ref = torch.empty_like(x), torch.empty_like(x)
    out = torch.full_like(x, float('nan'))
    d = L.i64s(dims)
    assert lib.pcs_conv1d(L.dtcode(x), L.ptr(x), L.ptr(t1), 3, d, 2, L.ptr(hb), kb, offb, st) == 0
    assert lib.pcs_conv1d(L.dtcode(x), L.ptr(t1), L.ptr(ref), 3, d, 1, L.ptr(ha), ka, offa, st) == 0
    assert lib.pcs_conv2d_sep_planes(L.dtcode(x), L.ptr(x), L.ptr(out), dims[0], dims[1], dims[2], L.ptr(ha), ka,
                                     offa, L.ptr(hb), kb, offb, 0, st) == 0
    torch.cuda.synchronize()
    assert not torch.isnan(out).any()  # every output written
    assert rel(host(out), host(ref)) < TOL[dtype]


def _c1_np(x, h, off, axis):
    """out[i] = sum_t h[t] x[i + off - t] along `axis`, zero outside (pcs_conv1d's definition)."""
    out = np.zeros_like(x)
    n = x.shape[axis]
    for t, ht in enumerate(h):
        s = off - t
        lo, hi = max(0, -s), min(n, n - s)
        if lo >= hi:
            continue
        dst = [slice(None)] * x.ndim
        src = [slice(None)] * x.ndim
        dst[axis], src[axis] = slice(lo, hi), slice(lo + s, hi + s)
        out[tuple(dst)] += ht * x[tuple(src)]
    return out


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
@pytest.mark.parametrize('ka,offa,kb,offb', [(15, 7, 15, 7), (15, 14, 15, 0), (6, 2, 9, 8), (3, 0, 5, 1), (1, 0, 2, 1)])
@pytest.mark.parametrize('dims', [(4, 200, 264), (2, 1100, 128), (9, 17, 36), (3, 70, 4), (1, 5, 8), (12, 64, 256),
                                  (600, 64, 64), (40, 300, 260)])
def test_conv2d_sep_ata_planes(A, dtype, ka, offa, kb, offb, dims):
    """pcs_conv2d_sep_ata_planes == C_a^T C_b^T C_b C_a per plane (four Convolve1D passes in
    NumPy, fp64): ragged strips and row segments, planes thinner than the 28-row vertical reach,
    offsets that need the horizontal tap padding (kb=5, offb=1); more tasks than resident workgroups
    (600 planes: one task per workgroup, later ones start as earlier ones finish)."""
    from pycsou_amd import _lib as L
    rng = np.random.default_rng(ka * 7 + kb + dims[2] + dims[1])
    xn = rng.standard_normal(dims)
    ha_n, hb_n = rng.standard_normal(ka), rng.standard_normal(kb)
    ref = _c1_np(_c1_np(xn, ha_n, offa, 1), hb_n, offb, 2)
    ref = _c1_np(_c1_np(ref, hb_n[::-1], kb - 1 - offb, 2), ha_n[::-1], ka - 1 - offa, 1)
    x = dev(xn.astype(dtype))
    ha, hb = dev(ha_n.astype(dtype)), dev(hb_n.astype(dtype))
    out = torch.full_like(x, float('nan'))
    lib, st = L.load(), L.stream()
    assert lib.pcs_conv2d_sep_ata_planes(L.dtcode(x), L.ptr(x), L.ptr(out), dims[0], dims[1], dims[2], L.ptr(ha), ka,
                                         offa, L.ptr(hb), kb, offb, st) == 0
    torch.cuda.synchronize()
    assert not torch.isnan(out).any()  # every output written
    assert rel(host(out), ref) < 10 * TOL[dtype]


def test_conv2d_sep_ata_planes_unsupported(A):
    """Layouts the strip kernel does not take return PCS_EUNSUPPORTED (-3) without launching:
    odd widths, and a 15-tap horizontal filter whose offset is 1 mod 4 (no padding freedom)."""
    from pycsou_amd import _lib as L
    x = torch.zeros((2, 16, 20), dtype=torch.float64, device='cuda')
    h = torch.ones(15, dtype=torch.float64, device='cuda')
    lib, st = L.load(), L.stream()
    assert lib.pcs_conv2d_sep_ata_planes(L.PCS_F64, L.ptr(x), L.ptr(x.clone()), 2, 16, 20, L.ptr(h), 15, 7, L.ptr(h), 15,
                                         5, st) == -3
    y = torch.zeros((2, 16, 21), dtype=torch.float64, device='cuda')
    assert lib.pcs_conv2d_sep_ata_planes(L.PCS_F64, L.ptr(y), L.ptr(y.clone()), 2, 16, 21, L.ptr(h), 15, 7, L.ptr(h), 15,
                                         7, st) == -3


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
@pytest.mark.parametrize('gkind', ['null', 'l1', 'nonneg', 'segment'])
@pytest.mark.parametrize('n', [1, 1000, 300001])
def test_apgd_step(A, dtype, gkind, n):
    """pcs_apgd_step == the reference update (proxalgs.py:586-601) restated in NumPy:
    x_t = G.prox(x - tau g, tau), x' = x_t + a (x_t - aux), and the two diagnostics norms."""
    from oracle import pycsou_ref as OR
    from pycsou_amd import _lib as L
    _, O = A
    rng = np.random.default_rng(n)
    x, g, aux = (rng.standard_normal(n).astype(dtype) for _ in range(3))
    tau, a, lam, seg = 0.37, 0.61, 0.8, (-0.25, 0.5)
    v = x.astype(np.float64) - tau * g.astype(np.float64)
    if gkind == 'l1':
        xt = OR.prox_l1(v, tau * lam)
    elif gkind == 'nonneg':
        xt = np.maximum(v, 0)
    elif gkind == 'segment':
        xt = np.clip(v, *seg)
    else:
        xt = v
    xn_ref = xt + a * (xt - aux)
    kind = {'null': L.PCS_G_NULL, 'l1': L.PCS_APGD_G_L1, 'nonneg': L.PCS_G_NONNEG, 'segment': L.PCS_G_SEGMENT}[gkind]
    xn, xtd, sums = O.apgd_step(dev(x), dev(g), dev(aux), tau, a, kind, lam, seg)
    tol = 10 * TOL[dtype]
    assert rel(host(xtd), xt) < tol and rel(host(xn), xn_ref) < tol
    d2, n2 = host(sums)
    xn_h = host(xn).astype(np.float64)
    assert abs(d2 - np.sum((x.astype(np.float64) - xn_h) ** 2)) <= 1e-9 * max(1.0, d2)
    assert abs(n2 - np.sum(x.astype(np.float64) ** 2)) <= 1e-9 * n2


def test_convolve1d_lipschitz_doctest(A):
    """Known answers of core/linop.py:262-266 and 299-303 (Convolve1D of a half-zeroed 5-tap
    Hann window on a 30-sample signal): three largest singular values round to 0.5 and the
    Lipschitz constant rounds to 0.5."""
    from scipy import signal
    from pycsou_amd.linop.conv import Convolve1D
    sig = np.repeat([0., 1., 0.], 10)
    filt = signal.windows.hann(5)
    filt[filt.size // 2:] = 0
    op = Convolve1D(size=sig.size, filter=filt)
    np.testing.assert_array_equal(np.round(op.singularvals(k=3, which='LM', tol=1e-3), 2), [0.5, 0.5, 0.5])
    op.compute_lipschitz_cst(tol=1e-2)
    assert np.round(op.lipschitz_cst, 1) == 0.5

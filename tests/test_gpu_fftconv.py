"""FFT-domain Convolve2D (pcs_fftconv2d: rocFFT on the zero-padded grid) for PSFs wider than the
direct correlation's 31 taps -- pycsou/linop/conv.py:167-295 with the reference default
method='fft' (scipy.signal.fftconvolve, mode 'same' at pycsou's offset).

Checked against scipy.signal.convolve(mode='same') (odd PSFs: offset K//2) and the oracle's
restatement (even PSFs: offset K//2 - 1), forward and adjoint, fp64 to 1e-12 and fp32 to 2e-6
relative; the adjoint by a dot test; a PDS deconvolution with a 41 x 41 PSF through the fused
engine's gradient buffer against the generic path.
"""

import numpy as np
import pytest
import torch

from oracle import pylops1 as P
from tests.cases import rel

pytestmark = pytest.mark.gpu


def _psf(kh, kw, seed):
    rng = np.random.default_rng(seed)
    r0, r1 = np.arange(kh) - (kh - 1) / 2, np.arange(kw) - (kw - 1) / 2
    yy, xx = np.meshgrid(r0, r1, indexing='ij')
    h = np.exp(-0.5 * ((xx * 0.8 + yy * 0.6) ** 2 / 60.0 + (yy * 0.8 - xx * 0.6) ** 2 / 12.0))
    h += 0.05 * rng.uniform(0, 1, (kh, kw))  # non-separable, no symmetry
    return h / h.sum()


@pytest.mark.parametrize('shape, k', [((300, 260), (63, 63)), ((257, 1000), (33, 47)), ((96, 70), (64, 40)),
                                      ((40, 37), (63, 63))])
@pytest.mark.parametrize('dtype', [np.float64, np.float32])
def test_fftconv_vs_reference(shape, k, dtype):
    from scipy import signal

    from pycsou_amd.linop.conv import Convolve2D
    h = _psf(*k, seed=k[0])
    N = shape[0] * shape[1]
    C = Convolve2D(N, h, shape)
    assert C.plan(torch.float64, False) is None, 'PSF wider than the direct tiers: the FFT path'
    x = np.random.default_rng(1).standard_normal(N)
    off = tuple(P.pycsou_offset(n) for n in k)
    ref_op = P.Convolve2D(N, h, shape, offset=off)
    fwd_ref, adj_ref = ref_op.matvec(x), ref_op.rmatvec(x)
    if k[0] % 2 and k[1] % 2:  # centred: scipy's 'same'
        np.testing.assert_allclose(fwd_ref, signal.convolve(x.reshape(shape), h, mode='same').ravel(), rtol=0,
                                   atol=1e-12 * np.abs(fwd_ref).max())
    xd = torch.as_tensor(x.astype(dtype)).cuda()
    fwd = C(xd).cpu().numpy()
    adj = C.adjoint(xd).cpu().numpy()
    tol = 1e-12 if dtype == np.float64 else 2e-6
    assert fwd.dtype == dtype and adj.dtype == dtype
    assert rel(fwd, fwd_ref) < tol, rel(fwd, fwd_ref)
    assert rel(adj, adj_ref) < tol, rel(adj, adj_ref)


@pytest.mark.parametrize('block', [64, 100])
@pytest.mark.parametrize('shape, k', [((300, 260), (63, 63)), ((257, 1000), (33, 47)), ((96, 70), (64, 40))])
@pytest.mark.parametrize('dtype', [np.float64, np.float32])
def test_fftconv_blocked_vs_reference(shape, k, dtype, block, monkeypatch):
    """The overlap-add block path (the default once an axis exceeds 2048 samples, e.g. 4096^2):
    PCS_FFT_BLOCK set small when the plan is created, so 2 x 2 and larger block grids with uneven
    last blocks run -- multi-block pad, the crop's block-candidate sums, the adjoint's negative
    offsets -- forward and adjoint against the oracle."""
    from pycsou_amd.linop.conv import Convolve2D
    monkeypatch.setenv('PCS_FFT_BLOCK', str(block))
    h = _psf(*k, seed=k[0] + 1)
    N = shape[0] * shape[1]
    C = Convolve2D(N, h, shape)  # plan created below, with the block override in the environment
    x = np.random.default_rng(4).standard_normal(N)
    ref_op = P.Convolve2D(N, h, shape, offset=tuple(P.pycsou_offset(n) for n in k))
    xd = torch.as_tensor(x.astype(dtype)).cuda()
    fwd = C(xd).cpu().numpy()
    adj = C.adjoint(xd).cpu().numpy()
    tol = 1e-12 if dtype == np.float64 else 3e-6
    assert rel(fwd, ref_op.matvec(x)) < tol, rel(fwd, ref_op.matvec(x))
    assert rel(adj, ref_op.rmatvec(x)) < tol, rel(adj, ref_op.rmatvec(x))
    # residual form through the blocks too
    y = torch.as_tensor(np.random.default_rng(5).standard_normal(N).astype(dtype)).cuda()
    r = C._apply_minus(xd, y).cpu().numpy()
    assert rel(r, fwd - y.cpu().numpy()) < tol


@pytest.mark.parametrize('block', [64, 100])
def test_fftconv_blocked_adjoint_dot_test(block, monkeypatch):
    from pycsou_amd.linop.conv import Convolve2D
    monkeypatch.setenv('PCS_FFT_BLOCK', str(block))
    shape, h = (130, 190), _psf(63, 35, seed=3)
    N = shape[0] * shape[1]
    C = Convolve2D(N, h, shape)
    rng = np.random.default_rng(2)
    u, v = torch.as_tensor(rng.standard_normal(N)).cuda(), torch.as_tensor(rng.standard_normal(N)).cuda()
    lhs = float(torch.dot(C(u), v))
    rhs = float(torch.dot(u, C.adjoint(v)))
    assert abs(lhs - rhs) <= 1e-12 * max(abs(lhs), 1.0)


def test_fftconv_apply_validates_buffers():
    """A wrong-length, non-contiguous or wrong-dtype buffer is a ValueError before any device call."""
    from pycsou_amd.linop.conv import Convolve2D
    shape = (64, 80)
    N = shape[0] * shape[1]
    f = Convolve2D(N, _psf(41, 41, seed=1), shape).fft(torch.float64)
    x = torch.zeros(N, dtype=torch.float64, device='cuda')
    with pytest.raises(ValueError):
        f.apply(torch.zeros(N - 1, dtype=torch.float64, device='cuda'))
    with pytest.raises(ValueError):
        f.apply(x, out=torch.zeros(2 * N, dtype=torch.float64, device='cuda')[::2])
    with pytest.raises(ValueError):
        f.apply(x, b=torch.zeros(N + 4, dtype=torch.float64, device='cuda'), beta=-1.0)
    with pytest.raises(ValueError):
        f.apply(x, out=torch.zeros(N, dtype=torch.float32, device='cuda'))


def test_fftconv_adjoint_dot_test():
    from pycsou_amd.linop.conv import Convolve2D
    shape, h = (130, 190), _psf(63, 35, seed=3)
    N = shape[0] * shape[1]
    C = Convolve2D(N, h, shape)
    rng = np.random.default_rng(2)
    u, v = torch.as_tensor(rng.standard_normal(N)).cuda(), torch.as_tensor(rng.standard_normal(N)).cuda()
    lhs = float(torch.dot(C(u), v))
    rhs = float(torch.dot(u, C.adjoint(v)))
    assert abs(lhs - rhs) <= 1e-12 * max(abs(lhs), 1.0)


def test_fftconv_residual_form():
    """Conv x - y in one call (the data-fidelity residual the PDS gradient buffer uses)."""
    from pycsou_amd.linop.conv import Convolve2D
    shape, h = (150, 128), _psf(45, 45, seed=4)
    N = shape[0] * shape[1]
    C = Convolve2D(N, h, shape)
    rng = np.random.default_rng(5)
    x, y = torch.as_tensor(rng.standard_normal(N)).cuda(), torch.as_tensor(rng.standard_normal(N)).cuda()
    r = C._apply_minus(x, y)
    assert rel(r.cpu().numpy(), (C(x) - y).cpu().numpy()) < 1e-14


@pytest.mark.parametrize('kind', ['forward', 'centered'])
def test_pds_large_psf_fused_vs_generic(kind):
    """PDS TV deconvolution with a 41 x 41 non-separable PSF: grad F through the FFT plan into the
    fused engine's gradient buffer (GRADBUF) against the generic per-operator path, fp64."""
    from pycsou_amd.func.loss import SquaredL2Loss
    from pycsou_amd.func.penalty import L21Norm
    from pycsou_amd.linop.conv import Convolve2D
    from pycsou_amd.linop.diff import Gradient
    from pycsou_amd.opt.proxalgs import PDS
    shape = (96, 128)
    N = shape[0] * shape[1]
    h = _psf(41, 41, seed=6)
    y = np.random.default_rng(7).uniform(0, 1, N)
    out = {}
    for mode in ('fused', 'generic'):
        C = Convolve2D(N, h, shape)
        C.lipschitz_cst = C.diff_lipschitz_cst = 1.0
        K = Gradient(shape, kind=kind)
        K.lipschitz_cst = K.diff_lipschitz_cst = np.sqrt(8.0)
        pds = PDS(dim=N, F=(1 / 2) * SquaredL2Loss(dim=N, data=y) * C,
                  H=0.05 * L21Norm(dim=2 * N, groups=np.tile(np.arange(N), 2)), K=K, x0=np.zeros(N), z0=np.zeros(2 * N),
                  max_iter=9, min_iter=9, accuracy_threshold=0.0, verbose=None, engine=mode)
        est, _, _ = pds.iterate()
        assert (pds._engine is not None) == (mode == 'fused')
        out[mode] = est
    assert rel(out['fused']['primal_variable'], out['generic']['primal_variable']) < 1e-11
    assert rel(out['fused']['dual_variable'], out['generic']['dual_variable']) < 1e-11

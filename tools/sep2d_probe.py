"""Time pcs_conv2d_sep_planes (both orders) against the two pcs_conv1d passes on a 512^3 fp32
volume (diagnostics; PCS_SEP2D_BLOCKS overrides the persistent grid)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pycsou_amd import _lib as L  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    n = int(os.environ.get('PCS_N', '512'))
    dt = torch.float64 if os.environ.get('PCS_DTYPE') == 'f64' else torch.float32
    lib, st = L.load(), L.stream()
    x = torch.randn(n, n, n, device='cuda', dtype=dt)
    y, t = torch.empty_like(x), torch.empty_like(x)
    h = torch.randn(15, device='cuda', dtype=dt)
    d = L.i64s((n, n, n))
    code = L.dtcode(x)
    us = {
        'sep2d_vfirst': timeit(lambda: lib.pcs_conv2d_sep_planes(code, L.ptr(x), L.ptr(y), n, n, n, L.ptr(h), 15, 7,
                                                                 L.ptr(h), 15, 7, 1, st)),
        'sep2d_hfirst': timeit(lambda: lib.pcs_conv2d_sep_planes(code, L.ptr(x), L.ptr(y), n, n, n, L.ptr(h), 15, 7,
                                                                 L.ptr(h), 15, 7, 0, st)),
        'conv1d_axis1': timeit(lambda: lib.pcs_conv1d(code, L.ptr(x), L.ptr(t), 3, d, 1, L.ptr(h), 15, 7, st)),
        'conv1d_axis2': timeit(lambda: lib.pcs_conv1d(code, L.ptr(x), L.ptr(t), 3, d, 2, L.ptr(h), 15, 7, st)),
        'conv1d_axis0': timeit(lambda: lib.pcs_conv1d(code, L.ptr(x), L.ptr(t), 3, d, 0, L.ptr(h), 15, 7, st)),
        'copy': timeit(lambda: y.copy_(x)),
    }
    gb = 2 * x.numel() * x.element_size() / 1e9
    print(os.environ.get('PCS_SEP2D_BLOCKS', 'default'),
          {k: f'{v:.0f}us {gb / (v * 1e-6) / 1e3:.2f}TB/s' for k, v in us.items()}, flush=True)


if __name__ == '__main__':
    main()

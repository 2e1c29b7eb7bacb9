"""Time the H-first pcs_conv2d_sep_planes on a volume against a plain copy (diagnostics).
PCS_N (edge, default 512), PCS_DTYPE (f32 / f64); PCS_SEP2D_TILE=1 selects the tile kernel."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pycsou_amd import _lib as L  # noqa: E402
from tools.sep2d_probe import timeit  # noqa: E402


def main():
    n = int(os.environ.get('PCS_N', '512'))
    dt = torch.float64 if os.environ.get('PCS_DTYPE') == 'f64' else torch.float32
    lib, st = L.load(), L.stream()
    x = torch.randn(n, n, n, device='cuda', dtype=dt)
    y = torch.empty_like(x)
    h = torch.randn(15, device='cuda', dtype=dt)
    code = L.dtcode(x)
    us = {'sep2d_hfirst': timeit(lambda: lib.pcs_conv2d_sep_planes(code, L.ptr(x), L.ptr(y), n, n, n, L.ptr(h), 15, 7,
                                                                   L.ptr(h), 15, 7, 0, st)),
          'copy': timeit(lambda: y.copy_(x))}
    gb = 2 * x.numel() * x.element_size() / 1e9
    print('tile' if os.environ.get('PCS_SEP2D_TILE') == '1' else 'march', n, str(dt),
          {k: f'{v:.0f}us {gb / (v * 1e-6) / 1e3:.2f}TB/s' for k, v in us.items()}, flush=True)


if __name__ == '__main__':
    main()

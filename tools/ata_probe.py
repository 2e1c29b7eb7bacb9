"""Time the in-plane normal operator C12^T C12 of the 3-D engine: one pcs_conv2d_sep_ata_planes
launch (both of its kernels) against the two pcs_conv2d_sep_planes launches (forward, flipped) it
replaces, on the C4 (512^3 f32) and C5 (1024^3 f64) volumes.  HIP events, median of 10 after 3 warm-up launches."""
import os
import sys
import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pycsou_amd import _lib as L  # noqa: E402


def med_ms(fn, n=10):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


def main():
    lib = L.load()
    # PCS_ATA_CASES: comma list of NP:N:dtype (NP planes of N x N), default the C4 and C5 volumes
    cases = os.environ.get('PCS_ATA_CASES', '512:512:f32,1024:1024:f64')
    for c in cases.split(','):
        npl, n, d = c.split(':')
        npl, n, dt = int(npl), int(n), torch.float64 if d == 'f64' else torch.float32
        x = torch.randn(npl, n, n, dtype=dt, device='cuda')
        t, g = torch.empty_like(x), torch.empty_like(x)
        r = np.arange(15) - 7.0
        h = np.exp(-0.5 * (r / 2.0) ** 2)
        h /= h.sum()
        hd = torch.as_tensor(h, dtype=dt, device='cuda')
        hf = torch.flip(hd, [0]).contiguous()
        code, st = L.dtcode(x), L.stream()

        def two():
            assert lib.pcs_conv2d_sep_planes(code, L.ptr(x), L.ptr(t), npl, n, n, L.ptr(hd), 15, 7, L.ptr(hd), 15, 7,
                                             0, st) == 0
            assert lib.pcs_conv2d_sep_planes(code, L.ptr(t), L.ptr(g), npl, n, n, L.ptr(hf), 15, 7, L.ptr(hf), 15, 7,
                                             0, st) == 0

        def one():
            assert lib.pcs_conv2d_sep_ata_planes(code, L.ptr(x), L.ptr(t), npl, n, n, L.ptr(hd), 15, 7, L.ptr(hd), 15,
                                                 7, st) == 0
        t2 = med_ms(two)
        for kern in os.environ.get('PCS_ATA_KERNELS', '2pass,4pass').split(','):  # k_sep2d_nrm (two 29-tap passes) / k_sep2d_ata (four 15-tap)
            os.environ['PCS_ATA_KERNEL'] = kern
            t1 = med_ms(one)
            d = (g - t).abs().max().item() / g.abs().max().item()
            print(f'{os.environ.get("PCS_LIB_PATH", "default")} {npl}x{n}x{n} {dt}: two passes {t2:.3f} ms, ata[{kern}] '
                  f'{t1:.3f} ms, max rel diff {d:.2e}', flush=True)
        os.environ.pop('PCS_ATA_KERNEL')
        del x, t, g


if __name__ == '__main__':
    main()

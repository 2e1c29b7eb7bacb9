"""Standalone Convolve2D timing (a9): one forward pass at n x n, k x k PSF, fp32/fp64, through
the public operator (packed plan -> pcs_conv2d_planned), HIP events on the launch stream.
Prints one JSON line per case: ms per pass, TFLOP/s (2 k^2 flop per pixel) and GB/s
(read x + write out)."""
import argparse
import json
import sys
import os

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=4096)
    ap.add_argument('--ks', default='15')
    ap.add_argument('--dtypes', default='f32')
    ap.add_argument('--iters', type=int, default=50)
    ap.add_argument('--raw', action='store_true', help='pcs_conv2d (raw PSF) instead of the plan')
    args = ap.parse_args()
    from pycsou_amd.linop.conv import Convolve2D
    from pycsou_amd import _lib as L, _ops as O
    n = args.n
    for dt in args.dtypes.split(','):
        dtype = torch.float32 if dt == 'f32' else torch.float64
        for k in map(int, args.ks.split(',')):
            rng = np.random.default_rng(0)
            h = rng.standard_normal((k, k))
            op = Convolve2D(n * n, h, (n, n))
            x = torch.randn(n * n, device='cuda', dtype=dtype)
            out = torch.empty_like(x)
            plan = op.plan(dtype, False)

            def run():
                if args.raw:
                    return O.conv2d(x, (n, n), op._h.get(dtype), k, k, k // 2, k // 2)
                return O.conv2d_planned(x, (n, n), plan, out=out)
            for _ in range(5):
                run()
            torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(args.iters):
                run()
            ev[1].record()
            torch.cuda.synchronize()
            ms = ev[0].elapsed_time(ev[1]) / args.iters
            flop = 2.0 * k * k * n * n
            byt = 2.0 * n * n * x.element_size()
            print(json.dumps({'n': n, 'k': k, 'dtype': dt, 'raw': args.raw, 'ms': round(ms, 4),
                              'tflops': round(flop / ms / 1e9, 2), 'GBps': round(byt / ms / 1e6, 1)}), flush=True)


if __name__ == '__main__':
    main()

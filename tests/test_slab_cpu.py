"""Row-slab decomposition and its transport on the CPU (gloo, world_size 2 and 3).

The GPU step kernel is replaced by a stand-in with the same data dependencies (own rows
computed from rows i-h .. i+h of the halo'd buffer), so the layout, the halo exchange
and the sum gathering of pycsou_amd.parallel are checked without a GPU; the kernel in
slab mode is covered by tests/test_gpu_slab.py.
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pycsou_amd.parallel.slab import DistComm, SlabLayout, gather_rows, row_split

N0, N1, ITERS = 41, 9, 6
W = np.array([0.05, -0.1, 0.2, 0.5, 0.2, -0.1, 0.05])  # 7-row stencil (h = 3)


def _stencil_global(x, w):
    h = len(w) // 2
    n0 = x.shape[0]
    xp = np.zeros((n0 + 2 * h, x.shape[1]))
    xp[h:h + n0] = x
    return sum(w[k] * xp[k:k + n0] for k in range(len(w)))


def _reference(x0, z0):
    x, z0c, z1c = x0.copy(), z0[0].copy(), z0[1].copy()
    sums = []
    for _ in range(ITERS):
        xn = _stencil_global(x, W)
        z0n = _stencil_global(z0c, np.array([0.25, 0.5, 0.25])) + xn
        z1n = _stencil_global(z1c, np.array([-0.5, 1.0, 0.5]))
        sums.append([((xn - x) ** 2).sum(), (x ** 2).sum()])
        x, z0c, z1c = xn, z0n, z1n
    return x, z0c, z1c, np.array(sums)


def _worker(rank, world, port, x0, z0, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        comm = DistComm()
        lay = SlabLayout(N0, N1, rank, world)
        hx, hz = 3, 1
        X = [lay.window(torch.as_tensor(x0.ravel()), hx) for _ in range(2)]
        Z = [torch.cat([lay.window(torch.as_tensor(z0[c].ravel()), hz) for c in (0, 1)]) for _ in range(2)]
        halos = [lay.halo_pairs([(X[q], hx, 0), (Z[q], hz, 0), (Z[q], hz, 1)]) for q in (0, 1)]
        R = lay.rows
        sums = []
        for it in range(ITERS):
            p = it % 2
            xin = X[p].view(R + 2 * hx, N1)
            xo = X[1 - p].view(R + 2 * hx, N1)
            gr = lay.row0 + np.arange(-hx, R + hx)
            valid = torch.as_tensor(((gr >= 0) & (gr < N0)).astype(np.float64))[:, None]
            xm = xin * valid  # rows outside the image read as zero, whatever the halo holds
            new = sum(W[k] * xm[k:k + R] for k in range(7))
            xo[hx:hx + R] = new
            for c, w, add in ((0, (0.25, 0.5, 0.25), True), (1, (-0.5, 1.0, 0.5), False)):
                zin = lay.rows_view(Z[p], hz, -hz, R + hz, c).view(R + 2, N1)
                g1 = lay.row0 + np.arange(-1, R + 1)
                zm = zin * torch.as_tensor(((g1 >= 0) & (g1 < N0)).astype(np.float64))[:, None]
                zn = sum(w[k] * zm[k:k + R] for k in range(3)) + (new if add else 0)
                lay.rows_view(Z[1 - p], hz, 0, R, c).copy_(zn.ravel())
            loc = torch.tensor([((new - xin[hx:hx + R]) ** 2).sum(), (xin[hx:hx + R] ** 2).sum(), 0., 0.],
                               dtype=torch.float64)
            g = torch.zeros(4 * world, dtype=torch.float64)
            comm.allgather(loc, g)
            sums.append(g.view(world, 4)[:, :2].sum(0).numpy())
            comm.exchange(halos[1 - p])
        q = ITERS % 2
        x = gather_rows(lay.rows_view(X[q], hx, 0, R).clone(), N0, N1, world, rank, comm)
        z0g = gather_rows(lay.rows_view(Z[q], hz, 0, R, 0).clone(), N0, N1, world, rank, comm)
        z1g = gather_rows(lay.rows_view(Z[q], hz, 0, R, 1).clone(), N0, N1, world, rank, comm)
        if rank == 0:
            np.savez(out, x=x.numpy(), z0=z0g.numpy(), z1=z1g.numpy(), sums=np.array(sums))
    finally:
        dist.destroy_process_group()


def _port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.parametrize('world', [2, 3])
def test_slab_exchange_gloo(world, tmp_path):
    rng = np.random.default_rng(world)
    x0 = rng.standard_normal((N0, N1))
    z0 = rng.standard_normal((2, N0, N1))
    out = str(tmp_path / 'res.npz')
    mp.spawn(_worker, args=(world, _port(), x0, z0, out), nprocs=world, join=True)
    r = np.load(out)
    x, z0c, z1c, sums = _reference(x0, z0)
    np.testing.assert_allclose(r['x'].reshape(N0, N1), x, rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(r['z0'].reshape(N0, N1), z0c, rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(r['z1'].reshape(N0, N1), z1c, rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(r['sums'], sums, rtol=1e-12)


@pytest.mark.parametrize('n0,world', [(10, 3), (4096 * 8, 8), (7, 7), (100, 1)])
def test_row_split_partition(n0, world):
    spans = [row_split(n0, world, r) for r in range(world)]
    assert spans[0][0] == 0
    assert all(a[0] + a[1] == b[0] for a, b in zip(spans, spans[1:]))
    assert spans[-1][0] + spans[-1][1] == n0
    assert max(s[1] for s in spans) - min(s[1] for s in spans) <= 1


def test_window_and_views():
    lay = SlabLayout(10, 3, 1, 3)  # rows 4..6 (rows 4,5,6 -> row0 4? split 4,3,3)
    assert (lay.row0, lay.rows) == (4, 3)
    g = torch.arange(30, dtype=torch.float64)
    w = lay.window(g, 2)
    assert w.numel() == (3 + 4) * 3
    np.testing.assert_array_equal(w.numpy(), g[6:27].numpy())
    assert torch.equal(lay.rows_view(w, 2, 0, 3), g[12:21])
    top = SlabLayout(10, 3, 0, 3)
    wt = top.window(g, 2)
    assert torch.equal(wt[:6], torch.zeros(6, dtype=torch.float64))  # above the image
    pairs = lay.halo_pairs([(w, 2, 0)])
    assert sorted(pairs) == [0, 2]
    (s_up, r_up), = pairs[0]
    assert torch.equal(s_up, g[12:18]) and torch.equal(r_up, g[6:12])

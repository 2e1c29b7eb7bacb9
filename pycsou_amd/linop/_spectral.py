"""Exact operator norms of the structured operators on the path (host, banded fp64 bisection).

The reference computes every ``lipschitz_cst`` with ARPACK (``pycsou/core/linop.py:279-321``:
``svds`` / ``eigsh`` with k=1, tens to thousands of operator applications at 4096^2).  The
operators here act along one axis of a C-order array, so their Gram matrices are Kronecker
structured:

* ``FirstDerivative`` / ``SecondDerivative`` / ``Convolve1D`` along axis k:
  K = I (x) A (x) I, ||K||^2 = lambda_max(A^T A) for the 1-D n_k x n_k matrix A;
* ``Gradient`` = [D_0; D_1; ...]: K^T K = sum_k I (x) D_k^T D_k (x) I (a Kronecker sum of PSD
  terms), ||K||^2 = sum_k lambda_max(D_k^T D_k);
* a separable ``Convolve2D`` h = c r^T: K = C_0 (x) C_1, ||K|| = ||C_0|| ||C_1||; a composition
  of ``Convolve1D`` along distinct axes of one shape likewise multiplies.

A^T A of a banded 1-D stencil / filter is banded (bandwidth <= 2 x the reach), so lambda_max is
found by bisection on positive definiteness of mu I - A^T A (a banded Cholesky per test, O(n b^2)):
10-50 ms for n = 4096, instead of seconds of device Lanczos (a banded eigensolver's
tridiagonal reduction is O(n^2 b): 0.44 s for the 15-tap blur at n = 4096).  The value returned
is the smallest mu found with a Cholesky factor, so it lies above lambda_max (relative 1e-14, plus Cholesky's backward error) and
step sizes built from it stay on the safe side of tau sigma ||K||^2 <= 1
(``pycsou/opt/proxalgs.py:280-301``).
"""

import numpy as np
import scipy.sparse as sp
from scipy.linalg import cholesky_banded


def _lam_max_gram(A, rtol=1e-14):
    """lambda_max(A^T A) for a sparse banded n x n matrix A, from above: the smallest mu found for
    which mu I - A^T A has a banded Cholesky factor (positive definite, so mu > lambda_max), by
    bisection between max diag(A^T A) (<= lambda_max) and the Gershgorin bound (>= lambda_max).
    Each test is O(n b^2) (LAPACK pbtrf); about 47 of them reach rtol."""
    G = (A.T @ A).tocsr()
    n = G.shape[0]
    diag = G.diagonal()
    lo = float(diag.max()) if n else 0.0
    hi = float(abs(G).sum(axis=0).max()) if n else 0.0
    if n <= 1 or hi <= 0.0:
        return hi
    offs = G.tocoo()
    b = int(np.max(np.abs(offs.col - offs.row)))
    band = np.zeros((b + 1, n))
    for k in range(b + 1):  # upper form: band[b - k, j] = G[j - k, j]
        band[b - k, k:] = -G.diagonal(k)
    hi *= 1.0 + 1e-12  # strictly above lambda_max (Gershgorin may be attained)

    def pd(mu):
        m = band.copy()
        m[b] += mu
        try:
            cholesky_banded(m, lower=False, check_finite=False)
            return True
        except np.linalg.LinAlgError:
            return False
    if b == 0:
        return hi
    while hi - lo > rtol * hi:
        mid = 0.5 * (lo + hi)
        if pd(mid):
            hi = mid
        else:
            lo = mid
    # a factor can exist for mu a few ulp of ||G|| below lambda_max (Cholesky's backward error):
    # step past that so the value stays above the exact lambda_max
    return hi * (1.0 + 4e-14) + 8 * (b + 1) * np.finfo(np.float64).eps * float(abs(G).sum(axis=0).max())


def deriv1_matrix(n, kind, edge, h):
    """PyLops 1.x FirstDerivative along one axis of length n (oracle/pylops1.py restates it)."""
    A = sp.lil_matrix((n, n))
    if kind == 'forward':
        for i in range(n - 1):
            A[i, i], A[i, i + 1] = -1.0 / h, 1.0 / h
    elif kind == 'backward':
        for i in range(1, n):
            A[i, i - 1], A[i, i] = -1.0 / h, 1.0 / h
    else:
        for i in range(1, n - 1):
            A[i, i - 1], A[i, i + 1] = -0.5 / h, 0.5 / h
        if edge and n >= 2:
            A[0, 0], A[0, 1] = -1.0 / h, 1.0 / h
            A[n - 1, n - 2], A[n - 1, n - 1] = -1.0 / h, 1.0 / h
    return A.tocsr()


def _deriv1_fast(n, kind, edge, h):
    """deriv1_matrix built from diagonals (O(n), no Python loop over rows)."""
    if n < 3:
        return deriv1_matrix(n, kind, edge, h)
    if kind == 'forward':
        d0 = np.full(n, -1.0 / h)
        d0[-1] = 0.0
        return sp.diags([d0, np.full(n - 1, 1.0 / h)], [0, 1], shape=(n, n), format='csr')
    if kind == 'backward':
        d0 = np.full(n, 1.0 / h)
        d0[0] = 0.0
        return sp.diags([np.full(n - 1, -1.0 / h), d0], [-1, 0], shape=(n, n), format='csr')
    lo = np.full(n - 1, -0.5 / h)
    up = np.full(n - 1, 0.5 / h)
    d0 = np.zeros(n)
    lo[-1] = 0.0  # row n-1 (set below)
    up[0] = 0.0   # row 0
    if edge:
        d0[0], up[0] = -1.0 / h, 1.0 / h
        lo[-1], d0[-1] = -1.0 / h, 1.0 / h
    return sp.diags([lo, d0, up], [-1, 0, 1], shape=(n, n), format='csr')


def deriv2_matrix(n, edge, h):
    """PyLops 1.x SecondDerivative along one axis (interior 3-point, one-sided ends with edge)."""
    A = sp.lil_matrix((n, n))
    h2 = h * h
    for i in range(1, n - 1):
        A[i, i - 1], A[i, i], A[i, i + 1] = 1.0 / h2, -2.0 / h2, 1.0 / h2
    if edge and n >= 3:
        A[0, 0], A[0, 1], A[0, 2] = 1.0 / h2, -2.0 / h2, 1.0 / h2
        A[n - 1, n - 3], A[n - 1, n - 2], A[n - 1, n - 1] = 1.0 / h2, -2.0 / h2, 1.0 / h2
    return A.tocsr()


def _deriv2_fast(n, edge, h):
    if n < 5:
        return deriv2_matrix(n, edge, h)
    h2 = h * h
    lo = np.full(n - 1, 1.0 / h2)
    d0 = np.full(n, -2.0 / h2)
    up = np.full(n - 1, 1.0 / h2)
    up[0] = d0[0] = 0.0
    lo[-1] = d0[-1] = 0.0
    A = sp.diags([lo, d0, up], [-1, 0, 1], shape=(n, n), format='lil')
    if edge:
        A[0, 0], A[0, 1], A[0, 2] = 1.0 / h2, -2.0 / h2, 1.0 / h2
        A[n - 1, n - 3], A[n - 1, n - 2], A[n - 1, n - 1] = 1.0 / h2, -2.0 / h2, 1.0 / h2
    return A.tocsr()


def conv1d_matrix(n, taps, off):
    """'same' zero-boundary convolution with pycsou's offset: out[i] = sum_j h[j] x[i + off - j]."""
    taps = np.asarray(taps, dtype=np.float64)
    k = taps.size
    diags, offsets = [], []
    for j in range(k):
        d = off - j  # column m = i + d
        if taps[j] == 0.0 or abs(d) >= n:
            continue
        diags.append(np.full(n - abs(d), taps[j]))
        offsets.append(d)
    if not diags:
        return sp.csr_matrix((n, n))
    return sp.diags(diags, offsets, shape=(n, n), format='csr')


def deriv1_norm2(n, kind, edge, h):
    """||FirstDerivative||^2 along an axis of length n."""
    return _lam_max_gram(_deriv1_fast(int(n), kind, bool(edge), float(h)))


def deriv2_norm2(n, edge, h):
    return _lam_max_gram(_deriv2_fast(int(n), bool(edge), float(h)))


def conv1d_norm2(n, taps, off):
    return _lam_max_gram(conv1d_matrix(int(n), taps, int(off)))

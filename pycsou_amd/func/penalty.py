"""Penalty functionals (``pycsou/func/penalty.py`` hot-path subset), gfx950 kernels.

* ``L1Norm`` (``penalty.py:194-245``): ``prox = x - tau*clip(x/tau, -1, 1)``.
* ``L2Norm`` (``penalty.py:23-70``): ``prox = x - tau*proj_l2_ball(x/tau, 1)``.
* ``L21Norm`` (``penalty.py:480-560``): same ``__new__`` dispatch (no groups / all distinct
  -> ``L1Norm``, one group -> ``L2Norm``).  The isotropic-TV grouping
  ``tile(arange(N), d)`` runs as one per-pixel kernel (the reference's O(G*N) Python loop
  becomes O(N)); any other labelling uses a segmented sum-of-squares + scale kernel pair.
* ``SquaredL2Norm`` (``penalty.py:73-131``): value / gradient, plus the closed-form prox
  ``x / (1 + 2 tau)`` that the reference lacks (new API).
* ``NonNegativeOrthant`` / ``Segment`` (``penalty.py:563-668``): indicator functionals
  whose projections are kernels.
"""

import numpy as np
import torch

from .. import _ops as O
from ..core.functional import DifferentiableFunctional
from .base import IndicatorFunctional, LpNorm


class L2Norm(LpNorm):
    def __init__(self, dim):
        super().__init__(dim=dim)

    def _apply(self, t):
        return float(np.sqrt(O.reduce_dev(0, t).item()))

    def _prox(self, t, tau):
        return O.prox_l2(t, tau)


class SquaredL2Norm(DifferentiableFunctional):
    def __init__(self, dim):
        super().__init__(dim=dim, data=None, is_linear=False, lipschitz_cst=np.inf, diff_lipschitz_cst=2)

    def _apply(self, t):
        return float(O.reduce_dev(0, t).item())

    def _jacT(self, t):
        return O.scale(t, 2.0)

    def _prox(self, t, tau):
        return O.prox_sql2(t, tau)

    def prox(self, x, tau):
        """New API: ``argmin_u tau*||u||^2 + 1/2 ||u - x||^2 = x / (1 + 2 tau)``."""
        return O.like(self._prox(O.to_dev(x), tau), x)


class L1Norm(LpNorm):
    def __init__(self, dim):
        super().__init__(dim=dim)

    def _apply(self, t):
        return float(O.reduce_dev(1, t).item())

    def _prox(self, t, tau):
        return O.prox_l1(t, tau)

    def _fenchel_scaled(self, w, sigma, lam):
        return O.fenchel_l1(w, sigma, lam)

    def soft(self, x, tau):
        from ..math.prox import soft
        return soft(x=x, tau=tau)


def _is_pixel_grouping(groups, dim):
    g = np.asarray(groups).reshape(-1)
    u = np.unique(g)
    if u.size == 0 or dim % u.size:
        return 0
    d = dim // u.size
    return d if np.array_equal(g, np.tile(u, d)) else 0


_CHUNK = 1 << 24


def _pixel_summary(g, dim):
    """O(n) test for the groupings TV builds, ``tile(u, d)`` with ``u`` strictly increasing
    (``np.tile(np.arange(npix), d)``): returns (u, d) -- u a view of g -- or None.  Avoids the
    three sorts of ``np.unique`` on 3e9 labels (C5: 1024^3 voxels x 3 components)."""
    n = g.size
    if n == 0 or n != dim or g.dtype.kind not in 'iu':
        return None
    m = None
    for a in range(0, n - 1, _CHUNK):  # first index where the labels stop increasing
        c = g[a:min(n, a + _CHUNK + 1)]
        hit = np.flatnonzero(c[1:] <= c[:-1])
        if hit.size:
            m = a + int(hit[0]) + 1
            break
    if m is None:
        return g, 1  # strictly increasing: all distinct
    if n % m:
        return None
    u = g[:m]
    for k in range(1, n // m):
        for a in range(0, m, _CHUNK):
            b = min(m, a + _CHUNK)
            if not np.array_equal(g[k * m + a:k * m + b], u[a:b]):
                return None
    return u, n // m


class L21Norm(LpNorm):
    """Mixed L2,1 norm over ``groups`` (``penalty.py:480-560``)."""

    def __new__(cls, dim, groups=None):
        if groups is None:
            return L1Norm(dim=dim)
        g = np.asarray(groups).reshape(-1)
        if g.dtype == object and np.all(g == None):  # noqa: E711
            return L1Norm(dim=dim)
        fast = _pixel_summary(g, dim)
        nuniq = fast[0].size if fast is not None else np.unique(g).size
        if nuniq == dim:
            return L1Norm(dim=dim)
        if nuniq == 1:
            return L2Norm(dim=dim)
        obj = super().__new__(cls)
        obj._fast = fast
        return obj

    def __init__(self, dim, groups):
        super().__init__(dim=dim)
        self.groups = np.asarray(groups).reshape(-1)
        fast = getattr(self, '_fast', None)
        if fast is not None:  # pixel groups: the sorted labels are the first component's
            self.groups_idxs, self.pixel_d = fast
            self._inv = None
        else:
            self.groups_idxs, inv = np.unique(self.groups, return_inverse=True)
            self.pixel_d = _is_pixel_grouping(self.groups, dim)   # d > 0 -> per-pixel kernel
            self._inv = inv.astype(np.int32)
        self._gid = None
        self._csr = None

    def _gid_dev(self):
        if self._gid is None:
            if self._inv is None:
                self._inv = np.unique(self.groups, return_inverse=True)[1].astype(np.int32)
            self._gid = torch.as_tensor(self._inv).to(O.device())
        return self._gid

    def _apply(self, t):
        if self.pixel_d:
            v = t.view(self.pixel_d, -1)
            return float(torch.sqrt((v.double() ** 2).sum(0)).sum())
        ss = torch.zeros(self.groups_idxs.size, dtype=torch.float64, device=t.device)
        ss.index_add_(0, self._gid_dev().long(), t.double() ** 2)
        return float(torch.sqrt(ss).sum())

    @staticmethod
    def _csr_host(inv, ngroups):
        """(order, offsets, largest group) of group indices `inv`: the elements group by group in ascending
        element order (a stable argsort), group g at order[off[g]:off[g + 1]]."""
        order = np.argsort(inv, kind='stable').astype(np.int32)
        counts = np.bincount(inv, minlength=ngroups)
        off = np.zeros(counts.size + 1, dtype=np.int64)
        np.cumsum(counts, out=off[1:])
        return order, off, int(counts.max()) if counts.size else 0

    def _csr_dev(self):
        """_csr_host of the labels on the device, for the deterministic group sums of pcs_prox_l21_groups."""
        if getattr(self, '_csr', None) is None:
            gid = self._gid_dev()
            order, off, maxlen = self._csr_host(self._inv, self.groups_idxs.size)
            self._csr = (torch.as_tensor(order).to(gid.device), torch.as_tensor(off).to(gid.device), maxlen)
        return self._csr

    def _prox(self, t, tau):
        if self.pixel_d:
            return O.prox_l21_pixel(t, tau, self.pixel_d)
        order, off, maxlen = self._csr_dev()
        return O.prox_l21_groups(t, tau, self._gid_dev(), self.groups_idxs.size, order, off, maxlen)

    def _fenchel_scaled(self, w, sigma, lam):
        if self.pixel_d:
            return O.fenchel_l21_pixel(w, sigma, lam, self.pixel_d)
        v = O.scale(w, 1.0 / sigma)
        return O.axpby(w, self._prox(v, (1.0 / sigma) * lam), 1.0, -sigma)


def NonNegativeOrthant(dim):
    """``penalty.py:563-612``."""
    return IndicatorFunctional(dim=dim, condition_func=lambda t: bool(torch.all(t >= 0)),
                               projection_func=lambda t: O.proj_nonneg(t), kind='nonneg')


def Segment(dim, a=0, b=1):
    """``penalty.py:615-668``."""
    return IndicatorFunctional(dim=dim, condition_func=lambda t: bool(torch.all((t >= a) & (t <= b))),
                               projection_func=lambda t: O.proj_segment(t, a, b), kind='segment',
                               params=(float(a), float(b)))


def L2Ball(dim, radius):
    """``penalty.py:134-191``: indicator of the L2 ball (projection via the L2 prox identity)."""
    def proj(t):
        # proj_{r B2}(x) = x - prox_{r||.||}(x)  (Moreau)
        return O.axpby(t, O.prox_l2(t, radius), 1.0, -1.0)
    return IndicatorFunctional(dim=dim, condition_func=lambda t: float(torch.linalg.vector_norm(t)) <= radius,
                               projection_func=proj)


def LInftyBall(dim, radius):
    """``penalty.py:420-477``: indicator of the L-infinity ball (clip)."""
    return IndicatorFunctional(dim=dim, condition_func=lambda t: float(t.abs().max()) <= radius,
                               projection_func=lambda t: O.proj_segment(t, -radius, radius))

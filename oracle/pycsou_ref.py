"""NumPy restatement of the reference pycsou solver / prox / functional code.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).  Pinned against the
golden vectors in ``tests/golden/`` that ``tests/golden/make_golden.py``
produced with the real reference code.

Every function names the reference lines it restates.  The operation order
(and the per-iteration temporaries, ``np.linalg.norm`` diagnostics, pandas
``.loc`` row appends and ``deepcopy`` of the iterand) follow the reference so
that this module doubles as the CPU baseline that ``bench.py`` times on the
GPU box, where ``/root/reference`` does not exist.
"""

from copy import deepcopy

import numpy as np

try:
    from pandas import DataFrame
except Exception:  # pragma: no cover
    DataFrame = None


# --------------------------------------------------------------------------
# pycsou/math/prox.py
# --------------------------------------------------------------------------

def sign(x):
    """``pycsou/math/prox.py:61-64``."""
    x = np.asarray(x)
    y = np.asarray(0 * x)
    nz = np.abs(x) != 0
    y[nz] = np.conj(x[nz]) / np.abs(x[nz])
    return y


def soft(x, tau):
    """``pycsou/math/prox.py:114``."""
    return np.clip(np.abs(x) - tau, a_min=0, a_max=None) * sign(x)


def proj_linfty_ball(x, radius):
    """``pycsou/math/prox.py:253-256`` (mutates and returns its argument)."""
    y = x
    y[y > radius] = radius
    y[y < -radius] = -radius
    return y


def proj_l2_ball(x, radius):
    """``pycsou/math/prox.py:207-210``."""
    n = np.linalg.norm(x)
    if n <= radius:
        return x
    return radius * x / n


def proj_nonnegative_orthant(x):
    """``pycsou/math/prox.py:295-297`` (mutates its argument)."""
    y = np.real(x)
    y[y < 0] = 0
    return y


def proj_segment(x, a=0, b=1):
    """``pycsou/math/prox.py:340-343`` (mutates its argument)."""
    y = np.real(x)
    y[y < a] = a
    y[y > b] = b
    return y


# --------------------------------------------------------------------------
# pycsou/func/base.py, pycsou/func/penalty.py, pycsou/core/functional.py
# --------------------------------------------------------------------------

def prox_l1(x, tau):
    """``LpNorm.prox`` with ``proj_linfty_ball`` (``pycsou/func/base.py:239-240``,
    ``pycsou/func/penalty.py:238``)."""
    return x - tau * proj_linfty_ball(x / tau, radius=1)


def prox_l2(x, tau):
    """``LpNorm.prox`` with ``proj_l2_ball`` (``pycsou/func/penalty.py:67``)."""
    return x - tau * proj_l2_ball(x / tau, radius=1)


def group_norms(x, groups):
    """Per-group Euclidean norms in ``np.unique(groups)`` order
    (``pycsou/func/penalty.py:545,553,559-560``), vectorised."""
    ids, inv = np.unique(groups, return_inverse=True)
    return ids, inv, np.sqrt(np.bincount(inv, weights=x * x, minlength=ids.size))


def prox_l21(x, tau, groups):
    """``L21Norm.prox`` (``pycsou/func/penalty.py:551-557``): per group g,
    ``y_g = clip(1 - tau/||x_g||, 0) * x_g`` (zero-norm group -> 0)."""
    _, inv, n = group_norms(x, groups)
    with np.errstate(divide='ignore'):
        fac = np.clip(1 - tau / n, a_min=0, a_max=None)
    return fac[inv] * x


def prox_l21_pixel(x, tau, d):
    """``L21Norm.prox`` for the isotropic-TV grouping ``groups = tile(arange(N), d)``:
    the group of pixel p is ``{x[k*N + p] : k < d}``."""
    v = x.reshape(d, -1)
    n = np.sqrt(np.sum(v * v, axis=0))
    with np.errstate(divide='ignore'):
        fac = np.clip(1 - tau / n, a_min=0, a_max=None)
    return (fac[None, :] * v).ravel()


def l21_value_pixel(x, d):
    """``L21Norm.__call__`` (``pycsou/func/penalty.py:548-549``) for pixel groups."""
    v = x.reshape(d, -1)
    return float(np.sum(np.sqrt(np.sum(v * v, axis=0))))


def prox_sql2(x, tau):
    """New API (no reference prox): ``prox_{tau ||.||^2}(x) = x / (1 + 2 tau)``
    (definition ``pycsou/core/functional.py:100-103``)."""
    return x / (1 + 2 * tau)


def fenchel_prox(prox, z, sigma):
    """``ProximableFunctional.fenchel_prox`` (``pycsou/core/functional.py:207``)."""
    return z - sigma * prox(z / sigma, 1 / sigma)


def postcomp(prox, scale):
    """``ProxFuncPostComp.prox`` (``pycsou/core/functional.py:264-265``): ``(scale*f).prox(x,t) = f.prox(x, t*scale)``."""
    return lambda x, tau: prox(x, tau * scale)


# --------------------------------------------------------------------------
# pycsou/opt/proxalgs.py : step sizes
# --------------------------------------------------------------------------

def pds_step_sizes(beta, K_lip, has_H=True):
    """``PrimalDualSplitting.set_step_sizes`` (``pycsou/opt/proxalgs.py:280-301``)."""
    if beta > 0:
        if not has_H:
            return 2 / beta, 0
        if K_lip < np.inf:
            t = (1 / K_lip ** 2) * ((-beta / 4) + np.sqrt((beta ** 2 / 16) + K_lip ** 2))
            return t, t
        raise ValueError('Please compute the Lipschitz constant of the linear operator K')
    if not has_H:
        return 1, 0
    if K_lip < np.inf:
        return 1 / K_lip, 1 / K_lip
    raise ValueError('Please compute the Lipschitz constant of the linear operator K')


def pds_momentum(beta):
    """``PrimalDualSplitting.set_momentum_term`` (``pycsou/opt/proxalgs.py:312-316``)."""
    return 0.9 if beta > 0 else 1


# --------------------------------------------------------------------------
# pycsou/core/solver.py + proxalgs.py : the loops
# --------------------------------------------------------------------------

def _rel(old, new):
    n = np.linalg.norm(old)
    if n == 0:
        return np.inf
    return np.linalg.norm(old - new) / n


def pds(grad_F, prox_G, K, KT, fenchel_H, tau, sigma, rho, x0, z0, max_iter=500, min_iter=10,
        accuracy_threshold=1e-3, has_H=True, pandas_diagnostics=False, callback=None):
    """``GenericIterativeAlgorithm.iterate`` (``pycsou/core/solver.py:55-76``) driving
    ``PrimalDualSplitting.update_iterand`` (``pycsou/opt/proxalgs.py:343-355``) and
    ``update_diagnostics``/``stopping_metric`` (``proxalgs.py:360-394``).

    Returns ``(x, z, diag)`` with ``diag = {'primal': [...], 'dual': [...]}`` (one
    entry per executed iteration) and, if ``pandas_diagnostics``, a DataFrame in
    ``diag['frame']`` built exactly like the reference (one ``.loc`` row per
    iteration).
    """
    x, z = x0, z0
    old = deepcopy({'primal_variable': x0, 'dual_variable': z0})
    hist_p, hist_d = [], []
    frame = None
    if pandas_diagnostics:
        cols = ['Iter', 'Relative Improvement (primal variable)']
        if has_H:
            cols.append('Relative Improvement (dual variable)')
        frame = DataFrame(columns=cols)
    it = 0
    while ((it <= max_iter) and ((np.inf if it == 0 else hist_p[it - 1]) > accuracy_threshold)) or (it <= min_iter):
        x_temp = prox_G(x - tau * grad_F(x) - tau * KT(z), tau)
        if has_H:
            u = 2 * x_temp - x
            z_temp = fenchel_H(z + sigma * K(u), sigma)
            z = rho * z_temp + (1 - rho) * z
        x = rho * x_temp + (1 - rho) * x
        hist_p.append(_rel(old['primal_variable'], x))
        if has_H:
            hist_d.append(_rel(old['dual_variable'], z))
        if frame is not None:
            frame.loc[it, 'Iter'] = it
            frame.loc[it, 'Relative Improvement (primal variable)'] = hist_p[-1]
            if has_H:
                frame.loc[it, 'Relative Improvement (dual variable)'] = hist_d[-1]
        old = deepcopy({'primal_variable': x, 'dual_variable': z})
        if callback is not None:
            callback(it, x, z)
        it += 1
    return x, z, {'primal': hist_p, 'dual': hist_d, 'frame': frame, 'n_iter': it}


def apgd(grad_F, prox_G, tau, x0, acceleration='CD', d=75., max_iter=500, min_iter=10,
         accuracy_threshold=1e-3, pandas_diagnostics=False):
    """``AcceleratedProximalGradientDescent`` loop (``pycsou/opt/proxalgs.py:586-622``)."""
    x, x_old, t_old = x0, 0 * x0, 1
    old = deepcopy(x0)
    hist = []
    frame = DataFrame(columns=['Iter', 'Relative Improvement']) if pandas_diagnostics else None
    it = 0
    while ((it <= max_iter) and ((np.inf if it == 0 else hist[it - 1]) > accuracy_threshold)) or (it <= min_iter):
        x_temp = prox_G(x - tau * grad_F(x), tau)
        if acceleration == 'BT':
            t = (1 + np.sqrt(1 + 4 * t_old ** 2)) / 2
        elif acceleration == 'CD':
            t = (it + d) / d
        else:
            t = t_old = 1
        a = (t_old - 1) / t
        x = x_temp + a * (x_temp - x_old)
        x_old, t_old = x_temp, t
        hist.append(_rel(old, x))
        if frame is not None:
            frame.loc[it, 'Iter'] = it
            frame.loc[it, 'Relative Improvement'] = hist[-1]
        old = deepcopy(x)
        it += 1
    return x, {'iterand': x, 'past_aux': x_old, 'past_t': t_old}, {'hist': hist, 'frame': frame, 'n_iter': it}


# --------------------------------------------------------------------------
# Problem builders used by tests / bench (synthetic inputs of SURVEY 8(d))
# --------------------------------------------------------------------------

def gaussian_psf(size=15, sigma=2.0, dtype=np.float64):
    """15x15 Gaussian PSF, sigma = 2 px, normalised to sum 1."""
    r = np.arange(size) - (size - 1) / 2
    g = np.exp(-0.5 * (r / sigma) ** 2)
    h = np.outer(g, g)
    return (h / h.sum()).astype(dtype)


def gaussian_taps(size=15, sigma=2.0, dtype=np.float64):
    """Separable 1-D factor of :func:`gaussian_psf` (C4/C5 axis filters)."""
    r = np.arange(size) - (size - 1) / 2
    g = np.exp(-0.5 * (r / sigma) ** 2)
    return (g / g.sum()).astype(dtype)


def phantom(shape, n_rect=64, seed=0, dtype=np.float64):
    """Piecewise-constant phantom in [0, 1]: ``n_rect`` random axis-aligned boxes."""
    rng = np.random.default_rng(seed)
    x = np.zeros(shape, dtype=np.float64)
    for _ in range(n_rect):
        lo = [rng.integers(0, s) for s in shape]
        hi = [min(s, l + rng.integers(max(1, s // 16), max(2, s // 3))) for s, l in zip(shape, lo)]
        sl = tuple(slice(l, h) for l, h in zip(lo, hi))
        x[sl] = rng.uniform(0, 1)
    return x.astype(dtype)

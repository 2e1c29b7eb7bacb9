"""Proximal algorithms (mirrors ``pycsou/opt/proxalgs.py``).

Same classes, aliases, constructor signatures, validation errors, step-size and momentum
rules, iterand dicts and diagnostics DataFrame as the reference:

* ``PrimalDualSplitting`` / ``PDS`` (``proxalgs.py:27-394``)
* ``AcceleratedProximalGradientDescent`` / ``APGD`` (``proxalgs.py:400-622``)
* ``ChambollePockSplitting`` / ``CPS``, ``DouglasRachfordSplitting`` / ``DRS``,
  ``ForwardBackwardSplitting`` / ``FBS`` (``proxalgs.py:628-862``)

Execution: a PDS problem of the headline family (2-D TV denoising / deconvolution, see
``opt/engine.py``) runs on the fused hipGraph engine; every other composition runs the
reference iteration operator by operator on the GPU kernels (``update_iterand`` below),
with the diagnostics norms reduced on the device.
"""

import os
from numbers import Number

import numpy as np
import torch

from .. import _ops as O
from ..core.functional import ProximableFunctional
from ..core.linop import LinearOperator
from ..core.map import DifferentiableMap
from ..core.solver import GenericIterativeAlgorithm
from ..func.base import NullDifferentiableFunctional, NullProximableFunctional
from ..linop.base import IdentityOperator, NullOperator


def _frame(columns, rows):
    from pandas import DataFrame
    df = DataFrame(rows, columns=columns)
    df['Iter'] = df['Iter'].astype(int)
    return df


def _find_arrays(obj, depth=0, out=None):
    """Arrays (numpy / torch) referenced by a map tree (shifts, data): decides the output kind."""
    out = [] if out is None else out
    if depth > 8 or obj is None:
        return out
    for name in ('shift', 'data', 'mat'):
        v = getattr(obj, name, None)
        if isinstance(v, (np.ndarray, torch.Tensor)):
            out.append(v)
    for name in ('map', 'map1', 'map2', 'prox_func', 'Linop', 'LinOp1', 'LinOp2'):
        _find_arrays(getattr(obj, name, None), depth + 1, out)
    return out


def _wants_torch(*objs):
    for o in objs:
        if isinstance(o, torch.Tensor):
            return True
    for o in objs:
        for a in _find_arrays(o):
            if isinstance(a, torch.Tensor):
                return True
    return False


def _rel_improvement(old, new):
    """||old - new|| / ||old|| (inf if ||old|| == 0), proxalgs.py:370-383: both sums in one
    device pass, one read-back (API-level update_diagnostics; the solver loops use _DeviceLoop)."""
    d2, n2 = O.rel_sums(old, new, torch.empty(2, dtype=torch.float64, device=old.device)).tolist()
    if n2 == 0:
        return np.inf
    return float(np.sqrt(d2) / np.sqrt(n2))


class _DeviceLoop:
    """Loop control of the per-operator (generic) path on the device: after each iteration the
    relative-improvement sums are reduced on the GPU (pcs_rel_sums) and pcs_pds_finalize
    records the diagnostics row and the reference loop condition (solver.py:65-66,
    proxalgs.py:366-394) in a device control block -- the same one the fused engine uses.
    The host learns the stop decision from an asynchronous copy of that block, up to ``lag``
    iterations behind (no blocking .item() per iteration); iterations issued past the stop
    are discarded by the caller, which keeps the last ``lag + 2`` states."""

    # the device history starts at this many iterations and doubles as the loop issues more (a
    # max_iter of 1e9 with accuracy_threshold doing the stopping must not allocate 16 GB up front)
    HIST_CHUNK = 4096

    def __init__(self, max_iter, min_iter, thr, has_dual, device, lag=3, cap=None):
        from .. import _lib as L
        self.L, self.lib = L, L.gpu()
        max_iter, min_iter = int(max_iter), int(min_iter)
        self.total = max(min_iter, max_iter) + 1
        cap = min(self.total, self.HIST_CHUNK) if cap is None else int(cap)  # cap: rows up front (graph chunks)
        self.hist = torch.full((2 * cap + 2,), float('nan'), dtype=torch.float64, device=device)
        self.ctrl = torch.zeros(int(self.lib.pcs_ctrl_bytes()) // 8, dtype=torch.float64, device=device)
        self.sums = torch.zeros(4, dtype=torch.float64, device=device)
        L.check(self.lib.pcs_ctrl_init2(L.ptr(self.ctrl), min_iter, max_iter, float(thr), int(has_dual),
                                        int(self.hist.numel()), L.stream()), 'pcs_ctrl_init2')
        self.has_dual, self.lag = has_dual, lag
        self.pending = []  # (pinned host copy of (it, stopped), event)
        self.final = None
        self.issued = 0

    def _grow(self):
        """Before iteration `issued` is recorded: make room for its history row (and the stop test
        of the next), doubling the device buffer and its length in the control block -- both
        stream-ordered after every finalize already enqueued."""
        need = 2 * (self.issued + 2) + 2
        if need <= self.hist.numel():
            return
        cap = min(self.total, max(2 * ((self.hist.numel() - 2) // 2), self.issued + 2))
        new = torch.full((2 * cap + 2,), float('nan'), dtype=torch.float64, device=self.hist.device)
        new[:self.hist.numel()].copy_(self.hist)
        self.hist = new
        self.ctrl.view(torch.int32)[5].fill_(int(new.numel()))  # Ctrl.hist_len (pds_ctrl.hpp)

    def record(self, x_old, x, z_old=None, z=None):
        """Enqueue this iteration's sums + finalize and an async read-back of the control."""
        O.rel_sums(x_old, x, self.sums[0:2])
        if self.has_dual:
            O.rel_sums(z_old, z, self.sums[2:4])
        self.finalize()

    def finalize(self):
        """The loop control of the iteration whose sums are in ``sums``, and its read-back."""
        L = self.L
        self._grow()
        self.issued += 1
        L.check(self.lib.pcs_pds_finalize(L.ptr(self.sums), L.ptr(self.ctrl), L.ptr(self.hist), L.stream()),
                'pcs_pds_finalize')
        host = torch.empty(2, dtype=torch.int32, pin_memory=True)
        host.copy_(self.ctrl.view(torch.int32)[:2], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.pending.append((host, ev))

    def record_captured(self, x_old, x, z_old=None, z=None):
        """``record`` inside a graph capture: the sums and the loop control only (no read-back, no
        growth -- the history holds every row up front, ``cap``)."""
        L = self.L
        O.rel_sums(x_old, x, self.sums[0:2])
        if self.has_dual:
            O.rel_sums(z_old, z, self.sums[2:4])
        L.check(self.lib.pcs_pds_finalize(L.ptr(self.sums), L.ptr(self.ctrl), L.ptr(self.hist), L.stream()),
                'pcs_pds_finalize')

    def stream_rows(self, every, show):
        """``verbose``: show(k, row) for every resolved iteration k with k % every == 0, while the
        loop runs (solver.py:69-71 prints inside the loop) -- at most ``lag`` iterations late."""
        self._every, self._show, self._shown = int(every), show, 0

    def _emit(self, done):
        show = getattr(self, '_show', None)
        if show is None:
            return
        for k in range(self._shown, done):
            if k % self._every == 0:
                show(k, self.hist[2 * k:2 * k + 2].cpu().numpy())
        self._shown = max(self._shown, done)

    def poll(self, drain=False):
        """Resolve finished read-backs in order; returns the iteration count once the device
        stopped (None while it runs).  Blocks only to keep at most ``lag`` in flight."""
        while self.pending and self.final is None:
            host, ev = self.pending[0]
            if not (drain or len(self.pending) > self.lag or ev.query()):
                break
            ev.synchronize()
            self.pending.pop(0)
            self._emit(int(host[0]))
            if int(host[1]) != 0:
                self.final = int(host[0])
        return self.final

    def rows(self, n):
        h = self.hist[:2 * n].cpu().numpy().reshape(n, 2) if n > 0 else np.zeros((0, 2))
        return h


class PrimalDualSplitting(GenericIterativeAlgorithm):
    """Primal dual splitting (``pycsou/opt/proxalgs.py:27-394``)."""

    def __init__(self, dim, F=None, G=None, H=None, K=None, tau=None, sigma=None, rho=None, beta=None, x0=None,
                 z0=None, max_iter=500, min_iter=10, accuracy_threshold=1e-3, verbose=1, engine='auto'):
        self.dim = dim
        self._H = True
        if isinstance(F, DifferentiableMap):
            if F.shape[1] != dim:
                raise ValueError(f'F does not have the proper dimension: {F.shape[1]}!={dim}.')
            self.F = F
            if F.diff_lipschitz_cst < np.inf:
                self.beta = self.F.diff_lipschitz_cst if beta is None else beta
            elif (beta is not None) and isinstance(beta, Number):
                self.beta = beta
            else:
                raise ValueError('F must be a differentiable functional with Lipschitz-continuous gradient.')
        elif F is None:
            self.F = NullDifferentiableFunctional(dim=dim)
            self.beta = 0
        else:
            raise TypeError(f'F must be of type {DifferentiableMap}.')

        if isinstance(G, ProximableFunctional):
            if G.dim != dim:
                raise ValueError(f'G does not have the proper dimension: {G.dim}!={dim}.')
            self.G = G
        elif G is None:
            self.G = NullProximableFunctional(dim=dim)
        else:
            raise TypeError(f'G must be of type {ProximableFunctional}.')

        if isinstance(K, LinearOperator) and isinstance(H, ProximableFunctional):
            if (K.shape[1] != dim) or (K.shape[0] != H.dim):
                raise ValueError(f'Operator K with shape {K.shape} is inconsistent with functional H with dimension '
                                 f'{H.dim}.')
        if isinstance(H, ProximableFunctional):
            self.H = H
            if isinstance(K, LinearOperator):
                self.K = K
            elif K is None:
                self.K = IdentityOperator(size=H.dim)
                self.K.lipschitz_cst = self.K.diff_lipschitz_cst = 1
            else:
                raise TypeError(f'K must be of type {LinearOperator}.')
        elif H is None:
            self.H = NullProximableFunctional(dim=dim)
            self._H = False
            self.K = NullOperator(shape=(dim, dim))
            self.K.lipschitz_cst = self.K.diff_lipschitz_cst = 0
        else:
            raise TypeError(f'H must be of type {ProximableFunctional}.')

        if (tau is not None) and (sigma is not None):
            self.tau, self.sigma = tau, sigma
        elif (tau is not None) and (sigma is None):
            self.tau = self.sigma = tau
        elif (tau is None) and (sigma is not None):
            self.tau = self.sigma = sigma
        else:
            self.tau, self.sigma = self.set_step_sizes()
        self.rho = rho if rho is not None else self.set_momentum_term()

        self._torch_out = _wants_torch(x0, z0, F)
        self.x0 = x0 if x0 is not None else self.initialize_primal_variable()
        self.z0 = z0 if z0 is not None else self.initialize_dual_variable()
        self.engine_mode = engine
        self._engine = None
        objective_functional = (self.F + self.G) + (self.H * self.K)
        init_iterand = {'primal_variable': self.x0, 'dual_variable': self.z0}
        super().__init__(objective_functional=objective_functional, init_iterand=init_iterand, max_iter=max_iter,
                         min_iter=min_iter, accuracy_threshold=accuracy_threshold, verbose=verbose)

    # ---------------------------------------------------------------- reference rules
    def set_step_sizes(self):
        """``proxalgs.py:246-301``."""
        if self.beta > 0:
            if self._H is False:
                return 2 / self.beta, 0
            if self.K.lipschitz_cst < np.inf:
                t = (1 / (self.K.lipschitz_cst) ** 2) * ((-self.beta / 4) + np.sqrt((self.beta ** 2 / 16)
                                                                                    + self.K.lipschitz_cst ** 2))
                return t, t
        else:
            if self._H is False:
                return 1, 0
            if self.K.lipschitz_cst < np.inf:
                return 1 / self.K.lipschitz_cst, 1 / self.K.lipschitz_cst
        raise ValueError('Please compute the Lipschitz constant of the linear operator K by calling its method '
                         '"compute_lipschitz_cst()".')

    def set_momentum_term(self):
        """``proxalgs.py:303-316``."""
        return 0.9 if self.beta > 0 else 1

    def initialize_primal_variable(self):
        return np.zeros(shape=(self.dim,), dtype=np.float64)

    def initialize_dual_variable(self):
        if self._H is False:
            return None
        return np.zeros(shape=(self.H.dim,), dtype=np.float64)

    # ---------------------------------------------------------------- dtype / kind
    def _compute_dtype(self):
        for a in [self.x0] + _find_arrays(self.F):
            if isinstance(a, torch.Tensor) and a.dtype in (torch.float32, torch.float64):
                return a.dtype
            if isinstance(a, np.ndarray) and a.dtype in (np.float32, np.float64):
                return torch.float32 if a.dtype == np.float32 else torch.float64
        return torch.float64

    def _out(self, t):
        if t is None:
            return None
        return t if self._torch_out else t.detach().cpu().numpy()

    # ---------------------------------------------------------------- fused engine
    def _fused_spec(self):
        if self.engine_mode in (False, 'generic'):
            return None
        from .engine import match_masked_stencil2d, match_pds2d, match_stencil2d
        from .engine3d import match_pds3d
        F = None if isinstance(self.F, NullDifferentiableFunctional) else self.F
        if self.engine_mode == 'stencil':  # the general-stencil fused step only (tests, benchmarks)
            return match_stencil2d(F, self.G, self.H, self.K, self._H)
        K = self.K
        if (self._compute_dtype() == torch.float64 and len(getattr(K, 'dims', ())) == 2 and K.dims[1] >= 128
                and K.dims[1] % 4 == 0):
            # fp64 (the reference's default dtype) on images the row march covers: every 2-D K kind on
            # the general-stencil engine, whose march has an fp64 form (the forward-Gradient fp32
            # kernels do not); narrower images keep the tile kernels
            return (match_stencil2d(F, self.G, self.H, self.K, self._H) or match_pds2d(F, self.G, self.H, self.K, self._H)
                    or match_pds3d(F, self.G, self.H, self.K, self._H))
        return (match_pds2d(F, self.G, self.H, self.K, self._H) or match_stencil2d(F, self.G, self.H, self.K, self._H)
                or match_pds3d(F, self.G, self.H, self.K, self._H)
                or match_masked_stencil2d(F, self.G, self.H, self.K, self._H))

    def iterate(self):
        spec = self._fused_spec()
        if spec is None:
            if self.engine_mode in ('fused', 'stencil'):
                raise ValueError('problem does not match the fused PDS engine')
            return self._iterate_generic()
        from .engine import engine_class
        dtype = self._compute_dtype()
        x0 = O.to_dev(self.x0, dtype)
        z0 = O.to_dev(self.z0, dtype)
        eng = engine_class(spec)
        self._engine = eng(spec, dtype, self.tau, self.sigma, self.rho, x0, z0)
        n, x, z, hist = self._engine.run(self.max_iter, self.min_iter, self.accuracy_threshold, has_dual=True)
        self.iter = n
        rows = [[i, hist[i, 0], hist[i, 1]] for i in range(n)]
        self.diagnostics = _frame(['Iter', 'Relative Improvement (primal variable)',
                                   'Relative Improvement (dual variable)'], rows)
        if self.verbose is not None:
            # The reference prints row ``iter`` every ``verbose`` iterations while it loops
            # (solver.py:69-71, proxalgs.py:357-358); the fused loop never stops for the host,
            # so the same lines are printed from the device history once the run ends.
            for row in rows[::self.verbose]:
                self._rows = [row]
                self.print_diagnostics()
            self._rows = rows
        self.converged = True
        self.iterand = {'primal_variable': self._out(x), 'dual_variable': self._out(z)}
        return self.iterand, self.converged, self.diagnostics

    # ---------------------------------------------------------------- generic device path
    def _iterate_generic(self):
        """The reference loop (solver.py:55-76) operator by operator on the device, with the
        stopping rule evaluated on the device (``_DeviceLoop``): up to ``lag`` iterations are
        issued ahead of the stop decision and discarded if the reference would have stopped."""
        dtype = self._compute_dtype()
        state = {'primal_variable': O.to_dev(self.x0, dtype),
                 'dual_variable': None if self.z0 is None else O.to_dev(self.z0, dtype)}
        self.init_iterand_dev = dict(state)
        self._graph_used = False
        if self._graph_ok(state):
            out = self._iterate_generic_graph(state)
            if out is not None:
                return out
        loop = _DeviceLoop(self.max_iter, self.min_iter, self.accuracy_threshold, bool(self._H),
                           state['primal_variable'].device)
        if self.verbose is not None:
            def show(k, h):
                self._rows = [[k, h[0], h[1]] if self._H else [k, h[0]]]
                self.print_diagnostics()
            loop.stream_rows(self.verbose, show)
        states = {-1: state}
        i, n = 0, None
        while n is None:
            if i >= loop.total:
                n = loop.poll(drain=True)
                break
            new = self._update_dev(states[i - 1])
            loop.record(states[i - 1]['primal_variable'], new['primal_variable'],
                        states[i - 1]['dual_variable'], new['dual_variable'])
            states[i] = new
            states.pop(i - loop.lag - 3, None)
            i += 1
            n = loop.poll()
        self.iter = n
        h = loop.rows(n)
        self._rows = [[k, h[k, 0], h[k, 1]] if self._H else [k, h[k, 0]] for k in range(n)]
        self._state = states[n - 1]
        self.converged = True
        cols = ['Iter', 'Relative Improvement (primal variable)']
        if self._H:
            cols.append('Relative Improvement (dual variable)')
        self.diagnostics = _frame(cols, self._rows)
        self.iterand = {'primal_variable': self._out(self._state['primal_variable']),
                        'dual_variable': self._out(self._state['dual_variable'])}
        return self.iterand, self.converged, self.diagnostics

    # iterations per captured chunk of the generic path; the state ring holds two chunks
    GRAPH_CHUNK = 4
    GRAPH_RING_BYTES = 8 << 30

    def _graph_ok(self, state):
        """The generic loop runs as hipGraph chunks (``_iterate_generic_graph``) on a GPU unless
        PCS_GENERIC_GRAPH=0, when the state ring fits GRAPH_RING_BYTES and the history fits up front."""
        x = state['primal_variable']
        if os.environ.get('PCS_GENERIC_GRAPH', '1') == '0' or x.device.type != 'cuda':
            return False
        nbytes = sum(t.numel() * t.element_size() for t in state.values() if t is not None)
        total = max(int(self.max_iter), int(self.min_iter)) + 1
        return 2 * self.GRAPH_CHUNK * nbytes <= self.GRAPH_RING_BYTES and total <= (1 << 22)

    def _iterate_generic_graph(self, state):
        """The generic loop with its per-iteration launches captured: two hipGraphs of GRAPH_CHUNK
        iterations each write a ring of 2 x GRAPH_CHUNK states (iteration i -> slot i mod 2C, reading
        slot i - 1) and end with an asynchronous read-back of the loop control; they alternate, at
        most one chunk runs ahead of the one whose read-back the host waits for, so the state of the
        stopping iteration (always in the chunk that reports the stop) is never overwritten.
        Iterations past the stop are computed and discarded, as in the eager path (the finalize
        kernel ignores them).  The same launches as the eager loop, so the iterates and the
        diagnostics are bitwise the eager path's.  None if the capture fails (the eager path runs)."""
        C = self.GRAPH_CHUNK
        R = 2 * C
        x0, z0 = state['primal_variable'], state['dual_variable']
        total = max(int(self.max_iter), int(self.min_iter)) + 1
        loop = _DeviceLoop(self.max_iter, self.min_iter, self.accuracy_threshold, bool(self._H), x0.device,
                           cap=total + R + 2)
        X = [torch.empty_like(x0) for _ in range(R)]
        Z = [None if z0 is None else torch.empty_like(z0) for _ in range(R)]
        X[R - 1].copy_(x0)
        if z0 is not None:
            Z[R - 1].copy_(z0)
        # one eager iteration and reduction first (discarded): lazy library state (plans, workspaces) is
        # created outside the capture
        self._update_dev({'primal_variable': X[R - 1], 'dual_variable': Z[R - 1]})
        O.rel_sums(X[R - 1], X[R - 1], loop.sums[0:2])
        host = [torch.zeros(2, dtype=torch.int32, pin_memory=True) for _ in range(2)]
        torch.cuda.synchronize()
        graphs, pool = [], None
        try:
            for h in range(2):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool):
                    for j in range(C):
                        slot, prev = h * C + j, (h * C + j - 1) % R
                        self._update_dev({'primal_variable': X[prev], 'dual_variable': Z[prev]},
                                         out=(X[slot], Z[slot] if self._H else None))
                        loop.record_captured(X[prev], X[slot], Z[prev], Z[slot])
                    host[h].copy_(loop.ctrl.view(torch.int32)[:2], non_blocking=True)
                pool = g.pool()
                graphs.append(g)
        except Exception:  # noqa: BLE001 -- torch's capture errors and the ABI's HipError alike
            torch.cuda.synchronize()
            return None
        self._graph_used = True
        show = None
        if self.verbose is not None:
            every = int(self.verbose)

            def show(lo, hi):
                for k in range(lo, hi):
                    if k % every == 0:
                        h = loop.hist[2 * k:2 * k + 2].cpu().numpy()
                        self._rows = [[k, h[0], h[1]] if self._H else [k, h[0]]]
                        self.print_diagnostics()
        max_chunks = -(-total // C) + 2  # the control stops the loop by then (max_iter, history length)
        inflight, k, n, shown = [], 0, None, 0
        while n is None:
            if k < max_chunks:
                graphs[k % 2].replay()
                ev = torch.cuda.Event()
                ev.record()
                inflight.append((k, ev))
                k += 1
            if len(inflight) >= 2 or (k >= max_chunks and inflight):
                kc, ev = inflight.pop(0)
                ev.synchronize()
                it, stopped = int(host[kc % 2][0]), int(host[kc % 2][1])
                if show is not None:
                    show(shown, it)
                    shown = it
                if stopped:
                    n = it
            elif k >= max_chunks:
                raise RuntimeError('generic PDS loop: the device control never stopped')
        torch.cuda.synchronize()  # the chunk run ahead of the stop has finished with the ring
        self.iter = n
        h = loop.rows(n)
        self._rows = [[i, h[i, 0], h[i, 1]] if self._H else [i, h[i, 0]] for i in range(n)]
        last = (n - 1) % R
        self._state = {'primal_variable': X[last], 'dual_variable': Z[last] if self._H else None}
        self.converged = True
        cols = ['Iter', 'Relative Improvement (primal variable)']
        if self._H:
            cols.append('Relative Improvement (dual variable)')
        self.diagnostics = _frame(cols, self._rows)
        self.iterand = {'primal_variable': self._out(self._state['primal_variable']),
                        'dual_variable': self._out(self._state['dual_variable'])}
        return self.iterand, self.converged, self.diagnostics

    def _update_dev(self, st, out=None):
        """``PrimalDualSplitting.update_iterand`` (proxalgs.py:343-355) on device tensors (``out``: the
        (x, z) buffers the relaxation steps write)."""
        ox, oz = (None, None) if out is None else out
        x, z = st['primal_variable'], st['dual_variable']
        g = self.F._grad(x)
        if self._H:
            v = O.sub2(x, g, self.K._adj(z), self.tau, self.tau)
        else:
            v = O.axpby(x, g, 1.0, -self.tau)
        x_temp = self.G._prox(v, self.tau)
        if self._H:
            u = O.axpby(x_temp, x, 2.0, -1.0)
            w = O.axpby(z, self.K._apply(u), 1.0, self.sigma)
            z_temp = self.H._fenchel(w, self.sigma)
            z = O.axpby(z_temp, z, self.rho, 1 - self.rho, out=oz)
        x = O.axpby(x_temp, x, self.rho, 1 - self.rho, out=ox)
        return {'primal_variable': x, 'dual_variable': z}

    def update_iterand(self):
        if not hasattr(self, '_state') or self.iter == 0:
            dtype = self._compute_dtype()
            self._state = {'primal_variable': O.to_dev(self.x0, dtype),
                           'dual_variable': None if self.z0 is None else O.to_dev(self.z0, dtype)}
        self._state = self._update_dev(self._state)
        return {'primal_variable': self._out(self._state['primal_variable']),
                'dual_variable': self._out(self._state['dual_variable'])}

    def print_diagnostics(self):
        print(dict(zip(['Iter', 'Relative Improvement (primal variable)', 'Relative Improvement (dual variable)'],
                       self._rows[-1])))

    def stopping_metric(self):
        if self.iter == 0:
            return np.inf
        return self._rows[self.iter - 1][1]

    def update_diagnostics(self):
        row = [self.iter, _rel_improvement(self._old['primal_variable'], self._state['primal_variable'])]
        if self._H:
            row.append(_rel_improvement(self._old['dual_variable'], self._state['dual_variable']))
        self._rows.append(row)


PDS = PrimalDualSplitting


class AcceleratedProximalGradientDescent(GenericIterativeAlgorithm):
    """Accelerated proximal gradient descent (``pycsou/opt/proxalgs.py:400-622``)."""

    def __init__(self, dim, F=None, G=None, tau=None, acceleration='CD', beta=None, x0=None, max_iter=500,
                 min_iter=10, accuracy_threshold=1e-3, verbose=1, d=75.):
        self.dim = dim
        self.acceleration = acceleration
        self.d = d
        if isinstance(F, DifferentiableMap):
            if F.shape[1] != dim:
                raise ValueError(f'F does not have the proper dimension: {F.shape[1]}!={dim}.')
            self.F = F
            if F.diff_lipschitz_cst < np.inf:
                self.beta = self.F.diff_lipschitz_cst if beta is None else beta
            elif (beta is not None) and isinstance(beta, Number):
                self.beta = beta
            else:
                raise ValueError('F must be a differentiable functional with Lipschitz-continuous gradient.')
        elif F is None:
            self.F = NullDifferentiableFunctional(dim=dim)
            self.beta = 0
        else:
            raise TypeError(f'F must be of type {DifferentiableMap}.')
        if isinstance(G, ProximableFunctional):
            if G.dim != dim:
                raise ValueError(f'G does not have the proper dimension: {G.dim}!={dim}.')
            self.G = G
        elif G is None:
            self.G = NullProximableFunctional(dim=dim)
        else:
            raise TypeError(f'G must be of type {ProximableFunctional}.')
        self.tau = tau if tau is not None else self.set_step_size()
        self._torch_out = _wants_torch(x0, F)
        self.x0 = x0 if x0 is not None else self.initialize_iterate()
        objective_functional = self.F + self.G
        init_iterand = {'iterand': self.x0, 'past_aux': 0 * self.x0, 'past_t': 1}
        super().__init__(objective_functional=objective_functional, init_iterand=init_iterand, max_iter=max_iter,
                         min_iter=min_iter, accuracy_threshold=accuracy_threshold, verbose=verbose)

    def set_step_size(self):
        return 1 / self.beta

    def initialize_iterate(self):
        return np.zeros(shape=(self.dim,), dtype=np.float64)

    def _compute_dtype(self):
        for a in [self.x0] + _find_arrays(self.F):
            if isinstance(a, torch.Tensor) and a.dtype in (torch.float32, torch.float64):
                return a.dtype
            if isinstance(a, np.ndarray) and a.dtype in (np.float32, np.float64):
                return torch.float32 if a.dtype == np.float32 else torch.float64
        return torch.float64

    def _out(self, t):
        return t if self._torch_out else t.detach().cpu().numpy()

    def iterate(self):
        """The reference loop (solver.py:55-76) with the stopping rule evaluated on the device
        (``_DeviceLoop``; the fused step writes its two norms straight into the loop's sums)."""
        dtype = self._compute_dtype()
        x0 = O.to_dev(self.x0, dtype)
        loop = _DeviceLoop(self.max_iter, self.min_iter, self.accuracy_threshold, False, x0.device)
        if self.verbose is not None:
            def show(k, h):
                self._rows = [[k, h[0]]]
                self.print_diagnostics()
            loop.stream_rows(self.verbose, show)
        states = {-1: (x0, torch.zeros_like(x0), 1)}
        i, n = 0, None
        while n is None:
            if i >= loop.total:
                n = loop.poll(drain=True)
                break
            self.iter = i  # the 'CD' momentum reads the iteration index (proxalgs.py:596-598)
            new = self._update_dev(states[i - 1], sums_out=loop.sums[0:2])
            if self._sums is None:
                O.rel_sums(states[i - 1][0], new[0], loop.sums[0:2])
            loop.finalize()
            states[i] = new
            states.pop(i - loop.lag - 3, None)
            i += 1
            n = loop.poll()
        self.iter = n
        h = loop.rows(n)
        self._rows = [[k, h[k, 0]] for k in range(n)]
        self._state = states[n - 1]
        self.converged = True
        self.diagnostics = _frame(['Iter', 'Relative Improvement'], self._rows)
        x, aux, t = self._state
        self.iterand = {'iterand': self._out(x), 'past_aux': self._out(aux), 'past_t': t}
        return self.iterand, self.converged, self.diagnostics

    def _g_kind(self):
        """(kind, lam, seg) of G for the fused step (pcs_apgd_step), or None."""
        from .. import _lib as L
        from ..core.functional import ProxFuncPostComp
        from ..func.base import IndicatorFunctional
        from ..func.penalty import L1Norm
        G, lam = self.G, 1.0
        if isinstance(G, ProxFuncPostComp) and G.shift == 0 and isinstance(G.prox_func, L1Norm):
            G, lam = G.prox_func, float(G.scale)
        if isinstance(G, NullProximableFunctional):
            return L.PCS_G_NULL, 1.0, (0.0, 1.0)
        if isinstance(G, L1Norm):
            return L.PCS_APGD_G_L1, lam, (0.0, 1.0)
        if isinstance(G, IndicatorFunctional) and G.kind == 'nonneg':
            return L.PCS_G_NONNEG, 1.0, (0.0, 1.0)
        if isinstance(G, IndicatorFunctional) and G.kind == 'segment':
            return L.PCS_G_SEGMENT, 1.0, tuple(G.params)
        return None

    def _momentum(self, t_old):
        if self.acceleration == 'BT':
            t = (1 + np.sqrt(1 + 4 * t_old ** 2)) / 2
        elif self.acceleration == 'CD':
            t = (self.iter + self.d) / self.d
        else:
            t = t_old = 1
        return t, (t_old - 1) / t

    def _update_dev(self, st, sums_out=None):
        """``proxalgs.py:586-601``: G.prox, the momentum step and the diagnostics' two norms in
        one kernel (pcs_apgd_step) when G is null / lam*L1 / an orthant or segment indicator."""
        x, x_old, t_old = st
        t, a = self._momentum(t_old)
        gk = self._g_kind()
        if gk is not None:
            kind, lam, seg = gk
            xn, x_temp, self._sums = O.apgd_step(x, self.F._grad(x), x_old, self.tau, a, kind, lam, seg,
                                                 sums=sums_out)
            return (xn, x_temp, t)
        self._sums = None
        x_temp = self.G._prox(O.axpby(x, self.F._grad(x), 1.0, -self.tau), self.tau)
        x = O.axpby(x_temp, O.axpby(x_temp, x_old, 1.0, -1.0), 1.0, a)
        return (x, x_temp, t)

    def update_iterand(self):
        if not hasattr(self, '_state') or self.iter == 0:
            x0 = O.to_dev(self.x0, self._compute_dtype())
            self._state = (x0, torch.zeros_like(x0), 1)
        self._state = self._update_dev(self._state)
        x, aux, t = self._state
        return {'iterand': self._out(x), 'past_aux': self._out(aux), 'past_t': t}

    def print_diagnostics(self):
        print(dict(zip(['Iter', 'Relative Improvement'], self._rows[-1])))

    def stopping_metric(self):
        if self.iter == 0:
            return np.inf
        return self._rows[self.iter - 1][1]

    def update_diagnostics(self):
        sums = getattr(self, '_sums', None)
        if sums is None:
            self._rows.append([self.iter, _rel_improvement(self._old, self._state[0])])
            return
        d2, n2 = sums.tolist()  # ||x_old - x||^2, ||x_old||^2 from the fused step
        self._rows.append([self.iter, np.inf if n2 == 0 else float(np.sqrt(d2) / np.sqrt(n2))])


APGD = AcceleratedProximalGradientDescent


class ChambollePockSplitting(PrimalDualSplitting):
    """``proxalgs.py:628-716``: PDS with F = 0, rho = 1."""

    def __init__(self, dim, G=None, H=None, K=None, tau=None, sigma=None, rho=1, x0=None, z0=None, max_iter=500,
                 min_iter=10, accuracy_threshold=1e-3, verbose=1):
        super().__init__(dim=dim, F=None, G=G, H=H, K=K, tau=tau, sigma=sigma, rho=rho, x0=x0, z0=z0,
                         max_iter=max_iter, min_iter=min_iter, accuracy_threshold=accuracy_threshold, verbose=verbose)


CPS = ChambollePockSplitting


class DouglasRachfordSplitting(PrimalDualSplitting):
    """``proxalgs.py:719-781``: PDS with F = 0, K = I, sigma = 1/tau, rho = 1."""

    def __init__(self, dim, G=None, H=None, tau=1., x0=None, z0=None, max_iter=500, min_iter=10,
                 accuracy_threshold=1e-3, verbose=1):
        super().__init__(dim=dim, F=None, G=G, H=H, K=None, tau=tau, sigma=1 / tau, rho=1, x0=x0, z0=z0,
                         max_iter=max_iter, min_iter=min_iter, accuracy_threshold=accuracy_threshold, verbose=verbose)


DRS = DouglasRachfordSplitting


class ForwardBackwardSplitting(PrimalDualSplitting):
    """``proxalgs.py:784-862``: PDS with H = 0."""

    def __init__(self, dim, F=None, G=None, tau=None, rho=1, x0=None, max_iter=500, min_iter=10,
                 accuracy_threshold=1e-3, verbose=1):
        super().__init__(dim=dim, F=F, G=G, H=None, K=None, tau=tau, rho=rho, x0=x0, max_iter=max_iter,
                         min_iter=min_iter, accuracy_threshold=accuracy_threshold, verbose=verbose)


FBS = ForwardBackwardSplitting

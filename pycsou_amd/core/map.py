"""Map algebra with Lipschitz bookkeeping (mirrors ``pycsou/core/map.py``).

Semantics kept from the reference (the solvers and user scripts depend on them):

* ``Map(shape)`` -- ``shape = (range_dim, domain_dim)``; ``is_functional`` iff range 1
  (``map.py:94-112``).
* ``+`` -> ``MapSum`` / ``DiffMapSum`` (shapes must be range-broadcastable,
  ``map.py:349-357``); ``*`` / ``@`` with a number inserts a ``HomothetyMap``; with an
  array it evaluates; with a map it composes (``map.py:253-304, 534-561``).
* Lipschitz propagation: sum -> sum of constants; composition -> product, and the
  gradient-Lipschitz rule of ``DiffMapComp`` (``map.py:596-607``), including the
  ``HomothetyMap`` special case that makes ``(1/2)*SquaredL2Loss`` have beta = 1.

Evaluation is split in two layers: ``__call__`` / ``jacobianT`` accept NumPy or torch
and return the same kind; ``_apply`` / ``_jacT`` work on flat device tensors and are
what the solvers call.
"""

from numbers import Number

import numpy as np
import torch

from .. import _ops as O
from ..util.misc import is_range_broadcastable, range_broadcast_shape


def _mul(a, b):
    """Product of two jacobianT factors: operator*vector applies, vector*scalar scales,
    operator*operator composes (the ``*`` of ``map.py:610``)."""
    from .linop import LinearOperator
    if isinstance(a, LinearOperator):
        if isinstance(b, torch.Tensor):
            return a._apply(b)
        return a * b
    if isinstance(a, torch.Tensor):
        if isinstance(b, Number):
            return O.scale(a, b)
        if isinstance(b, torch.Tensor) and b.numel() == 1:
            return O.scale(a, float(b.item()))
    if isinstance(a, Number):
        if isinstance(b, torch.Tensor):
            return O.scale(b, a)
        if isinstance(b, Number):
            return a * b
    raise NotImplementedError(f'cannot multiply {type(a).__name__} by {type(b).__name__}')


class Map:
    """Base class of all maps ``R^N -> R^M`` (``pycsou/core/map.py:20-334``)."""

    def __init__(self, shape, is_linear=False, is_differentiable=False):
        if len(shape) > 2:
            raise NotImplementedError('Shapes of map objects must be tuples of length 2 (tensorial maps not supported).')
        self.shape = tuple(shape)
        self.is_linear = is_linear
        self.is_functional = self.shape[0] == 1
        self.is_differentiable = is_differentiable

    # -- evaluation
    def _apply(self, t):
        raise NotImplementedError

    def __call__(self, arg):
        if isinstance(arg, Number):
            arg = np.asarray([arg], dtype=float)
        t = O.to_dev(arg)
        out = self._apply(t)
        if isinstance(out, torch.Tensor):
            return O.like(out, arg)
        return out

    def apply_along_axis(self, arr, axis=0):
        if arr.shape[axis] != self.shape[1]:
            raise ValueError(f"Array size along specified axis and the map domain's dimension differ: "
                             f"{arr.shape[axis]} != {self.shape[1]}.")
        return np.apply_along_axis(func1d=self.__call__, axis=axis, arr=np.asarray(arr))

    def shifter(self, shift):
        return MapShifted(map=self, shift=shift)

    # -- algebra
    def __add__(self, other):
        if isinstance(other, Map):
            return MapSum(self, other)
        raise NotImplementedError

    def __radd__(self, other):
        if isinstance(other, Map):
            return MapSum(other, self)
        raise NotImplementedError

    def __mul__(self, other):
        if isinstance(other, Number):
            from ..linop.base import HomothetyMap
            other = HomothetyMap(constant=other, size=self.shape[1])
        if O.is_array(other):
            return self(other)
        if isinstance(other, Map):
            return MapComp(self, other)
        raise NotImplementedError

    def __rmul__(self, other):
        if isinstance(other, Number):
            from ..linop.base import HomothetyMap
            other = HomothetyMap(constant=other, size=self.shape[0])
        if isinstance(other, Map):
            return MapComp(other, self)
        raise NotImplementedError

    def __matmul__(self, other):
        return self.__mul__(other)

    def __neg__(self):
        return self.__mul__(-1)

    def __sub__(self, other):
        return self.__add__(other.__neg__())

    def __pow__(self, power):
        if type(power) is int:
            out = self
            for _ in range(1, power):
                out = self.__mul__(out)
            return out
        raise NotImplementedError

    def __truediv__(self, scalar):
        if isinstance(scalar, Number):
            return self.__mul__(1 / scalar)
        raise NotImplementedError


def _shift_dev(shift, like=None):
    if isinstance(shift, Number):
        return shift
    dtype = None if like is None else like.dtype
    return O.to_dev(shift, dtype)


class MapShifted(Map):
    """``x -> map(x + shift)`` (``map.py:337-346``)."""

    def __init__(self, map, shift):
        self.map = map
        self.shift = shift
        if O.numel(shift) != map.shape[1]:
            raise TypeError('Invalid shift size.')
        self._shift_cache = {}
        Map.__init__(self, shape=map.shape, is_linear=map.is_linear, is_differentiable=map.is_differentiable)

    def _shifted(self, t):
        key = (t.dtype, t.device)
        s = self._shift_cache.get(key)
        if s is None:
            s = _shift_dev(self.shift, t)
            self._shift_cache[key] = s
        if isinstance(s, Number):
            return O.axpby(t, None, 1.0, 0.0) if s == 0 else torch.add(t, s)
        return O.add(t, s)

    def _apply(self, t):
        return self.map._apply(self._shifted(t))


class MapSum(Map):
    """``map1 + map2`` (``map.py:349-360``)."""

    def __init__(self, map1, map2):
        if not is_range_broadcastable(map1.shape, map2.shape):
            raise ValueError('Cannot sum two maps with inconsistent range or domain sizes.')
        Map.__init__(self, shape=range_broadcast_shape(map1.shape, map2.shape),
                     is_linear=map1.is_linear & map2.is_linear,
                     is_differentiable=map1.is_differentiable & map2.is_differentiable)
        self.map1, self.map2 = map1, map2

    def _apply(self, t):
        a, b = self.map1._apply(t), self.map2._apply(t)
        if isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor):
            return O.add(a, b)
        return a + b


class MapComp(Map):
    """``map1 o map2`` (``map.py:375-387``)."""

    def __init__(self, map1, map2):
        if map1.shape[1] != map2.shape[0] and map2.shape[0] != 1 and map1.shape[1] != 1:
            raise ValueError('Cannot compose two maps with inconsistent range or domain sizes.')
        Map.__init__(self, shape=(map1.shape[0], map2.shape[1]), is_linear=map1.is_linear & map2.is_linear,
                     is_differentiable=map1.is_differentiable & map2.is_differentiable)
        self.map1, self.map2 = map1, map2

    def _apply(self, t):
        return self.map1._apply(self.map2._apply(t))


class DifferentiableMap(Map):
    """Differentiable map with ``lipschitz_cst`` / ``diff_lipschitz_cst`` (``map.py:390-561``)."""

    def __init__(self, shape, is_linear=False, lipschitz_cst=np.inf, diff_lipschitz_cst=np.inf):
        Map.__init__(self, shape=shape, is_linear=is_linear, is_differentiable=True)
        self.lipschitz_cst = lipschitz_cst
        self.diff_lipschitz_cst = diff_lipschitz_cst

    def _jacT(self, t):
        """Device-level jacobianT: returns a device tensor, a number or a LinearOperator."""
        raise NotImplementedError

    def jacobianT(self, arg):
        t = None if arg is None else O.to_dev(arg)
        out = self._jacT(t)
        if isinstance(out, torch.Tensor):
            return O.like(out, arg)
        return out

    def gradient(self, arg):
        return self.jacobianT(arg)

    def _grad(self, t):
        return self._jacT(t)

    def compute_lipschitz_cst(self):
        pass

    def compute_diff_lipschitz_cst(self):
        pass

    def shifter(self, shift):
        return DiffMapShifted(map=self, shift=shift)

    def __add__(self, other):
        if isinstance(other, DifferentiableMap):
            return DiffMapSum(self, other)
        if isinstance(other, Map):
            return MapSum(self, other)
        raise NotImplementedError

    def __radd__(self, other):
        if isinstance(other, DifferentiableMap):
            return DiffMapSum(self, other)
        if isinstance(other, Map):
            return MapSum(self, other)
        raise NotImplementedError

    def __mul__(self, other):
        if isinstance(other, Number):
            from ..linop.base import HomothetyMap
            other = HomothetyMap(constant=other, size=self.shape[1])
        if O.is_array(other):
            return self(other)
        if isinstance(other, DifferentiableMap):
            return DiffMapComp(self, other)
        if isinstance(other, Map):
            return MapComp(self, other)
        raise NotImplementedError

    def __rmul__(self, other):
        if isinstance(other, Number):
            from ..linop.base import HomothetyMap
            other = HomothetyMap(constant=other, size=self.shape[0])
        if isinstance(other, DifferentiableMap):
            return DiffMapComp(other, self)
        if isinstance(other, Map):
            return MapComp(other, self)
        raise NotImplementedError


class DiffMapShifted(MapShifted, DifferentiableMap):
    """``map.py:564-572``."""

    def __init__(self, map, shift):
        MapShifted.__init__(self, map=map, shift=shift)
        DifferentiableMap.__init__(self, shape=self.shape, is_linear=self.is_linear, lipschitz_cst=map.lipschitz_cst,
                                   diff_lipschitz_cst=map.diff_lipschitz_cst)

    def _jacT(self, t):
        return self.map._jacT(self._shifted(t))


class DiffMapSum(MapSum, DifferentiableMap):
    """``map.py:575-583``."""

    def __init__(self, map1, map2):
        MapSum.__init__(self, map1=map1, map2=map2)
        DifferentiableMap.__init__(self, shape=self.shape, is_linear=self.is_linear,
                                   lipschitz_cst=map1.lipschitz_cst + map2.lipschitz_cst,
                                   diff_lipschitz_cst=map1.diff_lipschitz_cst + map2.diff_lipschitz_cst)

    def _jacT(self, t):
        a, b = self.map1._jacT(t), self.map2._jacT(t)
        if isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor):
            return O.add(a, b)
        return a + b


class DiffMapComp(MapComp, DifferentiableMap):
    """``map1 o map2`` with the chain rule ``J^T = J2^T(x) * J1^T(map2(x))`` (``map.py:596-610``)."""

    def __init__(self, map1, map2):
        from ..linop.base import HomothetyMap
        MapComp.__init__(self, map1=map1, map2=map2)
        lip = map2.lipschitz_cst * map1.lipschitz_cst
        if isinstance(map1, HomothetyMap):
            dlip = map1.diff_lipschitz_cst * map2.diff_lipschitz_cst
        else:
            dlip = map1.diff_lipschitz_cst * map2.diff_lipschitz_cst * map2.lipschitz_cst
        DifferentiableMap.__init__(self, shape=self.shape, is_linear=self.is_linear, lipschitz_cst=lip,
                                   diff_lipschitz_cst=dlip)

    def _jacT(self, t):
        from .linop import LinearOperator
        j2 = self.map2._jacT(t)
        # A linear map1's jacobianT does not depend on its argument: skip evaluating
        # map2(x) (the reference computes it and, for the loss, discards ||r-y||^2).
        if isinstance(self.map1, LinearOperator):
            j1 = self.map1._jacT(None)
        else:
            j1 = self.map1._jacT(self.map2._apply(t))
        return _mul(j2, j1)


# ---------------------------------------------------------------- stacks (map.py:613-958)
def _sections(block_sizes):
    """Offsets of ``np.split(x, np.cumsum(block_sizes))``: block i is ``[o[i], o[i+1])``."""
    return [0] + [int(s) for s in np.cumsum(block_sizes)]


def _as_flat(v, like):
    """A block result as a flat device tensor (functionals return numbers)."""
    if isinstance(v, torch.Tensor):
        return v.reshape(-1)
    return torch.as_tensor(np.asarray(v, dtype=np.float64).reshape(-1), device=like.device,
                           dtype=like.dtype if like.dtype.is_floating_point else torch.float64)


def _cat(parts, like):
    """np.concatenate of flat device blocks into one new buffer (one copy per block)."""
    parts = [_as_flat(p, like) for p in parts]
    out = torch.empty(sum(p.numel() for p in parts), dtype=parts[0].dtype, device=parts[0].device)
    o = 0
    for p in parts:
        out[o:o + p.numel()].copy_(p)
        o += p.numel()
    return out


class MapStack(Map):
    """Vertical (``axis=0``: ``x -> (f_1(x), ..., f_k(x))``) or horizontal (``axis=1``:
    ``(x_1, ..., x_k) -> sum_i f_i(x_i)``) stacking (``map.py:613-743``).  The blocks run one
    after the other on the current stream; ``n_jobs`` / ``joblib_backend`` are accepted for
    API compatibility (the reference's joblib fan-out has no GPU counterpart)."""

    def __init__(self, *maps, axis, n_jobs=1, joblib_backend='loky'):
        self.maps = list(maps)
        if np.abs(axis) > 1:
            ValueError('Axis must be one of {0, 1,-1}.')  # the reference builds but does not raise (map.py:703-704)
        self.axis = int(axis)
        self.is_linear_list = [m.is_linear for m in self.maps]
        self.is_differentiable_list = [m.is_differentiable for m in self.maps]
        self.shapes = np.array([m.shape for m in self.maps])
        self.block_sizes = [m.shape[axis] for m in self.maps]
        self.sections = np.cumsum(self.block_sizes)
        self._off = _sections(self.block_sizes)
        self.n_jobs = n_jobs
        self.joblib_backend = joblib_backend
        if not self.is_valid_stack():
            raise ValueError('Inconsistent map shapes for  stacking.')
        Map.__init__(self, shape=self.get_shape(), is_linear=bool(np.prod(self.is_linear_list).astype(bool)),
                     is_differentiable=bool(np.prod(self.is_differentiable_list).astype(bool)))

    def is_valid_stack(self):
        col_sizes = [m.shape[1 - self.axis] for m in self.maps]
        return np.unique(col_sizes).size == 1

    def get_shape(self):
        sizes = [m.shape[self.axis] for m in self.maps]
        if self.axis == 0:
            return int(np.sum(sizes).astype(int)), self.maps[0].shape[1 - self.axis]
        return self.maps[0].shape[1 - self.axis], int(np.sum(sizes).astype(int))

    def _split(self, t):
        o = self._off
        return [t[o[i]:o[i + 1]] for i in range(len(self.maps))]

    def _apply(self, t):
        if self.axis == 0:
            return _cat([m._apply(t) for m in self.maps], t)
        result = 0
        for m, xi in zip(self.maps, self._split(t)):
            r = m._apply(xi)
            if isinstance(result, torch.Tensor) and isinstance(r, torch.Tensor):
                result = O.add(result, r)
            else:
                result = result + r
        return result


class MapVStack(MapStack):
    """``MapStack(*maps, axis=0)`` (``map.py:746-780``)."""

    def __init__(self, *maps, n_jobs=1, joblib_backend='loky'):
        super().__init__(*maps, axis=0, n_jobs=n_jobs, joblib_backend=joblib_backend)


class MapHStack(MapStack):
    """``MapStack(*maps, axis=1)`` (``map.py:783-825``)."""

    def __init__(self, *maps, n_jobs=1, joblib_backend='loky'):
        super().__init__(*maps, axis=1, n_jobs=n_jobs, joblib_backend=joblib_backend)


class DiffMapStack(MapStack, DifferentiableMap):
    """Stack of differentiable maps (``map.py:828-942``): vertical stacks have Lipschitz
    constants ``sqrt(sum L_i^2)``, horizontal ones ``max L_i``; ``jacobianT`` is the
    horizontal (resp. vertical) stack of the blocks' jacobianT."""

    def __init__(self, *diffmaps, axis, n_jobs=1, joblib_backend='loky'):
        MapStack.__init__(self, *diffmaps, axis=axis, n_jobs=n_jobs, joblib_backend=joblib_backend)
        if axis == 0:
            lip = np.sqrt(np.sum([m.lipschitz_cst ** 2 for m in self.maps]))
            dlip = np.sqrt(np.sum([m.diff_lipschitz_cst ** 2 for m in self.maps]))
        else:
            lip = np.max([m.lipschitz_cst for m in self.maps])
            dlip = np.max([m.diff_lipschitz_cst for m in self.maps])
        DifferentiableMap.__init__(self, shape=self.shape, is_linear=self.is_linear, lipschitz_cst=lip,
                                   diff_lipschitz_cst=dlip)

    def _jacT(self, t):
        from ..func.base import ExplicitLinearFunctional
        from ..linop.base import LinOpHStack, LinOpVStack

        def wrap(j):
            return ExplicitLinearFunctional(j) if isinstance(j, torch.Tensor) else j

        if self.axis == 0:
            return LinOpVStack(*[wrap(m._jacT(t)) for m in self.maps], n_jobs=self.n_jobs,
                               joblib_backend=self.joblib_backend)
        return LinOpHStack(*[wrap(m._jacT(xi)) for m, xi in zip(self.maps, self._split(t))], n_jobs=self.n_jobs,
                           joblib_backend=self.joblib_backend)


class DiffMapVStack(DiffMapStack):
    """``map.py:945-955``."""

    def __init__(self, *diffmaps, n_jobs=1, joblib_backend='loky'):
        super().__init__(*diffmaps, axis=0, n_jobs=n_jobs, joblib_backend=joblib_backend)


class DiffMapHStack(DiffMapStack):
    """``map.py:958-968``."""

    def __init__(self, *diffmaps, n_jobs=1, joblib_backend='loky'):
        super().__init__(*diffmaps, axis=1, n_jobs=n_jobs, joblib_backend=joblib_backend)

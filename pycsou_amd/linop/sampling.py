"""Sampling operators on the GPU (``pycsou/linop/sampling.py:25-391``).

``Masking`` (``sampling.py:125-196``), ``DownSampling`` (``sampling.py:199-391``) and
``SubSampling`` (``sampling.py:25-122`` -> ``pylops.Restriction``) keep the reference's
constructors, shape rules and errors.  The boolean mask / index list becomes int32 gather
indices and the inverse map once, on the host; forward and adjoint are the gather kernels
``pcs_gather`` / ``pcs_gather_or_zero`` (``csrc/sampling.hip``).
"""

import numpy as np
import torch

from .. import _ops as O
from ..core.linop import LinearOperator


class _Gather(LinearOperator):
    """y = x[idx]; adjoint x = 0, x[idx] = y (repeated indices: the last one wins)."""

    def _set_indices(self, idx, n):
        idx = np.asarray(idx, dtype=np.int64).reshape(-1)
        if n >= 2 ** 31:
            raise NotImplementedError('sampling operators index with int32 (size < 2^31)')
        inv = np.full(n, -1, dtype=np.int32)
        inv[idx] = np.arange(idx.size, dtype=np.int32)  # NumPy fancy assignment: last wins
        self._idx_host, self._inv_host = idx.astype(np.int32), inv
        self._idx = self._inv = None

    def _dev(self):
        if self._idx is None:
            self._idx = torch.as_tensor(self._idx_host).to(O.device())
            self._inv = torch.as_tensor(self._inv_host).to(O.device())
        return self._idx, self._inv

    def _apply(self, t):
        return O.gather(t, self._dev()[0])

    def _adj(self, t):
        return O.gather_or_zero(t, self._dev()[1])


class Masking(_Gather):
    """``sampling.py:125-196``: extract the entries marked ``True`` in ``sampling_bool``."""

    def __init__(self, size, sampling_bool, dtype=np.float64):
        self.sampling_bool = np.asarray(sampling_bool).reshape(-1).astype(bool)
        self.input_size = size
        self.nb_of_samples = self.sampling_bool[self.sampling_bool == True].size  # noqa: E712
        if self.sampling_bool.size != size:
            raise ValueError('Invalid size of boolean sampling array.')
        super().__init__(shape=(self.nb_of_samples, self.input_size), dtype=dtype)
        self._set_indices(np.flatnonzero(self.sampling_bool), size)


class DownSampling(Masking):
    """``sampling.py:199-391``: keep one sample every ``downsampling_factor`` along every axis
    (or along ``axis``); ``output_shape`` as the reference computes it."""

    def __init__(self, size, downsampling_factor, shape=None, axis=None, dtype=np.float64):
        if type(downsampling_factor) is int:
            if (shape is not None) and (axis is None):
                self.downsampling_factor = len(shape) * (downsampling_factor,)
            else:
                self.downsampling_factor = (downsampling_factor,)
        else:
            self.downsampling_factor = tuple(downsampling_factor)
        if shape is not None:
            if size != np.prod(shape):
                raise ValueError(f'Array size {size} is incompatible with array shape {shape}.')
            if (axis is not None) and (axis > len(shape) - 1):
                raise ValueError(f'Array size {size} is incompatible with array shape {shape}.')
        if (shape is None) and (len(self.downsampling_factor) > 1):
            raise ValueError('Please specify an array shape for multidimensional downsampling.')
        elif (shape is not None) and (axis is None) and (len(shape) != len(self.downsampling_factor)):
            raise ValueError(f'Inconsistent downsampling factors {downsampling_factor} for array of shape {shape}.')
        self.input_size = size
        self.input_shape = shape
        self.axis = axis
        self.downsampling_mask = self.compute_downsampling_mask()
        if self.input_shape is None:
            self.output_shape = None
        elif len(self.downsampling_factor) > 1:
            self.output_shape = tuple(int(np.sum(np.arange(n) % f == 0))
                                      for n, f in zip(self.input_shape, self.downsampling_factor))
        else:
            out = list(self.input_shape)
            out[self.axis] = int(np.sum(np.arange(self.input_shape[self.axis]) % self.downsampling_factor[0] == 0))
            self.output_shape = tuple(out)
        super().__init__(size=self.input_size, sampling_bool=self.downsampling_mask, dtype=dtype)

    def compute_downsampling_mask(self):
        if self.input_shape is None:
            return (np.arange(self.input_size) % self.downsampling_factor[0]) == 0
        if len(self.downsampling_factor) > 1:
            mask = True
            for ax in range(len(self.input_shape)):
                keep = (np.arange(self.input_shape[ax]) % self.downsampling_factor[ax]) == 0
                keep = keep.reshape(keep.shape + (len(self.input_shape) - 1) * (1,))
                mask = mask * np.swapaxes(keep, 0, ax)
        else:
            mask = np.zeros(shape=self.input_shape, dtype=bool)
            mask = np.swapaxes(mask, 0, self.axis)
            mask[(np.arange(self.input_shape[self.axis]) % self.downsampling_factor[0]) == 0, ...] = True
            mask = np.swapaxes(mask, 0, self.axis)
        return np.asarray(mask).reshape(-1)


class SubSamplingOp(_Gather):
    """``pylops.Restriction(M, iava, dims, dir)``: ``x.take(iava, axis)`` (C order)."""

    def __init__(self, size, sampling_indices, shape=None, axis=0, dtype='float64'):
        iava = np.asarray(sampling_indices, dtype=np.int64).reshape(-1)
        dims = (size,) if shape is None else tuple(int(s) for s in shape)
        if int(np.prod(dims)) != size:
            raise ValueError('shape and size are not compatible')
        idx = np.arange(size, dtype=np.int64).reshape(dims).take(iava, axis=axis).reshape(-1)
        super().__init__(shape=(idx.size, size), dtype=np.dtype(dtype))
        self.sampling_indices, self.input_shape, self.axis = iava, shape, axis
        out = list(dims)
        out[axis] = iava.size
        self.output_shape = tuple(out)
        self._set_indices(idx, size)


def SubSampling(size, sampling_indices, shape=None, axis=0, dtype='float64'):
    """``pycsou/linop/sampling.py:25-122``."""
    return SubSamplingOp(size, sampling_indices, shape=shape, axis=axis, dtype=dtype)

"""pycsou_amd -- MI355X-native engine behind the pycsou proximal-splitting API.

Same module layout as the reference (``core``, ``linop``, ``func``, ``math``, ``opt``):
scripts written against ``pycsou`` run unchanged after ``pycsou_amd.install_alias()``
(or ``import pycsou_amd as pycsou``).  All compute runs in the gfx950 HIP kernels of
``lib/libpycsou_hip.so`` through the C ABI in ``include/pycsou_hip.h``.
"""

import sys

__version__ = '0.1.0'

_SUBMODULES = ('core', 'core.map', 'core.linop', 'core.functional', 'core.solver', 'linop', 'linop.base',
               'linop.conv', 'linop.diff', 'func', 'func.base', 'func.penalty', 'func.loss', 'math', 'math.prox',
               'opt', 'opt.proxalgs', 'util', 'util.misc')


def install_alias(name='pycsou'):
    """Register this package under ``name`` so ``from pycsou.opt.proxalgs import PDS`` works."""
    import importlib
    sys.modules[name] = sys.modules[__name__]
    for sub in _SUBMODULES:
        sys.modules[f'{name}.{sub}'] = importlib.import_module(f'{__name__}.{sub}')

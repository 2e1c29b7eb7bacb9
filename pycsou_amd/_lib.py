"""ctypes binding of libpycsou_hip.so (the C ABI declared in include/pycsou_hip.h).

There is exactly one compute path: the gfx950 HIP kernels in this library.  If the
library is missing or no ROCm GPU is visible, every compute call raises -- there is
no NumPy / PyTorch fallback.
"""

import ctypes
import os

import torch  # noqa: F401  -- must be imported first: its libamdhip64.so.7 is the one we bind to

_HERE = os.path.dirname(os.path.abspath(__file__))
# PCS_LIB_PATH: diagnostics only (e.g. an ablation build of the same sources).
LIB_PATH = os.environ.get('PCS_LIB_PATH') or os.path.join(_HERE, 'lib', 'libpycsou_hip.so')

PCS_F32, PCS_F64 = 0, 1
PCS_FORWARD, PCS_BACKWARD, PCS_CENTERED = 0, 1, 2
PCS_H_L1, PCS_H_L21 = 0, 1
PCS_K_GRAD_FORWARD, PCS_K_GRAD_BACKWARD, PCS_K_GRAD_CENTERED, PCS_K_LAPLACIAN = 0, 1, 2, 3
PCS_G_NULL, PCS_G_NONNEG, PCS_G_SEGMENT = 0, 1, 2
PCS_APGD_G_L1 = 3
PCS_F_NULL, PCS_F_DENOISE, PCS_F_SEPCONV, PCS_F_GRADBUF, PCS_F_CONV2D, PCS_F_CONV0 = 0, 1, 2, 3, 4, 5
PCS_M_NONE, PCS_M_L1LOSS = 0, 1
# pcs_pds2d_path: the kernel family of a fused 2-D step
(PCS_PATH_TILE, PCS_PATH_MARCH, PCS_PATH_NMARCH, PCS_PATH_PT, PCS_PATH_SMARCH, PCS_PATH_SMARCH_NX, PCS_PATH_NM64,
 PCS_PATH_CONV2D) = range(1, 9)
PCS_PATH_FUSED_NORMAL = (PCS_PATH_NMARCH, PCS_PATH_NM64)  # grad F = N x - Conv^T y inside the one launch
KINDS = {'forward': PCS_FORWARD, 'backward': PCS_BACKWARD, 'centered': PCS_CENTERED}

_c_int, _c_i64, _c_dbl, _vp = ctypes.c_int, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p
_pi64 = ctypes.POINTER(ctypes.c_int64)
_pdbl = ctypes.POINTER(ctypes.c_double)


class PdsArgs(ctypes.Structure):
    """Mirror of pcs_pds2d_args."""
    _fields_ = [('dtype', _c_int), ('fkind', _c_int), ('hkind', _c_int), ('gkind', _c_int),
                ('n0', _c_i64), ('n1', _c_i64), ('row0', _c_i64), ('rows', _c_i64),
                ('halo_x', _c_int), ('halo_z', _c_int), ('halo_y', _c_int), ('half', _c_int),
                ('taps0', _vp), ('taps1', _vp),
                ('tau', _c_dbl), ('sigma', _c_dbl), ('rho', _c_dbl), ('lam', _c_dbl),
                ('step0', _c_dbl), ('step1', _c_dbl), ('seg_a', _c_dbl), ('seg_b', _c_dbl),
                ('x', _vp), ('xn', _vp), ('z', _vp), ('zn', _vp), ('y', _vp), ('gbuf', _vp),
                ('partials', _vp), ('ctrl', _vp), ('hist', _vp), ('ws', _vp),
                ('sums_out', _vp), ('pre_partials', _vp), ('n_pre', _c_i64),
                ('cty', _vp), ('ntaps', _vp),
                ('kkind', _c_int), ('edge', _c_int), ('w0', _c_dbl), ('w1', _c_dbl),
                ('conv_fwd', _vp), ('conv_adj', _vp), ('conv_tier', _c_int), ('pad3', _c_int), ('rbuf', _vp),
                ('mkind', _c_int), ('pad4', _c_int), ('ym', _vp), ('zm', _vp), ('zmn', _vp),
                ('fin_partials', _vp)]


class StencilArgs(ctypes.Structure):
    """Mirror of pcs_pds2d_stencil_args."""
    _fields_ = [('dtype', _c_int), ('kkind', _c_int), ('fkind', _c_int), ('hkind', _c_int), ('gkind', _c_int),
                ('edge', _c_int), ('n0', _c_i64), ('n1', _c_i64),
                ('tau', _c_dbl), ('sigma', _c_dbl), ('rho', _c_dbl), ('lam', _c_dbl), ('step0', _c_dbl),
                ('step1', _c_dbl), ('w0', _c_dbl), ('w1', _c_dbl), ('seg_a', _c_dbl), ('seg_b', _c_dbl),
                ('x', _vp), ('xn', _vp), ('z', _vp), ('zn', _vp), ('g', _vp),
                ('partials', _vp), ('ctrl', _vp), ('hist', _vp), ('ws', _vp)]


class Pds3Args(ctypes.Structure):
    """Mirror of pcs_pds3d_args."""
    _fields_ = [('dtype', _c_int), ('fkind', _c_int), ('hkind', _c_int), ('gkind', _c_int),
                ('n0', _c_i64), ('n1', _c_i64), ('n2', _c_i64), ('plane0', _c_i64), ('planes', _c_i64),
                ('halo_x', _c_int), ('halo_z', _c_int), ('halo_g', _c_int), ('pad', _c_int),
                ('tau', _c_dbl), ('sigma', _c_dbl), ('rho', _c_dbl), ('lam', _c_dbl),
                ('step0', _c_dbl), ('step1', _c_dbl), ('step2', _c_dbl), ('seg_a', _c_dbl), ('seg_b', _c_dbl),
                ('x', _vp), ('xn', _vp), ('z', _vp), ('zn', _vp), ('g', _vp),
                ('partials', _vp), ('ctrl', _vp), ('hist', _vp), ('ws', _vp), ('kkind', _c_int), ('edge', _c_int),
                ('conv0_w', _vp), ('conv0_taps', _vp), ('conv0_k', _c_int), ('conv0_off', _c_int)]


class HaloSet(ctypes.Structure):
    """Mirror of pcs_halo_set."""
    _fields_ = [('nbuf', _c_int), ('pad', _c_int), ('send_lo', _vp * 4), ('recv_lo', _vp * 4),
                ('send_hi', _vp * 4), ('recv_hi', _vp * 4), ('bytes', _c_i64 * 4)]


class Slab2DDesc(ctypes.Structure):
    """Mirror of pcs_slab2d_desc."""
    _fields_ = [('world', _c_int), ('rank', _c_int), ('step', PdsArgs * 2), ('halo', HaloSet * 2),
                ('ctrl', _vp), ('hist', _vp), ('band', _c_i64), ('overlap', _c_int), ('pad2', _c_int)]


DEEP_MAX = 8


class SlabDeepDesc(ctypes.Structure):
    """Mirror of pcs_slab2d_deep_desc (ABI 9)."""
    _fields_ = [('world', _c_int), ('rank', _c_int), ('depth', _c_int), ('nbuf', _c_int), ('reach', _c_int),
                ('local', _c_int), ('step', PdsArgs * DEEP_MAX), ('halo', HaloSet * DEEP_MAX), ('ctrl', _vp),
                ('hist', _vp)]

# name -> (restype, argtypes)
_SIGS = {
    'pcs_abi_version': (_c_int, []),
    'pcs_deriv1_fwd': (_c_int, [_c_int, _vp, _vp, _c_int, _pi64, _c_int, _c_dbl, _c_int, _c_int, _vp]),
    'pcs_deriv1_adj': (_c_int, [_c_int, _vp, _vp, _c_int, _pi64, _c_int, _c_dbl, _c_int, _c_int, _vp]),
    'pcs_deriv2_fwd': (_c_int, [_c_int, _vp, _vp, _c_int, _pi64, _c_int, _c_dbl, _c_int, _vp]),
    'pcs_deriv2_adj': (_c_int, [_c_int, _vp, _vp, _c_int, _pi64, _c_int, _c_dbl, _c_int, _vp]),
    'pcs_gather': (_c_int, [_c_int, _vp, _vp, _vp, _c_i64, _vp]),
    'pcs_gather_or_zero': (_c_int, [_c_int, _vp, _vp, _vp, _c_i64, _vp]),
    'pcs_grad_fwd': (_c_int, [_c_int, _vp, _vp, _c_int, _pi64, _pdbl, _c_int, _c_int, _vp]),
    'pcs_grad_adj': (_c_int, [_c_int, _vp, _vp, _c_int, _pi64, _pdbl, _c_int, _c_int, _vp]),
    'pcs_lap_fwd': (_c_int, [_c_int, _vp, _vp, _pi64, _pdbl, _pdbl, _c_int, _vp]),
    'pcs_lap_adj': (_c_int, [_c_int, _vp, _vp, _pi64, _pdbl, _pdbl, _c_int, _vp]),
    'pcs_conv2d': (_c_int, [_c_int, _vp, _vp, _c_i64, _c_i64, _vp, _c_int, _c_int, _c_int, _c_int, _vp, _c_dbl,
                            _vp]),
    'pcs_conv2d_plan_tier': (_c_int, [_c_int, _c_int, _c_int, _c_int]),
    'pcs_conv2d_plan_bytes': (_c_i64, [_c_int, _c_int, _c_int, _c_int, _c_int]),
    'pcs_conv2d_plan_pack': (_c_int, [_c_int, _pdbl, _c_int, _c_int, _c_int, _c_int, _c_int, _vp]),
    'pcs_conv2d_planned': (_c_int, [_c_int, _vp, _vp, _c_i64, _c_i64, _vp, _c_int, _vp, _c_dbl, _vp]),
    'pcs_conv1d': (_c_int, [_c_int, _vp, _vp, _c_int, _pi64, _c_int, _vp, _c_int, _c_int, _vp]),
    'pcs_conv2d_sep_planes': (_c_int, [_c_int, _vp, _vp, _c_i64, _c_i64, _c_i64, _vp, _c_int, _c_int, _vp, _c_int,
                                        _c_int, _c_int, _vp]),
    'pcs_conv2d_sep_ata_planes': (_c_int, [_c_int, _vp, _vp, _c_i64, _c_i64, _c_i64, _vp, _c_int, _c_int, _vp,
                                            _c_int, _c_int, _vp]),
    'pcs_conv0_residual_adjoint': (_c_int, [_c_int, _vp, _vp, _vp, _c_i64, _c_i64, _vp, _c_int, _c_int, _c_i64,
                                             _c_i64, _c_i64, _c_i64, _vp]),
    'pcs_prox_l1': (_c_int, [_c_int, _vp, _vp, _c_i64, _c_dbl, _vp]),
    'pcs_fenchel_l1': (_c_int, [_c_int, _vp, _vp, _c_i64, _c_dbl, _c_dbl, _vp]),
    'pcs_prox_l21_pixel': (_c_int, [_c_int, _vp, _vp, _c_i64, _c_int, _c_dbl, _vp]),
    'pcs_fenchel_l21_pixel': (_c_int, [_c_int, _vp, _vp, _c_i64, _c_int, _c_dbl, _c_dbl, _vp]),
    'pcs_prox_l21_labels': (_c_int, [_c_int, _vp, _vp, _c_i64, _vp, _c_i64, _c_dbl, _vp, _vp]),
    'pcs_prox_l21_groups': (_c_int, [_c_int, _vp, _vp, _c_i64, _vp, _c_i64, _vp, _vp, _c_i64, _c_dbl, _vp, _vp]),
    'pcs_prox_l2': (_c_int, [_c_int, _vp, _vp, _c_i64, _c_dbl, _vp, _vp]),
    'pcs_prox_sql2': (_c_int, [_c_int, _vp, _vp, _c_i64, _c_dbl, _vp]),
    'pcs_proj_nonneg': (_c_int, [_c_int, _vp, _vp, _c_i64, _vp]),
    'pcs_proj_segment': (_c_int, [_c_int, _vp, _vp, _c_i64, _c_dbl, _c_dbl, _vp]),
    'pcs_axpby': (_c_int, [_c_int, _vp, _vp, _vp, _c_i64, _c_dbl, _c_dbl, _vp]),
    'pcs_mul': (_c_int, [_c_int, _vp, _vp, _vp, _c_i64, _vp]),
    'pcs_rel_sums': (_c_int, [_c_int, _vp, _vp, _c_i64, _vp, _vp, _vp]),
    'pcs_sub2': (_c_int, [_c_int, _vp, _vp, _vp, _vp, _c_i64, _c_dbl, _c_dbl, _vp]),
    'pcs_reduce_ws_bytes': (_c_i64, []),
    'pcs_reduce': (_c_int, [_c_int, _c_int, _vp, _vp, _c_i64, _vp, _vp, _vp]),
    'pcs_apgd_step': (_c_int, [_c_int, _vp, _vp, _vp, _vp, _vp, _c_i64, _c_dbl, _c_dbl, _c_int, _c_dbl, _c_dbl,
                                _c_dbl, _vp, _vp, _vp]),
    'pcs_pds2d_halo_x': (_c_int, [_c_int]),
    'pcs_pds2d_ntaps_len': (_c_int, [_c_int]),
    'pcs_pds2d_nblocks': (_c_i64, [ctypes.POINTER(PdsArgs)]),
    'pcs_pds2d_ws_bytes': (_c_i64, [ctypes.POINTER(PdsArgs)]),
    'pcs_pds2d_step': (_c_int, [ctypes.POINTER(PdsArgs), _vp]),
    'pcs_fftconv2d_grid': (_c_i64, [_c_i64, _c_int]),
    'pcs_fftconv2d_create': (_c_int, [_c_int, _c_i64, _c_i64, _pdbl, _c_int, _c_int, _c_int, _c_int,
                                      ctypes.POINTER(_vp)]),
    'pcs_fftconv2d_apply': (_c_int, [_vp, _vp, _vp, _c_int, _vp, _c_dbl, _vp]),
    'pcs_fftconv2d_destroy': (_c_int, [_vp]),
    'pcs_pds2d_supported': (_c_int, [ctypes.POINTER(PdsArgs)]),
    'pcs_pds2d_path': (_c_int, [ctypes.POINTER(PdsArgs)]),
    'pcs_pds2d_run': (_c_int, [ctypes.POINTER(PdsArgs), _c_i64, _vp]),
    'pcs_pds2d_stencil_nblocks': (_c_i64, [ctypes.POINTER(StencilArgs)]),
    'pcs_pds2d_stencil_ws_bytes': (_c_i64, [ctypes.POINTER(StencilArgs)]),
    'pcs_pds2d_stencil_step': (_c_int, [ctypes.POINTER(StencilArgs), _vp]),
    'pcs_pds2d_stencil_run': (_c_int, [ctypes.POINTER(StencilArgs), _c_i64, _vp]),
    'pcs_pds2d_nblocks_bands': (_c_i64, [ctypes.POINTER(PdsArgs), _c_i64, _c_i64, _c_i64, _c_i64]),
    'pcs_pds2d_step_bands': (_c_int, [ctypes.POINTER(PdsArgs), _c_i64, _c_i64, _c_i64, _c_i64, _vp]),
    'pcs_comm_available': (_c_int, []),
    'pcs_comm_id_bytes': (_c_int, []),
    'pcs_comm_unique_id': (_c_int, [_vp]),
    'pcs_comm_init': (_c_int, [_vp, _c_int, _c_int, ctypes.POINTER(_vp)]),
    'pcs_comm_destroy': (_c_int, [_vp]),
    'pcs_allgather_f64': (_c_int, [_vp, _c_int, _vp, _vp, _c_i64, _vp]),
    'pcs_halo_exchange': (_c_int, [_vp, _c_int, _c_int, ctypes.POINTER(HaloSet), _vp]),
    'pcs_slab2d_create': (_c_int, [ctypes.POINTER(Slab2DDesc), _vp, ctypes.POINTER(_vp)]),
    'pcs_slab2d_overlapped': (_c_int, [_vp]),
    'pcs_slab2d_run': (_c_int, [_vp, _c_i64, _c_int, _vp]),
    'pcs_slab2d_destroy': (_c_int, [_vp]),
    'pcs_slab2d_deep_create': (_c_int, [ctypes.POINTER(SlabDeepDesc), _vp, ctypes.POINTER(_vp)]),
    'pcs_slab2d_deep_run': (_c_int, [_vp, _c_i64, _c_int, _vp]),
    'pcs_slab2d_deep_run_local': (_c_int, [ctypes.POINTER(_vp), _c_int, _c_i64, _c_int, _vp]),
    'pcs_slab2d_deep_destroy': (_c_int, [_vp]),
    'pcs_pds_reduce_finalize_k': (_c_int, [_vp, _c_int, _c_int, _vp, _vp, _vp]),
    'pcs_pds3d_nblocks': (_c_i64, [ctypes.POINTER(Pds3Args)]),
    'pcs_pds3d_ws_bytes': (_c_i64, [ctypes.POINTER(Pds3Args)]),
    'pcs_pds3d_step': (_c_int, [ctypes.POINTER(Pds3Args), _vp]),
    'pcs_pds3d_nblocks_bands': (_c_i64, [ctypes.POINTER(Pds3Args), _c_i64, _c_i64, _c_i64, _c_i64]),
    'pcs_pds3d_step_bands': (_c_int, [ctypes.POINTER(Pds3Args), _c_i64, _c_i64, _c_i64, _c_i64, _vp]),
    'pcs_ctrl_bytes': (_c_i64, []),
    'pcs_ctrl_init': (_c_int, [_vp, _c_int, _c_int, _c_dbl, _c_int, _vp]),
    'pcs_ctrl_init2': (_c_int, [_vp, _c_int, _c_int, _c_dbl, _c_int, _c_int, _vp]),
    'pcs_reduce_partials': (_c_int, [_vp, _c_i64, _vp, _vp]),
    'pcs_pds_finalize': (_c_int, [_vp, _vp, _vp, _vp]),
    'pcs_pds_reduce_finalize': (_c_int, [_vp, _c_i64, _vp, _vp, _vp]),
    'pcs_pds_finalize_pending': (_c_int, [_vp, _c_i64, _vp, _vp, _vp]),
}

EXPORTS = tuple(_SIGS)
_lib = None


class HipError(ValueError):
    """A C-ABI entry point returned a nonzero status (the reference raises ValueError
    for invalid shapes/parameters; launch failures are reported the same way)."""


# the argument-struct layout these declarations assume (pcs_abi_version(), include/pycsou_hip.h)
ABI_VERSION = 10


def load():
    """Load and declare the library (no GPU needed to load it).  A library built from other
    sources than these declarations (a stale .so) is refused: its argument structs would not match."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f'pycsou_amd: {LIB_PATH} is not built -- run `make` (or __graft_entry__.build()). '
                               'There is no CPU fallback.')
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        if lib.pcs_abi_version() != ABI_VERSION:
            raise RuntimeError(f'pycsou_amd: {LIB_PATH} has ABI {lib.pcs_abi_version()}, these bindings expect '
                               f'{ABI_VERSION} -- rebuild it with `make`')
        _lib = lib
    return _lib


def gpu():
    """Library handle for a compute call: requires a visible ROCm GPU."""
    lib = load()
    if not torch.cuda.is_available():
        raise RuntimeError('pycsou_amd: no ROCm GPU is visible; the gfx950 HIP kernels are the only compute path.')
    return lib


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def check(rc, name):
    if rc != 0:
        raise HipError(f'{name} returned status {rc}')
    return rc


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def i64s(vals):
    return (ctypes.c_int64 * len(vals))(*[int(v) for v in vals])


def dbls(vals):
    return (ctypes.c_double * len(vals))(*[float(v) for v in vals])


def dtcode(t):
    if t.dtype == torch.float32:
        return PCS_F32
    if t.dtype == torch.float64:
        return PCS_F64
    raise TypeError(f'pycsou_amd kernels support float32/float64, got {t.dtype}')

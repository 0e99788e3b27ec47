"""ctypes binding of libgp2d.so (include/gp2d.h).

The HIP engine is the only compute path: if the shared library is missing or
fails to load, every compute entry point raises ``NativeLibraryError``; there is
no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GP2D_LIB", os.path.join(_HERE, "libgp2d.so"))
ABI_VERSION = 11         # GP2D_ABI_VERSION in include/gp2d.h

FAMILY_VECTOR2D, FAMILY_ARD_RBF, FAMILY_VECTOR_ST = 0, 1, 2
KIND_SCALAR, KIND_DIVFREE, KIND_CURLFREE, KIND_MIXED = 0, 1, 2, 3
VAR_LATENT, VAR_NOISY, VAR_CLIPPED = 0, 1, 2
COMM_INT32, COMM_FLOAT64 = 2, 8
COMM_SUM, COMM_MAX, COMM_MIN = 0, 1, 2

# every symbol declared in include/gp2d.h
EXPORTS = (
    "gp2d_abi_version", "gp2d_build_info", "gp2d_padded_points", "gp2d_block_dim", "gp2d_kernel_diag",
    "gp2d_assemble", "gp2d_factor_sets", "gp2d_factor_warm", "gp2d_factor_set_of", "gp2d_factor_join", "gp2d_potrf_workspace", "gp2d_potrf", "gp2d_trtri_workspace", "gp2d_trtri",
    "gp2d_potrf_inv_workspace", "gp2d_potrf_inv", "gp2d_potrf_batched", "gp2d_trtri_batched_workspace",
    "gp2d_trtri_batched",
    "gp2d_potrs_workspace", "gp2d_potrs_inv", "gp2d_predict_workspace", "gp2d_predict",
    "gp2d_ozaki_nmod", "gp2d_ozaki_wres_bytes", "gp2d_ozaki_prepare", "gp2d_ozaki_prepare_async", "gp2d_ozaki_prepare_packed",
    "gp2d_ozaki_guard_workspace", "gp2d_ozaki_guard", "gp2d_ozaki_error_model", "gp2d_ozaki_guard_bits",
    "gp2d_predict_ozaki_workspace", "gp2d_predict_ozaki_workspace_nmod",
    "gp2d_predict_ozaki", "gp2d_ozaki_nmod_apriori", "gp2d_ozaki_kstar_bytes", "gp2d_ozaki_kstar",
    "gp2d_predict_ozaki_planes_workspace", "gp2d_predict_ozaki_planes", "gp2d_ozaki_set_skip", "gp2d_morton_codes",
    "gp2d_morton_sort_workspace", "gp2d_morton_sort", "gp2d_gather_rows", "gp2d_obs_pad", "gp2d_lml", "gp2d_lml_grad_count",
    "gp2d_lml_grad_workspace", "gp2d_lml_grad",
    "gp2d_kernel_grad_count", "gp2d_kernel_grad_workspace", "gp2d_kernel_grad",
    "gp2d_gemm", "gp2d_transpose", "gp2d_comm_id_bytes", "gp2d_comm_unique_id", "gp2d_comm_init",
    "gp2d_comm_destroy", "gp2d_comm_size", "gp2d_bcast", "gp2d_allgather", "gp2d_allreduce", "gp2d_sendrecv",
    "gp2d_stream_create_cumask", "gp2d_stream_destroy", "gp2d_status_flip",
    "gp2d_dfact_sb", "gp2d_dfact_panel_doubles", "gp2d_dfact_workspace", "gp2d_dfact_panel", "gp2d_dfact_update",
    "gp2d_dfact_invstep", "gp2d_dfact_zpart", "gp2d_dfact_zsum", "gp2d_dfact_alpha_workspace", "gp2d_dfact_alpha_blocks",
    "gp2d_assemble_cols", "gp2d_copy2d", "gp2d_zero_upper", "gp2d_pack_lower_doubles", "gp2d_pack_lower",
    "gp2d_timing_enable", "gp2d_timing_read", "gp2d_trace_mark", "gp2d_last_error",
)


class NativeLibraryError(RuntimeError):
    pass


class GP2DError(RuntimeError):
    pass


class KernelDesc(ctypes.Structure):
    _fields_ = [
        ("family", ctypes.c_int32),
        ("kind", ctypes.c_int32),
        ("l_df", ctypes.c_double),
        ("l_cf", ctypes.c_double),
        ("ratio", ctypes.c_double),
        ("dim", ctypes.c_int32),
        ("nterms", ctypes.c_int32),
        ("var", ctypes.c_double * 2),
        ("ls", (ctypes.c_double * 3) * 2),
    ]


_lib = None
_lock = threading.Lock()

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_D = ctypes.c_double
_I = ctypes.c_int
_SZ = ctypes.c_size_t
_KP = ctypes.POINTER(KernelDesc)

_SIGS = {
    "gp2d_abi_version": (_I, []),
    "gp2d_build_info": (ctypes.c_char_p, []),
    "gp2d_padded_points": (_I64, [_I64]),
    "gp2d_block_dim": (_I, [_KP]),
    "gp2d_kernel_diag": (_D, [_KP]),
    "gp2d_assemble": (_I, [_P, _I64, _I64, _P, _I64, _I64, _KP, _D, _I, _P, _I64, _P]),
    "gp2d_factor_sets": (_I, [_I]),
    "gp2d_factor_warm": (_I, [_I, _P]),
    "gp2d_factor_set_of": (_I, [_P]),
    "gp2d_factor_join": (_I, [_I]),
    "gp2d_potrf_workspace": (_SZ, [_I64]),
    "gp2d_potrf": (_I, [_P, _I64, _I64, _P, _P, _P, _SZ, _P]),
    "gp2d_trtri_workspace": (_SZ, [_I64]),
    "gp2d_trtri": (_I, [_P, _I64, _I64, _P, _P, _SZ, _P]),
    "gp2d_potrf_inv_workspace": (_SZ, [_I64]),
    "gp2d_potrf_inv": (_I, [_P, _I64, _I64, _P, _P, _P, _SZ, _P]),
    "gp2d_potrf_batched": (_I, [_P, _I64, _I64, _I64, _I, _P, _P, _P]),
    "gp2d_trtri_batched_workspace": (_SZ, [_I64, _I]),
    "gp2d_trtri_batched": (_I, [_P, _I64, _I64, _I64, _I, _P, _P, _SZ, _P]),
    "gp2d_potrs_workspace": (_SZ, [_I64]),
    "gp2d_potrs_inv": (_I, [_P, _I64, _I64, _P, _P, _P, _SZ, _P]),
    "gp2d_predict_workspace": (_SZ, [_I64, _I64, _I]),
    "gp2d_predict": (_I, [_P, _I64, _I64, _P, _P, _I64, _I64, _P, _I64, _KP, _I, _D, _I, _P, _P, _I64, _P, _SZ, _P]),
    "gp2d_ozaki_nmod": (_I, [_I64]),
    "gp2d_ozaki_wres_bytes": (_SZ, [_I64]),
    "gp2d_ozaki_prepare": (_I, [_P, _I64, _I64, _KP, _I, _I, _P, _P, ctypes.POINTER(_I), _P]),
    "gp2d_ozaki_nmod_apriori": (_I, [_I64, _KP, _D, _I, _I]),
    "gp2d_ozaki_prepare_async": (_I, [_P, _I64, _I64, _KP, _D, _I, _I, _P, _P, ctypes.POINTER(_I), _P]),
    "gp2d_ozaki_prepare_packed": (_I, [_P, _I64, _KP, _D, _I, _I, _P, _P, ctypes.POINTER(_I), _P]),
    "gp2d_ozaki_guard_workspace": (_SZ, [_I64]),
    "gp2d_ozaki_guard": (_I, [_P, _I64, _I64, _I64, _I64, _D, _P, _P, _SZ, _P]),
    "gp2d_ozaki_error_model": (_D, [_D, _D, _I, _I]),
    "gp2d_ozaki_guard_bits": (_I, [_D, _D, _D, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "gp2d_ozaki_kstar_bytes": (_SZ, [_I64, _I64, _I64, _I]),
    "gp2d_ozaki_kstar": (_I, [_P, _I64, _I64, _P, _I64, _KP, _I, _I, _I64, _P, _SZ, _P]),
    "gp2d_predict_ozaki_planes_workspace": (_SZ, [_I64, _I64]),
    "gp2d_predict_ozaki_planes": (_I, [_P, _P, _I, _I, _I64, _P, _P, _I64, _I64, _P, _I64, _KP, _I, _D, _P, _I, _I,
                                       _P, _P, _P, _I64, _P, _SZ, _P]),
    "gp2d_predict_ozaki_workspace": (_SZ, [_I64, _I64]),
    "gp2d_predict_ozaki_workspace_nmod": (_SZ, [_I64, _I64, _I]),
    "gp2d_ozaki_set_skip": (None, [_I]),
    "gp2d_morton_codes": (_I, [_P, _I64, _I, _P, _P, _P]),
    "gp2d_morton_sort_workspace": (_SZ, [_I64]),
    "gp2d_morton_sort": (_I, [_P, _I64, _I, _P, _P, _P, _SZ, _P]),
    "gp2d_gather_rows": (_I, [_P, _P, _I64, _I64, _P, _P]),
    "gp2d_obs_pad": (_I, [_P, _I64, _I64, _I, _P, _P, _P]),
    "gp2d_predict_ozaki": (_I, [_P, _P, _I, _I, _I64, _P, _P, _I64, _I64, _P, _I64, _KP, _I, _D, _I, _P, _P, _P,
                                _I64, _P, _SZ, _P]),
    "gp2d_lml": (_I, [_P, _I64, _I64, _P, _P, _I64, _P, _P]),
    "gp2d_lml_grad_count": (_I, [_KP]),
    "gp2d_lml_grad_workspace": (_SZ, [_I64]),
    "gp2d_lml_grad": (_I, [_P, _I64, _I64, _P, _P, _I64, _I64, _KP, _P, _P, _SZ, _P]),
    "gp2d_kernel_grad_count": (_I, [_KP]),
    "gp2d_kernel_grad_workspace": (_SZ, [_I64, _I64]),
    "gp2d_kernel_grad": (_I, [_P, _I64, _P, _I64, _KP, _P, _I64, _P, _P, _SZ, _P]),
    "gp2d_gemm": (_I, [_I, _I64, _I64, _I64, _D, _P, _I64, _P, _I64, _D, _P, _I64, _P]),
    "gp2d_transpose": (_I, [_P, _I64, _I64, _P, _P]),
    "gp2d_comm_id_bytes": (_SZ, []),
    "gp2d_comm_unique_id": (_I, [_P]),
    "gp2d_comm_init": (_I, [ctypes.POINTER(_P), _I, _P, _I, _I]),
    "gp2d_comm_destroy": (_I, [_P]),
    "gp2d_comm_size": (_I, [_P, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "gp2d_bcast": (_I, [_P, _SZ, _I, _P, _P]),
    "gp2d_allgather": (_I, [_P, _P, _SZ, _P, _P]),
    "gp2d_allreduce": (_I, [_P, _SZ, _I, _I, _P, _P]),
    "gp2d_sendrecv": (_I, [_P, _I, _P, _I, _SZ, _P, _P]),
    "gp2d_stream_create_cumask": (_I, [_I, _I, ctypes.POINTER(_P)]),
    "gp2d_stream_destroy": (_I, [_P]),
    "gp2d_status_flip": (_I, [_P, _I, _P]),
    "gp2d_dfact_sb": (_I, []),
    "gp2d_dfact_panel_doubles": (_SZ, [_I64]),
    "gp2d_dfact_workspace": (_SZ, [_I64]),
    "gp2d_dfact_panel": (_I, [_P, _I64, _I64, _I, _P, _P, _P, _SZ, _P]),
    "gp2d_dfact_update": (_I, [_P, _I64, _I64, _I, _P, _I, _I, _I, _I, _P]),
    "gp2d_dfact_invstep": (_I, [_P, _I64, _I64, _I, _P, _I, _I, _P, _SZ, _P]),
    "gp2d_dfact_zpart": (_I, [_P, _I64, _I64, _I, _I, _I, _P, _P, _P]),
    "gp2d_dfact_zsum": (_I, [_P, _I, _I64, _P, _P]),
    "gp2d_dfact_alpha_workspace": (_SZ, [_I64, _I]),
    "gp2d_dfact_alpha_blocks": (_I, [_P, _I64, _I64, _I, _I, _I, _P, _P, _P, _SZ, _P]),
    "gp2d_assemble_cols": (_I, [_P, _I64, _I64, _KP, _D, _P, _I64, _I64, _I64, _P]),
    "gp2d_copy2d": (_I, [_P, _I64, _P, _I64, _I64, _I64, _P]),
    "gp2d_zero_upper": (_I, [_P, _I64, _I64, _P]),
    "gp2d_pack_lower_doubles": (_SZ, [_I64]),
    "gp2d_pack_lower": (_I, [_P, _I64, _I64, _P, _I, _P]),
    "gp2d_timing_enable": (None, [_I]),
    "gp2d_trace_mark": (_I, [_I, _P]),
    "gp2d_timing_read": (_I, [ctypes.POINTER(_D), ctypes.POINTER(_I64), ctypes.POINTER(_D)]),
    "gp2d_last_error": (ctypes.c_char_p, []),
}


def lib():
    """Load libgp2d.so once; raise NativeLibraryError (never fall back) on failure."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryError(
                f"gp2d HIP engine not built: {LIB_PATH} is missing (run `python __graft_entry__.py build`)")
        try:
            L = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - depends on the ROCm install
            raise NativeLibraryError(f"cannot load {LIB_PATH}: {e}") from e
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.gp2d_abi_version() != ABI_VERSION:
            raise NativeLibraryError("libgp2d.so ABI version mismatch")
        if not L.gp2d_build_info().startswith(b"release "):   # a measurement build never ships
            raise NativeLibraryError(f"{LIB_PATH} is not a release build: {L.gp2d_build_info()!r}")
        _lib = L
        return _lib


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().gp2d_last_error().decode(errors="replace")
        raise GP2DError(f"{what} failed (rc={rc}): {msg}")


def vector_kernel_desc(kind: int, l_df: float, l_cf: float = 1.0, ratio: float = 1.0) -> KernelDesc:
    k = KernelDesc()
    k.family = FAMILY_VECTOR2D
    k.kind = int(kind)
    k.l_df = float(l_df)
    k.l_cf = float(l_cf)
    k.ratio = float(ratio)
    return k


def vector_st_kernel_desc(kind: int, l_df: float, l_cf: float, ratio: float, var_t: float, l_t: float) -> KernelDesc:
    """Spatio-temporal product Kt(var_t, l_t) × vector kernel on (T, Y, X) points."""
    k = vector_kernel_desc(kind, l_df, l_cf, ratio)
    k.family = FAMILY_VECTOR_ST
    k.dim = 3
    k.var[0] = float(var_t)
    k.ls[0][0] = float(l_t)
    return k


def ard_kernel_desc(variances, lengthscales) -> KernelDesc:
    k = KernelDesc()
    k.family = FAMILY_ARD_RBF
    k.nterms = len(variances)
    if not 1 <= k.nterms <= 2:
        raise ValueError("ARD family supports 1 or 2 RBF terms")
    dim = len(lengthscales[0])
    if not 1 <= dim <= 3:
        raise ValueError("ARD family supports 1..3 input dimensions")
    k.dim = dim
    for t in range(k.nterms):
        k.var[t] = float(variances[t])
        ls = list(lengthscales[t])
        if len(ls) != dim:
            raise ValueError("all RBF terms must have the same input dimension")
        for d in range(dim):
            k.ls[t][d] = float(ls[d])
    return k

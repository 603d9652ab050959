"""Loader for libfltee_agg.so (the HIP library behind include/fltee_agg.h).

The product path has no CPU fallback: if the library is missing the import of
any compute entry point raises.  Build it with `make -C fl-tee_amd` (or
`__graft_entry__.build()`).
"""
import ctypes
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# FLTEE_LIB: another build of the same library (A/B runs of two builds, scripts/ab_env.py)
LIB_PATH = os.environ.get("FLTEE_LIB") or os.path.join(PKG_ROOT, "lib", "libfltee_agg.so")

# include/fltee_agg.h
SUCCESS = 0x0
ERROR_UNEXPECTED = 0x1
ERROR_INVALID_PARAMETER = 0x2
ERROR_OUT_OF_MEMORY = 0x3
ERROR_INVALID_ENCLAVE_ID = 0x2002

ALG_ADVANCED, ALG_NIPS19, ALG_BASELINE, ALG_NON_OBLIVIOUS, ALG_PATH_ORAM, ALG_OPTIMIZED = 1, 2, 3, 4, 5, 6
ALG_CODES = {  # src/option.py:131-145
    "advanced": ALG_ADVANCED, "nips19": ALG_NIPS19, "baseline": ALG_BASELINE,
    "non_oblivious": ALG_NON_OBLIVIOUS, "path_oram": ALG_PATH_ORAM, "optimized": ALG_OPTIMIZED,
}

DEV_ERR_DENSE_ORDER = 0x1
DEV_ERR_INDEX_RANGE = 0x2
DEV_ERR_FOLD_OVERFLOW = 0x4  # retired in round 6: never set

OPT_DENSE = 0x1
OPT_DP = 0x2
OPT_CLIP = 0x4
OPT_ACCUMULATE = 0x8
OPT_NO_AVERAGE = 0x10
OPT_K_REQ = 0x20
OPT_ORAM_TREE = 0x40
OPT_ORAM_LAZY = 0x80


class DeviceOpts(ctypes.Structure):
    """struct fltee_device_opts."""
    _fields_ = [
        ("flags", ctypes.c_uint32),
        ("sigma", ctypes.c_float),
        ("clipping", ctypes.c_float),
        ("seed", ctypes.c_uint64),
        ("k_req", ctypes.c_size_t),
        ("batch", ctypes.c_size_t),
        ("n_avg", ctypes.c_size_t),
        ("fold_halo", ctypes.c_size_t),
        ("d_status", ctypes.c_void_p),
    ]


# every symbol declared in include/fltee_agg.h, with its ctypes signature
_P, _S, _U32, _U64, _F, _U8 = (ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                               ctypes.c_uint64, ctypes.c_float, ctypes.c_uint8)
SIGNATURES = {
    "fltee_device_init": (_U32, [ctypes.c_int, _P]),
    "fltee_device_fini": (_U32, [_U64]),
    "ecall_fl_init": (_U32, [_U64, _P, _U32, _P, _S, _S, _S, _F, _F, _F, _F, _U32, _U8, _U8]),
    "ecall_start_round": (_U32, [_U64, _P, _U32, _U32, _S, _P]),
    "ecall_secure_aggregation": (_U32, [_U64, _P, _U32, _U32, _P, _S, _P, _S, _S, _S, _U32, _P, _P]),
    "ecall_client_size_optimized_secure_aggregation":
        (_U32, [_U64, _P, _U32, _U32, _S, _P, _S, _P, _S, _S, _U32, _P, _P]),
    "fltee_aggregate_device": (_U32, [_U32, _P, _S, _S, _S, _P, ctypes.POINTER(DeviceOpts), _P]),
    "fltee_workspace_bytes": (_S, [_U32, _S, _S, _S, ctypes.POINTER(DeviceOpts)]),
    "fltee_reserve": (_U32, [_U32, _S, _S, _S, ctypes.POINTER(DeviceOpts)]),
    "fltee_decrypt_device": (_U32, [_P, _S, _P, _S, _P, _P]),
    "fltee_device_status": (_U32, [_P, _P]),
    "fltee_sum_rows_device": (_U32, [_P, _S, _S, _F, _P, _P]),
    "fltee_dp_noise_device": (_U32, [_P, _S, _F, _F, _S, _U64, _P]),
    "fltee_bitonic_device": (_U32, [_P, _S, _U32, _U32, _P]),
    "fltee_fold_device": (_U32, [_P, _P, _S, _S, _S, _P, _P]),
    "fltee_laplace_r_device": (_U32, [_S, _S, _S, _U64, _P, _P, _P]),
    "fltee_client_topk_device": (_U32, [_P, _S, _S, _S, _P, _P]),
    "fltee_client_serialize_dense_device": (_U32, [_P, _S, _S, _P, _P]),
    "fltee_client_clip_device": (_U32, [_P, _S, _S, _F, _P]),
    "fltee_encrypt_device": (_U32, [_P, _S, _P, _S, _P, _P]),
    "fltee_advanced_init_range_device": (_U32, [_P, _S, _S, _S, _S, _P, _P]),
    "fltee_bitonic_range_sort_device": (_U32, [_P, _S, _S, _U32, _U32, _P]),
    "fltee_bitonic_range_sort_padded_device": (_U32, [_P, _S, _S, _S, _U32, _U32, _P]),
    "fltee_bitonic_range_merge_device": (_U32, [_P, _S, _S, _U32, _U32, _U32, _P]),
    "fltee_bitonic_range_exchange_device": (_U32, [_P, _P, _S, _S, _S, _U32, _U32, _U32, _P]),
    "fltee_bitonic_range_steps_device": (_U32, [_P, _S, _S, _U32, _U32, _U32, _U32, _U32, _P]),
    "fltee_fold_context": (_S, [_S]),
    "fltee_fold_side_bytes": (_S, [_S, _S]),
    "fltee_fold_range_device": (_U32, [_P, _P, _S, _S, _S, ctypes.c_int64, _S, _S, _P, _P]),
    "fltee_fold_range_total_device": (_U32, [_P, _S, _S, _P, _P]),
    "fltee_fold_range_patch_device": (_U32, [_P, _S, _S, ctypes.c_int64, _S, _S, _P, _P, _S, _P]),
    "fltee_compact_range_device": (_U32, [_P, _S, _S, _P, _P, _F, _P, _P]),
    "fltee_nips19_build_range_device": (_U32, [_P, _S, _P, _S, _S, _S, _S, _P, _P]),
    "fltee_safe_aggregate_device": (_U32, [_P, _S, _S, _P, _P]),
    "fltee_select_device": (_U32, [_P, _S, _S, _P, _S, _P, _P]),
    "fltee_ordered_list_device": (_U32, [_P, _S, _S, _F, _P, _P]),
    "fltee_debug_set_seed": (None, [_U64]),
    "fltee_set_path_oram_tree": (None, [ctypes.c_int]),
    "fltee_set_advanced_exact_runs": (None, [ctypes.c_int]),
    "fltee_version": (ctypes.c_char_p, []),
    "fltee_device_init_multi": (_U32, [_P, ctypes.c_int, _P]),
    "fltee_device_count": (ctypes.c_int, [_U64]),
}
EXTRA_SIGNATURES = {  # test hooks not in the public header
    "fltee_debug_aes_block": (None, [_P, _P, _P]),
    "fltee_debug_set_dense_variant": (None, [ctypes.c_int]),
    "fltee_debug_set_oram_bucket": (None, [ctypes.c_int]),
    "fltee_debug_set_aes_variant": (None, [ctypes.c_int]),
    "fltee_debug_read_floor": (ctypes.c_int, [_P, _S, _P, ctypes.c_uint, _P]),
    "fltee_debug_network_plan": (_S, [_U32, _U32, _U32, ctypes.c_int, _P, _S]),
    "fltee_debug_pad_units": (None, [_U32] * 8 + [_P]),
    "fltee_debug_set_advanced_compaction": (None, [ctypes.c_int]),
    "fltee_debug_set_compact_variant": (None, [ctypes.c_int]),
    "fltee_debug_set_fused_init": (None, [ctypes.c_int]),
    "fltee_debug_set_nips19_fused_select": (None, [ctypes.c_int]),
    "fltee_debug_net_stats": (None, [_P, _P, ctypes.c_int]),
    "fltee_debug_net_timing": (None, [ctypes.c_int, _P]),
    "fltee_debug_session_round_keys": (ctypes.c_int, [_P, _S, _P, ctypes.c_int]),
    "fltee_debug_net_log": (_S, [_S, ctypes.c_char_p, _S, _P, _P]),
    "fltee_debug_set_fold_compact": (None, [ctypes.c_int]),
    "fltee_debug_set_pad_skip": (None, [ctypes.c_int]),
    "fltee_debug_set_radix_order": (None, [ctypes.c_int]),
    "fltee_debug_set_swizzle": (None, [ctypes.c_int]),
    "fltee_debug_sort_fused": (_U32, [_U32, _P, _S, _P, _S, _P, _S, _S,
                                       _U32, _P]),
}

_lib = None


def lib():
    """Load the HIP library (raises if it was not built: no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `make -C {PKG_ROOT}` "
                "(the aggregation path has no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        ab = bool(os.environ.get("FLTEE_LIB"))  # an A/B build of an older source may lack a hook
        for name, (res, args) in {**SIGNATURES, **EXTRA_SIGNATURES}.items():
            if ab and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib

"""ctypes binding of librifraf_hip.so (the C-ABI in include/rifraf_hip.h).

This is the only way the host reaches the hot path: there is no CPU fallback.
If the shared library is missing, cannot be loaded, or no HIP device is
present, every engine entry point raises instead of computing anything.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_int8, c_int32, c_int64, c_uint8, c_void_p

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("RIFRAF_HIP_LIB", os.path.join(PKG_DIR, "librifraf_hip.so"))

RF_FWD, RF_BWD, RF_SKEW, RF_TRIM = 1, 2, 4, 8
RF_BAND_A, RF_BAND_B = 0, 1
RF_ERR_NEED_HOST = -5
RF_ABI_VERSION = 1

# every symbol include/rifraf_hip.h declares, with its ctypes signature
_SIGNATURES = {
    "rf_abi_version": (c_int, []),
    "rf_create": (c_int, [c_int, POINTER(c_void_p)]),
    "rf_destroy": (c_int, [c_void_p]),
    "rf_last_error": (c_char_p, [c_void_p]),
    "rf_reserve": (c_int, [c_void_p, c_int64]),
    "rf_release_bands": (c_int, [c_void_p]),
    "rf_device_bytes": (c_int64, [c_void_p]),
    "rf_set_sequences_codes": (c_int, [c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_double, c_double, c_double]),
    "rf_set_sequences_codes_prep": (c_int, [c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                            c_void_p, c_double, c_double, c_double] + [c_void_p] * 5),
    "rf_code_stats": (c_int, [c_void_p, POINTER(c_int64), POINTER(c_int64), POINTER(c_int64), POINTER(c_int64)]),
    "rf_set_sequences": (c_int, [c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rf_set_templates": (c_int, [c_void_p, c_int32, c_int32, c_void_p, c_void_p]),
    "rf_set_templates_ids": (c_int, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p]),
    "rf_rifraf_batch": (c_int, [c_void_p, c_int32, c_void_p] + [c_void_p] * 14),
    "rf_batch_fetch": (c_int, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64]),
    "rf_rifraf_batch_ref": (c_int, [c_void_p, c_int32] + [c_void_p] * 21),
    "rf_batch_fetch_ref": (c_int, [c_void_p, c_int32] + [c_void_p] * 6),
    "rf_batch_release": (None, [c_void_p]),
    "rf_aln_error_sums": (c_int, [c_void_p, c_int32] + [c_void_p] * 7),
    "rf_qv_probs": (c_int, [c_void_p, c_int32] + [c_void_p] * 8),
    "rf_host_julia_sums": (c_int, [c_int64, c_void_p, c_void_p, c_void_p]),
    "rf_host_seq_sums": (c_int, [c_int64, c_void_p, c_void_p, c_void_p]),
    "rf_host_tables_from_codes": (c_int, [c_int64] + [c_void_p] * 5 + [c_double] * 3 + [c_void_p] * 6),
    "rf_host_code_seq_sums": (c_int, [c_int64] + [c_void_p] * 5),
    "rf_host_code_prep": (c_int, [c_int64] + [c_void_p] * 8),
    "rf_host_lse_finish": (c_int, [c_int64] + [c_void_p] * 4),
    "rf_host_qv_prep": (c_int, [c_int64] + [c_void_p] * 8),
    "rf_host_qv_finish": (c_int, [c_int64] + [c_void_p] * 6),
    "rf_realign": (c_int, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p]),
    "rf_realign_jobs": (c_int, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rf_backtrace": (c_int, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rf_score": (c_int, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_void_p, c_void_p]),
    "rf_alignment_proposals": (c_int, [c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_void_p]),
    "rf_score_dense": (c_int, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p]),
    "rf_score_dense_dev": (c_int, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p]),
    "rf_slot_geometry": (c_int, [c_void_p, c_int32, c_int32, POINTER(c_int32), POINTER(c_int32),
                                 POINTER(c_int32), POINTER(c_int32)]),
    "rf_download_band": (c_int, [c_void_p, c_int32, c_int32, c_void_p]),
    "rf_last_timing": (c_int, [c_void_p, POINTER(c_double), POINTER(c_double), POINTER(c_double)]),
    "rf_last_backtrace_ms": (c_int, [c_void_p, POINTER(c_double)]),
    "rf_last_codon_ms": (c_int, [c_void_p, POINTER(c_double)]),
    "rf_set_option": (c_int, [c_void_p, c_int32, c_int32]),
    "rf_get_option": (c_int, [c_void_p, c_int32, POINTER(c_int32)]),
}

# rf_set_option keys (include/rifraf_hip.h RF_OPT_*)
OPTIONS = {"score_mode": 1, "score_kernel": 2, "lean_lds_kb": 4, "dp_psplit": 10,
           "dp_np8": 11, "dp_np8_lean": 12, "dp_streams": 13, "bt_win_kb": 15, "stage_kb": 16,
           "band_pad": 17, "dp_wide": 18, "aln_sums_host": 19,
           "aln_marks_min": 22, "sync_block": 23, "dp_nl64": 24, "dp_lat": 26,
           "score_wgs": 27, "seg_wgs": 28, "dp_pfit": 29, "dp_mc": 30, "bt_nw": 31}
# symbolic values of the enum-like options
OPTION_VALUES = {"score_mode": {"auto": 0, "fused": 1, "split": 2},
                 "score_kernel": {"auto": 0, "general": 1, "seg": 2, "ws": 3}}



class BatchParams(ctypes.Structure):
    """rf_batch_params (include/rifraf_hip.h)."""
    _fields_ = [("max_iters", c_int32), ("min_dist", c_int32), ("bandwidth", c_int32),
                ("do_alignment_proposals", c_int32), ("batch_fixed", c_int32), ("batch_size", c_int32),
                ("batch_threshold", c_double), ("batch_randomness", c_double), ("batch_mult", c_double),
                ("est_n_errors", c_void_p), ("seed", c_void_p)]


class BatchRefParams(ctypes.Structure):
    """rf_batch_ref_params (include/rifraf_hip.h)."""
    _fields_ = [("do_frame", c_int32), ("do_refine", c_int32), ("seed_indels", c_int32),
                ("indel_correction_only", c_int32), ("max_ref_indel_mults", c_int32), ("pad", c_int32),
                ("ref_error_mult", c_double)]


class BatchRef(ctypes.Structure):
    """rf_batch_ref (include/rifraf_hip.h): one cluster's reference record."""
    _fields_ = [("ref_seq", c_int32), ("edit_seq", c_int32), ("ref_slot", c_int32), ("scratch_slot", c_int32),
                ("ref_off", c_int64), ("ref_len", c_int64)]


# rf_ref_callback: (user, cluster, event, value, thr*) -> 0 / nonzero
RefCallback = ctypes.CFUNCTYPE(c_int, c_void_p, c_int32, c_int32, c_double, POINTER(c_double))


_lib = None
_load_error = None


class EngineUnavailable(RuntimeError):
    """The HIP engine cannot run here (library missing or no GPU)."""


def load(path: str | None = None):
    """Load librifraf_hip.so and bind every C-ABI symbol (raises if absent)."""
    global _lib, _load_error
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise EngineUnavailable(
            f"{p} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    try:
        lib = ctypes.CDLL(p)
    except OSError as e:  # pragma: no cover - environment dependent
        _load_error = e
        raise EngineUnavailable(f"cannot load {p}: {e}") from e
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError = missing export: loud
        fn.restype = res
        fn.argtypes = args
    if lib.rf_abi_version() != RF_ABI_VERSION:
        raise EngineUnavailable("librifraf_hip.so ABI version mismatch")
    if path is None:
        _lib = lib
    return lib


def ptr(a: np.ndarray | None):
    """Pointer to a contiguous numpy array (None -> NULL)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return a.ctypes.data_as(c_void_p)


__all__ = ["load", "ptr", "EngineUnavailable", "RF_FWD", "RF_BWD", "RF_SKEW", "RF_TRIM",
           "RF_BAND_A", "RF_BAND_B", "RF_ERR_NEED_HOST", "_SIGNATURES", "c_int8", "c_uint8"]

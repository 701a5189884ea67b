"""ctypes binding of libsglm_hip.so (C ABI: include/sglm_hip.h).

There is no fallback: if the shared library is missing or no ROCm GPU is visible, every
entry point raises ``HipEngineUnavailable``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# SGLM_LIB: another build of the same library (kernel-variant A/B runs)
LIB_PATH = os.environ.get("SGLM_LIB") or os.path.join(_HERE, "libsglm_hip.so")

_i32, _i64, _u64, _f32, _vp, _sz = C.c_int32, C.c_int64, C.c_uint64, C.c_float, C.c_void_p, C.c_size_t

# name -> (restype, argtypes); kept in the order of include/sglm_hip.h
SIGNATURES = {
    "sglm_last_error": (C.c_char_p, []),
    "sglm_version": (C.c_int, []),
    "sglm_timeshift_expand": (C.c_int, [_vp, _i64, _i64, _i64, _vp, _vp, _i32, _vp, _i64, _i64,
                                        _i64, _i64, _i32, _u64, _vp]),
    "sglm_timeshift_gather": (C.c_int, [_vp, _i64, _i64, _i64, _vp, _vp, _i32, _vp, _i64, _i64,
                                        _i64, _vp, _i32, _u64, _vp]),
    "sglm_pack_design": (C.c_int, [_vp, _i32, _i64, _i32, _i64, _i64, _i32, _vp, _vp, _i64,
                                   _i32, _vp, _vp]),
    "sglm_pack_design_rows": (C.c_int, [_vp, _i32, _i64, _i32, _i64, _i64, _i32, _vp, _vp, _i64,
                                        _i32, _i64, _vp, _vp]),
    "sglm_pack_design_rows_cf": (C.c_int, [_vp, _i32, _i64, _i32, _i64, _i64, _i32, _vp, _vp,
                                           _i64, _i32, _i64, _vp, _vp, _vp]),
    "sglm_gemv_eta": (C.c_int, [_vp, _i32, _i64, _i32, _i64, _vp, _i32, _vp, _vp]),
    "sglm_link_update": (C.c_int, [_i32, _f32, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp,
                                   _vp, _vp, _vp, _vp, _vp, _vp]),
    "sglm_link_update_rp": (C.c_int, [_i32, _f32, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp,
                                      _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp]),
    "sglm_xtr_work_bytes": (_sz, [_i32, _i32, _i64]),
    "sglm_xtr": (C.c_int, [_vp, _i32, _i64, _i32, _i64, _vp, _i32, _vp, _vp, _vp]),
    "sglm_syrk_work_bytes": (_sz, [_i32, _i32, _i32]),
    "sglm_syrk": (C.c_int, [_vp, _i64, _i32, _i64, _vp, _vp, _i32, _i32, _vp, _vp, _vp]),
    "sglm_syrk_masked": (C.c_int, [_vp, _i64, _i32, _i64, _vp, _vp, _i32, _i32, _vp, _vp, _vp, _vp,
                                   _vp, _vp]),
    "sglm_pack_bits": (C.c_int, [_vp, _i64, _i32, _vp, _vp, _vp]),
    "sglm_pack_bits_rows": (C.c_int, [_vp, _i64, _i32, _vp, _i64, _vp, _vp, _vp]),
    "sglm_compact_rbits": (C.c_int, [_vp, _i64, _i32, _vp, _i64, _vp, _vp]),
    "sglm_compact_bits": (C.c_int, [_vp, _i64, _i32, _vp, _i64, _vp, _vp]),
    "sglm_gather_w": (C.c_int, [_vp, _i64, _vp, _i32, _vp, _i64, _vp]),
    "sglm_syrk_cbits": (C.c_int, [_vp, _i32, _vp, _i32, _i32, _vp, _vp, _vp]),
    "sglm_lag_gram_w": (C.c_int, [_vp, _vp, _vp, _i32, _i32, _vp, _vp, _i32, _i32, _i32,
                                  _i32, _i32, _i32, _vp, _i64, _vp, _i32, _vp, _i32, _i32,
                                  _vp, _vp]),
    "sglm_lag_rowwords": (C.c_int, [_vp, _i32, _i32, _i32, _vp, _vp]),
    "sglm_pack_bits_t": (C.c_int, [_vp, _i64, _i32, _vp, _vp, _vp]),
    "sglm_eta_bits_work_bytes": (_sz, [_i32, _i32]),
    "sglm_gemv_eta_bits": (C.c_int, [_vp, _i64, _i32, _vp, _i32, _vp, _i32, _vp, _vp, _vp]),
    "sglm_xtr_bits_work_bytes": (_sz, [_i32, _i32, _i64]),
    "sglm_xtr_bits": (C.c_int, [_vp, _i64, _i32, _i64, _vp, _i32, _vp, _vp, _vp]),
    "sglm_xtr_bits_packed_work_bytes": (_sz, [_i32, _i32, _i64]),
    "sglm_xtr_bits_packed": (C.c_int, [_vp, _i64, _i32, _i64, _vp, _i32, _vp, _vp, _vp, _vp]),
    "sglm_xtr_bits_packed_bp": (C.c_int, [_vp, _i64, _i32, _i64, _vp, _i32, _i32, _vp, _vp, _vp,
                                          _vp]),
    "sglm_xtr_bits_int_work_bytes": (_sz, [_i32, _i32, _i64]),
    "sglm_xtr_bits_int": (C.c_int, [_vp, _i64, _i32, _i64, _vp, _i32, _vp, _vp, _vp]),
    "sglm_event_bits": (C.c_int, [_vp, _i64, _i32, _i64, _vp, _i64, _vp]),
    "sglm_lag_bits": (C.c_int, [_vp, _i64, _vp, _vp, _i32, _i64, _i64, _i64, _i32, _vp, _vp, _vp]),
    "sglm_digit_planes": (C.c_int, [_vp, _i64, _vp, _i64, _i64, _vp, _vp, _vp, _i32, _i32, _vp, _i64, _vp]),
    "sglm_center_gram": (C.c_int, [_vp, _i32, _i32, _vp, _i32, _i32, _vp, _vp]),
    "sglm_enet_cd_shared": (C.c_int, [_vp, _i32, _vp, _i32, _vp, _vp, _vp, _i32, C.c_double,
                                      _vp, _vp, _vp]),
    "sglm_enet_cd_fits_per_wg": (_i32, [_i32]),
    "sglm_enet_cd_grouped": (C.c_int, [_vp, _i32, _vp, _i32, _i32, _vp, _vp, _vp, _vp, _i32,
                                       C.c_double, _vp, _vp, _vp]),
    "sglm_gram_ss_work_bytes": (_sz, [_i32, _i32]),
    "sglm_gram_ss": (C.c_int, [_vp, _i32, _i32, _vp, _vp, _i32, _i32, _vp, _i32, _vp, _vp, _vp,
                               _vp, _vp, _vp, _vp]),
    "sglm_syrk_f32": (C.c_int, [_vp, _i64, _i32, _i64, _vp, _vp, _i32, _i32, _vp, _vp, _vp]),
    "sglm_chol_work_bytes": (_sz, [_i32, _i32]),
    "sglm_chol_solve_ex": (C.c_int, [_vp, _i32, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _i32, _i32,
                                     _vp, _vp]),
    "sglm_chol_solve_inv": (C.c_int, [_vp, _vp, _i32, _vp, _vp, _vp, _i32, _i32, _vp, _i32,
                                      _vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp]),
    "sglm_chol_solve_mixed": (C.c_int, [_vp, _i32, _vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _i32,
                                        _vp, _vp]),
    "sglm_chol_factor": (C.c_int, [_vp, _vp, _i32, _vp, _i32, _vp, _vp, _vp, _i32, _vp, _vp]),
    "sglm_chol_invert": (C.c_int, [_vp, _vp, _i32, _vp, _i32, _i32, _vp, _vp]),
    "sglm_chol_graph_cache_size": (_i32, []),
    "sglm_chol_graph_cache_clear": (C.c_int, []),
    "sglm_chol_solve_alias": (C.c_int, [_vp, _i32, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _i32, _vp,
                                        _vp]),
    "sglm_chol64_work_bytes": (_sz, [_i32, _i32]),
    "sglm_chol64_factor": (C.c_int, [_vp, _i32, _vp, _vp, _vp, _vp, _i32, C.c_double, _vp, _vp,
                                     _vp, _vp, _vp, _vp]),
    "sglm_chol64_factor_mixed": (C.c_int, [_vp, _i32, _vp, _vp, _vp, _vp, _i32, C.c_double, _vp,
                                           _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "sglm_chol64_solve": (C.c_int, [_vp, _i32, _vp, _vp, _vp, _i32, _vp, _vp, _vp]),
    "sglm_chol64_solve_add": (C.c_int, [_vp, _i32, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp]),
    "sglm_chol64_resid": (C.c_int, [_vp, _i32, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _i32, _vp,
                                    _vp, _vp, _vp, _vp, _vp]),
    "sglm_chol64_minnorm_work_bytes": (_sz, [_i32, _i32]),
    "sglm_chol64_minnorm": (C.c_int, [_vp, _i32, _i32, _vp, _vp, _vp, _i32, _vp, _vp, _i32, _vp,
                                      _vp, _vp]),
    "sglm_step_scalars": (C.c_int, [_i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp]),
    "sglm_step_update": (C.c_int, [_i32, _i32, _vp, _vp, _vp, _vp, _vp]),
    "sglm_aa_step": (C.c_int, [_i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "sglm_step_decide": (C.c_int, [_i32, _vp, _vp, _vp, _i32, _vp, C.c_double, C.c_double,
                                   C.c_double, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                   _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "sglm_mask_stats_work_bytes": (_sz, [_i32, _i32, _i64]),
    "sglm_mask_stats": (C.c_int, [_vp, _i64, _i32, _vp, _i32, _i64, _vp, C.c_double, _vp, _vp,
                                  _vp]),
    "sglm_rowsum_work_bytes": (_sz, [_i32, _i32, _i64]),
    "sglm_loss_trials": (C.c_int, [_i32, _f32, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp,
                                   _vp, _vp, _i32, _vp, _vp, _vp]),
    "sglm_loss_trials_max": (C.c_int, [_i32, _f32, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _vp,
                                       _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp]),
    "sglm_eta_axpy": (C.c_int, [_i64, _i64, _i32, _vp, _vp, _vp, _vp, _vp]),
    "sglm_eta_axpy_max": (C.c_int, [_i64, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "sglm_eta_pair_absmax": (C.c_int, [_i64, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "sglm_score_sums": (C.c_int, [_i32, _f32, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp,
                                  _vp, _vp]),
    "sglm_lag_tile_rows": (_i32, []),
    "sglm_lag_xtr_work_bytes": (_sz, [_i32, _i32, _i32, _i64]),
    "sglm_lag_gram_work_bytes": (_sz, [_i32, _i32, _i32]),
    "sglm_lag_gram_w_work_bytes": (_sz, [_i32, _i32, _i32, _i32]),
    "sglm_lag_gram_w_timing": (C.c_int, [_i32, _vp, _vp]),
    "sglm_xtr_prefer": (C.c_int, [_i32]),
    "sglm_lag_gram": (C.c_int, [_vp, _vp, _vp, _i64, _vp, _i32, _i32, _i32, _i32, _i32, _i64,
                                _i64, _i64, _i32, _vp, _i64, _vp, _i32, _vp, _vp, _vp]),
    "sglm_lag_gram_pc": (C.c_int, [_vp, _vp, _vp, _i64, _vp, _i32, _i32, _i32, _i32, _i32, _i64,
                                   _i64, _i64, _i32, _i32, _vp, _i64, _vp, _i32, _vp, _vp, _vp]),
    "sglm_mixed_work_bytes": (_sz, [_i32, _i32, _i64]),
    "sglm_mixed_wc": (C.c_int, [_vp, _i64, _vp, _i32, _vp, _i64, _i32, _i64, _i64, _vp, _vp]),
    "sglm_mixed_gram": (C.c_int, [_i32, _vp, _i64, _vp, _i32, _vp, _i64, _i32, _i64, _vp, _i32,
                                  _vp, _vp, _vp, _vp]),
    "sglm_mixed_xtr": (C.c_int, [_i32, _vp, _i64, _i64, _vp, _vp, _i32, _vp, _i64, _i32, _i64,
                                 _vp, _i32, _vp, _vp, _vp, _vp]),
    "sglm_mixed_eta": (C.c_int, [_vp, _i64, _i32, _i64, _vp, _vp, _i32, _vp, _i32, _vp, _i64,
                                 _vp]),
    "sglm_mixed_to_h": (C.c_int, [_vp, _i32, _i32, _i32, _vp, _vp, _vp, _vp]),
    "sglm_lag_xtr": (C.c_int, [_vp, _vp, _vp, _vp, _i32, _i32, _i32, _i64, _i64, _i32, _vp, _i64,
                               _vp, _i32, _vp, _vp, _vp]),
    "sglm_group_rows_work_bytes": (_sz, [_i64]),
    "sglm_group_rows": (C.c_int, [_vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "sglm_trial_lookup": (C.c_int, [_vp, _i64, _vp, _i64, _vp, _vp]),
    "sglm_dm_heatmap": (C.c_int, [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _i64,
                                  _vp]),
    "sglm_dm_licks": (C.c_int, [_vp, _i32, _vp, _i32, _i64, _vp, _vp, _vp]),
    "sglm_dm_counters": (C.c_int, [_vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                   _vp, _vp]),
    "sglm_dm_pull": (C.c_int, [_vp, _i64, _vp, _vp, _vp, _vp, _i32, _vp, _vp]),
    "sglm_dm_heatmap_k": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp,
                                    _i64, _vp]),
    "sglm_dm_counters_k": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp,
                                     _vp, _vp, _vp, _vp]),
    "sglm_dm_pull_k": (C.c_int, [_vp, _vp, _i64, _vp, _vp, _vp, _vp, _i32, _vp, _vp]),
    "sglm_trial_map": (C.c_int, [_i64, _vp, _vp, _i64, _vp, _vp, _i64, _vp, _i32, _vp, _i64, _vp,
                                 _vp]),
    "sglm_trial_map_u8": (C.c_int, [_i64, _vp, _vp, _i64, _vp, _vp, _i64, _vp, _i32, _vp, _i64,
                                    _vp, _vp]),
    "sglm_zero_groups_flag": (C.c_int, [_i64, _vp, _vp, _vp, _vp, _i64, _vp, _i32, _vp, _vp,
                                        _vp]),
    "sglm_host_masks": (C.c_int, [_i32, _vp, _vp, _vp, _i64, _i64, _vp, _vp, _vp, _i32]),
    "sglm_host_copy": (C.c_int, [_vp, _vp, _i64, _i32]),
    "sglm_host_gather_cols": (C.c_int, [_vp, _vp, _i32, _i64, _i32, _vp, _i32]),
    "sglm_host_pack_bits_cols": (C.c_int, [_vp, _vp, _i32, _i64, _vp, _vp, _vp, _i32]),
    "sglm_host_group_rows": (C.c_int, [_vp, _i64, _vp, _i32, _i64, _vp, _vp, _i32]),
    "sglm_host_group_runs": (C.c_int, [_vp, _vp, _vp, _i64, _vp, _i32, _i64, _vp, _vp, _i32]),
    "sglm_scatter_rows": (C.c_int, [_i64, _vp, _i64, _vp, _i32, _vp, _i64, _vp]),
    "sglm_signal_trials_work_bytes": (_sz, [_i64]),
    "sglm_signal_trials": (C.c_int, [_vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp,
                                     _vp, _vp]),
    "sglm_prep_work_bytes": (_sz, [_i64]),
    "sglm_prep_session": (C.c_int, [_vp, _i64, _i64, _i32, _vp, _i64, _vp, _vp]),
}


class HipEngineUnavailable(RuntimeError):
    """The MI355X engine cannot run here (library not built, or no GPU)."""


class HipEngineError(RuntimeError):
    """A libsglm_hip call returned an error status."""


_lock = threading.Lock()
_lib = None


def load(path: str = LIB_PATH):
    """Load the shared library and attach signatures (no GPU needed)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(path):
                raise HipEngineUnavailable(
                    f"{path} not found: build it with `python -c 'import __graft_entry__ as g; "
                    f"g.build()'` (hipcc --offload-arch=gfx950). There is no CPU fallback.")
            lib = C.CDLL(path)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def call(name: str, *args):
    """Invoke an int-returning entry point and raise on a non-zero status."""
    lib = load()
    st = getattr(lib, name)(*args)
    if st != 0:
        msg = lib.sglm_last_error().decode(errors="replace")
        raise HipEngineError(f"{name} failed with status {st}: {msg}")
    return st


def query(name: str, *args) -> int:
    return int(getattr(load(), name)(*args))

"""ctypes binding of ``libalignn_hip.so`` (the C ABI declared in ``include/alignn_hip.h``).

The library is built in-tree (``csrc/Makefile`` -> ``alignn_mi355x/libalignn_hip.so``).  There is no
CPU or PyTorch fallback: if the library is missing or cannot be loaded, :func:`lib` raises.
``torch`` is imported first so that the HIP runtime torch ships (SONAME ``libamdhip64.so.7``) is
the one the library binds to — one runtime, one device context, shared streams.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must load torch's HIP runtime before the library)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ALIGNN_HIP_LIB") or os.path.join(_HERE, "libalignn_hip.so")  # override: kernel A/B runs

c_i64 = ctypes.c_int64
c_i32 = ctypes.c_int32
c_u64 = ctypes.c_uint64
c_f32 = ctypes.c_float
c_f64 = ctypes.c_double
c_vp = ctypes.c_void_p


class GemmArgs(ctypes.Structure):
    _fields_ = [
        ("M", c_i64), ("N", c_i64), ("K", c_i64), ("batch", c_i64),
        ("A", c_vp), ("sam", c_i64), ("sak", c_i64), ("sab", c_i64),
        ("B", c_vp), ("sbk", c_i64), ("sbn", c_i64), ("sbb", c_i64),
        ("C", c_vp), ("scm", c_i64), ("scn", c_i64), ("scb", c_i64),
        ("bias", c_vp), ("sbias_b", c_i64),
        ("rowscale", c_vp), ("srs_m", c_i64), ("srs_b", c_i64),
        ("bias2", c_vp), ("sb2_b", c_i64),
        ("mask", c_vp), ("smk_m", c_i64), ("smk_n", c_i64),
        ("alpha", c_f32), ("beta", c_f32),
        ("relu", c_i32), ("split_k", c_i32),
        ("workspace", c_vp), ("workspace_elems", c_i64),
        ("reduce_batch", c_i32), ("tile", c_i32),
        ("c_rows", c_vp),
        ("rowsum", c_vp),
    ]


class Schedule(ctypes.Structure):
    _fields_ = [("light", c_vp), ("n_light", c_i64), ("heavy", c_vp), ("n_heavy", c_i64),
                ("flags", c_i32), ("reserved", c_i32)]


SCHED_WAVE_ITEMS = 2


ENCBWD_MAX_LAYERS = 8


class EncBwdArgs(ctypes.Structure):
    _fields_ = [("n", c_i64), ("T", c_i64), ("D", c_i32), ("H", c_i32), ("L", c_i32), ("kin", c_i32),
                ("dst_at", c_vp), ("off_dst", c_vp), ("x", c_vp), ("ldx", c_i64), ("w1", c_vp), ("b1", c_vp),
                ("U", c_vp * ENCBWD_MAX_LAYERS), ("Vd", c_vp * ENCBWD_MAX_LAYERS),
                ("dz", c_vp * ENCBWD_MAX_LAYERS), ("alpha", c_vp * ENCBWD_MAX_LAYERS),
                ("dW1", c_vp), ("db1", c_vp), ("accumulate", c_i32),
                ("workspace", c_vp), ("workspace_elems", c_i64)]


_SIGNATURES = {
    "alignn_version": ([], c_i32),
    "alignn_last_error": ([], ctypes.c_char_p),
    "alignn_set_step_seed": ([c_vp], None),
    "alignn_gemm_f32": ([ctypes.POINTER(GemmArgs), c_vp], c_i32),
    "alignn_gemm_workspace": ([ctypes.POINTER(GemmArgs)], c_i64),
    "alignn_copy_many": ([c_i32, c_vp, c_vp, c_vp, c_vp], c_i32),
    "alignn_gemm_path": ([ctypes.POINTER(GemmArgs)], c_i32),
    "alignn_colsum_f32": ([c_vp, c_i64, c_i64, c_i64, c_vp, c_i32, c_vp, c_vp], c_i32),
    "alignn_wcolsum2_f32": ([c_i64, c_i64, c_i32, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i32, c_vp,
                             c_vp], c_i32),
    "alignn_graph_prep": ([c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp], c_i32),
    "alignn_schedule_build": ([c_vp, c_i64, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp], c_i32),
    "alignn_gather_rows_f32": ([c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp], c_i32),
    "alignn_scatter_rows_f32": ([c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i32, c_vp], c_i32),
    "alignn_tconv_fwd": ([c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64,
                          c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_u64, c_vp], c_i32),
    "alignn_tconv_family": ([c_i32, c_i32, c_vp, c_vp, c_vp], c_i32),
    "alignn_tconv_bwd_src_by_bf16": ([c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp,
                                      c_vp, c_i64, c_vp], c_i32),
    "alignn_tconv_fwd_ex": ([c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp,
                             c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_u64, c_vp], c_i32),
    "alignn_tconv_bwd_dst_ex": ([c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp,
                                 c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                                 c_vp, c_i64, c_i32, c_f32, c_u64, c_vp], c_i32),
    "alignn_lg_fwd_bf16": ([c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp,
                            c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_u64, c_vp], c_i32),
    "alignn_lg_bwd_dst_bf16": ([c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp,
                                c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_f32,
                                c_u64, c_vp], c_i32),
    "alignn_lg_fwd_x": ([c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp,
                         c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_u64, c_vp], c_i32),
    "alignn_lg_bwd_dst_x": ([c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp,
                             c_vp, c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp,
                             c_vp, c_vp, c_f32, c_u64, c_vp], c_i32),
    "alignn_cast_bf16_f32": ([c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp], c_i32),
    "alignn_linear_smallk_bf16out": ([c_vp, c_i64, c_i64, c_i32, c_vp, c_i64, c_vp, c_i64, c_i32, c_vp, c_i64, c_vp],
                                     c_i32),
    "alignn_tconv_bwd_dst": ([c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                              c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64,
                              c_i32, c_f32, c_u64, c_vp], c_i32),
    "alignn_tconv_bwd_src": ([c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                              c_i64, c_vp], c_i32),
    "alignn_tconv_bwd_src_by": ([c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                                 c_i64, c_vp], c_i32),
    "alignn_gate_ln_fwd": ([c_i64, c_i32, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp,
                            c_vp, c_vp, c_f32, c_u64, c_vp], c_i32),
    "alignn_gate_ln_bwd": ([c_i64, c_i32, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                            c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_f32, c_u64, c_vp], c_i32),
    "alignn_gate_ln_fwd_rows": ([c_i64, c_i32, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64,
                                 c_vp, c_vp, c_vp, c_f32, c_u64, c_vp], c_i32),
    "alignn_gate_ln_bwd_rows": ([c_i64, c_i32, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                 c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_f32, c_u64, c_vp], c_i32),
    "alignn_gate_ln_bwd_partials": ([c_i64, c_i32, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                                     c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_f32, c_u64, c_vp], c_i32),
    "alignn_gate_ln_bwd_partials_add": ([c_i64, c_i32, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp,
                                         c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_f32, c_u64, c_vp], c_i32),
    "alignn_gate_ln_bwd_reduce": ([c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp], c_i32),
    "alignn_readout_feats_fwd": ([c_i64, c_i32, c_vp, c_vp, c_vp, c_i32, c_vp, c_i32, c_vp, c_f32, c_u64, c_vp],
                                 c_i32),
    "alignn_readout_pool_bwd": ([c_i64, c_i64, c_i32, c_vp, c_i64, c_vp, c_vp, c_vp, c_i32, c_f32, c_u64, c_vp],
                                c_i32),
    "alignn_dropout_f32": ([c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_f32, c_u64, c_vp], c_i32),
    "alignn_hetero_nll": ([c_i64, c_i32, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_f32, c_f32, c_vp, c_vp, c_i64, c_vp],
                          c_i32),
    "alignn_hetero_nll_amp": ([c_i64, c_i32, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_f32, c_f32, c_vp, c_vp, c_i64,
                               c_vp], c_i32),
    "alignn_add_noise_f32": ([c_i64, c_vp, c_f32, c_u64, c_vp], c_i32),
    "alignn_noisy_copy2_f32": ([c_i64, c_vp, c_vp, c_u64, c_i64, c_vp, c_vp, c_u64, c_f32, c_vp], c_i32),
    "alignn_ensemble_moments": ([c_i32, c_i64, c_i32, c_vp, c_i64, c_i64, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                 c_vp, c_vp, c_vp], c_i32),
    "alignn_member_mean_f32": ([c_i32, c_i64, c_vp, c_i64, c_vp, c_vp], c_i32),
    "alignn_grad_norm_f32": ([c_vp, c_i64, c_vp, c_vp, c_vp], c_i32),
    "alignn_collate_rows_f32": ([c_i32, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp], c_i32),
    "alignn_collate_index_i64": ([c_i32, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp], c_i32),
    "alignn_collate_batchvec": ([c_i32, c_vp, c_vp, c_i64, c_vp, c_vp], c_i32),
    "alignn_collate_rows_std_f32": ([c_i32, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp, c_i32,
                                     c_vp], c_i32),
    "alignn_ghost_edges_i64": ([c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp], c_i32),
    "alignn_segment_finite_f32": ([c_i32, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp], c_i32),
    "alignn_feature_stats_workspace": ([c_i32, c_i64], c_i64),
    "alignn_feature_stats_f64": ([c_i32, c_vp, c_i64, c_vp, c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_i64, c_vp], c_i32),
    "alignn_col_center_sq_f32": ([c_vp, c_i64, c_i32, c_vp, c_vp, c_vp], c_i32),
    "alignn_standardize_f32": ([c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp], c_i32),
    "alignn_row_sqnorm_f32": ([c_vp, c_i64, c_i32, c_vp, c_vp], c_i32),
    "alignn_knn_select_weights": ([c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, c_i32, c_vp, c_i32, c_f32, c_f32, c_f32,
                                   c_vp, c_vp, c_vp], c_i32),
    "alignn_linear_smallk_f32": ([c_vp, c_i64, c_i64, c_i32, c_vp, c_i64, c_vp, c_i64, c_i32, c_vp, c_i64, c_vp],
                                 c_i32),
    "alignn_gemm_tn_smalln_workspace": ([c_i64, c_i64, c_i32], c_i64),
    "alignn_gemm_tn_smalln_f32": ([c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_i32, c_vp, c_i64, c_vp, c_i32, c_vp,
                                   c_i64, c_vp], c_i32),
    "alignn_enc_bwd_workspace": ([c_i32, c_i32], c_i64),
    "alignn_enc_bwd_f32": ([ctypes.POINTER(EncBwdArgs), c_vp], c_i32),
    "alignn_enc_bwd_bf16": ([ctypes.POINTER(EncBwdArgs), c_vp, c_i64, c_vp], c_i32),
    "alignn_gate_ln_bwd_workspace": ([c_i64, c_i32], c_i64),
    "alignn_plan_begin": ([c_vp], c_i32),
    "alignn_plan_note_wait": ([c_vp, c_vp], c_i32),
    "alignn_plan_end": ([], c_vp),
    "alignn_plan_abort": ([], c_i32),
    "alignn_plan_replay": ([c_vp, c_vp], c_i32),
    "alignn_plan_replay_serial": ([c_vp, c_vp], c_i32),
    "alignn_plan_info": ([c_vp, c_vp, c_vp, c_vp, c_vp], c_i32),
    "alignn_plan_entries": ([c_vp, c_vp, c_vp, c_i64], c_i64),
    "alignn_plan_destroy": ([c_vp], c_i32),
    "alignn_plan_note_timestamp": ([c_vp], c_i32),
    "alignn_plan_elapsed_ms": ([c_vp, c_i32, c_i32, c_vp], c_i32),
    "alignn_plan_check_ptrs": ([c_vp, c_vp, c_i64, c_vp, c_vp, c_vp], c_i32),
    "alignn_plan_refs": ([c_vp, c_vp, c_i64, c_vp], c_i32),
    "alignn_graph_census": ([c_vp, c_vp, c_vp], c_i32),
    "alignn_plan_check_deps": ([c_vp, c_vp, c_vp, c_vp, c_vp], c_i32),
    "alignn_stream_create": ([c_i32, ctypes.POINTER(c_vp)], c_i32),
    "alignn_stream_create_dedicated": ([ctypes.POINTER(c_vp)], c_i32),
    "alignn_stream_destroy": ([c_vp], c_i32),
    "alignn_fill_f32": ([c_vp, c_i64, c_f32, c_vp], c_i32),
    "alignn_add_f32": ([c_vp, c_vp, c_i64, c_vp], c_i32),
    "alignn_set_i64": ([c_vp, c_i64, c_vp], c_i32),
    "alignn_copy_f32": ([c_vp, c_vp, c_i64, c_vp], c_i32),
    "alignn_adamw_f32": ([c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_f64, c_f64, c_f64, c_f64, c_f64, c_f64, c_vp, c_f32,
                          c_vp, c_vp], c_i32),
    "alignn_adamw_f32_dev": ([c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_f64, c_f64, c_f64, c_f64, c_vp, c_f32,
                              c_vp, c_vp], c_i32),
    "alignn_colsum_bf16": ([c_vp, c_i64, c_i64, c_i64, c_vp, c_i32, c_vp, c_vp], c_i32),
    "alignn_gate_ln_fwd_ex": ([c_i64, c_i32, c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64,
                               c_vp, c_i64, c_vp, c_vp, c_vp, c_f32, c_u64, c_vp], c_i32),
    "alignn_gate_ln_fwd_ex2": ([c_i64, c_i32, c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64,
                                c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_f32, c_u64, c_vp], c_i32),
    "alignn_gate_ln_bwd_partials_ex": ([c_i64, c_i32, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_vp, c_vp,
                                        c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_f32, c_u64, c_vp], c_i32),
    "alignn_grad_norm_amp_f32": ([c_vp, c_i64, c_vp, c_vp, c_vp, c_vp], c_i32),
    "alignn_adamw_amp_f32_dev": ([c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_f64, c_f64, c_f64, c_f64, c_vp, c_f32,
                                  c_vp, c_vp, c_i32, c_vp], c_i32),
}

EXPORTED = tuple(_SIGNATURES.keys())

_lib = None
_lock = threading.Lock()


class AlignnHipError(RuntimeError):
    pass


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load the library and declare every signature (no GPU work happens here)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise AlignnHipError(
                f"libalignn_hip.so not found at {path}: build it with `make -C "
                f"gnn-elasticity-predictor_amd/csrc` or __graft_entry__.build() (there is no CPU fallback)")
        lib_ = ctypes.CDLL(path)
        for name, (argtypes, restype) in _SIGNATURES.items():
            fn = getattr(lib_, name)
            fn.argtypes = argtypes
            fn.restype = restype
        _lib = lib_
        return _lib


def lib() -> ctypes.CDLL:
    return _lib if _lib is not None else load()


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().alignn_last_error()
        msg = msg.decode() if msg else ""
        raise AlignnHipError(f"{what} failed (code {rc}): {msg}")

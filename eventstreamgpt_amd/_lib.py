"""ctypes binding of the C ABI in ``include/esgpt_amd.h`` (libesgpt_amd.so, built in-tree for gfx950).

This is the exact binding a maintainer would add on the reference side. The library is
loaded after ``torch`` so that it shares torch's HIP runtime (both link ``libamdhip64.so.7``; the dynamic loader
reuses the already-loaded copy), which makes torch's streams and allocations valid handles for the kernels.

There is NO fallback: if the library is missing or no gfx950 device is visible, every product op raises.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ESGPT_AMD_LIB", os.path.join(_HERE, "libesgpt_amd.so"))

ESGPT_OK, ESGPT_ERR_INVALID_ARG, ESGPT_ERR_LAUNCH, ESGPT_ERR_UNSUPPORTED = 0, 1, 2, 3
F32, BF16 = 0, 1
FLAG_BAD_INDEX, FLAG_TTE_NAN, FLAG_TTE_NO_OBS, FLAG_BAD_LABEL, FLAG_PEER_RANK = 1, 2, 4, 8, 16
EMB_NORMALIZE, EMB_STATIC, EMB_TIME, EMB_CUMSUM, EMB_TIME_ABS = 1, 2, 4, 8, 16
BAG_JOINT, BAG_CAT, BAG_NUM = 0, 1, 2
TERM_SINGLE, TERM_MULTI, TERM_MVREG, TERM_UVREG = 1, 2, 3, 4
TTE_EXP, TTE_LNM = 1, 2
LOSS_PATH_AUTO, LOSS_PATH_STREAM, LOSS_PATH_ROW_STAGED, LOSS_PATH_GENERIC = 0, 1, 2, 3
GEMM_K_CONTIG, GEMM_MN_CONTIG = 0, 1
MAX_TERMS = 16

_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_f32 = ctypes.c_float
_int = ctypes.c_int
_sz = ctypes.c_size_t


class EsgptLrSchedule(ctypes.Structure):
    """esgpt_lr_schedule: kind 0 = constant init_lr, 1 = polynomial decay with warmup (esgpt_adamw_prepare)."""
    _fields_ = [("kind", ctypes.c_int64), ("warmup", ctypes.c_int64), ("total", ctypes.c_int64),
                ("power", ctypes.c_double), ("init_lr", ctypes.c_double), ("end_lr", ctypes.c_double)]


class EsgptBatch(ctypes.Structure):
    _fields_ = [
        ("dyn_idx", _vp), ("dyn_meas", _vp), ("dyn_vals", _vp), ("dyn_vmask", _vp), ("event_mask", _vp),
        ("time_delta", _vp), ("time_abs", _vp), ("st_idx", _vp), ("st_meas", _vp),
        ("B", _i64), ("L", _i64), ("M", _i64), ("S", _i64),
    ]


class EsgptBuckets(ctypes.Structure):
    _fields_ = [("G", _i64), ("cat_bits", ctypes.c_uint64 * 8), ("num_bits", ctypes.c_uint64 * 8)]


class EsgptLossTerm(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("meas_idx", ctypes.c_int32), ("vocab_start", ctypes.c_int32),
                ("vocab_end", ctypes.c_int32), ("col", ctypes.c_int32), ("obs_col", ctypes.c_int32),
                ("level", ctypes.c_int32), ("pad", ctypes.c_int32)]


class EsgptTTESpec(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("K", ctypes.c_int32), ("col", ctypes.c_int32), ("pad", ctypes.c_int32),
                ("mean_log", _f32), ("std_log", _f32)]


_PB = ctypes.POINTER(EsgptBatch)
_PK = ctypes.POINTER(EsgptBuckets)


class EsgptPackSeg(ctypes.Structure):
    """``esgpt_pack_seg``: dst[0 .. n) = cast(src[0 .. n)), dst[n .. n_pad) = 0."""
    _fields_ = [("src", _vp), ("dst", _vp), ("n", _i64), ("n_pad", _i64), ("dst_dtype", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]

class EsgptColsumJob(ctypes.Structure):
    """``esgpt_colsum_job``: sums[c] = sum_b part[b * width + c]."""
    _fields_ = [("part", _vp), ("n_parts", _i64), ("width", _i64), ("sums", _vp)]


SIGNATURES = {
    "esgpt_version": (ctypes.c_char_p, []),
    "esgpt_adamw_chunk": (_i64, []),
    "esgpt_adamw": (_int, [_vp, _vp, _i64, _f32, _f32, _f32, _f32, _f32, _i64, _vp, _vp, _vp]),
    "esgpt_adamw_prepare": (_int, [_vp, _vp, _int, _int, _vp, ctypes.c_double, ctypes.c_double, _vp, _vp, _vp, _vp]),
    "esgpt_adamw_prepare_ex": (_int, [_vp, _vp, _int, _int, _vp, ctypes.c_double, ctypes.c_double, _vp, _vp, _vp,
                                      _vp, _i64, _vp, _vp, _i64, _vp]),
    "esgpt_adamw_prepare_tab": (_int, [_vp, _vp, _int, _int, _vp, ctypes.c_double, ctypes.c_double, _vp, _vp, _vp,
                                       _vp, _i64, _vp, _vp, _i64, _vp, _vp]),
    "esgpt_host_words_alloc": (_int, [_i64, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p)]),
    "esgpt_host_words_free": (_int, [_vp]),
    "esgpt_adamw_dev": (_int, [_vp, _vp, _i64, _vp, _f32, _f32, _f32, _f32, _vp, _vp, _vp]),
    "esgpt_device_arch_ok": (_int, []),
    "esgpt_pack": (_int, [_vp, _i64, _vp]),
    "esgpt_embed_joint_fwd": (_int, [_PB, _PK, _vp, _i64, _i64, _vp, _vp, _int, _f32, _f32, _vp, _vp, _vp]),
    "esgpt_attn_path": (_int, [_i64, _i64, _i64, _i64, _i64, _i64, _int]),
    "esgpt_event_times": (_int, [_PB, _vp, _vp]),
    "esgpt_embed_joint_fwd_ex": (_int, [_PB, _PK, _vp, _int, _i64, _i64, _vp, _vp, _int, _f32, _f32, _vp, _vp, _vp]),
    "esgpt_embed_split_bags_fwd": (_int, [_PB, _PK, _vp, _i64, _vp, _i64, _i64, _int, _f32, _f32, _f32, _vp, _vp,
                                          _vp]),
    "esgpt_embed_epilogue_fwd": (_int, [_PB, _i64, _i64, _vp, _vp, _vp, _int, _vp, _vp]),
    "esgpt_embed_epilogue_bwd": (_int, [_PB, _i64, _i64, _vp, _int, _vp, _vp]),
    "esgpt_embed_epilogue_bwd_ex": (_int, [_PB, _i64, _i64, _vp, _int, _vp, _int, _vp]),
    "esgpt_split_proj_prep": (_int, [_vp, _i64, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _vp, _f32, _f32, _vp, _vp,
                                     _int, _vp]),
    "esgpt_split_proj_post": (_int, [_vp, _i64, _vp, _vp, _vp, _i64, _i64, _i64, _f32, _f32, _vp, _vp, _vp, _vp,
                                     _int, _vp]),
    "esgpt_embed_bag_bwd_workspace": (_sz, [_PB, _i64, _i64, _i64]),
    "esgpt_embed_bag_bwd": (_int, [_PB, _PK, _int, _int, _f32, _f32, _vp, _i64, _i64, _i64, _vp, _vp, _sz, _vp]),
    "esgpt_attn_fwd": (_int, [_vp, _vp, _vp, _i64, _i64, _vp, _i64, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64,
                              _i64, _f32, _vp, _int, _vp]),
    "esgpt_attn_keep_words": (_i64, [_i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _int, _f32]),
    "esgpt_attn_fwd_ex": (_int, [_vp, _vp, _vp, _i64, _i64, _vp, _i64, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64,
                                 _i64, _f32, _vp, _int, _vp, _vp]),
    "esgpt_attn_bwd_ex": (_int, [_vp, _vp, _vp, _i64, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp,
                                 _i64, _i64, _i64, _i64, _i64, _i64, _i64, _f32, _vp, _vp, _int, _vp, _sz, _vp, _vp]),
    "esgpt_attn_bwd_lead": (_int, [_vp, _vp, _vp, _i64, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp,
                                   _i64, _i64, _i64, _i64, _i64, _i64, _i64, _f32, _vp, _vp, _int, _vp, _sz, _vp, _i64,
                                   _vp]),
    "esgpt_row_tiles": (_int, [_vp, _i64, _i64, _vp, _vp]),
    "esgpt_gemm_row_tiles": (_int, [_vp]),
    "esgpt_attn_bwd_workspace": (_sz, [_i64, _i64, _i64, _i64, _i64]),
    "esgpt_residual_fwd": (_int, [_vp, _vp, _int, _vp, _i64, _i64, _f32, _vp, _i64, _i64, _vp, _vp]),
    "esgpt_residual_bwd": (_int, [_vp, _vp, _i64, _i64, _f32, _vp, _i64, _i64, _vp, _vp, _int, _vp]),
    "esgpt_na_split_fwd": (_int, [_vp, _vp, _i64, _i64, _i64, _vp, _vp]),
    "esgpt_na_split_bwd": (_int, [_vp, _vp, _i64, _i64, _i64, _vp, _vp]),
    "esgpt_na_assemble_fwd": (_int, [_vp, _vp, _i64, _i64, _i64, _i64, _vp, _vp]),
    "esgpt_na_assemble_bwd": (_int, [_vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp]),
    "esgpt_na_head_split_fwd": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _int, _vp]),
    "esgpt_na_head_split_bwd": (_int, [_vp, _vp, _int, _i64, _i64, _i64, _vp, _vp]),
    "esgpt_attn_bwd_counters": (_i64, [_i64, _i64, _i64]),
    "esgpt_attn_bwd": (_int, [_vp, _vp, _vp, _i64, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _i64,
                              _i64, _i64, _i64, _i64, _i64, _i64, _f32, _vp, _int, _vp, _sz, _vp, _vp]),
    "esgpt_kv_append": (_int, [_vp, _i64, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _int, _vp]),
    "esgpt_attn_decode": (_int, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64,
                                 _int, _vp]),
    "esgpt_residual_ln_partials": (_i64, [_i64]),
    "esgpt_residual_ln_fwd": (_int, [_vp, _vp, _int, _vp, _vp, _f32, _vp, _vp, _vp, _f32, _i64, _i64, _vp, _vp, _int,
                                     _vp, _vp, _vp]),
    "esgpt_residual_ln_counters": (_i64, [_i64]),
    "esgpt_residual_ln_fwd_ex": (_int, [_vp, _vp, _int, _vp, _vp, _f32, _vp, _vp, _vp, _f32, _i64, _i64, _i64, _vp,
                                        _vp, _int, _vp, _vp, _vp]),
    "esgpt_residual_ln_bwd_ex": (_int, [_vp, _vp, _int, _vp, _vp, _vp, _vp, _vp, _f32, _vp, _i64, _i64, _i64, _vp,
                                        _vp, _int, _vp, _vp, _vp]),
    "esgpt_residual_ln_bwd": (_int, [_vp, _vp, _int, _vp, _vp, _vp, _vp, _vp, _f32, _vp, _i64, _i64, _vp, _vp, _int,
                                     _vp, _vp, _vp, _vp]),
    "esgpt_colsum_jobs": (_int, [ctypes.POINTER(EsgptColsumJob), _i64, _vp]),
    "esgpt_bias_act_fwd": (_int, [_vp, _vp, _int, _i64, _i64, _vp, _int, _vp]),
    "esgpt_bias_act_partials": (_i64, [_i64]),
    "esgpt_bias_act_bwd": (_int, [_vp, _vp, _vp, _int, _i64, _i64, _vp, _vp, _vp, _int, _vp]),
    "esgpt_gemm_workspace": (_sz, [_i64, _i64, _i64]),
    "esgpt_gemm_counters": (_i64, [_i64, _i64]),
    "esgpt_gemm_bf16": (_int, [_int, _vp, _i64, _int, _vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _i64, _int, _int,
                               _vp, _sz, _vp, _vp]),
    "esgpt_linear_fwd": (_int, [_vp, _i64, _vp, _i64, _i64, _i64, _vp, _int, _vp, _vp, _i64, _vp]),
    "esgpt_linear_bwd_workspace": (_sz, [_i64, _i64, _i64, _int]),
    "esgpt_linear_bwd": (_int, [_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i64, _vp, _int, _vp, _i64, _vp, _i64, _vp,
                                _vp, _vp, _sz, _vp, _vp]),
    "esgpt_linear_bwd_ex": (_int, [_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i64, _vp, _int, _vp, _i64, _vp, _i64, _vp,
                                   _vp, _vp, _sz, _vp, _vp, _i64, _vp]),
    "esgpt_linear_bwd_split": (_int, [_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i64, _vp, _int, _vp, _i64, _vp, _i64,
                                      _vp, _vp, _vp, _sz, _vp, _vp, _i64, _vp, _vp]),
    "esgpt_gemm_f32": (_int, [_int, _vp, _i64, _int, _vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _i64, _int, _vp,
                              _sz, _vp, _vp]),
    "esgpt_linear_fwd_f32": (_int, [_vp, _i64, _vp, _i64, _i64, _i64, _vp, _int, _vp, _vp, _i64, _vp]),
    "esgpt_linear_bwd_f32_workspace": (_sz, [_i64, _i64, _i64, _int]),
    "esgpt_linear_bwd_f32": (_int, [_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i64, _vp, _int, _vp, _i64, _vp, _i64,
                                    _vp, _vp, _vp, _sz, _vp, _vp, _i64, _vp]),
    "esgpt_stream_wait": (_int, [_vp, _vp]),
    "esgpt_seed_bank": (_int, [_vp, _vp, _i64, _vp]),
    "esgpt_step_begin": (_int, [_vp, _vp, _i64, _vp, _vp]),
    "esgpt_column_sum_partials": (_i64, [_i64]),
    "esgpt_column_sum": (_int, [_vp, _int, _i64, _i64, _vp, _vp, _vp]),
    "esgpt_collate_shape": (_int, [_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "esgpt_collate": (_int, [_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _int,
                             _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _int]),
    "esgpt_output_loss_workspace": (_sz, [_i64, _i64, _int]),
    "esgpt_output_loss": (_int, [_PB, _vp, _i64, _i64, _int, _vp, _vp, _i64, _int, ctypes.POINTER(EsgptLossTerm),
                                 _int, ctypes.POINTER(EsgptTTESpec), _vp, _vp, _vp, _vp, _vp, _sz, _vp, _vp]),
    "esgpt_output_loss_ex": (_int, [_PB, _vp, _i64, _i64, _int, _vp, _vp, _i64, _int, ctypes.POINTER(EsgptLossTerm),
                                    _int, ctypes.POINTER(EsgptTTESpec), _vp, _vp, _vp, _vp, _vp, _sz, _vp, _int,
                                    _vp]),
}

_lib = None


class HipExtensionMissing(RuntimeError):
    pass


def load(require_device: bool = True):
    """Returns the loaded library; raises loudly if it (or, with ``require_device``, a GPU) is unavailable."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise HipExtensionMissing(
                f"eventstreamgpt_amd: HIP library not found at {LIB_PATH}. Build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (or `make -C eventstreamgpt_amd/csrc`)."
            )
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    if require_device and not torch.cuda.is_available():
        raise HipExtensionMissing("eventstreamgpt_amd: no HIP device visible; the product path has no CPU fallback.")
    return _lib


def check(status: int, what: str):
    if status != ESGPT_OK:
        names = {1: "invalid argument", 2: "launch failure", 3: "unsupported configuration"}
        raise RuntimeError(f"eventstreamgpt_amd: {what} failed: {names.get(status, status)}")


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    raise TypeError(f"eventstreamgpt_amd: unsupported activation dtype {dt}")

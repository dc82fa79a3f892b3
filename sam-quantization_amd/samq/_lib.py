"""ctypes binding of libsamq_hip.so (the C ABI declared in include/samq.h).

The library is built in-tree (``make -C sam-quantization_amd`` or ``__graft_entry__.build()``)
and loaded from this directory.  There is NO fallback: if the library is missing or fails to
load, importing the product ops raises immediately.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

# SAMQ_LIB=tuning selects the tuning build (make tuning: adds timing-only tile configs) and
# SAMQ_LIB=<path>.so a kernel-variant build for A/B runs; tools only
_sel = os.environ.get("SAMQ_LIB", "")
LIB_PATH = (Path(_sel) if _sel.endswith(".so") else Path(__file__).resolve().parent / (
    "libsamq_hip_tuning.so" if _sel == "tuning" else "libsamq_hip.so"))

SAMQ_OK = 0
SAMQ_ERR_INVALID = -1
SAMQ_ERR_UNSUPPORTED = -2
SAMQ_ERR_HIP = -3

EPI_BIAS = 0
EPI_BIAS_GELU = 1
EPI_RESADD_F32 = 2
EPI_F32 = 3
EPI_Q8 = 4
EPI_Q8_GELU = 5
EPI_Q8_RES = 6
EPI_RESADD_LNF = 7
EPI_BIAS_LNF = 8
EPI_GELU_LNF = 9

BF_W8 = 0
BF_W4 = 1

Q_IN_F16 = 1
Q_OUT_FQ = 2

MM_PER_ROW = 0
MM_PER_COL = 1
MM_ALL = 2
LN_IN_F16 = 1
LN_OUT_F32 = 2
LN_IN_I8 = 4
LN_OUT_I8 = 8
LN_DELTA_F16 = 16

_vp = ctypes.c_void_p
_i32 = ctypes.c_int
_i64 = ctypes.c_int64
_f32 = ctypes.c_float

# name -> (restype, argtypes); must match include/samq.h exactly
SIGNATURES = {
    "samq_last_error": (ctypes.c_char_p, []),
    "samq_version": (_i32, []),
    "samq_w4_packed_words": (ctypes.c_size_t, [_i32, _i32]),
    "samq_w4_repack": (_i32, [_vp, _vp, _i32, _i32, _vp]),
    "samq_w4_repack_layout": (_i32, [_vp, _vp, _i32, _i32, _i32, _vp]),
    "samq_w4a16_gemm": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _i32, _i32, _i32, _i32, _vp]),
    "samq_w4a16_gemm_cfg": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _i32, _i32, _i32, _i32, _i32, _vp]),
    "samq_w4a16_gemm_lnf": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _i32, _i32, _i32, _i32, _i32,
                                   _vp, _vp, _vp, _vp, _vp, _vp, _f32, _vp]),
    "samq_w8_repack": (_i32, [_vp, _vp, _i32, _i32, _vp]),
    "samq_w8a8_gemm": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _i32, _i32, _i32, _i32,
                              _f32, _f32, _f32, _f32, _vp]),
    "samq_w4a8_gemm": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _i32, _i32, _i32, _i32,
                              _f32, _f32, _vp]),
    "samq_w4a8_gemm_cfg": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _i32, _i32, _i32, _i32,
                                  _f32, _f32, _i32, _vp]),
    "samq_w4a8_gemm_rs": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _i32, _i32, _i32, _f32, _f32,
                                 _vp, _vp, _i32, _vp]),
    "samq_i8_gemm_cfg": (_i32, [_vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _i32, _i32, _i32,
                                _i32, _f32, _f32, _f32, _f32, _i32, _vp]),
    "samq_w8a8_conv_gemm": (_i32, [_vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32,
                                   _f32, _f32, _f32, _f32, _vp]),
    "samq_add_layernorm": (_i32, [_vp, _vp, _vp, _vp, _vp, _i64, _i32, _f32, _i32, _f32, _vp]),
    "samq_quantize": (_i32, [_vp, _vp, _i64, _f32, _i32, _vp]),
    "samq_minmax_workspace": (ctypes.c_size_t, [_i64, _i32, _i32]),
    "samq_minmax": (_i32, [_vp, _i64, _i32, _i32, _i32, _vp, _vp, _i32, _vp, ctypes.c_size_t, _vp]),
    "samq_silu_mul": (_i32, [_vp, _vp, _vp, _i64, _vp]),
    "samq_w4a16_gated_mlp": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp, _i64, _i32, _i32, _i32, _i32, _vp]),
    "samq_layernorm": (_i32, [_vp, _vp, _vp, _vp, _i64, _i32, _f32, _i32, _vp]),
    "samq_layernorm_mean": (_i32, [_vp, _vp, _vp, _vp, _i64, _i32, _f32, _i32, _vp, _vp]),
    "samq_layernorm_q": (_i32, [_vp, _vp, _vp, _vp, _i64, _i32, _f32, _i32, _f32, _f32, _vp]),
    "samq_layernorm_q_rs": (_i32, [_vp, _vp, _vp, _vp, _i64, _i32, _f32, _i32, _f32, _f32, _vp, _vp, _vp]),
    "samq_rel_attention": (_i32, [_vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _f32, _vp]),
    "samq_rel_attention_q": (_i32, [_vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _f32, _f32, _vp]),
    "samq_attention_relbias": (_i32, [_vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _f32, _vp]),
    "samq_rel_attention_q8": (_i32, [_vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _f32, _f32,
                                     _f32, _f32, _f32, _vp]),
    "samq_rel_attention_q8_rows": (_i32, [_vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _f32, _f32,
                                          _f32, _f32, _f32, _i32, _i32, _vp, _vp]),
    "samq_w8a8_gemm_v16": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp, _i64, _i32, _i32, _i32, _f32, _f32, _vp, _i32, _i64,
                                  _i32, _vp]),
    "samq_patch_embed": (_i32, [_vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _vp]),
    "samq_patch_embed_f32": (_i32, [_vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _vp]),
    "samq_patch_embed_u8": (_i32, [_vp, _i32, _i32, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _i32, _i32, _i32, _i32,
                                   _i32, _vp]),
    "samq_conv1x1_f32": (_i32, [_vp, _vp, _vp, _i64, _i32, _i32, _vp]),
    "samq_conv3x3_nhwc": (_i32, [_vp, _vp, _vp, _i32, _i32, _i32, _i32, _vp]),
}


class SamqError(RuntimeError):
    pass


_LIB = None


def load() -> ctypes.CDLL:
    """Load (once) and return the HIP library; raise loudly if it is unavailable."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not LIB_PATH.exists():
        raise ImportError(
            f"samq: HIP library not found at {LIB_PATH}; build it with "
            f"`make -C {LIB_PATH.parent.parent}` (hipcc --offload-arch=gfx950). "
            "There is no CPU or PyTorch fallback.")
    lib = ctypes.CDLL(str(LIB_PATH), mode=os.RTLD_NOW | getattr(os, "RTLD_GLOBAL", 0))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def check(status: int, what: str = "") -> None:
    """Map a C status to the reference's exception types (see include/samq.h)."""
    if status == SAMQ_OK:
        return
    msg = load().samq_last_error().decode(errors="replace")
    if what:
        msg = f"{what}: {msg}"
    if status == SAMQ_ERR_INVALID:
        raise AssertionError(msg)
    if status == SAMQ_ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    raise SamqError(msg)


def exported_symbols():
    return list(SIGNATURES)

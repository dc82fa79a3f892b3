"""Torch-facing wrappers of the HIP kernels (device memory + current stream plumbing only).

Every op enqueues on ``torch.cuda.current_stream()`` and returns caller-owned tensors; no op
falls back to PyTorch or the CPU -- a non-CUDA tensor is an error.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _lib

EPI_BIAS = _lib.EPI_BIAS
EPI_BIAS_GELU = _lib.EPI_BIAS_GELU
EPI_RESADD_F32 = _lib.EPI_RESADD_F32
EPI_F32 = _lib.EPI_F32


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _need_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("samq ops run on the GPU only (HIP); got a CPU tensor")


# ----------------------------------------------------------------------------- W4A16
def w4_repack(qweight: torch.Tensor, layout: int = 0) -> torch.Tensor:
    """Reference ``qweight`` int32 (K/8, N) -> kernel fragment layout (flat int32 K*N/8).
    ``layout`` 0 = the product layout expected by the default GEMM dispatch."""
    _need_cuda(qweight)
    assert qweight.dtype == torch.int32 and qweight.dim() == 2
    k, n = qweight.shape[0] * 8, qweight.shape[1]
    out = torch.empty(k * n // 8, dtype=torch.int32, device=qweight.device)
    lib = _lib.load()
    if layout:
        st = lib.samq_w4_repack_layout(_ptr(qweight.contiguous()), _ptr(out), k, n, layout, _stream())
    else:
        st = lib.samq_w4_repack(_ptr(qweight.contiguous()), _ptr(out), k, n, _stream())
    _lib.check(st, "w4_repack")
    return out


def w4a16_gemm(a: torch.Tensor, wpacked: torch.Tensor, scales: torch.Tensor, qzeros: torch.Tensor,
               bias: Optional[torch.Tensor], n: int, groupsize: int, epilogue: int = EPI_BIAS,
               out: Optional[torch.Tensor] = None, cfg: int = 0) -> torch.Tensor:
    """``epilogue(a @ W4 * s + bias)`` for a (..., K) fp16 (last dim contiguous)."""
    _need_cuda(a, wpacked, scales, qzeros, bias)
    assert a.dtype == torch.float16, "A must be float16"
    k = a.shape[-1]
    a2 = a.reshape(-1, k)
    if a2.stride(-1) != 1:
        a2 = a2.contiguous()
    m = a2.shape[0]
    if out is None:
        dt = torch.float32 if epilogue in (EPI_RESADD_F32, EPI_F32) else torch.float16
        out = torch.empty(a.shape[:-1] + (n,), dtype=dt, device=a.device)
        assert epilogue != EPI_RESADD_F32, "residual epilogue needs an out tensor"
    o2 = out.reshape(-1, n)
    assert o2.stride(-1) == 1 and o2.shape[0] == m
    if bias is not None:
        assert bias.dtype == torch.float16 and bias.numel() == n
    status = _lib.load().samq_w4a16_gemm_cfg(
        _ptr(a2), a2.stride(0), _ptr(wpacked), _ptr(scales), _ptr(qzeros), _ptr(bias), _ptr(o2), o2.stride(0),
        m, n, k, groupsize, epilogue, cfg, _stream())
    _lib.check(status, "w4a16_gemm")
    return out


# ----------------------------------------------------------------------------- LayerNorm
def layernorm(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float = 1e-6,
              out: Optional[torch.Tensor] = None, out_dtype: torch.dtype = torch.float16) -> torch.Tensor:
    """Row LayerNorm over the last dim; x f32 or f16 -> f16 (or f32); gamma/beta f32."""
    _need_cuda(x, gamma, beta)
    c = x.shape[-1]
    assert x.is_contiguous() and x.dtype in (torch.float32, torch.float16)
    assert gamma.dtype == torch.float32 and beta.dtype == torch.float32
    if out is None:
        out = torch.empty(x.shape, dtype=out_dtype, device=x.device)
    assert out.is_contiguous() and out.dtype in (torch.float16, torch.float32)
    flags = (_lib.LN_IN_F16 if x.dtype == torch.float16 else 0) | (_lib.LN_OUT_F32 if out.dtype == torch.float32 else 0)
    rows = x.numel() // c
    _lib.check(_lib.load().samq_layernorm(_ptr(x), _ptr(out), _ptr(gamma), _ptr(beta), rows, c, float(eps), flags,
                                          _stream()), "layernorm")
    return out


# ----------------------------------------------------------------------------- attention
def rel_attention(qkv: torch.Tensor, qkv_bias: Optional[torch.Tensor], rel_pos_h: torch.Tensor,
                  rel_pos_w: torch.Tensor, heads: int, window: int, sm_scale: float,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """qkv f16 (B, H, W, 3C) -> out f16 (B, H, W, C); windowed (window > 0) or global."""
    _need_cuda(qkv, qkv_bias, rel_pos_h, rel_pos_w)
    b, h, w, c3 = qkv.shape
    c = c3 // 3
    hd = c // heads
    assert qkv.dtype == torch.float16 and qkv.is_contiguous()
    assert rel_pos_h.dtype == torch.float16 and rel_pos_w.dtype == torch.float16
    if out is None:
        out = torch.empty((b, h, w, c), dtype=torch.float16, device=qkv.device)
    _lib.check(_lib.load().samq_rel_attention(_ptr(qkv), _ptr(qkv_bias), _ptr(rel_pos_h.contiguous()),
                                              _ptr(rel_pos_w.contiguous()), _ptr(out), b, h, w, heads, hd, window,
                                              float(sm_scale), _stream()), "rel_attention")
    return out


def attention_relbias(inp: torch.Tensor, rel_h: torch.Tensor, rel_w: torch.Tensor, heads: int, hd: int,
                      sm_scale: float) -> torch.Tensor:
    """Reference ``fused_attention.forward`` semantics with precomputed rel_h / rel_w."""
    _need_cuda(inp, rel_h, rel_w)
    b, h, w, c3 = inp.shape
    assert h == w, "the reference kernel requires square grids (emb_len = rel.shape[-1])"
    out = torch.empty((b, h, w, c3 // 3), dtype=inp.dtype, device=inp.device)
    _lib.check(_lib.load().samq_attention_relbias(_ptr(inp.contiguous()), _ptr(rel_h.half().contiguous()),
                                                  _ptr(rel_w.half().contiguous()), _ptr(out), b, h, heads, hd,
                                                  float(sm_scale), _stream()), "attention_relbias")
    return out

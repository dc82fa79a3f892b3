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
EPI_Q8 = _lib.EPI_Q8
EPI_Q8_GELU = _lib.EPI_Q8_GELU
EPI_Q8_RES = _lib.EPI_Q8_RES
EPI_RESADD_LNF = _lib.EPI_RESADD_LNF
EPI_BIAS_LNF = _lib.EPI_BIAS_LNF
EPI_GELU_LNF = _lib.EPI_GELU_LNF

# W4A16 tile configs of the product library (include/samq.h, samq_w4a16_gemm_cfg); 0 = automatic
W4A16_CFGS = frozenset((1, 2, 3, 4, 5, 6, 7, 9, 21, 22, 23, 24, 25, 26, 29, 30, 31, 55, 56, 57, 58, 62, 64, 65, 100, 101, 104, 107, 108, 109, 110, 111, 112, 113, 114))
_Q8_EPIS = (EPI_Q8, EPI_Q8_GELU, EPI_Q8_RES)


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


def w4_interleave32(gate_packed: torch.Tensor, up_packed: torch.Tensor, gate_scales: torch.Tensor,
                    up_scales: torch.Tensor, gate_qzeros: torch.Tensor, up_qzeros: torch.Tensor, n: int):
    """The samq_w4a16_gated_mlp operand layout: two repacked (layout 1) int4 matrices of N columns
    -> one of 2N whose 32-column blocks alternate gate block j / up block j (each block is one
    contiguous run of K/64 KiB in the repacked layout), scales (G, N) / qzeros (G, N/8) the same."""
    _need_cuda(gate_packed, up_packed, gate_scales, up_scales, gate_qzeros, up_qzeros)
    assert n % 32 == 0 and gate_packed.numel() == up_packed.numel()
    nb = n // 32
    w = torch.stack([gate_packed.view(nb, -1), up_packed.view(nb, -1)], 1).reshape(-1).contiguous()
    g = gate_scales.shape[0]
    s = torch.stack([gate_scales.reshape(g, nb, 32), up_scales.reshape(g, nb, 32)], 2).reshape(g, 2 * n).contiguous()
    z = torch.stack([gate_qzeros.reshape(g, nb, 4), up_qzeros.reshape(g, nb, 4)], 2).reshape(g, n // 4).contiguous()
    return w, s, z


def w4a16_gated_mlp(a: torch.Tensor, wpacked2: torch.Tensor, scales2: torch.Tensor, qzeros2: torch.Tensor,
                    n: int, groupsize: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``silu(a . Wgate) * (a . Wup)`` f16 (..., N) in ONE launch (samq_w4a16_gated_mlp) from the
    ``w4_interleave32`` operands of the two projections."""
    _need_cuda(a, wpacked2, scales2, qzeros2)
    assert a.dtype == torch.float16 and a.stride(-1) == 1
    # the kernel's 256-column tiles over the interleaved 2N columns; the reference's
    # triton_llama_mlp_4 asserts N % 256 already (gptq_triton/fused_mlp.py:437)
    assert n % 128 == 0, "w4a16_gated_mlp: N must be a multiple of 128"
    k = a.shape[-1]
    x = a.reshape(-1, k)
    m = x.shape[0]
    if out is None:
        out = torch.empty(a.shape[:-1] + (n,), dtype=torch.float16, device=a.device)
    assert out.is_contiguous() and out.dtype == torch.float16 and out.numel() == m * n
    _lib.check(_lib.load().samq_w4a16_gated_mlp(_ptr(x), x.stride(0), _ptr(wpacked2), _ptr(scales2), _ptr(qzeros2),
                                                _ptr(out), n, m, 2 * n, k, groupsize, _stream()),
               "w4a16_gated_mlp")
    return out


def w4a16_gemm_lnf(a: torch.Tensor, wpacked: torch.Tensor, scales: torch.Tensor, qzeros: torch.Tensor,
                   bias: Optional[torch.Tensor], n: int, groupsize: int, epilogue: int, out: torch.Tensor,
                   stats: torch.Tensor, mu: torch.Tensor, gamma: Optional[torch.Tensor] = None,
                   aout: Optional[torch.Tensor] = None, gw: Optional[torch.Tensor] = None,
                   bw: Optional[torch.Tensor] = None, eps: float = 1e-6, cfg: int = 0) -> torch.Tensor:
    """The W4A16 GEMM with a LayerNorm folded into its epilogue (samq_w4a16_gemm_lnf,
    include/samq.h): ``EPI_RESADD_LNF`` -- out f32 residual += y, then aout = f16((x - mu) * gamma)
    and the per-row partial sums ``stats``; ``EPI_BIAS_LNF`` / ``EPI_GELU_LNF`` -- out f16 =
    LN(x) . W + bias (GELU) from a = that aout, ``stats`` and gw = gamma . W, bw = beta . W; mu += delta."""
    _need_cuda(a, wpacked, scales, qzeros, bias, out, stats, mu, gamma, aout, gw, bw)
    assert a.dtype == torch.float16 and a.is_contiguous() and out.is_contiguous()
    k = a.shape[-1]
    m = a.numel() // k
    assert out.numel() == m * n and stats.dtype == torch.float32 and mu.dtype == torch.float32 and mu.numel() >= m
    if epilogue == EPI_RESADD_LNF:
        assert out.dtype == torch.float32 and gamma is not None and aout is not None and aout.numel() == m * n
        assert stats.numel() >= m * (n // 64) * 2
    else:
        assert out.dtype == torch.float16 and gw is not None and bw is not None and stats.numel() >= m * (k // 64) * 2
    status = _lib.load().samq_w4a16_gemm_lnf(
        _ptr(a), k, _ptr(wpacked), _ptr(scales), _ptr(qzeros), _ptr(bias), _ptr(out), n, m, n, k, groupsize,
        epilogue, cfg, _ptr(gamma), _ptr(gw), _ptr(bw), _ptr(stats), _ptr(mu), _ptr(aout), float(eps), _stream())
    _lib.check(status, "w4a16_gemm_lnf")
    return out


# ----------------------------------------------------------------------------- LayerNorm
def layernorm(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float = 1e-6,
              out: Optional[torch.Tensor] = None, out_dtype: torch.dtype = torch.float16,
              rows_per_wave: int = 0, mean_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Row LayerNorm over the last dim; x f32 or f16 -> f16 (or f32); gamma/beta f32.
    ``rows_per_wave`` (1, 2, 4; 0 = library default) is a tuning knob (SAMQ_LN_RPW)."""
    _need_cuda(x, gamma, beta)
    c = x.shape[-1]
    assert x.is_contiguous() and x.dtype in (torch.float32, torch.float16)
    assert gamma.dtype == torch.float32 and beta.dtype == torch.float32
    if out is None:
        out = torch.empty(x.shape, dtype=out_dtype, device=x.device)
    assert out.is_contiguous() and out.dtype in (torch.float16, torch.float32)
    flags = (_lib.LN_IN_F16 if x.dtype == torch.float16 else 0) | (_lib.LN_OUT_F32 if out.dtype == torch.float32 else 0)
    flags |= rows_per_wave << 16
    rows = x.numel() // c
    if mean_out is not None:
        assert mean_out.dtype == torch.float32 and mean_out.numel() >= rows and mean_out.is_cuda
        _lib.check(_lib.load().samq_layernorm_mean(_ptr(x), _ptr(out), _ptr(gamma), _ptr(beta), rows, c, float(eps),
                                                   flags, _ptr(mean_out), _stream()), "layernorm_mean")
        return out
    _lib.check(_lib.load().samq_layernorm(_ptr(x), _ptr(out), _ptr(gamma), _ptr(beta), rows, c, float(eps), flags,
                                          _stream()), "layernorm")
    return out


def add_layernorm(x: torch.Tensor, delta: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float = 1e-6,
                  out: Optional[torch.Tensor] = None, out_scale: float = 0.0, rows_per_wave: int = 0) -> torch.Tensor:
    """x (f32, in place) += delta (f16 or f32, same shape); returns LayerNorm(x) as f16, or as int8
    codes q(LN(x), out_scale) when ``out`` is int8 (samq_add_layernorm: the residual add of the
    preceding GEMM moved out of its epilogue)."""
    _need_cuda(x, delta, gamma, beta)
    c = x.shape[-1]
    assert x.is_contiguous() and x.dtype == torch.float32 and delta.is_contiguous()
    assert delta.dtype in (torch.float16, torch.float32) and delta.numel() == x.numel()
    assert gamma.dtype == torch.float32 and beta.dtype == torch.float32
    if out is None:
        out = torch.empty(x.shape, dtype=torch.int8 if out_scale > 0 else torch.float16, device=x.device)
    assert out.is_contiguous() and out.dtype in (torch.float16, torch.int8) and out.numel() == x.numel()
    flags = (_lib.LN_DELTA_F16 if delta.dtype == torch.float16 else 0) | (_lib.LN_OUT_I8 if out.dtype == torch.int8
                                                                           else 0)
    flags |= rows_per_wave << 16
    _lib.check(_lib.load().samq_add_layernorm(_ptr(x), _ptr(delta), _ptr(out), _ptr(gamma), _ptr(beta), x.numel() // c,
                                              c, float(eps), flags, float(out_scale), _stream()), "add_layernorm")
    return out


# ----------------------------------------------------------------------------- patch embed / neck
def patch_embed(img: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], pos: Optional[torch.Tensor],
                patch: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """img f16 (B, Cin, S, S) -> f32 (B, S/p, S/p, N) = Conv2d(k=p, stride=p)(img) + bias + pos;
    weight f16 (N, Cin*p*p), bias f32 (N,), pos f32 (S/p, S/p, N) or None.  With img and weight
    both f32 the whole GEMM runs in fp32 (``samq_patch_embed_f32``, the W4A8 embedding)."""
    _need_cuda(img, weight, bias, pos)
    b, cin, s, s2 = img.shape
    f32 = img.dtype == torch.float32
    dt = torch.float32 if f32 else torch.float16
    assert s == s2 and img.dtype == dt and img.is_contiguous()
    n = weight.shape[0]
    assert weight.dtype == dt and weight.is_contiguous() and weight.shape[1] == cin * patch * patch
    assert bias is None or (bias.dtype == torch.float32 and bias.is_contiguous())
    assert pos is None or (pos.dtype == torch.float32 and pos.is_contiguous() and pos.numel() == (s // patch) ** 2 * n)
    g = s // patch
    if out is None:
        out = torch.empty((b, g, g, n), dtype=torch.float32, device=img.device)
    assert out.dtype == torch.float32 and out.is_contiguous() and out.numel() == b * g * g * n
    fn = _lib.load().samq_patch_embed_f32 if f32 else _lib.load().samq_patch_embed
    _lib.check(fn(_ptr(img), _ptr(weight), _ptr(bias), _ptr(pos), _ptr(out), b, cin, s, patch, n, _stream()),
               "patch_embed")
    return out


def patch_embed_u8(img: torch.Tensor, pixel_mean: torch.Tensor, pixel_std: torch.Tensor, weight: torch.Tensor,
                   bias: Optional[torch.Tensor], pos: Optional[torch.Tensor], patch: int, img_size: int,
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Raw uint8 pixels (B, Cin, h, w), h, w <= img_size -> f32 (B, S/p, S/p, N): Sam.preprocess
    (normalise by pixel mean / std, zero-pad to img_size) fused into the patch-embedding GEMM.
    weight f16 (fp16 MFMA) or f32 (fp32 MFMA, the W4A8 embedding)."""
    _need_cuda(img, pixel_mean, pixel_std, weight, bias, pos)
    assert img.dtype == torch.uint8 and img.dim() == 4 and img.is_contiguous()
    b, cin, h, w = img.shape
    mean = pixel_mean.reshape(-1).float().contiguous()
    std = pixel_std.reshape(-1).float().contiguous()
    assert mean.numel() == cin and std.numel() == cin
    n = weight.shape[0]
    assert weight.dtype in (torch.float16, torch.float32) and weight.is_contiguous()
    assert weight.shape[1] == cin * patch * patch
    g = img_size // patch
    if out is None:
        out = torch.empty((b, g, g, n), dtype=torch.float32, device=img.device)
    assert out.dtype == torch.float32 and out.is_contiguous() and out.numel() == b * g * g * n
    _lib.check(_lib.load().samq_patch_embed_u8(_ptr(img), h, w, _ptr(mean), _ptr(std), _ptr(weight),
                                               int(weight.dtype == torch.float32), _ptr(bias), _ptr(pos), _ptr(out),
                                               b, cin, img_size, patch, n, _stream()), "patch_embed_u8")
    return out


def conv1x1_f32(x: torch.Tensor, weight: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """x f32 (..., K) tokens -> f16 (..., N) = x . weight^T (1x1 conv, no bias); weight f16 (N, K)."""
    _need_cuda(x, weight)
    k = x.shape[-1]
    n = weight.shape[0]
    assert x.dtype == torch.float32 and x.is_contiguous() and weight.dtype == torch.float16 and weight.shape[1] == k
    if out is None:
        out = torch.empty(x.shape[:-1] + (n,), dtype=torch.float16, device=x.device)
    assert out.dtype == torch.float16 and out.is_contiguous()
    _lib.check(_lib.load().samq_conv1x1_f32(_ptr(x), _ptr(weight.contiguous()), _ptr(out), x.numel() // k, n, k,
                                            _stream()), "conv1x1")
    return out


def conv3x3_nhwc(x: torch.Tensor, weight_tap_major: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """x f16 (B, G, G, Cin) -> f16 (B, G, G, N): 3x3 conv, padding 1, no bias; weight f16 (N, 3, 3, Cin)."""
    _need_cuda(x, weight_tap_major)
    b, g, g2, cin = x.shape
    assert g == g2 and x.dtype == torch.float16 and x.is_contiguous()
    w = weight_tap_major
    n = w.shape[0]
    assert w.dtype == torch.float16 and w.is_contiguous() and tuple(w.shape[1:]) == (3, 3, cin)
    if out is None:
        out = torch.empty((b, g, g, n), dtype=torch.float16, device=x.device)
    assert out.dtype == torch.float16 and out.is_contiguous()
    _lib.check(_lib.load().samq_conv3x3_nhwc(_ptr(x), _ptr(w), _ptr(out), b, g, cin, n, _stream()), "conv3x3")
    return out


# ----------------------------------------------------------------------------- attention
def rel_attention(qkv: torch.Tensor, qkv_bias: Optional[torch.Tensor], rel_pos_h: torch.Tensor,
                  rel_pos_w: torch.Tensor, heads: int, window: int, sm_scale: float,
                  out: Optional[torch.Tensor] = None, out_scale: float = 0.0) -> torch.Tensor:
    """qkv f16 (B, H, W, 3C) -> out f16 (B, H, W, C); windowed (window > 0) or global.
    out_scale > 0: out int8 codes of the fp16 output quantised with out_scale (samq_rel_attention_q,
    the W4A8 proj-input QAct folded into the store)."""
    _need_cuda(qkv, qkv_bias, rel_pos_h, rel_pos_w)
    b, h, w, c3 = qkv.shape
    c = c3 // 3
    hd = c // heads
    assert qkv.dtype == torch.float16 and qkv.is_contiguous()
    assert rel_pos_h.dtype == torch.float16 and rel_pos_w.dtype == torch.float16
    odt = torch.int8 if out_scale > 0 else torch.float16
    if out is None:
        out = torch.empty((b, h, w, c), dtype=odt, device=qkv.device)
    assert out.dtype == odt and out.is_contiguous()
    args = (_ptr(qkv), _ptr(qkv_bias), _ptr(rel_pos_h.contiguous()), _ptr(rel_pos_w.contiguous()), _ptr(out),
            b, h, w, heads, hd, window, float(sm_scale))
    if out_scale > 0:
        _lib.check(_lib.load().samq_rel_attention_q(*args, float(out_scale), _stream()), "rel_attention_q")
    else:
        _lib.check(_lib.load().samq_rel_attention(*args, _stream()), "rel_attention")
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


# ----------------------------------------------------------------------------- int8 activations
def quantize(x: torch.Tensor, scale: float, fake: bool = False, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fq_vit QAct (quant mode): int8 codes ``clamp(round(x / s), -128, 127)`` (or, with
    ``fake``, the f32 value ``codes * s``).  x f32 / f16 contiguous."""
    _need_cuda(x)
    assert x.is_contiguous() and x.dtype in (torch.float32, torch.float16)
    if out is None:
        out = torch.empty(x.shape, dtype=torch.float32 if fake else torch.int8, device=x.device)
    flags = (_lib.Q_IN_F16 if x.dtype == torch.float16 else 0) | (_lib.Q_OUT_FQ if fake else 0)
    _lib.check(_lib.load().samq_quantize(_ptr(x), _ptr(out), x.numel(), float(scale), flags, _stream()), "quantize")
    return out


def minmax_update(x2d: torch.Tensor, axis: int, max_val: Optional[torch.Tensor] = None,
                  min_val: Optional[torch.Tensor] = None):
    """fq_vit ``MinmaxObserver.update`` core on the GPU (``samq_minmax``): running max / min of a
    contiguous (rows, C) f32 / f16 tensor per row (``MM_PER_ROW``), per column (``MM_PER_COL``)
    or over everything (``MM_ALL``, 0-dim results).  ``max_val`` / ``min_val`` None -> fresh f32
    tensors; else they are merged in place (f32, contiguous, matching shape)."""
    _need_cuda(x2d)
    assert x2d.dim() == 2 and x2d.is_contiguous() and x2d.dtype in (torch.float32, torch.float16)
    rows, c = x2d.shape
    shape = {_lib.MM_PER_ROW: (rows,), _lib.MM_PER_COL: (c,), _lib.MM_ALL: ()}[axis]
    init = max_val is None
    if init:
        max_val = torch.empty(shape, dtype=torch.float32, device=x2d.device)
        min_val = torch.empty(shape, dtype=torch.float32, device=x2d.device)
    for t in (max_val, min_val):
        assert t.dtype == torch.float32 and t.is_contiguous() and tuple(t.shape) == shape and t.device == x2d.device
    lib = _lib.load()
    nws = lib.samq_minmax_workspace(rows, c, axis)
    ws = torch.empty(max(nws, 1), dtype=torch.float32, device=x2d.device)
    _lib.check(lib.samq_minmax(_ptr(x2d), rows, c, int(x2d.dtype == torch.float16), axis, _ptr(max_val),
                               _ptr(min_val), int(init), _ptr(ws), nws, _stream()), "minmax")
    return max_val, min_val


def layernorm_q(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float, in_scale: float = 0.0,
                out_scale: float = 0.0, out_dtype: torch.dtype = torch.int8,
                out: Optional[torch.Tensor] = None, rows_per_wave: int = 0,
                rowsum: Optional[torch.Tensor] = None, zero_rows: Optional[torch.Tensor] = None) -> torch.Tensor:
    """LayerNorm with int8 codes on either side: x int8 (codes * in_scale) / f32 / f16;
    out int8 codes (q(y, out_scale)), f32 fake-quant (out_dtype f32 with out_scale > 0), f16 or f32.
    ``rows_per_wave`` (1, 2, 4; 0 = library default) as in ``layernorm``.  ``rowsum`` (int32 [rows],
    int8-code output only): the output rows' code sums (``samq_layernorm_q_rs``, the W4A8 GEMM's
    row sums); ``zero_rows`` (int32 [rows]) is zeroed on the way."""
    if rowsum is not None:
        return _layernorm_q_rs(x, gamma, beta, eps, in_scale, out_scale, out, rows_per_wave, rowsum, zero_rows)
    _need_cuda(x, gamma, beta)
    c = x.shape[-1]
    assert x.is_contiguous() and gamma.dtype == torch.float32 and beta.dtype == torch.float32
    if out is None:
        out = torch.empty(x.shape, dtype=out_dtype, device=x.device)
    flags = 0
    if x.dtype == torch.int8:
        flags |= _lib.LN_IN_I8
    elif x.dtype == torch.float16:
        flags |= _lib.LN_IN_F16
    if out.dtype == torch.int8:
        flags |= _lib.LN_OUT_I8
    elif out.dtype == torch.float32:
        flags |= _lib.LN_OUT_F32 | (_lib.LN_OUT_I8 if out_scale > 0 else 0)
    flags |= rows_per_wave << 16
    _lib.check(_lib.load().samq_layernorm_q(_ptr(x), _ptr(out), _ptr(gamma), _ptr(beta), x.numel() // c, c,
                                            float(eps), flags, float(in_scale), float(out_scale), _stream()),
               "layernorm_q")
    return out


def _rows_i32(t: Optional[torch.Tensor], rows: int, what: str) -> None:
    if t is not None:
        assert t.dtype == torch.int32 and t.is_contiguous() and t.numel() >= rows, f"{what}: int32 [rows] expected"


def _layernorm_q_rs(x, gamma, beta, eps, in_scale, out_scale, out, rows_per_wave, rowsum, zero_rows):
    _need_cuda(x, gamma, beta, rowsum, zero_rows)
    c = x.shape[-1]
    rows = x.numel() // c
    assert x.is_contiguous() and gamma.dtype == torch.float32 and beta.dtype == torch.float32
    _rows_i32(rowsum, rows, "layernorm_q rowsum")
    _rows_i32(zero_rows, rows, "layernorm_q zero_rows")
    if out is None:
        out = torch.empty(x.shape, dtype=torch.int8, device=x.device)
    assert out.dtype == torch.int8, "layernorm_q: row sums need int8-code output"
    flags = _lib.LN_OUT_I8 | (rows_per_wave << 16)
    if x.dtype == torch.int8:
        flags |= _lib.LN_IN_I8
    elif x.dtype == torch.float16:
        flags |= _lib.LN_IN_F16
    _lib.check(_lib.load().samq_layernorm_q_rs(_ptr(x), _ptr(out), _ptr(gamma), _ptr(beta), rows, c, float(eps), flags,
                                               float(in_scale), float(out_scale), _ptr(rowsum), _ptr(zero_rows),
                                               _stream()), "layernorm_q_rs")
    return out


def w8_repack(w: torch.Tensor) -> torch.Tensor:
    """int8 weight codes [N, K] (QLinear / flattened QConv2d layout) -> int8 MFMA fragment order."""
    _need_cuda(w)
    assert w.dtype == torch.int8 and w.dim() == 2
    w = w.contiguous()
    n, k = w.shape
    out = torch.empty(n * k, dtype=torch.int8, device=w.device)
    _lib.check(_lib.load().samq_w8_repack(_ptr(w), _ptr(out), k, n, _stream()), "w8_repack")
    return out


def _i8_out(a2, n, epilogue, out, shape):
    if out is None:
        if epilogue in _Q8_EPIS:
            dt = torch.int8
        elif epilogue in (EPI_RESADD_F32, EPI_F32):
            dt = torch.float32
        else:
            dt = torch.float16
        assert epilogue != EPI_RESADD_F32, "residual epilogue needs an out tensor"
        out = torch.empty(shape + (n,), dtype=dt, device=a2.device)
    o2 = out.reshape(-1, n)
    assert o2.stride(-1) == 1 and o2.shape[0] == a2.shape[0]
    return out, o2


def i8_gemm(a: torch.Tensor, bfmt: int, wpacked: torch.Tensor, wscale: torch.Tensor, n: int,
            bias: Optional[torch.Tensor] = None, qzeros: Optional[torch.Tensor] = None, epilogue: int = EPI_BIAS,
            a_scale: float = 1.0, out_scale: float = 0.0, mid_scale: float = 0.0, res_scale: float = 0.0,
            res: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None, cfg: int = 0) -> torch.Tensor:
    """int8 codes a (..., K) x packed weights (bfmt 0: W8 from w8_repack, 1: GPTQ W4 layout 3)."""
    _need_cuda(a, wpacked, wscale, bias, qzeros, res)
    assert a.dtype == torch.int8 and wscale.dtype == torch.float32
    assert bias is None or bias.dtype == torch.float32
    k = a.shape[-1]
    a2 = a.reshape(-1, k)
    out, o2 = _i8_out(a2, n, epilogue, out, tuple(a.shape[:-1]))
    r2 = None if res is None else res.reshape(-1, n)
    status = _lib.load().samq_i8_gemm_cfg(
        _ptr(a2), a2.stride(0), bfmt, _ptr(wpacked), _ptr(wscale), _ptr(qzeros), _ptr(bias), _ptr(o2), o2.stride(0),
        _ptr(r2), 0 if r2 is None else r2.stride(0), a2.shape[0], n, k, epilogue, float(a_scale), float(mid_scale),
        float(res_scale), float(out_scale), cfg, _stream())
    _lib.check(status, "i8_gemm")
    return out


def w8a8_gemm(a, wpacked, wscale, n, bias=None, epilogue=EPI_Q8, a_scale=1.0, out_scale=0.0, mid_scale=0.0,
              res_scale=0.0, res=None, out=None, cfg=0):
    """fq_vit QLinear on int8 codes: ``epilogue(float(sum a w) * a_scale * wscale[n] + bias[n])``."""
    return i8_gemm(a, _lib.BF_W8, wpacked, wscale, n, bias, None, epilogue, a_scale, out_scale, mid_scale,
                   res_scale, res, out, cfg)


def w8a8_gemm_v16(a, wpacked, wscale, n, bias, a_scale, out_scale, v16, v_col0, out=None, cfg=0):
    """``w8a8_gemm`` with the Q8 epilogue that also stores the codes of columns [v_col0, n) as fp16
    into ``v16`` (rows x (n - v_col0)): the fq_vit qkv projection feeding ``rel_attention_q8(v16=)``."""
    _need_cuda(a, wpacked, wscale, bias, v16)
    assert a.dtype == torch.int8 and wscale.dtype == torch.float32 and v16.dtype == torch.float16
    k = a.shape[-1]
    a2 = a.reshape(-1, k)
    out, o2 = _i8_out(a2, n, EPI_Q8, out, tuple(a.shape[:-1]))
    v2 = v16.reshape(a2.shape[0], -1)
    assert v2.is_contiguous() and v2.shape[1] >= n - v_col0
    _lib.check(_lib.load().samq_w8a8_gemm_v16(
        _ptr(a2), a2.stride(0), _ptr(wpacked), _ptr(wscale), _ptr(bias), _ptr(o2), o2.stride(0), a2.shape[0], n, k,
        float(a_scale), float(out_scale), _ptr(v2), int(v_col0), v2.stride(0), cfg, _stream()), "w8a8_gemm_v16")
    return out


def w8a8_conv_gemm(x: torch.Tensor, mode: int, wpacked: torch.Tensor, wscale: torch.Tensor, n: int,
                   bias: Optional[torch.Tensor] = None, epilogue: int = EPI_Q8, a_scale: float = 1.0,
                   out_scale: float = 0.0, mid_scale: float = 0.0, res_scale: float = 0.0,
                   res: Optional[torch.Tensor] = None, rmod: int = 0) -> torch.Tensor:
    """fq_vit QConv2d on int8 codes as an implicit GEMM (``samq_w8a8_conv_gemm``): mode 1 = the
    16x16 / stride-16 PatchEmbed on NCHW codes (B, Cin, S, S); mode 2 = the 3x3 / pad-1 neck conv on
    NHWC codes (B, G, G, Cin).  Returns int8 codes (B, G, G, n)."""
    _need_cuda(x, wpacked, wscale, bias, res)
    assert x.dtype == torch.int8 and x.is_contiguous() and wscale.dtype == torch.float32
    if mode == 1:
        b, cin, side, _ = x.shape
        g = side // 16
    else:
        b, g, _, cin = x.shape
        side = g
    out = torch.empty((b, g, g, n), dtype=torch.int8, device=x.device)
    _lib.check(_lib.load().samq_w8a8_conv_gemm(_ptr(x), mode, b, cin, side, _ptr(wpacked), _ptr(wscale), _ptr(bias),
                                               _ptr(out), _ptr(res), rmod, n, epilogue, float(a_scale),
                                               float(mid_scale), float(res_scale), float(out_scale), _stream()),
               "w8a8_conv_gemm")
    return out


def w4a8_gemm(a, wpacked3, wscale, qzeros, n, bias=None, epilogue=EPI_BIAS, a_scale=1.0, out_scale=0.0,
              out=None, groupsize=-1, cfg=0, rowsum=None, rowsum_out=None):
    """GPTQ int4 weights (repacked layout 3) x int8 activation codes (cfg 0 = library pick).
    ``groupsize`` -1 (per-channel, ``wscale`` f32 [N]) or a multiple of 128 (grouped:
    ``wscale`` f32 [G, N], ``qzeros`` [G, N/8]; samq_w4a8_gemm_cfg).  Per-channel only:
    ``rowsum`` (int32 [M]) = the input rows' code sums from their producer (the zero-point
    ping-pong then skips its own), ``rowsum_out`` (int32 [M], zeroed by the caller; int8-code
    epilogues) accumulates the output rows' code sums (``samq_w4a8_gemm_rs``)."""
    if (rowsum is not None or rowsum_out is not None) and groupsize in (-1, a.shape[-1]):
        _need_cuda(a, wpacked3, wscale, bias, qzeros, rowsum, rowsum_out)
        assert a.dtype == torch.int8 and wscale.dtype == torch.float32
        assert bias is None or bias.dtype == torch.float32
        k = a.shape[-1]
        a2 = a.reshape(-1, k)
        _rows_i32(rowsum, a2.shape[0], "w4a8_gemm rowsum")
        _rows_i32(rowsum_out, a2.shape[0], "w4a8_gemm rowsum_out")
        out, o2 = _i8_out(a2, n, epilogue, out, tuple(a.shape[:-1]))
        status = _lib.load().samq_w4a8_gemm_rs(
            _ptr(a2), a2.stride(0), _ptr(wpacked3), _ptr(wscale), _ptr(qzeros), _ptr(bias), _ptr(o2), o2.stride(0),
            a2.shape[0], n, k, epilogue, float(a_scale), float(out_scale), _ptr(rowsum), _ptr(rowsum_out), cfg,
            _stream())
        _lib.check(status, "w4a8_gemm_rs")
        return out
    if groupsize in (-1, a.shape[-1]):
        return i8_gemm(a, _lib.BF_W4, wpacked3, wscale, n, bias, qzeros, epilogue, a_scale, out_scale, out=out,
                       cfg=cfg)
    if groupsize <= 0 or groupsize % 128:
        raise NotImplementedError("w4a8_gemm: grouped weights need groupsize % 128 == 0 (the int8 K tile)")
    _need_cuda(a, wpacked3, wscale, bias, qzeros)
    assert a.dtype == torch.int8 and wscale.dtype == torch.float32
    assert bias is None or bias.dtype == torch.float32
    k = a.shape[-1]
    assert wscale.numel() == ((k + groupsize - 1) // groupsize) * n, "w4a8_gemm: wscale must be f32 [G, N]"
    a2 = a.reshape(-1, k)
    out, o2 = _i8_out(a2, n, epilogue, out, tuple(a.shape[:-1]))
    status = _lib.load().samq_w4a8_gemm_cfg(
        _ptr(a2), a2.stride(0), _ptr(wpacked3), _ptr(wscale), _ptr(qzeros), _ptr(bias), _ptr(o2), o2.stride(0),
        a2.shape[0], n, k, groupsize, epilogue, float(a_scale), float(out_scale), cfg, _stream())
    _lib.check(status, "w4a8_gemm")
    return out


def rel_attention_q8(qkv: torch.Tensor, qkv_bias: Optional[torch.Tensor], rel_pos_h: torch.Tensor,
                     rel_pos_w: torch.Tensor, heads: int, window: int, sm_scale: float, s_qkv: float, s_a1: float,
                     s_a2: float, s_out: float, out: Optional[torch.Tensor] = None,
                     rows: Optional[tuple] = None, v16: Optional[torch.Tensor] = None) -> torch.Tensor:
    """W8A8 attention on int8 qkv codes (B, H, W, 3C) -> int8 output codes (B, H, W, C).
    ``rows = (row0, n)``: only the queries (global) / windows (windowed) of grid rows
    [row0, row0 + n) are computed (``samq_rel_attention_q8_rows``).  ``v16``: the V codes as fp16
    (B, H, W, C) from ``w8a8_gemm_v16`` (the global kernel then stages V unconverted)."""
    if v16 is not None:
        _need_cuda(v16)
        assert v16.dtype == torch.float16 and v16.is_contiguous() and v16.numel() == qkv.numel() // 3
    _need_cuda(qkv, qkv_bias, rel_pos_h, rel_pos_w)
    b, h, w, c3 = qkv.shape
    c = c3 // 3
    assert qkv.dtype == torch.int8 and qkv.is_contiguous()
    assert rel_pos_h.dtype == torch.float32 and rel_pos_w.dtype == torch.float32
    assert qkv_bias is None or qkv_bias.dtype == torch.float32
    if out is None:
        out = torch.empty((b, h, w, c), dtype=torch.int8, device=qkv.device)
    r0, nr = rows if rows is not None else (0, -1)
    _lib.check(_lib.load().samq_rel_attention_q8_rows(
        _ptr(qkv), _ptr(qkv_bias), _ptr(rel_pos_h.contiguous()), _ptr(rel_pos_w.contiguous()), _ptr(out), b, h, w,
        heads, c // heads, window, float(sm_scale), float(s_qkv), float(s_a1), float(s_a2), float(s_out), int(r0),
        int(nr), _ptr(v16), _stream()), "rel_attention_q8")
    return out


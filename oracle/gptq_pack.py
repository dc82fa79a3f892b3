"""Bit-exact GPTQ int4 packing, unpacking and dequantisation (numpy).

TEST INFRASTRUCTURE (oracle) -- see ``oracle/__init__.py``.

Packed layout (the on-disk / module-buffer contract of ``QuantLinear``,
reference ``gptq_triton/quant_linear.py:81-109``):

* ``qweight``  int32 ``(K/8, N)``: word ``qweight[k//8, n]`` holds input feature ``k`` of
  output ``n`` in bits ``4*(k%8) .. 4*(k%8)+3``;
* ``qzeros``   int32 ``(G, N/8)``: word ``qzeros[g, n//8]`` holds ``zero-1`` of output ``n``
  in bits ``4*(n%8)..``; a zero point of 0 is stored as -1 and, because packing ORs
  ``-1 << 4j``, sets every higher nibble of that word (quirk 4 of SURVEY.md §0);
* ``scales``   fp16  ``(G, N)``; ``G = ceil(K / groupsize)``.

The kernel decodes ``q = (qweight >> 4*(k%8)) & 0xF`` and ``zp = ((qzeros >> 4*(n%8)) & 0xF) + 1``
(``quant_linear.py:299-339``) so the effective weight is ``s * (q - zp)``.
"""
from __future__ import annotations

import numpy as np

MASK32 = np.int64(0xFFFFFFFF)


def _to_int32(a64: np.ndarray) -> np.ndarray:
    return (a64 & MASK32).astype(np.uint32).view(np.int32)


# ---------------------------------------------------------------- RTN quantizer
def rtn_find_params(w: np.ndarray, bits: int = 4):
    """Asymmetric per-row min/max parameters.

    Restates ``gptq.Quantizer.find_params`` (reference ``gptq.py:218-299``) for
    ``perchannel=True, sym=False, mse=False, weight=True``: the range always contains 0,
    all-zero rows get ``[-1, 1]``, ``scale = (xmax-xmin)/maxq``, ``zero = round(-xmin/scale)``.
    ``w``: (rows, cols) float32.  Returns fp32 ``scale, zero`` of shape (rows,).
    """
    w = np.asarray(w, dtype=np.float32)
    maxq = np.float32(2 ** bits - 1)
    xmin = np.minimum(w.min(axis=1), np.float32(0))
    xmax = np.maximum(w.max(axis=1), np.float32(0))
    both0 = (xmin == 0) & (xmax == 0)
    xmin = np.where(both0, np.float32(-1), xmin).astype(np.float32)
    xmax = np.where(both0, np.float32(1), xmax).astype(np.float32)
    scale = ((xmax - xmin) / maxq).astype(np.float32)
    zero = np.round(-xmin / scale).astype(np.float32)  # numpy round = half-to-even, as torch.round
    return scale, zero


def rtn_quantize(w: np.ndarray, scale: np.ndarray, zero: np.ndarray, bits: int = 4) -> np.ndarray:
    """Fake-quantised weight ``scale*(clamp(round(w/scale)+zero, 0, maxq) - zero)``.

    Restates ``gptq.quantize`` (reference ``gptq.py:183-187``); ``scale``/``zero`` broadcast
    against ``w`` (pass them as column vectors for per-row parameters).
    """
    maxq = np.float32(2 ** bits - 1)
    q = np.clip(np.round(w / scale) + zero, 0, maxq)
    return (scale * (q - zero)).astype(np.float32)


def rtn_quantize_linear(w: np.ndarray, groupsize: int = -1, bits: int = 4):
    """RTN-quantise a Linear weight ``w`` (N, K) per output row and per K-group.

    Returns ``(w_fake (N,K) fp32, scale (N,G) fp32, zero (N,G) fp32)`` -- the same triple
    ``GPTQ.fasterquant`` hands to ``pack_linear`` (``gptq.py:115-171``) but without the
    Hessian error feedback (round-to-nearest), which is what the fixtures use.
    """
    w = np.asarray(w, dtype=np.float32)
    n, k = w.shape
    g = k if groupsize == -1 else groupsize
    ngroups = (k + g - 1) // g
    scales = np.zeros((n, ngroups), np.float32)
    zeros = np.zeros((n, ngroups), np.float32)
    fake = np.empty_like(w)
    for gi in range(ngroups):
        cols = slice(gi * g, min(k, (gi + 1) * g))
        s, z = rtn_find_params(w[:, cols], bits)
        scales[:, gi], zeros[:, gi] = s, z
        fake[:, cols] = rtn_quantize(w[:, cols], s[:, None], z[:, None], bits)
    return fake, scales, zeros


# ---------------------------------------------------------------- packing
def pack_linear(weight: np.ndarray, scales: np.ndarray, zeros: np.ndarray, groupsize: int, bits: int = 4):
    """Pack a fake-quantised weight into ``(qweight, qzeros, scales_fp16)``.

    Restates ``pack_linear`` (reference ``gptq4sam.py:434-497``), including its exact
    rounding ``q = round((w + zero*scale) / scale)`` with fp32 ``scale`` per group of the
    ORIGINAL column index, the fp16 cast of the stored scales, and the ``zero-1`` packing
    whose sign-extension corrupts higher nibbles when a zero point is 0 (quirk 4).

    weight (N, K) fp32; scales/zeros (N, G) fp32 (as returned by the quantizer).
    """
    assert bits == 4
    weight = np.asarray(weight, np.float32)
    n, k = weight.shape
    g = k if groupsize == -1 else groupsize
    s_t = np.ascontiguousarray(np.asarray(scales, np.float32).T)  # (G, N)
    z_t = np.ascontiguousarray(np.asarray(zeros, np.float32).T)   # (G, N)
    sz = (z_t * s_t).astype(np.float32)
    gidx = np.arange(k) // g
    # intweight[k, n]
    iw = np.round((weight.T + sz[gidx]) / s_t[gidx]).astype(np.int64)
    qweight = np.zeros((k // 8, n), np.int64)
    for j in range(8):
        qweight |= iw[j::8] << (4 * j)
    zi = (z_t - 1).astype(np.int64)  # (G, N), may be -1
    qzeros = np.zeros((z_t.shape[0], n // 8), np.int64)
    for j in range(8):
        qzeros |= zi[:, j::8] << (4 * j)
    return _to_int32(qweight), _to_int32(qzeros), s_t.astype(np.float16)


def unpack_qweight(qweight: np.ndarray) -> np.ndarray:
    """int32 (K/8, N) -> uint8 codes q (K, N); ``quant_linear.py:292-294, 336``."""
    u = np.asarray(qweight).view(np.uint32).astype(np.int64)
    kk, n = u.shape
    out = np.empty((kk * 8, n), np.uint8)
    for j in range(8):
        out[j::8] = (u >> (4 * j)) & 0xF
    return out


def unpack_zeros(qzeros: np.ndarray) -> np.ndarray:
    """int32 (G, N/8) -> decoded zero points ``nibble+1`` (G, N); ``quant_linear.py:312-313``."""
    u = np.asarray(qzeros).view(np.uint32).astype(np.int64)
    g, nn8 = u.shape
    out = np.empty((g, nn8 * 8), np.int64)
    for j in range(8):
        out[:, j::8] = ((u >> (4 * j)) & 0xF) + 1
    return out


def dequant_g1(qweight, scales, qzeros, groupsize: int) -> np.ndarray:
    """Oracle G1 weight (K, N) fp32: ``float(s16) * (q - zp)`` -- the CPU fake-quant path."""
    q = unpack_qweight(qweight).astype(np.float32)
    zp = unpack_zeros(qzeros).astype(np.float32)
    s = np.asarray(scales).astype(np.float32)
    k = q.shape[0]
    g = k if groupsize == -1 else groupsize
    gidx = np.arange(k) // g
    return (s[gidx] * (q - zp[gidx])).astype(np.float32)


def dequant_g2(qweight, scales, qzeros, groupsize: int) -> np.ndarray:
    """Oracle G2 weight (K, N) fp16: the Triton kernel's fp16 dequant
    ``fp16(q*s) - fp16(zp*s)`` (``quant_linear.py:312-313, 336-339``)."""
    q = unpack_qweight(qweight).astype(np.float16)
    zp = unpack_zeros(qzeros).astype(np.float16)
    s = np.asarray(scales).astype(np.float16)
    k = q.shape[0]
    g = k if groupsize == -1 else groupsize
    gidx = np.arange(k) // g
    zs = (zp * s).astype(np.float16)          # (G, N) fp16 product
    return ((q * s[gidx]).astype(np.float16) - zs[gidx]).astype(np.float16)


def matmul4_g1(a: np.ndarray, qweight, scales, qzeros, groupsize: int, bias=None) -> np.ndarray:
    """fp32 ``a @ W_g1 + bias`` (a: (M,K))."""
    w = dequant_g1(qweight, scales, qzeros, groupsize)
    c = np.asarray(a, np.float32) @ w
    if bias is not None:
        c = c + np.asarray(bias, np.float32)
    return c


def matmul4_g2(a: np.ndarray, qweight, scales, qzeros, groupsize: int, bias=None) -> np.ndarray:
    """Triton semantics: fp16 operands, fp32 accumulate, fp16 store, fp16 ``c + bias``
    (``quant_linear.py:341-352, 431-435``)."""
    w = dequant_g2(qweight, scales, qzeros, groupsize).astype(np.float32)
    c = (np.asarray(a, np.float16).astype(np.float32) @ w).astype(np.float16)
    if bias is not None:
        c = (c + np.asarray(bias, np.float16)).astype(np.float16)
    return c

"""``QuantAttention`` / ``make_quant_attn`` / ``forward`` -- the reference's
``gptq_triton.fused_attention`` API (``gptq_triton/fused_attention.py``) on the HIP kernels.

``QuantAttention.forward(x)`` takes the already window-partitioned ``(B', h, w, C)`` tensor like
the reference (``:107-149``) and runs: qkv projection (HIP W4A16 GEMM when ``qkv_proj`` is a
``QuantLinear``) -> HIP attention with the decomposed relative-position bias computed in-kernel
(no ``rel_h``/``rel_w`` tensors, no ``torch.full`` output init) -> output projection.
The whole-encoder fast path (``samq.engine``) goes further and skips the partition copies.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn as nn

from . import ops
from .modeling import Attention, get_rel_pos


def make_quant_attn(model: nn.Module) -> None:
    """Replace every SAM ``Attention`` by ``QuantAttention`` (reference ``:12-43``)."""
    for name, m in list(model.named_modules()):
        if not isinstance(m, Attention):
            continue
        attn = QuantAttention(m.qkv, m.proj, m.num_heads, m.scale, m.use_rel_pos,
                              m.rel_pos_h if m.use_rel_pos else None,
                              m.rel_pos_w if m.use_rel_pos else None)
        attn.window_size = getattr(m, "window_size", 0)
        parent_name, _, child = name.rpartition(".")
        parent = model.get_submodule(parent_name) if parent_name else model
        setattr(parent, child, attn)


def add_decomposed_rel_pos(q: torch.Tensor, rel_pos_h: torch.Tensor, rel_pos_w: torch.Tensor,
                           q_size: Tuple[int, int], k_size: Tuple[int, int]):
    """``(rel_h, rel_w)`` bias tensors of the reference helper (``:46-80``), including its
    indexing of the width table by the query ROW (batch-broadcast of ``Rw``)."""
    rh = get_rel_pos(q_size[0], k_size[0], rel_pos_h)
    rw = get_rel_pos(q_size[1], k_size[1], rel_pos_w)
    return torch.matmul(q, rh.transpose(1, 2)), torch.matmul(q, rw.transpose(1, 2))


class QuantAttention(nn.Module):
    """Attention with fused rel-pos softmax (reference ``:83-149``)."""

    def __init__(self, qkv_proj, o_proj, num_heads, scale, use_rel_pos, rel_pos_h=None, rel_pos_w=None):
        super().__init__()
        self.qkv_proj = qkv_proj
        self.o_proj = o_proj
        self.num_heads = num_heads
        self.scale = scale
        self.rel_pos_h = rel_pos_h
        self.rel_pos_w = rel_pos_w
        self.use_rel_pos = use_rel_pos
        self.window_size = 0
        self._tables = {}

    def rel_tables(self, side: int):
        """fp16 relative-position tables of length 2*side-1 (interpolated like get_rel_pos)."""
        key = (side, self.rel_pos_h.data_ptr(), self.rel_pos_h._version, self.rel_pos_w._version)
        t = self._tables.get(side)
        if t is None or t[0] != key:
            def fit(tab):
                span = 2 * side - 1
                if tab.shape[0] != span:
                    tab = torch.nn.functional.interpolate(tab.float().t().unsqueeze(0), size=span,
                                                          mode="linear").squeeze(0).t()
                return tab.detach().to(torch.float16).contiguous()
            t = (key, fit(self.rel_pos_h), fit(self.rel_pos_w))
            self._tables[side] = t
        return t[1], t[2]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not self.use_rel_pos:
            raise NotImplementedError
        b, h, w, _ = x.shape
        assert h == w, "QuantAttention expects square token grids"
        qkv = self.qkv_proj(x)
        if qkv.dtype != torch.float16:
            qkv = qkv.half()
        relh, relw = self.rel_tables(h)
        o = ops.rel_attention(qkv.contiguous(), None, relh, relw, self.num_heads, 0, self.scale)
        return self.o_proj(o.to(x.dtype))


def forward(inp: torch.Tensor, pos_emb1: torch.Tensor, pos_emb2: torch.Tensor, head_num: int,
            hidden_dim: int, sm_scale: float) -> torch.Tensor:
    """Reference functional kernel entry (``:312-358``): softmax(q.k*s + rel_h + rel_w).v
    from the packed qkv tensor ``inp`` (B, h, w, 3*heads*hd) with precomputed bias tensors."""
    return ops.attention_relbias(inp, pos_emb1, pos_emb2, head_num, hidden_dim, sm_scale)

"""``gptq_triton.fused_mlp`` API on the HIP kernels (API parity).

The reference fuses ``silu(A . Wgate) * (A . Wup)`` for LLaMA MLPs (``fused_mlp.py``:
``make_fused_mlp`` ``:13-27``, ``autotune_warmup`` ``:30-71``, ``QuantLlamaMLP`` ``:74-112``,
``llama_mlp_fused_4_kernel`` ``:230-383``, ``triton_llama_mlp_4`` ``:391-477``).  SAM has no such
MLP (its ``make_fused_mlp`` even references an undefined ``LlamaMLP``); this module keeps the
names, arguments, buffers and asserts so code written against it runs, and fuses like the
reference: both int4 GEMMs and ``silu(g) * u`` in ONE launch (``samq_w4a16_gated_mlp``: the two
packed weights interleaved in 32-column blocks, so each wave tile holds a gate block and its up
block and the epilogue multiplies them in registers; exact integer weights, fp32 accumulate, G1
numerics).  Biases of gate/up are ignored, as in the reference kernel.
"""
from __future__ import annotations

import functools

import torch
import torch.nn as nn

from . import _lib, ops


def _gated_operands(gate_qweight, gate_scales, gate_qzeros, up_qweight, up_scales, up_qzeros):
    n = gate_qweight.shape[1]
    return ops.w4_interleave32(ops.w4_repack(gate_qweight), ops.w4_repack(up_qweight), gate_scales, up_scales,
                               gate_qzeros, up_qzeros, n)


def triton_llama_mlp_4(groupsize: int, a: torch.Tensor, gate_qweight: torch.Tensor, gate_scales: torch.Tensor,
                       gate_qzeros: torch.Tensor, up_qweight: torch.Tensor, up_scales: torch.Tensor,
                       up_qzeros: torch.Tensor, _operands=None) -> torch.Tensor:
    """``silu(gate(a)) * up(a)``, a (..., K) fp16 -> (..., N) fp16 (reference ``:391-477``): both
    int4 GEMMs and the gate product in one HIP launch (samq_w4a16_gated_mlp; ``_operands`` = the
    cached ``ops.w4_interleave32`` buffers of a ``QuantLlamaMLP``)."""
    assert (gate_qweight.shape == up_qweight.shape and gate_scales.shape == up_scales.shape
            and gate_qzeros.shape == up_qzeros.shape), "All weights must have the same shape"
    assert a.shape[-1] == gate_qweight.shape[0] * 8, "A must be a multiple of 8 in the last dimension"
    assert a.is_contiguous(), "A must be contiguous"
    k, n = a.shape[-1], gate_qweight.shape[1]
    assert k % 128 == 0, "K must be a multiple of 16, 32, 64, and 128"
    assert n % 256 == 0, "N must be a multiple of 16, 32, 64, 128, and 256"
    gs = k if groupsize == -1 else groupsize
    assert gs % 128 == 0, "groupsize must be a multiple of 32, 64, and 128"
    gs = -1 if gs == k else gs
    w2, s2, z2 = _operands if _operands is not None else _gated_operands(
        gate_qweight, gate_scales, gate_qzeros, up_qweight, up_scales, up_qzeros)
    return ops.w4a16_gated_mlp(a, w2, s2, z2, n, gs)


llama_mlp_4 = triton_llama_mlp_4


class QuantLlamaMLP(nn.Module):
    """``down_proj(silu(gate_proj(x)) * up_proj(x))`` with only the gate/up packed buffers kept
    (reference ``:74-112``)."""

    def __init__(self, gate_proj, down_proj, up_proj):
        super().__init__()
        assert gate_proj.groupsize == up_proj.groupsize
        self.register_buffer("gate_proj_qweight", gate_proj.qweight)
        self.register_buffer("gate_proj_scales", gate_proj.scales)
        self.register_buffer("gate_proj_qzeros", gate_proj.qzeros)
        self.register_buffer("up_proj_qweight", up_proj.qweight)
        self.register_buffer("up_proj_scales", up_proj.scales)
        self.register_buffer("up_proj_qzeros", up_proj.qzeros)
        self.groupsize = gate_proj.groupsize
        self.infeatures = gate_proj.infeatures
        self.outfeatures = down_proj.outfeatures
        self.down_proj = down_proj

    def gated_operands(self):
        """The interleaved gate/up operands of the fused kernel, built once and rebuilt when any of
        the six packed buffers moves or is written (data pointer / in-place version counter)."""
        bufs = (self.gate_proj_qweight, self.gate_proj_scales, self.gate_proj_qzeros, self.up_proj_qweight,
                self.up_proj_scales, self.up_proj_qzeros)
        key = tuple((b.data_ptr(), b._version) for b in bufs)
        if getattr(self, "_gated", None) is None or self._gated[0] != key:
            self._gated = (key, _gated_operands(self.gate_proj_qweight, self.gate_proj_scales, self.gate_proj_qzeros,
                                                self.up_proj_qweight, self.up_proj_scales, self.up_proj_qzeros))
        return self._gated[1]

    def forward(self, x):
        gs = -1 if self.groupsize == self.infeatures else self.groupsize
        return self.down_proj(triton_llama_mlp_4(gs, x, self.gate_proj_qweight, self.gate_proj_scales,
                                                 self.gate_proj_qzeros, self.up_proj_qweight, self.up_proj_scales,
                                                 self.up_proj_qzeros, _operands=self.gated_operands()))


def make_fused_mlp(m: nn.Module, parent_name: str = "") -> nn.Module:
    """Replace every LLaMA-style MLP (class named ``LlamaMLP`` with gate/up/down ``QuantLinear``)
    by ``QuantLlamaMLP`` (reference ``:13-27``)."""
    if type(m).__name__ == "LlamaMLP" and all(hasattr(m, a) for a in ("gate_proj", "up_proj", "down_proj")):
        return QuantLlamaMLP(m.gate_proj, m.down_proj, m.up_proj)
    for name, child in m.named_children():
        new = make_fused_mlp(child, parent_name=f"{parent_name}.{name}")
        if isinstance(new, QuantLlamaMLP):
            setattr(m, name, new)
    return m


def autotune_warmup(model: nn.Module):
    """One warm-up call per unique K (reference ``:30-71``); there is no autotuner."""
    mods = {m.infeatures: m for m in model.modules() if isinstance(m, QuantLlamaMLP)}
    print(f"FusedMLP Warmup: Found {len(mods)} unique K values.")

    def run(mrows, mod):
        a = torch.randn(1, mrows, mod.infeatures, dtype=torch.float16, device=mod.gate_proj_qweight.device)
        gs = -1 if mod.groupsize == mod.infeatures else mod.groupsize
        triton_llama_mlp_4(gs, a, mod.gate_proj_qweight, mod.gate_proj_scales, mod.gate_proj_qzeros,
                           mod.up_proj_qweight, mod.up_proj_scales, mod.up_proj_qzeros)

    return (functools.partial(run, mod=m) for m in mods.values())

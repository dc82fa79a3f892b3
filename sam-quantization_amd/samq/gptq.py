"""Producer side of the GPTQ int4 checkpoint format (RTN subset).

* ``Quantizer``      -- asymmetric per-channel min/max parameters (reference ``gptq.py:200-299``,
                        ``perchannel=True, sym=False``; ``mse`` grid search not used by the SAM scripts);
* ``pack_linear``    -- bit-identical to the reference's packing (``gptq4sam.py:434-497``),
                        vectorised in torch so it runs on the GPU in milliseconds per layer;
* ``quantize_rtn``   -- round-to-nearest quantisation of every encoder Linear -> QuantLinear;
* ``save_quant``     -- ``model.pt`` + ``quant_config.json`` exactly as ``gptq4sam.py:651-663`` writes.

The Hessian-based GPTQ update (``gptq.py:62-171``) is the remaining part of row f3.
"""
from __future__ import annotations

import json
import math
from pathlib import Path

import torch
import torch.nn as nn

from .quant_linear import QuantLinear, make_quant


class Quantizer:
    def __init__(self, bits: int = 4):
        self.maxq = 2 ** bits - 1

    def find_params(self, w: torch.Tensor):
        """Per-row ``scale, zero`` (fp32) for ``w`` (rows, cols)."""
        w = w.float()
        zero_t = torch.zeros(w.shape[0], device=w.device)
        xmin = torch.minimum(w.min(1).values, zero_t)
        xmax = torch.maximum(w.max(1).values, zero_t)
        both0 = (xmin == 0) & (xmax == 0)
        xmin = torch.where(both0, torch.full_like(xmin, -1), xmin)
        xmax = torch.where(both0, torch.full_like(xmax, 1), xmax)
        scale = (xmax - xmin) / self.maxq
        zero = torch.round(-xmin / scale)
        return scale, zero

    def quantize(self, w, scale, zero):
        q = torch.clamp(torch.round(w / scale) + zero, 0, self.maxq)
        return scale * (q - zero)


def rtn(w: torch.Tensor, groupsize: int = -1, bits: int = 4):
    """RTN fake quant of a Linear weight (N, K): ``(w_fake, scale (N,G), zero (N,G))``."""
    n, k = w.shape
    g = k if groupsize == -1 else groupsize
    qz = Quantizer(bits)
    fake = torch.empty_like(w, dtype=torch.float32)
    scales, zeros = [], []
    for s0 in range(0, k, g):
        blk = w[:, s0:s0 + g].float()
        s, z = qz.find_params(blk)
        fake[:, s0:s0 + g] = qz.quantize(blk, s[:, None], z[:, None])
        scales.append(s)
        zeros.append(z)
    return fake, torch.stack(scales, 1), torch.stack(zeros, 1)


def pack_linear(quant: QuantLinear, weight: torch.Tensor, scales: torch.Tensor, zeros: torch.Tensor,
                bias: torch.Tensor | None) -> None:
    """Fill ``quant``'s ``qweight/qzeros/scales/bias`` from a fake-quantised weight (N, K) and
    its ``scales/zeros`` (N, G), bit-identically to the reference ``pack_linear``."""
    dev = quant.qweight.device
    s_t = scales.t().contiguous().float().to(dev)      # (G, N)
    z_t = zeros.t().contiguous().float().to(dev)
    k = quant.infeatures
    gidx = torch.arange(k, device=dev) // quant.groupsize
    w = weight.to(dev)
    iw = torch.round((w.t() + (z_t * s_t)[gidx]) / s_t[gidx]).to(torch.int64)  # (K, N)
    qw = torch.zeros((k // 8, iw.shape[1]), dtype=torch.int64, device=dev)
    for j in range(8):
        qw |= iw[j::8] << (4 * j)
    zi = (z_t - 1).to(torch.int64)
    qz = torch.zeros((zi.shape[0], zi.shape[1] // 8), dtype=torch.int64, device=dev)
    for j in range(8):
        qz |= zi[:, j::8] << (4 * j)
    def to32(a):  # two's-complement wrap of the low 32 bits (int32 OR semantics of the reference)
        a = a & 0xFFFFFFFF
        return torch.where(a >= 2 ** 31, a - 2 ** 32, a).to(torch.int32)

    quant.qweight.copy_(to32(qw))
    quant.qzeros.copy_(to32(qz))
    quant.scales.copy_(s_t.to(torch.float16))
    if quant.bias is not None and bias is not None:
        quant.bias.copy_(bias.to(torch.float16))


@torch.no_grad()
def quantize_rtn(module: nn.Module, groupsize: int = -1, bits: int = 4, device=None) -> nn.Module:
    """Replace every ``nn.Linear`` of ``module`` by a packed ``QuantLinear`` (RTN weights)."""
    dense = {n: m for n, m in module.named_modules() if isinstance(m, nn.Linear)}
    make_quant(module, bits, groupsize)
    for name, m in module.named_modules():
        if isinstance(m, QuantLinear) and name in dense:
            lin = dense[name]
            if device is not None:
                m.to(device)
            w = lin.weight.detach().to(m.qweight.device).float()
            fake, s, z = rtn(w, groupsize, bits)
            pack_linear(m, fake, s, z, None if lin.bias is None else lin.bias.detach().to(m.qweight.device))
    return module


def save_quant(model: nn.Module, path, wbits: int = 4, groupsize: int = -1) -> None:
    """Write ``<path>/model.pt`` + ``<path>/quant_config.json`` (reference ``gptq4sam.py:651-663``)."""
    p = Path(path)
    p.mkdir(parents=True, exist_ok=True)
    torch.save({k: v.detach().cpu() for k, v in model.state_dict().items()}, p / "model.pt")
    (p / "quant_config.json").write_text(json.dumps({"wbits": wbits, "groupsize": groupsize}))


def num_groups(k: int, groupsize: int) -> int:
    return math.ceil(k / (k if groupsize == -1 else groupsize))

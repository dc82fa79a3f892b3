"""Producer side of the GPTQ int4 checkpoint format, on the GPU.

* ``Quantizer``      -- asymmetric per-channel min/max parameters (reference ``gptq.py:200-299``,
                        ``perchannel=True, sym=False``; ``mse`` grid search not used by the SAM scripts);
* ``GPTQ``           -- Hessian accumulation + the blockwise optimal-brain-quantiser update
                        (reference ``gptq.py:15-171``), in fp32 torch on the layer's device;
* ``sam_sequential`` -- the reference's block-by-block calibration of the SAM encoder
                        (``gptq4sam.py:280-431``, true-sequential groups qkv / proj / lin1+lin2);
* ``pack_linear``    -- bit-identical to the reference's packing (``gptq4sam.py:434-497``),
                        vectorised in torch so it runs on the GPU in milliseconds per layer;
* ``quantize_rtn`` / ``quantize_gptq`` -- RTN or GPTQ weights of every encoder Linear -> QuantLinear;
* ``save_quant``     -- ``model.pt`` + ``quant_config.json`` exactly as ``gptq4sam.py:651-663`` writes.
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


class GPTQ:
    """Second-order weight quantisation of one ``nn.Linear`` (reference ``gptq.py:15-171``).

    ``add_batch`` keeps H = 2/n sum x x^T as a running mean where, as in the reference's SAM
    variant, every call counts as ONE sample whatever its batch (``gptq.py:33-34``).
    ``fasterquant`` inverts the damped Hessian through Cholesky factors and quantises column by
    column inside blocks of ``blocksize``, pushing each column's scaled error onto the columns
    not yet quantised; group parameters are taken from the error-updated weights at each group
    start.  The layer's weight is replaced by the fake-quantised one; returns ``(scale, zero)``
    of shape (rows, groups).
    """

    def __init__(self, layer: nn.Module, bits: int = 4):
        self.layer = layer
        w = layer.weight.data
        self.rows, self.columns = w.shape[0], w[0].numel()
        self.dev = w.device
        self.H = torch.zeros((self.columns, self.columns), device=self.dev, dtype=torch.float32)
        self.nsamples = 0
        self.quantizer = Quantizer(bits)

    def add_batch(self, inp: torch.Tensor, out=None) -> None:
        x = inp.reshape(-1, inp.shape[-1]).t().float()          # (columns, tokens)
        self.H *= self.nsamples / (self.nsamples + 1)
        self.nsamples += 1
        x = math.sqrt(2.0 / self.nsamples) * x
        self.H += x @ x.t()

    @torch.no_grad()
    def fasterquant(self, blocksize: int = 128, percdamp: float = 0.01, groupsize: int = -1,
                    actorder: bool = False):
        W = self.layer.weight.data.clone().reshape(self.rows, -1).float()
        qz = self.quantizer
        scale, zero = qz.find_params(W)
        H = self.H
        self.H = None
        dead = torch.diagonal(H) == 0
        H[dead, dead] = 1.0
        W[:, dead] = 0.0
        perm = None
        if actorder:
            perm = torch.argsort(torch.diagonal(H), descending=True)
            W, H = W[:, perm], H[perm][:, perm]
        idx = torch.arange(self.columns, device=self.dev)
        H[idx, idx] += percdamp * torch.mean(torch.diagonal(H))
        L = torch.linalg.cholesky(H)
        Hinv = torch.linalg.cholesky(torch.cholesky_inverse(L), upper=True)
        Q = torch.zeros_like(W)
        scales, zeros = [], []
        for i1 in range(0, self.columns, blocksize):
            i2 = min(i1 + blocksize, self.columns)
            W1 = W[:, i1:i2].clone()
            Err1 = torch.zeros_like(W1)
            Hinv1 = Hinv[i1:i2, i1:i2]
            for i in range(i2 - i1):
                col = i1 + i
                if groupsize != -1 and col % groupsize == 0:
                    # the reference reads the OUTER W here: columns of the current block as of the
                    # block start, later columns as of the last block update (gptq.py:113-117)
                    scale, zero = qz.find_params(W[:, col:col + groupsize])
                    scales.append(scale)
                    zeros.append(zero)
                w = W1[:, i]
                q = qz.quantize(w, scale, zero)
                Q[:, col] = q
                err = (w - q) / Hinv1[i, i]
                W1[:, i:] -= err[:, None] * Hinv1[i, i:][None, :]
                Err1[:, i] = err
            W[:, i2:] -= Err1 @ Hinv[i1:i2, i2:]
        if perm is not None:
            Q = Q[:, torch.argsort(perm)]
        self.layer.weight.data = Q.reshape(self.layer.weight.shape).to(self.layer.weight.dtype)
        if not scales:
            scales, zeros = [scale], [zero]
        return torch.stack(scales, 1), torch.stack(zeros, 1)


@torch.no_grad()
def sam_sequential(encoder: nn.Module, images, groupsize: int = -1, percdamp: float = 0.01,
                   act_order: bool = False, true_sequential: bool = True, bits: int = 4) -> dict:
    """GPTQ-quantise every block Linear of a float SAM encoder, block by block, on calibration
    ``images`` (reference ``gptq4sam.py:280-431``).  Returns ``{name: (scale, zero)}``; the
    Linear weights are replaced by their fake-quantised values (pack with ``pack_gptq``)."""
    inps = []
    for img in images:
        x = encoder.patch_embed(img)
        if encoder.pos_embed is not None:
            x = x + encoder.pos_embed
        inps.append(x)
    groups = [["attn.qkv"], ["attn.proj"], ["mlp.lin1", "mlp.lin2"]] if true_sequential else None
    params = {}
    for bi, blk in enumerate(encoder.blocks):
        full = {n: m for n, m in blk.named_modules() if isinstance(m, nn.Linear)}
        for names in (groups or [list(full)]):
            g = {n: GPTQ(full[n], bits) for n in names}
            hooks = [full[n].register_forward_hook(lambda m, i, o, n=n: g[n].add_batch(i[0].data))
                     for n in names]
            for x in inps:
                blk(x)
            for h in hooks:
                h.remove()
            for n in names:
                params[f"blocks.{bi}.{n}"] = g[n].fasterquant(percdamp=percdamp, groupsize=groupsize,
                                                              actorder=act_order)
        inps = [blk(x) for x in inps]
    return params


@torch.no_grad()
def pack_gptq(encoder: nn.Module, params: dict, groupsize: int = -1, bits: int = 4) -> nn.Module:
    """``sam_pack`` (reference ``gptq4sam.py:434-451``): swap the calibrated Linears for packed
    ``QuantLinear`` (bit-identical packing of the fake-quantised weights and their scale / zero)."""
    dense = {n: m for n, m in encoder.named_modules() if isinstance(m, nn.Linear) and n in params}
    make_quant(encoder, bits, groupsize)
    for name, m in encoder.named_modules():
        if isinstance(m, QuantLinear) and name in dense:
            lin = dense[name]
            m.to(lin.weight.device)
            s, z = params[name]
            pack_linear(m, lin.weight.detach().float(), s, z, None if lin.bias is None else lin.bias.detach())
    return encoder


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

"""fq_vit W8A8 fake-quant restatement of the SAM image encoder (oracle F).

TEST INFRASTRUCTURE (oracle) -- see ``oracle/__init__.py``.

Semantics restated (configuration of ``quant_fq-vit.sh:1`` / ``fq_vit/test_quant.py:229-231``:
``Config(ptf=False, lis=False, quant_method='minmax')`` then ``cfg.BIT_TYPE_A = int8``):

* weights (``QLinear`` ``fq_vit/models/ptq/layers.py:160-200``, ``QConv2d`` ``:11-74``):
  int8, symmetric, per output channel, ``MinmaxObserver`` (``observer/minmax.py:14-50``):
  ``s = max(-min, max) / 127.5`` clamped at fp32 eps, zero point 0;
* activations (``QAct`` ``layers.py:203-242``): int8 symmetric, layer-wise (one scalar per
  QAct), min/max accumulated over every calibration forward;
* fake quant (``quantizer/uniform.py:23-45``): ``(clamp(round(x / s + zp), lo, hi) - zp) * s``
  with a TRUE division and round-half-to-even;
* ``QIntLayerNorm`` / ``QIntSoftmax`` / ``QIntLayerNorm2D`` return the float op on their first
  line (``layers.py:258, 379``, ``fq_vit/models/sam/common.py:108``): plain LayerNorm (eps 1e-6
  in blocks, **1e-5** in the neck), plain softmax, no softmax quantiser;
* the 11 per-block activation quantisers and their positions follow
  ``fq_vit/models/sam/image_encoder.py:310-331`` (Block), ``:437-478`` (Attention),
  ``common.py:65-73`` (MLPBlock); the 4 encoder-level ones ``:192-213``; the neck's 4 ``:207-211``.

QAct names mirror the fq_vit module paths so the scales can be compared key-by-key with the
reference's ``quantizer.scale`` buffers.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .sam_ref import rel_bias, window_partition, window_unpartition, layernorm2d, _t

EPS32 = torch.finfo(torch.float32).eps
QLO, QHI = -128.0, 127.0


def sym_scale(vmin: torch.Tensor, vmax: torch.Tensor) -> torch.Tensor:
    """``MinmaxObserver.get_quantization_params`` symmetric branch (``minmax.py:41-44``)."""
    return (torch.max(-vmin, vmax) / ((QHI - QLO) / 2)).clamp(min=EPS32)


def fake_quant(x: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    """``UniformQuantizer.quant`` + ``dequantize`` with zero point 0 (``uniform.py:23-45``)."""
    return torch.clamp(torch.round(x / s), QLO, QHI) * s


def weight_fake_quant(w: torch.Tensor):
    """Per-output-channel symmetric int8 fake quant; returns ``(w_fq, s (out,), q int8)``."""
    flat = w.reshape(w.shape[0], -1)
    s = sym_scale(flat.min(dim=1).values, flat.max(dim=1).values)
    shape = (-1,) + (1,) * (w.dim() - 1)
    q = torch.clamp(torch.round(w / s.reshape(shape)), QLO, QHI)
    return q * s.reshape(shape), s, q.to(torch.int8)


class FQEncoderOracle:
    """W8A8 fake-quant SAM encoder (fp32 CPU).  Usage::

        o = FQEncoderOracle(cfg, state)
        o.calibrate([img0, img1])       # float forwards, observers accumulate
        out = o(img)                    # quant forward
    """

    WEIGHTS = ("patch_embed.proj", "neck.0", "neck.2")

    def __init__(self, cfg: dict, state: dict, dtype: torch.dtype = torch.float32):
        # dtype float64: the same fake-quant function evaluated with (nearly) exact arithmetic --
        # used by the tests to measure how far fp32 rounding alone moves the reference's codes
        self.cfg = cfg
        self.dtype = dtype
        self.p = {k: _t(v, dtype) for k, v in state.items()}
        self.minmax: dict[str, tuple[torch.Tensor, torch.Tensor]] = {}
        self.scales: dict[str, torch.Tensor] = {}
        self.mode = "float"  # "float" | "calib" | "quant"
        # weight fake quant is data independent: observer sees the same weight every call
        self.wq: dict[str, torch.Tensor] = {}
        self.wscale: dict[str, torch.Tensor] = {}
        names = list(self.WEIGHTS) + [f"blocks.{i}.{s}" for i in range(cfg["depth"])
                                      for s in ("attn.qkv", "attn.proj", "mlp.lin1", "mlp.lin2")]
        for n in names:
            wfq, s, _ = weight_fake_quant(self.p[n + ".weight"].float())   # fp32 scales (the model's)
            self.wq[n], self.wscale[n] = wfq.to(dtype), s

    # -- activation quantiser points ------------------------------------------------------
    def qact(self, name: str, x: torch.Tensor) -> torch.Tensor:
        if self.mode == "calib":
            lo, hi = x.min(), x.max()
            if name in self.minmax:
                plo, phi = self.minmax[name]
                lo, hi = torch.minimum(lo, plo), torch.maximum(hi, phi)
            self.minmax[name] = (lo, hi)
            return x
        if self.mode == "quant":
            return fake_quant(x, self.scales[name])
        return x

    def w(self, name: str) -> torch.Tensor:
        return self.wq[name] if self.mode == "quant" else self.p[name + ".weight"]

    def finalize(self):
        self.scales = {k: sym_scale(lo, hi) for k, (lo, hi) in self.minmax.items()}

    def set_scales(self, scales: dict) -> None:
        """Use calibrated activation scales (e.g. the reference's ``quantizer.scale`` buffers)."""
        self.scales = {k: torch.tensor(float(v), dtype=torch.float32).to(self.dtype) for k, v in scales.items()}
        self.mode = "quant"

    # -- graph -----------------------------------------------------------------------------
    def attention(self, pre: str, x: torch.Tensor) -> torch.Tensor:
        p, heads = self.p, self.cfg["num_heads"]
        bq, h, w, c = x.shape
        d = c // heads
        qkv = F.linear(x.reshape(bq, h * w, c), self.w(pre + "qkv"), p[pre + "qkv.bias"])
        qkv = self.qact(pre + "qact1", qkv)
        qkv = qkv.reshape(bq, h * w, 3, heads, d).permute(2, 0, 3, 1, 4)
        q, k, v = qkv.reshape(3, bq * heads, h * w, d).unbind(0)
        scores = (q * (d ** -0.5)) @ k.transpose(-2, -1)
        scores = self.qact(pre + "qact_attn1", scores)
        rel_h, rel_w = rel_bias(q.reshape(bq * heads, h, w, d), p[pre + "rel_pos_h"],
                                p[pre + "rel_pos_w"], h, w)
        scores = (scores.view(bq * heads, h, w, h, w) + rel_h[..., :, None]
                  + rel_w[..., None, :]).view(bq * heads, h * w, h * w)
        scores = self.qact(pre + "use_rel_pos_qact", scores)
        probs = F.softmax(scores, dim=-1)
        o = (probs @ v).view(bq, heads, h, w, d).permute(0, 2, 3, 1, 4).reshape(bq, h, w, c)
        o = self.qact(pre + "qact2", o)
        o = F.linear(o, self.w(pre + "proj"), p[pre + "proj.bias"])
        return self.qact(pre + "qact3", o)

    def block(self, i: int, x: torch.Tensor) -> torch.Tensor:
        p, cfg = self.p, self.cfg
        pre = f"blocks.{i}."
        c = cfg["embed_dim"]
        win = 0 if i in cfg["global_attn_indexes"] else cfg["window_size"]
        shortcut = x
        y = self.qact(pre + "qact1", F.layer_norm(x, (c,), p[pre + "norm1.weight"],
                                                   p[pre + "norm1.bias"], eps=1e-6))
        h, w = y.shape[1], y.shape[2]
        if win > 0:
            y, pad_hw = window_partition(y, win)
        y = self.attention(pre + "attn.", y)
        if win > 0:
            y = window_unpartition(y, win, pad_hw, (h, w))
        x = self.qact(pre + "qact2", shortcut + y)
        z = self.qact(pre + "qact3", F.layer_norm(x, (c,), p[pre + "norm2.weight"],
                                                   p[pre + "norm2.bias"], eps=1e-6))
        z = F.gelu(F.linear(z, self.w(pre + "mlp.lin1"), p[pre + "mlp.lin1.bias"]))
        z = self.qact(pre + "mlp.qact1", z)
        z = self.qact(pre + "mlp.qact2", F.linear(z, self.w(pre + "mlp.lin2"), p[pre + "mlp.lin2.bias"]))
        return self.qact(pre + "qact4", x + z)

    @torch.no_grad()
    def forward(self, img) -> torch.Tensor:
        p, cfg = self.p, self.cfg
        x = self.qact("qact_input", _t(img, self.dtype))
        x = F.conv2d(x, self.w("patch_embed.proj"), p["patch_embed.proj.bias"], stride=cfg["patch_size"])
        x = self.qact("patch_embed.qact", x).permute(0, 2, 3, 1)
        x = x + self.qact("qact_pos", p["pos_embed"])
        x = self.qact("qact1", x)
        for i in range(cfg["depth"]):
            x = self.block(i, x)
        y = x.permute(0, 3, 1, 2)
        y = self.qact("qacts.0", F.conv2d(y, self.w("neck.0")))
        y = self.qact("qacts.1", layernorm2d(y, p["neck.1.weight"], p["neck.1.bias"], eps=1e-5))
        y = self.qact("qacts.2", F.conv2d(y, self.w("neck.2"), padding=1))
        return self.qact("qacts.3", layernorm2d(y, p["neck.3.weight"], p["neck.3.bias"], eps=1e-5))

    @torch.no_grad()
    def calibrate(self, images) -> None:
        """``model_open_calibrate`` .. ``model_close_calibrate`` (``test_quant.py:284-294``)."""
        self.mode = "calib"
        for img in images:
            self.forward(img)
        self.finalize()
        self.mode = "quant"

    def __call__(self, img):
        return self.forward(img)

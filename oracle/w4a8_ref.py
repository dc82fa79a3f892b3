"""W4A8 oracle: GPTQ int4 weights x fq_vit int8 activations (SURVEY.md §8c "Oracle W4A8").

TEST INFRASTRUCTURE (oracle) -- see ``oracle/__init__.py``.

No single reference path runs int4 weights with int8 activations, so (as the survey prescribes)
this oracle is a COMPOSITION of two reference pieces:

* the W4 fake-quant encoder of oracle G1 (``sam_ref.EncoderOracle`` with the GPTQ-packed
  weights decoded as ``s * (q - (z + 1))``, ``gptq_triton/quant_linear.py:292-313``);
* an fq_vit ``QAct`` (``fq_vit/models/ptq/layers.py:203-242``) in front of every QuantLinear:
  int8 symmetric, layer-wise ``MinmaxObserver`` (``observer/minmax.py:14-50``) and the uniform
  fake quantiser ``clamp(round(x / s), -128, 127) * s`` (``quantizer/uniform.py:23-45``).

Calibration: float forwards of the W4 model with the observers on each Linear input (the fq_vit
calibrate mode returns the unquantised input, ``layers.py:232-239``); padded window tokens are
part of the observed tensors exactly as in the reference graph.  Parity of this composition is
therefore pinned only through its two pinned halves (G1 goldens, fq_vit goldens).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .fq_ref import fake_quant, sym_scale
from .sam_ref import EncoderOracle, attention_core, window_partition, window_unpartition


class W4A8EncoderOracle(EncoderOracle):
    """``EncoderOracle`` (G1 weights) with int8 fake quant on the input of every block Linear.
    Scale names are the Linear paths: ``blocks.{i}.attn.qkv`` / ``.attn.proj`` / ``.mlp.lin1`` /
    ``.mlp.lin2``."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.mode = "float"      # "float" | "calib" | "quant"
        self.minmax: dict = {}
        self.scales: dict = {}

    def qin(self, name: str, x: torch.Tensor) -> torch.Tensor:
        if self.mode == "calib":
            lo, hi = x.min(), x.max()
            if name in self.minmax:
                lo, hi = torch.minimum(lo, self.minmax[name][0]), torch.maximum(hi, self.minmax[name][1])
            self.minmax[name] = (lo, hi)
            return x
        if self.mode == "quant":
            return fake_quant(x, self.scales[name].to(x.dtype))
        return x

    def block(self, i: int, x: torch.Tensor) -> torch.Tensor:
        return self.block_taps(i, x)["out"]

    def block_taps(self, i: int, x: torch.Tensor) -> dict:
        """One block with every intermediate recorded (the stage-local parity taps): ``ln1`` /
        ``ln2`` the LayerNorm outputs (natural token layout, before the int8 quantiser), ``qkv``
        the qkv projection and ``att`` the attention output (natural layout: window padding
        cropped), ``x1`` the residual after proj, ``h`` GELU(lin1), ``out`` the block output."""
        cfg, p = self.cfg, self.p
        pre = f"blocks.{i}."
        c = cfg["embed_dim"]
        win = 0 if i in cfg["global_attn_indexes"] else cfg["window_size"]
        t = {"x": x}
        y = F.layer_norm(x, (c,), p[pre + "norm1.weight"], p[pre + "norm1.bias"], eps=1e-6)
        t["ln1"] = y
        h, w = y.shape[1], y.shape[2]
        if win > 0:
            y, pad_hw = window_partition(y, win)
        qkv = F.linear(self.qin(pre + "attn.qkv", y), p[pre + "attn.qkv.weight"], p.get(pre + "attn.qkv.bias"))
        o = attention_core(qkv, cfg["num_heads"], p[pre + "attn.rel_pos_h"], p[pre + "attn.rel_pos_w"])
        t["qkv"] = window_unpartition(qkv, win, pad_hw, (h, w)) if win > 0 else qkv
        t["att"] = window_unpartition(o, win, pad_hw, (h, w)) if win > 0 else o
        y = F.linear(self.qin(pre + "attn.proj", o), p[pre + "attn.proj.weight"], p.get(pre + "attn.proj.bias"))
        if win > 0:
            y = window_unpartition(y, win, pad_hw, (h, w))
        x = x + y
        t["x1"] = x
        z = F.layer_norm(x, (c,), p[pre + "norm2.weight"], p[pre + "norm2.bias"], eps=1e-6)
        t["ln2"] = z
        z = F.gelu(F.linear(self.qin(pre + "mlp.lin1", z), p[pre + "mlp.lin1.weight"], p.get(pre + "mlp.lin1.bias")))
        t["h"] = z
        z = F.linear(self.qin(pre + "mlp.lin2", z), p[pre + "mlp.lin2.weight"], p.get(pre + "mlp.lin2.bias"))
        t["out"] = x + z
        return t

    def attention(self, i: int, qkv: torch.Tensor) -> torch.Tensor:
        """The block-``i`` attention core on a natural-layout qkv (windowed blocks partition it
        with the pad tokens' q/k/v = the qkv bias, which is what the zero-padded LN output
        projects to), cropped back to the natural layout."""
        cfg, p = self.cfg, self.p
        pre = f"blocks.{i}."
        win = 0 if i in cfg["global_attn_indexes"] else cfg["window_size"]
        h, w = qkv.shape[1], qkv.shape[2]
        if win > 0:
            bias = p.get(pre + "attn.qkv.bias")
            real, _ = window_partition(torch.ones_like(qkv[..., :1]), win)
            qkv, pad_hw = window_partition(qkv, win)
            if bias is not None:
                qkv = torch.where(real > 0, qkv, bias.to(qkv.dtype))
        o = attention_core(qkv, cfg["num_heads"], p[pre + "attn.rel_pos_h"], p[pre + "attn.rel_pos_w"])
        return window_unpartition(o, win, pad_hw, (h, w)) if win > 0 else o

    @torch.no_grad()
    def calibrate(self, images) -> None:
        self.mode = "calib"
        for img in images:
            self(img)
        self.scales = {k: sym_scale(lo, hi) for k, (lo, hi) in self.minmax.items()}
        self.mode = "quant"

    def set_scales(self, scales: dict) -> None:
        self.scales = {k: torch.tensor(float(v), dtype=torch.float32) for k, v in scales.items()}
        self.mode = "quant"

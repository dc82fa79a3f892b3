"""fp32 / fp16 CPU restatement of the SAM ViT image encoder (oracles G1 and G2).

TEST INFRASTRUCTURE (oracle) -- see ``oracle/__init__.py``.

Restates ``segment_anything/modeling/image_encoder.py`` (``ImageEncoderViT.forward``
``:106-118``, ``Block.forward`` ``:189-207``, ``Attention.forward`` ``:243-265``,
``get_rel_pos`` ``:336-366``, ``add_decomposed_rel_pos`` ``:369-408``, ``PatchEmbed``
``:411-442``), ``common.py`` (``MLPBlock`` ``:13-27`` exact-erf GELU, ``LayerNorm2d``
``:31-43`` eps 1e-6) with two deliberate differences from that file:

* windowing is batch- and size-generic (as ``fq_vit/models/sam/image_encoder.py:481-536``)
  instead of the hard-coded ``B=1, 64x64, pad 6, C=1280`` of ``image_encoder.py:297-328``
  (identical results wherever the hard-coded version runs);
* nothing else: in particular the relative-position term keeps the reference's
  indexing ``rel_w[b,h,w,k] = sum_c q[b,h,w,c] * Rw[h,k,c]`` -- the table row follows the
  query ROW ``h`` (quirk 1, ``image_encoder.py:402``, ``fused_attention.py:78``).

``precision="fp32"`` is oracle G1 (the "CPU fake-quant path"): every op in fp32, quantised
Linear weights given as dequantised fp32 ``s*(q-zp)``.  ``precision="fp16"`` is the
fp16-faithful dataflow of the reference's GPU path (``gptq4sam_infer.py:218`` ``.half()``)
and, with ``oracle.gptq_pack.dequant_g2`` weights, oracle G2.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from . import gptq_pack


def _t(x, dtype):
    if isinstance(x, np.ndarray):
        x = torch.from_numpy(np.ascontiguousarray(x))
    return x.to(dtype)


def rel_pos_table(q_size: int, k_size: int, table: torch.Tensor) -> torch.Tensor:
    """(q_size, k_size, C) gathered relative-position rows (``get_rel_pos``, ``:336-366``)."""
    span = int(2 * max(q_size, k_size) - 1)
    if table.shape[0] != span:
        t = F.interpolate(table.t().unsqueeze(0).float(), size=span, mode="linear")
        table = t.squeeze(0).t().to(table.dtype)
    qf = max(k_size / q_size, 1.0)
    kf = max(q_size / k_size, 1.0)
    qi = torch.arange(q_size)[:, None] * qf
    ki = torch.arange(k_size)[None, :] * kf
    idx = (qi - ki) + (k_size - 1) * kf
    return table[idx.long()]


def rel_bias(q: torch.Tensor, rel_pos_h, rel_pos_w, side_h: int, side_w: int):
    """Decomposed relative-position terms, quirk-1 indexing.

    q: (B', h, w, d)  ->  rel_h (B', h, w, kh), rel_w (B', h, w, kw) with
    ``rel_h[..,i,j,k] = q[..,i,j,:] . Rh[i,k,:]`` and ``rel_w[..,i,j,k] = q[..,i,j,:] . Rw[i,k,:]``.
    """
    rh = rel_pos_table(side_h, side_h, rel_pos_h)  # (h, kh, d)
    rw = rel_pos_table(side_w, side_w, rel_pos_w)  # (w, kw, d) -- indexed by ROW i below
    rel_h = torch.einsum("bijd,ikd->bijk", q, rh)
    rel_w = torch.einsum("bijd,ikd->bijk", q, rw)
    return rel_h, rel_w


def attention(x, qkv_w, qkv_b, proj_w, proj_b, heads: int, rel_pos_h, rel_pos_w):
    """Multi-head attention with decomposed rel-pos; x: (B', h, w, C)."""
    o = attention_core(F.linear(x, qkv_w, qkv_b), heads, rel_pos_h, rel_pos_w)
    return F.linear(o, proj_w, proj_b)


def attention_core(qkv, heads: int, rel_pos_h, rel_pos_w):
    """softmax(q.k*scale + rel_h + rel_w).v from the qkv projection (B', h, w, 3C) -> (B', h, w, C)
    (``Attention.forward`` ``:243-265`` minus the two Linears)."""
    bq, h, w, c3 = qkv.shape
    c = c3 // 3
    d = c // heads
    qkv = qkv.reshape(bq, h * w, 3, heads, d).permute(2, 0, 3, 1, 4)
    q, k, v = qkv.reshape(3, bq * heads, h * w, d).unbind(0)
    scores = (q * (d ** -0.5)) @ k.transpose(-2, -1)
    rel_h, rel_w = rel_bias(q.reshape(bq * heads, h, w, d), rel_pos_h, rel_pos_w, h, w)
    scores = (scores.view(bq * heads, h, w, h, w) + rel_h[..., :, None] + rel_w[..., None, :])
    scores = scores.view(bq * heads, h * w, h * w)
    probs = scores.softmax(dim=-1)
    return (probs @ v).view(bq, heads, h, w, d).permute(0, 2, 3, 1, 4).reshape(bq, h, w, c)


def window_partition(x: torch.Tensor, win: int):
    b, h, w, c = x.shape
    ph, pw = (-h) % win, (-w) % win
    if ph or pw:
        x = F.pad(x, (0, 0, 0, pw, 0, ph))
    hp, wp = h + ph, w + pw
    x = x.view(b, hp // win, win, wp // win, win, c).permute(0, 1, 3, 2, 4, 5)
    return x.reshape(-1, win, win, c), (hp, wp)


def window_unpartition(xw: torch.Tensor, win: int, hp_wp, hw):
    hp, wp = hp_wp
    h, w = hw
    b = xw.shape[0] // ((hp // win) * (wp // win))
    x = xw.view(b, hp // win, wp // win, win, win, -1).permute(0, 1, 3, 2, 4, 5)
    x = x.reshape(b, hp, wp, -1)
    return x[:, :h, :w, :]


def layernorm2d(x, weight, bias, eps=1e-6):
    mu = x.mean(1, keepdim=True)
    var = (x - mu).pow(2).mean(1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * weight[:, None, None] + bias[:, None, None]


class EncoderOracle:
    """Functional SAM ``ImageEncoderViT`` on CPU.

    ``state``: numpy/torch state dict with reference key names (``oracle.synth``).
    ``linear_weights``: optional ``{name: W (out,in)}`` overriding ``<name>.weight`` (e.g.
    dequantised GPTQ weights); ``linear_bias``: optional override of biases.
    """

    def __init__(self, cfg: dict, state: dict, precision: str = "fp32",
                 linear_weights: dict | None = None, linear_bias: dict | None = None):
        self.cfg = cfg
        self.dtype = {"fp32": torch.float32, "fp16": torch.float16, "fp64": torch.float64}[precision]
        self.p = {k: _t(v, self.dtype) for k, v in state.items()}
        for name, wt in (linear_weights or {}).items():
            self.p[name + ".weight"] = _t(wt, self.dtype)
        for name, bt in (linear_bias or {}).items():
            self.p[name + ".bias"] = None if bt is None else _t(bt, self.dtype)

    def block(self, i: int, x: torch.Tensor) -> torch.Tensor:
        cfg, p = self.cfg, self.p
        pre = f"blocks.{i}."
        c = cfg["embed_dim"]
        win = 0 if i in cfg["global_attn_indexes"] else cfg["window_size"]
        shortcut = x
        y = F.layer_norm(x, (c,), p[pre + "norm1.weight"], p[pre + "norm1.bias"], eps=1e-6)
        h, w = y.shape[1], y.shape[2]
        if win > 0:
            y, pad_hw = window_partition(y, win)
        y = attention(y, p[pre + "attn.qkv.weight"], p.get(pre + "attn.qkv.bias"),
                      p[pre + "attn.proj.weight"], p.get(pre + "attn.proj.bias"),
                      cfg["num_heads"], p[pre + "attn.rel_pos_h"], p[pre + "attn.rel_pos_w"])
        if win > 0:
            y = window_unpartition(y, win, pad_hw, (h, w))
        x = shortcut + y
        z = F.layer_norm(x, (c,), p[pre + "norm2.weight"], p[pre + "norm2.bias"], eps=1e-6)
        z = F.linear(z, p[pre + "mlp.lin1.weight"], p.get(pre + "mlp.lin1.bias"))
        z = F.gelu(z)
        z = F.linear(z, p[pre + "mlp.lin2.weight"], p.get(pre + "mlp.lin2.bias"))
        return x + z

    def embed(self, img: torch.Tensor) -> torch.Tensor:
        p = self.p
        x = F.conv2d(img, p["patch_embed.proj.weight"], p["patch_embed.proj.bias"],
                     stride=self.cfg["patch_size"])
        return x.permute(0, 2, 3, 1) + p["pos_embed"]

    def neck(self, x: torch.Tensor) -> torch.Tensor:
        p = self.p
        y = F.conv2d(x.permute(0, 3, 1, 2), p["neck.0.weight"])
        y = layernorm2d(y, p["neck.1.weight"], p["neck.1.bias"])
        y = F.conv2d(y, p["neck.2.weight"], padding=1)
        return layernorm2d(y, p["neck.3.weight"], p["neck.3.bias"])

    @torch.no_grad()
    def __call__(self, img, return_tokens: bool = False):
        x = self.embed(_t(img, self.dtype))
        for i in range(self.cfg["depth"]):
            x = self.block(i, x)
        out = self.neck(x)
        return (out, x) if return_tokens else out


def quantized_linear_weights(qstate: dict, names, groupsize: int, mode: str = "g1") -> dict:
    """Dequantise ``{name.qweight, name.qzeros, name.scales}`` into ``{name: W (out,in)}``."""
    fn = {"g1": gptq_pack.dequant_g1, "g2": gptq_pack.dequant_g2}[mode]
    return {n: fn(qstate[n + ".qweight"], qstate[n + ".scales"], qstate[n + ".qzeros"], groupsize).T
            for n in names}


def quantize_encoder_state(state: dict, names, groupsize: int = -1):
    """RTN-quantise + pack every Linear in ``names`` (numpy).  Returns the packed
    ``{name.qweight, name.qzeros, name.scales, name.bias(fp16)}`` dict."""
    out = {}
    for n in names:
        w = state[n + ".weight"]
        fake, s, z = gptq_pack.rtn_quantize_linear(w, groupsize)
        qw, qz, sc = gptq_pack.pack_linear(fake, s, z, groupsize)
        out[n + ".qweight"], out[n + ".qzeros"], out[n + ".scales"] = qw, qz, sc
        out[n + ".bias"] = np.asarray(state[n + ".bias"], np.float16)
    return out


def gelu_erf(x):
    return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))

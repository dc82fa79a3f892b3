"""SAM ViT image encoder module tree (host side of the hot path).

Module names, constructor arguments and ``state_dict`` keys follow the reference's
``segment_anything/modeling/image_encoder.py`` (``ImageEncoderViT`` ``:17-118``, ``Block``
``:141-207``, ``Attention`` ``:210-265``, ``PatchEmbed`` ``:411-442``) and ``common.py``
(``MLPBlock``, ``LayerNorm2d``), so reference checkpoints (``model.pt``) load unchanged and
``make_quant`` / ``make_quant_attn`` find the same ``nn.Linear`` / ``Attention`` slots.

Behavioural notes:
* windowing is batch- and size-generic (the reference hard-codes B=1 / 64x64 / C=1280,
  ``image_encoder.py:297-328``; results are identical wherever that version runs);
* the relative-position width term keeps the reference's query-ROW table indexing (quirk 1);
* once the encoder is quantized (``load_quant``) and on a GPU, ``ImageEncoderViT.forward``
  runs the fused HIP engine (``samq.engine``); the plain module forward below is the float
  model (used before quantization, e.g. for calibration), not the hot path.
"""
from __future__ import annotations

from typing import Optional, Tuple, Type

import torch
import torch.nn as nn
import torch.nn.functional as F


class MLPBlock(nn.Module):
    def __init__(self, embedding_dim: int, mlp_dim: int, act: Type[nn.Module] = nn.GELU):
        super().__init__()
        self.lin1 = nn.Linear(embedding_dim, mlp_dim)
        self.lin2 = nn.Linear(mlp_dim, embedding_dim)
        self.act = act()

    def forward(self, x):
        return self.lin2(self.act(self.lin1(x)))


class LayerNorm2d(nn.Module):
    def __init__(self, num_channels: int, eps: float = 1e-6):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(num_channels))
        self.bias = nn.Parameter(torch.zeros(num_channels))
        self.eps = eps

    def forward(self, x):
        mu = x.mean(1, keepdim=True)
        var = (x - mu).pow(2).mean(1, keepdim=True)
        return (x - mu) * torch.rsqrt(var + self.eps) * self.weight[:, None, None] + self.bias[:, None, None]


def get_rel_pos(q_size: int, k_size: int, rel_pos: torch.Tensor) -> torch.Tensor:
    """(q_size, k_size, C) relative-position rows, linearly resampled if the table length
    differs from 2*max(q,k)-1 (reference ``image_encoder.py:336-366``)."""
    span = int(2 * max(q_size, k_size) - 1)
    if rel_pos.shape[0] != span:
        t = F.interpolate(rel_pos.reshape(1, rel_pos.shape[0], -1).permute(0, 2, 1), size=span, mode="linear")
        rel_pos = t.reshape(-1, span).permute(1, 0)
    qf, kf = max(k_size / q_size, 1.0), max(q_size / k_size, 1.0)
    coords = (torch.arange(q_size, device=rel_pos.device)[:, None] * qf
              - torch.arange(k_size, device=rel_pos.device)[None, :] * kf + (k_size - 1) * kf)
    return rel_pos[coords.long()]


def window_partition(x: torch.Tensor, window_size: int):
    b, h, w, c = x.shape
    ph, pw = (-h) % window_size, (-w) % window_size
    if ph or pw:
        x = F.pad(x, (0, 0, 0, pw, 0, ph))
    hp, wp = h + ph, w + pw
    x = x.view(b, hp // window_size, window_size, wp // window_size, window_size, c)
    return x.permute(0, 1, 3, 2, 4, 5).reshape(-1, window_size, window_size, c), (hp, wp)


def window_unpartition(windows: torch.Tensor, window_size: int, pad_hw, hw) -> torch.Tensor:
    hp, wp = pad_hw
    h, w = hw
    b = windows.shape[0] // ((hp // window_size) * (wp // window_size))
    x = windows.view(b, hp // window_size, wp // window_size, window_size, window_size, -1)
    x = x.permute(0, 1, 3, 2, 4, 5).reshape(b, hp, wp, -1)
    return x[:, :h, :w, :].contiguous()


class Attention(nn.Module):
    def __init__(self, dim: int, num_heads: int = 8, qkv_bias: bool = True, use_rel_pos: bool = False,
                 rel_pos_zero_init: bool = True, input_size: Optional[Tuple[int, int]] = None):
        super().__init__()
        self.num_heads = num_heads
        self.scale = (dim // num_heads) ** -0.5
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.proj = nn.Linear(dim, dim)
        self.use_rel_pos = use_rel_pos
        if use_rel_pos:
            assert input_size is not None, "Input size must be provided if using relative positional encoding."
            self.rel_pos_h = nn.Parameter(torch.zeros(2 * input_size[0] - 1, dim // num_heads))
            self.rel_pos_w = nn.Parameter(torch.zeros(2 * input_size[1] - 1, dim // num_heads))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        b, h, w, c = x.shape
        nh = self.num_heads
        d = c // nh
        qkv = self.qkv(x).reshape(b, h * w, 3, nh, d).permute(2, 0, 3, 1, 4).reshape(3, b * nh, h * w, d)
        q, k, v = qkv.unbind(0)
        attn = (q * self.scale) @ k.transpose(-2, -1)
        if self.use_rel_pos:
            rh = get_rel_pos(h, h, self.rel_pos_h)
            rw = get_rel_pos(w, w, self.rel_pos_w)
            rq = q.reshape(b * nh, h, w, d)
            rel_h = torch.einsum("bijd,ikd->bijk", rq, rh)
            rel_w = torch.einsum("bijd,ikd->bijk", rq, rw)  # query-row indexing (reference quirk)
            attn = (attn.view(b * nh, h, w, h, w) + rel_h[..., :, None] + rel_w[..., None, :]).view(b * nh, h * w, h * w)
        attn = attn.softmax(dim=-1)
        x = (attn @ v).view(b, nh, h, w, d).permute(0, 2, 3, 1, 4).reshape(b, h, w, c)
        return self.proj(x)


class Block(nn.Module):
    def __init__(self, dim: int, num_heads: int, mlp_ratio: float = 4.0, qkv_bias: bool = True,
                 norm_layer: Type[nn.Module] = nn.LayerNorm, act_layer: Type[nn.Module] = nn.GELU,
                 use_rel_pos: bool = False, rel_pos_zero_init: bool = True, window_size: int = 0,
                 input_size: Optional[Tuple[int, int]] = None):
        super().__init__()
        self.norm1 = norm_layer(dim)
        self.attn = Attention(dim, num_heads=num_heads, qkv_bias=qkv_bias, use_rel_pos=use_rel_pos,
                              rel_pos_zero_init=rel_pos_zero_init,
                              input_size=input_size if window_size == 0 else (window_size, window_size))
        self.attn.window_size = window_size
        self.norm2 = norm_layer(dim)
        self.mlp = MLPBlock(dim, int(dim * mlp_ratio), act_layer)
        self.window_size = window_size

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        shortcut = x
        x = self.norm1(x)
        h, w = x.shape[1], x.shape[2]
        if self.window_size > 0:
            x, pad_hw = window_partition(x, self.window_size)
        x = self.attn(x)
        if self.window_size > 0:
            x = window_unpartition(x, self.window_size, pad_hw, (h, w))
        x = shortcut + x
        return x + self.mlp(self.norm2(x))


class PatchEmbed(nn.Module):
    def __init__(self, kernel_size=(16, 16), stride=(16, 16), padding=(0, 0), in_chans: int = 3, embed_dim: int = 768):
        super().__init__()
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=kernel_size, stride=stride, padding=padding)

    def forward(self, x):
        return self.proj(x).permute(0, 2, 3, 1)


class ImageEncoderViT(nn.Module):
    def __init__(self, img_size: int = 1024, patch_size: int = 16, in_chans: int = 3, embed_dim: int = 768,
                 depth: int = 12, num_heads: int = 12, mlp_ratio: float = 4.0, out_chans: int = 256,
                 qkv_bias: bool = True, norm_layer: Type[nn.Module] = nn.LayerNorm,
                 act_layer: Type[nn.Module] = nn.GELU, use_abs_pos: bool = True, use_rel_pos: bool = False,
                 rel_pos_zero_init: bool = True, window_size: int = 0, global_attn_indexes: Tuple[int, ...] = ()):
        super().__init__()
        self.img_size = img_size
        self.patch_size = patch_size
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.window_size = window_size
        self.global_attn_indexes = tuple(global_attn_indexes)
        self.patch_embed = PatchEmbed((patch_size, patch_size), (patch_size, patch_size), in_chans=in_chans,
                                      embed_dim=embed_dim)
        self.pos_embed: Optional[nn.Parameter] = None
        if use_abs_pos:
            self.pos_embed = nn.Parameter(torch.zeros(1, img_size // patch_size, img_size // patch_size, embed_dim))
        self.blocks = nn.ModuleList([
            Block(embed_dim, num_heads, mlp_ratio, qkv_bias, norm_layer, act_layer, use_rel_pos, rel_pos_zero_init,
                  window_size if i not in global_attn_indexes else 0,
                  (img_size // patch_size, img_size // patch_size))
            for i in range(depth)])
        self.neck = nn.Sequential(
            nn.Conv2d(embed_dim, out_chans, kernel_size=1, bias=False),
            LayerNorm2d(out_chans),
            nn.Conv2d(out_chans, out_chans, kernel_size=3, padding=1, bias=False),
            LayerNorm2d(out_chans))
        self._engine = None

    # -- fused HIP path -------------------------------------------------------------------
    def is_quantized(self) -> bool:
        from .quant_linear import QuantLinear
        return any(isinstance(m, QuantLinear) for m in self.modules())

    def engine(self):
        from .engine import EncoderEngine
        if self._engine is None or not self._engine.valid_for(self):
            self._engine = EncoderEngine(self)
        return self._engine

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.is_quantized():
            if not x.is_cuda:
                raise RuntimeError("the quantized SAM encoder runs on the GPU only (no CPU fallback)")
            return self.engine()(x)
        return self.module_forward(x)

    def module_forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.patch_embed(x)
        if self.pos_embed is not None:
            x = x + self.pos_embed
        for blk in self.blocks:
            x = blk(x)
        return self.neck(x.permute(0, 3, 1, 2))

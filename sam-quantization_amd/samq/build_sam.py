"""SAM model registry (encoder side): ``sam_model_registry`` / ``build_sam_vit_{h,l,b}``.

Hyper-parameters restate the reference registry (``segment_anything/build_sam.py:14-107``):
patch 16, image 1024, window 14, mlp_ratio 4, LayerNorm eps 1e-6, qkv bias, relative positions,
out_chans 256, pixel mean/std.  The returned ``Sam`` container holds the image encoder (the hot
path) and the preprocessing constants; the prompt encoder / mask decoder are the next rows of
SURVEY.md §8f (f2) and are not built here -- their checkpoint keys are ignored on load
(``load_quant`` loads ``model.pt`` non-strictly, as the reference does, ``__init__.py:50``).
"""
from __future__ import annotations

from functools import partial

import torch
import torch.nn as nn
import torch.nn.functional as F

from .modeling import ImageEncoderViT

VIT_HPARAMS = {
    "vit_h": dict(encoder_embed_dim=1280, encoder_depth=32, encoder_num_heads=16,
                  encoder_global_attn_indexes=[7, 15, 23, 31]),
    "vit_l": dict(encoder_embed_dim=1024, encoder_depth=24, encoder_num_heads=16,
                  encoder_global_attn_indexes=[5, 11, 17, 23]),
    "vit_b": dict(encoder_embed_dim=768, encoder_depth=12, encoder_num_heads=12,
                  encoder_global_attn_indexes=[2, 5, 8, 11]),
}


class Sam(nn.Module):
    """Encoder-side SAM container (reference ``segment_anything/modeling/sam.py``)."""

    mask_threshold: float = 0.0
    image_format: str = "RGB"

    def __init__(self, image_encoder: ImageEncoderViT, pixel_mean=(123.675, 116.28, 103.53),
                 pixel_std=(58.395, 57.12, 57.375)):
        super().__init__()
        self.image_encoder = image_encoder
        self.register_buffer("pixel_mean", torch.tensor(pixel_mean).view(-1, 1, 1), False)
        self.register_buffer("pixel_std", torch.tensor(pixel_std).view(-1, 1, 1), False)

    @property
    def device(self):
        return self.pixel_mean.device

    def preprocess(self, x: torch.Tensor) -> torch.Tensor:
        """Normalise pixels and zero-pad to a square (reference ``sam.py:164-174``)."""
        x = (x - self.pixel_mean) / self.pixel_std
        h, w = x.shape[-2:]
        s = self.image_encoder.img_size
        return F.pad(x, (0, s - w, 0, s - h), value=0)


def build_image_encoder(encoder_embed_dim, encoder_depth, encoder_num_heads, encoder_global_attn_indexes,
                        img_size: int = 1024) -> ImageEncoderViT:
    return ImageEncoderViT(depth=encoder_depth, embed_dim=encoder_embed_dim, img_size=img_size, mlp_ratio=4,
                           norm_layer=partial(torch.nn.LayerNorm, eps=1e-6), num_heads=encoder_num_heads,
                           patch_size=16, qkv_bias=True, use_rel_pos=True,
                           global_attn_indexes=encoder_global_attn_indexes, window_size=14, out_chans=256)


def _build_sam(checkpoint=None, img_size: int = 1024, **hp) -> Sam:
    sam = Sam(build_image_encoder(img_size=img_size, **hp))
    sam.eval()
    if checkpoint is not None:
        sd = torch.load(checkpoint, map_location="cpu", weights_only=True)
        sam.load_state_dict(sd, strict=False)
    return sam


def build_sam_vit_h(checkpoint=None, img_size: int = 1024):
    return _build_sam(checkpoint, img_size, **VIT_HPARAMS["vit_h"])


def build_sam_vit_l(checkpoint=None, img_size: int = 1024):
    return _build_sam(checkpoint, img_size, **VIT_HPARAMS["vit_l"])


def build_sam_vit_b(checkpoint=None, img_size: int = 1024):
    return _build_sam(checkpoint, img_size, **VIT_HPARAMS["vit_b"])


build_sam = build_sam_vit_h

sam_model_registry = {
    "default": build_sam_vit_h,
    "vit_h": build_sam_vit_h,
    "vit_l": build_sam_vit_l,
    "vit_b": build_sam_vit_b,
}

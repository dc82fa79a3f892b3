"""SAM model registry: ``sam_model_registry`` / ``build_sam_vit_{h,l,b}``.

Hyper-parameters restate the reference registry (``segment_anything/build_sam.py:14-107``):
patch 16, image 1024, window 14, mlp_ratio 4, LayerNorm eps 1e-6, qkv bias, relative positions,
out_chans 256, pixel mean/std, prompt encoder / mask decoder (``samq.sam_decoder``).  The image
encoder is the hot path; the prompt side is small torch compute used for masks / mask IoU.
"""
from __future__ import annotations

from functools import partial

import torch
import torch.nn as nn
import torch.nn.functional as F

from .modeling import ImageEncoderViT
from .sam_decoder import build_prompt_decoder, postprocess_masks

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

    def __init__(self, image_encoder: ImageEncoderViT, prompt_encoder=None, mask_decoder=None,
                 pixel_mean=(123.675, 116.28, 103.53), pixel_std=(58.395, 57.12, 57.375)):
        super().__init__()
        self.image_encoder = image_encoder
        if prompt_encoder is None and mask_decoder is None:
            prompt_encoder, mask_decoder = build_prompt_decoder(image_encoder.neck[0].weight.shape[0],
                                                                image_encoder.img_size)
        self.prompt_encoder = prompt_encoder
        self.mask_decoder = mask_decoder
        self.register_buffer("pixel_mean", torch.tensor(pixel_mean).view(-1, 1, 1), False)
        self.register_buffer("pixel_std", torch.tensor(pixel_std).view(-1, 1, 1), False)

    @property
    def device(self):
        return self.pixel_mean.device

    @torch.no_grad()
    def forward(self, batched_input, multimask_output: bool):
        """Reference ``Sam.forward`` (``sam.py:53-131``): encode the batch once (HIP engine), then
        one prompt-encoder + mask-decoder round per image."""
        imgs = torch.stack([self.preprocess(r["image"].float()) for r in batched_input], dim=0)
        p = next(self.image_encoder.parameters(), None)
        dt = p.dtype if p is not None and p.is_floating_point() else torch.float32
        emb = self.image_encoder(imgs.to(dt)).float()
        outs = []
        for rec, e in zip(batched_input, emb):
            pts = (rec["point_coords"], rec["point_labels"]) if "point_coords" in rec else None
            sparse, dense = self.prompt_encoder(points=pts, boxes=rec.get("boxes"), masks=rec.get("mask_inputs"))
            low, iou = self.mask_decoder(e[None], self.prompt_encoder.get_dense_pe(), sparse, dense, multimask_output)
            masks = self.postprocess_masks(low, rec["image"].shape[-2:], rec["original_size"])
            outs.append({"masks": masks > self.mask_threshold, "iou_predictions": iou, "low_res_logits": low})
        return outs

    def postprocess_masks(self, masks, input_size, original_size):
        return postprocess_masks(masks, self.image_encoder.img_size, input_size, original_size)

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

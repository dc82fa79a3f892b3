"""Random-init SAM encoders of the real architecture, GPTQ-packed on the GPU (for bench / smoke).

There are no checkpoints offline; the benchmark uses random weights of the named architecture
(Linear/conv ~ N(0, 0.02), rel-pos / pos-embed ~ N(0, 0.1), LN affine ~ 1 +- 0.05) quantised by
RTN into the reference's packed int4 format (``samq.gptq``), then loaded like a checkpoint.
"""
from __future__ import annotations

import torch

from .build_sam import VIT_HPARAMS, build_image_encoder
from .fused_attention import make_quant_attn
from .gptq import quantize_rtn


@torch.no_grad()
def random_quant_encoder(name: str = "vit_h", groupsize: int = -1, device="cuda", seed: int = 0,
                         img_size: int = 1024, depth: int | None = None, quantize: bool = True, init: bool = True):
    hp = dict(VIT_HPARAMS[name])
    if depth is not None:
        hp["encoder_depth"] = depth
        hp["encoder_global_attn_indexes"] = [i for i in hp["encoder_global_attn_indexes"] if i < depth]
    enc = build_image_encoder(img_size=img_size, **hp)
    if not init:  # receiver of a weight broadcast: just the quantised module tree
        from .quant_linear import make_quant
        make_quant(enc, 4, groupsize)
        make_quant_attn(enc)
        return enc.to(device)
    g = torch.Generator(device="cpu").manual_seed(seed)
    for name_, p in enc.named_parameters():
        if name_.endswith("norm1.weight") or name_.endswith("norm2.weight") or name_ in ("neck.1.weight", "neck.3.weight"):
            p.copy_(1 + 0.05 * torch.randn(p.shape, generator=g))
        elif "rel_pos" in name_ or name_ == "pos_embed":
            p.copy_(0.1 * torch.randn(p.shape, generator=g))
        else:
            p.copy_(0.02 * torch.randn(p.shape, generator=g))
    enc = enc.to(device)
    if quantize:
        quantize_rtn(enc, groupsize=groupsize, device=device)
        make_quant_attn(enc)
    return enc


def flops_per_image(enc) -> dict:
    """Algorithmic FLOPs of one image (2 FLOP / MAC), de-padded: window padding tokens are not
    computed by the fused engine (their q/k/v are the qkv bias), so they are not counted."""
    from .quant_linear import QuantLinear
    patch = enc.patch_embed.proj.kernel_size[0]
    g = enc.img_size // patch
    t = g * g
    c = enc.pos_embed.shape[-1]
    lin = 0
    for blk in enc.blocks:
        for m in blk.modules():
            if isinstance(m, QuantLinear):
                lin += 2 * t * m.infeatures * m.outfeatures
            elif isinstance(m, torch.nn.Linear):
                lin += 2 * t * m.in_features * m.out_features
    att = rel = 0
    for blk in enc.blocks:
        heads = blk.attn.num_heads
        d = c // heads
        if blk.window_size > 0:
            keys, side = blk.window_size ** 2, blk.window_size
        else:
            keys, side = t, g
        att += 2 * 2 * t * keys * d * heads
        rel += 2 * 2 * t * side * d * heads
    oc = enc.neck[0].weight.shape[0]
    pe = 2 * t * c * 3 * patch ** 2
    neck = 2 * t * c * oc + 2 * t * oc * oc * 9
    return dict(linear=lin, attention=att, relpos=rel, patch_embed=pe, neck=neck,
                total=lin + att + rel + pe + neck)


def random_fq_encoder(name: str = "vit_b", device="cuda", seed: int = 0, img_size: int = 1024,
                      calib_images: int = 1, depth: int | None = None):
    """fq_vit W8A8 encoder with random weights (same init as ``random_quant_encoder``), calibrated
    on ``calib_images`` seeded standard-normal images (the reference's calibration sequence, run on
    ``device``) and switched to quant mode."""
    from .fq_vit import build_fq_image_encoder
    enc = build_fq_image_encoder(name, img_size=img_size, depth=depth)
    g = torch.Generator(device="cpu").manual_seed(seed)
    with torch.no_grad():
        for name_, p in enc.named_parameters():
            if name_.endswith("norm1.weight") or name_.endswith("norm2.weight") or name_ in ("neck.1.weight",
                                                                                           "neck.3.weight"):
                p.copy_(1 + 0.05 * torch.randn(p.shape, generator=g))
            elif "rel_pos" in name_ or name_ == "pos_embed":
                p.copy_(0.1 * torch.randn(p.shape, generator=g))
            else:
                p.copy_(0.02 * torch.randn(p.shape, generator=g))
    enc = enc.to(device).eval()
    imgs = [torch.randn((1, 3, img_size, img_size), generator=g).to(device) for _ in range(calib_images)]
    enc.calibrate_with(imgs)
    return enc

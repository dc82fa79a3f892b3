"""Deterministic synthetic SAM image-encoder weights and images (numpy PCG64).

TEST INFRASTRUCTURE (oracle) -- see ``oracle/__init__.py``.

There are no checkpoints in this environment, so every parity fixture, test and bench
run builds its weights here from a seed.  The generator is pure numpy (PCG64), so the
same seed gives bit-identical weights in this container and on the GPU box.

Hyper-parameters restate the reference registry (``segment_anything/build_sam.py:14-44``,
``_build_sam`` ``:55-107``): patch 16, window 14, mlp_ratio 4, out_chans 256, qkv bias,
relative positions on.  Key names follow ``ImageEncoderViT``'s ``state_dict``.
"""
from __future__ import annotations

import numpy as np

VIT_CONFIGS = {
    # embed_dim, depth, heads, global attention block indexes
    "vit_h": dict(embed_dim=1280, depth=32, num_heads=16, global_attn_indexes=(7, 15, 23, 31)),
    "vit_l": dict(embed_dim=1024, depth=24, num_heads=16, global_attn_indexes=(5, 11, 17, 23)),
    "vit_b": dict(embed_dim=768, depth=12, num_heads=12, global_attn_indexes=(2, 5, 8, 11)),
}


def encoder_config(name: str = "vit_h", depth: int | None = None, global_attn_indexes=None,
                   img_size: int = 1024) -> dict:
    cfg = dict(VIT_CONFIGS[name])
    if depth is not None:
        cfg["depth"] = depth
    if global_attn_indexes is not None:
        cfg["global_attn_indexes"] = tuple(global_attn_indexes)
    cfg.update(img_size=img_size, patch_size=16, window_size=14, mlp_ratio=4, out_chans=256,
               in_chans=3, name=name)
    return cfg


def make_encoder_state(cfg: dict, seed: int = 0, std: float = 0.02) -> dict:
    """fp32 numpy state dict of an ``ImageEncoderViT`` (reference key names)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    c = cfg["embed_dim"]
    heads = cfg["num_heads"]
    hd = c // heads
    p = cfg["patch_size"]
    grid = cfg["img_size"] // p
    hidden = int(c * cfg["mlp_ratio"])
    oc = cfg["out_chans"]

    def n(shape, s):
        return (rng.standard_normal(shape, dtype=np.float32) * np.float32(s)).astype(np.float32)

    sd = {
        "patch_embed.proj.weight": n((c, cfg["in_chans"], p, p), std),
        "patch_embed.proj.bias": n((c,), std),
        "pos_embed": n((1, grid, grid, c), 0.1),
    }
    for i in range(cfg["depth"]):
        pre = f"blocks.{i}."
        win = 0 if i in cfg["global_attn_indexes"] else cfg["window_size"]
        side = grid if win == 0 else win
        sd[pre + "norm1.weight"] = (1.0 + n((c,), 0.05)).astype(np.float32)
        sd[pre + "norm1.bias"] = n((c,), std)
        sd[pre + "attn.qkv.weight"] = n((3 * c, c), std)
        sd[pre + "attn.qkv.bias"] = n((3 * c,), std)
        sd[pre + "attn.proj.weight"] = n((c, c), std)
        sd[pre + "attn.proj.bias"] = n((c,), std)
        sd[pre + "attn.rel_pos_h"] = n((2 * side - 1, hd), 0.1)
        sd[pre + "attn.rel_pos_w"] = n((2 * side - 1, hd), 0.1)
        sd[pre + "norm2.weight"] = (1.0 + n((c,), 0.05)).astype(np.float32)
        sd[pre + "norm2.bias"] = n((c,), std)
        sd[pre + "mlp.lin1.weight"] = n((hidden, c), std)
        sd[pre + "mlp.lin1.bias"] = n((hidden,), std)
        sd[pre + "mlp.lin2.weight"] = n((c, hidden), std)
        sd[pre + "mlp.lin2.bias"] = n((c,), std)
    sd["neck.0.weight"] = n((oc, c, 1, 1), std)
    sd["neck.1.weight"] = (1.0 + n((oc,), 0.05)).astype(np.float32)
    sd["neck.1.bias"] = n((oc,), std)
    sd["neck.2.weight"] = n((oc, oc, 3, 3), std)
    sd["neck.3.weight"] = (1.0 + n((oc,), 0.05)).astype(np.float32)
    sd["neck.3.bias"] = n((oc,), std)
    return sd


LINEAR_SUFFIXES = ("attn.qkv", "attn.proj", "mlp.lin1", "mlp.lin2")


def linear_names(cfg: dict):
    return [f"blocks.{i}.{s}" for i in range(cfg["depth"]) for s in LINEAR_SUFFIXES]


def make_images(batch: int, img_size: int = 1024, seed: int = 1) -> np.ndarray:
    """Standard-normal images (B,3,H,W) fp32, like ``bench_speed``'s ``torch.randn``
    input (reference ``gptq4sam_infer.py:64``)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.standard_normal((batch, 3, img_size, img_size), dtype=np.float32)


def make_decoder_state(shapes: dict, seed: int = 300) -> dict:
    """Seeded weights for the SAM prompt encoder + mask decoder, given ``{key: shape}`` (taken
    from the module's own ``state_dict``, so the reference and our modules receive the same
    tensors).  Keys are visited in sorted order.  Embeddings and the Fourier matrix ~ N(0, 1);
    LayerNorm weight 1 + N(0, 0.1), bias N(0, 0.1); other biases N(0, 0.02); matrices and conv
    kernels N(0, 1/fan_in)."""
    import re
    unit = re.compile(r"(point_embeddings\.\d+|not_a_point_embed|no_mask_embed|iou_token|mask_tokens)\.weight$"
                      r"|positional_encoding_gaussian_matrix$")
    rng = np.random.Generator(np.random.PCG64(seed))
    out = {}
    for k in sorted(shapes):
        shape = tuple(shapes[k])
        z = rng.standard_normal(shape).astype(np.float32)
        ln = len(shape) == 1 and len(tuple(shapes.get(k.rsplit(".", 1)[0] + ".weight", ()))) == 1
        if unit.search(k):
            out[k] = z
        elif ln and k.endswith(".weight"):
            out[k] = (1.0 + 0.1 * z).astype(np.float32)
        elif len(shape) == 1:
            out[k] = ((0.1 if ln else 0.02) * z).astype(np.float32)
        else:
            out[k] = (z / np.sqrt(float(np.prod(shape[1:])))).astype(np.float32)
    return out


DECODER_PROMPTS = [
    dict(points=[[512.0, 512.0]], labels=[1]),
    dict(points=[[200.0, 300.0]], labels=[1]),
    dict(points=[[700.0, 150.0], [650.0, 220.0]], labels=[1, 0]),
    dict(points=[[120.0, 880.0], [900.0, 900.0], [500.0, 640.0]], labels=[1, 1, 0]),
    dict(box=[300.0, 260.0, 760.0, 700.0]),
]

"""samq -- MI355X-native (gfx950) quantized SAM image-encoder hot path.

Drop-in for the reference's ``gptq_triton`` package (``gptq_triton/__init__.py``): same public
names -- ``load_quant``, ``autotune_warmup``, ``QuantLinear``, ``make_quant``,
``triton_matmul4`` (alias of ``matmul4``), ``QuantAttention``, ``make_quant_attn`` -- backed by
hand-written HIP kernels in ``libsamq_hip.so`` (C ABI: ``include/samq.h``).  No Triton, no
CUDA shims, no CPU fallback.
"""
from __future__ import annotations

import itertools
import json
from pathlib import Path
from typing import Optional

import torch

from . import _lib, ops, quant_linear, fused_attention  # noqa: F401
from .build_sam import Sam, build_sam, build_sam_vit_b, build_sam_vit_h, build_sam_vit_l, sam_model_registry  # noqa
from .fused_attention import QuantAttention, make_quant_attn
from .modeling import ImageEncoderViT
from .quant_linear import (QuantLinear, calibrate_act_quant, make_act_quant, make_quant, matmul4,  # noqa: F401
                           triton_matmul4)
from . import fq_vit  # noqa: F401
from .sam_decoder import ResizeLongestSide, SamPredictor, mask_iou  # noqa: F401

__all__ = [
    "load_quant", "autotune_warmup", "QuantLinear", "make_quant", "matmul4", "triton_matmul4",
    "QuantAttention", "make_quant_attn", "ImageEncoderViT", "Sam", "sam_model_registry",
    "make_act_quant", "calibrate_act_quant", "fq_vit", "SamPredictor", "ResizeLongestSide", "mask_iou",
]


def load_quant(model, checkpoint: str, warmup_autotune: bool = True, device: Optional[str] = "cuda",
               fuse_mlp: Optional[bool] = None, sub_module: Optional[str] = None):
    """Load a GPTQ-quantised checkpoint into ``model`` (reference ``gptq_triton/__init__.py:15-81``).

    Reads ``quant_config.json`` ({"wbits", "groupsize"}), swaps every Linear of ``sub_module``
    for ``QuantLinear``, loads ``model.safetensors`` (strict) or ``model.pt`` (non-strict), drops
    all-zero biases, swaps every SAM ``Attention`` for ``QuantAttention``, moves to ``device``
    and (``warmup_autotune``) repacks the weights for the kernels.  ``fuse_mlp`` is accepted for
    API compatibility: the reference's fused MLP is a LLaMA gated MLP that SAM does not have
    (``make_fused_mlp`` references an undefined ``LlamaMLP``); SAM's lin1+GELU fusion is always
    on in the encoder engine, so ``fuse_mlp=True`` raises ``NotImplementedError`` and
    ``None``/``False`` are no-ops.
    """
    ckpt = Path(checkpoint)
    cfg = json.loads((ckpt / "quant_config.json").read_text())
    wbits, groupsize = cfg["wbits"], cfg["groupsize"]
    target = getattr(model, sub_module) if sub_module else model
    make_quant(target, wbits, groupsize)
    print("Loading model ...")
    if (ckpt / "model.safetensors").exists():
        from safetensors.torch import load_file as safe_load
        model.load_state_dict(safe_load(str(ckpt / "model.safetensors")))
    elif (ckpt / "model.pt").exists():
        model.load_state_dict(torch.load(ckpt / "model.pt", map_location="cpu", weights_only=True), strict=False)
    else:
        raise FileNotFoundError(
            f"Could not find model checkpoint at {checkpoint}; please ensure that the path is correct and "
            "contains a `model.pt` or `model.safetensors` file.")
    for m in model.modules():
        if isinstance(m, QuantLinear) and m.bias is not None and bool((m.bias == 0).all()):
            m.bias = None
    make_quant_attn(target)
    if fuse_mlp:
        raise NotImplementedError("fuse_mlp: SAM has no gated (LLaMA) MLP; lin1+GELU is fused in the engine")
    if device is not None:
        model = model.to(device)
    if warmup_autotune:
        if device is None:
            raise ValueError("You must specify a device when warmup_autotune is True.")
        autotune_warmup(model)
    print("Done.")
    return model


def autotune_warmup(model):
    """Repack every QuantLinear once and run one GEMM per unique (K, N) shape (reference
    ``gptq_triton/__init__.py:84-104``; there is no autotuner to warm)."""
    with torch.no_grad():
        for fn in itertools.chain(quant_linear.autotune_warmup(model)):
            fn(256)

#!/usr/bin/env python3
"""Producer of GPTQ-packed SAM checkpoints (reference ``gptq4sam.py``, main ``:596-663``).

Same positional arguments and quantisation flags as the reference CLI: build SAM from
``model_path`` (``sam_model_registry``), GPTQ-calibrate every image-encoder Linear block by block
(``sam_sequential``, reference ``:280-414``; Hessians + Cholesky OBQ on the GPU when one is
present), pack them into the reference's int4 ``QuantLinear`` buffers (``sam_pack`` /
``pack_linear``, ``:417-497``, bit-identical) and write ``<save>/model.pt`` +
``<save>/quant_config.json`` (``:651-663``) -- exactly what ``gptq4sam_infer.py --save`` and
``samq.load_quant`` read.

Calibration data: the reference draws ``--nsamples`` SBD training images through its RITM data
pipeline (not available offline).  Here ``dataset_dir`` may hold image files (png/jpg), fed
through ``SamPredictor``'s preprocessing (``ResizeLongestSide`` + ``Sam.preprocess``); without
it (or with ``--synthetic``) the calibration images are seeded standard-normal 1024x1024
tensors.  ``--synthetic`` also replaces the checkpoint by the seeded random-init weights that
bench.py uses.  ``--nearest`` is the reference's RTN baseline.
"""
from __future__ import annotations

import argparse
import json
import random
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent / "sam-quantization_amd"))

import samq  # noqa: E402
from samq.gptq import pack_gptq, quantize_rtn, sam_sequential, save_quant  # noqa: E402


def calibration_images(model, dataset_dir, nsamples: int, seed: int, device, img_size: int):
    """``nsamples`` preprocessed (1, 3, S, S) images: files of ``dataset_dir`` if it holds any,
    else seeded N(0, 1) tensors (the bench / reference ``bench_speed`` input distribution)."""
    files = []
    if dataset_dir and Path(dataset_dir).is_dir():
        files = sorted(p for p in Path(dataset_dir).rglob("*") if p.suffix.lower() in (".png", ".jpg", ".jpeg"))
    out = []
    if files:
        from PIL import Image
        from samq.sam_decoder import ResizeLongestSide
        tf = ResizeLongestSide(img_size)
        for f in files[:nsamples]:
            im = tf.apply_image(np.array(Image.open(f).convert("RGB")))
            t = torch.as_tensor(im).permute(2, 0, 1).contiguous()[None].float()
            out.append(model.preprocess(t.to(model.pixel_mean.device)).to(device))
    g = torch.Generator().manual_seed(seed)
    while len(out) < nsamples:
        out.append(torch.randn((1, 3, img_size, img_size), generator=g).to(device))
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("model_path", type=str, nargs="?", default=None, help="SAM checkpoint (.pth state dict)")
    ap.add_argument("dataset_dir", type=str, nargs="?", default=None, help="calibration images (png/jpg)")
    ap.add_argument("--batch_size", type=int, default=1)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--nsamples", type=int, default=128)
    ap.add_argument("--percdamp", type=float, default=0.01)
    ap.add_argument("--nearest", action="store_true", help="RTN baseline instead of GPTQ")
    ap.add_argument("--wbits", type=int, default=4, choices=[2, 3, 4, 8, 16])
    ap.add_argument("--groupsize", type=int, default=-1)
    ap.add_argument("--sym", action="store_true")
    ap.add_argument("--new-eval", action="store_true")
    ap.add_argument("--act-order", action="store_true")
    ap.add_argument("--true-sequential", action="store_true")
    ap.add_argument("--num_workers", action="store_true")
    ap.add_argument("--save", type=str, required=True)
    ap.add_argument("--synthetic", action="store_true", help="seeded random-init weights instead of model_path")
    ap.add_argument("--model-type", default="vit_h", choices=list(samq.sam_model_registry))
    ap.add_argument("--img-size", type=int, default=1024)
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    args = ap.parse_args(argv)
    assert args.batch_size == 1, "Batch size must be 1 for calibration."   # reference :588
    if args.wbits != 4:
        raise NotImplementedError("only 4-bit QuantLinear is supported (reference quant_linear.py:72-73)")
    if args.sym:
        raise NotImplementedError("symmetric GPTQ is not wired to the packed int4 format here")
    if args.act_order and args.groupsize != -1:
        # reference quirk 8: pack_linear assigns groups by the ORIGINAL column
        # while fasterquant chose them over the permuted ones -> a wrong checkpoint
        raise ValueError("--act-order with --groupsize produces an inconsistent checkpoint in the reference")

    if not (args.synthetic or args.model_path):
        ap.error("pass a SAM checkpoint (model_path) or --synthetic")

    torch.manual_seed(args.seed)
    np.random.seed(args.seed)
    random.seed(args.seed)
    dev = torch.device(args.device)
    model = samq.sam_model_registry[args.model_type](
        checkpoint=None if args.synthetic else args.model_path, img_size=args.img_size)
    if args.synthetic:
        from samq.synthetic import random_quant_encoder
        enc = random_quant_encoder(args.model_type, device="cpu", seed=args.seed, img_size=args.img_size,
                                   quantize=False)
        model.image_encoder.load_state_dict(enc.state_dict())
    model.eval()
    if dev.type == "cuda":
        model.half()   # reference :635 (GPTQ accumulates its Hessians in fp32 either way)
    enc = model.image_encoder.to(dev)
    dt = next(enc.parameters()).dtype
    if args.nearest:
        quantize_rtn(enc, groupsize=args.groupsize, device=dev)
    else:
        imgs = [x.to(dt) for x in calibration_images(model.to(dev), args.dataset_dir, args.nsamples, args.seed,
                                                     dev, args.img_size)]
        params = sam_sequential(enc, imgs, groupsize=args.groupsize, percdamp=args.percdamp,
                                act_order=args.act_order, true_sequential=args.true_sequential)
        pack_gptq(enc, params, groupsize=args.groupsize)
    save_quant(model, args.save, args.wbits, args.groupsize)
    print(json.dumps({"saved": str(Path(args.save) / "model.pt"), "wbits": args.wbits, "groupsize": args.groupsize,
                      "method": "rtn" if args.nearest else "gptq", "nsamples": 0 if args.nearest else args.nsamples}))
    return model


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Entry point of the quantized SAM image-encoder hot path (reference ``gptq4sam_infer.py``).

Same positional arguments and quantisation flags as the reference CLI (``:105-168``); the flow
is the reference's ``main`` (``:170-225``): build SAM (``sam_model_registry``), ``.half()``,
``load_quant(model, --save, sub_module="image_encoder", fuse_mlp=False)``, then
``bench_speed(model.image_encoder, (B,3,1024,1024), fp16, "cuda")``.

Additions: ``--synthetic`` quantises a random-init model by RTN when no checkpoint directory
is given (there are no checkpoints offline); ``--model-type`` (vit_h/vit_l/vit_b);
``--bench-batch``.  The SBD click-mIoU evaluation (``script/evaluation2.py``) needs the dataset
and the mask decoder and is not part of this build yet: ``dataset_dir`` is
accepted and ignored.
"""
from __future__ import annotations

import argparse
import random
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent / "sam-quantization_amd"))

import samq  # noqa: E402


@torch.no_grad()
def bench_speed(model, inp_shape, dtype, device, num_iters=100, warmup_iters=25):
    """Reference ``bench_speed`` (``gptq4sam_infer.py:59-79``): warm-up + timed forwards of a
    randn input, device-synchronised wall clock; returns mean seconds per iteration."""
    model.to(device)
    model.eval()
    inp = torch.randn(inp_shape, dtype=dtype).to(device)
    print("Warm up...")
    for _ in range(warmup_iters):
        model(inp)
    print("Speed test...")
    torch.cuda.synchronize()
    tik = time.time()
    for _ in range(num_iters):
        model(inp)
    torch.cuda.synchronize()
    tok = time.time()
    per = (tok - tik) / num_iters
    print(f"Average time per iteration: {per}  ({inp_shape[0] / per:.2f} img/s)")
    return per


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("model_path", type=str, nargs="?", default=None, help="SAM checkpoint (unused by the encoder bench)")
    ap.add_argument("dataset_dir", type=str, nargs="?", default=None, help="SBD directory (evaluation not built yet)")
    ap.add_argument("--batch_size", type=int, default=1)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--nsamples", type=int, default=128)
    ap.add_argument("--percdamp", type=float, default=0.01)
    ap.add_argument("--nearest", action="store_true")
    ap.add_argument("--wbits", type=int, default=4, choices=[2, 3, 4, 8, 16])
    ap.add_argument("--groupsize", type=int, default=-1)
    ap.add_argument("--sym", action="store_true")
    ap.add_argument("--new-eval", action="store_true")
    ap.add_argument("--act-order", action="store_true")
    ap.add_argument("--true-sequential", action="store_true")
    ap.add_argument("--num_workers", action="store_true")
    ap.add_argument("--save", type=str, default=None, help="directory with model.pt + quant_config.json")
    ap.add_argument("--synthetic", action="store_true", help="random-init RTN-quantised model if --save is absent")
    ap.add_argument("--model-type", default="vit_h", choices=list(samq.sam_model_registry))
    ap.add_argument("--bench-batch", type=int, default=1)
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=25)
    args = ap.parse_args(argv)

    torch.manual_seed(args.seed)
    np.random.seed(args.seed)
    random.seed(args.seed)
    device = "cuda"
    model = samq.sam_model_registry[args.model_type](checkpoint=None)
    model.half()
    if args.save:
        model = samq.load_quant(model, args.save, sub_module="image_encoder", fuse_mlp=False)
    elif args.synthetic:
        from samq.synthetic import random_quant_encoder
        model.image_encoder = random_quant_encoder(args.model_type, args.groupsize, device=device)
    else:
        ap.error("pass --save <quantised checkpoint dir> or --synthetic")
    return bench_speed(model.image_encoder, (args.bench_batch, 3, 1024, 1024), torch.float16, device,
                       num_iters=args.iters, warmup_iters=args.warmup)


if __name__ == "__main__":
    main()

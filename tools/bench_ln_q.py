"""Micro-benchmark of the W4A8 LayerNorm with int8 output codes (ViT-H rows, HIP events), against the
fp16-output LayerNorm on the same rows.

    python tools/bench_ln_q.py
"""
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "sam-quantization_amd"))
from samq import ops  # noqa: E402

dev = torch.device("cuda:0")
for rows, c in ((8192, 1280), (16384, 1280)):
    xs = [torch.randn(rows, c, device=dev) for _ in range(4)]   # rotate past the MALL
    w, b = torch.randn(c, device=dev), torch.randn(c, device=dev)
    y16 = torch.empty(rows, c, device=dev, dtype=torch.float16)
    y8 = torch.empty(rows, c, device=dev, dtype=torch.int8)
    runs = {"f16": (lambda x: ops.layernorm(x, w, b, 1e-6, out=y16), 6),
            "i8": (lambda x: ops.layernorm_q(x, w, b, 1e-6, out_scale=0.03, out=y8), 5)}
    for name, (fn, bpe) in runs.items():
        for _ in range(3):
            fn(xs[0])
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(48):
            fn(xs[i % 4])
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 48 * 1e3
        print(f"layernorm rows={rows} C={c} out={name}: {us:.1f} us  {rows * c * bpe / us / 1e3:.0f} GB/s", flush=True)

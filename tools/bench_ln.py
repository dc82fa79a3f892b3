"""Micro-benchmark of the encoder LayerNorm (f32 residual rows -> f16), ViT-H B=4 geometry."""
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "sam-quantization_amd"))
from samq import ops  # noqa: E402

dev = torch.device("cuda:0")
for rows, c, rpw in ((16384, 1280, 1), (16384, 1280, 2), (16384, 1280, 4), (4096, 768, 1), (4096, 768, 2),
                     (4096, 768, 4)):
    xs = [torch.randn(rows, c, device=dev) for _ in range(4)]   # 4 x 84 MB rotate past the 256 MB MALL
    x = xs[0]
    w, b = torch.randn(c, device=dev), torch.randn(c, device=dev)
    y = torch.empty(rows, c, device=dev, dtype=torch.float16)
    for _ in range(3):
        ops.layernorm(x, w, b, 1e-6, out=y, rows_per_wave=rpw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(48):
        ops.layernorm(xs[i % 4], w, b, 1e-6, out=y, rows_per_wave=rpw)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 48 * 1e3
    ref = torch.nn.functional.layer_norm(xs[3], (c,), w, b, 1e-6)
    err = (y.float() - ref).abs().max().item()
    print(f"layernorm rows={rows} C={c} rpw={rpw}: {us:.1f} us  {rows * c * 6 / us / 1e3:.0f} GB/s  max-abs vs torch {err:.2e}")

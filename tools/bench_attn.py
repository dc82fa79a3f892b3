"""Micro-benchmark of the rel-pos attention kernel on the ViT-H geometries (HIP events).

    python tools/bench_attn.py [--batch 4] [--iters 20]
"""
import argparse
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "sam-quantization_amd"))
from samq import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--heads", type=int, default=16)
    ap.add_argument("--hd", type=int, default=80)
    ap.add_argument("--window-only", action="store_true")
    ap.add_argument("--global-only", action="store_true")
    ap.add_argument("--q8", action="store_true", help="int8 output codes (the W4A8 proj-input QAct store)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    b, g, heads, d = args.batch, 64, args.heads, args.hd
    c = heads * d
    qkv = (torch.randn(b, g, g, 3 * c, device=dev) * 0.5).half()
    bias = (torch.randn(3 * c, device=dev) * 0.1).half()
    for window in ((14,) if args.window_only else (0,) if args.global_only else (14, 0)):
        side = window or g
        rh = (torch.randn(2 * side - 1, d, device=dev) * 0.1).half()
        rw = (torch.randn(2 * side - 1, d, device=dev) * 0.1).half()
        out = torch.empty(b, g, g, c, device=dev, dtype=torch.int8 if args.q8 else torch.float16)
        kw = dict(out_scale=0.02) if args.q8 else {}
        for _ in range(3):
            ops.rel_attention(qkv, bias, rh, rw, heads, window, d ** -0.5, out=out, **kw)
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                ops.rel_attention(qkv, bias, rh, rw, heads, window, d ** -0.5, out=out, **kw)
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / args.iters * 1e3)
        t = g * g
        keys = window * window if window else t
        fl = 4.0 * b * heads * t * keys * d
        byt = b * t * 3 * c * 2 + b * t * c * 2
        print(f"attention{' q8' if args.q8 else ''} window={window:2d} B={b}: {best:8.1f} us  {fl / best / 1e6:7.1f} TF/s  "
              f"{byt / best / 1e3:7.1f} GB/s (qkv read once + out)")


if __name__ == "__main__":
    main()

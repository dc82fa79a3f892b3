"""Micro-benchmark of the W8A8 (fq_vit) attention kernels on the vit_b geometry (64 x 64 grid,
12 heads of 64, windows of 14 and global), HIP events on the launch stream; outputs of every
run compared with the first (determinism).  ``SAMQ_LIB`` selects a variant library.

    python tools/bench_attn_q8.py [--batch 1] [--iters 20]
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
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--window-only", action="store_true")
    ap.add_argument("--global-only", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    b, side, heads, d = args.batch, 64, 12, 64
    c = heads * d
    qkv = torch.randint(-100, 100, (b, side, side, 3 * c), generator=g, device=dev, dtype=torch.int8)
    bias = torch.randn(3 * c, generator=g, device=dev) * 0.1
    stream = torch.cuda.current_stream()
    for window in ((14,) if args.window_only else ((0,) if args.global_only else (14, 0))):
        s = 2 * (window or side) - 1
        rh = torch.randn(s, d, generator=g, device=dev) * 0.1
        rw = torch.randn(s, d, generator=g, device=dev) * 0.1

        v16 = qkv[..., 2 * c:].to(torch.float16).contiguous() if window == 0 else None

        def run(v=None):
            return ops.rel_attention_q8(qkv, bias if window else None, rh, rw, heads, window, d ** -0.5, 0.05, 0.08,
                                        0.1, 0.03, v16=v)
        ref = run()
        if v16 is not None:   # round 6: the global kernel staging V from the fp16 copy (the engine's path)
            assert torch.equal(run(v16), ref)
            b16 = 1e9
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(args.iters):
                    run(v16)
                e1.record(stream)
                torch.cuda.synchronize()
                b16 = min(b16, e0.elapsed_time(e1) / args.iters * 1e3)
            print(f"attention_q8 window= 0 B={b} with fp16 V: {b16:8.1f} us", flush=True)
        best = 1e9
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.iters):
                run()
            e1.record(stream)
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / args.iters * 1e3)
        same = torch.equal(run(), ref)
        keys = (window * window) if window else side * side
        nq = b * side * side
        gop = 2 * 2 * nq * keys * d * heads / 1e9
        print(f"attention_q8 window={window:2d} B={b}: {best:8.1f} us  {gop / best * 1e3:7.1f} TOPS (q.k + p.v)  "
              f"deterministic: {same}", flush=True)


if __name__ == "__main__":
    main()

"""Micro-benchmark of the W4A16 GEMM tile configs on the ViT-H projection shapes.

    python tools/bench_gemm.py [--m 16384] [--cfgs 1,2,3,6] [--iters 30]

Times every (shape, cfg, epilogue) with HIP events on the launch stream, interleaved rounds in
one process (guide §5.4 rule 24), and checks each output against cfg 3 on the same inputs.
"""
import argparse
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "sam-quantization_amd"))
from samq import ops  # noqa: E402
from samq.gptq import rtn, pack_linear  # noqa: E402
from samq.quant_linear import QuantLinear  # noqa: E402

SHAPES = {"qkv": (1280, 3840, ops.EPI_BIAS), "proj": (1280, 1280, ops.EPI_RESADD_F32),
          "lin1": (1280, 5120, ops.EPI_BIAS_GELU), "lin2": (5120, 1280, ops.EPI_RESADD_F32)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=16384)
    ap.add_argument("--cfgs", default="1,2,3,6")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--shapes", default="qkv,proj,lin1,lin2")
    ap.add_argument("--epi", default="native", help="native | bias (force EPI_BIAS)")
    ap.add_argument("--torch", action="store_true", help="also time dense fp16 torch.matmul")
    ap.add_argument("--groupsize", type=int, default=-1)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    cfgs = [int(c) for c in args.cfgs.split(",")]
    m = args.m
    results = {}
    for name in args.shapes.split(","):
        k, n, epi = SHAPES[name]
        if args.epi == "bias":
            epi = ops.EPI_BIAS
        gs = args.groupsize
        q = QuantLinear(4, gs, k, n, True).to(dev)
        w = torch.randn(n, k, device=dev) * 0.02
        fake, s, z = rtn(w, gs)
        pack_linear(q, fake, s, z, torch.randn(n, device=dev) * 0.02)
        packed = q.prepare()
        # layout-2 weights exist only in the tuning build (SAMQ_LIB=tuning, make tuning)
        packed2 = ops.w4_repack(q.qweight, layout=2) if any(40 <= c < 50 for c in cfgs) else None
        pk = lambda c: packed2 if 40 <= c < 50 else packed  # noqa: E731
        a = torch.randn(m, k, device=dev).half()
        f32 = epi in (ops.EPI_RESADD_F32, ops.EPI_F32)
        outs = {}
        for c in cfgs + [3]:
            out = torch.zeros(m, n, device=dev, dtype=torch.float32 if f32 else torch.float16)
            try:
                ops.w4a16_gemm(a, pk(c), q.scales, q.qzeros, q.bias, n, gs, epi, out=out, cfg=c)
            except AssertionError as e:
                print(f"{name} cfg {c}: skipped ({e})")
                continue
            outs[c] = out
        torch.cuda.synchronize()
        ref = outs[3].float()
        times = {c: [] for c in outs}
        stream = torch.cuda.current_stream()
        for _ in range(3):
            for c in outs:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ops.w4a16_gemm(a, pk(c), q.scales, q.qzeros, q.bias, n, gs, epi, out=outs[c], cfg=c)
                e0.record(stream)
                for _ in range(args.iters):
                    ops.w4a16_gemm(a, pk(c), q.scales, q.qzeros, q.bias, n, gs, epi, out=outs[c], cfg=c)
                e1.record(stream)
                torch.cuda.synchronize()
                times[c].append(e0.elapsed_time(e1) / args.iters * 1e3)
        flops = 2.0 * m * n * k
        for c in outs:
            us = min(times[c])
            # residual epilogues accumulate: compare a fresh single launch instead
            o = torch.zeros_like(outs[c])
            ops.w4a16_gemm(a, pk(c), q.scales, q.qzeros, q.bias, n, gs, epi, out=o, cfg=c)
            r = torch.zeros_like(outs[3])
            ops.w4a16_gemm(a, packed, q.scales, q.qzeros, q.bias, n, gs, epi, out=r, cfg=3)
            err = (o.float() - r.float()).abs().max().item()
            print(f"{name:5s} M={m} K={k} N={n} cfg {c}: {us:8.1f} us  {flops / us / 1e6:7.1f} TF/s  "
                  f"({flops / us / 1e6 / 2500 * 100:4.1f}% fp16 peak)  maxdiff vs cfg3 {err:.2e}")
            results[(name, c)] = us
    if args.torch:
        # vendor reference point: dense fp16 x fp16 hipBLASLt GEMM of the same shapes
        for name in args.shapes.split(","):
            k, n, _ = SHAPES[name]
            a = torch.randn(m, k, device=dev).half()
            b = torch.randn(k, n, device=dev).half()
            for _ in range(3):
                torch.matmul(a, b)
            torch.cuda.synchronize()
            best = 1e9
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    torch.matmul(a, b)
                e1.record()
                torch.cuda.synchronize()
                best = min(best, e0.elapsed_time(e1) / args.iters * 1e3)
            fl = 2.0 * m * n * k
            print(f"{name:5s} torch.matmul fp16 (hipBLASLt): {best:8.1f} us  {fl / best / 1e6:7.1f} TF/s")
            results[(name, "torch")] = best
    tot = {}
    for (name, c), us in results.items():
        tot.setdefault(c, 0.0)
        tot[c] += us
    print("sum over shapes:", {c: round(v, 1) for c, v in tot.items()})


if __name__ == "__main__":
    main()

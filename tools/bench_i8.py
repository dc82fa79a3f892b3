"""Micro-benchmark of the W4A8 int8-MFMA GEMM tile configs (81 256x256, 82 128x256, 83 128x128)
on the ViT-H projection shapes, with HIP events on the launch stream; outputs checked equal to
cfg 82 (int32-exact sums: every config must agree bit for bit).

    python tools/bench_i8.py [--m 16384,32768] [--cfgs 81,82,83]
(cfg 100 + c: tile config c with the zero-point row sums supplied by the producer, round 6)
"""
import argparse
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "sam-quantization_amd"))
from samq import _lib, ops  # noqa: E402
from samq.gptq import rtn, pack_linear  # noqa: E402
from samq.quant_linear import QuantLinear  # noqa: E402

SHAPES = {"qkv": (1280, 3840, ops.EPI_BIAS), "proj": (1280, 1280, ops.EPI_RESADD_F32),
          "lin1": (1280, 5120, ops.EPI_Q8_GELU), "lin2": (5120, 1280, ops.EPI_RESADD_F32)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="16384,32768")
    ap.add_argument("--cfgs", default="81,82,83")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--w8-vitb", action="store_true", help="W8A8 vit_b shapes (int8 weights, EPI_Q8)")
    ap.add_argument("--w8-vith", action="store_true",
                    help="ViT-H W4A8 shapes and epilogues on int8-expanded weights (values in [-15, 15], BF_W8)")
    args = ap.parse_args()
    if args.w8_vitb:
        return w8_vitb(args)
    if args.w8_vith:
        return w8_vith(args)
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    cfgs = [int(c) for c in args.cfgs.split(",")]
    for m in (int(x) for x in args.m.split(",")):
        tot = {c: 0.0 for c in cfgs}
        for name, (k, n, epi) in SHAPES.items():
            q = QuantLinear(4, -1, k, n, True).to(dev)
            w = torch.randn(n, k, device=dev) * 0.02
            fake, s, z = rtn(w)
            pack_linear(q, fake, s, z, torch.randn(n, device=dev) * 0.02)
            wb = q.prepare_w4a8()
            a = torch.randint(-127, 128, (m, k), device=dev, dtype=torch.int8)
            osc = 0.05 if epi == ops.EPI_Q8_GELU else 0.0

            rs = a.to(torch.int32).sum(1, dtype=torch.int32)
            rso = torch.zeros(m, device=dev, dtype=torch.int32)

            def run(c, out):
                if c >= 100:   # cfg c - 100 with the producer-side row sums (round 6: samq_w4a8_gemm_rs;
                    # lin1 also accumulates its output row sums, as in the engine)
                    return ops.w4a8_gemm(a, wb["packed"], wb["scale"], q.qzeros, n, wb["bias"], epi, 0.02, osc,
                                         out=out, cfg=c - 100, rowsum=rs,
                                         rowsum_out=rso if epi == ops.EPI_Q8_GELU else None)
                return ops.i8_gemm(a, _lib.BF_W4, wb["packed"], wb["scale"], n, wb["bias"], q.qzeros, epi,
                                   0.02, osc, out=out, cfg=c)
            if epi == ops.EPI_RESADD_F32:
                ref = torch.zeros(m, n, device=dev, dtype=torch.float32)
                run(82, ref)
            else:
                ref = run(82, None)
            stream = torch.cuda.current_stream()
            for c in cfgs:
                o = torch.zeros_like(ref)
                run(c, o)
                same = torch.equal(o, ref)
                best = 1e9
                for _ in range(3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(args.iters):
                        run(c, o)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    best = min(best, e0.elapsed_time(e1) / args.iters * 1e3)
                tot[c] += best
                fl = 2.0 * m * n * k
                print(f"{name:5s} M={m} cfg {c}: {best:8.1f} us  {fl / best / 1e6:7.1f} TOPS "
                      f"({fl / best / 1e6 / 5000 * 100:4.1f}% int8 peak)  identical to cfg 82: {same}", flush=True)
        print(f"M={m} per-block GEMM total: " + "  ".join(f"cfg {c} {t:.1f} us" for c, t in tot.items()), flush=True)


def w8_vith(args):
    """The ViT-H W4A8 shapes and epilogues with the int4 weights expanded to int8 (q - zp in [-15, 15]):
    the int8 GEMM without any in-kernel unpack (BF_W8 kernels), timed like main()."""
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    cfgs = [int(c) for c in args.cfgs.split(",")]
    for m in (int(x) for x in args.m.split(",")):
        tot = {c: 0.0 for c in cfgs}
        for name, (k, n, epi) in SHAPES.items():
            w = torch.randint(-15, 16, (n, k), device=dev, dtype=torch.int8)
            packed = ops.w8_repack(w)
            ws = torch.rand(n, device=dev) * 0.01
            bias = torch.randn(n, device=dev) * 0.02
            a = torch.randint(-127, 128, (m, k), device=dev, dtype=torch.int8)
            osc = 0.05 if epi == ops.EPI_Q8_GELU else 0.0

            def run(c, out):
                return ops.i8_gemm(a, _lib.BF_W8, packed, ws, n, bias, None, epi, 0.02, osc, out=out, cfg=c)
            stream = torch.cuda.current_stream()
            for c in cfgs:
                o = torch.zeros(m, n, device=dev, dtype=torch.float32) if epi == ops.EPI_RESADD_F32 else None
                o = run(c, o)
                best = 1e9
                for _ in range(3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(args.iters):
                        run(c, o)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    best = min(best, e0.elapsed_time(e1) / args.iters * 1e3)
                tot[c] += best
                fl = 2.0 * m * n * k
                print(f"w8 {name:5s} M={m} cfg {c}: {best:8.1f} us  {fl / best / 1e6:7.1f} TOPS "
                      f"({fl / best / 1e6 / 5000 * 100:4.1f}% int8 peak)", flush=True)
        print(f"w8 M={m} per-block GEMM total: " + "  ".join(f"cfg {c} {t:.1f} us" for c, t in tot.items()), flush=True)


def w8_vitb(args):
    """fq_vit W8A8 vit_b projection shapes (M = 4096 per image), quantising epilogue."""
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    cfgs = [int(c) for c in args.cfgs.split(",")]
    shapes = {"qkv": (768, 2304), "proj": (768, 768), "lin1": (768, 3072), "lin2": (3072, 768)}
    for m in (int(x) for x in args.m.split(",")):
        tot = {c: 0.0 for c in cfgs}
        for name, (k, n) in shapes.items():
            w = torch.randint(-127, 128, (n, k), device=dev, dtype=torch.int8)
            packed = ops.w8_repack(w)
            ws = torch.rand(n, device=dev) * 0.01
            bias = torch.randn(n, device=dev) * 0.02
            a = torch.randint(-127, 128, (m, k), device=dev, dtype=torch.int8)

            def run(c):
                return ops.w8a8_gemm(a, packed, ws, n, bias, ops.EPI_Q8, 0.02, 0.05) if c == 0 else \
                    ops.i8_gemm(a, _lib.BF_W8, packed, ws, n, bias, None, ops.EPI_Q8, 0.02, 0.05, cfg=c)
            ref = run(0)
            stream = torch.cuda.current_stream()
            for c in cfgs:
                same = torch.equal(run(c), ref)
                best = 1e9
                for _ in range(3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(args.iters):
                        run(c)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    best = min(best, e0.elapsed_time(e1) / args.iters * 1e3)
                tot[c] += best
                fl = 2.0 * m * n * k
                print(f"w8 {name:5s} M={m} cfg {c}: {best:7.1f} us  {fl / best / 1e6:7.1f} TOPS  "
                      f"identical to default pick: {same}", flush=True)
        print(f"w8 M={m} per-block GEMM total: " + "  ".join(f"cfg {c} {t:.1f} us" for c, t in tot.items()),
              flush=True)


if __name__ == "__main__":
    main()

"""Isolated cost of the LayerNorm-fold epilogues: each ViT-H projection at M rows with its plain
epilogue vs its LN-fold epilogue, plus the standalone LayerNorm the fold replaces.

    python tools/bench_lnf.py [--m 8192] [--iters 30]

HIP events on the launch stream, interleaved rounds (min of 3).
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


def layer(k, n, dev):
    q = QuantLinear(4, -1, k, n, True).to(dev)
    w = torch.randn(n, k, device=dev) * 0.02
    fake, s, z = rtn(w, -1)
    pack_linear(q, fake, s, z, torch.randn(n, device=dev) * 0.02)
    q.prepare()
    return q


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m, c = args.m, 1280
    x = torch.randn(m, c, device=dev)
    g = torch.rand(c, device=dev) + 0.5
    b = torch.randn(c, device=dev) * 0.1
    xn = torch.empty(m, c, device=dev, dtype=torch.float16)
    mu = torch.zeros(m, device=dev)
    stats = torch.zeros(m, c // 64, 2, device=dev)
    ops.layernorm(x, g, b, 1e-6, out=xn, mean_out=mu)
    cases = {}
    for name, k, n, plain, lnf in (("qkv", c, 3 * c, ops.EPI_BIAS, ops.EPI_BIAS_LNF),
                                   ("proj", c, c, ops.EPI_RESADD_F32, ops.EPI_RESADD_LNF),
                                   ("lin1", c, 4 * c, ops.EPI_BIAS_GELU, ops.EPI_GELU_LNF),
                                   ("lin2", 4 * c, c, ops.EPI_RESADD_F32, ops.EPI_RESADD_LNF)):
        q = layer(k, n, dev)
        a = torch.randn(m, k, device=dev).half()
        if plain in (ops.EPI_RESADD_F32,):
            out = torch.zeros(m, n, device=dev)
            cases[name] = lambda q=q, a=a, out=out, e=plain: q.forward_epilogue(a, e, out=out)
            cases[name + "_lnf"] = (lambda q=q, a=a, out=out, e=lnf:
                                    q.forward_lnf(a, e, out, stats, mu, gamma=g, aout=xn))
        else:
            out = torch.empty(m, n, device=dev, dtype=torch.float16)
            gw, bw = q.ln_fold_constants(g, b)
            cases[name] = lambda q=q, a=a, out=out, e=plain: q.forward_epilogue(a, e, out=out)
            cases[name + "_lnf"] = (lambda q=q, out=out, e=lnf, gw=gw, bw=bw:
                                    q.forward_lnf(xn, e, out, stats, mu, gw=gw, bw=bw, eps=1e-6))
    cases["layernorm"] = lambda: ops.layernorm(x, g, b, 1e-6, out=xn)
    # keep mu / x bounded: the residual cases accumulate into x-sized buffers, mu drifts by delta
    stream = torch.cuda.current_stream()
    times = {k: [] for k in cases}
    for _ in range(3):
        for k, f in cases.items():
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.iters):
                f()
            e1.record(stream)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / args.iters * 1e3)
            mu.zero_()
    for k in cases:
        print(f"{k:12s} {min(times[k]):8.1f} us")
    tot_plain = sum(min(times[k]) for k in ("qkv", "proj", "lin1", "lin2")) + 2 * min(times["layernorm"])
    tot_lnf = sum(min(times[k + "_lnf"]) for k in ("qkv", "proj", "lin1", "lin2"))
    print(f"block GEMMs + 2 LN: plain {tot_plain:.1f} us, folded {tot_lnf:.1f} us")


if __name__ == "__main__":
    main()

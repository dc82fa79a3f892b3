"""Interleaved A/B of global-attention kernel variants of the tuning build (SAMQ_LIB=tuning,
SAMQ_ATTN_DBG read per launch): ViT-H global geometry, B images; outputs compared with variant 0.
    SAMQ_LIB=tuning python tools/attn_variant_ab.py [dbg,dbg,...] [batch] [rounds]"""
import os
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "sam-quantization_amd"))
from samq import ops  # noqa: E402

variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,8").split(",")]
b = int(sys.argv[2]) if len(sys.argv) > 2 else 2
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 6
dev = torch.device("cuda:0")
g, heads, d = 64, 16, 80
c = heads * d
gen = torch.Generator(device=dev).manual_seed(5)
qkv = (torch.randn(b, g, g, 3 * c, device=dev, generator=gen) * 0.5).half()
bias = (torch.randn(3 * c, device=dev, generator=gen) * 0.1).half()
rh = (torch.randn(2 * g - 1, d, device=dev, generator=gen) * 0.1).half()
rw = (torch.randn(2 * g - 1, d, device=dev, generator=gen) * 0.1).half()
outs, times = {}, {v: [] for v in variants}
for v in variants:
    os.environ["SAMQ_ATTN_DBG"] = str(v)
    outs[v] = ops.rel_attention(qkv, bias, rh, rw, heads, 0, d ** -0.5)
torch.cuda.synchronize()
for _ in range(rounds):
    for v in variants:
        os.environ["SAMQ_ATTN_DBG"] = str(v)
        out = torch.empty_like(outs[v])
        for _ in range(2):
            ops.rel_attention(qkv, bias, rh, rw, heads, 0, d ** -0.5, out=out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            ops.rel_attention(qkv, bias, rh, rw, heads, 0, d ** -0.5, out=out)
        e1.record()
        torch.cuda.synchronize()
        times[v].append(e0.elapsed_time(e1) / 10 * 1e3)
ref = outs[variants[0]].float()
for v in variants:
    ts = sorted(times[v])
    err = float((outs[v].float() - ref).abs().max())
    print(f"global attention B={b} dbg={v}: median {ts[len(ts) // 2]:.1f} us  min {ts[0]:.1f} us  "
          f"max-abs vs dbg {variants[0]}: {err:.3e}", flush=True)

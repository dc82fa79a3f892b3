"""A/B of window-attention variants of the tuning build (SAMQ_LIB=tuning; SAMQ_ATTN_WIN read per
launch): accuracy against the fp32 oracle (fp16 output max-abs; W4A8 int8 store: codes off by one)
and interleaved timing at the ViT-H 2-image geometry.
    SAMQ_LIB=tuning python tools/win_variant_ab.py [variants] [rounds]"""
import os
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "sam-quantization_amd"))
sys.path.insert(0, str(REPO / "tests"))
sys.path.insert(0, str(REPO))
from samq import ops  # noqa: E402
from test_gpu_kernels import _attn_case  # noqa: E402

variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,1").split(",")]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 6
dev = torch.device("cuda:0")
torch.set_num_threads(16)
qkv16, bq, rph, rpw, ref = _attn_case(2, 64, 64, 16, 80, 14, seed=77)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
args = (t(qkv16), t(bq), t(rph), t(rpw), 16, 14, 80 ** -0.5)
s = float(np.abs(ref).max() / 100)
codes = np.clip(np.rint(ref / np.float32(s)), -128, 127)
times = {v: [] for v in variants}
first = {}
for v in variants:
    os.environ["SAMQ_ATTN_WIN"] = str(v)
    o16 = ops.rel_attention(*args).float().cpu().numpy()
    o8 = ops.rel_attention(*args, out_scale=s).cpu().numpy().astype(np.int32)
    first.setdefault("o16", o16)
    first.setdefault("o8", o8)
    print(f"window variant {v}: identical to variant {variants[0]}: fp16 {np.array_equal(o16, first['o16'])}, "
          f"int8 {np.array_equal(o8, first['o8'])}", flush=True)
    print(f"window variant {v}: fp16 out max-abs vs oracle {np.abs(o16 - ref).max():.3e}, int8 codes off by one "
          f"{float((o8 != codes).mean()):.2e} (max |d| {int(np.abs(o8 - codes).max())})", flush=True)
out = torch.empty(qkv16.shape[:3] + (1280,), dtype=torch.float16, device=dev)
for _ in range(rounds):
    for v in variants:
        os.environ["SAMQ_ATTN_WIN"] = str(v)
        for _ in range(2):
            ops.rel_attention(*args, out=out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ops.rel_attention(*args, out=out)
        e1.record()
        torch.cuda.synchronize()
        times[v].append(e0.elapsed_time(e1) / 20 * 1e3)
for v in variants:
    ts = sorted(times[v])
    print(f"window variant {v}: median {ts[len(ts) // 2]:.2f} us  min {ts[0]:.2f} us", flush=True)
# the int8-code store (W4A8 proj input): timing per variant
out8 = torch.empty(qkv16.shape[:3] + (1280,), dtype=torch.int8, device=dev)
t8 = {v: [] for v in variants}
for _ in range(rounds):
    for v in variants:
        os.environ["SAMQ_ATTN_WIN"] = str(v)
        for _ in range(2):
            ops.rel_attention(*args, out_scale=s, out=out8)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ops.rel_attention(*args, out_scale=s, out=out8)
        e1.record()
        torch.cuda.synchronize()
        t8[v].append(e0.elapsed_time(e1) / 20 * 1e3)
for v in variants:
    ts = sorted(t8[v])
    print(f"window variant {v} int8 store: median {ts[len(ts) // 2]:.2f} us  min {ts[0]:.2f} us", flush=True)

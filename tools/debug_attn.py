"""Localise attention-kernel errors: per (image, head, query row) max-abs vs the oracle."""
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "sam-quantization_amd"), str(REPO / "tests")]
from test_gpu_kernels import _attn_case  # noqa: E402
from samq import ops  # noqa: E402

dev = torch.device("cuda:0")
for (b, h, w, heads, d, win) in [(1, 64, 64, 2, 80, 0), (2, 64, 64, 2, 80, 0), (2, 64, 64, 1, 80, 0),
                                 (2, 32, 32, 2, 80, 0), (2, 64, 64, 2, 64, 0), (1, 64, 64, 16, 80, 0)]:
    qkv16, bq, rph, rpw, ref = _attn_case(b, h, w, heads, d, win, seed=h * 100 + w + d + win)
    out = ops.rel_attention(torch.from_numpy(qkv16).to(dev), torch.from_numpy(bq).to(dev),
                            torch.from_numpy(rph).to(dev), torch.from_numpy(rpw).to(dev), heads, win, d ** -0.5)
    o = out.float().cpu().numpy().reshape(b, h, w, heads, d)
    r = ref.reshape(b, h, w, heads, d)
    e = np.abs(o - r)
    print(f"case b={b} S={h} heads={heads} d={d}: max {e.max():.3e}")
    per = e.max(axis=(2, 4))  # (b, h, heads)
    for bi in range(b):
        for hh in range(heads):
            rows = np.nonzero(per[bi, :, hh] > 5e-3)[0]
            print(f"   img {bi} head {hh}: max {per[bi, :, hh].max():.3e} bad rows {rows[:20].tolist()}{'...' if len(rows) > 20 else ''}")
        if bi == 0 and per[bi].max() > 5e-3:
            row = int(np.argmax(per[bi].max(axis=1)))
            cols = e[bi, row].max(axis=(1, 2))
            print(f"   img0 worst row {row}: bad cols {np.nonzero(cols > 5e-3)[0][:32].tolist()}")

"""Debug aid: ping-pong GEMM configs vs the v3 kernel on small K / M / N, error pattern per tile."""
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "sam-quantization_amd"))
from samq import ops  # noqa: E402
from samq.gptq import rtn, pack_linear  # noqa: E402
from samq.quant_linear import QuantLinear  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
cfgs = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "51,52").split(",")]
for (m, k, n) in [(256, 1280, 1280), (2048, 1280, 3840), (4096, 1280, 3840), (16384, 1280, 3840), (16384, 256, 256)]:
    q = QuantLinear(4, -1, k, n, True).to(dev)
    w = torch.randn(n, k, device=dev) * 0.02
    fake, s, z = rtn(w)
    pack_linear(q, fake, s, z, torch.randn(n, device=dev) * 0.02)
    packed = q.prepare()
    a = torch.randn(m, k, device=dev).half()
    ref = ops.w4a16_gemm(a, packed, q.scales, q.qzeros, q.bias, n, -1, ops.EPI_BIAS, cfg=22).float()
    for c in cfgs:
        if n % 256:
            continue
        out = ops.w4a16_gemm(a, packed, q.scales, q.qzeros, q.bias, n, -1, ops.EPI_BIAS, cfg=c).float()
        torch.cuda.synchronize()
        err = (out - ref).abs()
        bad = err > 1e-2
        rows = bad.any(1).nonzero().flatten().tolist()
        cols = bad.any(0).nonzero().flatten().tolist()
        print(f"M={m} K={k} N={n} cfg {c}: maxdiff {err.max().item():.3e} bad {int(bad.sum())} "
              f"rows {rows[:8]}..({len(rows)}) cols {cols[:8]}..({len(cols)}) "
              f"ratio {float((out[bad] / ref[bad]).mean()) if bad.any() else 0:.3f}")

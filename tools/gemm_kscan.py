"""Time the W4A16 GEMM at fixed M, N over K to split fixed per-tile cost (prologue / epilogue /
tail) from the per-K-step cost:  t(K) = a + b*K."""
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "sam-quantization_amd"))
from samq import ops  # noqa: E402
from samq.gptq import rtn, pack_linear  # noqa: E402
from samq.quant_linear import QuantLinear  # noqa: E402

dev = torch.device("cuda")
m = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
cfgs = [int(c) for c in (sys.argv[2] if len(sys.argv) > 2 else "22").split(",")]
for n, epi in ((3840, ops.EPI_BIAS), (1280, ops.EPI_RESADD_F32)):
    for cfg in cfgs:
        pts = []
        for k in ([int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else (640, 1280, 2560, 5120)):
            q = QuantLinear(4, -1, k, n, True).to(dev)
            fake, s, z = rtn(torch.randn(n, k, device=dev) * 0.02)
            pack_linear(q, fake, s, z, torch.randn(n, device=dev) * 0.02)
            a = torch.randn(m, k, device=dev).half()
            out = torch.zeros(m, n, device=dev, dtype=torch.float32 if epi == ops.EPI_RESADD_F32 else torch.float16)
            packed = q.prepare()
            f = lambda: ops.w4a16_gemm(a, packed, q.scales, q.qzeros, q.bias, n, -1, epi, out=out, cfg=cfg)  # noqa
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            best = 1e9
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    f()
                e1.record()
                torch.cuda.synchronize()
                best = min(best, e0.elapsed_time(e1) / 20 * 1e3)
            pts.append((k, best))
        ks = torch.tensor([p[0] for p in pts], dtype=torch.float64)
        ts = torch.tensor([p[1] for p in pts], dtype=torch.float64)
        A = torch.stack([torch.ones_like(ks), ks], 1)
        sol = torch.linalg.lstsq(A, ts[:, None]).solution.squeeze()
        print(f"N={n} cfg {cfg}: " + "  ".join(f"K={k}: {t:.1f}us ({2*m*n*k/t/1e6:.0f} TF)" for k, t in pts)
              + f" | fit t = {sol[0]:.1f} + {sol[1]*1000:.2f}*K/1000 us")

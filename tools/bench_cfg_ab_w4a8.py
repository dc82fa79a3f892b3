"""Interleaved in-graph A/B of per-layer W4A8 int8-MFMA tile configs (ViT-H, B=8, bench.py's model
setup): each variant is captured once, the graphs replayed in rounds A B C A B C ...
usage: python tools/bench_cfg_ab_w4a8.py [lanes] [rounds]"""
import sys
import time
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "sam-quantization_amd"))
import samq  # noqa: E402
from samq.synthetic import random_quant_encoder  # noqa: E402

dev = torch.device("cuda:0")
lanes = int(sys.argv[1]) if len(sys.argv) > 1 else 2
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 6
VARIANTS = {"pick": {}, "res=ln32": {"res": "ln32"}}   # round 4: residual adds in the LayerNorm-q kernels
if len(sys.argv) > 3:   # variants as "name:layer=cfg,res=ln32,skip_win=1;name:..." (pick always first)
    VARIANTS = {"pick": {}}
    for v in sys.argv[3].split(";"):
        name, spec = v.split(":")
        VARIANTS[name] = {kv.split("=")[0]: (kv.split("=")[1] if kv.split("=")[0] == "res" else int(kv.split("=")[1]))
                          for kv in spec.split(",")}

enc = random_quant_encoder("vit_h", -1, device=dev)
enc.half()
samq.make_act_quant(enc)
gcal = torch.Generator(device="cpu").manual_seed(99)
samq.calibrate_act_quant(enc, enc.module_forward, [torch.randn((1, 3, 1024, 1024), generator=gcal).to(dev, torch.float16)])
eng = enc.engine()
g = torch.Generator(device=dev).manual_seed(1234)
img = torch.randn((8, 3, 1024, 1024), generator=g, device=dev, dtype=torch.float16)
graphs, ref = {}, None
rpw0 = eng.ln_rpw   # the engine's default is "pick"
for name, cfg in VARIANTS.items():
    eng.res_mode = cfg.get("res", "epi")
    eng.ln_rpw = cfg.get("ln_rpw", rpw0)
    eng.lane_priority = cfg.get("prio", 0)   # round 6: lane 0's stream at high priority
    eng.rowsums = {0: False, 1: True, 2: "ln"}[cfg.get("rowsums", 1)]   # round 6: producer-side row sums
    eng.skip = frozenset(k[5:] for k in cfg if k.startswith("skip_"))   # timing-only
    for p in eng.plans:
        for lay in ("qkv", "proj", "lin1", "lin2"):
            getattr(p, lay).i8_cfg = cfg.get(lay, 0)
    graph, out = eng.capture(img, lanes=lanes)
    graph.replay()
    torch.cuda.synchronize()
    ref = out.clone() if ref is None else ref
    graphs[name] = (graph, torch.equal(out, ref))
times = {k: [] for k in graphs}
for _ in range(rounds):
    for name, (graph, _) in graphs.items():
        for _ in range(2):
            graph.replay()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            graph.replay()
        torch.cuda.synchronize()
        times[name].append((time.perf_counter() - t) / 5 * 1e3)
for name, ts in times.items():
    ts = sorted(ts)
    med = ts[len(ts) // 2]
    print(f"lanes={lanes} {name:18s} median {med:.3f} ms/step  min {ts[0]:.3f}  ({8 / med * 1e3:.1f} img/s)  "
          f"bit-identical: {graphs[name][1]}")

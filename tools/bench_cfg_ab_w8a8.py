"""Interleaved A/B of per-layer W8 tile configs INSIDE the timed W8A8 HIP graph (fq_vit vit_b,
B=1): each variant is captured once and the graphs are replayed in rounds A B C A B C ...
usage: python tools/bench_cfg_ab_w8a8.py [rounds] ["name:layer=cfg,layer=cfg;name:..."]"""
import sys
import time
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "sam-quantization_amd"))
from samq.synthetic import random_fq_encoder  # noqa: E402

dev = torch.device("cuda:0")
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 8
VARIANTS = {"pick": {}}
spec = sys.argv[2] if len(sys.argv) > 2 else (
    "all87:qkv=87,proj=87,lin1=87,lin2=87;all88:qkv=88,proj=88,lin1=88,lin2=88;"
    "all89:qkv=89,proj=89,lin1=89,lin2=89")
for v in spec.split(";"):
    name, kv = v.split(":")
    VARIANTS[name] = {x.split("=")[0]: int(x.split("=")[1]) for x in kv.split(",")}

enc = random_fq_encoder("vit_b", device=dev)
eng = enc.engine()
g = torch.Generator(device=dev).manual_seed(1234)
img = torch.randn((1, 3, 1024, 1024), generator=g, device=dev)
graphs, ref = {}, None
rpw0, lanes0 = eng.ln_rpw, eng.row_lanes   # the engine's defaults are "pick"
for name, cfg in VARIANTS.items():
    eng.ln_rpw = cfg.get("ln_rpw", rpw0)
    eng.row_lanes = cfg.get("lanes", lanes0)   # round 6: one image as two row lanes
    eng.v16 = bool(cfg.get("v16", 1))            # round 6: fp16 V copy for the global attention
    for bl in eng.blocks:
        for lay in ("qkv", "proj", "lin1", "lin2"):
            bl[lay]["cfg"] = cfg.get(lay, 0)
    graph, out = eng.capture(img)
    graph.replay()
    torch.cuda.synchronize()
    ref = out.clone() if ref is None else ref
    graphs[name] = (graph, torch.equal(out, ref))
times = {k: [] for k in graphs}
for _ in range(rounds):
    for name, (graph, _) in graphs.items():
        for _ in range(3):
            graph.replay()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(20):
            graph.replay()
        torch.cuda.synchronize()
        times[name].append((time.perf_counter() - t) / 20 * 1e3)
for name, ts in times.items():
    ts.sort()
    print(f"w8a8 {name:12s} median {ts[len(ts) // 2]:.4f} ms/step  min {ts[0]:.4f}  "
          f"({1 / ts[len(ts) // 2] * 1e3:.1f} img/s)  bit-identical: {graphs[name][1]}", flush=True)

"""Interleaved A/B of per-layer W4A16 tile configs INSIDE the timed HIP graph (ViT-H, B=4):
each variant is captured once and the graphs are replayed in rounds A B C A B C ... so box drift
hits every variant alike.  usage: python tools/bench_cfg_ab.py [lanes] [rounds]"""
import sys
import time
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "sam-quantization_amd"))
from samq.synthetic import random_quant_encoder  # noqa: E402

dev = torch.device("cuda:0")
lanes = int(sys.argv[1]) if len(sys.argv) > 1 else 2
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 6
VARIANTS = {"pick": {}, "proj=22": {"proj": 22}, "proj=22,lin2=22": {"proj": 22, "lin2": 22},
            "proj=22,lin1=22": {"proj": 22, "lin1": 22}, "proj=25,lin1=25": {"proj": 25, "lin1": 25}}
if len(sys.argv) > 3:   # variants as "name:layer=cfg,layer=cfg;name:..." (pick always first)
    VARIANTS = {"pick": {}}
    for v in sys.argv[3].split(";"):
        name, spec = v.split(":")
        VARIANTS[name] = {kv.split("=")[0]: (kv.split("=")[1] if kv.split("=")[0] == "res" else int(kv.split("=")[1]))
                          for kv in spec.split(",")}

import os  # noqa: E402
enc = random_quant_encoder("vit_h", int(os.environ.get("SAMQ_AB_GS", "-1")), device=dev)   # groupsize
eng = enc.engine()
g = torch.Generator(device=dev).manual_seed(1234)
img = torch.randn((4, 3, 1024, 1024), generator=g, device=dev, dtype=torch.float16)
graphs, ref = {}, None
for name, cfg in VARIANTS.items():
    eng.ln_rpw = cfg.get("ln_rpw", 0)
    eng.lane_priority = cfg.get("prio", 0)   # round 6: lane 0's stream at high priority
    eng.res_mode = cfg.get("res", "epi")   # where the proj / lin2 residual adds run (engine.res_mode)
    eng.skip = frozenset(k[5:] for k in cfg if k.startswith("skip_"))   # timing-only: "skip_ln=1" etc.
    for p in eng.plans:
        for lay in ("qkv", "proj", "lin1", "lin2"):
            getattr(p, lay).gemm_cfg = cfg.get(lay, 0)
    envs = {k[4:]: str(v) for k, v in cfg.items() if k.startswith("env_")}   # tuning-build knobs, e.g.
    for k, v in envs.items():                                                # "env_SAMQ_ATTN_WIN=8"
        os.environ[k] = v
    graph, out = eng.capture(img, lanes=lanes)
    for k in envs:
        del os.environ[k]
    graph.replay()
    torch.cuda.synchronize()
    ref = out.clone() if ref is None else ref
    graphs[name] = (graph, torch.equal(out, ref), float((out.float() - ref.float()).abs().max()))
times = {k: [] for k in graphs}
for _ in range(rounds):
    for name, (graph, *_) in graphs.items():
        for _ in range(3):
            graph.replay()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(10):
            graph.replay()
        torch.cuda.synchronize()
        times[name].append((time.perf_counter() - t) / 10 * 1e3)
for name, ts in times.items():
    ts.sort()
    print(f"lanes={lanes} {name:16s} median {ts[len(ts) // 2]:.3f} ms/step  min {ts[0]:.3f}  "
          f"({4 / ts[len(ts) // 2] * 1e3:.1f} img/s)  bit-identical: {graphs[name][1]} "
          f"(max-abs vs pick {graphs[name][2]:.2e})", flush=True)

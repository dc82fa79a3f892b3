"""Encoder step time vs ``lanes`` (image groups as concurrent kernel chains on separate HIP
streams, one HIP graph): ViT-H W4A16 at B=4 / B=8 and W4A8 at B=8; checks lanes>1 is
bit-identical to lanes=1."""
import sys
import time
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "sam-quantization_amd"))
import samq  # noqa: E402
from samq.synthetic import random_quant_encoder  # noqa: E402

dev = torch.device("cuda:0")
which = sys.argv[1:] or ["w4a16"]


def step_ms(fn, n=12):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


for mode in which:
    enc = random_quant_encoder("vit_h", -1, device=dev)
    if mode == "w4a8":
        enc.half()
        samq.make_act_quant(enc)
        gcal = torch.Generator(device="cpu").manual_seed(99)
        cal = torch.randn((1, 3, 1024, 1024), generator=gcal).to(dev, torch.float16)
        samq.calibrate_act_quant(enc, enc.module_forward, [cal])
    eng = enc.engine()
    for batch in ((4, 8) if mode == "w4a16" else (8,)):
        g = torch.Generator(device=dev).manual_seed(1234)
        img = torch.randn((batch, 3, 1024, 1024), generator=g, device=dev, dtype=torch.float16)
        base = None
        for lanes in (1, 2, 4):
            graph, out = eng.capture(img, lanes=lanes)
            ms = step_ms(graph.replay)
            ms_eager = step_ms(lambda: eng(img, lanes=lanes))
            graph.replay()
            torch.cuda.synchronize()
            if base is None:
                base = out.clone()
            same = torch.equal(out, base)
            print(f"{mode} B={batch} lanes={lanes}: {ms:.2f} ms/step  {batch / ms * 1e3:.1f} img/s  "
                  f"eager {ms_eager:.2f} ms  bit-identical to lanes=1: {same}", flush=True)
            del graph
        if mode == "w4a16":   # lin1 tile A/B inside the 2-lane graph (cfg 22 vs the default pick)
            for cfg in (22, 0):
                for p in eng.plans:
                    p.lin1.gemm_cfg = cfg
                graph, out = eng.capture(img, lanes=2)
                ms = step_ms(graph.replay)
                graph.replay()
                torch.cuda.synchronize()
                print(f"{mode} B={batch} lanes=2 lin1 cfg {cfg or 'pick'}: {ms:.2f} ms/step  "
                      f"bit-identical to lanes=1: {torch.equal(out, base)}", flush=True)
                del graph

"""Where does the W4A16 engine's output for image 0 start to depend on the batch?"""
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "sam-quantization_amd"), str(REPO / "tests")]
from _encoder_helpers import oracle_vith, product_encoder  # noqa: E402
from oracle import synth  # noqa: E402
from samq import ops  # noqa: E402

cuda = torch.device("cuda")
cfg, st, names, q = oracle_vith(4, 7, global_idx=(3,))
enc = product_encoder(cfg, st, names, q, -1, cuda)
eng = enc.engine()
x1 = torch.from_numpy(synth.make_images(1, seed=3)).to(cuda)
x2 = torch.cat([x1, torch.flip(x1, dims=[-1])])
for k in range(0, 5):
    a = eng.tokens(x1, upto=k)
    b = eng.tokens(x2, upto=k)[:1]
    print(f"after {k} blocks: max diff {(a - b).abs().max().item():.3e}")
# per-op check inside block 0 with identical inputs
bufs1, bufs2 = eng.buffers(1), eng.buffers(2)
eng.embed(x1, bufs1["x"])
eng.embed(x2, bufs2["x"])
p = eng.plans[0]
for nm, fn in (("ln1", lambda bf: ops.layernorm(bf["x"], p.ln1_w, p.ln1_b, p.ln1_eps, out=bf["xn"])),
               ("qkv", lambda bf: p.qkv.forward_epilogue(bf["xn"], ops.EPI_BIAS, out=bf["qkv"])),
               ("attn", lambda bf: ops.rel_attention(bf["qkv"], p.qkv_bias, p.relh, p.relw, p.heads, p.window, p.scale,
                                                     out=bf["att"])),
               ("proj", lambda bf: p.proj.forward_epilogue(bf["att"], ops.EPI_RESADD_F32, out=bf["x"]))):
    fn(bufs1)
    fn(bufs2)
    key = {"ln1": "xn", "qkv": "qkv", "attn": "att", "proj": "x"}[nm]
    print(nm, (bufs1[key][:1].float() - bufs2[key][:1].float()).abs().max().item())

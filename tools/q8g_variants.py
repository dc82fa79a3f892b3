"""Tuning-build check of the W8A8 global attention variants (SAMQ_Q8G_PVAR, row64 kernel): codes of
each variant vs the round-4 form (0) and vs the test's numpy reference, on test_rel_attention_q8's
1 x 64 x 64 global case.  usage: SAMQ_LIB=tuning python tools/q8g_variants.py"""
import os
import subprocess
import sys

if len(sys.argv) > 1:   # child: one variant, codes to the given file
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "sam-quantization_amd"))
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
    from samq import ops
    from test_w8a8 import _attn_ref
    cuda = torch.device("cuda:0")
    b, hw, window, heads, d = 1, 64, 0, 2, 64
    c = heads * d
    rng = np.random.Generator(np.random.PCG64(hw + window))
    qkv = rng.integers(-128, 128, (b, hw, hw, 3 * c), dtype=np.int8)
    relh = (rng.standard_normal((2 * hw - 1, d), dtype=np.float32) * 0.5).astype(np.float32)
    relw = (rng.standard_normal((2 * hw - 1, d), dtype=np.float32) * 0.5).astype(np.float32)
    bias = (rng.standard_normal(3 * c, dtype=np.float32) * 0.3).astype(np.float32)
    s_qkv, s1, s2, s_o = np.float32(0.02), np.float32(2.0 / 127.5), np.float32(6.0 / 127.5), np.float32(2.6 / 127.5)
    out = ops.rel_attention_q8(torch.from_numpy(qkv).to(cuda), torch.from_numpy(bias).to(cuda),
                               torch.from_numpy(relh).to(cuda), torch.from_numpy(relw).to(cuda), heads, window,
                               d ** -0.5, float(s_qkv), float(s1), float(s2), float(s_o))
    np.save(sys.argv[1], out.cpu().numpy())
    if not os.path.exists(sys.argv[1] + ".ref.npy"):
        np.save(sys.argv[1] + ".ref.npy", _attn_ref(qkv, bias, relh, relw, heads, window, s_qkv, s1, s2, s_o))
    sys.exit(0)

import numpy as np
res = {}
for v in (0, 1, 2, 3):
    f = f"/tmp/q8g_v{v}.npy"
    env = dict(os.environ, SAMQ_LIB="tuning", SAMQ_Q8G_PVAR=str(v))
    r = subprocess.run([sys.executable, __file__, f], env=env)
    if r.returncode:
        sys.exit(r.returncode)
    res[v] = np.load(f).astype(np.int32)
ref = np.load("/tmp/q8g_v0.npy.ref.npy")
for v, o in res.items():
    d0 = np.abs(o - res[0])
    dr = np.abs(o - ref)
    print(f"PVAR {v}: vs round-4 max {d0.max()} frac {np.mean(d0 > 0):.2e} | vs reference max {dr.max()} frac>0 {np.mean(dr > 0):.2e}")

"""Phase timing of the window-attention kernel from a stamps build (diagnostic only).

    SAMQ_LIB=<abs path>/build_ab/attention_stamps.so python tools/attn_stamps.py
Stamps (s_memtime, shader clock) per wave: 0 start, 1 loads issued, 2 after the K/V barrier,
then per pass p: 3+5p rel-pos done, 4+5p QK done, 5+5p softmax done, 6+5p PV done, 7+5p stored.
"""
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "sam-quantization_amd"))
from samq import ops, _lib  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    b, g, heads, d = 2, 64, 16, 80
    c = heads * d
    qkv = (torch.randn(b, g, g, 3 * c, device=dev) * 0.5).half()
    bias = (torch.randn(3 * c, device=dev) * 0.1).half()
    rh = (torch.randn(27, d, device=dev) * 0.1).half()
    rw = (torch.randn(27, d, device=dev) * 0.1).half()
    out = torch.empty(b, g, g, c, device=dev, dtype=torch.float16)
    for _ in range(5):
        ops.rel_attention(qkv, bias, rh, rw, heads, 14, d ** -0.5, out=out)
    torch.cuda.synchronize()
    n = 4096 * 4 * 16
    buf = (ctypes.c_ulonglong * n)()
    lib = _lib.load()
    assert lib.samq_debug_stamps(buf, n) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 4, 16).astype(np.int64)[:800]
    t0 = st[:, :, 0].min()
    print("kernel span (cycles):", st[:, :, :].max() - t0)
    names = ["loads issued", "K/V barrier", "p0 relpos", "p0 QK", "p0 softmax", "p0 PV", "p0 store",
             "p1 relpos", "p1 QK", "p1 softmax", "p1 PV", "p1 store"]
    for w in range(4):
        row = st[:, w, :]
        np1 = 13 if w < 3 else 8
        dif = np.diff(row[:, :np1], axis=1)
        print(f"wave {w}: " + "  ".join(f"{names[i]} {np.median(dif[:, i]):7.0f}" for i in range(np1 - 1)))
    life = np.maximum(st[:, :3, 12].max(1), st[:, 3, 7]) - st[:, :, 0].min(1)
    print("WG lifetime median", np.median(life))


if __name__ == "__main__":
    main()

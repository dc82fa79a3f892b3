"""gptq_triton.fused_mlp API parity: QuantLlamaMLP / triton_llama_mlp_4 /
make_fused_mlp.  Oracle: fp32 silu(A.W1) * (A.W2) with the G1-decoded int4 weights
(``oracle.gptq_pack.dequant_g1``); tolerance: fp16 output rounding of values up to |8|."""
import numpy as np
import pytest
import torch
import torch.nn as nn

from oracle import gptq_pack


def _packed(k, n, seed, groupsize=-1):
    rng = np.random.Generator(np.random.PCG64(seed))
    w = rng.standard_normal((n, k), dtype=np.float32) * np.float32(0.05)
    fake, s, z = gptq_pack.rtn_quantize_linear(w, groupsize)
    return gptq_pack.pack_linear(fake, s, z, groupsize)


def test_fused_mlp_asserts_and_swap_cpu():
    import samq
    from samq.fused_mlp import QuantLlamaMLP, make_fused_mlp, triton_llama_mlp_4
    qw, qz, sc = (torch.from_numpy(x) for x in _packed(256, 256, 1))
    qw2, qz2, sc2 = (torch.from_numpy(x) for x in _packed(256, 512, 2))
    a = torch.zeros(4, 256, dtype=torch.float16)
    with pytest.raises(AssertionError, match="same shape"):
        triton_llama_mlp_4(-1, a, qw, sc, qz, qw2, sc2, qz2)
    with pytest.raises(AssertionError, match="multiple of 8"):
        triton_llama_mlp_4(-1, torch.zeros(4, 128, dtype=torch.float16), qw, sc, qz, qw, sc, qz)

    class LlamaMLP(nn.Module):
        def __init__(self):
            super().__init__()
            self.gate_proj = samq.QuantLinear(4, -1, 256, 512, False)
            self.up_proj = samq.QuantLinear(4, -1, 256, 512, False)
            self.down_proj = samq.QuantLinear(4, -1, 512, 256, False)

    model = nn.Sequential(nn.Identity(), LlamaMLP())
    make_fused_mlp(model)
    assert isinstance(model[1], QuantLlamaMLP) and model[1].infeatures == 256 and model[1].outfeatures == 256
    assert set(n for n, _ in model[1].named_buffers()) >= {"gate_proj_qweight", "up_proj_scales", "down_proj.qweight"}


@pytest.mark.gpu
@pytest.mark.parametrize("groupsize", [-1, 128])
def test_triton_llama_mlp_4_vs_oracle(cuda, groupsize):
    from samq.fused_mlp import triton_llama_mlp_4
    k, n, m = 1024, 768, 77
    g, u = _packed(k, n, 3, groupsize), _packed(k, n, 4, groupsize)
    rng = np.random.Generator(np.random.PCG64(5))
    a = rng.standard_normal((m, k), dtype=np.float32).astype(np.float16)
    wg = gptq_pack.dequant_g1(g[0], g[2], g[1], groupsize)
    wu = gptq_pack.dequant_g1(u[0], u[2], u[1], groupsize)
    xg, xu = a.astype(np.float32) @ wg, a.astype(np.float32) @ wu
    ref = xg / (1 + np.exp(-xg)) * xu
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(cuda)  # noqa: E731
    out = triton_llama_mlp_4(groupsize, t(a).view(1, m, k), t(g[0]), t(g[2]), t(g[1]), t(u[0]), t(u[2]), t(u[1]))
    assert out.shape == (1, m, n) and out.dtype == torch.float16
    err = np.abs(out.float().cpu().numpy()[0] - ref).max()
    assert err <= 2e-3 * max(1.0, np.abs(ref).max()), err

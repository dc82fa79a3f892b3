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
@pytest.mark.parametrize("groupsize,m", [(-1, 77), (128, 77), (-1, 1), (128, 300), (-1, 1000)])
def test_triton_llama_mlp_4_vs_oracle(cuda, groupsize, m):
    """One fused launch (samq_w4a16_gated_mlp) vs the fp32 oracle, M from decode (1) to 1000."""
    from samq.fused_mlp import triton_llama_mlp_4
    k, n = 1024, 768
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


@pytest.mark.gpu
def test_gated_mlp_one_launch_matches_two_gemms_and_module(cuda):
    """The fused kernel equals the unfused composition (two EPI_F32 int4 GEMMs + samq_silu_mul) up
    to fp16 output rounding, and QuantLlamaMLP.forward (cached interleaved operands) runs it."""
    import samq
    from samq import _lib, ops
    from samq.fused_mlp import QuantLlamaMLP
    k, n, m = 512, 1024, 4096
    g, u = _packed(k, n, 6), _packed(k, n, 7)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(cuda)  # noqa: E731
    a = (torch.randn(m, k, generator=torch.Generator().manual_seed(3)) * 0.5).half().to(cuda)
    gp, up = ops.w4_repack(t(g[0])), ops.w4_repack(t(u[0]))
    w2, s2, z2 = ops.w4_interleave32(gp, up, t(g[2]), t(u[2]), t(g[1]), t(u[1]), n)
    fused = ops.w4a16_gated_mlp(a, w2, s2, z2, n, -1)
    xg = ops.w4a16_gemm(a, gp, t(g[2]), t(g[1]), None, n, -1, ops.EPI_F32)
    xu = ops.w4a16_gemm(a, up, t(u[2]), t(u[1]), None, n, -1, ops.EPI_F32)
    ref = torch.empty(m, n, dtype=torch.float16, device=cuda)
    _lib.check(_lib.load().samq_silu_mul(xg.data_ptr(), xu.data_ptr(), ref.data_ptr(), ref.numel(), ops._stream()),
               "silu_mul")
    d = (fused.float() - ref.float()).abs()
    tol = 2e-3 * ref.float().abs() + 1e-3
    assert bool((d <= tol).all()), float(d.max())

    gate = samq.QuantLinear(4, -1, k, n, False).to(cuda)
    upl = samq.QuantLinear(4, -1, k, n, False).to(cuda)
    down = samq.QuantLinear(4, -1, n, k, False).to(cuda)
    for lin, pk in ((gate, g), (upl, u)):
        lin.qweight.copy_(t(pk[0]))
        lin.qzeros.copy_(t(pk[1]))
        lin.scales.copy_(t(pk[2]))
    dq, dz, ds = _packed(n, k, 8)
    down.qweight.copy_(t(dq))
    down.qzeros.copy_(t(dz))
    down.scales.copy_(t(ds))
    mlp = QuantLlamaMLP(gate, down, upl)
    y = mlp(a.view(2, m // 2, k))
    y_ref = down(ref.view(2, m // 2, n))
    assert y.shape == (2, m // 2, k)
    assert (y.float() - y_ref.float()).abs().max().item() <= 5e-3 * max(1.0, y_ref.float().abs().max().item())
    assert mlp._gated is not None and mlp(a.view(2, m // 2, k)).equal(y)
    mlp.up_proj_scales.mul_(2)            # in-place weight update: the cached operands are rebuilt
    y2 = mlp(a.view(2, m // 2, k))
    assert (y2.float() - 2 * y.float()).abs().max().item() <= 1e-2 * max(1.0, y.float().abs().max().item())

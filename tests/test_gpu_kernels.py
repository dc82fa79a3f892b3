"""GPU parity of the HIP kernels vs the CPU oracle (called through the C ABI).

Tolerances (stated per test): fp16 outputs are compared at a few fp16 ulps of the output
magnitude against an fp32 oracle fed the SAME fp16 inputs and the SAME packed int4 weights.
"""
import math

import numpy as np
import pytest
import torch

from oracle import gptq_pack, sam_ref

pytestmark = pytest.mark.gpu


def _packed_layer(k, n, groupsize, seed, zero_quirk=True):
    rng = np.random.Generator(np.random.PCG64(seed))
    w = rng.standard_normal((n, k), dtype=np.float32) * np.float32(0.02)
    if zero_quirk:
        w[5] = np.abs(w[5])  # a zero point of 0 (quirk 4)
    fake, s, z = gptq_pack.rtn_quantize_linear(w, groupsize)
    qw, qz, sc = gptq_pack.pack_linear(fake, s, z, groupsize)
    bias = (rng.standard_normal(n, dtype=np.float32) * np.float32(0.02)).astype(np.float16)
    return qw, qz, sc, bias


def _dev(a, cuda):
    return torch.from_numpy(np.ascontiguousarray(a)).to(cuda)


def _close(out, ref, rel):
    out = out.float().cpu().numpy() if torch.is_tensor(out) else out
    err = np.abs(out - ref).max()
    scale = max(1.0, float(np.abs(ref).max()))
    assert err <= rel * scale, f"max-abs {err:.3e} > {rel * scale:.3e}"
    return err


CFGS = [(1, 512), (2, 256), (3, 256), (4, 192), (5, 96), (6, 512), (7, 512), (9, 512), (21, 512), (22, 512),
        (23, 256), (24, 256), (25, 512), (26, 192)]


@pytest.mark.parametrize("cfg,n", CFGS)
@pytest.mark.parametrize("groupsize", [-1, 128])
def test_w4a16_gemm_configs(cuda, cfg, n, groupsize):
    from samq import ops
    m, k = 333, 1280  # ragged M
    qw, qz, sc, bias = _packed_layer(k, n, groupsize, seed=cfg * 7 + (groupsize > 0))
    rng = np.random.Generator(np.random.PCG64(cfg))
    a = rng.standard_normal((m, k), dtype=np.float32).astype(np.float16)
    ref = gptq_pack.matmul4_g1(a, qw, sc, qz, groupsize, bias)
    packed = ops.w4_repack(_dev(qw, cuda))
    out = ops.w4a16_gemm(_dev(a, cuda), packed, _dev(sc, cuda), _dev(qz, cuda), _dev(bias, cuda), n, groupsize,
                         ops.EPI_BIAS, cfg=cfg)
    torch.cuda.synchronize()
    # fp16 output rounding (2^-11 rel) + grouped fp16(q*s) weight rounding
    _close(out, ref, 2e-3 if groupsize == -1 else 4e-3)


@pytest.mark.parametrize("epi", ["gelu", "resadd", "f32"])
def test_w4a16_gemm_epilogues(cuda, epi):
    from samq import ops
    m, k, n = 517, 2560, 768
    qw, qz, sc, bias = _packed_layer(k, n, -1, seed=11)
    rng = np.random.Generator(np.random.PCG64(12))
    a = rng.standard_normal((m, k), dtype=np.float32).astype(np.float16)
    y = gptq_pack.matmul4_g1(a, qw, sc, qz, -1, bias)
    packed = ops.w4_repack(_dev(qw, cuda))
    args = (_dev(a, cuda), packed, _dev(sc, cuda), _dev(qz, cuda), _dev(bias, cuda), n, -1)
    if epi == "gelu":
        ref = sam_ref.gelu_erf(torch.from_numpy(y)).numpy()
        out = ops.w4a16_gemm(*args, ops.EPI_BIAS_GELU)
        _close(out, ref, 2e-3)
    elif epi == "resadd":
        r0 = rng.standard_normal((m, n), dtype=np.float32)
        res = _dev(r0, cuda)
        ops.w4a16_gemm(*args, ops.EPI_RESADD_F32, out=res)
        _close(res, r0 + y, 2e-5)
    else:
        out = ops.w4a16_gemm(*args, ops.EPI_F32)
        _close(out, y, 2e-5)


def _epi_check(ops, cuda, a, y, packed, sc, qz, bias, n, groupsize, epi, cfg, rng):
    args = (_dev(a, cuda), packed, _dev(sc, cuda), _dev(qz, cuda), _dev(bias, cuda), n, groupsize)
    tol = 2e-3 if groupsize == -1 else 4e-3
    if epi == "bias":
        _close(ops.w4a16_gemm(*args, ops.EPI_BIAS, cfg=cfg), y, tol)
    elif epi == "gelu":
        _close(ops.w4a16_gemm(*args, ops.EPI_BIAS_GELU, cfg=cfg), sam_ref.gelu_erf(torch.from_numpy(y)).numpy(), tol)
    elif epi == "resadd":
        r0 = rng.standard_normal(y.shape, dtype=np.float32)
        res = _dev(r0, cuda)
        ops.w4a16_gemm(*args, ops.EPI_RESADD_F32, out=res, cfg=cfg)
        _close(res, r0 + y, 2e-5 if groupsize == -1 else 4e-3)
    else:
        _close(ops.w4a16_gemm(*args, ops.EPI_F32, cfg=cfg), y, 2e-5 if groupsize == -1 else 4e-3)


@pytest.mark.parametrize("cfg", [55, 56, 57, 58, 62, 64, 65, 100, 101, 104, 107, 108, 109, 110, 111])
@pytest.mark.parametrize("epi", ["bias", "gelu", "resadd", "f32"])
def test_w4a16_gemm_pingpong(cuda, cfg, epi):
    """v6 ping-pong kernels (256-row tiles, 2 staggered wave groups, 3/4-slot LDS-DMA rings):
    ragged M, short and long K (1 .. 40 K tiles, so the ring prologue / retire paths all run).
    cfg 104 (transposed accumulators, f16-staged epilogue) has the f16 epilogues only and refuses
    the f32 ones with NotImplementedError (SAMQ_ERR_UNSUPPORTED)."""
    from samq import ops
    if cfg == 104 and epi in ("resadd", "f32"):
        qw, qz, sc, bias = _packed_layer(256, 256, -1, seed=104)
        a = torch.zeros((256, 256), dtype=torch.float16, device=cuda)
        e = ops.EPI_RESADD_F32 if epi == "resadd" else ops.EPI_F32
        out = torch.zeros((256, 256), dtype=torch.float32, device=cuda)
        with pytest.raises(NotImplementedError):
            ops.w4a16_gemm(a, ops.w4_repack(_dev(qw, cuda)), _dev(sc, cuda), _dev(qz, cuda), _dev(bias, cuda), 256,
                           -1, e, out=out, cfg=104)
        return
    for m, k, n in ((333, 1280, 512), (300, 64, 256), (260, 192, 256), (513, 2560, 768)):
        qw, qz, sc, bias = _packed_layer(k, n, -1, seed=cfg * 13 + k)
        rng = np.random.Generator(np.random.PCG64(cfg + k))
        a = rng.standard_normal((m, k), dtype=np.float32).astype(np.float16)
        y = gptq_pack.matmul4_g1(a, qw, sc, qz, -1, bias)
        _epi_check(ops, cuda, a, y, ops.w4_repack(_dev(qw, cuda)), sc, qz, bias, n, -1, epi, cfg, rng)


@pytest.mark.parametrize("cfg,base", [(107, 57), (108, 64), (111, 57)])
@pytest.mark.parametrize("epi", ["bias", "gelu", "resadd", "f32"])
def test_w4a16_gemm_persistent_matches(cuda, cfg, base, epi):
    """The persistent ping-pong form (one workgroup per CU looping over the tiles) computes every
    tile exactly like its one-tile-per-workgroup twin, and cfg 111 (cfg 57 with the transposed
    f16-staged epilogue) like cfg 57: bit-identical at M = 16384, N = 1280
    (320 tiles on <= 256 workgroups, so workgroups run two tiles) and at a ragged M."""
    from samq import ops
    for m, k, n in ((16384, 1280, 1280), (9000, 640, 768)):
        qw, qz, sc, bias = _packed_layer(k, n, -1, seed=cfg + k)
        g = torch.Generator(device=cuda).manual_seed(m)
        a = torch.randn((m, k), generator=g, device=cuda).half()
        packed = ops.w4_repack(_dev(qw, cuda))
        args = (a, packed, _dev(sc, cuda), _dev(qz, cuda), _dev(bias, cuda), n, -1)
        e = {"bias": ops.EPI_BIAS, "gelu": ops.EPI_BIAS_GELU, "resadd": ops.EPI_RESADD_F32, "f32": ops.EPI_F32}[epi]
        if e == ops.EPI_RESADD_F32:
            r0 = torch.randn((m, n), generator=g, device=cuda)
            o1, o2 = r0.clone(), r0.clone()
            ops.w4a16_gemm(*args, e, out=o1, cfg=base)
            ops.w4a16_gemm(*args, e, out=o2, cfg=cfg)
        else:
            o1 = ops.w4a16_gemm(*args, e, cfg=base)
            o2 = ops.w4a16_gemm(*args, e, cfg=cfg)
        torch.cuda.synchronize()
        assert torch.equal(o1, o2), (m, k, n)


@pytest.mark.parametrize("cfg", [57, 64, 114])
@pytest.mark.parametrize("groupsize", [64, 128, 256])
@pytest.mark.parametrize("epi", ["bias", "gelu", "resadd", "f32"])
def test_w4a16_gemm_pingpong_grouped(cuda, cfg, groupsize, epi):
    """Grouped weights on the ping-pong kernels (the group's scale / zero row staged with every K
    tile, fp16((q - zp) * s) in the unpack; reference quant_linear.py:324-335): ragged M, K of
    1 .. 40 K tiles, every epilogue, against the oracle."""
    from samq import ops
    for m, k, n in ((333, 1280, 512), (300, max(64, groupsize), 256), (260, 3 * groupsize, 256), (513, 2560, 768)):
        qw, qz, sc, bias = _packed_layer(k, n, groupsize, seed=cfg * 17 + k + groupsize)
        rng = np.random.Generator(np.random.PCG64(cfg + k + groupsize))
        a = rng.standard_normal((m, k), dtype=np.float32).astype(np.float16)
        y = gptq_pack.matmul4_g1(a, qw, sc, qz, groupsize, bias)
        _epi_check(ops, cuda, a, y, ops.w4_repack(_dev(qw, cuda)), sc, qz, bias, n, groupsize, epi, cfg, rng)


@pytest.mark.parametrize("cfg,base", [(112, 114), (113, 64)])
@pytest.mark.parametrize("groupsize", [64, 128, 192, 256])
def test_w4a16_grouped_register_rows(cuda, cfg, base, groupsize):
    """Grouped ping-pong with register rows (the group's scale / zero words loaded into VGPRs ahead
    of the group, counted in the ring's vmcnt; 4 ring slots; cfg 112, selectable) against the
    ring-row form (cfg 114 = the grouped cfg 57, the group row as one more LDS-DMA piece per
    stage): identical bits (same unpack, same MFMA order) for 1 .. 80 K tiles, 1 .. 4 K tiles per
    group, every epilogue, plus the oracle at the largest K.  Groupsize 192 (3 K tiles per group)
    runs multi-group shapes too: K = 576 / 960 / 1152 (3, 5, 6 groups; at K = 960 the ring's last
    stages fall inside the last group)."""
    from samq import ops
    shapes = [(300, 64 * t, 256) for t in (1, 2, 3, 4, 5, 7)] + [(300, 576, 256), (300, 960, 256), (260, 1152, 256)] \
        + [(333, 1280, 512), (8192, 1280, 1280), (520, 5120, 1280)]
    for m, k, n in shapes:
        if k % groupsize:
            continue
        qw, qz, sc, bias = _packed_layer(k, n, groupsize, seed=k + groupsize + cfg)
        g = torch.Generator(device=cuda).manual_seed(k + groupsize)
        a = torch.randn((m, k), generator=g, device=cuda).half()
        packed = ops.w4_repack(_dev(qw, cuda))
        args = (a, packed, _dev(sc, cuda), _dev(qz, cuda), _dev(bias, cuda), n, groupsize)
        for e in (ops.EPI_BIAS, ops.EPI_BIAS_GELU, ops.EPI_RESADD_F32, ops.EPI_F32):
            if e == ops.EPI_RESADD_F32:
                r0 = torch.randn((m, n), generator=g, device=cuda)
                o1, o2 = r0.clone(), r0.clone()
                ops.w4a16_gemm(*args, e, out=o1, cfg=base)
                ops.w4a16_gemm(*args, e, out=o2, cfg=cfg)
            else:
                o1 = ops.w4a16_gemm(*args, e, cfg=base)
                o2 = ops.w4a16_gemm(*args, e, cfg=cfg)
            torch.cuda.synchronize()
            assert torch.equal(o1, o2), (m, k, n, e)
    y = gptq_pack.matmul4_g1(a.cpu().numpy(), qw, sc, qz, groupsize, bias)
    _close(ops.w4a16_gemm(*args, ops.EPI_BIAS, cfg=cfg), y, 4e-3)


@pytest.mark.parametrize("groupsize", [-1, 128])
def test_w4a16_gemm_auto_pick_wide(cuda, groupsize):
    """The automatic tile choice below one 2-image lane (M = 4133: the v3 128x256 tiles) at a
    ViT-H wide shape, per-channel and grouped, against the oracle."""
    from samq import ops
    m, k, n = 4133, 1280, 2304
    qw, qz, sc, bias = _packed_layer(k, n, groupsize, seed=77 + (groupsize > 0))
    rng = np.random.Generator(np.random.PCG64(78))
    a = rng.standard_normal((m, k), dtype=np.float32).astype(np.float16)
    y = gptq_pack.matmul4_g1(a, qw, sc, qz, groupsize, bias)
    packed = ops.w4_repack(_dev(qw, cuda))
    for epi in ("bias", "gelu", "resadd"):
        _epi_check(ops, cuda, a, y, packed, sc, qz, bias, n, groupsize, epi, 0, rng)


@pytest.mark.parametrize("n", [1280, 2560])
@pytest.mark.parametrize("groupsize", [-1, 128])
def test_w4a16_gemm_auto_pick_lane(cuda, n, groupsize):
    """The automatic tile choice at one 2-image lane (M = 8192): the 16x16x32 ping-pong (cfg 64)
    for the N = 1280 projections, the 32x32x16 one (cfg 57) for wide N, per-channel and grouped
    -- against the oracle, and bit-identical to the explicit config."""
    from samq import ops
    m, k = 8192, 1280
    qw, qz, sc, bias = _packed_layer(k, n, groupsize, seed=91 + n + groupsize)
    rng = np.random.Generator(np.random.PCG64(92))
    a = rng.standard_normal((m, k), dtype=np.float32).astype(np.float16)
    y = gptq_pack.matmul4_g1(a, qw, sc, qz, groupsize, bias)
    packed = ops.w4_repack(_dev(qw, cuda))
    for epi in ("bias", "resadd"):
        _epi_check(ops, cuda, a, y, packed, sc, qz, bias, n, groupsize, epi, 0, rng)
    args = (_dev(a, cuda), packed, _dev(sc, cuda), _dev(qz, cuda), _dev(bias, cuda), n, groupsize)
    auto = ops.w4a16_gemm(*args, ops.EPI_BIAS, cfg=0)
    assert torch.equal(auto, ops.w4a16_gemm(*args, ops.EPI_BIAS, cfg=64 if n < 2048 and groupsize == -1 else 57))


@pytest.mark.parametrize("tag", ["gm1", "g128"])
def test_matmul4_functional_vs_reference_golden(cuda, golden_dir, tag):
    """``triton_matmul4`` drop-in on the reference's own fixture: within fp16 rounding of the
    fp32 fake-quant path (G1); the reference Triton output (G2) differs by its fp16 dequant."""
    from samq import triton_matmul4
    f = np.load(golden_dir / f"matmul4_{tag}.npz", allow_pickle=False)
    g = int(f["groupsize"])
    out = triton_matmul4(g, _dev(f["a"], cuda), _dev(f["qweight"], cuda), _dev(f["scales"], cuda),
                         _dev(f["qzeros"], cuda), _dev(f["bias"], cuda)).float().cpu().numpy()
    g1 = gptq_pack.matmul4_g1(f["a"], f["qweight"], f["scales"], f["qzeros"], g, f["bias"])
    _close(out, g1, 2e-3)
    assert np.abs(out - f["out"].astype(np.float32)).max() < 5e-3


def test_matmul4_rejects_bad_k(cuda):
    from samq import triton_matmul4
    a = torch.zeros(4, 96, dtype=torch.float16, device=cuda)
    with pytest.raises(AssertionError):
        triton_matmul4(-1, a, torch.zeros(12, 64, dtype=torch.int32, device=cuda),
                       torch.zeros(1, 64, dtype=torch.float16, device=cuda),
                       torch.zeros(1, 8, dtype=torch.int32, device=cuda))
    with pytest.raises(AssertionError):  # K != 8 * qweight rows
        triton_matmul4(-1, torch.zeros(4, 128, dtype=torch.float16, device=cuda),
                       torch.zeros(8, 64, dtype=torch.int32, device=cuda),
                       torch.zeros(1, 64, dtype=torch.float16, device=cuda),
                       torch.zeros(1, 8, dtype=torch.int32, device=cuda))


@pytest.mark.parametrize("rpw", [0, 1, 2, 4])
@pytest.mark.parametrize("c", [256, 768, 1280])
@pytest.mark.parametrize("in_dtype", [torch.float32, torch.float16])
def test_layernorm(cuda, c, in_dtype, rpw):
    """1001 rows: ragged against every rows-per-wave grid (4 waves x rpw rows per workgroup)."""
    from samq import ops
    g = torch.Generator().manual_seed(c)
    x = (torch.randn(1001, c, generator=g) * 3 + 1.5).to(in_dtype)
    w = 1 + 0.1 * torch.randn(c, generator=g)
    b = 0.1 * torch.randn(c, generator=g)
    ref = torch.nn.functional.layer_norm(x.float(), (c,), w, b, eps=1e-6).numpy()
    out = ops.layernorm(x.to(cuda), w.to(cuda), b.to(cuda), 1e-6, rows_per_wave=rpw)
    _close(out, ref, 1.5e-3)
    out32 = ops.layernorm(x.to(cuda), w.to(cuda), b.to(cuda), 1e-6, out_dtype=torch.float32, rows_per_wave=rpw)
    _close(out32, ref, 2e-5)


@pytest.mark.parametrize("c", [768, 1280])
@pytest.mark.parametrize("delta_dtype", [torch.float16, torch.float32])
@pytest.mark.parametrize("q8", [False, True])
def test_add_layernorm(cuda, c, delta_dtype, q8):
    """samq_add_layernorm: x += delta in place (bit-identical to the f32 add of the GEMM's
    residual epilogue), then LayerNorm(x) as f16 or as int8 codes (fq_vit quantiser)."""
    from samq import ops
    g = torch.Generator().manual_seed(c + q8)
    x = torch.randn(1003, c, generator=g) * 3 + 1.5
    d = (torch.randn(1003, c, generator=g) * 0.7).to(delta_dtype)
    w = 1 + 0.1 * torch.randn(c, generator=g)
    b = 0.1 * torch.randn(c, generator=g)
    xs = x + d.float()
    ref = torch.nn.functional.layer_norm(xs, (c,), w, b, eps=1e-6)
    xd = x.to(cuda)
    if q8:
        s = 0.03
        out = ops.add_layernorm(xd, d.to(cuda), w.to(cuda), b.to(cuda), 1e-6, out_scale=s)
        codes = torch.clamp(torch.round(ref / s), -128, 127)
        diff = (out.cpu().to(torch.int64) - codes.to(torch.int64)).abs()
        assert out.dtype == torch.int8 and int(diff.max()) <= 1 and float((diff > 0).double().mean()) < 1e-3
    else:
        out = ops.add_layernorm(xd, d.to(cuda), w.to(cuda), b.to(cuda), 1e-6)
        _close(out, ref.numpy(), 1.5e-3)
    torch.cuda.synchronize()
    assert torch.equal(xd.cpu(), xs)


def _attn_case(b, h, w, heads, d, window, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    c = heads * d
    x = rng.standard_normal((b, h, w, c), dtype=np.float32)
    wq = rng.standard_normal((3 * c, c), dtype=np.float32) * np.float32(0.6 / math.sqrt(c))
    bq = (rng.standard_normal(3 * c, dtype=np.float32) * np.float32(0.3)).astype(np.float16)
    side = window if window else h
    rph = (rng.standard_normal((2 * side - 1, d), dtype=np.float32) * np.float32(0.3)).astype(np.float16)
    rpw = (rng.standard_normal((2 * side - 1, d), dtype=np.float32) * np.float32(0.3)).astype(np.float16)
    # qkv as the GPU sees it (fp16); the oracle uses the same fp16 values
    qkv16 = (x @ wq.T + bq.astype(np.float32)).astype(np.float16)
    t = torch.from_numpy
    if window:
        # oracle: partition the LN output (zero pad) -> Linear -> pad tokens get exactly the bias
        xw, pad_hw = sam_ref.window_partition(t(x), window)
        qkvw = (xw @ t(wq).T + t(bq.astype(np.float32))).half().float()
        o = sam_ref.attention_core(qkvw, heads, t(rph).float(), t(rpw).float())
        ref = sam_ref.window_unpartition(o, window, pad_hw, (h, w)).numpy()
    else:
        ref = sam_ref.attention_core(t(qkv16).float(), heads, t(rph).float(), t(rpw).float()).numpy()
    return qkv16, bq, rph, rpw, ref


@pytest.mark.parametrize("b,h,w,heads,d,window", [
    (2, 64, 64, 2, 80, 14),     # ViT-H windowed geometry (25 windows, pad 6)
    (1, 20, 33, 3, 64, 14),     # ragged grid, vit_b head dim
    (4, 64, 64, 16, 80, 14),    # ViT-H B=4 windowed: 1600 (window, head) items, ~6 per persistent workgroup
    (3, 64, 64, 12, 64, 14),    # vit_b B=3 windowed: 900 items (a ragged last round)
    (2, 64, 64, 2, 80, 0),      # ViT-H global
    (1, 32, 32, 2, 64, 0),
    (3, 16, 16, 2, 80, 0),
    (2, 14, 14, 2, 80, 0),      # pre-partitioned window as a global 14x14 grid (QuantAttention module path)
    (2, 64, 64, 4, 80, 0),      # ViT-H global, heads * B % 8 == 0: the 32x32-MFMA kernel
    (1, 64, 64, 8, 80, 0),
    (1, 64, 64, 1, 80, 0),      # heads * B == 1: the 3-D grid launch (no XCD remap)
    (1, 32, 32, 1, 64, 0),
])
def test_rel_attention(cuda, b, h, w, heads, d, window):
    from samq import ops
    qkv16, bq, rph, rpw, ref = _attn_case(b, h, w, heads, d, window, seed=h * 100 + w + d + window)
    args = (_dev(qkv16, cuda), _dev(bq, cuda), _dev(rph, cuda), _dev(rpw, cuda), heads, window, d ** -0.5)
    out = ops.rel_attention(*args)
    torch.cuda.synchronize()
    # fp16 P (2^-11) and fp16 output rounding on |o| <~ 2
    _close(out, ref, 2.5e-3)
    # deterministic: a second launch is bit-identical (no LDS ring race)
    for _ in range(3):
        assert torch.equal(ops.rel_attention(*args), out)


@pytest.mark.parametrize("b,h,w,heads,d,window", [
    (2, 64, 64, 16, 80, 14),    # ViT-H windowed lane (two-workgroups-per-CU window kernel)
    (2, 64, 64, 16, 80, 0),     # ViT-H global lane (streaming kernel)
    (1, 20, 33, 3, 64, 14),     # ragged grid, vit_b head dim
    (3, 16, 16, 2, 80, 0),      # resident small global grid
])
def test_rel_attention_q_out(cuda, b, h, w, heads, d, window):
    """samq_rel_attention_q (the W4A8 proj-input QAct folded into the attention store) quantises the
    f32 attention output itself (round 4; round 3 quantised its fp16 rounding, bit-identical to
    samq_rel_attention + samq_quantize): against that fp16 composition every code is within one
    step, and against the oracle's fake quant of its f32 attention the codes are within one step
    and no further off than the fp16 composition's."""
    from samq import ops
    qkv16, bq, rph, rpw, ref = _attn_case(b, h, w, heads, d, window, seed=7 + h + window)
    args = (_dev(qkv16, cuda), _dev(bq, cuda), _dev(rph, cuda), _dev(rpw, cuda), heads, window, d ** -0.5)
    s = 0.011
    o16 = ops.rel_attention(*args)
    via16 = ops.quantize(o16, s).cpu().numpy().astype(np.int32)
    got = ops.rel_attention(*args, out_scale=s)
    torch.cuda.synchronize()
    assert got.dtype == torch.int8
    got = got.cpu().numpy().astype(np.int32)
    assert np.abs(got - via16).max() <= 1
    codes = np.clip(np.rint(ref / np.float32(s)), -128, 127)
    f_got, f_16 = float((got != codes).mean()), float((via16 != codes).mean())
    print(f"\n[attn q8] codes off by one vs oracle: f32 store {f_got:.2e}, via fp16 {f_16:.2e}")
    assert np.abs(got - codes).max() <= 1 and f_got <= f_16 + 1e-4


@pytest.mark.parametrize("s,d", [(64, 80), (32, 64)])
def test_attention_relbias_single_head(cuda, s, d):
    """fused_attention.forward (samq_attention_relbias) at B = 1, heads = 1: the streaming kernel's
    3-D grid launch, whose y / z extents are 1 (regression: the XCD remap is keyed on the
    launcher's flag, not on the grid shape)."""
    from samq import fused_attention
    qkv16, _, rph, rpw, ref = _attn_case(1, s, s, 1, d, 0, seed=s + d)
    qkv = _dev(qkv16, cuda)
    q = qkv.reshape(1, s * s, 3, 1, d).permute(2, 0, 3, 1, 4).reshape(3, 1, s, s, d)[0]
    rel_h, rel_w = fused_attention.add_decomposed_rel_pos(q, _dev(rph, cuda), _dev(rpw, cuda), (s, s), (s, s))
    o = fused_attention.forward(qkv, rel_h, rel_w, 1, d, d ** -0.5)
    torch.cuda.synchronize()
    _close(o.reshape(ref.shape), ref, 3e-3)


@pytest.mark.parametrize("tag", ["win", "glob"])
def test_attention_functional_and_module_vs_reference_golden(cuda, golden_dir, tag):
    import samq
    from samq import fused_attention
    f = np.load(golden_dir / f"attn_{tag}.npz", allow_pickle=False)
    heads = int(f["heads"])
    qkv = _dev(f["qkv"], cuda)
    b, s = qkv.shape[0], qkv.shape[1]
    d = qkv.shape[-1] // 3 // heads
    q = qkv.reshape(b, s * s, 3, heads, d).permute(2, 0, 3, 1, 4).reshape(3, b * heads, s, s, d)[0]
    rel_h, rel_w = fused_attention.add_decomposed_rel_pos(q, _dev(f["rel_pos_h"], cuda), _dev(f["rel_pos_w"], cuda),
                                                          (s, s), (s, s))
    o = fused_attention.forward(qkv, rel_h, rel_w, heads, d, d ** -0.5)
    _close(o, f["attn_out"].astype(np.float32), 3e-3)
    # module path: QuantAttention with fp16 nn.Linear projections, as the reference test builds it
    c = heads * d
    lq, lp = torch.nn.Linear(c, 3 * c).half().to(cuda), torch.nn.Linear(c, c).half().to(cuda)
    with torch.no_grad():
        lq.weight.copy_(_dev(f["wqkv"], cuda)); lq.bias.copy_(_dev(f["bqkv"], cuda))
        lp.weight.copy_(_dev(f["wp"], cuda)); lp.bias.copy_(_dev(f["bp"], cuda))
    qa = samq.QuantAttention(lq, lp, heads, d ** -0.5, True, torch.nn.Parameter(_dev(f["rel_pos_h"], cuda)),
                             torch.nn.Parameter(_dev(f["rel_pos_w"], cuda)))
    with torch.no_grad():
        y = qa(_dev(f["x"], cuda))
    _close(y, f["out"].astype(np.float32), 4e-3)


# ----------------------------------------------------------------------------- patch embed / neck (§8f f4)
def test_patch_embed_vs_conv(cuda):
    """Implicit-GEMM PatchEmbed (+bias +pos_embed) vs torch Conv2d in fp32 on the same fp16 values
    (fp32 accumulation: only the summation order differs)."""
    from samq import ops
    g = torch.Generator().manual_seed(5)
    b, c, p, s = 2, 768, 16, 256
    img = torch.randn(b, 3, s, s, generator=g).half()
    w = (torch.randn(c, 3, p, p, generator=g) * 0.02).half()
    bias = torch.randn(c, generator=g) * 0.02
    pos = torch.randn(1, s // p, s // p, c, generator=g) * 0.1
    ref = torch.nn.functional.conv2d(img.float(), w.float(), bias, stride=p).permute(0, 2, 3, 1) + pos
    out = ops.patch_embed(img.to(cuda), w.reshape(c, -1).contiguous().to(cuda), bias.to(cuda), pos[0].contiguous().to(cuda), p)
    torch.cuda.synchronize()
    _close(out, ref.numpy(), 2e-5)


@pytest.mark.parametrize("b,s,c", [(2, 256, 768), (1, 1024, 1280)])
def test_patch_embed_f32_vs_conv(cuda, b, s, c):
    """fp32 PatchEmbed (the W4A8 embedding: split-fp16 MFMA, x = hi + lo' 2^-11, three products
    per fragment pair) vs torch Conv2d in float64 on the same fp32 values: within fp32-level
    rounding of a 768-term sum (2e-6 of the output scale)."""
    from samq import ops
    g = torch.Generator().manual_seed(s + c)
    p = 16
    img = torch.randn(b, 3, s, s, generator=g)
    w = torch.randn(c, 3, p, p, generator=g) * 0.02
    bias = torch.randn(c, generator=g) * 0.02
    pos = torch.randn(1, s // p, s // p, c, generator=g) * 0.1
    ref = (torch.nn.functional.conv2d(img.double(), w.double(), bias.double(), stride=p).permute(0, 2, 3, 1)
           + pos.double())
    out = ops.patch_embed(img.to(cuda), w.reshape(c, -1).contiguous().to(cuda), bias.to(cuda),
                          pos[0].contiguous().to(cuda), p)
    torch.cuda.synchronize()
    _close(out, ref.float().numpy(), 2e-6)


def test_patch_embed_u8_f32_weights_vs_conv(cuda):
    """Raw uint8 pixels (Sam.preprocess fused: normalise + zero-pad a 200 x 240 image to 256) with
    fp32 weights -- the W4A8 predictor path, split-fp16 MFMA -- vs float64 torch on the same
    normalised fp32 values."""
    from samq import ops
    g = torch.Generator().manual_seed(11)
    b, c, p, s, h, w_ = 2, 768, 16, 256, 200, 240
    img = torch.randint(0, 256, (b, 3, h, w_), generator=g, dtype=torch.uint8)
    mean = torch.tensor([123.675, 116.28, 103.53])
    std = torch.tensor([58.395, 57.12, 57.375])
    w = torch.randn(c, 3, p, p, generator=g) * 0.02
    bias = torch.randn(c, generator=g) * 0.02
    pos = torch.randn(1, s // p, s // p, c, generator=g) * 0.1
    x = torch.zeros(b, 3, s, s)
    x[:, :, :h, :w_] = (img.float() - mean.view(1, 3, 1, 1)) / std.view(1, 3, 1, 1)
    ref = (torch.nn.functional.conv2d(x.double(), w.double(), bias.double(), stride=p).permute(0, 2, 3, 1)
           + pos.double())
    out = ops.patch_embed_u8(img.to(cuda), mean.to(cuda), std.to(cuda), w.reshape(c, -1).contiguous().to(cuda),
                             bias.to(cuda), pos[0].contiguous().to(cuda), p, s)
    torch.cuda.synchronize()
    _close(out, ref.float().numpy(), 2e-6)


@pytest.mark.parametrize("b,g,cin,n", [(2, 16, 768, 256), (1, 64, 1280, 256)])
def test_neck_convs_vs_conv(cuda, b, g, cin, n):
    """Neck 1x1 (fp32 tokens -> fp16) and 3x3 pad-1 NHWC implicit GEMMs vs torch Conv2d (fp32 on
    the same fp16 values; outputs rounded to fp16)."""
    from samq import ops
    gen = torch.Generator().manual_seed(g + cin)
    x = torch.randn(b, g, g, cin, generator=gen)
    w1 = (torch.randn(n, cin, 1, 1, generator=gen) * 0.03).half()
    w2 = (torch.randn(n, n, 3, 3, generator=gen) * 0.03).half()
    y1 = ops.conv1x1_f32(x.to(cuda), w1.reshape(n, cin).contiguous().to(cuda))
    ref1 = torch.nn.functional.conv2d(x.half().float().permute(0, 3, 1, 2), w1.float()).permute(0, 2, 3, 1)
    _close(y1, ref1.numpy(), 2e-3)
    y2 = ops.conv3x3_nhwc(y1, w2.permute(0, 2, 3, 1).contiguous().to(cuda))
    ref2 = torch.nn.functional.conv2d(y1.float().cpu().permute(0, 3, 1, 2), w2.float(), padding=1).permute(0, 2, 3, 1)
    _close(y2, ref2.numpy(), 2e-3)


def test_conv_ops_reject_bad_shapes(cuda):
    from samq import ops
    with pytest.raises((AssertionError, NotImplementedError)):
        ops.conv1x1_f32(torch.zeros(8, 40, device=cuda), torch.zeros(128, 40, dtype=torch.float16, device=cuda))
    with pytest.raises((AssertionError, NotImplementedError)):
        ops.conv3x3_nhwc(torch.zeros(1, 8, 8, 48, dtype=torch.float16, device=cuda),
                         torch.zeros(128, 3, 3, 48, dtype=torch.float16, device=cuda))


# ----------------------------------------------------------------------------- LayerNorm fold
@pytest.mark.parametrize("groupsize", [-1, 128])
@pytest.mark.parametrize("m,cfg_p,cfg_c,c", [(8192, 0, 0, 1280), (333, 64, 57, 1280), (300, 57, 64, 1280),
                                             (300, 57, 64, 2048)])
def test_w4a16_gemm_lnf_chain(cuda, groupsize, m, cfg_p, cfg_c, c):
    """LayerNorm folded into the GEMMs around it (samq_w4a16_gemm_lnf): the residual producer
    (x += att.Wp + bp; a = f16((x - mu_p) gamma); per-row partial sums) followed by the consumer
    (GELU(LN(x).W1 + b1) from a, the sums and gamma.W1 / beta.W1) against the plain fp32 chain
    x' = x + att.Wp + bp -> LayerNorm -> W1 -> GELU (oracle G1 weights).  mu_p is the previous
    LayerNorm's mean, here a perturbed copy of the true row mean (what the engine carries)."""
    import samq
    from samq import ops
    n1 = 2560
    rng = np.random.Generator(np.random.PCG64(5 + m + groupsize + c))
    qwp, qzp, scp, bp = _packed_layer(c, c, groupsize, seed=3 + m)
    qw1, qz1, sc1, b1 = _packed_layer(c, n1, groupsize, seed=4 + m)
    att = (rng.standard_normal((m, c), dtype=np.float32)).astype(np.float16)
    x0 = (rng.standard_normal((m, c), dtype=np.float32) * 2 + rng.standard_normal((m, 1), dtype=np.float32) * 3)
    gamma = (1 + 0.2 * rng.standard_normal(c)).astype(np.float32)
    beta = (0.1 * rng.standard_normal(c)).astype(np.float32)
    eps = 1e-6
    # reference chain (fp32, G1 weights)
    xr = x0 + gptq_pack.matmul4_g1(att, qwp, scp, qzp, groupsize, bp)
    mean = xr.mean(1, keepdims=True)
    ln = (xr - mean) / np.sqrt(xr.var(1, keepdims=True) + eps) * gamma + beta
    y1 = gptq_pack.matmul4_g1(ln.astype(np.float32), qw1, sc1, qz1, groupsize, b1)
    ref = sam_ref.gelu_erf(torch.from_numpy(y1)).numpy()
    # product chain
    lin_p = samq.QuantLinear(4, groupsize, c, c, True).to(cuda)
    lin_1 = samq.QuantLinear(4, groupsize, c, n1, True).to(cuda)
    for lin, (qw, qz, sc, b) in ((lin_p, (qwp, qzp, scp, bp)), (lin_1, (qw1, qz1, sc1, b1))):
        lin.qweight.copy_(_dev(qw, cuda)); lin.qzeros.copy_(_dev(qz, cuda))
        lin.scales.copy_(_dev(sc, cuda)); lin.bias.copy_(_dev(b, cuda))
    lin_p.gemm_cfg, lin_1.gemm_cfg = cfg_p, cfg_c
    x = _dev(x0, cuda)
    mu = _dev((mean[:, 0] + 0.05 * rng.standard_normal(m)).astype(np.float32), cuda)
    stats = torch.empty((m, c // 64, 2), device=cuda)
    aout = torch.empty((m, c), dtype=torch.float16, device=cuda)
    g, bt = _dev(gamma, cuda), _dev(beta, cuda)
    lin_p.forward_lnf(_dev(att, cuda), ops.EPI_RESADD_LNF, x, stats, mu, gamma=g, aout=aout)
    torch.cuda.synchronize()
    _close(x, xr, 2e-5 if groupsize == -1 else 4e-3)              # the residual (grouped: fp16 weights)
    d = x.cpu().numpy() - mu.cpu().numpy()[:, None]                 # the fold algebra on the actual x
    _close(aout, d * gamma, 2e-3)                                  # f16 fold operand
    st = stats.cpu().numpy()
    np.testing.assert_allclose(st[..., 0].sum(1), d.sum(1), rtol=1e-4, atol=1e-2)
    np.testing.assert_allclose(st[..., 1].sum(1), (d * d).sum(1), rtol=1e-4)
    gw, bw = lin_1.ln_fold_constants(g, bt)
    out = torch.empty((m, n1), dtype=torch.float16, device=cuda)
    mu0 = mu.clone()
    lin_1.forward_lnf(aout, ops.EPI_GELU_LNF, out, stats, mu, gw=gw, bw=bw, eps=eps)
    torch.cuda.synchronize()
    err = _close(out, ref, 4e-3 if groupsize == -1 else 6e-3)
    print(f"\n[lnf] m={m} g={groupsize}: GELU(LN(x).W1+b1) folded vs fp32 chain max-abs {err:.2e}")
    np.testing.assert_allclose(mu.cpu().numpy(), mean[:, 0], rtol=0, atol=1e-4)   # mu_p + delta = mean
    # BIAS_LNF: the same without GELU
    mu.copy_(mu0)
    out2 = torch.empty((m, n1), dtype=torch.float16, device=cuda)
    lin_1.forward_lnf(aout, ops.EPI_BIAS_LNF, out2, stats, mu, gw=gw, bw=bw, eps=eps)
    torch.cuda.synchronize()
    _close(out2, y1, 4e-3 if groupsize == -1 else 6e-3)


def test_w4a16_gemm_lnf_rejects_non_pingpong(cuda):
    """The fold epilogues exist only in the ping-pong configs: others are SAMQ_ERR_UNSUPPORTED."""
    import samq
    from samq import ops
    lin = samq.QuantLinear(4, -1, 256, 256, True).to(cuda)
    lin.gemm_cfg = 22
    st = torch.zeros((64, 4, 2), device=cuda)
    mu = torch.zeros(64, device=cuda)
    with pytest.raises(NotImplementedError):
        lin.forward_lnf(torch.zeros((64, 256), dtype=torch.float16, device=cuda), ops.EPI_RESADD_LNF,
                        torch.zeros((64, 256), device=cuda), st, mu, gamma=torch.ones(256, device=cuda),
                        aout=torch.zeros((64, 256), dtype=torch.float16, device=cuda))


@pytest.mark.parametrize("groupsize,cfg,k,ok", [(64, 57, 1728, True), (64, 57, 1792, False), (64, 64, 2688, True),
                                                 (64, 64, 2752, False), (-1, 57, 3008, True), (-1, 57, 3072, False)])
def test_w4a16_gemm_lnf_consumer_k_limit(cuda, groupsize, cfg, k, ok):
    """the consumer stages 256 rows x K/64 partial-sum pairs in the LDS its ring frees;
    a K past the config's budget (grouped cfg 57: 1728) is SAMQ_ERR_UNSUPPORTED instead of a
    silent LDS overrun.  At the limit itself the launch runs (finite output)."""
    import samq
    from samq import ops
    m, n = 256, 256
    lin = samq.QuantLinear(4, groupsize, k, n, True).to(cuda)
    qw, qz, sc, b = _packed_layer(k, n, groupsize, seed=k + cfg)
    lin.qweight.copy_(_dev(qw, cuda)); lin.qzeros.copy_(_dev(qz, cuda))
    lin.scales.copy_(_dev(sc, cuda)); lin.bias.copy_(_dev(b, cuda))
    lin.gemm_cfg = cfg
    a = torch.randn((m, k), device=cuda).half()
    stats = torch.zeros((m, k // 64, 2), device=cuda)
    stats[..., 1] = 64.0                                   # unit variance per row
    mu = torch.zeros(m, device=cuda)
    gw, bw = lin.ln_fold_constants(torch.ones(k, device=cuda), torch.zeros(k, device=cuda))
    out = torch.empty((m, n), dtype=torch.float16, device=cuda)
    if ok:
        lin.forward_lnf(a, ops.EPI_BIAS_LNF, out, stats, mu, gw=gw, bw=bw, eps=1e-6)
        torch.cuda.synchronize()
        assert torch.isfinite(out).all()
    else:
        with pytest.raises(NotImplementedError):
            lin.forward_lnf(a, ops.EPI_BIAS_LNF, out, stats, mu, gw=gw, bw=bw, eps=1e-6)


@pytest.mark.gpu
def test_empty_batch_inputs(cuda):
    """Zero rows / zero images through every product entry point of the hot path (the engines'
    batch can be split into an empty shard on a rank): no launch fault, empty outputs of the right
    shape, and a following non-empty call still correct."""
    from samq import ops
    k, n = 256, 256
    qw, qz, sc, bias = _packed_layer(k, n, -1, seed=3)
    packed = ops.w4_repack(_dev(qw, cuda))
    args = (packed, _dev(sc, cuda), _dev(qz, cuda), _dev(bias, cuda), n, -1)
    a0 = torch.zeros((0, k), dtype=torch.float16, device=cuda)
    assert ops.w4a16_gemm(a0, *args, ops.EPI_BIAS).shape == (0, n)
    assert ops.w4a16_gemm(a0, *args, ops.EPI_BIAS_GELU).shape == (0, n)
    r0 = torch.zeros((0, n), dtype=torch.float32, device=cuda)
    ops.w4a16_gemm(a0, *args, ops.EPI_RESADD_F32, out=r0)
    # int8 paths
    w8 = torch.randint(-127, 128, (n, k), dtype=torch.int8, device=cuda)
    p8 = ops.w8_repack(w8)
    ws = torch.rand(n, device=cuda) * 0.01
    b32 = torch.zeros(n, device=cuda)
    a8 = torch.zeros((0, k), dtype=torch.int8, device=cuda)
    assert ops.w8a8_gemm(a8, p8, ws, n, b32, ops.EPI_Q8, 0.02, 0.05).shape == (0, n)
    assert ops.quantize(torch.zeros(0, device=cuda), 0.1).numel() == 0
    x0 = torch.zeros((0, 1280), dtype=torch.float32, device=cuda)
    g = torch.ones(1280, device=cuda)
    assert ops.layernorm(x0, g, torch.zeros(1280, device=cuda)).shape == (0, 1280)
    # attention over zero images (windowed and global)
    qkv0 = torch.zeros((0, 64, 64, 3 * 1280), dtype=torch.float16, device=cuda)
    rh = torch.zeros((127, 80), dtype=torch.float16, device=cuda)
    rw = torch.zeros((27, 80), dtype=torch.float16, device=cuda)
    assert ops.rel_attention(qkv0, None, rh, rh, 16, 0, 80 ** -0.5).shape == (0, 64, 64, 1280)
    assert ops.rel_attention(qkv0, None, rw, rw, 16, 14, 80 ** -0.5).shape == (0, 64, 64, 1280)
    torch.cuda.synchronize()
    # a normal call afterwards
    m = 300
    rng = np.random.Generator(np.random.PCG64(4))
    a = rng.standard_normal((m, k), dtype=np.float32).astype(np.float16)
    y = gptq_pack.matmul4_g1(a, qw, sc, qz, -1, bias)
    _close(ops.w4a16_gemm(_dev(a, cuda), *args, ops.EPI_BIAS), y, 2e-3)

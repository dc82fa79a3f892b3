"""W8A8 (fq_vit) path: the module mirror on CPU (calibration semantics vs the reference's goldens)
and the HIP int8 kernels / fused engine on the GPU (vs the CPU oracle F and the goldens).

Tolerances.  The reference sums fp32 products of fake-quant values; the kernels sum the int8
codes exactly and scale once, so the pre-quantisation values differ by fp32 rounding (~1e-6
relative) and a value lying that close to a rounding boundary of the next quantiser can land one
code apart.  Kernel tests therefore require: every code within +-1 of the reference and at most
a small stated fraction of codes off by one.  Encoder tests state the fraction of output codes
equal to the golden codes and the max-abs difference in units of the output scale.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import fq_ref, sam_ref, synth


def _golden_model(golden_dir, tag, img_size):
    g = np.load(golden_dir / f"fq_vitb_{tag}.npz", allow_pickle=False)
    meta = json.loads(str(g["meta"]))
    cfg = synth.encoder_config("vit_b", img_size=img_size)
    st = {k: v.astype(np.float16).astype(np.float32) for k, v in synth.make_encoder_state(cfg, seed=meta["seed"]).items()}
    return g, meta, cfg, st


def _product_fq(cfg, st, device="cpu"):
    from samq import fq_vit
    enc = fq_vit.build_fq_image_encoder("vit_b", img_size=cfg["img_size"])
    missing, unexpected = enc.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()}, strict=False)
    assert not unexpected, unexpected
    assert all("quantizer" in k for k in missing), missing
    return enc.to(device).eval()


# ----------------------------------------------------------------------------- CPU: module mirror
def test_fq_module_calibration_matches_reference_scales(golden_dir):
    """Our fq_vit module tree + calibration switches reproduce the reference's 140 activation
    scales and every per-channel weight scale bit for bit (same torch CPU ops)."""
    g, meta, cfg, st = _golden_model(golden_dir, "img256", 256)
    enc = _product_fq(cfg, st)
    enc.calibrate_with([torch.from_numpy(synth.make_images(1, 256, seed=s)) for s in meta["calib_seeds"]])
    names = list(g["act_scale_names"])
    from samq import fq_vit
    qa = fq_vit.act_quantizers(enc)
    assert set(qa) == set(names)
    mine = np.array([float(qa[n].quantizer.scale) for n in names], np.float32)
    np.testing.assert_array_equal(mine, g["act_scales"])
    mods = dict(enc.named_modules())
    for k in g.files:
        if k.startswith("wscale:"):
            np.testing.assert_array_equal(mods[k[7:]].quantizer.scale.numpy(), g[k])
    # quant-mode module graph on CPU (reference semantics, torch ops) == golden codes
    out = enc.module_forward(torch.from_numpy(synth.make_images(1, 256, seed=meta["test_seed"]))).detach().numpy()
    np.testing.assert_array_equal(np.round(out / g["out_scale"]), g["codes"].astype(np.float64))


def test_fq_quant_encoder_refuses_cpu(golden_dir):
    g, meta, cfg, st = _golden_model(golden_dir, "img256", 256)
    enc = _product_fq(cfg, st)
    from samq import fq_vit
    fq_vit.calibrate_weights(enc)
    fq_vit.set_act_scales(enc, dict(zip(g["act_scale_names"], g["act_scales"])))
    enc.model_quant()
    with pytest.raises(RuntimeError, match="GPU"):
        enc(torch.zeros(1, 3, 256, 256))


# ----------------------------------------------------------------------------- GPU: kernels
def _codes_close(out, ref, max_frac, what):
    out = out.astype(np.int64)
    ref = ref.astype(np.int64)
    d = np.abs(out - ref)
    frac = float((d > 0).mean())
    assert d.max() <= 1, f"{what}: code off by {d.max()}"
    assert frac <= max_frac, f"{what}: {frac:.2e} of codes off by one (> {max_frac:.1e})"
    return frac


def _rq(v, s):
    return np.clip(np.round(v / np.float32(s)), -128, 127)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [0, 81, 82, 83, 84, 87, 88, 89, 90, 91, 92])
def test_w8a8_gemm_epilogues(cuda, cfg):
    from samq import ops
    rng = np.random.Generator(np.random.PCG64(11 + cfg))
    m, k, n = 333, 768, 512
    a = rng.integers(-128, 128, (m, k), dtype=np.int8)
    w = rng.integers(-128, 128, (n, k), dtype=np.int8)
    ws = (rng.random(n, dtype=np.float32) * 1e-3 + 1e-4).astype(np.float32)
    bias = (rng.standard_normal(n, dtype=np.float32) * 0.5).astype(np.float32)
    a_s = np.float32(0.013)
    acc = a.astype(np.int64) @ w.astype(np.int64).T
    y = acc.astype(np.float64) * (np.float64(a_s) * ws.astype(np.float64)) + bias
    da, dw = torch.from_numpy(a).to(cuda), ops.w8_repack(torch.from_numpy(w).to(cuda))
    dws, db = torch.from_numpy(ws).to(cuda), torch.from_numpy(bias).to(cuda)
    f32 = ops.i8_gemm(da, 0, dw, dws, n, db, epilogue=ops.EPI_F32, a_scale=float(a_s), cfg=cfg).cpu().numpy()
    assert np.abs(f32 - y).max() <= 1e-5 * np.abs(y).max()
    s_o = np.float32(np.abs(y).max() / 127.5)
    q = ops.i8_gemm(da, 0, dw, dws, n, db, epilogue=ops.EPI_Q8, a_scale=float(a_s), out_scale=float(s_o), cfg=cfg)
    _codes_close(q.cpu().numpy(), _rq(y, s_o), 2e-4, "Q8")
    gl = 0.5 * y * (1 + np.vectorize(__import__("math").erf)(y / np.sqrt(2)))
    s_g = np.float32(np.abs(gl).max() / 127.5)
    qg = ops.i8_gemm(da, 0, dw, dws, n, db, epilogue=ops.EPI_Q8_GELU, a_scale=float(a_s), out_scale=float(s_g), cfg=cfg)
    _codes_close(qg.cpu().numpy(), _rq(gl, s_g), 2e-4, "Q8_GELU")
    res = rng.integers(-128, 128, (m, n), dtype=np.int8)
    s_r, s_mid = np.float32(0.02), np.float32(np.abs(y).max() / 127.5)
    mid = _rq(y, s_mid) * s_mid
    xr = res.astype(np.float32) * s_r + mid.astype(np.float32)
    s_x = np.float32(np.abs(xr).max() / 127.5)
    dres = torch.from_numpy(res).to(cuda)
    qr = ops.i8_gemm(da, 0, dw, dws, n, db, epilogue=ops.EPI_Q8_RES, a_scale=float(a_s), out_scale=float(s_x),
                     mid_scale=float(s_mid), res_scale=float(s_r), res=dres, out=dres, cfg=cfg)   # in place
    _codes_close(qr.cpu().numpy(), _rq(xr, s_x), 5e-4, "Q8_RES")


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [0, 81, 82, 83, 85, 86, 93])
def test_w4a8_gemm_exact_integer(cuda, cfg):
    """int4 (layout 3, incl. a zero point of 0 -> quirk 4) x int8: integer sums are exact."""
    from oracle import gptq_pack
    from samq import ops
    rng = np.random.Generator(np.random.PCG64(5 + cfg))
    m, k, n = 300, 1280, 512
    w = rng.standard_normal((n, k), dtype=np.float32) * np.float32(0.02)
    w[7] = np.abs(w[7])
    fake, s, z = gptq_pack.rtn_quantize_linear(w, -1)
    qw, qz, sc = gptq_pack.pack_linear(fake, s, z, -1)
    q = gptq_pack.unpack_qweight(qw).astype(np.int64)            # (K, N)
    zp = gptq_pack.unpack_zeros(qz).astype(np.int64)[0]          # (N,) decoded nibble + 1
    a = rng.integers(-128, 128, (m, k), dtype=np.int8)
    ref = a.astype(np.int64) @ (q - zp[None, :])
    packed = ops.w4_repack(torch.from_numpy(qw).to(cuda), layout=3)
    ones = torch.ones(n, dtype=torch.float32, device=cuda)
    out = ops.i8_gemm(torch.from_numpy(a).to(cuda), 1, packed, ones, n, None, torch.from_numpy(qz).to(cuda),
                      epilogue=ops.EPI_F32, a_scale=1.0, cfg=cfg)
    np.testing.assert_array_equal(out.cpu().numpy().astype(np.int64), ref)
    # scaled fp16 output with bias == activation * int4 dequant (fp32 ref, fp16 output rounding)
    a_s = np.float32(0.02)
    bias = (rng.standard_normal(n, dtype=np.float32) * 0.02).astype(np.float32)
    scf = sc.astype(np.float32).reshape(-1)
    y = ref.astype(np.float64) * (np.float64(a_s) * scf) + bias
    o16 = ops.w4a8_gemm(torch.from_numpy(a).to(cuda), packed, torch.from_numpy(scf).to(cuda),
                        torch.from_numpy(qz).to(cuda), n, torch.from_numpy(bias).to(cuda), ops.EPI_BIAS, float(a_s))
    assert np.abs(o16.float().cpu().numpy() - y).max() <= 1e-3 * max(1.0, np.abs(y).max())


@pytest.mark.gpu
@pytest.mark.parametrize("groupsize,k", [(128, 1280), (256, 5120), (512, 1280)])
@pytest.mark.parametrize("cfg", [0, 83, 84, 87, 88])
def test_w4a8_gemm_grouped(cuda, groupsize, k, cfg):
    """Grouped GPTQ weights on the int8 path (samq_w4a8_gemm_cfg; the reference applies per-group
    scale / zero rows, quant_linear.py:324-335): per group g the int32 sum of a * (q - zp[g]) is
    exact, scaled by s[g] in f32 and summed over the groups.  Reference: the exact integer group
    sums in int64, combined in float64.  Groupsize 512 on K = 1280 leaves a half group at the end;
    zero points include nibble 0 (quirk 4)."""
    from oracle import gptq_pack
    from samq import ops
    rng = np.random.Generator(np.random.PCG64(groupsize + k + cfg))
    m, n = 333, 512
    w = rng.standard_normal((n, k), dtype=np.float32) * np.float32(0.02)
    w[7] = np.abs(w[7])
    fake, s, z = gptq_pack.rtn_quantize_linear(w, groupsize)
    qw, qz, sc = gptq_pack.pack_linear(fake, s, z, groupsize)
    q = gptq_pack.unpack_qweight(qw).astype(np.int64)            # (K, N)
    zp = gptq_pack.unpack_zeros(qz).astype(np.int64)             # (G, N)
    scf = sc.astype(np.float32)                                  # (G, N)
    a = rng.integers(-128, 128, (m, k), dtype=np.int8)
    a_s = np.float32(0.013)
    bias = (rng.standard_normal(n, dtype=np.float32) * 0.02).astype(np.float32)
    y = np.zeros((m, n), np.float64)
    for g in range(zp.shape[0]):
        ks = slice(g * groupsize, min(k, (g + 1) * groupsize))
        pg = a[:, ks].astype(np.int64) @ (q[ks] - zp[g][None, :])
        y += pg.astype(np.float64) * scf[g].astype(np.float64)
    y = y * np.float64(a_s) + bias
    packed = ops.w4_repack(torch.from_numpy(qw).to(cuda), layout=3)
    args = (torch.from_numpy(a).to(cuda), packed, torch.from_numpy(scf).to(cuda).reshape(-1).contiguous(),
            torch.from_numpy(qz).to(cuda), n, torch.from_numpy(bias).to(cuda))
    o32 = ops.w4a8_gemm(*args, ops.EPI_F32, float(a_s), groupsize=groupsize, cfg=cfg).cpu().numpy()
    err = np.abs(o32 - y).max() / np.abs(y).max()
    print(f"\n[w4a8 grouped] g={groupsize} K={k} cfg {cfg}: f32 max rel err {err:.2e}")
    assert err <= 2e-6
    o16 = ops.w4a8_gemm(*args, ops.EPI_BIAS, float(a_s), groupsize=groupsize, cfg=cfg)
    assert np.abs(o16.float().cpu().numpy() - y).max() <= 1e-3 * max(1.0, np.abs(y).max())
    # quantising GELU epilogue: codes of GELU(y) within one step (ties of the f32 value)
    so = float(np.abs(y).max() / 100)
    c8 = ops.w4a8_gemm(*args, ops.EPI_Q8_GELU, float(a_s), out_scale=so, groupsize=groupsize, cfg=cfg)
    from oracle import sam_ref
    ref8 = torch.clamp(torch.round(sam_ref.gelu_erf(torch.from_numpy(y).float()) / so), -128, 127).numpy()
    d = np.abs(c8.cpu().numpy().astype(np.int64) - ref8.astype(np.int64))
    assert d.max() <= 1 and (d > 0).mean() <= 1e-3
    # per-channel weights (G = 1) through the same entry point stay on the per-channel kernels
    if cfg == 0:
        with pytest.raises(NotImplementedError):
            ops.w4a8_gemm(*args, ops.EPI_F32, float(a_s), groupsize=64)


@pytest.mark.gpu
@pytest.mark.parametrize("m,k,n", [(300, 1280, 512), (8192, 1280, 1280), (520, 5120, 1280), (77, 128, 256),
                                   (260, 256, 768), (8192, 1280, 5120), (1100, 640, 1408)])
@pytest.mark.parametrize("cfg", [85, 86, 93] + ([99] if os.environ.get("SAMQ_LIB") == "tuning" else []))
def test_w4a8_pingpong_matches_v3(cuda, m, k, n, cfg):
    """The W4A8 ping-pong kernels (cfg 85; cfg 86 = zero point applied through per-row sums of the
    int8 activations; cfg 93 = cfg 86 with the LDS-DMA pieces spread through the MFMA bursts) against the v3-style 256x256 kernel (cfg 81): all sum the same int32 products
    exactly and share the epilogue code, so every epilogue must agree BIT FOR BIT -- ragged M,
    K = 128 (one K tile, shorter than the lookahead), K = 256 (= the lookahead), and the lin2 depth
    K = 5120.  The weights include zero points of 0..15 (nibble + 1 = 1..16) and saturated codes.
    With SAMQ_LIB=tuning, cfg 99 (the tile ping-pong, tuning build only) runs the same checks: it
    needs K >= 512 (shorter K raise NotImplementedError) and is checked with four tiles per
    workgroup (N = 5120) and an odd tile count (1100 x 1408: 5 x 11 tiles, a last workgroup with one
    tile), against the 128x128 v3 kernel (cfg 83) where N is not a multiple of 256."""
    if n % 256 and cfg != 99:
        pytest.skip("256-column tiles")
    from oracle import gptq_pack
    from samq import ops
    rng = np.random.Generator(np.random.PCG64(m + k + n))
    w = rng.standard_normal((n, k), dtype=np.float32) * np.float32(0.02)
    w[7] = np.abs(w[7])   # an all-positive column: zero point nibble 0 (quirk 4)
    fake, s, z = gptq_pack.rtn_quantize_linear(w, -1)
    qw, qz, sc = gptq_pack.pack_linear(fake, s, z, -1)
    packed = ops.w4_repack(torch.from_numpy(qw).to(cuda), layout=3)
    a_np = rng.integers(-128, 128, (m, k), dtype=np.int8)
    a_np[:3] = 127     # saturated rows: the largest row sums
    a_np[3:5] = -128
    a = torch.from_numpy(a_np).to(cuda)
    scf = torch.from_numpy(sc.astype(np.float32).reshape(-1)).to(cuda)
    qzd = torch.from_numpy(qz).to(cuda)
    bias = torch.from_numpy(rng.standard_normal(n, dtype=np.float32) * np.float32(0.02)).to(cuda)
    a_s = 0.02
    if cfg == 99 and k < 512:
        with pytest.raises(NotImplementedError):
            ops.w4a8_gemm(a, packed, scf, qzd, n, bias, ops.EPI_BIAS, a_s, 0.0, cfg=cfg)
        return
    for epi, osc in ((ops.EPI_BIAS, 0.0), (ops.EPI_BIAS_GELU, 0.0), (ops.EPI_F32, 0.0), (ops.EPI_Q8, 0.05),
                     (ops.EPI_Q8_GELU, 0.03)):
        ref = ops.w4a8_gemm(a, packed, scf, qzd, n, bias, epi, a_s, osc, cfg=81 if n % 256 == 0 else 83)
        got = ops.w4a8_gemm(a, packed, scf, qzd, n, bias, epi, a_s, osc, cfg=cfg)
        assert torch.equal(got, ref), f"epilogue {epi}"
    res0 = torch.from_numpy(rng.standard_normal((m, n), dtype=np.float32)).to(cuda)
    r81, r85 = res0.clone(), res0.clone()
    ops.w4a8_gemm(a, packed, scf, qzd, n, bias, ops.EPI_RESADD_F32, a_s, out=r81, cfg=81 if n % 256 == 0 else 83)
    ops.w4a8_gemm(a, packed, scf, qzd, n, bias, ops.EPI_RESADD_F32, a_s, out=r85, cfg=cfg)
    assert torch.equal(r85, r81)


@pytest.mark.gpu
@pytest.mark.parametrize("m,k,n", [(300, 1280, 512), (8192, 1280, 1280), (520, 5120, 1280), (8192, 1280, 5120),
                                   (77, 128, 256)])
def test_w4a8_gemm_rowsums(cuda, m, k, n):
    """Zero-point row sums from the producer (samq_w4a8_gemm_rs, round 6): with ``rowsum`` = the exact
    int32 code sums of A the ping-pong GEMMs (cfg 86 / 93 and the automatic pick) give the same bits
    as summing A themselves, on every epilogue; ``rowsum_out`` (int8-code epilogues, any tile
    config) accumulates exactly the row sums of the codes written, on top of what the buffer held."""
    from oracle import gptq_pack
    from samq import ops
    rng = np.random.Generator(np.random.PCG64(m + 3 * k + n))
    w = rng.standard_normal((n, k), dtype=np.float32) * np.float32(0.02)
    w[7] = np.abs(w[7])
    fake, s, z = gptq_pack.rtn_quantize_linear(w, -1)
    qw, qz, sc = gptq_pack.pack_linear(fake, s, z, -1)
    packed = ops.w4_repack(torch.from_numpy(qw).to(cuda), layout=3)
    a_np = rng.integers(-128, 128, (m, k), dtype=np.int8)
    a_np[:3] = 127
    a_np[3:5] = -128
    a = torch.from_numpy(a_np).to(cuda)
    rs = a.to(torch.int32).sum(1, dtype=torch.int32).contiguous()
    scf = torch.from_numpy(sc.astype(np.float32).reshape(-1)).to(cuda)
    qzd = torch.from_numpy(qz).to(cuda)
    bias = torch.from_numpy(rng.standard_normal(n, dtype=np.float32) * np.float32(0.02)).to(cuda)
    cfgs = [0] + ([86, 93] if n % 256 == 0 else [])
    for cfg in cfgs:
        for epi, osc in ((ops.EPI_BIAS, 0.0), (ops.EPI_BIAS_GELU, 0.0), (ops.EPI_F32, 0.0), (ops.EPI_Q8, 0.05),
                         (ops.EPI_Q8_GELU, 0.03)):
            ref = ops.w4a8_gemm(a, packed, scf, qzd, n, bias, epi, 0.02, osc, cfg=cfg)
            got = ops.w4a8_gemm(a, packed, scf, qzd, n, bias, epi, 0.02, osc, cfg=cfg, rowsum=rs)
            assert torch.equal(got, ref), (cfg, epi)
            if epi in (ops.EPI_Q8, ops.EPI_Q8_GELU):
                acc = torch.full((m,), 5, dtype=torch.int32, device=cuda)
                got2 = ops.w4a8_gemm(a, packed, scf, qzd, n, bias, epi, 0.02, osc, cfg=cfg, rowsum_out=acc)
                assert torch.equal(got2, ref)
                assert torch.equal(acc, got2.to(torch.int32).sum(1, dtype=torch.int32) + 5), (cfg, epi)
        res0 = torch.from_numpy(rng.standard_normal((m, n), dtype=np.float32)).to(cuda)
        r1, r2 = res0.clone(), res0.clone()
        ops.w4a8_gemm(a, packed, scf, qzd, n, bias, ops.EPI_RESADD_F32, 0.02, out=r1, cfg=cfg)
        ops.w4a8_gemm(a, packed, scf, qzd, n, bias, ops.EPI_RESADD_F32, 0.02, out=r2, cfg=cfg, rowsum=rs)
        assert torch.equal(r1, r2), cfg
    if n % 256 == 0:   # the v3 kernels emit the same output sums
        acc = torch.zeros((m,), dtype=torch.int32, device=cuda)
        o3 = ops.w4a8_gemm(a, packed, scf, qzd, n, bias, ops.EPI_Q8_GELU, 0.02, 0.03, cfg=81, rowsum_out=acc)
        assert torch.equal(acc, o3.to(torch.int32).sum(1, dtype=torch.int32))
    with pytest.raises(AssertionError):   # output row sums of a non-code epilogue
        ops.w4a8_gemm(a, packed, scf, qzd, n, bias, ops.EPI_BIAS, 0.02, cfg=0,
                      rowsum_out=torch.zeros((m,), dtype=torch.int32, device=cuda))


@pytest.mark.gpu
def test_layernorm_q_rowsums(cuda):
    """LN-q with the output rows' code sums (samq_layernorm_q_rs): identical codes to samq_layernorm_q,
    rowsum = the exact int32 sum of each row's codes, zero_rows cleared; every rows-per-wave form
    and a ragged row count, ViT-H width."""
    from samq import ops
    rng = np.random.Generator(np.random.PCG64(11))
    rows, c = 1027, 1280
    x = torch.from_numpy(rng.standard_normal((rows, c), dtype=np.float32) * 2).to(cuda)
    g = torch.from_numpy((1 + 0.1 * rng.standard_normal(c)).astype(np.float32)).to(cuda)
    b = torch.from_numpy((0.1 * rng.standard_normal(c)).astype(np.float32)).to(cuda)
    ref = ops.layernorm_q(x, g, b, 1e-6, out_scale=0.021)
    for rpw in (0, 1, 2, 4):
        rs = torch.full((rows,), 3, dtype=torch.int32, device=cuda)
        zr = torch.full((rows,), 9, dtype=torch.int32, device=cuda)
        out = ops.layernorm_q(x, g, b, 1e-6, out_scale=0.021, rows_per_wave=rpw, rowsum=rs, zero_rows=zr)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), rpw
        assert torch.equal(rs, ref.to(torch.int32).sum(1, dtype=torch.int32)), rpw
        assert int(zr.abs().max()) == 0
    rs = torch.zeros((rows,), dtype=torch.int32, device=cuda)
    with pytest.raises(AssertionError):
        ops.layernorm_q(x, g, b, 1e-6, out_scale=0.0, rowsum=rs)


@pytest.mark.gpu
def test_quantize_and_layernorm_q(cuda):
    from samq import ops
    rng = np.random.Generator(np.random.PCG64(3))
    x = (rng.standard_normal((517, 768), dtype=np.float32) * 3).astype(np.float32)
    s = np.float32(0.037)
    codes = ops.quantize(torch.from_numpy(x).to(cuda), float(s)).cpu().numpy()
    ref = torch.clamp(torch.round(torch.from_numpy(x) / torch.tensor(s)), -128, 127).numpy()
    np.testing.assert_array_equal(codes.astype(np.float32), ref)
    fq = ops.quantize(torch.from_numpy(x).to(cuda), float(s), fake=True).cpu().numpy()
    np.testing.assert_array_equal(fq, ref * s)
    tail = ops.quantize(torch.from_numpy(x.reshape(-1)[:1003].copy()).to(cuda), float(s)).cpu().numpy()
    np.testing.assert_array_equal(tail.astype(np.float32), ref.reshape(-1)[:1003])
    # LN on int8 codes -> int8 codes (fq_vit norm1 + qact1 / neck LN2d + qacts)
    g = (1 + 0.1 * rng.standard_normal(768)).astype(np.float32)
    b = (0.1 * rng.standard_normal(768)).astype(np.float32)
    xc = codes.astype(np.int8)
    xf = torch.from_numpy(xc.astype(np.float32) * s)
    for eps in (1e-6, 1e-5):
        y = torch.nn.functional.layer_norm(xf, (768,), torch.from_numpy(g), torch.from_numpy(b), eps=eps).numpy()
        s_o = np.float32(np.abs(y).max() / 127.5)
        out = ops.layernorm_q(torch.from_numpy(xc).to(cuda), torch.from_numpy(g).to(cuda),
                              torch.from_numpy(b).to(cuda), eps, in_scale=float(s), out_scale=float(s_o))
        _codes_close(out.cpu().numpy(), _rq(y, s_o), 1e-3, "layernorm_q")
        fq32 = ops.layernorm_q(torch.from_numpy(xc).to(cuda), torch.from_numpy(g).to(cuda),
                               torch.from_numpy(b).to(cuda), eps, in_scale=float(s), out_scale=float(s_o),
                               out_dtype=torch.float32).cpu().numpy()
        np.testing.assert_array_equal(fq32, out.cpu().numpy().astype(np.float32) * s_o)
        # rows per wave (the W8A8 engine runs one): same codes, including the ragged last wave
        for rpw in (1, 2, 4):
            o2 = ops.layernorm_q(torch.from_numpy(xc).to(cuda), torch.from_numpy(g).to(cuda),
                                 torch.from_numpy(b).to(cuda), eps, in_scale=float(s), out_scale=float(s_o),
                                 rows_per_wave=rpw)
            assert torch.equal(o2.cpu(), out.cpu()), rpw


def _attn_ref(qkv_codes, bias, relh, relw, heads, window, s_qkv, s1, s2, s_o):
    """fq_vit Attention core (oracle F semantics) on fake-quant qkv values, with windowing."""
    b, h, w, c3 = qkv_codes.shape
    c = c3 // 3
    d = c // heads
    qkv = torch.from_numpy(qkv_codes.astype(np.float32) * s_qkv)
    if window > 0:
        # pad tokens project the zero-padded LN output: qkv = bias, then attn.qact1
        pad_val = fq_ref.fake_quant(torch.from_numpy(bias), torch.tensor(s_qkv))
        hp, wp = -(-h // window) * window, -(-w // window) * window
        full = pad_val.expand(b, hp, wp, c3).clone()
        full[:, :h, :w] = qkv
        qkv, _ = sam_ref.window_partition(full, window)
    bq, hh, ww, _ = qkv.shape
    t = qkv.reshape(bq, hh * ww, 3, heads, d).permute(2, 0, 3, 1, 4)
    q, k, v = t.reshape(3, bq * heads, hh * ww, d).unbind(0)
    sc = (q * (d ** -0.5)) @ k.transpose(-2, -1)
    sc = fq_ref.fake_quant(sc, torch.tensor(s1))
    rh, rw = sam_ref.rel_bias(q.reshape(bq * heads, hh, ww, d), torch.from_numpy(relh), torch.from_numpy(relw), hh, ww)
    sc = (sc.view(bq * heads, hh, ww, hh, ww) + rh[..., :, None] + rw[..., None, :]).view(bq * heads, hh * ww, hh * ww)
    sc = fq_ref.fake_quant(sc, torch.tensor(s2))
    o = (torch.softmax(sc, -1) @ v).view(bq, heads, hh, ww, d).permute(0, 2, 3, 1, 4).reshape(bq, hh, ww, c)
    if window > 0:
        o = sam_ref.window_unpartition(o, window, (hp, wp), (h, w))
    return np.clip(np.round((o / s_o).numpy()), -128, 127)


@pytest.mark.gpu
@pytest.mark.parametrize("b,hw,window", [(1, 20, 14), (2, 14, 14), (1, 16, 0), (1, 32, 0), (1, 64, 0)])
def test_rel_attention_q8(cuda, b, hw, window):
    from samq import ops
    heads, d = 2 if hw == 64 else 3, 64
    c = heads * d
    rng = np.random.Generator(np.random.PCG64(hw + window))
    qkv = rng.integers(-128, 128, (b, hw, hw, 3 * c), dtype=np.int8)
    side = window or hw
    relh = (rng.standard_normal((2 * side - 1, d), dtype=np.float32) * 0.5).astype(np.float32)
    relw = (rng.standard_normal((2 * side - 1, d), dtype=np.float32) * 0.5).astype(np.float32)
    bias = (rng.standard_normal(3 * c, dtype=np.float32) * 0.3).astype(np.float32)
    s_qkv = np.float32(0.02)
    # score scales chosen like minmax calibration would (max |score| / 127.5)
    s1, s2, s_o = np.float32(2.0 / 127.5), np.float32(6.0 / 127.5), np.float32(2.6 / 127.5)
    ref = _attn_ref(qkv, bias, relh, relw, heads, window, s_qkv, s1, s2, s_o)
    out = ops.rel_attention_q8(torch.from_numpy(qkv).to(cuda), torch.from_numpy(bias).to(cuda),
                               torch.from_numpy(relh).to(cuda), torch.from_numpy(relw).to(cuda), heads, window,
                               d ** -0.5, float(s_qkv), float(s1), float(s2), float(s_o))
    _codes_close(out.cpu().numpy(), ref, 5e-3, f"attention_q8 {b}x{hw} win {window}")


@pytest.mark.gpu
@pytest.mark.parametrize("window", [0, 14])
def test_rel_attention_q8_rows(cuda, window):
    """Row ranges of the W8A8 attention (samq_rel_attention_q8_rows, the row lanes' split): global --
    the queries of grid rows [r0, r0 + n) against every key; windows -- whole window rows, the last
    range running past the grid into the padded windows.  The union of the ranges gives the full
    launch's codes bit for bit; a range that cuts a window is refused."""
    from samq import ops
    heads, d, hw = 2, 64, 64
    c = heads * d
    rng = np.random.Generator(np.random.PCG64(77 + window))
    qkv = torch.from_numpy(rng.integers(-128, 128, (1, hw, hw, 3 * c), dtype=np.int8)).to(cuda)
    side = window or hw
    relh = torch.from_numpy((rng.standard_normal((2 * side - 1, d), dtype=np.float32) * 0.5)).to(cuda)
    relw = torch.from_numpy((rng.standard_normal((2 * side - 1, d), dtype=np.float32) * 0.5)).to(cuda)
    bias = torch.from_numpy((rng.standard_normal(3 * c, dtype=np.float32) * 0.3)).to(cuda)
    args = (qkv, bias, relh, relw, heads, window, d ** -0.5, 0.02, 2.0 / 127.5, 6.0 / 127.5, 2.6 / 127.5)
    full = ops.rel_attention_q8(*args)
    splits = [(0, 28), (28, 36)] if window else [(0, 28), (28, 36), (0, 1), (63, 1)]
    out = torch.zeros_like(full)
    for r0, n in splits[:2]:
        ops.rel_attention_q8(*args, out=out, rows=(r0, n))
    torch.cuda.synchronize()
    assert torch.equal(out, full)
    if not window:
        for r0, n in splits[2:]:
            one = torch.zeros_like(full)
            ops.rel_attention_q8(*args, out=one, rows=(r0, n))
            assert torch.equal(one[:, r0:r0 + n], full[:, r0:r0 + n]) and int(one[:, :r0].abs().sum()) == 0
    else:
        with pytest.raises(NotImplementedError):
            ops.rel_attention_q8(*args, out=out, rows=(20, 14))


@pytest.mark.gpu
def test_w8a8_fp16_v_path(cuda):
    """Round 6: the qkv GEMM's fp16 copy of the V codes (samq_w8a8_gemm_v16) equals its int8 codes
    (and leaves them unchanged), the global attention staged from it gives the same codes as from the
    int8 V, and the W8A8 engine with the path on / off is bit-identical (vit_b, 1024^2)."""
    from samq import ops
    from samq.synthetic import random_fq_encoder
    rng = np.random.Generator(np.random.PCG64(21))
    heads, d, hw = 12, 64, 64
    c = heads * d
    m, k = hw * hw, c
    a = torch.from_numpy(rng.integers(-128, 128, (m, k), dtype=np.int8)).to(cuda)
    w = torch.from_numpy(rng.integers(-128, 128, (3 * c, k), dtype=np.int8)).to(cuda)
    packed = ops.w8_repack(w)
    ws = torch.from_numpy(rng.random(3 * c, dtype=np.float32) * 1e-3).to(cuda)
    bias = torch.from_numpy(rng.standard_normal(3 * c, dtype=np.float32) * 0.1).to(cuda)
    ref = ops.w8a8_gemm(a, packed, ws, 3 * c, bias, ops.EPI_Q8, 0.02, 0.05)
    for cfg in (0, 89, 90, 84):
        v16 = torch.full((m, c), 7.0, dtype=torch.float16, device=cuda)
        got = ops.w8a8_gemm_v16(a, packed, ws, 3 * c, bias, 0.02, 0.05, v16, 2 * c, cfg=cfg)
        torch.cuda.synchronize()
        assert torch.equal(got, ref), cfg
        assert torch.equal(v16, ref[:, 2 * c:].to(torch.float16)), cfg
    qkv = ref.view(1, hw, hw, 3 * c)
    relh = torch.from_numpy((rng.standard_normal((127, d), dtype=np.float32) * 0.5)).to(cuda)
    relw = torch.from_numpy((rng.standard_normal((127, d), dtype=np.float32) * 0.5)).to(cuda)
    args = (qkv, None, relh, relw, heads, 0, d ** -0.5, 0.05, 2.0 / 127.5, 6.0 / 127.5, 2.6 / 127.5)
    o8 = ops.rel_attention_q8(*args)
    o16 = ops.rel_attention_q8(*args, v16=v16.view(1, hw, hw, c))
    torch.cuda.synchronize()
    assert torch.equal(o8, o16)
    enc = random_fq_encoder("vit_b", device=cuda)
    eng = enc.engine()
    img = torch.randn((1, 3, 1024, 1024), generator=torch.Generator(device=cuda).manual_seed(8), device=cuda)
    eng.v16 = False
    r0 = eng(img).clone()
    eng.v16 = True
    assert torch.equal(eng(img), r0)


@pytest.mark.gpu
def test_w8a8_row_lanes_bit_identical(cuda):
    """Config 2 geometry (vit_b W8A8, 1024^2, B = 1): the engine's opt-in row lanes (grid rows
    [0, 28) and [28, 64) as concurrent kernel chains, joined around the global blocks' attention)
    give the one-chain output bit for bit, eager and as a captured HIP graph replayed twice."""
    from samq.synthetic import random_fq_encoder
    enc = random_fq_encoder("vit_b", device=cuda)
    eng = enc.engine()
    img = torch.randn((1, 3, 1024, 1024), generator=torch.Generator(device=cuda).manual_seed(5), device=cuda)
    eng.row_lanes = 1
    ref = eng(img).clone()
    eng.row_lanes = 2
    assert eng._row_split(64) == 28
    got = eng(img)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    graph, gout = eng.capture(img)
    for _ in range(2):
        graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(gout, ref)


# ----------------------------------------------------------------------------- GPU: encoder
def _gpu_fq(cfg, st, g, device):
    from samq import fq_vit
    enc = _product_fq(cfg, st, device)
    fq_vit.calibrate_weights(enc)
    fq_vit.set_act_scales(enc, dict(zip(g["act_scale_names"], g["act_scales"])))
    enc.model_quant()
    return enc


def _cpu_reference_taps(cfg, st, g, img_t):
    """Our module graph in quant mode on the CPU (== the reference's goldens, see
    test_fq_module_calibration_matches_reference_scales) with every QAct output recorded."""
    from samq import fq_vit
    enc = _gpu_fq(cfg, st, g, "cpu")
    taps = {}
    for n, m in fq_vit.act_quantizers(enc).items():
        m.register_forward_hook(lambda mod, inp, out, n=n: taps.__setitem__(n, out.detach()))
    enc.module_forward(img_t)
    return taps


@pytest.mark.gpu
def test_w8a8_stage_local_parity(cuda, golden_dir):
    """Each fused W8A8 stage fed the reference's own int8 inputs reproduces the reference's output
    codes (all within +-1, <= 1e-4 of them off by one): LN+qact, qkv GEMM+qact, windowed and global
    attention (score quantisers, rel-pos, softmax, qact2), proj / lin2 GEMM + qact + residual +
    qact, lin1 GEMM + GELU + qact.  This is the kernel-level bit parity; the encoder-level
    statistics follow in test_w8a8_encoder_vs_golden."""
    from samq import ops
    g, meta, cfg, st = _golden_model(golden_dir, "img256", 256)
    img_t = torch.from_numpy(synth.make_images(1, 256, seed=meta["test_seed"]))
    ref = _cpu_reference_taps(cfg, st, g, img_t)
    scales = dict(zip(g["act_scale_names"], g["act_scales"]))
    eng = _gpu_fq(cfg, st, g, cuda).engine()
    c, gsz = cfg["embed_dim"], 256 // 16

    def codes(n, shape=None):
        t = torch.round(ref[n] / float(scales[n])).to(torch.int8)
        return (t if shape is None else t.reshape(shape)).to(cuda).contiguous()

    def check(what, out, n, natural=None):
        r = ref[n] if natural is None else natural
        rc = np.round(r.numpy() / scales[n]).reshape(-1)
        _codes_close(out.cpu().numpy().reshape(-1), rc, 1e-4, what)

    for i in range(cfg["depth"]):
        bl, pre = eng.blocks[i], f"blocks.{i}."
        xin_n = "qact1" if i == 0 else f"blocks.{i - 1}.qact4"
        s_in = float(scales[xin_n])
        check(pre + "LN1", ops.layernorm_q(codes(xin_n, (-1, c)), *bl["n1"], in_scale=s_in, out_scale=bl["s_ln1"]),
              pre + "qact1")
        win = bl["window"]
        qkv_ref = ref[pre + "attn.qact1"]
        ao_ref = ref[pre + "attn.qact2"]
        if win:
            hp = -(-gsz // win) * win
            qkv_ref = sam_ref.window_unpartition(qkv_ref.reshape(-1, win, win, 3 * c), win, (hp, hp), (gsz, gsz))
            ao_ref = sam_ref.window_unpartition(ao_ref, win, (hp, hp), (gsz, gsz))
        else:
            qkv_ref = qkv_ref.reshape(1, gsz, gsz, 3 * c)
        qkv = eng._gemm(codes(pre + "qact1", (-1, c)), bl["qkv"], ops.EPI_Q8, bl["s_ln1"], bl["s_qkv"])
        check(pre + "qkv", qkv, pre + "attn.qact1", qkv_ref)
        qc = torch.round(qkv_ref / float(scales[pre + "attn.qact1"])).to(torch.int8).to(cuda).contiguous()
        ao = ops.rel_attention_q8(qc, bl["qkv_bias"], bl["relh"], bl["relw"], bl["heads"], win, bl["scale"],
                                  bl["s_qkv"], bl["s_a1"], bl["s_a2"], bl["s_ao"])
        check(pre + f"attention (window {win})", ao, pre + "attn.qact2", ao_ref)
        aoc = torch.round(ao_ref / float(scales[pre + "attn.qact2"])).to(torch.int8).to(cuda).reshape(-1, c)
        x1 = codes(xin_n, (-1, c))
        eng._gemm(aoc.contiguous(), bl["proj"], ops.EPI_Q8_RES, bl["s_ao"], bl["s_x1"], mid=bl["s_proj"], res=x1,
                  res_scale=s_in, out=x1)
        check(pre + "proj+res", x1, pre + "qact2")
        check(pre + "LN2", ops.layernorm_q(codes(pre + "qact2", (-1, c)), *bl["n2"], in_scale=bl["s_x1"],
                                           out_scale=bl["s_ln2"]), pre + "qact3")
        check(pre + "lin1+gelu", eng._gemm(codes(pre + "qact3", (-1, c)), bl["lin1"], ops.EPI_Q8_GELU, bl["s_ln2"],
                                           bl["s_h"]), pre + "mlp.qact1")
        x3 = codes(pre + "qact2", (-1, c))
        eng._gemm(codes(pre + "mlp.qact1", (-1, 4 * c)), bl["lin2"], ops.EPI_Q8_RES, bl["s_h"], bl["s_x2"],
                  mid=bl["s_l2"], res=x3, res_scale=bl["s_x1"], out=x3)
        check(pre + "lin2+res", x3, pre + "qact4")


@pytest.mark.gpu
@pytest.mark.parametrize("tag,img", [("img256", 256), ("img1024", 1024)])
def test_w8a8_encoder_vs_golden(cuda, golden_dir, tag, img):
    """Fused HIP W8A8 engine with the reference's calibrated scales vs the reference's output codes.

    A W8A8 fake-quant encoder is chaotic at the code level: evaluating the SAME reference graph in
    float64 instead of float32 (oracle F, dtype=float64) already changes ~80% of the output codes
    by a few units (measured: 20.8% equal, mean |dcode| 1.53 at img 256), so no implementation can
    match the fp32 CPU codes bit for bit end to end (stage-level bit parity is
    test_w8a8_stage_local_parity).  Stated tolerance: our distance to the reference is at most
    1.25x the reference's own fp32-vs-fp64 distance (+0.05 codes), cosine similarity >= 0.995,
    max-abs <= 0.15 x absmax."""
    g, meta, cfg, st = _golden_model(golden_dir, tag, img)
    enc = _gpu_fq(cfg, st, g, cuda)
    img_np = synth.make_images(1, img, seed=meta["test_seed"])
    out = enc(torch.from_numpy(img_np).to(cuda)).float().cpu().numpy()
    s_out = float(g["out_scale"])
    codes = np.round(out / s_out)
    np.testing.assert_allclose(codes * s_out, out, rtol=0, atol=1e-5 * max(1.0, np.abs(out).max()))
    ref = g["codes"].astype(np.float64)
    o64 = fq_ref.FQEncoderOracle(cfg, st, dtype=torch.float64)
    o64.set_scales(dict(zip(g["act_scale_names"], g["act_scales"])))
    c64 = np.round(o64(img_np).numpy() / s_out)

    def stats(a, b):
        d = np.abs(a - b)
        cos = float((a * b).sum() / np.sqrt((a * a).sum() * (b * b).sum()))
        return float((d == 0).mean()), float(d.mean()), float(d.max()), cos

    ours, self_ = stats(codes, ref), stats(c64, ref)
    print(f"\nW8A8 vit_b {img}: ours vs reference: {ours[0] * 100:.2f}% codes equal, mean |dcode| {ours[1]:.3f}, "
          f"max {ours[2]:.0f}, cos {ours[3]:.5f} | reference fp64 vs fp32: {self_[0] * 100:.2f}% equal, "
          f"mean {self_[1]:.3f}, max {self_[2]:.0f}, cos {self_[3]:.5f} | ours vs fp64: "
          f"mean {stats(codes, c64)[1]:.3f}")
    assert ours[1] <= 1.25 * self_[1] + 0.05
    assert ours[3] >= 0.995
    assert ours[2] * s_out <= 0.15 * np.abs(ref).max() * s_out


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
def test_w8a8_conv_gemm_implicit_vs_im2col(cuda, mode):
    """The implicit-GEMM gathers (samq_w8a8_conv_gemm: 16x16 PatchEmbed on NCHW codes, 3x3 pad-1
    conv on NHWC codes) give exactly the codes of the explicit im2col + samq_w8a8_gemm path
    (int32-exact sums, same epilogue), incl. the per-image residual row (pos codes, rmod)."""
    from samq import ops
    import torch.nn.functional as F
    g = torch.Generator(device="cpu").manual_seed(30 + mode)
    b, n = 2, 256
    if mode == 1:
        cin, side = 3, 128
        x = torch.randint(-128, 128, (b, cin, side, side), generator=g, dtype=torch.int8)
        gg = side // 16
        cols = x.view(b, cin, gg, 16, gg, 16).permute(0, 2, 4, 1, 3, 5).reshape(b * gg * gg, cin * 256)
        w = torch.randint(-127, 128, (n, cin * 256), generator=g, dtype=torch.int8)
        wk = w
    else:
        cin, gg = 256, 12
        x = torch.randint(-128, 128, (b, gg, gg, cin), generator=g, dtype=torch.int8)
        pad = F.pad(x.float(), (0, 0, 1, 1, 1, 1))
        cols = pad.unfold(1, 3, 1).unfold(2, 3, 1).reshape(b * gg * gg, cin * 9).to(torch.int8)   # (c, ky, kx)
        w4 = torch.randint(-127, 128, (n, cin, 3, 3), generator=g, dtype=torch.int8)
        w = w4.reshape(n, -1)
        wk = w4.permute(0, 2, 3, 1).reshape(n, -1)    # tap-major for the implicit GEMM
    ws = (torch.rand(n, generator=g) * 0.01 + 0.001).float().to(cuda)
    bias = (torch.randn(n, generator=g) * 0.1).float().to(cuda)
    pos = torch.randint(-128, 128, (gg * gg, n), generator=g, dtype=torch.int8).to(cuda)
    packed = ops.w8_repack(w.to(cuda).contiguous())
    packed_k = ops.w8_repack(wk.to(cuda).contiguous())
    if mode == 1:
        ref = ops.w8a8_gemm(cols.to(cuda).contiguous(), packed, ws, n, bias, ops.EPI_Q8_RES, 0.02, 0.05, 0.04, 0.03,
                            pos.repeat(b, 1))
        out = ops.w8a8_conv_gemm(x.to(cuda).contiguous(), 1, packed_k, ws, n, bias, ops.EPI_Q8_RES, 0.02, 0.05,
                                 mid_scale=0.04, res_scale=0.03, res=pos, rmod=gg * gg)
    else:
        ref = ops.w8a8_gemm(cols.to(cuda).contiguous(), packed, ws, n, bias, ops.EPI_Q8, 0.02, 0.05)
        out = ops.w8a8_conv_gemm(x.to(cuda).contiguous(), 2, packed_k, ws, n, bias, ops.EPI_Q8, 0.02, 0.05)
    torch.cuda.synchronize()
    assert torch.equal(out.view(-1, n), ref.view(-1, n))

"""Pin the CPU oracle against golden vectors produced by the REFERENCE itself
(tests/golden/make_golden.py: reference pack_linear / gptq.Quantizer, Triton-interpreted
matmul4_kernel and _fwd_kernel1, segment_anything ImageEncoderViT, fq_vit W8A8 encoder)."""
import hashlib
import json

import numpy as np
import pytest
import torch

from oracle import fq_ref, gptq_pack, sam_ref, synth


def _load(golden_dir, name):
    return np.load(golden_dir / name, allow_pickle=False)


@pytest.mark.parametrize("tag,g", [("gm1", -1), ("g128", 128)])
def test_pack_bit_exact(golden_dir, tag, g):
    p = _load(golden_dir, f"pack_{tag}.npz")
    s, z = [], []
    # the oracle's RTN parameters equal the reference Quantizer's
    fake, s, z = gptq_pack.rtn_quantize_linear(p["w"], g)
    np.testing.assert_array_equal(s, p["scale"])
    np.testing.assert_array_equal(z, p["zero"])
    np.testing.assert_array_equal(fake, p["fake"])
    qw, qz, sc = gptq_pack.pack_linear(p["fake"], p["scale"], p["zero"], g)
    np.testing.assert_array_equal(qw, p["qweight"])
    np.testing.assert_array_equal(qz, p["qzeros"])
    np.testing.assert_array_equal(sc, p["scales"])


def test_zero_point_overflow_quirk(golden_dir):
    """zero point 0 on channel 3 -> stored -1 -> channels 3..7 of that word decode as 16."""
    p = _load(golden_dir, "pack_gm1.npz")
    assert p["zero"][3, 0] == 0
    zp = gptq_pack.unpack_zeros(p["qzeros"])
    assert (zp[0, 3:8] == 16).all()
    assert (zp[0, :3] == p["zero"][:3, 0]).all()  # decoded nibble+1 == zero


@pytest.mark.parametrize("tag", ["gm1", "g128"])
def test_matmul4_g2_matches_reference_kernel(golden_dir, tag):
    m = _load(golden_dir, f"matmul4_{tag}.npz")
    g = int(m["groupsize"])
    out = m["out"].astype(np.float32)
    g2 = gptq_pack.matmul4_g2(m["a"], m["qweight"], m["scales"], m["qzeros"], g, m["bias"]).astype(np.float32)
    # same fp16 operands, different fp32 summation order -> within 1 fp16 ulp
    assert np.abs(g2 - out).max() <= np.spacing(np.abs(out).max().astype(np.float16)).astype(np.float32)
    g1 = gptq_pack.matmul4_g1(m["a"], m["qweight"], m["scales"], m["qzeros"], g, m["bias"])
    assert np.abs(g1 - out).max() < 5e-3   # the reference's fp16 dequant error (quirk 5)


@pytest.mark.parametrize("tag", ["win", "glob"])
def test_attention_oracle_matches_reference_kernel(golden_dir, tag):
    f = _load(golden_dir, f"attn_{tag}.npz")
    t = lambda k: torch.from_numpy(f[k]).float()  # noqa: E731
    y = sam_ref.attention(t("x"), t("wqkv"), t("bqkv"), t("wp"), t("bp"), int(f["heads"]),
                          t("rel_pos_h"), t("rel_pos_w"))
    # reference runs in fp16 (Triton kernel + fp16 Linear); oracle in fp32
    assert (y - t("out")).abs().max().item() < 3e-3


def _vith_state(depth, seed):
    cfg = synth.encoder_config("vit_h", depth=depth, global_attn_indexes=(1,) if depth == 2 else None)
    st = {k: v.astype(np.float16).astype(np.float32) for k, v in synth.make_encoder_state(cfg, seed=seed).items()}
    return cfg, st


def test_encoder_g1_depth2_bit_exact(golden_dir):
    f = _load(golden_dir, "encoder_vith2.npz")
    meta = json.loads(str(f["meta"]))
    cfg, st = _vith_state(2, meta["seed"])
    names = synth.linear_names(cfg)
    q = sam_ref.quantize_encoder_state(st, names, -1)
    lw = sam_ref.quantized_linear_weights(q, names, -1)
    lb = {n: q[n + ".bias"].astype(np.float32) for n in names}
    out = sam_ref.EncoderOracle(cfg, st, linear_weights=lw, linear_bias=lb)(synth.make_images(1, seed=5)).numpy()
    assert np.abs(out - f["out"]).max() < 1e-5


def test_fq_vitb_img256_scales_and_codes(golden_dir):
    g = _load(golden_dir, "fq_vitb_img256.npz")
    meta = json.loads(str(g["meta"]))
    cfg = synth.encoder_config("vit_b", img_size=256)
    st = {k: v.astype(np.float16).astype(np.float32) for k, v in synth.make_encoder_state(cfg, seed=meta["seed"]).items()}
    o = fq_ref.FQEncoderOracle(cfg, st)
    o.calibrate([synth.make_images(1, 256, seed=s) for s in meta["calib_seeds"]])
    out = o(synth.make_images(1, 256, seed=meta["test_seed"])).numpy()
    names = list(g["act_scale_names"])
    assert len(names) == 140
    mine = np.array([o.scales[n].item() for n in names], np.float32)
    np.testing.assert_array_equal(mine, g["act_scales"])
    for k in g.files:
        if k.startswith("wscale:"):
            np.testing.assert_array_equal(o.wscale[k[7:]].numpy(), g[k])
    codes = np.round(out / g["out_scale"])
    np.testing.assert_array_equal(codes, g["codes"].astype(np.float64))


@pytest.mark.slow
def test_full_vith_packing_hashes(golden_dir):
    """Every packed buffer of the full 32-block ViT-H (reference pack_linear) == oracle's."""
    ref = json.loads((golden_dir / "packed_sha256_vith32.json").read_text())
    meta = json.loads(str(_load(golden_dir, "encoder_vith32.npz")["meta"]))
    cfg, st = _vith_state(32, meta["seed"])
    q = sam_ref.quantize_encoder_state(st, synth.linear_names(cfg), -1)
    for n, h in ref.items():
        d = hashlib.sha256()
        for k in ("qweight", "qzeros", "scales", "bias"):
            d.update(np.ascontiguousarray(q[f"{n}.{k}"]).tobytes())
        assert d.hexdigest() == h, n

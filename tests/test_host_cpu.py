"""Host-side logic on CPU: C-ABI exports, error mapping, product packer, module swaps,
checkpoint round trip (no GPU compute)."""
import ctypes
import json
import re

import numpy as np
import pytest
import torch

from conftest import REPO
from oracle import gptq_pack


def test_library_exports_every_header_symbol():
    from samq import _lib
    lib = _lib.load()
    header = (REPO / "include" / "samq.h").read_text()
    decl = set(re.findall(r"^\s*(?:const char\*|int|size_t)\s+(samq_\w+)\s*\(", header, re.M))
    assert decl, "no declarations parsed"
    assert decl == set(_lib.SIGNATURES), (decl ^ set(_lib.SIGNATURES))
    for name in decl:
        assert getattr(lib, name) is not None
    assert lib.samq_version() >= 100
    assert lib.samq_w4_packed_words(1280, 3840) == 1280 * 3840 // 8


def test_c_abi_rejects_bad_shapes_before_touching_the_device():
    from samq import _lib
    lib = _lib.load()
    st = lib.samq_w4a16_gemm(ctypes.c_void_p(16), 96, ctypes.c_void_p(16), ctypes.c_void_p(16), ctypes.c_void_p(16),
                             None, ctypes.c_void_p(16), 64, 8, 64, 96, -1, 0, None)
    assert st == _lib.SAMQ_ERR_INVALID
    assert "K must be a multiple of 64" in lib.samq_last_error().decode()
    with pytest.raises(AssertionError):
        _lib.check(st)
    st = lib.samq_rel_attention(ctypes.c_void_p(16), None, ctypes.c_void_p(16), ctypes.c_void_p(16),
                                ctypes.c_void_p(16), 1, 64, 64, 16, 96, 0, 0.1, None)
    assert st == _lib.SAMQ_ERR_UNSUPPORTED
    with pytest.raises(NotImplementedError):
        _lib.check(st)


def test_c_abi_empty_batch_is_a_no_op():
    """An empty batch (M / rows / n / B == 0) returns SAMQ_OK before any pointer is checked or a
    launch is made (an empty tensor's data pointer is null), while a negative size is still an
    error -- runs without a GPU since nothing reaches the device (include/samq.h conventions)."""
    from samq import _lib
    lib = _lib.load()
    assert lib.samq_w4a16_gemm(None, 1280, None, None, None, None, None, 3840, 0, 3840, 1280, -1, 0, None) == 0
    assert lib.samq_w4a16_gemm(None, 1280, None, None, None, None, None, 3840, -1, 3840, 1280, -1, 0,
                               None) == _lib.SAMQ_ERR_INVALID
    assert lib.samq_layernorm(None, None, None, None, 0, 1280, 1e-6, 0, None) == 0
    assert lib.samq_quantize(None, None, 0, 0.1, 0, None) == 0
    assert lib.samq_rel_attention(None, None, None, None, None, 0, 64, 64, 16, 80, 14, 0.1, None) == 0
    assert lib.samq_rel_attention(None, None, None, None, None, 1, 64, 64, 16, 80, 14, 0.1,
                                  None) == _lib.SAMQ_ERR_INVALID


def test_c_abi_rejects_timing_and_layout2_configs():
    """The product library exposes only tile configs that compute the GEMM on layout-1 weights:
    the tuning build's timing-only variants (27/28 no unpack, 70-73 no MFMA / no restaging) and the
    layout-2 v4 kernels (41-45) are rejected before any device work (no launch happens)."""
    from samq import _lib, ops
    from samq.quant_linear import QuantLinear
    lib = _lib.load()
    p = ctypes.c_void_p(4096)
    for cfg in range(1, 120):
        if cfg in ops.W4A16_CFGS:
            continue
        st = lib.samq_w4a16_gemm_cfg(p, 1280, p, p, p, None, p, 1280, 256, 1280, 1280, -1, 0, cfg, None)
        assert st == _lib.SAMQ_ERR_INVALID, cfg
    assert "unknown tile config" in lib.samq_last_error().decode() or "N not divisible" in lib.samq_last_error().decode()
    for cfg in (27, 41, 71):
        st = lib.samq_w4a16_gemm_cfg(p, 1280, p, p, p, None, p, 1280, 256, 1280, 1280, -1, 0, cfg, None)
        assert st == _lib.SAMQ_ERR_INVALID
    assert lib.samq_w4_repack_layout(p, p, 1280, 1280, 2, None) == _lib.SAMQ_ERR_INVALID
    q = QuantLinear(4, -1, 256, 256, True)
    for cfg in (71, 41, 27):
        with pytest.raises(ValueError):
            q.gemm_cfg = cfg
    q.gemm_cfg = 22
    assert q.gemm_cfg == 22


@pytest.mark.parametrize("tag,g", [("gm1", -1), ("g128", 128)])
def test_product_packer_bit_exact_vs_reference(golden_dir, tag, g):
    from samq.gptq import pack_linear, rtn
    from samq.quant_linear import QuantLinear
    p = np.load(golden_dir / f"pack_{tag}.npz", allow_pickle=False)
    w = torch.from_numpy(p["w"])
    fake, s, z = rtn(w, g)
    np.testing.assert_array_equal(s.numpy(), p["scale"])
    np.testing.assert_array_equal(z.numpy(), p["zero"])
    q = QuantLinear(4, g, 256, 128, True)
    pack_linear(q, fake, s, z, torch.from_numpy(p["bias"]))
    np.testing.assert_array_equal(q.qweight.numpy(), p["qweight"])
    np.testing.assert_array_equal(q.qzeros.numpy(), p["qzeros"])
    np.testing.assert_array_equal(q.scales.numpy(), p["scales"])
    np.testing.assert_array_equal(q.bias.numpy(), p["bias16"])


def test_quantlinear_buffers_match_reference_layout():
    from samq import QuantLinear
    q = QuantLinear(4, -1, 1280, 3840, True)
    sd = q.state_dict()
    assert set(sd) == {"qweight", "qzeros", "scales", "bias"}
    assert sd["qweight"].shape == (160, 3840) and sd["qweight"].dtype == torch.int32
    assert sd["qzeros"].shape == (1, 480) and sd["qzeros"].dtype == torch.int32
    assert sd["scales"].shape == (1, 3840) and sd["scales"].dtype == torch.float16
    q = QuantLinear(4, 128, 5120, 1280, False)
    assert q.qzeros.shape == (40, 160) and q.bias is None
    with pytest.raises(NotImplementedError):
        QuantLinear(3, -1, 64, 64, True)


def test_make_quant_and_attention_swap_and_load_quant_roundtrip(tmp_path):
    import samq
    from samq.gptq import quantize_rtn, save_quant
    torch.manual_seed(0)
    sam = samq.build_sam_vit_b(img_size=256)
    enc = sam.image_encoder
    n_lin = sum(isinstance(m, torch.nn.Linear) for m in enc.modules())
    assert n_lin == 48
    quantize_rtn(enc, groupsize=-1)
    assert sum(isinstance(m, samq.QuantLinear) for m in enc.modules()) == 48
    # zero one bias so load_quant drops it (reference __init__.py:57-61)
    enc.blocks[0].mlp.lin1.bias.zero_()
    save_quant(sam, tmp_path, 4, -1)
    cfg = json.loads((tmp_path / "quant_config.json").read_text())
    assert cfg == {"wbits": 4, "groupsize": -1}
    sam2 = samq.build_sam_vit_b(img_size=256)
    samq.load_quant(sam2, str(tmp_path), warmup_autotune=False, device=None, sub_module="image_encoder")
    e2 = sam2.image_encoder
    assert sum(isinstance(m, samq.QuantAttention) for m in e2.modules()) == 12
    assert e2.blocks[0].mlp.lin1.bias is None
    a, b = enc.state_dict(), sam2.state_dict()
    for k, v in a.items():
        kk = "image_encoder." + k.replace("attn.qkv.", "attn.qkv_proj.").replace("attn.proj.", "attn.o_proj.")
        if k == "blocks.0.mlp.lin1.bias":
            continue
        assert torch.equal(v, b[kk]), k
    with pytest.raises(FileNotFoundError):
        (tmp_path / "model.pt").unlink()
        samq.load_quant(samq.build_sam_vit_b(img_size=256), str(tmp_path), warmup_autotune=False, device=None,
                        sub_module="image_encoder")


def test_quantized_encoder_refuses_cpu():
    import samq
    from samq.gptq import quantize_rtn
    enc = samq.build_sam_vit_b(img_size=256).image_encoder
    quantize_rtn(enc)
    with pytest.raises(RuntimeError, match="GPU only"):
        enc(torch.zeros(1, 3, 256, 256))


def test_module_float_forward_matches_oracle():
    """The host module tree (float, unquantized) == the oracle restatement (same weights)."""
    import samq
    from oracle import sam_ref, synth
    cfg = synth.encoder_config("vit_b", img_size=256, depth=3, global_attn_indexes=(1,))
    st = synth.make_encoder_state(cfg, seed=3)
    enc = samq.ImageEncoderViT(img_size=256, embed_dim=768, depth=3, num_heads=12, mlp_ratio=4,
                               norm_layer=lambda d: torch.nn.LayerNorm(d, eps=1e-6), use_rel_pos=True,
                               global_attn_indexes=(1,), window_size=14)
    enc.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()})
    img = synth.make_images(1, 256, seed=4)
    with torch.no_grad():
        y = enc(torch.from_numpy(img)).numpy()
    ref = sam_ref.EncoderOracle(cfg, st)(img).numpy()
    assert np.abs(y - ref).max() < 1e-4


def test_w4_unpack_bit_trick_exact():
    """The GEMM kernels' int4 -> fp16 unpack (csrc/gemm_w4a16.hip w4_unpack): nibble groups 0/1 OR-ed
    into the mantissa under the exponents of 1024 / 64, groups 2/3 the same after one shift by 8,
    are the exact fp16 integers magic + q for every 32-bit word pattern tried."""
    import numpy as np
    rng = np.random.default_rng(0)
    w = rng.integers(0, 2 ** 32, size=20000, dtype=np.uint64).astype(np.uint32)
    w = np.concatenate([w, np.array([0, 0xFFFFFFFF, 0x88888888, 0x0F0F0F0F, 0xF0F0F0F0], np.uint32)])

    def f16(x):
        return np.frombuffer(np.ascontiguousarray(x, dtype=np.uint16).tobytes(), dtype=np.float16).astype(np.float32)

    w8 = w >> 8
    groups = [((w & 0x000F000F) | 0x64006400, 1024), ((w & 0x00F000F0) | 0x54005400, 64),
              ((w8 & 0x000F000F) | 0x64006400, 1024), ((w8 & 0x00F000F0) | 0x54005400, 64)]
    for i, (x, magic) in enumerate(groups):
        lo, hi = f16(x & 0xFFFF) - magic, f16(x >> 16) - magic
        assert np.array_equal(lo, (w >> (4 * i)) & 15)
        assert np.array_equal(hi, (w >> (16 + 4 * i)) & 15)


def test_bench_in_step_gemm_classifier_on_committed_profiles():
    """bench.is_proj_gemm picks exactly the projection GEMMs out of every committed in-step kernel
    trace (profiles/instep_*.json): the W4A8 int8 ping-pong GEMM (i8_gemm_pp2) included, attention /
    LayerNorm / convolution kernels excluded, and each trace's GEMM union interval is non-empty."""
    import json
    import sys
    from pathlib import Path
    repo = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(repo))
    import bench
    files = sorted((repo / "profiles").glob("instep_*.json"))
    assert files
    for f in files:
        mode = f.name.split("_")[1]
        d = json.loads(f.read_text())
        gemms = [k for k in d["kernels"] if bench.is_proj_gemm(mode, k)]
        assert gemms, f.name
        for k in d["kernels"]:
            if any(t in k for t in ("attention", "layernorm", "conv_gemm", "patch_embed", "quantize")):
                assert not bench.is_proj_gemm(mode, k), (f.name, k)
        assert d["gemm_union_ns"] > 0, f.name
    assert bench.is_proj_gemm("w4a8", "void samq::i8_gemm_pp2<5, 3, 2, 8>(signed char const*, long)")
    assert not bench.is_proj_gemm("w8a8", "void samq::i8_gemm_pp2<5, 3, 2, 8>(signed char const*, long)")


def test_bench_oracle_state_matches_test_oracle():
    """bench.py's parity leg rebuilds the oracle from the bench encoder's own state dict
    (``oracle_state``): on a small product encoder it must be the very oracle the GPU tests use
    (oracle G1 from the same packed buffers), output for output."""
    import sys
    from pathlib import Path
    import numpy as np
    import torch
    repo = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(repo))
    sys.path.insert(0, str(repo / "tests"))
    import bench
    from _encoder_helpers import oracle_g1, oracle_vith, product_encoder
    from oracle import sam_ref, synth
    cfg, st, names, q = oracle_vith(2, seed=3, name="vit_b", img_size=256, global_idx=(1,))
    enc = product_encoder(cfg, st, names, q, -1, "cpu")
    st2, lw, lb, _ = bench.oracle_state(enc, cfg, -1)
    img = synth.make_images(1, 256, seed=4)
    a = sam_ref.EncoderOracle(cfg, st2, linear_weights=lw, linear_bias=lb)(img).numpy()
    b = oracle_g1(cfg, st, names, q)(img).numpy()
    np.testing.assert_array_equal(a, b)


def test_bench_parity_report_cpu():
    """bench.parity_report (the BENCH line's parity stanza): max-abs vs the oracle and the mask IoU
    of the decoder run on both embeddings -- identical embeddings give IoU 1, a sign-flipped one
    does not."""
    import bench
    g = torch.Generator().manual_seed(0)
    ref = torch.randn((1, 256, 64, 64), generator=g) * 0.5
    rec = bench.parity_report("w4a16", ref.clone(), ref)
    assert rec["max_abs_vs_oracle"] == 0.0 and rec["pass"] is True
    assert rec["mask_iou_min"] == 1.0 and rec["masks"] == 20
    bad = bench.parity_report("w8a8", -ref, ref)
    assert bad["pass"] is False and bad["cosine"] < -0.99 and bad["mask_iou_min"] < 0.9


def test_bench_int8_parity_gate_cpu():
    """The int8 modes' parity stanza is gated against its reference points:
    the oracle's own fp64-vs-fp32 distance (mask IoU) and, for W4A8, the int8 activation noise
    (max-abs <= 1.5x, tests/test_w4a8.py:185); ``pass`` is a boolean, never null."""
    import bench
    g = torch.Generator().manual_seed(1)
    ref = torch.randn((1, 256, 64, 64), generator=g) * 0.5
    near = ref + 0.01 * torch.randn(ref.shape, generator=g)
    noise = ref + 0.05 * torch.randn(ref.shape, generator=g)
    pts = {"fp64": near, "int8_noise": noise}
    ok = bench.parity_report("w4a8", near.clone(), ref, pts)
    assert ok["pass"] is True and "fp64" in ok["reference_points"]
    assert ok["reference_points"]["fp64"]["mask_iou_mean"] > 0.9
    far = ref + 0.5 * torch.randn(ref.shape, generator=g)
    assert bench.parity_report("w4a8", far, ref, pts)["pass"] is False      # > 1.5x the noise
    assert bench.parity_report("w8a8", near.clone(), ref, {"fp64": near})["pass"] is True
    # half the channels sign-flipped: fails (cosine and masks)
    flip = ref.clone()
    flip[:, :128] = -flip[:, :128]
    rec = bench.parity_report("w8a8", flip, ref, {"fp64": ref.clone()})
    assert rec["pass"] is False
    assert bench.parity_report("w4a8", near.clone(), ref)["pass"] is True   # no points: absolute 0.35

"""The two CLI entry points of the path: ``gptq4sam.py`` (producer: GPTQ-calibrate + pack +
save, reference ``gptq4sam.py:596-663``) and ``gptq4sam_infer.py`` (consumer: ``load_quant`` +
``bench_speed``, reference ``gptq4sam_infer.py:170-225``), and ``load_quant`` on the GPU with
``warmup_autotune`` (reference ``gptq_triton/__init__.py:15-104``).

Parity: the encoder loaded from the produced checkpoint is compared with oracle G1 built from
the SAME saved buffers (dequantised ``s * (q - zp)``, fp32), tolerance 1e-2 max-abs (north star).
"""
import json
import sys

import numpy as np
import pytest
import torch

from conftest import REPO

sys.path.insert(0, str(REPO))


def _oracle_from_checkpoint(ckpt, name, img_size):
    from oracle import sam_ref, synth
    sd = torch.load(ckpt / "model.pt", map_location="cpu", weights_only=True)
    cfg = synth.encoder_config(name, img_size=img_size)
    names = synth.linear_names(cfg)
    pre = "image_encoder."
    q, st = {}, {}
    for k, v in sd.items():
        if not k.startswith(pre):
            continue
        k = k[len(pre):]
        if k.rsplit(".", 1)[0] in names:
            q[k] = v.numpy()
        else:
            st[k] = v.float().numpy()
    gs = json.loads((ckpt / "quant_config.json").read_text())["groupsize"]
    lw = sam_ref.quantized_linear_weights(q, names, gs)
    lb = {n: q[n + ".bias"].astype(np.float32) for n in names}
    return sam_ref.EncoderOracle(cfg, st, linear_weights=lw, linear_bias=lb)


def test_producer_cli_writes_a_loadable_checkpoint_cpu(tmp_path):
    """gptq4sam.py (GPTQ on 2 seeded calibration images, vit_b at 256 px on the CPU) writes
    model.pt + quant_config.json; load_quant reads them back into identical packed buffers."""
    import gptq4sam
    import samq
    model = gptq4sam.main(["--synthetic", "--model-type", "vit_b", "--img-size", "256", "--nsamples", "2",
                           "--true-sequential", "--save", str(tmp_path), "--device", "cpu"])
    assert json.loads((tmp_path / "quant_config.json").read_text()) == {"wbits": 4, "groupsize": -1}
    sam2 = samq.build_sam_vit_b(img_size=256)
    samq.load_quant(sam2, str(tmp_path), warmup_autotune=False, device=None, sub_module="image_encoder")
    ref = model.state_dict()
    got = sam2.state_dict()
    for k in [k for k in ref if k.endswith((".qweight", ".qzeros", ".scales"))]:
        kk = k.replace("attn.qkv.", "attn.qkv_proj.").replace("attn.proj.", "attn.o_proj.")
        assert torch.equal(ref[k].cpu(), got[kk]), k
    assert sum(isinstance(m, samq.QuantLinear) for m in sam2.image_encoder.modules()) == 48
    out = _oracle_from_checkpoint(tmp_path, "vit_b", 256)(np.zeros((1, 3, 256, 256), np.float32))
    assert out.shape == (1, 256, 16, 16) and torch.isfinite(out).all()
    with pytest.raises(NotImplementedError):
        gptq4sam.main(["--synthetic", "--wbits", "3", "--save", str(tmp_path)])
    with pytest.raises(ValueError):
        gptq4sam.main(["--synthetic", "--act-order", "--groupsize", "128", "--save", str(tmp_path)])


@pytest.mark.gpu
def test_producer_then_infer_entry_point_on_gpu(cuda, tmp_path):
    """Producer on the GPU (vit_b, 1024 px, GPTQ on 2 calibration images) -> gptq4sam_infer.main
    (--save: load_quant + bench_speed) -> load_quant(device="cuda", warmup_autotune=True) and the
    loaded encoder vs oracle G1 of the saved buffers."""
    import gptq4sam
    import gptq4sam_infer
    import samq
    from oracle import synth
    gptq4sam.main(["--synthetic", "--model-type", "vit_b", "--nsamples", "2", "--true-sequential",
                   "--save", str(tmp_path)])
    per = gptq4sam_infer.main(["--save", str(tmp_path), "--model-type", "vit_b", "--iters", "2", "--warmup", "1"])
    assert 0 < per < 10
    sam = samq.build_sam_vit_b()
    sam.half()
    samq.load_quant(sam, str(tmp_path), warmup_autotune=True, device="cuda", sub_module="image_encoder")
    img = synth.make_images(1, 1024, seed=21)
    with torch.no_grad():
        out = sam.image_encoder(torch.from_numpy(img).to(cuda).half()).float().cpu().numpy()
    ref = _oracle_from_checkpoint(tmp_path, "vit_b", 1024)(img).numpy()
    err = float(np.abs(out - ref).max())
    print(f"\n[parity] vit_b GPTQ checkpoint -> load_quant(cuda) engine vs oracle G1: max-abs {err:.3e}")
    assert err <= 1e-2


@pytest.mark.gpu
def test_infer_entry_point_synthetic(cuda):
    """gptq4sam_infer.main --synthetic (RTN-packed random vit_b): the reference bench_speed flow."""
    import gptq4sam_infer
    per = gptq4sam_infer.main(["--synthetic", "--model-type", "vit_b", "--iters", "2", "--warmup", "1"])
    assert 0 < per < 10

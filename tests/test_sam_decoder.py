"""Prompt encoder + mask decoder and predictor plumbing (f1); mask-IoU report.

Golden: the reference's ``PromptEncoder`` / ``MaskDecoder`` (seeded weights) applied to the
reference's own 32-block ViT-H W4 encoder output (tests/golden/masks_vith32.npz, made by
tests/golden/make_golden.py --only masks).  Masks are thresholded at 0 after the reference's
``postprocess_masks`` to 1024x1024, as in ``Sam.forward``.
"""
import json

import numpy as np
import pytest
import torch

from oracle import synth


def _decoder(device="cpu"):
    from samq.sam_decoder import build_prompt_decoder
    pe, md = build_prompt_decoder()
    shapes = {f"prompt_encoder.{k}": v.shape for k, v in pe.state_dict().items()}
    shapes.update({f"mask_decoder.{k}": v.shape for k, v in md.state_dict().items()})
    st = synth.make_decoder_state(shapes)
    pe.load_state_dict({k[15:]: torch.from_numpy(v) for k, v in st.items() if k.startswith("prompt_encoder.")})
    md.load_state_dict({k[13:]: torch.from_numpy(v) for k, v in st.items() if k.startswith("mask_decoder.")})
    return pe.to(device).eval(), md.to(device).eval()


def _run(pe, md, emb, pr, mm):
    dev = emb.device
    pts = box = None
    if "points" in pr:
        pts = (torch.tensor([pr["points"]], dtype=torch.float32, device=dev),
               torch.tensor([pr["labels"]], dtype=torch.int64, device=dev))
    if "box" in pr:
        box = torch.tensor([pr["box"]], dtype=torch.float32, device=dev)
    with torch.no_grad():
        sparse, dense = pe(points=pts, boxes=box, masks=None)
        return md(emb, pe.get_dense_pe(), sparse, dense, mm)


def _binary(low):
    from samq.sam_decoder import postprocess_masks
    return postprocess_masks(low.float(), 1024, (1024, 1024), (1024, 1024)) > 0.0


def test_decoder_matches_reference_on_reference_embedding(golden_dir):
    g = np.load(golden_dir / "masks_vith32.npz", allow_pickle=False)
    emb = torch.from_numpy(np.load(golden_dir / "encoder_vith32.npz")["out"].astype(np.float32))
    pe, md = _decoder()
    from samq import mask_iou
    for i, pr in enumerate(synth.DECODER_PROMPTS):
        for mm in (0, 1):
            low, iou = _run(pe, md, emb, pr, bool(mm))
            ref = torch.from_numpy(g[f"low_{i}_{mm}"].astype(np.float32))
            assert (low - ref).abs().max().item() <= 4e-3       # golden logits stored in fp16
            np.testing.assert_allclose(iou.numpy(), g[f"iou_{i}_{mm}"], atol=1e-4)
            assert mask_iou(_binary(low), _binary(ref)) >= 0.999


def test_predictor_plumbing_cpu():
    """SamPredictor.set_image (RGB uint8 HWC -> ResizeLongestSide -> Sam.preprocess -> encoder)
    + predict on the float model on the CPU (config 1 plumbing, small image)."""
    import samq
    from samq.build_sam import Sam, build_image_encoder
    enc = build_image_encoder(768, 2, 12, [1], img_size=256)
    sam = Sam(enc).eval()
    pred = samq.SamPredictor(sam)
    rng = np.random.Generator(np.random.PCG64(0))
    img = rng.integers(0, 256, (200, 160, 3), dtype=np.uint8)
    pred.set_image(img)
    assert pred.input_size == (256, 205) and pred.original_size == (200, 160)
    assert pred.get_image_embedding().shape == (1, 256, 16, 16)
    masks, iou, low = pred.predict(point_coords=np.array([[80.0, 100.0]]), point_labels=np.array([1]))
    assert masks.shape == (3, 200, 160) and masks.dtype == bool and iou.shape == (3,) and low.shape == (3, 64, 64)
    masks1, _, _ = pred.predict(box=np.array([10, 20, 150, 180]), multimask_output=False)
    assert masks1.shape == (1, 200, 160)
    with pytest.raises(RuntimeError):
        samq.SamPredictor(sam).predict(point_coords=np.array([[1.0, 1.0]]), point_labels=np.array([1]))


@pytest.mark.gpu
def test_mask_iou_hip_encoder_vs_reference(cuda, golden_dir):
    """North-star mask-IoU report: masks from our HIP ViT-H W4A16 embedding vs masks from the
    reference's embedding, same decoder and prompts.  Stated tolerance: IoU >= 0.97 for every
    prompt (encoder max-abs ~3e-3 moves only mask-boundary pixels)."""
    from _encoder_helpers import oracle_vith, product_encoder
    from samq import mask_iou
    f = np.load(golden_dir / "encoder_vith32.npz", allow_pickle=False)
    meta = json.loads(str(f["meta"]))
    cfg, st, names, q = oracle_vith(32, meta["seed"])
    enc = product_encoder(cfg, st, names, q, -1, cuda)
    img = torch.from_numpy(synth.make_images(1, seed=meta["image_seed"])).to(cuda)
    emb = enc.engine()(img, out_dtype=torch.float32)
    g = np.load(golden_dir / "masks_vith32.npz", allow_pickle=False)
    pe, md = _decoder(cuda)
    ious = []
    for i, pr in enumerate(synth.DECODER_PROMPTS):
        for mm in (0, 1):
            low, _ = _run(pe, md, emb, pr, bool(mm))
            ref = torch.from_numpy(g[f"low_{i}_{mm}"].astype(np.float32)).to(cuda)
            for j in range(low.shape[1]):
                ious.append(mask_iou(_binary(low[:, j:j + 1]), _binary(ref[:, j:j + 1])))
    print(f"\n[mask IoU] HIP W4A16 ViT-H vs reference embedding, {len(ious)} masks: "
          f"min {min(ious):.4f} mean {np.mean(ious):.4f}")
    assert min(ious) >= 0.97

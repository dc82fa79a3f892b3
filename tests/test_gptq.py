"""GPTQ producer: our GPTQ vs the reference's ``GPTQ`` on the same layer and
activations (tests/golden/gptq_layer.npz, made by make_golden.py --only gptq)."""
import numpy as np
import pytest
import torch


def _run(golden_dir, device, gs, act):
    from samq.gptq import GPTQ
    g = np.load(golden_dir / "gptq_layer.npz")
    lin = torch.nn.Linear(g["w"].shape[1], g["w"].shape[0], bias=False).to(device)
    lin.weight.data = torch.from_numpy(g["w"]).to(device)
    q = GPTQ(lin)
    for i in range(4):
        q.add_batch(torch.from_numpy(g[f"x{i}"]).to(device))
    scale, zero = q.fasterquant(percdamp=0.01, groupsize=gs, actorder=act)
    tag = f"g{gs}_a{int(act)}"
    return (lin.weight.data.cpu().numpy(), scale.cpu().numpy(), zero.cpu().numpy(),
            g[f"q_{tag}"], g[f"scale_{tag}"], g[f"zero_{tag}"])


@pytest.mark.parametrize("gs,act", [(-1, False), (-1, True), (128, False), (128, True)])
def test_gptq_matches_reference_cpu(golden_dir, gs, act):
    q, s, z, rq, rs, rz = _run(golden_dir, "cpu", gs, act)
    np.testing.assert_allclose(s, rs, rtol=1e-6)
    np.testing.assert_array_equal(z, rz)
    codes = np.round(q / np.repeat(s, q.shape[1] // s.shape[1], 1)) + np.repeat(z, q.shape[1] // z.shape[1], 1)
    rcodes = np.round(rq / np.repeat(rs, q.shape[1] // rs.shape[1], 1)) + np.repeat(rz, q.shape[1] // rz.shape[1], 1)
    assert (codes == rcodes).mean() >= 0.999
    assert np.abs(q - rq).max() <= 1e-5 + np.abs(rs).max() * (codes != rcodes).any()


@pytest.mark.gpu
@pytest.mark.parametrize("gs,act", [(-1, False), (128, True)])
def test_gptq_on_gpu_matches_reference(cuda, golden_dir, gs, act):
    """fp32 Cholesky / error feedback on the GPU: same scales/zeros, >= 99 % identical codes
    (a code one step away where the GPU's summation order moves a value across a rounding edge)."""
    q, s, z, rq, rs, rz = _run(golden_dir, cuda, gs, act)
    rep = q.shape[1] // s.shape[1]
    codes = np.round(q / np.repeat(s, rep, 1)) + np.repeat(z, rep, 1)
    rcodes = np.round(rq / np.repeat(rs, rep, 1)) + np.repeat(rz, rep, 1)
    eq = (codes == rcodes).mean()
    print(f"\nGPTQ GPU vs reference (g{gs}, act {act}): {eq * 100:.3f}% codes equal")
    np.testing.assert_allclose(s[:, :1], rs[:, :1], rtol=1e-5)
    assert eq >= 0.99 and np.abs(codes - rcodes).max() <= 1


@pytest.mark.gpu
def test_sam_sequential_gptq_pack_and_run(cuda):
    """gptq4sam's block-by-block calibration on a small encoder, packed into QuantLinear and run
    by the HIP engine; GPTQ's output error on the calibration image is below RTN's."""
    import samq
    from samq.gptq import pack_gptq, sam_sequential
    from samq.synthetic import random_quant_encoder
    torch.manual_seed(0)
    enc_f = random_quant_encoder("vit_b", depth=2, img_size=256, device=cuda, quantize=False)
    enc_r = random_quant_encoder("vit_b", depth=2, img_size=256, device=cuda, quantize=True)
    imgs = [torch.randn(1, 3, 256, 256, device=cuda) for _ in range(2)]
    with torch.no_grad():
        ref = enc_f.module_forward(imgs[0]).float()
    params = sam_sequential(enc_f, imgs, groupsize=-1)
    assert len(params) == 8
    pack_gptq(enc_f, params)
    samq.make_quant_attn(enc_f)
    out_g = enc_f.engine()(imgs[0], out_dtype=torch.float32)
    out_r = enc_r.engine()(imgs[0], out_dtype=torch.float32)
    eg, er = (out_g - ref).abs().mean().item(), (out_r - ref).abs().mean().item()
    print(f"\nmean-abs error vs float: GPTQ {eg:.4e}  RTN {er:.4e}")
    assert eg < er

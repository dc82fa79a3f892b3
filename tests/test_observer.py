"""fq_vit MinmaxObserver on the GPU (``observer/minmax.py:14-29``).

The HIP reduction (``samq_minmax``) must give exactly the torch statistics of the reference
observer (max / min are exact in any order): per row for weights, per column of the channel-last
view for activations, a scalar for layer_wise, merged over several updates, NaN / inf included.
On the GPU, ``calibrate_weights`` then reproduces the reference's golden per-channel weight
scales bit for bit.
"""
import numpy as np
import pytest
import torch

from oracle import synth


def _observer(module_type, mode, permute=True):
    from samq import fq_vit
    return fq_vit.build_observer("minmax", module_type, fq_vit.BIT_TYPE_DICT["int8"], mode, permute=permute)


CASES = [
    ("linear_weight", "channel_wise", (1280, 640), torch.float32),
    ("linear_weight", "layer_wise", (768, 3072), torch.float32),
    ("conv_weight", "channel_wise", (256, 128, 3, 3), torch.float32),
    ("activation", "layer_wise", (2, 64, 64, 768), torch.float32),
    ("activation", "channel_wise", (3, 50, 1280), torch.float32),
    ("activation", "channel_wise", (2, 256, 16, 16), torch.float32),   # 4-D: NCHW permute
    ("activation", "layer_wise", (4097, 33), torch.float16),
    ("activation", "channel_wise", (7, 5), torch.float32),
]


def test_minmax_abi_exports():
    """The observer entry points are part of the C ABI (loads without a GPU)."""
    from samq import _lib
    lib = _lib.load()
    assert lib.samq_minmax_workspace(0, 5, _lib.MM_ALL) == 0
    assert lib.samq_minmax_workspace(100, 64, _lib.MM_PER_ROW) == 0
    assert lib.samq_minmax_workspace(4096, 1280, _lib.MM_PER_COL) >= 2 * 1280


@pytest.mark.gpu
@pytest.mark.parametrize("module_type,mode,shape,dtype", CASES)
def test_minmax_observer_matches_torch(cuda, module_type, mode, shape, dtype):
    g = torch.Generator().manual_seed(sum(shape))
    ref, hip = _observer(module_type, mode), _observer(module_type, mode)
    for step in range(3):
        v = (torch.randn(shape, generator=g) * (1 + step) + 0.3 * step).to(dtype)
        if step == 2 and v.numel() > 10:
            flat = v.view(-1)
            flat[3] = float("inf")
            flat[-2] = float("-inf")
        ref.update(v)                 # CPU: the reference's torch ops
        hip.update(v.to(cuda))        # GPU: samq_minmax
        assert hip.max_val.is_cuda
        np.testing.assert_array_equal(hip.max_val.cpu().numpy(), ref.max_val.float().numpy())
        np.testing.assert_array_equal(hip.min_val.cpu().numpy(), ref.min_val.float().numpy())
    s_ref, z_ref = ref.get_quantization_params()
    s_hip, z_hip = hip.get_quantization_params()
    np.testing.assert_array_equal(s_hip.cpu().numpy(), s_ref.numpy())
    np.testing.assert_array_equal(z_hip.cpu().numpy(), z_ref.numpy())


@pytest.mark.gpu
def test_minmax_observer_nan_propagates(cuda):
    for module_type, mode in (("activation", "layer_wise"), ("activation", "channel_wise"),
                              ("linear_weight", "channel_wise")):
        v = torch.randn(300, 70)
        v[17, 5] = float("nan")
        ref, hip = _observer(module_type, mode), _observer(module_type, mode)
        ref.update(v)
        hip.update(v.to(cuda))
        np.testing.assert_array_equal(hip.max_val.cpu().numpy(), ref.max_val.numpy())
        np.testing.assert_array_equal(hip.min_val.cpu().numpy(), ref.min_val.numpy())


@pytest.mark.gpu
def test_calibrate_weights_on_gpu_matches_reference_golden(cuda, golden_dir):
    """Weight calibration of the fq_vit encoder on the GPU (HIP observers) gives the reference's
    golden per-channel weight scales bit for bit."""
    import json
    from samq import fq_vit
    g = np.load(golden_dir / "fq_vitb_img256.npz", allow_pickle=False)
    meta = json.loads(str(g["meta"]))
    cfg = synth.encoder_config("vit_b", img_size=256)
    st = {k: v.astype(np.float16).astype(np.float32) for k, v in synth.make_encoder_state(cfg, seed=meta["seed"]).items()}
    enc = fq_vit.build_fq_image_encoder("vit_b", img_size=256)
    enc.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()}, strict=False)
    enc = enc.to(cuda).eval()
    fq_vit.calibrate_weights(enc)
    mods = dict(enc.named_modules())
    n = 0
    for k in g.files:
        if k.startswith("wscale:"):
            q = mods[k[7:]]
            assert q.observer.max_val.is_cuda
            np.testing.assert_array_equal(q.quantizer.scale.cpu().numpy(), g[k])
            n += 1
    assert n > 0

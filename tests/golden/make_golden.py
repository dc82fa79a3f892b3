"""Generate the golden fixtures under tests/golden/ FROM THE REFERENCE ITSELF.

Run in the build container (needs /root/reference, read-only; never on the GPU box):

    TRITON_INTERPRET=1 python tests/golden/make_golden.py [--skip-full]

What it does (all on CPU, seeded, numpy PCG64 weights from ``oracle.synth``):

* ``pack_*.npz``      -- reference ``gptq.Quantizer`` RTN params + reference ``pack_linear``
                         (``gptq4sam.py:434-497``) bit layout, incl. a zero-point-0 channel
                         (quirk 4).  Inputs + packed outputs.
* ``matmul4_*.npz``   -- reference ``triton_matmul4`` (``gptq_triton/quant_linear.py:355``)
                         executed by the Triton interpreter: the reference's GPU semantics
                         (oracle G2) at real K/N with small M.
* ``attn_*.npz``      -- reference ``QuantAttention`` (``gptq_triton/fused_attention.py:107``,
                         Triton interpreter) on a windowed-shape and a global-shape input.
* ``encoder_vith2.npz``  -- reference ``segment_anything`` ``ImageEncoderViT`` (ViT-H dims,
                         depth 2: one windowed + one global block, B=1, 1024x1024) in fp32 with
                         the reference-packed int4 weights decoded (oracle G1).
* ``encoder_vith32.npz`` -- the same for the full 32-block ViT-H (fp16-stored output) plus a
                         sha256 of every reference-packed buffer of the model.
* ``masks_vith32.npz`` -- reference ``PromptEncoder`` + ``MaskDecoder`` (seeded weights,
                         ``oracle.synth.make_decoder_state``) on the reference encoder output of
                         ``encoder_vith32.npz`` for the prompts ``oracle.synth.DECODER_PROMPTS``:
                         low-res mask logits + IoU predictions (single- and multi-mask).
* ``gptq_layer.npz``  -- reference ``GPTQ.add_batch`` / ``fasterquant`` (``gptq.py:15-171``) on one
                         seeded Linear + 4 activation batches: fake-quant weights, scales, zeros
                         for groupsize -1 / 128 with act_order off / on.
* ``fq_vitb.npz``     -- reference fq_vit W8A8 ``ImageEncoderViT`` (vit_b dims, img 256 and
                         1024): calibrate on 2 seeded images (minmax, int8), then quant forward;
                         every QAct scale + weight scales + output codes.

Only OUTPUT data is committed; weights are regenerated from the seeds by ``oracle.synth``.
Import shims (none modify /root/reference): a stub ``segment_anything`` package module
(skips its ``__init__`` -> predictor -> torchvision), ``torch.empty(device='cuda')`` -> cpu
while ``gptq_triton.quant_linear`` allocates its workspace, ``get_device_capability`` ->
(8,0), a single autotune config, and ``pack_linear`` extracted with ``ast`` from
``gptq4sam.py`` (whose module imports need albumentations/cv2).
"""
from __future__ import annotations

import argparse
import ast
import hashlib
import json
import os
import sys
import time
import types
from pathlib import Path

os.environ.setdefault("TRITON_INTERPRET", "1")
sys.dont_write_bytecode = True

import numpy as np
import torch

REF = Path("/root/reference")
HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))

from oracle import synth, gptq_pack, sam_ref  # noqa: E402


# ----------------------------------------------------------------------------- shims
def import_reference():
    sys.path.insert(0, str(REF))
    sa = types.ModuleType("segment_anything")
    sa.__path__ = [str(REF / "segment_anything")]
    sys.modules["segment_anything"] = sa
    import segment_anything.modeling.image_encoder as ie  # noqa

    real_empty = torch.empty

    def cpu_empty(*a, **k):
        if str(k.get("device", "")) .startswith("cuda"):
            k["device"] = "cpu"
        return real_empty(*a, **k)

    torch.empty = cpu_empty
    try:
        import gptq_triton.quant_linear as ql
        import gptq_triton.fused_attention as fa
    finally:
        torch.empty = real_empty
    torch.cuda.get_device_capability = lambda *a, **k: (8, 0)
    ql.matmul4_kernel.configs = ql.matmul4_kernel.configs[:1]
    ql.matmul4_kernel.early_config_prune = None
    import gptq
    src = (REF / "gptq4sam.py").read_text()
    tree = ast.parse(src)
    fn = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "pack_linear"][0]
    ns = {"torch": torch, "Optional": __import__("typing").Optional}
    exec(compile(ast.Module(body=[fn], type_ignores=[]), "gptq4sam.py", "exec"), ns)
    return types.SimpleNamespace(ie=ie, ql=ql, fa=fa, gptq=gptq, pack_linear=ns["pack_linear"])


def ref_rtn(R, w: torch.Tensor, groupsize: int):
    """Reference RTN quantiser per group: gptq.Quantizer(4, perchannel, asym)."""
    n, k = w.shape
    g = k if groupsize == -1 else groupsize
    scales, zeros, fake = [], [], torch.empty_like(w)
    for s0 in range(0, k, g):
        q = R.gptq.Quantizer()
        q.configure(4, perchannel=True, sym=False, mse=False)
        blk = w[:, s0:s0 + g]
        q.find_params(blk, weight=True)
        fake[:, s0:s0 + g] = R.gptq.quantize(blk, q.scale, q.zero, q.maxq)
        scales.append(q.scale)
        zeros.append(q.zero)
    return fake, torch.cat(scales, 1), torch.cat(zeros, 1)


def ref_pack(R, fake: torch.Tensor, scale, zero, bias, groupsize: int):
    n, k = fake.shape
    g = k if groupsize == -1 else groupsize
    ng = (k + g - 1) // g
    quant = types.SimpleNamespace(
        bits=4, groupsize=g, infeatures=k, outfeatures=n,
        qweight=torch.zeros((k // 8, n), dtype=torch.int32),
        qzeros=torch.zeros((ng, n // 8), dtype=torch.int32),
        scales=torch.zeros((ng, n), dtype=torch.float16),
        bias=torch.zeros(n, dtype=torch.float16) if bias is not None else None)
    R.pack_linear(quant, fake, scale, zero, bias)
    return quant.qweight.numpy(), quant.qzeros.numpy(), quant.scales.numpy(), (
        None if quant.bias is None else quant.bias.numpy())


def fp16_round(state: dict) -> dict:
    return {k: v.astype(np.float16).astype(np.float32) for k, v in state.items()}


# ----------------------------------------------------------------------------- fixtures
def make_pack(R):
    rng = np.random.Generator(np.random.PCG64(123))
    out = {}
    for g in (-1, 128):
        w = rng.standard_normal((128, 256), dtype=np.float32) * np.float32(0.02)
        w[3] = np.abs(w[3])      # zero point 0 on channel 3 -> quirk 4
        w[17, :] = 0.0           # all-zero row -> [-1, 1] range
        fake, s, z = ref_rtn(R, torch.from_numpy(w), g)
        bias = torch.from_numpy(rng.standard_normal(128, dtype=np.float32) * np.float32(0.02))
        qw, qz, sc, b16 = ref_pack(R, fake, s, z, bias, g)
        tag = "gm1" if g == -1 else f"g{g}"
        out[tag] = dict(w=w, fake=fake.numpy(), scale=s.numpy(), zero=z.numpy(), bias=bias.numpy(),
                        qweight=qw, qzeros=qz, scales=sc, bias16=b16)
        np.savez_compressed(HERE / f"pack_{tag}.npz", **out[tag])
    return out


def make_matmul4(R, packs):
    rng = np.random.Generator(np.random.PCG64(7))
    for tag, p in packs.items():
        g = -1 if tag == "gm1" else int(tag[1:])
        a = rng.standard_normal((48, 256), dtype=np.float32).astype(np.float16)
        # reference kernel needs N % 256 == 0: tile the 128 packed columns twice
        qw = np.concatenate([p["qweight"], p["qweight"]], 1)
        qz = np.concatenate([p["qzeros"], p["qzeros"]], 1)
        sc = np.concatenate([p["scales"], p["scales"]], 1)
        b = np.concatenate([p["bias16"], p["bias16"]])
        t0 = time.time()
        c = R.ql.triton_matmul4(g if g != -1 else 256, torch.from_numpy(a), torch.from_numpy(qw),
                                torch.from_numpy(sc), torch.from_numpy(qz), torch.from_numpy(b))
        print(f"matmul4 {tag}: {time.time() - t0:.1f}s")
        np.savez_compressed(HERE / f"matmul4_{tag}.npz", a=a, qweight=qw, qzeros=qz, scales=sc,
                            bias=b, groupsize=np.int64(g), out=c.numpy().astype(np.float16))


def make_attn(R):
    rng = np.random.Generator(np.random.PCG64(11))
    heads, d = 2, 80
    c = heads * d
    for tag, (b, side) in {"win": (2, 14), "glob": (1, 16)}.items():
        x = (rng.standard_normal((b, side, side, c), dtype=np.float32)).astype(np.float16)
        wqkv = (rng.standard_normal((3 * c, c), dtype=np.float32) * np.float32(0.08)).astype(np.float16)
        bqkv = (rng.standard_normal((3 * c,), dtype=np.float32) * np.float32(0.02)).astype(np.float16)
        wp = (rng.standard_normal((c, c), dtype=np.float32) * np.float32(0.08)).astype(np.float16)
        bp = (rng.standard_normal((c,), dtype=np.float32) * np.float32(0.02)).astype(np.float16)
        rph = (rng.standard_normal((2 * side - 1, d), dtype=np.float32) * np.float32(0.1)).astype(np.float16)
        rpw = (rng.standard_normal((2 * side - 1, d), dtype=np.float32) * np.float32(0.1)).astype(np.float16)
        qkv = torch.nn.Linear(c, 3 * c).half()
        proj = torch.nn.Linear(c, c).half()
        with torch.no_grad():
            qkv.weight.copy_(torch.from_numpy(wqkv)); qkv.bias.copy_(torch.from_numpy(bqkv))
            proj.weight.copy_(torch.from_numpy(wp)); proj.bias.copy_(torch.from_numpy(bp))
        attn = R.fa.QuantAttention(qkv, proj, heads, d ** -0.5, True,
                                   torch.nn.Parameter(torch.from_numpy(rph)),
                                   torch.nn.Parameter(torch.from_numpy(rpw)))
        t0 = time.time()
        with torch.no_grad():
            # also capture the kernel's own output (before o_proj)
            qkv_out = qkv(torch.from_numpy(x))
            q = qkv_out.reshape(b, side * side, 3, heads, -1).permute(2, 0, 3, 1, 4).reshape(
                3, b * heads, side, side, -1)[0]
            rel_h, rel_w = R.fa.add_decomposed_rel_pos(q, attn.rel_pos_h, attn.rel_pos_w,
                                                       (side, side), (side, side))
            o_kernel = R.fa.forward(qkv_out, rel_h, rel_w, heads, d, d ** -0.5)
            y = attn(torch.from_numpy(x))
        print(f"attn {tag}: {time.time() - t0:.1f}s")
        np.savez_compressed(HERE / f"attn_{tag}.npz", x=x, wqkv=wqkv, bqkv=bqkv, wp=wp, bp=bp,
                            rel_pos_h=rph, rel_pos_w=rpw, heads=np.int64(heads),
                            qkv=qkv_out.numpy(), attn_out=o_kernel.numpy(), out=y.numpy())


def quantized_reference_weights(R, cfg, state, groupsize=-1, hashes=None):
    """Reference RTN + reference pack for every Linear; return G1-decoded weights."""
    lin_w, lin_b = {}, {}
    for name in synth.linear_names(cfg):
        w = torch.from_numpy(state[name + ".weight"])
        fake, s, z = ref_rtn(R, w, groupsize)
        qw, qz, sc, b16 = ref_pack(R, fake, s, z, torch.from_numpy(state[name + ".bias"]), groupsize)
        if hashes is not None:
            h = hashlib.sha256()
            for arr in (qw, qz, sc, b16):
                h.update(np.ascontiguousarray(arr).tobytes())
            hashes[name] = h.hexdigest()
        lin_w[name] = gptq_pack.dequant_g1(qw, sc, qz, groupsize).T
        lin_b[name] = b16.astype(np.float32)
    return lin_w, lin_b


def run_ref_encoder(R, cfg, state, lin_w, lin_b, img):
    enc = R.ie.ImageEncoderViT(
        depth=cfg["depth"], embed_dim=cfg["embed_dim"], img_size=cfg["img_size"], mlp_ratio=4,
        norm_layer=lambda d: torch.nn.LayerNorm(d, eps=1e-6), num_heads=cfg["num_heads"],
        patch_size=16, qkv_bias=True, use_rel_pos=True,
        global_attn_indexes=cfg["global_attn_indexes"], window_size=14, out_chans=256)
    sd = {k: torch.from_numpy(v) for k, v in state.items()}
    for n in lin_w:
        sd[n + ".weight"] = torch.from_numpy(np.ascontiguousarray(lin_w[n]))
        sd[n + ".bias"] = torch.from_numpy(lin_b[n])
    enc.load_state_dict(sd)
    enc.eval()
    with torch.no_grad():
        return enc(torch.from_numpy(img)).numpy()


def make_encoder(R, depth: int):
    cfg = synth.encoder_config("vit_h", depth=depth,
                               global_attn_indexes=(1,) if depth == 2 else None)
    seed = 100 + depth
    state = fp16_round(synth.make_encoder_state(cfg, seed=seed))
    img = synth.make_images(1, seed=5)
    hashes = {}
    t0 = time.time()
    lin_w, lin_b = quantized_reference_weights(R, cfg, state, -1, hashes)
    t1 = time.time()
    out = run_ref_encoder(R, cfg, state, lin_w, lin_b, img)
    print(f"encoder depth {depth}: pack {t1 - t0:.1f}s forward {time.time() - t1:.1f}s "
          f"absmax {np.abs(out).max():.3f}")
    meta = dict(model="vit_h", depth=depth, seed=seed, image_seed=5, groupsize=-1,
                global_attn_indexes=list(cfg["global_attn_indexes"]), state="fp16-rounded synth",
                torch=torch.__version__)
    if depth == 2:
        np.savez_compressed(HERE / "encoder_vith2.npz", out=out.astype(np.float32),
                            meta=json.dumps(meta))
    else:
        np.savez_compressed(HERE / "encoder_vith32.npz", out=out.astype(np.float16),
                            meta=json.dumps(meta))
    (HERE / f"packed_sha256_vith{depth}.json").write_text(json.dumps(hashes, indent=0, sort_keys=True))


def make_fq(img_size: int, tag: str):
    sys.path.insert(0, str(REF / "fq_vit"))
    from fq_vit.models.sam.image_encoder import ImageEncoderViT as FQEnc
    from fq_vit.models.ptq.layers import QIntLayerNorm
    from fq_vit.models.ptq import QAct, QConv2d, QLinear, QIntSoftmax
    from fq_vit.config import Config
    from models import BIT_TYPE_DICT
    from functools import partial
    cfgq = Config(False, False, "minmax")
    cfgq.BIT_TYPE_A = BIT_TYPE_DICT["int8"]
    cfg = synth.encoder_config("vit_b", img_size=img_size)
    enc = FQEnc(depth=12, embed_dim=768, img_size=img_size, mlp_ratio=4,
                norm_layer=partial(QIntLayerNorm, eps=1e-6), num_heads=12, patch_size=16,
                qkv_bias=True, use_rel_pos=True, global_attn_indexes=[2, 5, 8, 11], window_size=14,
                out_chans=256, quant=False, calibrate=False, cfg=cfgq)
    state = fp16_round(synth.make_encoder_state(cfg, seed=200 + img_size))
    sd = {k: torch.from_numpy(v) for k, v in state.items()}
    # fq_vit names: neck is a ModuleList with the same indices as the Sequential
    missing, unexpected = enc.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all(("quantizer" in m) or ("qact" in m) for m in missing), missing
    enc.eval()
    imgs = [synth.make_images(1, img_size, seed=s) for s in (21, 22)]
    test_img = synth.make_images(1, img_size, seed=23)
    mods = [m for m in enc.modules() if type(m) in (QConv2d, QLinear, QAct, QIntSoftmax)]
    t0 = time.time()
    with torch.no_grad():
        for m in mods:
            m.calibrate = True
        for i, im in enumerate(imgs):
            if i == len(imgs) - 1:
                for m in mods:
                    m.last_calibrate = True
            enc(torch.from_numpy(im))
        for m in mods:
            m.calibrate = False
            m.quant = True
        out = enc(torch.from_numpy(test_img)).numpy()
    print(f"fq vit_b {img_size}: {time.time() - t0:.1f}s absmax {np.abs(out).max():.3f}")
    scales = {}
    for name, m in enc.named_modules():
        if isinstance(m, QAct):
            scales[name] = float(m.quantizer.scale.reshape(-1)[0])
    wscales = {name: m.quantizer.scale.reshape(-1).numpy() for name, m in enc.named_modules()
               if isinstance(m, (QLinear, QConv2d))}
    s_out = scales["qacts.3"]
    codes = np.round(out / s_out)
    assert np.abs(codes * s_out - out).max() < 1e-5 * max(1.0, np.abs(out).max())
    np.savez_compressed(HERE / f"fq_vitb_{tag}.npz", codes=codes.astype(np.int8), out_scale=np.float32(s_out),
                        act_scale_names=np.array(list(scales.keys())),
                        act_scales=np.array(list(scales.values()), np.float32),
                        **{"wscale:" + k: v for k, v in wscales.items()},
                        meta=json.dumps(dict(img_size=img_size, seed=200 + img_size, calib_seeds=[21, 22],
                                             test_seed=23, torch=torch.__version__)))


def make_gptq():
    """Reference ``GPTQ`` (``gptq.py:15-171``) on one seeded Linear + calibration activations
    (CPU, fp32): fake-quant weights, scales, zeros for groupsize -1 / 128, act_order off / on."""
    import gptq as ref_gptq
    torch.cuda.synchronize = lambda *a, **k: None
    rng = np.random.Generator(np.random.PCG64(77))
    k, n = 256, 96
    w = (rng.standard_normal((n, k)) * 0.05).astype(np.float32)
    xs = [(rng.standard_normal((3, 50, k)) * np.linspace(0.2, 2.0, k)).astype(np.float32) for _ in range(4)]
    xs[0][..., 5] = 0.0   # a column with a zero Hessian diagonal is impossible with 4 batches; keep dead=False
    res = dict(w=w, **{f"x{i}": x for i, x in enumerate(xs)})
    for gs in (-1, 128):
        for act in (False, True):
            lin = torch.nn.Linear(k, n, bias=False)
            lin.weight.data = torch.from_numpy(w.copy())
            g = ref_gptq.GPTQ(lin)
            g.quantizer = ref_gptq.Quantizer()
            g.quantizer.configure(4, perchannel=True, sym=False, mse=False)
            for x in xs:
                g.add_batch(torch.from_numpy(x), None)
            scale, zero = g.fasterquant(percdamp=0.01, groupsize=gs, actorder=act)
            tag = f"g{gs}_a{int(act)}"
            res[f"q_{tag}"] = lin.weight.data.numpy().copy()
            res[f"scale_{tag}"] = scale.numpy()
            res[f"zero_{tag}"] = zero.numpy()
    np.savez_compressed(HERE / "gptq_layer.npz", **res)
    print("gptq:", {k_: v.shape for k_, v in res.items()})


def make_masks():
    """Reference prompt encoder + mask decoder on the golden ViT-H embedding (mask-IoU report)."""
    from segment_anything.modeling.prompt_encoder import PromptEncoder
    from segment_anything.modeling.mask_decoder import MaskDecoder
    from segment_anything.modeling.transformer import TwoWayTransformer
    torch.manual_seed(0)
    pe = PromptEncoder(embed_dim=256, image_embedding_size=(64, 64), input_image_size=(1024, 1024), mask_in_chans=16)
    md = MaskDecoder(num_multimask_outputs=3, transformer=TwoWayTransformer(depth=2, embedding_dim=256, mlp_dim=2048,
                                                                            num_heads=8),
                     transformer_dim=256, iou_head_depth=3, iou_head_hidden_dim=256)
    shapes = {f"prompt_encoder.{k}": v.shape for k, v in pe.state_dict().items()}
    shapes.update({f"mask_decoder.{k}": v.shape for k, v in md.state_dict().items()})
    st = synth.make_decoder_state(shapes)
    pe.load_state_dict({k[len("prompt_encoder."):]: torch.from_numpy(v) for k, v in st.items()
                        if k.startswith("prompt_encoder.")})
    md.load_state_dict({k[len("mask_decoder."):]: torch.from_numpy(v) for k, v in st.items()
                        if k.startswith("mask_decoder.")})
    pe.eval(), md.eval()
    emb = torch.from_numpy(np.load(HERE / "encoder_vith32.npz")["out"].astype(np.float32))
    res = {}
    with torch.no_grad():
        for i, pr in enumerate(synth.DECODER_PROMPTS):
            pts = None
            if "points" in pr:
                pts = (torch.tensor([pr["points"]], dtype=torch.float32), torch.tensor([pr["labels"]], dtype=torch.int64))
            box = torch.tensor([pr["box"]], dtype=torch.float32) if "box" in pr else None
            sparse, dense = pe(points=pts, boxes=box, masks=None)
            for mm in (False, True):
                low, iou = md(image_embeddings=emb, image_pe=pe.get_dense_pe(), sparse_prompt_embeddings=sparse,
                              dense_prompt_embeddings=dense, multimask_output=mm)
                res[f"low_{i}_{int(mm)}"] = low.numpy().astype(np.float16)
                res[f"iou_{i}_{int(mm)}"] = iou.numpy().astype(np.float32)
    np.savez_compressed(HERE / "masks_vith32.npz", **res,
                        meta=json.dumps(dict(decoder_seed=300, prompts=synth.DECODER_PROMPTS, torch=torch.__version__)))
    print("masks:", {k: v.shape for k, v in res.items() if k.startswith("low_")})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-full", action="store_true")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count() or 8)
    R = import_reference()
    only = set(args.only.split(",")) if args.only else None

    def want(x):
        return only is None or x in only

    if want("pack") or want("matmul4"):
        packs = make_pack(R)
        if want("matmul4"):
            make_matmul4(R, packs)
    if want("attn"):
        make_attn(R)
    if want("enc2"):
        make_encoder(R, 2)
    if want("fq"):
        make_fq(256, "img256")
        if not args.skip_full:
            make_fq(1024, "img1024")
    if want("enc32") and not args.skip_full:
        make_encoder(R, 32)
    if want("masks"):
        make_masks()
    if want("gptq"):
        make_gptq()


if __name__ == "__main__":
    main()

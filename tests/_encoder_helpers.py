"""Build the product encoder from oracle-generated weights (as a checkpoint would hold them)."""
import numpy as np
import torch

from oracle import sam_ref, synth


def oracle_vith(depth, seed, groupsize=-1, name="vit_h", img_size=1024, global_idx=None):
    cfg = synth.encoder_config(name, depth=depth, global_attn_indexes=global_idx, img_size=img_size)
    st = {k: v.astype(np.float16).astype(np.float32) for k, v in synth.make_encoder_state(cfg, seed=seed).items()}
    names = synth.linear_names(cfg)
    q = sam_ref.quantize_encoder_state(st, names, groupsize)
    return cfg, st, names, q


def oracle_g1(cfg, st, names, q, groupsize=-1):
    lw = sam_ref.quantized_linear_weights(q, names, groupsize)
    lb = {n: q[n + ".bias"].astype(np.float32) for n in names}
    return sam_ref.EncoderOracle(cfg, st, linear_weights=lw, linear_bias=lb)


def product_encoder(cfg, st, names, q, groupsize, device):
    """Our ImageEncoderViT with the packed weights loaded through ``load_state_dict`` exactly as
    ``load_quant`` does (make_quant -> load -> make_quant_attn -> .to(device))."""
    import samq
    from samq.build_sam import build_image_encoder
    enc = build_image_encoder(cfg["embed_dim"], cfg["depth"], cfg["num_heads"], list(cfg["global_attn_indexes"]),
                              img_size=cfg["img_size"])
    samq.make_quant(enc, 4, groupsize)
    lin = set(names)
    sd = {}
    for k, v in st.items():
        base = k.rsplit(".", 1)[0]
        if base in lin:
            continue
        sd[k] = torch.from_numpy(v).half()  # the reference model is .half() before saving
    for k, v in q.items():
        sd[k] = torch.from_numpy(np.ascontiguousarray(v))
    missing, unexpected = enc.load_state_dict(sd, strict=False)
    assert not unexpected and not missing, (missing, unexpected)
    samq.make_quant_attn(enc)
    return enc.to(device)

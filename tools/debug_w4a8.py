"""Per-op comparison of the W4A8 engine's first block with the W4A8 oracle (debug tool)."""
import sys
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "sam-quantization_amd"), str(REPO / "tests")]
import samq  # noqa: E402
from samq import ops  # noqa: E402
from oracle import synth, sam_ref  # noqa: E402
from oracle.fq_ref import fake_quant  # noqa: E402
from test_w4a8 import _oracle  # noqa: E402
from _encoder_helpers import product_encoder  # noqa: E402

cuda = torch.device("cuda")
cfg, st, names, q, o = _oracle(2, 7, global_idx=(1,))
enc = product_encoder(cfg, st, names, q, -1, cuda).half()
samq.make_act_quant(enc)
calib = [synth.make_images(1, 1024, seed=s) for s in (1, 2)]
o.calibrate(calib)
for n, m in enc.named_modules():
    if isinstance(m, samq.QuantLinear):
        m.act_quant.quantizer.update_quantization_params  # noqa
        key = n.replace("qkv_proj", "qkv").replace("o_proj", "proj")
        m.act_quant.quantizer.scale = torch.tensor(float(o.scales[key]), device=cuda)
        m.act_quant.quantizer.zero_point = torch.zeros((), dtype=torch.int64, device=cuda)
        m.act_quant.quant = True
x = synth.make_images(1, 1024, seed=9)
eng = enc.engine()
print("w4a8:", eng.w4a8)
bufs = eng.buffers(1)
eng.embed(torch.from_numpy(x).to(cuda).half(), bufs["x"])
x0 = o.embed(torch.from_numpy(x))
print("embed max diff", (bufs["x"].cpu() - x0).abs().max().item())
p = eng.plans[0]
c = cfg["embed_dim"]
pre = "blocks.0."
xo = x0
y = F.layer_norm(xo, (c,), o.p[pre + "norm1.weight"], o.p[pre + "norm1.bias"], eps=1e-6)
yq = fake_quant(y, o.scales[pre + "attn.qkv"])
ops.layernorm_q(bufs["x"], p.ln1_w, p.ln1_b, p.ln1_eps, out_scale=p.s_qkv, out=bufs["xn8"])
d = (bufs["xn8"].float().cpu() * p.s_qkv - yq).abs()
print("LN1 codes diff", (d > 1e-6).float().mean().item(), d.max().item(), "s", p.s_qkv, float(o.scales[pre + "attn.qkv"]))
qkv_ref = F.linear(yq, o.p[pre + "attn.qkv.weight"], o.p[pre + "attn.qkv.bias"])
p.qkv.forward_w4a8(bufs["xn8"], p.s_qkv, ops.EPI_BIAS, out=bufs["qkv"])
print("qkv max diff", (bufs["qkv"].float().cpu() - qkv_ref).abs().max().item(), "absmax", qkv_ref.abs().max().item())
# attention in natural layout via windows
win = p.window
yw, pad_hw = sam_ref.window_partition(yq, win)
qkv_w = F.linear(yw, o.p[pre + "attn.qkv.weight"], o.p[pre + "attn.qkv.bias"])
att_w = sam_ref.attention_core(qkv_w, cfg["num_heads"], o.p[pre + "attn.rel_pos_h"], o.p[pre + "attn.rel_pos_w"])
att_ref = sam_ref.window_unpartition(att_w, win, pad_hw, (64, 64))
ops.rel_attention(bufs["qkv"], p.qkv_bias, p.relh, p.relw, p.heads, p.window, p.scale, out=bufs["att"])
print("att max diff", (bufs["att"].float().cpu() - att_ref).abs().max().item(), "absmax", att_ref.abs().max().item())
aq_ref = fake_quant(att_ref, o.scales[pre + "attn.proj"])
ops.quantize(bufs["att"], p.s_proj, out=bufs["att8"])
d = (bufs["att8"].float().cpu() * p.s_proj - aq_ref).abs()
print("att codes diff frac", (d > 1e-6).float().mean().item(), "max", d.max().item() / p.s_proj)
proj_ref = F.linear(aq_ref, o.p[pre + "attn.proj.weight"], o.p[pre + "attn.proj.bias"])
x1_ref = xo + proj_ref
p.proj.forward_w4a8(bufs["att8"], p.s_proj, ops.EPI_RESADD_F32, out=bufs["x"])
print("x1 max diff", (bufs["x"].cpu() - x1_ref).abs().max().item())
z = F.layer_norm(x1_ref, (c,), o.p[pre + "norm2.weight"], o.p[pre + "norm2.bias"], eps=1e-6)
zq = fake_quant(z, o.scales[pre + "mlp.lin1"])
ops.layernorm_q(bufs["x"], p.ln2_w, p.ln2_b, p.ln2_eps, out_scale=p.s_lin1, out=bufs["xn8"])
d = (bufs["xn8"].float().cpu() * p.s_lin1 - zq).abs()
print("LN2 codes diff frac", (d > 1e-6).float().mean().item())
h = F.gelu(F.linear(zq, o.p[pre + "mlp.lin1.weight"], o.p[pre + "mlp.lin1.bias"]))
hq = fake_quant(h, o.scales[pre + "mlp.lin2"])
p.lin1.forward_w4a8(bufs["xn8"], p.s_lin1, ops.EPI_Q8_GELU, out=bufs["hid8"], out_scale=p.s_lin2)
d = (bufs["hid8"].float().cpu() * p.s_lin2 - hq).abs()
print("hid codes diff frac", (d > 1e-6).float().mean().item(), "max", d.max().item() / p.s_lin2)
x2_ref = x1_ref + F.linear(hq, o.p[pre + "mlp.lin2.weight"], o.p[pre + "mlp.lin2.bias"])
p.lin2.forward_w4a8(bufs["hid8"], p.s_lin2, ops.EPI_RESADD_F32, out=bufs["x"])
print("x2 max diff", (bufs["x"].cpu() - x2_ref).abs().max().item(), "absmax", x2_ref.abs().max().item())

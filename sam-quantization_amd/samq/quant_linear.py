"""``QuantLinear`` / ``make_quant`` / ``matmul4`` -- the reference's ``gptq_triton.quant_linear``
API (``gptq_triton/quant_linear.py``) on the HIP W4A16 kernel.

Same class/function names, constructor arguments, buffer names, dtypes and shapes as the
reference (so a ``model.pt`` written by ``gptq4sam.py`` loads unchanged), same exceptions.
Differences (documented in DESIGN.md):

* no module-global ``workspace`` (reference ``:13``): outputs are fresh tensors, so calls are
  reentrant, batch > 1 works and outputs never alias;
* the weight is repacked ONCE into the kernel's fragment order (non-persistent buffer
  ``wpacked``; rebuilt automatically if ``qweight`` changes);
* shape constraints are relaxed to ``K % 64 == 0`` and ``N % 32 == 0``; the reference's
  ``K != 8 * qweight.rows`` check still raises ``AssertionError``;
* the bias add is fused into the GEMM epilogue.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn

from . import _lib, ops


def make_quant(model: nn.Module, bits: int, groupsize: int) -> None:
    """Replace every ``nn.Linear`` except one named ``lm_head`` by ``QuantLinear``
    (reference ``quant_linear.py:15-36``)."""
    for name, m in list(model.named_modules()):
        if not isinstance(m, nn.Linear) or name == "lm_head":
            continue
        q = QuantLinear(bits, groupsize, m.in_features, m.out_features, m.bias is not None)
        parent_name, _, child = name.rpartition(".")
        parent = model.get_submodule(parent_name) if parent_name else model
        setattr(parent, child, q)


class QuantLinear(nn.Module):
    """GPTQ int4 Linear (reference ``quant_linear.py:66-116``)."""

    def __init__(self, bits: int, groupsize: int, infeatures: int, outfeatures: int, bias: bool):
        super().__init__()
        if bits not in [4]:
            raise NotImplementedError("Only 4 bits are supported.")
        groupsize = infeatures if groupsize == -1 else groupsize
        self.infeatures = infeatures
        self.outfeatures = outfeatures
        self.bits = bits
        self.groupsize = groupsize
        per_int = 32 // bits
        assert outfeatures % per_int == 0, "outfeatures must be a multiple of features_per_int"
        ng = math.ceil(infeatures / groupsize)
        self.register_buffer("qweight", torch.empty((infeatures // per_int, outfeatures), dtype=torch.int32))
        self.register_buffer("qzeros", torch.empty((ng, outfeatures // per_int), dtype=torch.int32))
        self.register_buffer("scales", torch.empty((ng, outfeatures), dtype=torch.float16))
        if bias:
            self.register_buffer("bias", torch.empty(outfeatures, dtype=torch.float16))
        else:
            self.register_parameter("bias", None)
        self.register_buffer("wpacked", None, persistent=False)
        self._packed_from = None
        # W4A8: an fq_vit QAct on the input (make_act_quant); None = W4A16
        self.act_quant = None
        self._w4a8 = None
        self.gemm_cfg = 0   # W4A16 tile config; 0 = the library's per-shape pick (tools/bench_lanes.py)

    @property
    def gemm_cfg(self) -> int:
        return self._gemm_cfg

    @gemm_cfg.setter
    def gemm_cfg(self, cfg: int) -> None:
        cfg = int(cfg)
        # the tuning build (SAMQ_LIB=tuning) also carries the timing-only / experimental configs;
        # its C ABI range-checks them itself (SAMQ_ERR_INVALID for unknown ones)
        if cfg != 0 and cfg not in ops.W4A16_CFGS and _lib.LIB_PATH.name != "libsamq_hip_tuning.so":
            raise ValueError(f"gemm_cfg {cfg} is not a product tile config (0 or one of {sorted(ops.W4A16_CFGS)})")
        self._gemm_cfg = cfg

    # -- kernel-side weight layout ------------------------------------------------------
    def prepare(self) -> torch.Tensor:
        """Repack ``qweight`` for the kernel (once; redone if the buffer was replaced)."""
        key = (self.qweight.data_ptr(), self.qweight.device, self.qweight._version)
        if self.wpacked is None or self._packed_from != key:
            self.wpacked = ops.w4_repack(self.qweight)
            self._packed_from = key
        return self.wpacked

    def prepare_w4a8(self) -> dict:
        """Kernel-side buffers of the W4A8 GEMM: int4 weights in the int8-MFMA fragment order
        (repack layout 3), f32 scales ([G, N]; G = 1 per-channel) and bias.  Grouped weights need
        a groupsize that is a multiple of 128 (the int8 kernel's K tile)."""
        if self.groupsize != self.infeatures and self.groupsize % 128:
            raise NotImplementedError("W4A8 with grouped weights needs groupsize % 128 == 0")
        key = (self.qweight.data_ptr(), self.qweight.device, self.qweight._version, self.scales._version)
        if self._w4a8 is None or self._w4a8["key"] != key:
            self._w4a8 = dict(key=key, packed=ops.w4_repack(self.qweight, layout=3),
                              scale=self.scales.float().reshape(-1).contiguous(),
                              bias=None if self.bias is None else self.bias.float().contiguous())
        return self._w4a8

    def act_scale(self) -> Optional[float]:
        """The calibrated int8 input scale in quant mode, else None (W4A16)."""
        aq = self.act_quant
        if aq is None or not aq.quant or aq.calibrate:
            return None
        sc = aq.quantizer.scale
        if sc is None or sc.numel() != 1:
            raise RuntimeError("QuantLinear.act_quant is not calibrated (layer-wise scale expected)")
        return float(sc.reshape(-1)[0])

    def forward_w4a8(self, codes: torch.Tensor, a_scale: float, epilogue: int, out: Optional[torch.Tensor] = None,
                     out_scale: float = 0.0, rowsum: Optional[torch.Tensor] = None,
                     rowsum_out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """int8 input codes (scale ``a_scale``) x int4 weights on the int8 MFMA.  Per-channel weights:
        ``rowsum`` / ``rowsum_out`` = the input / output rows' code sums (``ops.w4a8_gemm``)."""
        w = self.prepare_w4a8()
        gs = -1 if self.groupsize == self.infeatures else self.groupsize
        return ops.w4a8_gemm(codes, w["packed"], w["scale"], self.qzeros, self.outfeatures, w["bias"], epilogue,
                             a_scale, out_scale, out=out, groupsize=gs, cfg=getattr(self, "i8_cfg", 0),
                             rowsum=rowsum, rowsum_out=rowsum_out)

    def forward_lnf(self, x: torch.Tensor, epilogue: int, out: torch.Tensor, stats: torch.Tensor, mu: torch.Tensor,
                    **kw) -> torch.Tensor:
        """The W4A16 GEMM with a LayerNorm folded into its epilogue (ops.w4a16_gemm_lnf)."""
        return ops.w4a16_gemm_lnf(x, self.prepare(), self.scales, self.qzeros, self.bias, self.outfeatures,
                                  self.groupsize, epilogue, out, stats, mu, cfg=self.gemm_cfg, **kw)

    def ln_fold_constants(self, gamma: torch.Tensor, beta: torch.Tensor):
        """``(gamma . W, beta . W)`` f32 [N] for a LayerNorm folded into this layer's input, computed by
        this layer's own GEMM (so they carry exactly the weights the kernel multiplies: s (q - zp),
        or fp16((q - zp) s) per group) on [gamma_hi; gamma_lo; beta_hi; beta_lo] f16 rows (hi + lo
        split: the f32 LayerNorm parameters to ~2^-22)."""
        rows = []
        for v in (gamma, beta):
            v = v.float().reshape(1, -1)
            hi = v.half()
            rows += [hi, (v - hi.float()).half()]
        a = torch.cat(rows).contiguous()
        out = ops.w4a16_gemm(a, self.prepare(), self.scales, self.qzeros, None, self.outfeatures, self.groupsize,
                             ops.EPI_F32)
        return (out[0] + out[1]).contiguous(), (out[2] + out[3]).contiguous()

    def forward_epilogue(self, x: torch.Tensor, epilogue: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        assert x.shape[-1] == self.qweight.shape[0] * 8, "A must be a multiple of 8 in the last dimension"
        return ops.w4a16_gemm(x, self.prepare(), self.scales, self.qzeros, self.bias, self.outfeatures,
                              self.groupsize, epilogue, out=out, cfg=self.gemm_cfg)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.act_quant is not None:
            s = self.act_scale()
            if s is not None:
                codes = ops.quantize(x.contiguous(), s)
                return self.forward_w4a8(codes, s, ops.EPI_BIAS)
            if self.act_quant.calibrate:
                self.act_quant(x.float())          # observer pass (fq_vit calibrate mode)
        return self.forward_epilogue(x, ops.EPI_BIAS)

    def extra_repr(self) -> str:
        return f"infeatures={self.infeatures}, outfeatures={self.outfeatures}, bits={self.bits}, groupsize={self.groupsize}"


def matmul4(groupsize: int, a: torch.Tensor, qweight: torch.Tensor, scales: torch.Tensor, qzeros: torch.Tensor,
            bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Functional ``C = A x W4 + bias`` (reference ``triton_matmul4``, ``quant_linear.py:355-437``).

    ``a`` (..., K) fp16; ``qweight`` int32 (K/8, N); ``scales`` fp16 (G, N); ``qzeros`` int32
    (G, N/8); ``bias`` fp16 (N).  Returns a fresh fp16 (..., N).  The weight is repacked per
    call (use ``QuantLinear`` to repack once).
    """
    assert a.shape[-1] == qweight.shape[0] * 8, "A must be a multiple of 8 in the last dimension"
    k = a.shape[-1]
    gs = -1 if groupsize in (-1, k) else groupsize
    return ops.w4a16_gemm(a, ops.w4_repack(qweight), scales, qzeros,
                          None if bias is None else bias.reshape(-1), qweight.shape[1], gs, ops.EPI_BIAS)


# drop-in alias: the reference's name for the functional entry point
triton_matmul4 = matmul4


def autotune_warmup(model: nn.Module):
    """Reference ``quant_linear.autotune_warmup`` (``:39-63``) returns per-(K,N) warmup closures.
    There is no autotuner here (tile configs are chosen analytically); the closures repack the
    weights and run one GEMM per unique shape so first-call costs leave the timed region."""
    mods = [m for m in model.modules() if isinstance(m, QuantLinear)]
    seen = {}
    for m in mods:
        seen.setdefault((m.infeatures, m.outfeatures), m)

    def make(mod):
        def run(mrows: int):
            a = torch.randn(1, mrows, mod.infeatures, dtype=torch.float16, device=mod.qweight.device)
            mod(a)
        return run

    return (make(m) for m in seen.values())


# ----------------------------------------------------------------------------- W4A8
def make_act_quant(model: nn.Module, cfg=None) -> int:
    """Attach an fq_vit ``QAct`` (int8 symmetric, layer-wise minmax, ``fq_vit/models/ptq/layers.py:
    203-242``) to the input of every ``QuantLinear``: the W4A8 composition of SURVEY.md §8c.
    Calibrate with ``calibrate_act_quant``; returns the number of quantisers attached."""
    from .fq_vit import QAct, sam_w8a8_config
    cfg = cfg or sam_w8a8_config()
    n = 0
    for m in model.modules():
        if isinstance(m, QuantLinear):
            dev = m.qweight.device
            m.act_quant = QAct(bit_type=cfg.BIT_TYPE_A, calibration_mode=cfg.CALIBRATION_MODE_A,
                               observer_str=cfg.OBSERVER_A, quantizer_str=cfg.QUANTIZER_A).to(dev)
            n += 1
    return n


@torch.no_grad()
def calibrate_act_quant(model: nn.Module, run, images) -> None:
    """fq_vit calibration sequence (``test_quant.py:284-294``) over the W4A8 input quantisers:
    ``run(img)`` must execute the MODULE forward (e.g. ``encoder.module_forward``)."""
    aqs = [m.act_quant for m in model.modules() if isinstance(m, QuantLinear) and m.act_quant is not None]
    images = list(images)
    for q in aqs:
        q.quant, q.calibrate, q.last_calibrate = False, True, False
    for i, img in enumerate(images):
        if i == len(images) - 1:
            for q in aqs:
                q.last_calibrate = True
        run(img)
    for q in aqs:
        q.calibrate, q.last_calibrate, q.quant = False, False, True

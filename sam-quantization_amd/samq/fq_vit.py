"""fq_vit W8A8 SAM image encoder: module API of the reference + the fused HIP int8 engine.

Mirrors (names, constructor arguments, flags, ``quantizer.scale`` buffers) the reference's
``fq_vit`` package so calibrated state dicts load unchanged:

* ``Config`` (``fq_vit/config.py:4-43``), ``BIT_TYPE_DICT`` (``models/ptq/bit_type.py:7-47``);
* ``MinmaxObserver`` (``observer/minmax.py:14-50``, ``observer/base.py:16-29``),
  ``UniformQuantizer`` (``quantizer/uniform.py:9-45``, ``quantizer/base.py:15-49``);
* ``QConv2d`` / ``QLinear`` / ``QAct`` / ``QIntLayerNorm`` / ``QIntSoftmax``
  (``models/ptq/layers.py:11-74, 160-200, 203-242, 245-258, 306-379``), ``QIntLayerNorm2D``
  (``models/sam/common.py:93-108``);
* the SAM encoder ``ImageEncoderViT`` / ``Block`` / ``Attention`` / ``PatchEmbed`` /
  ``MLPBlock`` with the 140 activation quantisers at the reference positions
  (``models/sam/image_encoder.py:18-478, 615-668``, ``common.py:15-73``);
* calibration switches ``model_open_calibrate`` / ``model_open_last_calibrate`` /
  ``model_close_calibrate`` / ``model_quant`` / ``model_dequant`` (``models/sam/sam.py:208-235``).

Supported configuration = the one the reference's SAM path uses (``test_quant.py:229-231``):
``Config(ptf=False, lis=False, quant_method="minmax")`` with ``BIT_TYPE_A = int8``: int8
symmetric per-channel weights, int8 symmetric layer-wise activations (zero point 0), plain
LayerNorm / softmax.  Other configurations raise ``NotImplementedError`` in quant mode.

Float and calibration forwards run the reference graph with torch ops (this is the observer
pass, not the hot path).  In quant mode on a GPU the encoder's forward is the fused HIP engine
(``W8A8Engine``): int8 codes flow between kernels, every quantiser is folded into the producing
kernel's epilogue (GEMM epilogues, LayerNorm, attention) -- there is no CPU or torch fallback.
"""
from __future__ import annotations

from typing import Optional, Tuple, Type

import torch
import torch.nn as nn
import torch.nn.functional as F

from .modeling import get_rel_pos, window_partition, window_unpartition


# ----------------------------------------------------------------------------- bit types / config
class BitType:
    def __init__(self, bits: int, signed: bool, name: str):
        self.bits, self.signed, self.name = bits, signed, name

    @property
    def upper_bound(self) -> int:
        return 2 ** (self.bits - 1) - 1 if self.signed else 2 ** self.bits - 1

    @property
    def lower_bound(self) -> int:
        return -(2 ** (self.bits - 1)) if self.signed else 0

    @property
    def range(self) -> int:
        return 2 ** self.bits


BIT_TYPE_DICT = {name: BitType(b, s, name) for name, b, s in
                 (("int8", 8, True), ("uint8", 8, False), ("uint4", 4, False), ("int4", 4, True),
                  ("uint2", 2, False))}


class Config:
    """``fq_vit/config.py:4-43`` (same attribute names and defaults)."""

    def __init__(self, ptf: bool = True, lis: bool = True, quant_method: str = "minmax"):
        self.BIT_TYPE_W = BIT_TYPE_DICT["int8"]
        self.BIT_TYPE_A = BIT_TYPE_DICT["uint8"]
        self.OBSERVER_W = "minmax"
        self.OBSERVER_A = quant_method
        self.QUANTIZER_W = "uniform"
        self.QUANTIZER_A = "uniform"
        self.QUANTIZER_A_LN = "uniform"
        self.CALIBRATION_MODE_W = "channel_wise"
        self.CALIBRATION_MODE_A = "layer_wise"
        self.CALIBRATION_MODE_S = "layer_wise"
        if lis:
            self.INT_SOFTMAX = True
            self.BIT_TYPE_S = BIT_TYPE_DICT["uint4"]
            self.OBSERVER_S = "minmax"
            self.QUANTIZER_S = "log2"
        else:
            self.INT_SOFTMAX = False
            self.BIT_TYPE_S = BIT_TYPE_DICT["uint8"]
            self.OBSERVER_S = self.OBSERVER_A
            self.QUANTIZER_S = self.QUANTIZER_A
        if ptf:
            self.INT_NORM = True
            self.OBSERVER_A_LN = "ptf"
            self.CALIBRATION_MODE_A_LN = "channel_wise"
        else:
            self.INT_NORM = False
            self.OBSERVER_A_LN = self.OBSERVER_A
            self.CALIBRATION_MODE_A_LN = self.CALIBRATION_MODE_A


def sam_w8a8_config() -> Config:
    """The configuration of the reference's SAM W8A8 run (``quant_fq-vit.sh:1``,
    ``test_quant.py:229-231``)."""
    cfg = Config(False, False, "minmax")
    cfg.BIT_TYPE_A = BIT_TYPE_DICT["int8"]
    return cfg


# ----------------------------------------------------------------------------- observer / quantizer
class MinmaxObserver:
    """``observer/minmax.py:14-50``; running min / max (per channel, or reduced layer-wise)."""

    def __init__(self, module_type: str, bit_type: BitType, calibration_mode: str, permute: bool = True):
        if module_type not in ("conv_weight", "linear_weight", "activation"):
            raise NotImplementedError(module_type)
        self.module_type, self.bit_type, self.calibration_mode, self.permute = (
            module_type, bit_type, calibration_mode, permute)
        self.max_val = None
        self.min_val = None
        self.eps = torch.finfo(torch.float32).eps
        self.symmetric = bit_type.signed

    def reshape_tensor(self, v: torch.Tensor) -> torch.Tensor:
        v = v.detach()
        if self.module_type in ("conv_weight", "linear_weight"):
            return v.reshape(v.shape[0], -1)
        if v.dim() == 4 and self.permute:
            v = v.permute(0, 2, 3, 1)
        return v.reshape(-1, v.shape[-1]).transpose(0, 1)

    def update(self, v: torch.Tensor) -> None:
        if v.is_cuda:
            return self._update_hip(v)
        v = self.reshape_tensor(v)
        cur_max, cur_min = v.max(dim=1).values, v.min(dim=1).values
        self.max_val = cur_max if self.max_val is None else torch.max(cur_max, self.max_val)
        self.min_val = cur_min if self.min_val is None else torch.min(cur_min, self.min_val)
        if self.calibration_mode == "layer_wise":
            self.max_val = self.max_val.max()
            self.min_val = self.min_val.min()

    def _update_hip(self, v: torch.Tensor) -> None:
        """GPU tensors: the same statistics from one HIP reduction (``samq_minmax``) on the
        un-transposed layout -- rows of ``(out, -1)`` for weights, columns of the channel-last
        ``(-1, C)`` view for activations, everything for layer_wise.  Bit-identical to the torch
        path (max / min are exact); running values are f32 for f32 / f16 / bf16 inputs alike
        (the torch path keeps the input dtype: same values, as the inputs convert exactly)."""
        from . import ops, _lib
        v = v.detach()
        if v.dtype not in (torch.float32, torch.float16):
            v = v.float()
        if self.module_type in ("conv_weight", "linear_weight"):
            x2d = v.reshape(v.shape[0], -1).contiguous()
            per = _lib.MM_PER_ROW
        else:
            if v.dim() == 4 and self.permute:
                v = v.permute(0, 2, 3, 1)
            x2d = v.reshape(-1, v.shape[-1]).contiguous()
            per = _lib.MM_PER_COL
        axis = _lib.MM_ALL if self.calibration_mode == "layer_wise" else per
        if self.max_val is not None:
            want = () if axis == _lib.MM_ALL else (x2d.shape[0] if per == _lib.MM_PER_ROW else x2d.shape[1],)
            if tuple(self.max_val.shape) != want or self.max_val.dtype != torch.float32 or not self.max_val.is_cuda:
                raise ValueError(f"MinmaxObserver: running statistics of shape {tuple(self.max_val.shape)} "
                                 f"do not match this tensor's {want}")
            self.max_val, self.min_val = ops.minmax_update(x2d, axis, self.max_val.clone(), self.min_val.clone())
        else:
            self.max_val, self.min_val = ops.minmax_update(x2d, axis)

    def get_quantization_params(self, *args, **kwargs):
        qmax, qmin = self.bit_type.upper_bound, self.bit_type.lower_bound
        # fp32 division done as a correctly rounded f64 quotient: GPU torch divides by a Python
        # scalar through its reciprocal (1-ulp differences); the reference runs it on the CPU
        if self.symmetric:
            scale = (torch.max(-self.min_val, self.max_val).double() / (float(qmax - qmin) / 2)).float()
            scale.clamp_(self.eps)
            zero_point = torch.zeros_like(self.max_val, dtype=torch.int64)
        else:
            scale = ((self.max_val - self.min_val).double() / float(qmax - qmin)).float()
            scale.clamp_(self.eps)
            zero_point = (qmin - torch.round(self.min_val / scale)).clamp_(qmin, qmax)
        return scale, zero_point


def build_observer(observer_str, module_type, bit_type, calibration_mode, permute=True):
    """``observer/build.py:17-19`` (minmax only)."""
    if observer_str != "minmax":
        raise NotImplementedError(f"observer {observer_str!r}: only minmax is supported")
    return MinmaxObserver(module_type, bit_type, calibration_mode, permute=permute)


class UniformQuantizer(nn.Module):
    """``quantizer/uniform.py:9-45``: ``(clamp(round(x / s + zp), lo, hi) - zp) * s``."""

    def __init__(self, bit_type, observer, module_type, permute=True):
        super().__init__()
        self.bit_type, self.observer, self.module_type, self.permute = bit_type, observer, module_type, permute
        self.scale = None
        self.zero_point = None

    def update_quantization_params(self, *args, **kwargs):
        scale, zero = self.observer.get_quantization_params(*args, **kwargs)
        if "scale" in self._buffers:
            del self._buffers["scale"], self._buffers["zero_point"]
        else:
            del self.scale, self.zero_point
        self.register_buffer("scale", scale)
        self.register_buffer("zero_point", zero)

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        # calibrated checkpoints carry scale / zero_point buffers that do not exist before calibration
        for name in ("scale", "zero_point"):
            key = prefix + name
            if key in state_dict and name not in self._buffers:
                if name in self.__dict__:
                    del self.__dict__[name]
                self.register_buffer(name, torch.empty_like(state_dict[key]))
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                                      error_msgs)

    def get_reshape_range(self, inputs):
        if self.module_type == "conv_weight":
            return (-1, 1, 1, 1)
        if self.module_type == "linear_weight":
            return (-1, 1)
        nd = inputs.dim()
        if nd == 2:
            return (1, -1)
        if nd == 3:
            return (1, 1, -1)
        if nd == 4:
            return (1, -1, 1, 1) if self.permute else (1, 1, 1, -1)
        raise NotImplementedError

    def quant(self, inputs, scale=None, zero_point=None):
        scale = (self.scale if scale is None else scale).reshape(self.get_reshape_range(inputs))
        zero_point = (self.zero_point if zero_point is None else zero_point).reshape(self.get_reshape_range(inputs))
        return (inputs / scale + zero_point).round().clamp(self.bit_type.lower_bound, self.bit_type.upper_bound)

    def dequantize(self, inputs, scale=None, zero_point=None):
        scale = (self.scale if scale is None else scale).reshape(self.get_reshape_range(inputs))
        zero_point = (self.zero_point if zero_point is None else zero_point).reshape(self.get_reshape_range(inputs))
        return (inputs - zero_point) * scale

    def forward(self, inputs):
        return self.dequantize(self.quant(inputs))


def build_quantizer(quantizer_str, bit_type, observer, module_type, permute=True):
    """``quantizer/build.py:8-10`` (uniform only)."""
    if quantizer_str != "uniform":
        raise NotImplementedError(f"quantizer {quantizer_str!r}: only uniform is supported")
    return UniformQuantizer(bit_type, observer, module_type, permute=permute)


# ----------------------------------------------------------------------------- layers
class _QFlags:
    def _init_q(self, quant, calibrate, last_calibrate, bit_type, calibration_mode, observer_str, quantizer_str,
                module_type, permute=True):
        self.quant, self.calibrate, self.last_calibrate = quant, calibrate, last_calibrate
        self.bit_type, self.calibration_mode = bit_type, calibration_mode
        self.observer_str, self.quantizer_str, self.module_type = observer_str, quantizer_str, module_type
        self.observer = build_observer(observer_str, module_type, bit_type, calibration_mode, permute=permute)
        self.quantizer = build_quantizer(quantizer_str, bit_type, self.observer, module_type, permute=permute)

    def _observe(self, v, x):
        if self.calibrate:
            self.quantizer.observer.update(v)
            if self.last_calibrate:
                self.quantizer.update_quantization_params(x)


class QConv2d(nn.Conv2d, _QFlags):
    """``layers.py:11-74``: conv with per-output-channel int8 fake-quant weights in quant mode."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1, bias=True,
                 quant=False, calibrate=False, last_calibrate=False, bit_type=BIT_TYPE_DICT["int8"],
                 calibration_mode="layer_wise", observer_str="minmax", quantizer_str="uniform"):
        nn.Conv2d.__init__(self, in_channels, out_channels, kernel_size, stride=stride, padding=padding,
                           dilation=dilation, groups=groups, bias=bias)
        self._init_q(quant, calibrate, last_calibrate, bit_type, calibration_mode, observer_str, quantizer_str,
                     "conv_weight")

    def forward(self, x):
        self._observe(self.weight, x)
        w = self.quantizer(self.weight) if self.quant else self.weight
        return F.conv2d(x, w, self.bias, self.stride, self.padding, self.dilation, self.groups)


class QLinear(nn.Linear, _QFlags):
    """``layers.py:160-200``."""

    def __init__(self, in_features, out_features, bias=True, quant=False, calibrate=False, last_calibrate=False,
                 bit_type=BIT_TYPE_DICT["int8"], calibration_mode="layer_wise", observer_str="minmax",
                 quantizer_str="uniform"):
        nn.Linear.__init__(self, in_features, out_features, bias)
        self._init_q(quant, calibrate, last_calibrate, bit_type, calibration_mode, observer_str, quantizer_str,
                     "linear_weight")

    def forward(self, x):
        self._observe(self.weight, x)
        w = self.quantizer(self.weight) if self.quant else self.weight
        return F.linear(x, w, self.bias)


class QAct(nn.Module, _QFlags):
    """``layers.py:203-242``.  In quant mode on a GPU the fake quant runs in the HIP quantiser."""

    def __init__(self, quant=False, calibrate=False, last_calibrate=False, bit_type=BIT_TYPE_DICT["int8"],
                 calibration_mode="layer_wise", observer_str="minmax", quantizer_str="uniform", permute=True):
        nn.Module.__init__(self)
        self._init_q(quant, calibrate, last_calibrate, bit_type, calibration_mode, observer_str, quantizer_str,
                     "activation", permute=permute)

    def forward(self, x):
        self._observe(x, x)
        if not self.quant:
            return x
        if x.is_cuda and self.bit_type.signed and x.dtype == torch.float32 and self.quantizer.scale.numel() == 1:
            from . import ops
            return ops.quantize(x.contiguous(), float(self.quantizer.scale), fake=True)
        return self.quantizer(x)


class QIntLayerNorm(nn.LayerNorm):
    """``layers.py:245-258``: the float LayerNorm (the reference returns on its first line)."""

    def __init__(self, normalized_shape, eps=1e-5, elementwise_affine=True):
        super().__init__(normalized_shape, eps, elementwise_affine)
        assert isinstance(normalized_shape, int)
        self.mode = "ln"

    def forward(self, x, in_quantizer=None, out_quantizer=None, in_scale_expand=1):
        return super().forward(x)


class QIntLayerNorm2D(nn.Module):
    """``models/sam/common.py:93-108``: channel LayerNorm of NCHW maps (float path, eps 1e-5)."""

    def __init__(self, num_channels: int, eps: float = 1e-5):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(num_channels))
        self.bias = nn.Parameter(torch.zeros(num_channels))
        self.eps = eps
        self.mode = "ln"

    def forward(self, x, in_quantizer=None, out_quantizer=None):
        u = x.mean(1, keepdim=True)
        s = (x - u).pow(2).mean(1, keepdim=True)
        x = (x - u) / torch.sqrt(s + self.eps)
        return self.weight[:, None, None] * x + self.bias[:, None, None]


class QIntSoftmax(nn.Module):
    """``layers.py:306-379``: plain softmax (the reference returns ``F.softmax`` first)."""

    def __init__(self, log_i_softmax=False, quant=False, calibrate=False, last_calibrate=False,
                 bit_type=BIT_TYPE_DICT["int8"], calibration_mode="layer_wise", observer_str="minmax",
                 quantizer_str="uniform"):
        super().__init__()
        self.log_i_softmax, self.quant, self.calibrate, self.last_calibrate = (
            log_i_softmax, quant, calibrate, last_calibrate)
        self.bit_type = bit_type

    def forward(self, x, scale=None):
        return F.softmax(x, dim=-1)


def _qact(cfg: Config, quant: bool, calibrate: bool, ln: bool = False, permute: bool = True) -> QAct:
    if ln:
        return QAct(quant=quant, calibrate=calibrate, bit_type=cfg.BIT_TYPE_A,
                    calibration_mode=cfg.CALIBRATION_MODE_A_LN, observer_str=cfg.OBSERVER_A_LN,
                    quantizer_str=cfg.QUANTIZER_A_LN, permute=permute)
    return QAct(quant=quant, calibrate=calibrate, bit_type=cfg.BIT_TYPE_A, calibration_mode=cfg.CALIBRATION_MODE_A,
                observer_str=cfg.OBSERVER_A, quantizer_str=cfg.QUANTIZER_A, permute=permute)


def _qlinear(cfg: Config, i: int, o: int, bias: bool, quant: bool, calibrate: bool) -> QLinear:
    return QLinear(i, o, bias=bias, quant=quant, calibrate=calibrate, bit_type=cfg.BIT_TYPE_W,
                   calibration_mode=cfg.CALIBRATION_MODE_W, observer_str=cfg.OBSERVER_W,
                   quantizer_str=cfg.QUANTIZER_W)


def _qconv(cfg: Config, i: int, o: int, k: int, stride: int = 1, padding: int = 0, bias: bool = True,
           quant: bool = False, calibrate: bool = False) -> QConv2d:
    return QConv2d(i, o, k, stride=stride, padding=padding, bias=bias, quant=quant, calibrate=calibrate,
                   bit_type=cfg.BIT_TYPE_W, calibration_mode=cfg.CALIBRATION_MODE_W, observer_str=cfg.OBSERVER_W,
                   quantizer_str=cfg.QUANTIZER_W)


# ----------------------------------------------------------------------------- encoder modules
class MLPBlock(nn.Module):
    """``fq_vit/models/sam/common.py:15-73``."""

    def __init__(self, embedding_dim, mlp_dim, act: Type[nn.Module] = nn.GELU, quant=False, calibrate=False,
                 cfg: Optional[Config] = None):
        super().__init__()
        self.lin1 = _qlinear(cfg, embedding_dim, mlp_dim, True, quant, calibrate)
        self.qact1 = _qact(cfg, quant, calibrate)
        self.lin2 = _qlinear(cfg, mlp_dim, embedding_dim, True, quant, calibrate)
        self.qact2 = _qact(cfg, quant, calibrate)
        self.act = act()

    def forward(self, x):
        return self.qact2(self.lin2(self.qact1(self.act(self.lin1(x)))))


def add_decomposed_rel_pos(attn, q, rel_pos_h, rel_pos_w, q_size, k_size):
    """``segment_anything/modeling/image_encoder.py:369-408`` (quirk-1 width term by query row)."""
    q_h, q_w = q_size
    k_h, k_w = k_size
    rh = get_rel_pos(q_h, k_h, rel_pos_h)
    rw = get_rel_pos(q_w, k_w, rel_pos_w)
    b, _, dim = q.shape
    r_q = q.reshape(b, q_h, q_w, dim)
    rel_h = torch.einsum("bhwc,hkc->bhwk", r_q, rh)
    rel_w = torch.einsum("bhwc,hkc->bhwk", r_q, rw)
    attn = (attn.view(b, q_h, q_w, k_h, k_w) + rel_h[:, :, :, :, None] + rel_w[:, :, :, None, :])
    return attn.view(b, q_h * q_w, k_h * k_w)


class Attention(nn.Module):
    """``fq_vit/models/sam/image_encoder.py:334-478``."""

    def __init__(self, dim, num_heads=8, qkv_bias=True, use_rel_pos=False, rel_pos_zero_init=True,
                 input_size: Optional[Tuple[int, int]] = None, quant=False, calibrate=False,
                 cfg: Optional[Config] = None):
        super().__init__()
        self.num_heads = num_heads
        head_dim = dim // num_heads
        self.scale = head_dim ** -0.5
        self.qkv = _qlinear(cfg, dim, dim * 3, qkv_bias, quant, calibrate)
        self.qact_attn1 = _qact(cfg, quant, calibrate)
        self.qact1 = _qact(cfg, quant, calibrate)
        self.qact2 = _qact(cfg, quant, calibrate)
        self.proj = _qlinear(cfg, dim, dim, True, quant, calibrate)
        self.qact3 = _qact(cfg, quant, calibrate)
        self.use_rel_pos = use_rel_pos
        if use_rel_pos:
            assert input_size is not None
            self.rel_pos_h = nn.Parameter(torch.zeros(2 * input_size[0] - 1, head_dim))
            self.rel_pos_w = nn.Parameter(torch.zeros(2 * input_size[1] - 1, head_dim))
            self.use_rel_pos_qact = _qact(cfg, quant, calibrate)
        self.log_int_softmax = QIntSoftmax(log_i_softmax=cfg.INT_SOFTMAX, quant=quant, calibrate=calibrate,
                                           bit_type=cfg.BIT_TYPE_S, calibration_mode=cfg.CALIBRATION_MODE_S,
                                           observer_str=cfg.OBSERVER_S, quantizer_str=cfg.QUANTIZER_S)

    def forward(self, x):
        b, h, w, c = x.shape
        qkv = self.qact1(self.qkv(x.reshape(b, h * w, c))).reshape(b, h * w, 3, self.num_heads, -1)
        q, k, v = qkv.permute(2, 0, 3, 1, 4).reshape(3, b * self.num_heads, h * w, -1).unbind(0)
        attn = self.qact_attn1((q * self.scale) @ k.transpose(-2, -1))
        if self.use_rel_pos:
            attn = self.use_rel_pos_qact(add_decomposed_rel_pos(attn, q, self.rel_pos_h, self.rel_pos_w,
                                                                (h, w), (h, w)))
        attn = self.log_int_softmax(attn)
        x = (attn @ v).view(b, self.num_heads, h, w, -1).permute(0, 2, 3, 1, 4).reshape(b, h, w, -1)
        return self.qact3(self.proj(self.qact2(x)))


class Block(nn.Module):
    """``fq_vit/models/sam/image_encoder.py:216-331``."""

    def __init__(self, dim, num_heads, mlp_ratio=4.0, qkv_bias=True, norm_layer=nn.LayerNorm, act_layer=nn.GELU,
                 use_rel_pos=False, rel_pos_zero_init=True, window_size=0, input_size=None, quant=False,
                 calibrate=False, cfg: Optional[Config] = None):
        super().__init__()
        self.norm1 = norm_layer(dim)
        self.qact1 = _qact(cfg, quant, calibrate, ln=True, permute=False)
        self.attn = Attention(dim, num_heads=num_heads, qkv_bias=qkv_bias, use_rel_pos=use_rel_pos,
                              rel_pos_zero_init=rel_pos_zero_init,
                              input_size=input_size if window_size == 0 else (window_size, window_size),
                              quant=quant, calibrate=calibrate, cfg=cfg)
        self.qact2 = _qact(cfg, quant, calibrate, permute=False)
        self.norm2 = norm_layer(dim)
        self.qact3 = _qact(cfg, quant, calibrate, ln=True, permute=False)
        self.mlp = MLPBlock(dim, int(dim * mlp_ratio), act=act_layer, quant=quant, calibrate=calibrate, cfg=cfg)
        self.qact4 = _qact(cfg, quant, calibrate, permute=False)
        self.window_size = window_size

    def forward(self, x, last_quantizer=None):
        shortcut = x
        x = self.qact1(self.norm1(x))
        if self.window_size > 0:
            h, w = x.shape[1], x.shape[2]
            x, pad_hw = window_partition(x, self.window_size)
        x = self.attn(x)
        if self.window_size > 0:
            x = window_unpartition(x, self.window_size, pad_hw, (h, w))
        x = self.qact2(shortcut + x)
        return self.qact4(x + self.mlp(self.qact3(self.norm2(x))))


class PatchEmbed(nn.Module):
    """``fq_vit/models/sam/image_encoder.py:615-668``."""

    def __init__(self, kernel_size=(16, 16), stride=(16, 16), padding=(0, 0), in_chans=3, embed_dim=768,
                 quant=False, calibrate=False, cfg: Optional[Config] = None):
        super().__init__()
        self.proj = _qconv(cfg, in_chans, embed_dim, kernel_size[0], stride=stride[0], padding=padding[0],
                           quant=quant, calibrate=calibrate)
        self.qact = _qact(cfg, quant, calibrate)

    def forward(self, x):
        return self.qact(self.proj(x)).permute(0, 2, 3, 1)


class ImageEncoderViT(nn.Module):
    """``fq_vit/models/sam/image_encoder.py:18-213`` (W8A8 SAM ViT encoder)."""

    def __init__(self, img_size=1024, patch_size=16, in_chans=3, embed_dim=768, depth=12, num_heads=12,
                 mlp_ratio=4.0, out_chans=256, qkv_bias=True, norm_layer=nn.LayerNorm, act_layer=nn.GELU,
                 use_abs_pos=True, use_rel_pos=False, rel_pos_zero_init=True, window_size=0,
                 global_attn_indexes: Tuple[int, ...] = (), quant=False, calibrate=False,
                 cfg: Optional[Config] = None, input_quant=True):
        super().__init__()
        cfg = cfg or sam_w8a8_config()
        self.cfg = cfg
        self.img_size = img_size
        self.input_quant = input_quant
        self.qact_input = _qact(cfg, quant, calibrate)
        self.patch_embed = PatchEmbed(kernel_size=(patch_size, patch_size), stride=(patch_size, patch_size),
                                      in_chans=in_chans, embed_dim=embed_dim, quant=quant, calibrate=calibrate,
                                      cfg=cfg)
        self.pos_embed = None
        if use_abs_pos:
            self.pos_embed = nn.Parameter(torch.zeros(1, img_size // patch_size, img_size // patch_size, embed_dim))
        self.qact_pos = _qact(cfg, quant, calibrate, permute=False)
        self.qact1 = _qact(cfg, quant, calibrate, permute=False)
        self.blocks = nn.ModuleList([
            Block(dim=embed_dim, num_heads=num_heads, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, norm_layer=norm_layer,
                  act_layer=act_layer, use_rel_pos=use_rel_pos, rel_pos_zero_init=rel_pos_zero_init,
                  window_size=window_size if i not in global_attn_indexes else 0,
                  input_size=(img_size // patch_size, img_size // patch_size), quant=quant, calibrate=calibrate,
                  cfg=cfg)
            for i in range(depth)])
        self.neck = nn.ModuleList([
            _qconv(cfg, embed_dim, out_chans, 1, bias=False, quant=quant, calibrate=calibrate),
            QIntLayerNorm2D(out_chans),
            _qconv(cfg, out_chans, out_chans, 3, padding=1, bias=False, quant=quant, calibrate=calibrate),
            QIntLayerNorm2D(out_chans)])
        self.qacts = nn.ModuleList([_qact(cfg, quant, calibrate, ln=True) for _ in range(4)])
        self.global_attn_indexes = tuple(global_attn_indexes)
        self.window_size = window_size
        self._engine = None

    # -- calibration switches (fq_vit/models/sam/sam.py:208-235) ------------------------------------
    def _qmods(self):
        return [m for m in self.modules() if type(m) in (QConv2d, QLinear, QAct, QIntSoftmax)]

    def model_quant(self):
        for m in self._qmods():
            m.quant = True
        self._engine = None

    def model_dequant(self):
        for m in self._qmods():
            m.quant = False

    def model_open_calibrate(self):
        for m in self._qmods():
            m.calibrate = True

    def model_open_last_calibrate(self):
        for m in self._qmods():
            m.last_calibrate = True

    def model_close_calibrate(self):
        for m in self._qmods():
            m.calibrate = False
        self._engine = None

    @torch.no_grad()
    def calibrate_with(self, images) -> None:
        """The reference calibration sequence (``test_quant.py:284-294``): observe every image,
        compute the scales on the last one, close calibration and switch to quant mode."""
        images = list(images)
        self.model_open_calibrate()
        for i, img in enumerate(images):
            if i == len(images) - 1:
                self.model_open_last_calibrate()
            self.module_forward(img)
        self.model_close_calibrate()
        self.model_quant()

    def is_quant(self) -> bool:
        return all(m.quant for m in self._qmods() if not isinstance(m, QIntSoftmax))

    def engine(self) -> "W8A8Engine":
        if self._engine is None:
            self._engine = W8A8Engine(self)
        return self._engine

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.is_quant() and not any(m.calibrate for m in self._qmods()):
            if not x.is_cuda:
                raise RuntimeError("fq_vit ImageEncoderViT: the quantized encoder runs on the GPU (HIP) only")
            return self.engine().forward(x)
        return self.module_forward(x)

    def module_forward(self, x: torch.Tensor) -> torch.Tensor:
        """The reference's module graph (float / calibration mode)."""
        if self.input_quant:
            x = self.qact_input(x)
        x = self.patch_embed(x)
        if self.pos_embed is not None:
            x = x + self.qact_pos(self.pos_embed)
        x = self.qact1(x)
        for blk in self.blocks:
            x = blk(x)
        x = x.permute(0, 3, 1, 2)
        for i, mod in enumerate(self.neck):
            x = self.qacts[i](mod(x))
        return x


def build_fq_image_encoder(name: str = "vit_b", img_size: int = 1024, cfg: Optional[Config] = None,
                           depth: Optional[int] = None, quant=False, calibrate=False) -> ImageEncoderViT:
    """fq_vit ``build_sam_vit_*`` encoder part (``fq_vit/models/sam/build_sam.py``)."""
    from .build_sam import VIT_HPARAMS
    hp = VIT_HPARAMS[name]
    from functools import partial
    return ImageEncoderViT(depth=depth or hp["encoder_depth"], embed_dim=hp["encoder_embed_dim"], img_size=img_size,
                           mlp_ratio=4, norm_layer=partial(QIntLayerNorm, eps=1e-6),
                           num_heads=hp["encoder_num_heads"], patch_size=16, qkv_bias=True, use_rel_pos=True,
                           global_attn_indexes=hp["encoder_global_attn_indexes"],
                           window_size=14, out_chans=256, quant=quant, calibrate=calibrate,
                           cfg=cfg or sam_w8a8_config())


def act_quantizers(enc: nn.Module) -> dict:
    """name -> QAct, with the fq_vit module paths as names (``blocks.0.attn.qact1`` ...)."""
    return {n: m for n, m in enc.named_modules() if isinstance(m, QAct)}


@torch.no_grad()
def set_act_scales(enc: nn.Module, scales: dict) -> None:
    """Install calibrated layer-wise activation scales (what a calibrated checkpoint's
    ``quantizer.scale`` / ``zero_point`` buffers hold) on every named QAct."""
    qa = act_quantizers(enc)
    missing = set(qa) - set(scales)
    if missing:
        raise KeyError(f"no scale for {sorted(missing)[:4]} ...")
    for n, m in qa.items():
        q = m.quantizer
        dev = next(enc.parameters()).device
        sc = torch.as_tensor(scales[n], dtype=torch.float32, device=dev).reshape(())
        for name, val in (("scale", sc), ("zero_point", torch.zeros((), dtype=torch.int64, device=dev))):
            if name in q._buffers:
                q._buffers[name] = val
            else:
                if name in q.__dict__:
                    del q.__dict__[name]
                q.register_buffer(name, val)
    if isinstance(enc, ImageEncoderViT):
        enc._engine = None


@torch.no_grad()
def calibrate_weights(enc: nn.Module) -> None:
    """Weight quantisers only (data independent): observe each QLinear / QConv2d weight once and
    compute its per-channel scale (``layers.py:191-194`` with last_calibrate)."""
    for m in enc.modules():
        if isinstance(m, (QLinear, QConv2d)):
            m.observer.max_val = m.observer.min_val = None
            m.observer.update(m.weight)
            m.quantizer.update_quantization_params()
    if isinstance(enc, ImageEncoderViT):
        enc._engine = None


# ----------------------------------------------------------------------------- fused W8A8 engine
def _s(q: QAct) -> float:
    sc = q.quantizer.scale
    if sc is None:
        raise RuntimeError("fq_vit: activation quantizer is not calibrated")
    if sc.numel() != 1:
        raise NotImplementedError("W8A8 engine: only layer-wise activation scales are supported")
    if q.quantizer.zero_point is not None and int(q.quantizer.zero_point.reshape(-1)[0]) != 0:
        raise NotImplementedError("W8A8 engine: only symmetric (zero point 0) activations are supported")
    return float(sc.reshape(-1)[0])


class W8A8Engine:
    """Fused HIP forward of a calibrated fq_vit encoder (quant mode), int8 codes end to end.

    Per block (all quantisers folded into the producing kernel):
      LN1+qact1 -> int8 | qkv GEMM + attn.qact1 -> int8 | attention (qact_attn1, rel-pos,
      use_rel_pos_qact, softmax, attn.qact2) -> int8 | proj GEMM + attn.qact3 + residual +
      blk.qact2 -> int8 x | LN2+qact3 -> int8 | lin1 GEMM + GELU + mlp.qact1 -> int8 |
      lin2 GEMM + mlp.qact2 + residual + blk.qact4 -> int8 x.
    Patch embed: image quantiser (HIP) + an implicit GEMM gathering the 16x16 patches from the
    NCHW codes (``samq_w8a8_conv_gemm`` mode 1) whose epilogue applies patch_embed.qact, adds
    qact_pos(pos_embed) and applies qact1.  Neck: 1x1 GEMM + qacts.0, LN2d + qacts.1, 3x3 implicit
    GEMM over the NHWC codes with the zero padding in the gather (mode 2) + qacts.2, LN2d +
    qacts.3 -> f32.  No im2col / pad copies.
    """

    def __init__(self, enc: ImageEncoderViT):
        from . import ops
        cfg = enc.cfg
        if not (cfg.BIT_TYPE_A.signed and cfg.BIT_TYPE_A.bits == 8) or cfg.INT_NORM or cfg.INT_SOFTMAX:
            raise NotImplementedError("W8A8 engine supports Config(ptf=False, lis=False) with BIT_TYPE_A=int8")
        self.enc = enc
        # LayerNorm-q rows per wave: one (1024 workgroups for the 4096 vit_b rows instead of 512) --
        # in the W8A8 graph 1.6543 vs 1.6836 ms per image, bit-identical; the ViT-H W4A8 graph keeps
        # the library default (two: -2.2 % with one, profiles/r5_ln_rpw_ab.log)
        self.ln_rpw = 1
        # row lanes (round 6, opt-in): one image as two concurrent kernel chains over the token grid's
        # rows (split on a window boundary: per-row LayerNorm / GEMMs / residual, whole windows),
        # joined around the global blocks' attention (every query reads every key); the neck's 3x3
        # conv after the final join.  Bit-identical to one chain (per-row kernels, integer-exact
        # GEMMs on any tile).  Measured SLOWER in the W8A8 graph: 1.826 vs 1.664 ms per image
        # (profiles/r6_w8a8_row_lanes.log) -- the step is not made of inter-kernel gaps that a
        # second chain could fill; halving every launch costs more.  1 = one chain (default).
        self.row_lanes = 1
        # global blocks (64 x 64 grid): the qkv GEMM also stores the V codes as fp16
        # (samq_w8a8_gemm_v16) and the global attention stages them unconverted (round 6; same codes)
        self.v16 = True
        dev = enc.pos_embed.device
        if dev.type != "cuda":
            raise RuntimeError("W8A8 engine: move the encoder to the GPU first")
        self.dev = dev
        self.ops = ops
        self.embed_dim = enc.patch_embed.proj.weight.shape[0]
        self.patch = enc.patch_embed.proj.kernel_size[0]
        self.s_in = _s(enc.qact_input) if enc.input_quant else None
        if self.s_in is None:
            raise NotImplementedError("W8A8 engine: input_quant=False is not supported")
        self.layers = {}
        self.patch_w = self._weight(enc.patch_embed.proj)
        s_pos = _s(enc.qact_pos)
        self.pos_codes = ops.quantize(enc.pos_embed.detach().float().contiguous(), s_pos).reshape(-1, self.embed_dim)
        self.s_pos = s_pos
        self.s_pe = _s(enc.patch_embed.qact)
        self.s_x0 = _s(enc.qact1)
        self.blocks = []
        for blk in enc.blocks:
            a = blk.attn
            self.blocks.append(dict(
                window=blk.window_size, heads=a.num_heads, scale=a.scale,
                n1=(blk.norm1.weight.detach().float().contiguous(), blk.norm1.bias.detach().float().contiguous(),
                    blk.norm1.eps),
                n2=(blk.norm2.weight.detach().float().contiguous(), blk.norm2.bias.detach().float().contiguous(),
                    blk.norm2.eps),
                qkv=self._weight(a.qkv), proj=self._weight(a.proj), lin1=self._weight(blk.mlp.lin1),
                lin2=self._weight(blk.mlp.lin2),
                relh=a.rel_pos_h.detach().float().contiguous(), relw=a.rel_pos_w.detach().float().contiguous(),
                qkv_bias=a.qkv.bias.detach().float().contiguous() if a.qkv.bias is not None else None,
                s_ln1=_s(blk.qact1), s_qkv=_s(a.qact1), s_a1=_s(a.qact_attn1), s_a2=_s(a.use_rel_pos_qact),
                s_ao=_s(a.qact2), s_proj=_s(a.qact3), s_x1=_s(blk.qact2), s_ln2=_s(blk.qact3),
                s_h=_s(blk.mlp.qact1), s_l2=_s(blk.mlp.qact2), s_x2=_s(blk.qact4)))
        self.neck0 = self._weight(enc.neck[0])
        self.neck2 = self._weight(enc.neck[2], tap_major=True)
        self.ln_n1 = (enc.neck[1].weight.detach().float().contiguous(), enc.neck[1].bias.detach().float().contiguous(),
                      enc.neck[1].eps)
        self.ln_n3 = (enc.neck[3].weight.detach().float().contiguous(), enc.neck[3].bias.detach().float().contiguous(),
                      enc.neck[3].eps)
        self.s_q = [_s(q) for q in enc.qacts]

    def _weight(self, mod, tap_major: bool = False):
        """Per-output-channel symmetric int8 codes of a QLinear / QConv2d weight (the reference's
        ``quantizer(self.weight)``, layers.py:196-199) packed for the int8 MFMA GEMM.
        ``tap_major``: conv weight flattened (n, ky, kx, c), the implicit 3x3 GEMM's K order."""
        w = mod.weight.detach().float()
        n = w.shape[0]
        w2 = (w.permute(0, 2, 3, 1) if tap_major else w).reshape(n, -1)
        s = mod.quantizer.scale
        if s is None:
            raise RuntimeError("fq_vit: weight quantizer is not calibrated")
        s = s.detach().float().reshape(-1).to(w.device)
        # round(fp32(w / s)) with the correctly rounded fp32 quotient (uniform.py:31-36)
        codes = torch.clamp(torch.round((w2.double() / s.double()[:, None]).float()), -128, 127).to(torch.int8)
        bias = None if mod.bias is None else mod.bias.detach().float().contiguous()
        return dict(packed=self.ops.w8_repack(codes), scale=s.contiguous(), bias=bias, n=n, k=w2.shape[1],
                    cfg=0)   # i8 GEMM tile config (0: the library's pick)

    def _gemm(self, a, lw, epi, a_scale, out_scale, mid=0.0, res=None, res_scale=0.0, out=None):
        return self.ops.w8a8_gemm(a, lw["packed"], lw["scale"], lw["n"], lw["bias"], epi, a_scale, out_scale, mid,
                                  res_scale, res, out, cfg=lw["cfg"])

    @torch.no_grad()
    def forward(self, img: torch.Tensor, taps: Optional[dict] = None) -> torch.Tensor:
        """``taps`` (debugging / tests): if a dict, receives the fake-quant f32 value of every
        inter-kernel activation under the reference QAct name that produced it."""
        ops = self.ops

        def tap(name, codes, s):
            if taps is not None:
                taps[name] = codes.float() * s
        img = img.to(self.dev, torch.float32).contiguous()
        b, cin, hh, ww = img.shape
        p = self.patch
        gh, gw = hh // p, ww // p
        c = self.embed_dim
        codes = ops.quantize(img, self.s_in)
        if p == 16 and hh == ww:
            pw = self.patch_w
            x = ops.w8a8_conv_gemm(codes, 1, pw["packed"], pw["scale"], pw["n"], pw["bias"], ops.EPI_Q8_RES,
                                   self.s_in, self.s_x0, mid_scale=self.s_pe, res_scale=self.s_pos, res=self.pos_codes,
                                   rmod=gh * gw).view(b * gh * gw, c)
        else:   # other patch geometries: explicit im2col
            cols = codes.view(b, cin, gh, p, gw, p).permute(0, 2, 4, 1, 3, 5).reshape(b * gh * gw, cin * p * p)
            pos = self.pos_codes if b == 1 else self.pos_codes.repeat(b, 1)
            x = self._gemm(cols.contiguous(), self.patch_w, ops.EPI_Q8_RES, self.s_in, self.s_x0, mid=self.s_pe,
                           res=pos, res_scale=self.s_pos)
        s_x = self.s_x0
        tap("qact1", x.view(b, gh, gw, c), s_x)
        xn = torch.empty_like(x)
        ao = torch.empty_like(x)
        v16buf = None
        split = self._row_split(gh)
        if taps is None and split:
            s_x = self._blocks_row_lanes(x, xn, ao, b, gh, gw, c, split)
            return self._neck(x, s_x, b, gh, gw)
        for i, bl in enumerate(self.blocks):
            pre = f"blocks.{i}."
            g1, b1, e1 = bl["n1"]
            ops.layernorm_q(x, g1, b1, e1, in_scale=s_x, out_scale=bl["s_ln1"], out=xn, rows_per_wave=self.ln_rpw)
            tap(pre + "qact1", xn.view(b, gh, gw, c), bl["s_ln1"])
            v16 = None
            if self.v16 and bl["window"] == 0 and gh == 64 and gw == 64:
                # global block: the qkv GEMM also writes the V codes as fp16 for the attention's staging
                if v16buf is None:
                    v16buf = torch.empty((b, gh, gw, c), dtype=torch.float16, device=x.device)
                v16 = v16buf
                qkv = ops.w8a8_gemm_v16(xn, bl["qkv"]["packed"], bl["qkv"]["scale"], bl["qkv"]["n"], bl["qkv"]["bias"],
                                        bl["s_ln1"], bl["s_qkv"], v16, 2 * c, cfg=bl["qkv"]["cfg"]).view(b, gh, gw, 3 * c)
            else:
                qkv = self._gemm(xn, bl["qkv"], ops.EPI_Q8, bl["s_ln1"], bl["s_qkv"]).view(b, gh, gw, 3 * c)
            tap(pre + "attn.qact1", qkv, bl["s_qkv"])
            ops.rel_attention_q8(qkv, bl["qkv_bias"], bl["relh"], bl["relw"], bl["heads"], bl["window"],
                                 bl["scale"], bl["s_qkv"], bl["s_a1"], bl["s_a2"], bl["s_ao"],
                                 out=ao.view(b, gh, gw, c), v16=v16)
            tap(pre + "attn.qact2", ao.view(b, gh, gw, c), bl["s_ao"])
            self._gemm(ao, bl["proj"], ops.EPI_Q8_RES, bl["s_ao"], bl["s_x1"], mid=bl["s_proj"], res=x, res_scale=s_x,
                       out=x)
            tap(pre + "qact2", x.view(b, gh, gw, c), bl["s_x1"])
            g2, b2, e2 = bl["n2"]
            ops.layernorm_q(x, g2, b2, e2, in_scale=bl["s_x1"], out_scale=bl["s_ln2"], out=xn, rows_per_wave=self.ln_rpw)
            tap(pre + "qact3", xn.view(b, gh, gw, c), bl["s_ln2"])
            hbuf = self._gemm(xn, bl["lin1"], ops.EPI_Q8_GELU, bl["s_ln2"], bl["s_h"])
            tap(pre + "mlp.qact1", hbuf.view(b, gh, gw, -1), bl["s_h"])
            self._gemm(hbuf, bl["lin2"], ops.EPI_Q8_RES, bl["s_h"], bl["s_x2"], mid=bl["s_l2"], res=x,
                       res_scale=bl["s_x1"], out=x)
            s_x = bl["s_x2"]
            tap(pre + "qact4", x.view(b, gh, gw, c), s_x)
        return self._neck(x, s_x, b, gh, gw)

    def _row_split(self, gh: int) -> int:
        """First grid row of the second row lane (0: one chain): the window boundary nearest the
        middle, so every window lies in one lane."""
        if self.row_lanes <= 1:
            return 0
        wins = {bl["window"] for bl in self.blocks if bl["window"] > 0}
        step = max(wins) if wins else 1
        if len(wins) > 1 or gh < 2 * step:
            return 0
        return max(step, round(gh / 2 / step) * step)

    def _blocks_row_lanes(self, x, xn, ao, b, gh, gw, c, split):
        """The blocks as two kernel chains on their own HIP streams, lane 0 on grid rows [0, split),
        lane 1 on [split, gh).  Global blocks: both lanes' qkv rows are complete before either lane's
        attention reads every key, and neither lane's next qkv GEMM overwrites its rows before the
        other lane's global attention has read them -- two joins of the lanes through the forking
        stream.  (Pairwise cross-stream events in place of the joins crashed the HIP graph capture,
        tools/w8a8_lane_capture_probe.py.)  Returns the final activation scale."""
        ops = self.ops
        if b != 1:
            raise NotImplementedError("W8A8 row lanes: batch 1 (config 2); larger batches run one chain")
        ranges = ((0, split), (split, gh))
        cur = torch.cuda.current_stream()
        streams = self._lane_streams()

        def join():   # the lanes wait for each other, through the forking stream
            for st in streams:
                cur.wait_stream(st)
            for st in streams:
                st.wait_stream(cur)
        for st in streams:
            st.wait_stream(cur)
        # every buffer the lanes share is allocated on the forking stream (stream-ordered reuse stays
        # behind the final join)
        qkv_all = torch.empty((b * gh * gw, 3 * c), dtype=torch.int8, device=x.device)
        hid = torch.empty((b * gh * gw, self.blocks[0]["lin1"]["n"]), dtype=torch.int8, device=x.device)
        qkv = qkv_all.view(b, gh, gw, 3 * c)
        after_global = False
        s_x = self.s_x0
        for bl in self.blocks:
            glob = bl["window"] == 0
            if after_global:
                join()   # the previous global attention has read both lanes' qkv rows
            for li, (r0, r1) in enumerate(ranges):
                t0, t1 = r0 * gw, r1 * gw
                with torch.cuda.stream(streams[li]):
                    g1, b1, e1 = bl["n1"]
                    ops.layernorm_q(x[t0:t1], g1, b1, e1, in_scale=s_x, out_scale=bl["s_ln1"], out=xn[t0:t1],
                                    rows_per_wave=self.ln_rpw)
                    self._gemm(xn[t0:t1], bl["qkv"], ops.EPI_Q8, bl["s_ln1"], bl["s_qkv"], out=qkv_all[t0:t1])
            if glob:
                join()   # every key row is projected before any query reads it
            for li, (r0, r1) in enumerate(ranges):
                t0, t1 = r0 * gw, r1 * gw
                with torch.cuda.stream(streams[li]):
                    ops.rel_attention_q8(qkv, bl["qkv_bias"], bl["relh"], bl["relw"], bl["heads"], bl["window"],
                                         bl["scale"], bl["s_qkv"], bl["s_a1"], bl["s_a2"], bl["s_ao"],
                                         out=ao.view(b, gh, gw, c), rows=(r0, r1 - r0))
                    self._gemm(ao[t0:t1], bl["proj"], ops.EPI_Q8_RES, bl["s_ao"], bl["s_x1"], mid=bl["s_proj"],
                               res=x[t0:t1], res_scale=s_x, out=x[t0:t1])
                    g2, b2, e2 = bl["n2"]
                    ops.layernorm_q(x[t0:t1], g2, b2, e2, in_scale=bl["s_x1"], out_scale=bl["s_ln2"], out=xn[t0:t1],
                                    rows_per_wave=self.ln_rpw)
                    self._gemm(xn[t0:t1], bl["lin1"], ops.EPI_Q8_GELU, bl["s_ln2"], bl["s_h"], out=hid[t0:t1])
                    self._gemm(hid[t0:t1], bl["lin2"], ops.EPI_Q8_RES, bl["s_h"], bl["s_x2"], mid=bl["s_l2"],
                               res=x[t0:t1], res_scale=bl["s_x1"], out=x[t0:t1])
            after_global = glob
            s_x = bl["s_x2"]
        for st in streams:
            cur.wait_stream(st)
        return s_x

    def _lane_streams(self):
        ss = self.__dict__.get("_streams")
        if ss is None:
            ss = self._streams = [torch.cuda.Stream(device=self.dev) for _ in range(2)]
        return ss

    def _neck(self, x, s_x, b, gh, gw):
        ops = self.ops
        sq = self.s_q
        y0 = self._gemm(x, self.neck0, ops.EPI_Q8, s_x, sq[0])
        y1 = ops.layernorm_q(y0, self.ln_n1[0], self.ln_n1[1], self.ln_n1[2], in_scale=sq[0], out_scale=sq[1])
        oc = y1.shape[-1]
        n2 = self.neck2
        y2 = ops.w8a8_conv_gemm(y1.view(b, gh, gw, oc).contiguous(), 2, n2["packed"], n2["scale"], n2["n"], n2["bias"],
                                ops.EPI_Q8, sq[1], sq[2]).view(b * gh * gw, -1)
        y3 = ops.layernorm_q(y2, self.ln_n3[0], self.ln_n3[1], self.ln_n3[2], in_scale=sq[2], out_scale=sq[3],
                             out_dtype=torch.float32)
        return y3.view(b, gh, gw, oc).permute(0, 3, 1, 2)

    __call__ = forward

    def capture(self, img_static: torch.Tensor):
        """Record one forward into a HIP graph; returns ``(graph, out)`` (see EncoderEngine.capture)."""
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self.forward(img_static)
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = self.forward(img_static)
        return graph, out

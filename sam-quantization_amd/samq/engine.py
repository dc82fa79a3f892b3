"""Fused HIP forward of a quantized SAM ViT image encoder (the hot path).

Replaces, for a whole ``ImageEncoderViT`` (reference ``image_encoder.py:106-118``) after
``load_quant``, the reference's per-module dataflow (~20 launches and several
partition/permute/pad copies per block, fp16 residual) by 7 launches per block:

    xn  = LN1(x)                      samq_layernorm      f32 -> f16
    qkv = xn . Wqkv + b               samq_w4a16_gemm     EPI_BIAS         (natural token order)
    a   = attn(qkv)                   samq_rel_attention  windowed/global, rel-pos in-kernel,
                                                          window pad/crop folded into addressing
    x  += a . Wproj + b               samq_w4a16_gemm     EPI_RESADD_F32   (fp32 residual in place)
    xn  = LN2(x)                      samq_layernorm
    h   = GELU(xn . W1 + b1)          samq_w4a16_gemm     EPI_BIAS_GELU
    x  += h . W2 + b2                 samq_w4a16_gemm     EPI_RESADD_F32

The residual stream ``x`` stays fp32 in HBM (precision: SURVEY.md §7 "Hard parts").
Patch embedding (+bias +pos_embed) and the neck convolutions are implicit-GEMM HIP kernels
(``csrc/conv_gemm.hip``: patches gathered from the NCHW image, 3x3 taps from the NHWC map, no
im2col copies) plus the HIP LayerNorm; the only torch op left is the final NHWC -> NCHW view
change of the output.  W4A8 keeps its patch embedding in fp32 (``samq_patch_embed_f32``, the
fp32-MFMA twin of the implicit GEMM): its first int8 quantiser sits right behind it.
All activation buffers are allocated once per batch size and reused; ``capture()`` records the
whole forward into a HIP graph for launch-overhead-free replay.
"""
from __future__ import annotations

from collections import OrderedDict

import torch
import torch.nn.functional as F

from . import ops
from .quant_linear import QuantLinear


class _BlockPlan:
    __slots__ = ("ln1_w", "ln1_b", "ln1_eps", "qkv", "proj", "relh", "relw", "heads", "window", "scale",
                 "ln2_w", "ln2_b", "ln2_eps", "lin1", "lin2", "qkv_bias", "s_qkv", "s_proj", "s_lin1", "s_lin2",
                 "qkv_gw", "qkv_bw", "lin1_gw", "lin1_bw")


class EncoderEngine:
    def __init__(self, enc):
        from .fused_attention import QuantAttention
        self.enc = enc
        self.device = enc.pos_embed.device if enc.pos_embed is not None else next(enc.parameters()).device
        self.C = enc.embed_dim
        self.grid = enc.img_size // enc.patch_size
        self.ln_rpw = 0   # LayerNorm rows per wave (0 = library default; in-graph A/B knob)
        # fold norm2 / the next block's norm1 into the GEMMs around them (W4A16, >= 8192 rows per
        # chain: the ping-pong GEMMs carry the fold epilogues).  Off by default: measured in the
        # 2-lane bench graph the fold epilogues cost more than the two LayerNorm launches they
        # replace (isolated per block 358 vs 351 us, step 23.4 vs 23.0 ms)
        self.fold_ln = False
        # lanes > 1: lane i+1 starts after lane i's launch number ``lane_stagger`` (7 per block,
        # block 0 first; -1 = all lanes start together) -- an in-graph A/B knob
        self.lane_stagger = 1   # measured: +0.3 % over no stagger (profiles/r3_v9_lane_stagger.log)
        # where the residual adds of proj / lin2 run: "epi" = the GEMM's read-modify-write epilogue
        # (x += y in f32); "ln32" = the GEMM stores y (f32) and the next LayerNorm adds it
        # (samq_add_layernorm, bit-identical x); "ln16" = the same with y stored as f16
        self.res_mode = "epi"
        # W4A8 (per-channel weights, res_mode "epi"): the zero-point row sums S[m] of each int8 GEMM
        # input come from its producer -- LN-q for qkv / lin1, lin1's Q8_GELU epilogue (int32 atomics)
        # for lin2 -- instead of every column tile of the ping-pong GEMM re-summing its A rows;
        # bit-identical either way (an in-graph A/B knob)
        self.rowsums = True   # True, False, or "ln" (LN-q's sums only: lin2 sums its own rows)
        # lanes > 1: lane 0's HIP stream at high priority (its workgroups dispatched first, the
        # other lanes fill the CUs it leaves) -- an in-graph A/B knob, default off
        self.lane_priority = 0
        # timing-only A/B knob (tools): launches to leave out of the W4A16 block ("ln", "win",
        # "glob") -- the output is wrong; the empty default runs everything
        self.skip = frozenset()
        self.plans = []
        for blk in enc.blocks:
            attn = blk.attn
            p = _BlockPlan()
            if isinstance(attn, QuantAttention):
                qkv, proj = attn.qkv_proj, attn.o_proj
            else:
                qkv, proj = attn.qkv, attn.proj
            for lin in (qkv, proj, blk.mlp.lin1, blk.mlp.lin2):
                if not isinstance(lin, QuantLinear):
                    raise TypeError("EncoderEngine needs every encoder Linear quantized (load_quant / make_quant)")
                lin.prepare()
            if not attn.use_rel_pos:
                raise NotImplementedError
            p.qkv, p.proj, p.lin1, p.lin2 = qkv, proj, blk.mlp.lin1, blk.mlp.lin2
            p.qkv_bias = qkv.bias
            p.heads = attn.num_heads
            p.scale = float(attn.scale)
            p.window = blk.window_size
            side = blk.window_size if blk.window_size > 0 else self.grid
            p.relh, p.relw = self._tables(attn, side)
            p.ln1_w, p.ln1_b, p.ln1_eps = self._ln(blk.norm1)
            p.ln2_w, p.ln2_b, p.ln2_eps = self._ln(blk.norm2)
            p.s_qkv, p.s_proj, p.s_lin1, p.s_lin2 = (lin.act_scale() for lin in (qkv, proj, blk.mlp.lin1, blk.mlp.lin2))
            self.plans.append(p)
        # W4A8 when every block Linear has a calibrated int8 input quantiser in quant mode
        flags = [s is not None for p in self.plans for s in (p.s_qkv, p.s_proj, p.s_lin1, p.s_lin2)]
        if any(flags) and not all(flags):
            raise NotImplementedError("W4A8 engine: either all or none of the block Linears quantise their input")
        self.w4a8 = bool(flags) and all(flags)
        if self.w4a8:
            for p in self.plans:
                for lin in (p.qkv, p.proj, p.lin1, p.lin2):
                    lin.prepare_w4a8()
            # LN-q at four rows per wave in the 2-lane W4A8 graph: 34.58 vs 34.80 ms and 34.83 vs 34.99
            # (two boxes, interleaved, bit-identical, profiles/r6_ln_rpw_w4a8_ab.log); W4A16 keeps 2
            self.ln_rpw = 4
        self._fold_ready = False
        pe = enc.patch_embed.proj
        self.patch = pe.kernel_size[0]
        self.pe_w = pe.weight.detach().reshape(pe.weight.shape[0], -1).to(torch.float16).contiguous()
        # W4A8 embeds in fp32: the f32 weight copy is made here, on the construction stream,
        # before any lane fork (a lazy copy on lane 0's stream would race lane 1's first read)
        self.pe_w32 = self.pe_w.float().contiguous() if self.w4a8 else None
        self.pe_b = pe.bias.detach().float().contiguous() if pe.bias is not None else None
        self.pos = enc.pos_embed.detach().float().contiguous() if enc.pos_embed is not None else None
        n0, n1, n2, n3 = enc.neck
        self.n0_w = n0.weight.detach().reshape(n0.weight.shape[0], -1).to(torch.float16).contiguous()
        self.n1 = (n1.weight.detach().float().contiguous(), n1.bias.detach().float().contiguous(), float(n1.eps))
        self.n2_w = n2.weight.detach().reshape(n2.weight.shape[0], -1).to(torch.float16).contiguous()
        # 3x3 taps major, channels minor: a 16-byte A chunk of the implicit GEMM is 8 channels of one tap
        self.n2_w_tap = n2.weight.detach().permute(0, 2, 3, 1).to(torch.float16).contiguous()
        self.n3 = (n3.weight.detach().float().contiguous(), n3.bias.detach().float().contiguous(), float(n3.eps))
        self.out_chans = n0.weight.shape[0]
        self._pixel_norm = None
        self._bufs = OrderedDict()   # (images, lane) -> activation buffers, most recent last
        self.max_cached_batches = 2  # distinct per-lane batch sizes kept (captured graphs pin their own)
        self._key = self._make_key(enc)

    # ---------------------------------------------------------------- helpers
    @staticmethod
    def _make_key(enc):
        return tuple((id(m), getattr(m, "qweight", None) is not None and m.qweight._version, m.act_scale())
                     for m in enc.modules() if isinstance(m, QuantLinear))

    def valid_for(self, enc) -> bool:
        return enc is self.enc and self._make_key(enc) == self._key

    @staticmethod
    def _ln(norm):
        return (norm.weight.detach().float().contiguous(), norm.bias.detach().float().contiguous(), float(norm.eps))

    @staticmethod
    def _tables(attn, side):
        def fit(tab):
            span = 2 * side - 1
            t = tab.detach().float()
            if t.shape[0] != span:
                t = F.interpolate(t.t().unsqueeze(0), size=span, mode="linear").squeeze(0).t()
            return t.to(torch.float16).contiguous()
        return fit(attn.rel_pos_h), fit(attn.rel_pos_w)

    def buffers(self, b: int, lane: int = 0):
        """Activation buffers for a batch of ``b`` images; each concurrent lane (``forward``'s
        ``lanes``) owns its own set."""
        bufs = self._bufs.get((b, lane))
        if bufs is not None:
            self._bufs.move_to_end((b, lane))
        else:
            sizes = list(OrderedDict.fromkeys(k[0] for k in self._bufs))
            while len(sizes) >= self.max_cached_batches and sizes[0] != b:
                old = sizes.pop(0)   # evict the least recently used batch size (all its lanes)
                for k in [k for k in self._bufs if k[0] == old]:
                    del self._bufs[k]
            g, c, dev = self.grid, self.C, self.device
            hid = self.plans[0].lin1.outfeatures
            assert all(p.lin1.outfeatures == hid for p in self.plans)
            bufs = dict(
                x=torch.empty((b, g, g, c), dtype=torch.float32, device=dev),
                xn=torch.empty((b, g, g, c), dtype=torch.float16, device=dev),
                qkv=torch.empty((b, g, g, 3 * c), dtype=torch.float16, device=dev),
                att=torch.empty((b, g, g, c), dtype=torch.float16, device=dev),
                hid=torch.empty((b, g, g, hid), dtype=torch.float16, device=dev),
            )
            if not self.w4a8:   # LayerNorm fold: per-row partial sums (64-column blocks) and means
                bufs.update(stats=torch.empty((b * g * g, c // 64, 2), dtype=torch.float32, device=dev),
                            mu=torch.empty((b * g * g,), dtype=torch.float32, device=dev))
            if self.w4a8:
                bufs.update(xn8=torch.empty((b, g, g, c), dtype=torch.int8, device=dev),
                            att8=torch.empty((b, g, g, c), dtype=torch.int8, device=dev),
                            hid8=torch.empty((b, g, g, hid), dtype=torch.int8, device=dev),
                            rs_x=torch.empty((b * g * g,), dtype=torch.int32, device=dev),
                            rs_h=torch.empty((b * g * g,), dtype=torch.int32, device=dev))
                del bufs["xn"], bufs["hid"], bufs["att"]
            self._bufs[(b, lane)] = bufs
        return bufs

    def release(self) -> None:
        """Drop every cached activation buffer (graphs from ``capture`` keep their own alive)."""
        self._bufs.clear()

    # ---------------------------------------------------------------- stages
    def embed(self, img: torch.Tensor, x32: torch.Tensor) -> None:
        """Patch embedding + bias + pos_embed into the fp32 residual stream: one implicit-GEMM HIP
        kernel (patches read straight from the NCHW image).  W4A8 computes it in fp32
        (``samq_patch_embed_f32``): its first int8 quantiser sits right behind it.  A uint8 image
        (raw pixels, ``pixel_norm`` set by ``forward``) is normalised and zero-padded inside the
        same kernel (``Sam.preprocess`` fused, ``samq_patch_embed_u8``)."""
        p = self.patch
        pos = None if self.pos is None else self.pos[0]
        if "embed" in self.skip:   # timing-only (in-graph A/B): no patch embedding
            return
        if img.dtype == torch.uint8:
            if self._pixel_norm is None:
                raise ValueError("uint8 pixels need pixel_norm=(pixel_mean, pixel_std)")
            ops.patch_embed_u8(img.contiguous(), *self._pixel_norm, self.pe_w32 if self.w4a8 else self.pe_w, self.pe_b,
                               pos, p, self.enc.img_size, out=x32)
            return
        if not self.w4a8:
            ops.patch_embed(img.to(torch.float16).contiguous(), self.pe_w, self.pe_b, pos, p, out=x32)
            return
        ops.patch_embed(img.to(torch.float32).contiguous(), self.pe_w32, self.pe_b, pos, p, out=x32)

    def block_w4a8(self, p: _BlockPlan, bufs, mark=None, first: bool = True, last: bool = True) -> None:
        """W4A8 block: int8 codes into every GEMM (fq_vit QAct on each QuantLinear input, folded
        into LN / the GELU epilogue / the attention's store), int8 MFMA GEMMs.  ``mark(k)``,
        ``first`` / ``last`` and ``res_mode`` as in ``block`` ("ln16" stores f32 deltas here too:
        the int8 GEMMs have no f16 residual output)."""
        mark = mark or (lambda k: None)
        x, xn8, qkv, att8, hid8 = bufs["x"], bufs["xn8"], bufs["qkv"], bufs["att8"], bufs["hid8"]
        late = self.res_mode != "epi"
        rs = self.rowsums and not late and all(lin.groupsize in (-1, lin.infeatures)
                                               for lin in (p.qkv, p.lin1, p.lin2))
        rs_x = bufs["rs_x"] if rs else None
        rs_h = bufs["rs_h"] if rs and self.rowsums != "ln" else None
        if late and not first:
            ops.add_layernorm(x, self._delta(bufs, torch.float32), p.ln1_w, p.ln1_b, p.ln1_eps, out=xn8,
                              out_scale=p.s_qkv)
        else:
            ops.layernorm_q(x, p.ln1_w, p.ln1_b, p.ln1_eps, out_scale=p.s_qkv, out=xn8, rows_per_wave=self.ln_rpw,
                            rowsum=rs_x)
        mark(0)
        p.qkv.forward_w4a8(xn8, p.s_qkv, ops.EPI_BIAS, out=qkv, rowsum=rs_x)
        mark(1)
        if ("win" if p.window else "glob") not in self.skip:
            ops.rel_attention(qkv, p.qkv_bias, p.relh, p.relw, p.heads, p.window, p.scale, out=att8,
                              out_scale=p.s_proj)
        mark(2)
        if late:
            p.proj.forward_w4a8(att8, p.s_proj, ops.EPI_F32, out=self._delta(bufs, torch.float32))
            mark(3)
            ops.add_layernorm(x, self._delta(bufs, torch.float32), p.ln2_w, p.ln2_b, p.ln2_eps, out=xn8,
                              out_scale=p.s_lin1)
        else:
            p.proj.forward_w4a8(att8, p.s_proj, ops.EPI_RESADD_F32, out=x)
            mark(3)
            ops.layernorm_q(x, p.ln2_w, p.ln2_b, p.ln2_eps, out_scale=p.s_lin1, out=xn8, rows_per_wave=self.ln_rpw,
                            rowsum=rs_x, zero_rows=rs_h)
        mark(4)
        p.lin1.forward_w4a8(xn8, p.s_lin1, ops.EPI_Q8_GELU, out=hid8, out_scale=p.s_lin2, rowsum=rs_x, rowsum_out=rs_h)
        mark(5)
        if late and not last:
            p.lin2.forward_w4a8(hid8, p.s_lin2, ops.EPI_F32, out=self._delta(bufs, torch.float32))
        else:
            p.lin2.forward_w4a8(hid8, p.s_lin2, ops.EPI_RESADD_F32, out=x, rowsum=rs_h)
        mark(6)

    # ---------------------------------------------------------------- LayerNorm fold
    def _fold_usable(self, rows: int) -> bool:
        """The fold epilogues live in the ping-pong GEMMs (configs 57 / 64), which the library picks
        from 8192 rows up; every block Linear must use that pick (gemm_cfg 0, 57 or 64)."""
        if self.w4a8 or not self.fold_ln or rows < 8192 or self.C % 256:
            return False
        return all(lin.gemm_cfg in (0, 57, 64) and lin.outfeatures % 256 == 0
                   for p in self.plans for lin in (p.qkv, p.proj, p.lin1, p.lin2))

    def _prepare_fold(self) -> None:
        """gamma . W and beta . W of every folded LayerNorm's consumer (norm1 -> qkv for blocks >= 1,
        norm2 -> lin1), from the layers' own GEMMs -- once per engine."""
        if self._fold_ready:
            return
        for p in self.plans:
            p.qkv_gw, p.qkv_bw = p.qkv.ln_fold_constants(p.ln1_w, p.ln1_b)
            p.lin1_gw, p.lin1_bw = p.lin1.ln_fold_constants(p.ln2_w, p.ln2_b)
        self._fold_ready = True

    def block_fold(self, i: int, bufs, mark=None) -> None:
        """W4A16 block with the LayerNorms folded into the GEMMs (samq_w4a16_gemm_lnf, include/samq.h):
        proj's residual epilogue emits f16((x - mu) * gamma2) + per-row partial sums, lin1's
        epilogue applies LN2 algebraically (rstd * (acc - delta * gamma2.W1) + beta2.W1 + b1, GELU);
        lin2's residual epilogue does the same for the next block's norm1 and its qkv consumes it.
        Block 0's norm1 stays a LayerNorm kernel (it also writes the row means mu).  ``mark(k)``
        runs at the place of ``block``'s launch k (a folded LayerNorm's mark right after the
        launch that absorbed it), so the lane stagger gates at the same point as unfolded."""
        mark = mark or (lambda k: None)
        p = self.plans[i]
        x, xn, qkv, att, hid = bufs["x"], bufs["xn"], bufs["qkv"], bufs["att"], bufs["hid"]
        st, mu = bufs["stats"], bufs["mu"]
        if i == 0:
            ops.layernorm(x, p.ln1_w, p.ln1_b, p.ln1_eps, out=xn, rows_per_wave=self.ln_rpw, mean_out=mu)
            mark(0)
            p.qkv.forward_epilogue(xn, ops.EPI_BIAS, out=qkv)
        else:
            mark(0)   # norm1 was folded into the previous block's lin2
            p.qkv.forward_lnf(xn, ops.EPI_BIAS_LNF, qkv, st, mu, gw=p.qkv_gw, bw=p.qkv_bw, eps=p.ln1_eps)
        mark(1)
        ops.rel_attention(qkv, p.qkv_bias, p.relh, p.relw, p.heads, p.window, p.scale, out=att)
        mark(2)
        p.proj.forward_lnf(att, ops.EPI_RESADD_LNF, x, st, mu, gamma=p.ln2_w, aout=xn)
        mark(3)
        mark(4)   # norm2 folded into proj (producer) / lin1 (consumer)
        p.lin1.forward_lnf(xn, ops.EPI_GELU_LNF, hid, st, mu, gw=p.lin1_gw, bw=p.lin1_bw, eps=p.ln2_eps)
        mark(5)
        if i + 1 < len(self.plans):
            p.lin2.forward_lnf(hid, ops.EPI_RESADD_LNF, x, st, mu, gamma=self.plans[i + 1].ln1_w, aout=xn)
        else:
            p.lin2.forward_epilogue(hid, ops.EPI_RESADD_F32, out=x)
        mark(6)

    def _delta(self, bufs, dtype=None) -> torch.Tensor:
        """The proj / lin2 output the next LayerNorm adds to x (res_mode "ln32": f32, "ln16": f16),
        allocated with the lane's buffers on first use."""
        dtype = dtype or (torch.float16 if self.res_mode == "ln16" else torch.float32)
        key = "delta16" if dtype == torch.float16 else "delta32"
        t = bufs.get(key)
        if t is None:
            t = bufs[key] = torch.empty(bufs["x"].shape, dtype=dtype, device=bufs["x"].device)
        return t

    def _res_add_ln(self, x, bufs, w, b, eps, out, pending: bool) -> None:
        """The LayerNorm in front of a block half; with ``pending`` (res_mode != "epi") the
        preceding GEMM's output (``_delta``) is first added to x (samq_add_layernorm)."""
        if pending:
            ops.add_layernorm(x, self._delta(bufs), w, b, eps, out=out, rows_per_wave=self.ln_rpw)
        else:
            ops.layernorm(x, w, b, eps, out=out, rows_per_wave=self.ln_rpw)

    def block(self, p: _BlockPlan, bufs, mark=None, first: bool = True, last: bool = True) -> None:
        """One W4A16 block (7 launches).  ``mark(k)`` (lane stagger) runs after launch k.  With
        ``res_mode`` "ln32" / "ln16" the residual adds run in the LayerNorms: proj and lin2 store
        y into ``delta`` and the next LayerNorm adds it (``first``: x is complete on entry; ``last``:
        lin2 adds in its own epilogue so x is complete for the neck)."""
        if self.w4a8:
            return self.block_w4a8(p, bufs, mark, first, last)
        mark = mark or (lambda k: None)
        x, xn, qkv, att, hid = bufs["x"], bufs["xn"], bufs["qkv"], bufs["att"], bufs["hid"]
        late = self.res_mode != "epi"
        res_epi = ops.EPI_BIAS if self.res_mode == "ln16" else ops.EPI_F32
        if "ln" not in self.skip:
            self._res_add_ln(x, bufs, p.ln1_w, p.ln1_b, p.ln1_eps, xn, late and not first)
        mark(0)
        p.qkv.forward_epilogue(xn, ops.EPI_BIAS, out=qkv)
        mark(1)
        if ("win" if p.window else "glob") not in self.skip:
            ops.rel_attention(qkv, p.qkv_bias, p.relh, p.relw, p.heads, p.window, p.scale, out=att)
        mark(2)
        if late:
            p.proj.forward_epilogue(att, res_epi, out=self._delta(bufs))
        else:
            p.proj.forward_epilogue(att, ops.EPI_RESADD_F32, out=x)
        mark(3)
        if "ln" not in self.skip:
            self._res_add_ln(x, bufs, p.ln2_w, p.ln2_b, p.ln2_eps, xn, late)
        mark(4)
        p.lin1.forward_epilogue(xn, ops.EPI_BIAS_GELU, out=hid)
        mark(5)
        if late and not last:
            p.lin2.forward_epilogue(hid, res_epi, out=self._delta(bufs))
        else:
            p.lin2.forward_epilogue(hid, ops.EPI_RESADD_F32, out=x)
        mark(6)

    def neck(self, x32: torch.Tensor, out_dtype) -> torch.Tensor:
        """Neck (image_encoder.py:88-104) on NHWC tokens: 1x1 conv (HIP, fp32 tokens -> fp16),
        LayerNorm2d (HIP), 3x3 conv (HIP implicit GEMM, zero padding in the gather), LayerNorm2d."""
        b, g = x32.shape[0], self.grid
        if "neck" in self.skip:   # timing-only (in-graph A/B): no neck
            return torch.empty((b, self.n0_w.shape[0], g, g), dtype=out_dtype or torch.float16, device=x32.device)
        y = ops.conv1x1_f32(x32, self.n0_w)                                                # (b, g, g, oc) f16
        y = ops.layernorm(y, *self.n1[:2], eps=self.n1[2])                                 # LN2d (NHWC rows)
        y = ops.conv3x3_nhwc(y, self.n2_w_tap)                                             # 3x3, pad 1
        y = ops.layernorm(y, *self.n3[:2], eps=self.n3[2], out_dtype=torch.float32)
        return y.permute(0, 3, 1, 2).to(out_dtype)

    # ---------------------------------------------------------------- forward
    @torch.no_grad()
    def forward(self, img: torch.Tensor, out_dtype=None, lanes: int = 1, pixel_norm=None) -> torch.Tensor:
        """Whole encoder forward.  ``lanes > 1`` splits the batch into that many image groups,
        each run as its own kernel chain on its own HIP stream (images are independent: per-token
        LN, per-image attention).  Kernels of one lane fill the CUs another lane leaves idle —
        the last partial round of GEMM tiles (N=1280: 1.25 rounds of 256 CUs at B=4), and the
        HBM-bound LayerNorm under the MFMA-bound GEMMs.  Every kernel is batch-invariant, so the
        result is bit-identical to ``lanes=1`` (tests/test_gpu_encoder.py).

        Returns ``(B, out_chans, H, W)`` in channels-last memory (an NCHW view of the engine's
        NHWC tokens) for every ``lanes``; ``lanes`` must divide the batch (``ValueError``).
        ``img`` may be raw uint8 pixels (B, 3, h, w) with ``pixel_norm=(pixel_mean, pixel_std)``:
        the normalise + zero-pad of ``Sam.preprocess`` then runs inside the patch embedding."""
        assert img.is_cuda, "EncoderEngine runs on the GPU only"
        if img.dtype == torch.uint8:
            # raw (B, 3, h, w) pixels, h, w <= img_size: Sam.preprocess runs inside the patch embedding
            self._pixel_norm = tuple(t.reshape(-1).float().contiguous() for t in pixel_norm) if pixel_norm else None
            out_dtype = out_dtype or torch.float32
        out_dtype = out_dtype or img.dtype
        b = img.shape[0]
        per_chain = b // min(max(lanes, 1), b) if lanes > 1 and b >= 2 else b
        if self._fold_usable(per_chain * self.grid * self.grid):
            self._prepare_fold()   # on the current stream, before any lane fork
        if lanes <= 1 or b < 2:
            return self._forward(img, self.buffers(b), out_dtype)
        lanes = min(lanes, b)
        if b % lanes:
            raise ValueError(f"batch {b} does not split into {lanes} lanes")
        bl = b // lanes
        cur = torch.cuda.current_stream()
        streams = self._lane_streams(lanes)
        for s in streams:
            s.wait_stream(cur)
        outs = []
        gate = None   # lane stagger: lane i starts once lane i-1 has issued its first launches
        for i, s in enumerate(streams):
            with torch.cuda.stream(s):
                if gate is not None:
                    s.wait_event(gate)
                ev = torch.cuda.Event() if self.lane_stagger >= 0 and i + 1 < lanes else None
                outs.append(self._forward(img[i * bl:(i + 1) * bl], self.buffers(bl, i), out_dtype, ev))
                gate = ev
        n, c, h, w = outs[0].shape
        out = torch.empty((b, h, w, c), dtype=out_dtype, device=img.device).permute(0, 3, 1, 2)
        for i, s in enumerate(streams):  # nothing was enqueued on ``cur`` since the fork
            with torch.cuda.stream(s):
                out[i * bl:(i + 1) * bl].copy_(outs[i])
            cur.wait_stream(s)
        return out

    def _lane_streams(self, lanes: int):
        cache = self.__dict__.setdefault("_streams", {})
        ss = cache.get((lanes, self.lane_priority))
        if ss is None:
            hi = torch.cuda.Stream.priority_range()[1]   # the numerically lowest = highest priority
            ss = cache[(lanes, self.lane_priority)] = [
                torch.cuda.Stream(device=self.device, priority=hi if (self.lane_priority and i == 0) else 0)
                for i in range(lanes)]
        return ss

    def _forward(self, img: torch.Tensor, bufs, out_dtype, gate_event=None) -> torch.Tensor:
        self.embed(img, bufs["x"])
        fold = self._fold_ready and self._fold_usable(bufs["x"].numel() // self.C)
        for i, p in enumerate(self.plans):
            mark = None
            if gate_event is not None and i == self.lane_stagger // 7:
                k0 = self.lane_stagger % 7
                mark = lambda k, k0=k0: gate_event.record() if k == k0 else None  # noqa: E731
            if fold:
                self.block_fold(i, bufs, mark)
            else:
                self.block(p, bufs, mark, first=i == 0, last=i + 1 == len(self.plans))
        if gate_event is not None and self.lane_stagger // 7 >= len(self.plans):
            gate_event.record()
        return self.neck(bufs["x"], out_dtype)

    __call__ = forward

    @torch.no_grad()
    def tokens(self, img: torch.Tensor, upto: int | None = None) -> torch.Tensor:
        """fp32 residual stream after ``upto`` blocks (debug / parity helper)."""
        bufs = self.buffers(img.shape[0])
        self.embed(img, bufs["x"])
        n = len(self.plans) if upto is None else upto
        for i, p in enumerate(self.plans[:n]):
            self.block(p, bufs, first=i == 0, last=i + 1 == n)
        return bufs["x"].clone()

    def capture(self, img_static: torch.Tensor, out_dtype=None, lanes: int = 1):
        """Record one forward on ``img_static`` into a HIP graph; returns ``(graph, out)``;
        ``graph.replay()`` recomputes ``out`` from the current contents of ``img_static``."""
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self.forward(img_static, out_dtype, lanes)
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = self.forward(img_static, out_dtype, lanes)
        # the graph replays into these buffers: keep them alive with it, whatever the cache evicts
        b = img_static.shape[0]
        nl = min(lanes, b) if lanes > 1 and b >= 2 else 1
        graph.samq_buffers = [self._bufs[(b // nl, i)] for i in range(nl)]
        return graph, out

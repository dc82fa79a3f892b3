/*
 * libsamq_hip.so -- C ABI of the MI355X (gfx950) quantized SAM image-encoder hot path.
 *
 * Drop-in boundary for the reference's Python/Triton path (zhanglei1172/sam-quantization):
 * every entry point below names the reference interface it replaces (file:line, relative to
 * the reference repository).  Conventions:
 *   - all tensor arguments are DEVICE pointers on the current HIP device, caller-owned and
 *     caller-allocated (no globals: the reference's shared `workspace`,
 *     gptq_triton/quant_linear.py:13, is gone, so calls are reentrant);
 *   - every launch is enqueued on the explicit `stream` (0 = legacy default stream);
 *     nothing synchronises the host, so a caller may capture any sequence into a hipGraph;
 *   - return 0 on success, a negative SAMQ_ERR_* on failure; samq_last_error() returns a
 *     thread-local message.  The Python layer maps SAMQ_ERR_INVALID -> AssertionError
 *     (the reference's shape asserts, quant_linear.py:378-399), SAMQ_ERR_UNSUPPORTED ->
 *     NotImplementedError (quant_linear.py:72-73, fused_attention.py:134-135) and
 *     SAMQ_ERR_HIP -> RuntimeError;
 *   - an empty batch (zero rows / tokens / images: M, rows, n or B == 0) returns 0 before any
 *     pointer is checked or dereferenced (an empty tensor's data pointer may be null).
 * Data types: "f16" = IEEE binary16, "f32" = binary32; int4 weights use the reference's
 * GPTQ packing (qweight int32 (K/8,N), qzeros int32 (G,N/8), scales f16 (G,N),
 * gptq4sam.py:434-497) -- repacked once per layer by samq_w4_repack.
 */
#ifndef SAMQ_H
#define SAMQ_H

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SAMQ_OK 0
#define SAMQ_ERR_INVALID (-1)
#define SAMQ_ERR_UNSUPPORTED (-2)
#define SAMQ_ERR_HIP (-3)

/* GEMM epilogues (y = acc * scale[n] + bias[n]) */
#define SAMQ_EPI_BIAS 0        /* C f16  = y                        (QuantLinear.forward)     */
#define SAMQ_EPI_BIAS_GELU 1   /* C f16  = GELU_erf(y)              (MLPBlock lin1 + act)     */
#define SAMQ_EPI_RESADD_F32 2  /* C f32 += y (in place)             (Block residual adds)     */
#define SAMQ_EPI_F32 3         /* C f32  = y                                                  */
/* int8-activation GEMMs only (samq_w8a8_gemm / samq_w4a8_gemm); C = int8 codes, q(v, s) =
 * clamp(round_half_even(v / s), -128, 127) (fq_vit quantizer/uniform.py:23-45) */
#define SAMQ_EPI_Q8 4          /* C i8 = q(y, out_scale)                  (Linear -> QAct)        */
#define SAMQ_EPI_Q8_GELU 5     /* C i8 = q(GELU(y), out_scale)            (lin1 -> GELU -> QAct)  */
#define SAMQ_EPI_Q8_RES 6      /* C i8 = q(R*res_scale + q(y,mid)*mid, out_scale)  (residual)   */

/* Thread-local description of the last failure on this thread ("" if none). */
const char* samq_last_error(void);
/* ABI version of this library (major*100 + minor). */
int samq_version(void);

/* ---------------------------------------------------------------- W4A16 (GPTQ int4) */

/* Number of int32 words of the repacked weight of a K x N layer (= K*N/8). */
size_t samq_w4_packed_words(int K, int N);

/* Repack a reference `QuantLinear.qweight` (int32 (K/8, N), gptq_triton/quant_linear.py:81-85)
 * into the kernel's MFMA-fragment order.  K % 64 == 0, N % 32 == 0.  Called once per layer
 * by load_quant (replaces the reference's per-call B-tile addressing, quant_linear.py:292-294). */
int samq_w4_repack(const int32_t* qweight, int32_t* packed, int K, int N, hipStream_t stream);

/* Same with an explicit fragment layout: 1 = the W4A16 layout (32x32x16 MFMA order, what
 * samq_w4_repack produces and every samq_w4a16_gemm_cfg config of this library consumes),
 * 3 = the W4A8 layout (samq_w4a8_gemm / samq_i8_gemm_cfg).  Layout 2 exists only in the
 * tuning build (make tuning); this library rejects it with SAMQ_ERR_INVALID. */
int samq_w4_repack_layout(const int32_t* qweight, int32_t* packed, int K, int N, int layout,
                          hipStream_t stream);

/* C = epilogue(A[M,K] (f16, row stride lda) x W4[K,N]).  Replaces triton_matmul4 +
 * matmul4_kernel (gptq_triton/quant_linear.py:355-437, 231-352) and the separate `c + bias`
 * (:434-435).  wpacked from samq_w4_repack; scales f16 (G,N); qzeros int32 (G,N/8);
 * bias f16 (N) or NULL; groupsize -1 (== K) or a multiple of 64.  C is f16 for
 * SAMQ_EPI_BIAS / SAMQ_EPI_BIAS_GELU and f32 (row stride ldc) for the F32 epilogues.
 * Shapes: K % 64 == 0, N % 32 == 0 (a superset of the reference's K%128/N%256). */
int samq_w4a16_gemm(const void* A, int64_t lda, const int32_t* wpacked, const void* scales,
                    const int32_t* qzeros, const void* bias, void* C, int64_t ldc, int M, int N,
                    int K, int groupsize, int epilogue, hipStream_t stream);

/* Same with an explicit tile configuration (0 = automatic); for tests and in-graph A/B runs.
 * All accept layout-1 weights and compute the same result (up to fp32 summation order):
 *   1 256x256  2 256x128  3 128x128  4 64x64  5 64x32  6 128x256 (1 wave row)  7 256x256
 *   (8 waves in N)  9 128x256                               -- v1, register-staged
 *   21 256x256  22 128x256  23 128x128  24 256x128  25 128x256  26 64x64
 *   29 128x320  30 256x320  31 128x320                      -- v3, LDS-DMA ring
 *   55 56 57 58 62 64 65 (groupsize == K only)             -- v6 ping-pong, 256x256
 * Any other value (the tuning build's timing-only and layout-2 configs) returns
 * SAMQ_ERR_INVALID. */
int samq_w4a16_gemm_cfg(const void* A, int64_t lda, const int32_t* wpacked, const void* scales,
                        const int32_t* qzeros, const void* bias, void* C, int64_t ldc, int M,
                        int N, int K, int groupsize, int epilogue, int cfg, hipStream_t stream);

/* LayerNorm folded into the projection GEMMs around it (the W4A16 encoder block's norm2 between
 * proj and lin1, and the next block's norm1 between lin2 and qkv; image_encoder.py:194-207):
 * the HBM round trip of a standalone LayerNorm (read the f32 residual, write the f16 normalised
 * rows) is replaced by exact algebra,  LN(x).W = rstd*((x - mu_p)*gamma).W - rstd*delta*(gamma.W)
 * + beta.W,  with mu_p the row mean of the PREVIOUS LayerNorm of the same row (so the f16 operand
 * (x - mu_p)*gamma carries no large mean) and delta = mean(x) - mu_p from per-row partial sums:
 *   SAMQ_EPI_RESADD_LNF (producer, C f32 [M,N] residual x += y in place), then
 *     aout f16 [M,N] = f16((x_new - mu[r]) * gamma[n]) and, per 64-column block b,
 *     stats[(r*(N/64) + b)*2 + {0,1}] = sum over the block of (x_new - mu[r]), (x_new - mu[r])^2;
 *   SAMQ_EPI_BIAS_LNF / SAMQ_EPI_GELU_LNF (consumer, A = the producer's aout, K = its N):
 *     delta = S1/K, rstd = 1/sqrt(S2/K - delta^2 + eps) from stats[r, 0..K/64),
 *     C f16 = y = rstd*(acc*scale[n] - delta*gw[n]) + bw[n] + bias[n]  (GELU_erf(y) for GELU_LNF),
 *     gw = gamma.W, bw = beta.W (f32 [N], the next LayerNorm's weights times this layer's dequantised
 *     weight); the tiles of column block 0 set mu[r] += delta (the next producer's mu_p). */
#define SAMQ_EPI_RESADD_LNF 7
#define SAMQ_EPI_BIAS_LNF 8
#define SAMQ_EPI_GELU_LNF 9
#define SAMQ_EPI_SILU_MUL 10   /* internal: the samq_w4a16_gated_mlp epilogue */
/* samq_w4a16_gemm_cfg with the LayerNorm-fold epilogues above (ping-pong configs 57 / 64 / 0 =
 * automatic at M >= 8192 only, else SAMQ_ERR_UNSUPPORTED): gamma f32 [N] (producer), gw / bw f32
 * [N] (consumer), stats f32, mu f32 [M], aout f16 [M,N] (producer), eps of the folded LayerNorm.
 * The consumer stages its 256 rows' partial sums in LDS: K <= 3008 (cfg 57) / 3968 (cfg 64) for
 * per-channel weights, K <= 1728 / 2688 for grouped ones (3-slot rings), else SAMQ_ERR_UNSUPPORTED. */
int samq_w4a16_gemm_lnf(const void* A, int64_t lda, const int32_t* wpacked, const void* scales,
                        const int32_t* qzeros, const void* bias, void* C, int64_t ldc, int M, int N, int K,
                        int groupsize, int epilogue, int cfg, const float* gamma, const float* gw,
                        const float* bw, float* stats, float* mu, void* aout, float eps, hipStream_t stream);

/* ---------------------------------------------------------------- int8 activations */

/* fq_vit int8 weights: W int8 [N][K] row-major (QLinear / flattened QConv2d weight codes,
 * fq_vit/models/ptq/layers.py:160-200, 11-74) -> int8 MFMA fragment order (K*N bytes).
 * K % 128 == 0, N % 32 == 0, 16-byte aligned pointers. */
int samq_w8_repack(const int8_t* w, int8_t* packed, int K, int N, hipStream_t stream);

/* W8A8 GEMM (fq_vit QLinear in quant mode, layers.py:190-200, fed by the int8 codes of the
 * preceding QAct, layers.py:203-242):  y[m,n] = float(sum_k A[m,k] W[n,k]) * a_scale *
 * wscale[n] + bias[n] (int32 exact sum), then the epilogue (SAMQ_EPI_*; Q8_RES reads the int8
 * residual codes R (row stride ldr; may alias C) with res_scale and quantises y with mid_scale
 * first when mid_scale > 0).  A int8 [M,K] (16-byte aligned, lda % 16 == 0); wpacked from
 * samq_w8_repack; wscale/bias f32 [N] (bias may be NULL); K % 128 == 0, N % 64 == 0. */
int samq_w8a8_gemm(const int8_t* A, int64_t lda, const int8_t* wpacked, const float* wscale,
                   const float* bias, void* C, int64_t ldc, const int8_t* R, int64_t ldr, int M,
                   int N, int K, int epilogue, float a_scale, float mid_scale, float res_scale,
                   float out_scale, hipStream_t stream);

/* W4A8 GEMM: GPTQ int4 weights (QuantLinear buffers, gptq_triton/quant_linear.py:81-85, repacked
 * with samq_w4_repack_layout(..., layout 3, ...)) x int8 activation codes (fq_vit QAct on the
 * QuantLinear input, SURVEY.md §8c "Oracle W4A8"): y = float(sum_k A (q - zp)) * a_scale *
 * wscale[n] + bias[n]; wscale = the QuantLinear scales as f32 [G, N] (G = 1 per-channel);
 * epilogues BIAS/BIAS_GELU (f16 out), RESADD_F32/F32, Q8/Q8_GELU.  groupsize -1 (== K), or a
 * multiple of 128 (grouped weights, quant_linear.py:324-335: per group g = k / groupsize the
 * exact int32 sum over the group times wscale[g, n], summed in f32; qzeros [G, N/8]); other
 * groupsizes SAMQ_ERR_UNSUPPORTED. */
int samq_w4a8_gemm(const int8_t* A, int64_t lda, const int32_t* wpacked, const float* wscale,
                   const int32_t* qzeros, const float* bias, void* C, int64_t ldc, int M, int N,
                   int K, int groupsize, int epilogue, float a_scale, float out_scale,
                   hipStream_t stream);
/* The same with an explicit tile config (0 = automatic; per-channel: as samq_i8_gemm_cfg; grouped:
 * 83 128x128, 84 64x64, 87 128x64, 88 64x128). */
int samq_w4a8_gemm_cfg(const int8_t* A, int64_t lda, const int32_t* wpacked, const float* wscale,
                       const int32_t* qzeros, const float* bias, void* C, int64_t ldc, int M, int N,
                       int K, int groupsize, int epilogue, float a_scale, float out_scale, int cfg,
                       hipStream_t stream);

/* samq_w8a8_gemm with the Q8 epilogue (the fq_vit qkv QLinear + attn.qact1) that also stores the
 * codes of output columns [v_col0, N) as fp16 values into v16 [M, ldv] (column c at c - v_col0): the V
 * third of qkv for samq_rel_attention_q8_rows' v16 (round 6).  v_col0 % 64 == 0. */
int samq_w8a8_gemm_v16(const int8_t* A, int64_t lda, const int8_t* wpacked, const float* wscale,
                       const float* bias, int8_t* C, int64_t ldc, int M, int N, int K, float a_scale,
                       float out_scale, void* v16, int v_col0, int64_t ldv, int cfg, hipStream_t stream);

/* Per-channel W4A8 GEMM with the zero point's row sums moved to the producers (round 6):
 * rowsum_in (optional, int32 [M]) = S[m] = sum_k A[m, k] of the int8 input rows -- the zero-point
 * ping-pong (cfg 86 / 93) then subtracts zp[n] * S[m] without re-summing A per column tile; kernels
 * without the row-sum form ignore it.  rowsum_out (optional, int32 [M], ZEROED by the caller;
 * epilogue Q8 / Q8_GELU only) accumulates the row sums of the int8 output codes with atomics, the
 * next GEMM's rowsum_in (replaces the per-tile row sums of quant_linear.py:299-343's zero-point
 * subtraction; fq_vit uniform.py:23-45 codes).  Outputs are bit-identical to samq_w4a8_gemm_cfg. */
int samq_w4a8_gemm_rs(const int8_t* A, int64_t lda, const int32_t* wpacked, const float* wscale,
                      const int32_t* qzeros, const float* bias, void* C, int64_t ldc, int M, int N, int K,
                      int epilogue, float a_scale, float out_scale, const int32_t* rowsum_in,
                      int32_t* rowsum_out, int cfg, hipStream_t stream);

/* Both int8 GEMMs with an explicit weight format (0 = W8 packed, 1 = W4 layout 3) and tile
 * config (0 = automatic; 81 256x256, 82 128x256, 83 128x128, 84 64x64); for tuning and tests. */
int samq_i8_gemm_cfg(const int8_t* A, int64_t lda, int bfmt, const void* wpacked, const float* wscale,
                     const int32_t* qzeros, const float* bias, void* C, int64_t ldc, const int8_t* R,
                     int64_t ldr, int M, int N, int K, int epilogue, float a_scale, float mid_scale,
                     float res_scale, float out_scale, int cfg, hipStream_t stream);

/* W8A8 convolution as an implicit GEMM (fq_vit QConv2d on int8 codes, layers.py:11-74): the A
 * operand is gathered from the code map by the LDS-DMA loader, no im2col copy.
 *   mode 1 (PatchEmbed, fq_vit image_encoder.py PatchEmbed): x int8 [B, Cin, side, side] NCHW,
 *     16x16 patches stride 16; weight codes flattened (n, c, kh, kw) (K = Cin*256);
 *   mode 2 (neck 3x3, padding 1, image_encoder.py:88-104): x int8 [B, side, side, Cin] NHWC,
 *     Cin % 128 == 0; weight codes permuted to (n, ky, kx, c) (K = 9*Cin).
 * Weights from samq_w8_repack; output C int8 [B*G*G, N] codes (row stride N) with epilogue Q8 or
 * Q8_RES as samq_w8a8_gemm; Q8_RES reads residual codes R [rmod, N] at row (r % rmod) when
 * rmod > 0 (the pos_embed codes shared by every image), else R [B*G*G, N]. */
int samq_w8a8_conv_gemm(const int8_t* x, int mode, int B, int Cin, int side, const int8_t* wpacked,
                        const float* wscale, const float* bias, void* C, const int8_t* R, int rmod,
                        int N, int epilogue, float a_scale, float mid_scale, float res_scale,
                        float out_scale, hipStream_t stream);

/* Elementwise activation quantiser (fq_vit QAct in quant mode, layers.py:232-242 ->
 * UniformQuantizer.forward, quantizer/base.py:43-49, uniform.py:23-45, zero point 0):
 * codes[i] = q(x[i], scale); x f32 (or f16 with SAMQ_Q_IN_F16); with SAMQ_Q_OUT_FQ the output is
 * the f32 fake-quant value codes*scale instead of int8 codes. */
#define SAMQ_Q_IN_F16 1
#define SAMQ_Q_OUT_FQ 2
int samq_quantize(const void* x, void* y, int64_t n, float scale, int flags, hipStream_t stream);

/* Running min / max of a calibration tensor viewed as (rows, C) row-major -- fq_vit
 * MinmaxObserver.update (observer/minmax.py:14-29, reshape_tensor observer/base.py:16-29):
 *   SAMQ_MM_PER_ROW: one value per row     (conv / linear weights, v.reshape(out, -1));
 *   SAMQ_MM_PER_COL: one value per column  (channel-last activations, channel_wise);
 *   SAMQ_MM_ALL:     one scalar            (layer_wise).
 * x f32 (f16 with in_f16); max_io / min_io f32 (rows, C or 1 values): overwritten when init != 0,
 * else merged with max(old, new) / min(old, new).  NaN propagates as in torch.max / torch.min.
 * PER_COL and ALL need a float workspace of samq_minmax_workspace(rows, C, axis) elements. */
#define SAMQ_MM_PER_ROW 0
#define SAMQ_MM_PER_COL 1
#define SAMQ_MM_ALL 2
size_t samq_minmax_workspace(int64_t rows, int C, int axis);
int samq_minmax(const void* x, int64_t rows, int C, int in_f16, int axis, float* max_io, float* min_io,
                int init, float* workspace, size_t workspace_floats, hipStream_t stream);

/* Fused gated MLP in ONE launch: C f16 [M, N] = silu(A . Wg) * (A . Wu) with both int4 weight
 * sets in one packed matrix of 2N columns whose 32-column blocks alternate gate block j, up
 * block j (the samq_w4_repack layout-1 blocks interleaved; scales / qzeros interleaved the same
 * way, N2 = 2N, N2 % 256 == 0): each wave's 64-column tile holds a gate block and its up block,
 * the epilogue multiplies them in registers.  fp32 accumulate, exact integer weights (G1).
 * Replaces llama_mlp_fused_4_kernel / triton_llama_mlp_4 (gptq_triton/fused_mlp.py:230-388,
 * 391-477); biases are ignored as there. */
int samq_w4a16_gated_mlp(const void* A, int64_t lda, const int32_t* wpacked, const void* scales,
                         const int32_t* qzeros, void* C, int64_t ldc, int M, int N2, int K, int groupsize,
                         hipStream_t stream);

/* Gated-MLP activation: out f16[i] = silu(gate[i]) * up[i] (f32 inputs).  With two
 * samq_w4a16_gemm(..., SAMQ_EPI_F32) calls it replaces triton_llama_mlp_4 /
 * llama_mlp_fused_4_kernel (gptq_triton/fused_mlp.py:391-477, 230-388). */
int samq_silu_mul(const float* gate, const float* up, void* out, int64_t n, hipStream_t stream);

/* ---------------------------------------------------------------- normalisation */

/* y[r,:] = LayerNorm(x[r,:]) * gamma + beta over C channels (row stride C), f32 statistics.
 * flags: SAMQ_LN_IN_F16 -> x is f16 (else f32); SAMQ_LN_OUT_F32 -> y is f32 (else f16).
 * gamma/beta f32.  Replaces nn.LayerNorm(eps=1e-6) of Block.norm1/norm2
 * (segment_anything/modeling/image_encoder.py:184,187,194,205; build_sam.py:72) and the
 * channel LayerNorm2d of the neck on NHWC tokens (segment_anything/modeling/common.py:31-43). */
#define SAMQ_LN_IN_F16 1
#define SAMQ_LN_OUT_F32 2
/* tuning: rows per wave (1, 2 or 4; 0 = the library default) in bits 16-18 of flags */
#define SAMQ_LN_RPW(n) ((n) << 16)
int samq_layernorm(const void* x, void* y, const float* gamma, const float* beta, int64_t rows,
                   int C, float eps, int flags, hipStream_t stream);
/* samq_layernorm that also writes the row means (f32 [rows]) -- the mu_p of the first folded
 * LayerNorm (SAMQ_EPI_RESADD_LNF) downstream. */
int samq_layernorm_mean(const void* x, void* y, const float* gamma, const float* beta, int64_t rows,
                        int C, float eps, int flags, float* mean_out, hipStream_t stream);

/* LayerNorm with int8 activation codes on either side (fq_vit QIntLayerNorm = nn.LayerNorm
 * between two QActs, layers.py:245-258, fq_vit/models/sam/image_encoder.py:310-331; neck
 * QIntLayerNorm2D eps 1e-5, fq_vit/models/sam/common.py:93-108):
 *   SAMQ_LN_IN_I8:  x = int8 codes * in_scale (else f32 / f16 per SAMQ_LN_IN_F16);
 *   SAMQ_LN_OUT_I8: y = q(LN(x), out_scale) int8 codes; with SAMQ_LN_OUT_F32 as well, y is the
 *   f32 fake-quant value q(..)*out_scale (else f16 / f32 per SAMQ_LN_OUT_F32). */
#define SAMQ_LN_IN_I8 4
#define SAMQ_LN_OUT_I8 8
int samq_layernorm_q(const void* x, void* y, const float* gamma, const float* beta, int64_t rows,
                     int C, float eps, int flags, float in_scale, float out_scale,
                     hipStream_t stream);
/* samq_layernorm_q with int8-code output (SAMQ_LN_OUT_I8) plus rowsum[r] = sum_c y[r, c] (int32
 * [rows], the W4A8 GEMM's rowsum_in) and, when zero_rows is not null, zero_rows[r] = 0 (the
 * accumulator of the next int8-code GEMM's rowsum_out). */
int samq_layernorm_q_rs(const void* x, void* y, const float* gamma, const float* beta, int64_t rows,
                        int C, float eps, int flags, float in_scale, float out_scale, int32_t* rowsum,
                        int32_t* zero_rows, hipStream_t stream);

/* Residual add + LayerNorm (Block.forward's x = x + attn(...) / x = x + mlp(...) followed by the
 * next norm, image_encoder.py:199-207): x f32 [rows, C] += delta (f16 with SAMQ_LN_DELTA_F16,
 * else f32 -- the preceding GEMM's plain-stored output), written back in place, then
 * y = LayerNorm(x) (f16, or int8 codes q(LN(x), out_scale) with SAMQ_LN_OUT_I8).  C <= 1280. */
#define SAMQ_LN_DELTA_F16 16
int samq_add_layernorm(void* x, const void* delta, void* y, const float* gamma, const float* beta,
                       int64_t rows, int C, float eps, int flags, float out_scale, hipStream_t stream);

/* ---------------------------------------------------------------- attention */

/* Multi-head attention with in-kernel decomposed relative-position bias over an image token
 * grid, windowed or global, reading Q/K/V straight from the qkv projection output.
 * Replaces QuantAttention.forward's attention part -- add_decomposed_rel_pos + the Triton
 * `_fwd_kernel1` + `forward` (gptq_triton/fused_attention.py:46-80, 107-149, 159-358) -- AND
 * the window_partition / window_unpartition copies around it
 * (segment_anything/modeling/image_encoder.py:195-202, 282-333):
 *   qkv  f16 [B, H, W, 3, heads, hd]  (the qkv Linear output, natural token order)
 *   out  f16 [B, H, W, heads*hd]      (natural token order; window padding cropped)
 *   window = 0: global attention over the H x W grid (requires H == W, H % 16 == 0);
 *   window = S > 0: attention inside S x S windows of the grid zero-padded to a multiple of S;
 *     padded tokens are keys/values whose q/k/v equal the qkv bias (the reference projects the
 *     zero-padded LayerNorm output), given by qkv_bias (f16 [3*heads*hd]) or zeros if NULL;
 *   rel_pos_h / rel_pos_w f16 [2*side-1, hd] with side = window or H; the width term uses the
 *     query ROW as the table index (reference quirk, image_encoder.py:402 /
 *     fused_attention.py:78).  hd in {64, 80}; side <= 64 and (window == 0 => side % 16 == 0).
 *   sm_scale multiplies q.k (the reference passes head_dim**-0.5). */
int samq_rel_attention(const void* qkv, const void* qkv_bias, const void* rel_pos_h,
                       const void* rel_pos_w, void* out, int B, int H, int W, int heads, int hd,
                       int window, float sm_scale, hipStream_t stream);

/* samq_rel_attention with the W4A8 proj input quantiser folded into its store: out int8
 * [B, H, W, heads*hd] = clamp(rne(fp16(o) / out_scale), -128, 127) -- the fq_vit QAct on the
 * QuantLinear input (fq_vit/models/ptq/layers.py:203-242, quantizer/uniform.py:31-36) applied to
 * the fp16 attention output, bit-identical to samq_rel_attention + samq_quantize.  out_scale > 0. */
int samq_rel_attention_q(const void* qkv, const void* qkv_bias, const void* rel_pos_h,
                         const void* rel_pos_w, int8_t* out, int B, int H, int W, int heads, int hd,
                         int window, float sm_scale, float out_scale, hipStream_t stream);

/* Reference functional API `fused_attention.forward(inp, pos_emb1, pos_emb2, head_num,
 * hidden_dim, sm_scale)` (gptq_triton/fused_attention.py:312-358): attention over each of B
 * independent S x S grids with PRECOMPUTED bias terms rel_h, rel_w f16 [B*heads, S, S, S]
 * (bias[m, n] = rel_h[m, n // S] + rel_w[m, n % S]).  inp f16 [B, S, S, 3*heads*hd],
 * out f16 [B, S, S, heads*hd]. */
int samq_attention_relbias(const void* inp, const void* rel_h, const void* rel_w, void* out, int B,
                           int S, int heads, int hd, float sm_scale, hipStream_t stream);

/* W8A8 attention (fq_vit quant-mode Attention.forward, fq_vit/models/sam/image_encoder.py:437-478,
 * with window_partition / window_unpartition :282-333 folded in) on int8 codes:
 *   qkv  int8 [B, H, W, 3, heads, hd] codes of attn.qact1 (scale s_qkv), natural token order;
 *   scores = q8((q*s_qkv*sm_scale).(k*s_qkv), s_a1) * s_a1            (qact_attn1)
 *   scores = q8(scores + rel_h + rel_w, s_a2) * s_a2                   (use_rel_pos_qact; rel_w
 *            indexed by the query ROW, quirk 1; rel tables f32 [2*side-1, hd])
 *   out  int8 [B, H, W, heads*hd] = q8(softmax(scores) . (v*s_qkv), s_out)     (qact2)
 * window > 0: S x S windows over the grid padded to a multiple of S (pad tokens' q/k/v =
 * q8(qkv_bias f32 [3*heads*hd], s_qkv), or 0 if qkv_bias is NULL), window <= 16;
 * window == 0: global over an H == W <= 64 grid.  hd must be 64 (else SAMQ_ERR_UNSUPPORTED). */
int samq_rel_attention_q8(const int8_t* qkv, const float* qkv_bias, const float* rel_pos_h,
                          const float* rel_pos_w, int8_t* out, int B, int H, int W, int heads,
                          int hd, int window, float sm_scale, float s_qkv, float s_a1, float s_a2,
                          float s_out, hipStream_t stream);
/* samq_rel_attention_q8 over a range of the grid's rows (round 6: the W8A8 engine's opt-in row lanes
 * run one image as two concurrent kernel chains): global (window == 0, H == W == 64) -- the queries of
 * grid rows [row0, row0 + rows) against all keys; windows -- the windows of rows [row0, row0 + rows),
 * row0 a multiple of window and rows too unless the range ends at H.  rows < 0: the whole grid.
 * v16 (optional, 16-byte aligned): the V codes as fp16 [B, H, W, heads*hd] (samq_w8a8_gemm_v16) --
 * the 64 x 64 global kernel then stages V without converting it; same output codes. */
int samq_rel_attention_q8_rows(const int8_t* qkv, const float* qkv_bias, const float* rel_pos_h,
                               const float* rel_pos_w, int8_t* out, int B, int H, int W, int heads, int hd,
                               int window, float sm_scale, float s_qkv, float s_a1, float s_a2, float s_out,
                               int row0, int rows, const void* v16, hipStream_t stream);

/* ---------------------------------------------------------------- patch embedding / neck */

/* PatchEmbed (segment_anything/modeling/image_encoder.py:411-442) + pos_embed add (:108-110)
 * as one implicit GEMM: img f16 [B, Cin, S, S] (NCHW, S = img_size), weight f16 [N, Cin*p*p]
 * (the Conv2d weight flattened (c, kh, kw)), bias f32 [N] or NULL, pos f32 [(S/p)^2, N] or NULL
 * -> out f32 [B, S/p, S/p, N] (the residual stream; fp32 accumulate, no fp16 rounding).
 * patch % 8 == 0, Cin*p*p % 32 == 0, N % 128 == 0. */
int samq_patch_embed(const void* img, const void* weight, const float* bias, const float* pos, float* out,
                     int B, int Cin, int img_size, int patch, int N, hipStream_t stream);

/* The same in fp32 end to end (img f32, weight f32, fp32 MFMA): the W4A8 encoder's patch
 * embedding, whose int8 quantiser follows directly (fq_vit image_encoder.py PatchEmbed + QAct).
 * patch % 4 == 0, Cin*p*p % 16 == 0, N % 128 == 0. */
int samq_patch_embed_f32(const float* img, const float* weight, const float* bias, const float* pos,
                         float* out, int B, int Cin, int img_size, int patch, int N, hipStream_t stream);

/* PatchEmbed straight from RAW pixels (SamPredictor.set_image -> set_torch_image,
 * segment_anything/predictor.py:34-90): img uint8 [B, Cin, h, w] (NCHW, h, w <= img_size) is
 * normalised in the A-operand gather exactly as Sam.preprocess does (modeling/sam.py:164-174):
 * (pixel - pixel_mean[c]) / pixel_std[c] (f32 [Cin] each), zero-padded to img_size x img_size;
 * then as samq_patch_embed (weight f16) or, with weight_f32, as samq_patch_embed_f32. */
int samq_patch_embed_u8(const uint8_t* img, int h, int w, const float* pixel_mean, const float* pixel_std,
                        const void* weight, int weight_f32, const float* bias, const float* pos, float* out,
                        int B, int Cin, int img_size, int patch, int N, hipStream_t stream);

/* Neck 1x1 conv, no bias (image_encoder.py:88-104 neck[0]) on the fp32 token rows:
 * x f32 [M, K] (converted to f16 on load, as the reference's fp16 neck), weight f16 [N, K]
 * -> out f16 [M, N].  K % 32 == 0, N % 128 == 0. */
int samq_conv1x1_f32(const float* x, const void* weight, void* out, int64_t M, int N, int K,
                     hipStream_t stream);

/* Neck 3x3 conv, padding 1, no bias (neck[2]) on an NHWC f16 map: x f16 [B, G, G, Cin],
 * weight f16 [N, 3, 3, Cin] (the Conv2d weight permuted (n, ky, kx, c)) -> out f16 [B, G, G, N].
 * Cin % 32 == 0, N % 128 == 0. */
int samq_conv3x3_nhwc(const void* x, const void* weight, void* out, int B, int G, int Cin, int N,
                      hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* SAMQ_H */

// Row LayerNorm (f32 statistics, f16 output) for the ViT blocks' norm1 / norm2.
// Reference: nn.LayerNorm(eps=1e-6) (segment_anything/build_sam.py:72) applied in
// Block.forward (segment_anything/modeling/image_encoder.py:194, 205).  HBM-bound: one wave
// per row, 16-byte vector loads, the row held in registers (two-pass mean / variance).
#include "common.h"

namespace samq {

// IN: 0 f32, 1 f16, 2 int8 codes (x = code * in_scale)
// OUT: 0 f16, 1 f32, 2 int8 codes q(y, out_scale), 3 f32 fake-quant q(y, out_scale) * out_scale
enum { LN_F32 = 0, LN_F16 = 1, LN_I8 = 2, LN_FQ32 = 3 };

__device__ __forceinline__ float ln_q8(float v, float s) {   // fq_vit uniform.py:31-36
  return q8_exact(v, s, 1.0f / s);   // the reciprocal is loop-invariant (hoisted)
}

// ADD (f32 input only): the residual add of the GEMM before the LayerNorm runs here instead of in
// that GEMM's epilogue -- x += delta (delta f16 when ADD == 1, f32 when ADD == 2; the GEMM wrote
// y = acc * s + b with a plain store), x written back in place, then the LayerNorm of the new x.
// f32 delta: the same fp32 add as the GEMM's read-modify-write epilogue (bit-identical x).  The ADD
// variants read AND write the residual through ``xres`` (plain, non-const: the buffer is updated in
// place); ``xin`` (const restrict) is the input of the ADD == 0 variants only.
template <int IN, int OUT, int VPT, int RPW, int ADD = 0>
__global__ __launch_bounds__(256) void layernorm_kernel(const void* __restrict__ xin, void* __restrict__ y,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, int64_t rows, int C,
                                                        float eps, float in_scale, float out_scale,
                                                        float* __restrict__ mean_out,
                                                        const void* __restrict__ delta = nullptr,
                                                        float* xres = nullptr, int* __restrict__ rs_out = nullptr,
                                                        int* __restrict__ rs_zero = nullptr) {
  static_assert(ADD == 0 || IN == LN_F32, "residual add: f32 rows");
  const int lane = threadIdx.x & 63;
  const int64_t row0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (row0 >= rows) return;
  const int nvec = C / 4;
  // all RPW rows' loads are issued before the first reduction: RPW x VPT 16-byte loads in flight
  float4_t v[RPW][VPT];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int64_t row = row0 + r < rows ? row0 + r : rows - 1;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int j = lane + 64 * i;
      if (j < nvec) {
        if (IN == LN_F16) {
          const half4_t h = ((const half4_t*)xin)[row * nvec + j];
          v[r][i] = float4_t{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
        } else if (IN == LN_I8) {
          const uint32_t w = ((const uint32_t*)xin)[row * nvec + j];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[r][i][e] = (float)(int8_t)((w >> (8 * e)) & 0xFFu) * in_scale;
        } else {
          v[r][i] = ADD != 0 ? ((const float4_t*)xres)[row * nvec + j] : ((const float4_t*)xin)[row * nvec + j];
          if constexpr (ADD == 1) {
            const half4_t h = ((const half4_t*)delta)[row * nvec + j];
            v[r][i] += float4_t{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
          } else if constexpr (ADD == 2) {
            v[r][i] += ((const float4_t*)delta)[row * nvec + j];
          }
        }
      } else {
        v[r][i] = float4_t{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  if constexpr (ADD != 0) {   // the new residual rows back in place
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int64_t row = row0 + r;
      if (row < rows) {
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
          const int j = lane + 64 * i;
          if (j < nvec) ((float4_t*)xres)[row * nvec + j] = v[r][i];
        }
      }
    }
  }
  // int8-code output (the W4A8 LN-q): gamma / beta loaded beside the rows, not behind the
  // reductions (measured: LN-q 26.1 -> 21.3 us at 16384 rows, W4A8 step +0.6 %; the f16-output
  // LayerNorm of W4A16 runs inside the other lane's GEMMs and lost 0.5 % with it: late loads there)
  constexpr bool EARLY_GB = OUT == LN_I8;
  float4_t gv[EARLY_GB ? VPT : 1], bv[EARLY_GB ? VPT : 1];
  if constexpr (EARLY_GB) {
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int j = lane + 64 * i;
      gv[i] = j < nvec ? ((const float4_t*)gamma)[j] : float4_t{0.f, 0.f, 0.f, 0.f};
      bv[i] = j < nvec ? ((const float4_t*)beta)[j] : float4_t{0.f, 0.f, 0.f, 0.f};
    }
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int64_t row = row0 + r;
    if (row >= rows) break;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) s += v[r][i][0] + v[r][i][1] + v[r][i][2] + v[r][i][3];
    const float mean = wave_sum_valu(s) / (float)C;
    if (mean_out && lane == 0) mean_out[row] = mean;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int j = lane + 64 * i;
      if (j < nvec) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = v[r][i][e] - mean;
          q += d * d;
        }
      }
    }
    const float rstd = rsqrtf(wave_sum_valu(q) / (float)C + eps);
    int rsi = 0;   // LN_I8 with rs_out: the row's codes summed (the W4A8 GEMM's zero-point row sum)
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int j = lane + 64 * i;
      if (j < nvec) {
        const float4_t g = EARLY_GB ? gv[EARLY_GB ? i : 0] : ((const float4_t*)gamma)[j];
        const float4_t b = EARLY_GB ? bv[EARLY_GB ? i : 0] : ((const float4_t*)beta)[j];
        float4_t o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (v[r][i][e] - mean) * rstd * g[e] + b[e];
        if (OUT == LN_F32) {
          ((float4_t*)y)[row * nvec + j] = o;
        } else if (OUT == LN_FQ32) {
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = ln_q8(o[e], out_scale) * out_scale;
          ((float4_t*)y)[row * nvec + j] = o;
        } else if (OUT == LN_I8) {
          const float inv = 1.0f / out_scale, lim = 130.0f * out_scale;   // (loop-invariant: hoisted)
          const float2_t c01 = q8_exact2(float2_t{o[0], o[1]}, out_scale, inv, lim);
          const float2_t c23 = q8_exact2(float2_t{o[2], o[3]}, out_scale, inv, lim);
          const uint32_t wq = q8_pack4(c01.x, c01.y, c23.x, c23.y);
          ((uint32_t*)y)[row * nvec + j] = wq;
          if (rs_out) rsi = __builtin_amdgcn_sdot4((int)wq, 0x01010101, rsi, false);
        } else {
          ((half4_t*)y)[row * nvec + j] = half4_t{(_Float16)o[0], (_Float16)o[1], (_Float16)o[2], (_Float16)o[3]};
        }
      }
    }
    if (OUT == LN_I8 && rs_out) {   // |sum| <= 128 C < 2^24: the f32 wave sum is exact
      const float t = wave_sum_valu((float)rsi);
      if (lane == 0) rs_out[row] = (int)t;
    }
    if (rs_zero && lane == 0) rs_zero[row] = 0;   // the next GEMM's rs_out accumulator
  }
}

}  // namespace samq

using namespace samq;

// rows per wave: SAMQ_LN_RPW(n) in flags (0 = default; rows wider than 1280 channels use 1)
#define SAMQ_LN_DEFAULT_RPW 2   // measured: ViT-H rows 33.0 -> 27.3 us uncached (tools/bench_ln.py)
static int ln_rpw(int flags) {
  const int r = (flags >> 16) & 7;
  return r == 0 ? SAMQ_LN_DEFAULT_RPW : r;
}

static int ln_launch(const void* x, void* y, const float* gamma, const float* beta, int64_t rows, int C, float eps,
                     int in, int out, float in_scale, float out_scale, int rpw, hipStream_t stream,
                     float* mean_out = nullptr, int* rs_out = nullptr, int* rs_zero = nullptr) {
  if (rows == 0) return SAMQ_OK;   // empty batch: no work, data pointers may be null
  SAMQ_REQUIRE(x && y && gamma && beta, SAMQ_ERR_INVALID, "layernorm: null pointer");
  SAMQ_REQUIRE(C > 0 && C % 4 == 0 && C <= 4096, SAMQ_ERR_INVALID, "layernorm: C must be a multiple of 4, <= 4096");
  if (rows <= 0) return SAMQ_OK;
  SAMQ_REQUIRE(rpw == 1 || rpw == 2 || rpw == 4, SAMQ_ERR_INVALID, "layernorm: rows per wave must be 1, 2 or 4");
  const int vpt = (C / 4 + 63) / 64;
  if (vpt > 5) rpw = 1;
  const dim3 grid((unsigned)((rows + 4 * rpw - 1) / (4 * rpw)));
#define LN_R(I, O, V) \
  do { \
    if (rpw == 1) hipLaunchKernelGGL((layernorm_kernel<I, O, V, 1>), grid, dim3(256), 0, stream, x, y, gamma, beta, rows, C, eps, in_scale, out_scale, mean_out, nullptr, nullptr, rs_out, rs_zero); \
    else if (rpw == 2) hipLaunchKernelGGL((layernorm_kernel<I, O, V, 2>), grid, dim3(256), 0, stream, x, y, gamma, beta, rows, C, eps, in_scale, out_scale, mean_out, nullptr, nullptr, rs_out, rs_zero); \
    else hipLaunchKernelGGL((layernorm_kernel<I, O, V, 4>), grid, dim3(256), 0, stream, x, y, gamma, beta, rows, C, eps, in_scale, out_scale, mean_out, nullptr, nullptr, rs_out, rs_zero); \
  } while (0)
#define LN_V(I, O) \
  do { \
    if (vpt <= 1) LN_R(I, O, 1); \
    else if (vpt <= 3) LN_R(I, O, 3); \
    else if (vpt <= 4) LN_R(I, O, 4); \
    else if (vpt <= 5) LN_R(I, O, 5); \
    else LN_R(I, O, 16); \
  } while (0)
#define LN_O(I) \
  do { \
    switch (out) { case LN_F16: LN_V(I, LN_F16); break; case LN_F32: LN_V(I, LN_F32); break; \
                   case LN_I8: LN_V(I, LN_I8); break; default: LN_V(I, LN_FQ32); break; } \
  } while (0)
  switch (in) { case LN_F16: LN_O(LN_F16); break; case LN_I8: LN_O(LN_I8); break; default: LN_O(LN_F32); break; }
#undef LN_O
#undef LN_V
#undef LN_R
  SAMQ_LAUNCH_CHECK("layernorm launch");
  return SAMQ_OK;
}

extern "C" int samq_layernorm(const void* x, void* y, const float* gamma, const float* beta, int64_t rows, int C,
                              float eps, int flags, hipStream_t stream) {
  return ln_launch(x, y, gamma, beta, rows, C, eps, (flags & SAMQ_LN_IN_F16) ? LN_F16 : LN_F32,
                   (flags & SAMQ_LN_OUT_F32) ? LN_F32 : LN_F16, 1.f, 1.f, ln_rpw(flags), stream);
}

extern "C" int samq_layernorm_mean(const void* x, void* y, const float* gamma, const float* beta, int64_t rows,
                                   int C, float eps, int flags, float* mean_out, hipStream_t stream) {
  SAMQ_REQUIRE(mean_out, SAMQ_ERR_INVALID, "layernorm_mean: null mean_out");
  return ln_launch(x, y, gamma, beta, rows, C, eps, (flags & SAMQ_LN_IN_F16) ? LN_F16 : LN_F32,
                   (flags & SAMQ_LN_OUT_F32) ? LN_F32 : LN_F16, 1.f, 1.f, ln_rpw(flags), stream, mean_out);
}

// x += delta (f16 [rows, C] with SAMQ_LN_DELTA_F16, else f32), in place, then y = LN(x) (f16, or
// int8 codes q(LN(x), out_scale) with SAMQ_LN_OUT_I8): the residual add of the preceding GEMM
// moved out of its epilogue.  Rows of C <= 1280 (the ViT-H / vit_b widths).
extern "C" int samq_add_layernorm(void* x, const void* delta, void* y, const float* gamma, const float* beta,
                                  int64_t rows, int C, float eps, int flags, float out_scale, hipStream_t stream) {
  if (rows == 0) return SAMQ_OK;   // empty batch: no work, data pointers may be null
  SAMQ_REQUIRE(x && delta && y && gamma && beta, SAMQ_ERR_INVALID, "add_layernorm: null pointer");
  SAMQ_REQUIRE(C > 0 && C % 4 == 0 && C <= 1280, SAMQ_ERR_INVALID, "add_layernorm: C must be a multiple of 4, <= 1280");
  SAMQ_REQUIRE(!(flags & SAMQ_LN_OUT_I8) || out_scale > 0.f, SAMQ_ERR_INVALID, "add_layernorm: out_scale must be > 0");
  if (rows <= 0) return SAMQ_OK;
  const int rpw = ln_rpw(flags);
  SAMQ_REQUIRE(rpw == 1 || rpw == 2 || rpw == 4, SAMQ_ERR_INVALID, "add_layernorm: rows per wave must be 1, 2 or 4");
  const dim3 grid((unsigned)((rows + 4 * rpw - 1) / (4 * rpw)));
  const bool i8 = (flags & SAMQ_LN_OUT_I8) != 0, d16 = (flags & SAMQ_LN_DELTA_F16) != 0;
  const int vpt = (C / 4 + 63) / 64;
#define ALN(O, V, R, A) hipLaunchKernelGGL((layernorm_kernel<LN_F32, O, V, R, A>), grid, dim3(256), 0, stream, \
                                           (const void*)nullptr, y, gamma, beta, rows, C, eps, 1.f, out_scale, nullptr, \
                                           delta, (float*)x)
#define ALN_R(O, V, A) do { if (rpw == 1) ALN(O, V, 1, A); else if (rpw == 2) ALN(O, V, 2, A); else ALN(O, V, 4, A); } while (0)
#define ALN_V(O, A) do { if (vpt <= 3) ALN_R(O, 3, A); else if (vpt <= 4) ALN_R(O, 4, A); else ALN_R(O, 5, A); } while (0)
  if (i8) { if (d16) ALN_V(LN_I8, 1); else ALN_V(LN_I8, 2); }
  else { if (d16) ALN_V(LN_F16, 1); else ALN_V(LN_F16, 2); }
#undef ALN_V
#undef ALN_R
#undef ALN
  SAMQ_LAUNCH_CHECK("add_layernorm launch");
  return SAMQ_OK;
}

extern "C" int samq_layernorm_q(const void* x, void* y, const float* gamma, const float* beta, int64_t rows, int C,
                                float eps, int flags, float in_scale, float out_scale, hipStream_t stream) {
  SAMQ_REQUIRE(!(flags & SAMQ_LN_IN_I8) || in_scale > 0.f, SAMQ_ERR_INVALID, "layernorm_q: in_scale must be > 0");
  SAMQ_REQUIRE(!(flags & SAMQ_LN_OUT_I8) || out_scale > 0.f, SAMQ_ERR_INVALID, "layernorm_q: out_scale must be > 0");
  const int in = (flags & SAMQ_LN_IN_I8) ? LN_I8 : ((flags & SAMQ_LN_IN_F16) ? LN_F16 : LN_F32);
  const int out = (flags & SAMQ_LN_OUT_I8) ? ((flags & SAMQ_LN_OUT_F32) ? LN_FQ32 : LN_I8)
                                           : ((flags & SAMQ_LN_OUT_F32) ? LN_F32 : LN_F16);
  return ln_launch(x, y, gamma, beta, rows, C, eps, in, out, in_scale, out_scale, ln_rpw(flags), stream);
}

// LN-q with the output rows' code sums (round 6): rowsum[r] = sum_c y[r, c] (int8 codes, SAMQ_LN_OUT_I8
// required) for the W4A8 zero-point GEMM that reads y; zero_rows (optional) [rows] int32 set to 0 --
// the accumulator the next int8-code GEMM epilogue adds its output row sums into
extern "C" int samq_layernorm_q_rs(const void* x, void* y, const float* gamma, const float* beta, int64_t rows, int C,
                                   float eps, int flags, float in_scale, float out_scale, int32_t* rowsum,
                                   int32_t* zero_rows, hipStream_t stream) {
  SAMQ_REQUIRE((flags & SAMQ_LN_OUT_I8) && !(flags & SAMQ_LN_OUT_F32), SAMQ_ERR_INVALID,
               "layernorm_q_rs: row sums of int8-code outputs only (SAMQ_LN_OUT_I8)");
  SAMQ_REQUIRE(rows == 0 || rowsum, SAMQ_ERR_INVALID, "layernorm_q_rs: null rowsum");
  SAMQ_REQUIRE(!(flags & SAMQ_LN_IN_I8) || in_scale > 0.f, SAMQ_ERR_INVALID, "layernorm_q_rs: in_scale must be > 0");
  SAMQ_REQUIRE(out_scale > 0.f, SAMQ_ERR_INVALID, "layernorm_q_rs: out_scale must be > 0");
  const int in = (flags & SAMQ_LN_IN_I8) ? LN_I8 : ((flags & SAMQ_LN_IN_F16) ? LN_F16 : LN_F32);
  return ln_launch(x, y, gamma, beta, rows, C, eps, in, LN_I8, in_scale, out_scale, ln_rpw(flags), stream, nullptr,
                   rowsum, zero_rows);
}

// Row LayerNorm (f32 statistics, f16 output) for the ViT blocks' norm1 / norm2.
// Reference: nn.LayerNorm(eps=1e-6) (segment_anything/build_sam.py:72) applied in
// Block.forward (segment_anything/modeling/image_encoder.py:194, 205).  HBM-bound: one wave
// per row, 16-byte vector loads, the row held in registers (two-pass mean / variance).
#include "common.h"

namespace samq {

template <bool IN_F16, bool OUT_F32, int VPT>  // VPT = float4 (or half4) vectors per lane
__global__ __launch_bounds__(256) void layernorm_kernel(const void* __restrict__ xin, void* __restrict__ y,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, int64_t rows, int C,
                                                        float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nvec = C / 4;
  float4_t v[VPT];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int j = lane + 64 * i;
    if (j < nvec) {
      if (IN_F16) {
        const half4_t h = ((const half4_t*)xin)[row * nvec + j];
        v[i] = float4_t{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
      } else {
        v[i] = ((const float4_t*)xin)[row * nvec + j];
      }
      s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
    } else {
      v[i] = float4_t{0.f, 0.f, 0.f, 0.f};
    }
  }
  const float mean = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int j = lane + 64 * i;
    if (j < nvec) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[i][e] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)C + eps);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int j = lane + 64 * i;
    if (j < nvec) {
      const float4_t g = ((const float4_t*)gamma)[j];
      const float4_t b = ((const float4_t*)beta)[j];
      float4_t o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (v[i][e] - mean) * rstd * g[e] + b[e];
      if (OUT_F32) {
        ((float4_t*)y)[row * nvec + j] = o;
      } else {
        ((half4_t*)y)[row * nvec + j] = half4_t{(_Float16)o[0], (_Float16)o[1], (_Float16)o[2], (_Float16)o[3]};
      }
    }
  }
}

}  // namespace samq

using namespace samq;

extern "C" int samq_layernorm(const void* x, void* y, const float* gamma, const float* beta, int64_t rows, int C,
                              float eps, int flags, hipStream_t stream) {
  SAMQ_REQUIRE(x && y && gamma && beta, SAMQ_ERR_INVALID, "layernorm: null pointer");
  SAMQ_REQUIRE(C > 0 && C % 4 == 0 && C <= 4096, SAMQ_ERR_INVALID, "layernorm: C must be a multiple of 4, <= 4096");
  if (rows <= 0) return SAMQ_OK;
  const dim3 grid((unsigned)((rows + 3) / 4));
  const int vpt = (C / 4 + 63) / 64;
  const bool in16 = flags & SAMQ_LN_IN_F16, out32 = flags & SAMQ_LN_OUT_F32;
#define LN_V(I, O) \
  do { \
    if (vpt <= 1) hipLaunchKernelGGL((layernorm_kernel<I, O, 1>), grid, dim3(256), 0, stream, x, y, gamma, beta, rows, C, eps); \
    else if (vpt <= 3) hipLaunchKernelGGL((layernorm_kernel<I, O, 3>), grid, dim3(256), 0, stream, x, y, gamma, beta, rows, C, eps); \
    else if (vpt <= 4) hipLaunchKernelGGL((layernorm_kernel<I, O, 4>), grid, dim3(256), 0, stream, x, y, gamma, beta, rows, C, eps); \
    else if (vpt <= 5) hipLaunchKernelGGL((layernorm_kernel<I, O, 5>), grid, dim3(256), 0, stream, x, y, gamma, beta, rows, C, eps); \
    else hipLaunchKernelGGL((layernorm_kernel<I, O, 16>), grid, dim3(256), 0, stream, x, y, gamma, beta, rows, C, eps); \
  } while (0)
  if (in16) { if (out32) LN_V(true, true); else LN_V(true, false); }
  else { if (out32) LN_V(false, true); else LN_V(false, false); }
#undef LN_V
  SAMQ_LAUNCH_CHECK("layernorm launch");
  return SAMQ_OK;
}

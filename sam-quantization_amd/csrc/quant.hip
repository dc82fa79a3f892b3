// Elementwise activation quantiser: fq_vit QAct in quant mode (fq_vit/models/ptq/layers.py:232-242
// -> BaseQuantizer.forward, quantizer/base.py:43-49 -> UniformQuantizer.quant/dequantize,
// quantizer/uniform.py:23-45) with the int8 symmetric layer-wise configuration (zero point 0):
//   code = clamp(round_half_even(x / s), -128, 127)   (the correctly rounded quotient, via q8_exact)
// Output int8 codes (consumed by the int8 GEMMs / attention) or the f32 fake-quant value.
// HBM-bound: 4 elements per lane per step, grid-stride.
#include "common.h"

namespace samq {

template <bool IN_F16, bool OUT_FQ>
__global__ __launch_bounds__(256) void quantize_kernel(const void* __restrict__ x, void* __restrict__ y, int64_t n,
                                                       float s) {
  const float inv = 1.0f / s;   // q8_exact (common.h): multiply + two Markstein corrections
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4 + (n & 3); i += stride) {
    // vector part [0, n4) then the scalar tail (n & 3 elements) on the first lanes
    const bool tail = i >= n4;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    int cnt = 4;
    int64_t base = i * 4;
    if (!tail) {
      if (IN_F16) {
        const half4_t h = ((const half4_t*)x)[i];
        v[0] = (float)h[0]; v[1] = (float)h[1]; v[2] = (float)h[2]; v[3] = (float)h[3];
      } else {
        const float4_t f = ((const float4_t*)x)[i];
        v[0] = f[0]; v[1] = f[1]; v[2] = f[2]; v[3] = f[3];
      }
    } else {
      base = n4 * 4 + (i - n4);
      cnt = 1;
      v[0] = IN_F16 ? (float)((const _Float16*)x)[base] : ((const float*)x)[base];
    }
    float q[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) q[e] = q8_exact(v[e], s, inv);
    if (OUT_FQ) {
      if (cnt == 4) ((float4_t*)y)[i] = float4_t{q[0] * s, q[1] * s, q[2] * s, q[3] * s};
      else ((float*)y)[base] = q[0] * s;
    } else {
      if (cnt == 4) {
        uint32_t w = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) w |= ((uint32_t)(int)q[e] & 0xFFu) << (8 * e);
        ((uint32_t*)y)[i] = w;
      } else {
        ((int8_t*)y)[base] = (int8_t)(int)q[0];
      }
    }
  }
}

}  // namespace samq

using namespace samq;

extern "C" int samq_quantize(const void* x, void* y, int64_t n, float scale, int flags, hipStream_t stream) {
  if (n == 0) return SAMQ_OK;   // empty batch: no work, data pointers may be null
  SAMQ_REQUIRE(x && y, SAMQ_ERR_INVALID, "quantize: null pointer");
  SAMQ_REQUIRE(scale > 0.f, SAMQ_ERR_INVALID, "quantize: scale must be > 0");
  SAMQ_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0, SAMQ_ERR_INVALID,
               "quantize: pointers must be 16-byte aligned");
  if (n <= 0) return SAMQ_OK;
  const int64_t work = n / 4 + (n & 3);
  const int blocks = (int)((work + 255) / 256 < 16384 ? (work + 255) / 256 : 16384);
  const bool f16 = flags & SAMQ_Q_IN_F16, fq = flags & SAMQ_Q_OUT_FQ;
  if (f16) {
    if (fq) hipLaunchKernelGGL((quantize_kernel<true, true>), dim3(blocks), dim3(256), 0, stream, x, y, n, scale);
    else hipLaunchKernelGGL((quantize_kernel<true, false>), dim3(blocks), dim3(256), 0, stream, x, y, n, scale);
  } else {
    if (fq) hipLaunchKernelGGL((quantize_kernel<false, true>), dim3(blocks), dim3(256), 0, stream, x, y, n, scale);
    else hipLaunchKernelGGL((quantize_kernel<false, false>), dim3(blocks), dim3(256), 0, stream, x, y, n, scale);
  }
  SAMQ_LAUNCH_CHECK("quantize launch");
  return SAMQ_OK;
}

// ------------------------------------------------------------------ gated MLP activation
// out = silu(gate) * up (f32 in, f16 out): the activation / product of the reference's fused
// LLaMA MLP kernel (gptq_triton/fused_mlp.py:230-388, silu :386-388), whose two int4 GEMMs run
// as samq_w4a16_gemm with the f32 epilogue.
namespace samq {
__global__ __launch_bounds__(256) void silu_mul_kernel(const float* __restrict__ g, const float* __restrict__ u,
                                                       _Float16* __restrict__ out, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    const float x = g[i];
    out[i] = (_Float16)(x / (1.0f + expf(-x)) * u[i]);
  }
}
}  // namespace samq

extern "C" int samq_silu_mul(const float* gate, const float* up, void* out, int64_t n, hipStream_t stream) {
  if (n == 0) return SAMQ_OK;   // empty batch: no work, data pointers may be null
  SAMQ_REQUIRE(gate && up && out, SAMQ_ERR_INVALID, "silu_mul: null pointer");
  if (n <= 0) return SAMQ_OK;
  const int blocks = (int)((n + 255) / 256 < 16384 ? (n + 255) / 256 : 16384);
  hipLaunchKernelGGL(samq::silu_mul_kernel, dim3(blocks), dim3(256), 0, stream, gate, up, (_Float16*)out, n);
  SAMQ_LAUNCH_CHECK("silu_mul launch");
  return SAMQ_OK;
}

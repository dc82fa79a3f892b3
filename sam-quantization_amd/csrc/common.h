// Shared device helpers and the C-ABI error plumbing for libsamq_hip.so (gfx950 / CDNA4).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <type_traits>

#include "../../include/samq.h"

namespace samq {

typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float float4_t __attribute__((ext_vector_type(4)));
typedef float float16_t __attribute__((ext_vector_type(16)));
typedef int int4_t __attribute__((ext_vector_type(4)));
typedef int int16_t_v __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef short short4_t __attribute__((ext_vector_type(4)));
typedef signed char char8_t_v __attribute__((ext_vector_type(8)));

#define SAMQ_GLOBAL __attribute__((address_space(1)))
#define SAMQ_LDS __attribute__((address_space(3)))

// ---------------------------------------------------------------- error state
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int check_hip(hipError_t e, const char* what);

#define SAMQ_REQUIRE(cond, code, msg)                  \
  do {                                                 \
    if (!(cond)) return ::samq::fail((code), (msg));   \
  } while (0)

#define SAMQ_LAUNCH_CHECK(what) \
  do { hipError_t _e = hipGetLastError(); if (_e != hipSuccess) return ::samq::check_hip(_e, what); } while (0)

// ---------------------------------------------------------------- device helpers
__device__ __forceinline__ float gelu_erf(float x) {
  // nn.GELU() default (exact erf form), reference segment_anything/modeling/common.py:25-26
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f));
}

// GELU(x) = x * Phi(x) with erf from Abramowitz & Stegun 7.1.26 (|error of erf| <= 1.5e-7, i.e. far
// below the fp16 rounding of the GEMM output), rearranged for the fewest VALU issues:
//   GELU(x) = 0.5 x + 0.5 |x| erf(|x|/sqrt2) = relu(x) - |x| * (0.5 P(t)) * exp(-x^2/2),
//   t = 1 / (1 + p |x|/sqrt2),  P(t) = t (a1 + t (a2 + t (a3 + t (a4 + t a5)))),
// with 0.5 folded into the a_i and 1/sqrt2, log2(e) into the |x| scalings: 11 plain VALU (abs / neg
// as source modifiers) + v_rcp + v_exp per element, vs 15 + 2 for the textbook order.  Max |error|
// against the exact erf form 3.3e-7 over [-12, 12] (fp32 emulation).
__device__ __forceinline__ float gelu_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.2316418883f, ax, 1.0f));   // p / sqrt2 = 0.3275911 / 1.41421
  float poly = fmaf(0.5307027145f, t, -0.7265760135f);                    // 0.5 * a5, 0.5 * a4
  poly = fmaf(poly, t, 0.7107068705f);                                    // 0.5 * a3
  poly = fmaf(poly, t, -0.142248368f);                                    // 0.5 * a2
  poly = fmaf(poly, t, 0.127414796f);                                     // 0.5 * a1
  poly *= t;
  const float u = ax * 0.84932180028801904272f;                           // sqrt(log2(e) / 2)
  const float e = __builtin_amdgcn_exp2f(-(u * u));                       // exp(-x^2 / 2)
  return fmaf(-ax, poly * e, fmaxf(x, 0.0f));
}

typedef float float2_t __attribute__((ext_vector_type(2)));

// gelu_fast on two values with packed fp32 math (v_pk_fma_f32 / v_pk_mul_f32 carry two values per
// instruction: twice the VALU rate in an epilogue, where no MFMA shares the issue): the same IEEE
// operations in the same order as gelu_fast, so each half is bit-identical to it
__device__ __forceinline__ float2_t gelu_fast2(float2_t x) {
  const float2_t ax = __builtin_elementwise_abs(x);
  const float2_t d = __builtin_elementwise_fma((float2_t)(0.2316418883f), ax, (float2_t)(1.0f));
  const float2_t t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  float2_t poly = __builtin_elementwise_fma((float2_t)(0.5307027145f), t, (float2_t)(-0.7265760135f));
  poly = __builtin_elementwise_fma(poly, t, (float2_t)(0.7107068705f));
  poly = __builtin_elementwise_fma(poly, t, (float2_t)(-0.142248368f));
  poly = __builtin_elementwise_fma(poly, t, (float2_t)(0.127414796f));
  poly = poly * t;
  const float2_t u = ax * (float2_t)(0.84932180028801904272f);
  const float2_t nu2 = -(u * u);
  const float2_t e = {__builtin_amdgcn_exp2f(nu2.x), __builtin_amdgcn_exp2f(nu2.y)};
  const float2_t m = {fmaxf(x.x, 0.0f), fmaxf(x.y, 0.0f)};
  return __builtin_elementwise_fma(-ax, poly * e, m);
}

// GELU on two values with erf from Abramowitz & Stegun 7.1.28, erf(z) = 1 - (1 + a1 z + .. + a6 z^6)^-16
// (|error of erf| <= 3e-7): no exp2, one v_rcp, the 16th power as four packed squarings; 1/sqrt2
// and 2^(1/16) folded into the coefficients so r = 0.5 / p^16 directly and
//   GELU(x) = relu(x) - |x| r.
// 11 packed + 4 plain VALU + 2 v_rcp per pair (gelu_fast2: 10 + 4 + 2 v_rcp + 2 v_exp; the
// transcendentals issue at 8 cycles).  Max |error| against the exact erf form 7.1e-7 over
// [-15, 15] (fp32 emulation) -- twice gelu_fast's, far below an int8 code step or an fp16 ulp.
__device__ __forceinline__ float2_t gelu_r16_2(float2_t x) {
  const float2_t ax = __builtin_elementwise_abs(x);
  float2_t p = __builtin_elementwise_fma((float2_t)(5.6212996640e-06f), ax, (float2_t)(5.1055209009e-05f));
  p = __builtin_elementwise_fma(p, ax, (float2_t)(3.9686137011e-05f));
  p = __builtin_elementwise_fma(p, ax, (float2_t)(3.4227392389e-03f));
  p = __builtin_elementwise_fma(p, ax, (float2_t)(2.2076998457e-02f));
  p = __builtin_elementwise_fma(p, ax, (float2_t)(5.2075163037e-02f));
  p = __builtin_elementwise_fma(p, ax, (float2_t)(1.0442737824e+00f));
  p = p * p;
  p = p * p;
  p = p * p;
  p = p * p;
  const float2_t r = {__builtin_amdgcn_rcpf(p.x), __builtin_amdgcn_rcpf(p.y)};
  const float2_t m = {fmaxf(x.x, 0.0f), fmaxf(x.y, 0.0f)};
  return __builtin_elementwise_fma(-ax, r, m);
}

// gelu_r16_2 on N pairs at once, stage by stage across the pairs: the per-pair form is a chain of
// ~12 dependent packed ops (Horner, four squarings, rcp), which at two waves per SIMD left the VALU
// waiting on each result (the compiler padded the chains with s_nop); N independent chains in
// lockstep fill those slots.  Same operations, same results as gelu_r16_2 per pair.
template <int N>
__device__ __forceinline__ void gelu_r16_n(float2_t (&x)[N]) {
  float2_t ax[N], p[N];
#pragma unroll
  for (int n = 0; n < N; ++n) {
    ax[n] = __builtin_elementwise_abs(x[n]);
    p[n] = __builtin_elementwise_fma((float2_t)(5.6212996640e-06f), ax[n], (float2_t)(5.1055209009e-05f));
  }
#pragma unroll
  for (int n = 0; n < N; ++n) p[n] = __builtin_elementwise_fma(p[n], ax[n], (float2_t)(3.9686137011e-05f));
#pragma unroll
  for (int n = 0; n < N; ++n) p[n] = __builtin_elementwise_fma(p[n], ax[n], (float2_t)(3.4227392389e-03f));
#pragma unroll
  for (int n = 0; n < N; ++n) p[n] = __builtin_elementwise_fma(p[n], ax[n], (float2_t)(2.2076998457e-02f));
#pragma unroll
  for (int n = 0; n < N; ++n) p[n] = __builtin_elementwise_fma(p[n], ax[n], (float2_t)(5.2075163037e-02f));
#pragma unroll
  for (int n = 0; n < N; ++n) p[n] = __builtin_elementwise_fma(p[n], ax[n], (float2_t)(1.0442737824e+00f));
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int n = 0; n < N; ++n) p[n] = p[n] * p[n];
#pragma unroll
  for (int n = 0; n < N; ++n) {
    const float2_t r = {__builtin_amdgcn_rcpf(p[n].x), __builtin_amdgcn_rcpf(p[n].y)};
    const float2_t m = {fmaxf(x[n].x, 0.0f), fmaxf(x[n].y, 0.0f)};
    x[n] = __builtin_elementwise_fma(-ax[n], r, m);
  }
}

// clamp(round_half_even(v / s), -128, 127) with the reference's CORRECTLY ROUNDED quotient (fq_vit
// quantizer/uniform.py:31-36), branch-free.  q0 = fl(v * inv) with inv = fl(1/s) can be ~1.5 ulp
// off v/s -- outside Markstein's precondition (a faithful q) -- so one correction is not provably
// fl(v / s) (it failed on none of ~6e6 adversarial operands, but a quotient within ~2^-22 ulp of a
// rounding midpoint could flip).  The first correction q1 = fl(q0 + fl(v - s q0) inv) is faithful
// (error ~0.5 ulp + 2^-23 ulp); the second, q2 = fl(q1 + (v - s q1) inv) with an EXACT remainder,
// is fl(v / s) by Markstein's theorem (inv within half an ulp of 1/s, round to nearest, no
// overflow / subnormal quotient in the quantiser's range).  Four FMAs, no division, no branch;
// tools/check_markstein.py checks both forms against exact rational division.  Non-finite q0
// (overflow) keeps q0, so the clamp sees +-inf as the true division would.
__device__ __forceinline__ float q8_exact(float v, float s, float inv) {
  const float q = v * inv;
  const float q1 = __builtin_fmaf(__builtin_fmaf(-q, s, v), inv, q);
  const float q2 = __builtin_fmaf(__builtin_fmaf(-q1, s, v), inv, q1);
  const float r = __builtin_rintf(__builtin_isfinite(q) ? q2 : q);
  return fminf(fmaxf(r, -128.f), 127.f);
}

// q8_exact on a packed pair (v_pk_mul / v_pk_fma: the same IEEE operations, so each half is
// bit-identical to q8_exact), with |v| first clamped to lim (>= 128.5 s: every larger |v| gives the
// same saturated code, and the quotients stay finite -- no isfinite select) and the code clamp on
// v_med3.  Returns the codes as floats in [-128, 127].
__device__ __forceinline__ float2_t q8_exact2(float2_t v, float s, float inv, float lim) {
  v = float2_t{__builtin_amdgcn_fmed3f(v.x, -lim, lim), __builtin_amdgcn_fmed3f(v.y, -lim, lim)};
  const float2_t sv = (float2_t)(s), iv = (float2_t)(inv);
  const float2_t q = v * iv;
  const float2_t q1 = __builtin_elementwise_fma(__builtin_elementwise_fma(-q, sv, v), iv, q);
  const float2_t q2 = __builtin_elementwise_fma(__builtin_elementwise_fma(-q1, sv, v), iv, q1);
  return float2_t{__builtin_amdgcn_fmed3f(__builtin_rintf(q2.x), -128.f, 127.f),
                  __builtin_amdgcn_fmed3f(__builtin_rintf(q2.y), -128.f, 127.f)};
}
// round_half_even(v * fl(1/s)), NOT clamped: the quotient by one reciprocal multiply (<= 1.5 ulp from
// v / s, so a code differs from the exact quotient's only within ~1e-7 of a rounding midpoint); the
// clamp to [-128, 127] is q8_pack4's saturating conversion.  For the GELU epilogues only: the GELU in
// front of it is itself an approximation (|error| 7.1e-7, gelu_r16_2), so the exact quotient of
// q8_exact2 buys nothing there; 3 VALU per pair instead of 11.
__device__ __forceinline__ float2_t q8_recip2(float2_t v, float inv) {
  const float2_t q = v * (float2_t)(inv);
  return float2_t{__builtin_rintf(q.x), __builtin_rintf(q.y)};
}
// four codes (integer floats) -> their int8 bytes in one dword: v_cvt_pk_u8_f32 of code + 128 per
// byte, then the sign bit flipped back per byte.  The conversion saturates to [0, 255] (and rounds to
// nearest even; gfx950, tools/probe_cvt_u8.hip -> profiles/r6_probe_cvt_u8.log), so codes outside
// [-128, 127] come out clamped
__device__ __forceinline__ uint32_t q8_pack4(float c0, float c1, float c2, float c3) {
  uint32_t w = __builtin_amdgcn_cvt_pk_u8_f32(c0 + 128.f, 0, 0u);
  w = __builtin_amdgcn_cvt_pk_u8_f32(c1 + 128.f, 1, w);
  w = __builtin_amdgcn_cvt_pk_u8_f32(c2 + 128.f, 2, w);
  w = __builtin_amdgcn_cvt_pk_u8_f32(c3 + 128.f, 3, w);
  return w ^ 0x80808080u;
}

// max over the four 16-lane rows of a wave at the same column (lane ^ 16, ^ 32, ^ 48): two VALU
// permlane swaps (v_permlane16_swap / v_permlane32_swap of a value with itself: results 0 / 1 hold
// the row pair's two values) instead of three LDS bpermutes
__device__ __forceinline__ float max_rows4(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(int, v), __builtin_bit_cast(int, v), false, false);
  v = fmaxf(__builtin_bit_cast(float, (int)a[0]), __builtin_bit_cast(float, (int)a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(int, v), __builtin_bit_cast(int, v), false, false);
  return fmaxf(__builtin_bit_cast(float, (int)b[0]), __builtin_bit_cast(float, (int)b[1]));
}

// sum over the 64 lanes on the VALU: DPP within 16-lane rows (quad_perm xor 1, xor 2, then the
// half-row and row mirrors -- value-equivalent to xor 4 / xor 8 once the smaller groups agree),
// then v_permlane16_swap / v_permlane32_swap across rows; no LDS round trips
__device__ __forceinline__ float wave_sum_valu(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, true));
  const auto a = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(int, v), __builtin_bit_cast(int, v), false, false);
  v = __builtin_bit_cast(float, (int)a[0]) + __builtin_bit_cast(float, (int)a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(int, v), __builtin_bit_cast(int, v), false, false);
  return __builtin_bit_cast(float, (int)b[0]) + __builtin_bit_cast(float, (int)b[1]);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware remap of a 1-D workgroup id: consecutive logical ids share an XCD
// (MI355X deals workgroups round-robin over 8 XCDs; speed only, never correctness).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, k = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}


template <int N, typename F, int I = 0>
__device__ __forceinline__ void static_for(F&& f) {   // f(integral_constant<int, 0..N-1>)
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, F, I + 1>(static_cast<F&&>(f));
  }
}

}  // namespace samq

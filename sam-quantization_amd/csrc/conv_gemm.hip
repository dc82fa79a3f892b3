// Implicit-GEMM convolutions of the encoder's patch embedding and neck on fp16 MFMA.
//
// Replaces the last vendor-BLAS / im2col pieces of the encoder forward:
//  * PatchEmbed: Conv2d(3, C, 16, stride 16) + pos_embed add (segment_anything/modeling/
//    image_encoder.py:411-442, :108-110): the 16x16 patches are gathered straight from the NCHW
//    image into the A operand (no im2col copy), bias and the absolute position embedding are
//    added in the fp32 epilogue, the fp32 residual stream is written directly;
//  * the same from RAW uint8 pixels (SamPredictor.set_image, predictor.py:34-90): the gather
//    applies Sam.preprocess (sam.py:164-174) itself -- (pixel - mean[c]) / std[c], and the zero
//    padding of an h x w image (h, w <= img_size) to the square input -- so the normalised fp32
//    image never exists in HBM (3 MB of uint8 read instead of 12 MB of fp32 written + read);
//  * neck conv 1x1 (C -> 256, no bias, image_encoder.py:88-104): A = the fp32 residual tokens,
//    converted to fp16 while staged (the reference runs the neck in fp16);
//  * neck conv 3x3 pad 1 (256 -> 256, no bias): A gathered from the NHWC fp16 feature map with
//    zero padding; the weight is pre-permuted to (n, ky, kx, c) so a 64-byte A chunk is 32
//    contiguous channels of one tap.
// Small GEMMs (0.3 % of the encoder FLOPs): a plain 128x128x32 LDS double-buffered tile on
// v_mfma_f32_32x32x16_f16, 4 waves of 64x64, fp32 accumulation.
#include "common.h"

namespace samq {

enum { CG_PATCH = 0, CG_1X1_F32 = 1, CG_3X3 = 2, CG_PATCH_U8 = 3 };

struct ConvArgs {
  const void* x;        // PATCH: image f16 [B][Cin][G*P][G*P]; 1X1_F32: f32 [M][K]; 3X3: f16 [B][G][G][Cin]
  const _Float16* w;    // f16 [N][K]  (3X3: K ordered (ky, kx, c))
  const float* bias;    // PATCH: f32 [N] or null
  const float* pos;     // PATCH: f32 [G*G][N] or null
  void* out;            // PATCH: f32 [M][N]; else f16 [M][N]
  int M, N, K;
  int G, P, Cin;
  const float* mean;    // PATCH_U8: per-channel pixel mean / std (Sam.pixel_mean / pixel_std)
  const float* stdv;
  int ih, iw;           // PATCH_U8: real image rows / columns (<= G*P; the rest is zero padding)
};

// one normalised pixel of a raw uint8 NCHW image (Sam.preprocess), 0 in the padding
__device__ __forceinline__ float pixel_norm(const ConvArgs& a, const uint8_t* img, int b, int c, int y, int x) {
  if (y >= a.ih || x >= a.iw) return 0.f;
  const float v = (float)img[(((int64_t)b * a.Cin + c) * a.ih + y) * a.iw + x];
  return (v - a.mean[c]) / a.stdv[c];
}

template <int MODE>
__device__ __forceinline__ half8_t conv_load_a(const ConvArgs& a, int t, int k) {
  // t: token index (< M), k: first of 8 consecutive reduction indices
  const int gg = a.G * a.G;
  const int b = t / gg, gy = (t / a.G) % a.G, gx = t % a.G;
  if (MODE == CG_PATCH_U8) {
    const int pp = a.P * a.P;
    const int c = k / pp, rem = k - c * pp, kh = rem / a.P, kw = rem - kh * a.P;
    const uint8_t* img = (const uint8_t*)a.x;
    half8_t r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (_Float16)pixel_norm(a, img, b, c, gy * a.P + kh, gx * a.P + kw + j);
    return r;
  } else if (MODE == CG_PATCH) {
    const int pp = a.P * a.P;
    const int c = k / pp, rem = k - c * pp, kh = rem / a.P, kw = rem - kh * a.P;
    const int side = a.G * a.P;
    const _Float16* src = (const _Float16*)a.x + (((int64_t)b * a.Cin + c) * side + gy * a.P + kh) * side +
                          gx * a.P + kw;
    return *(const half8_t*)src;
  } else if (MODE == CG_1X1_F32) {
    const float4_t* src = (const float4_t*)((const float*)a.x + (int64_t)t * a.K + k);
    const float4_t v0 = src[0], v1 = src[1];
    return half8_t{(_Float16)v0[0], (_Float16)v0[1], (_Float16)v0[2], (_Float16)v0[3],
                   (_Float16)v1[0], (_Float16)v1[1], (_Float16)v1[2], (_Float16)v1[3]};
  } else {
    const int tap = k / a.Cin, c0 = k - tap * a.Cin;
    const int sy = gy + tap / 3 - 1, sx = gx + tap % 3 - 1;
    if (sy < 0 || sy >= a.G || sx < 0 || sx >= a.G) return half8_t{};
    return *(const half8_t*)((const _Float16*)a.x + (((int64_t)b * a.G + sy) * a.G + sx) * a.Cin + c0);
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void conv_gemm_kernel(ConvArgs a) {
  constexpr int BM = 128, BN = 128, BK = 32;
  constexpr int PITCH = BK * 2 + 16;   // 80-byte LDS rows: the 32 row reads of a fragment spread over banks
  constexpr int BUF = (BM + BN) * PITCH;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = a.N / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (bid / tiles_n) * BM;
  const int n0 = (bid % tiles_n) * BN;
  const int kt_count = a.K / BK;

  // staging: chunk c = tid + 256 j (j = 0, 1) -> row c / 4, 8 k-values at (c % 4) * 8
  half8_t ra[2], rb[2];
  auto load = [&](int kt) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = tid + 256 * j;
      const int row = c >> 2, k = kt * BK + (c & 3) * 8;
      int t = m0 + row;
      t = t < a.M ? t : a.M - 1;
      ra[j] = conv_load_a<MODE>(a, t, k);
      rb[j] = *(const half8_t*)(a.w + (int64_t)(n0 + row) * a.K + k);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = tid + 256 * j;
      const int row = c >> 2, off = (c & 3) * 16;
      *(half8_t*)(smem + buf * BUF + row * PITCH + off) = ra[j];
      *(half8_t*)(smem + buf * BUF + (BM + row) * PITCH + off) = rb[j];
    }
  };

  float16_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][t][r] = 0.f;

  const int hsel = lane >> 5;
  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < kt_count; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < kt_count) load(kt + 1);
    const char* base = smem + buf * BUF;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      half8_t af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[i] = *(const half8_t*)(base + (wm * 64 + i * 32 + (lane & 31)) * PITCH + (s * 16 + 8 * hsel) * 2);
#pragma unroll
      for (int t = 0; t < 2; ++t)
        bf[t] = *(const half8_t*)(base + (BM + wn * 64 + t * 32 + (lane & 31)) * PITCH + (s * 16 + 8 * hsel) * 2);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i], bf[t], acc[i][t], 0, 0, 0);
    }
    if (kt + 1 < kt_count) {
      store(buf ^ 1);   // the other buffer was last read before the previous barrier
      __syncthreads();
    }
  }

  // epilogue: lane owns column (lane & 31) of each 32x32 tile, 16 rows
  const int gg = a.G * a.G;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int col = n0 + wn * 64 + t * 32 + (lane & 31);
    const float bcol = ((MODE == CG_PATCH || MODE == CG_PATCH_U8) && a.bias) ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hsel;
        if (row >= a.M) continue;
        float v = acc[i][t][r];
        if (MODE == CG_PATCH || MODE == CG_PATCH_U8) {
          v += bcol;
          if (a.pos) v += a.pos[(int64_t)(row % gg) * a.N + col];
          ((float*)a.out)[(int64_t)row * a.N + col] = v;
        } else {
          ((_Float16*)a.out)[(int64_t)row * a.N + col] = (_Float16)v;
        }
      }
    }
  }
}

// fp32 patch embedding (the W4A8 engine: its first int8 quantiser sits right behind it, so the
// embedding keeps the reference's fp32 arithmetic): the same implicit GEMM on
// v_mfma_f32_32x32x2_f32, 128x128x16 tiles, fp32 image / weight / accumulation.
template <bool U8>
__global__ __launch_bounds__(256) void patch_embed_f32_kernel(ConvArgs a) {
  constexpr int BM = 128, BN = 128, BK = 16;
  constexpr int PITCH = BK + 1;   // floats; odd pitch spreads a fragment's 32 rows over the banks
  constexpr int BUF = (BM + BN) * PITCH;
  __shared__ float smem[2 * BUF];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = a.N / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (bid / tiles_n) * BM;
  const int n0 = (bid % tiles_n) * BN;
  const int kt_count = a.K / BK;
  const int gg = a.G * a.G, pp = a.P * a.P, side = a.G * a.P;

  // staging: float4 chunk c = tid + 256 j (j = 0, 1) -> row c / 4, 4 k-values at (c % 4) * 4
  float4_t ra[2], rb[2];
  auto load = [&](int kt) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = tid + 256 * j;
      const int row = c >> 2, k = kt * BK + (c & 3) * 4;
      int t = m0 + row;
      t = t < a.M ? t : a.M - 1;
      const int b = t / gg, gy = (t / a.G) % a.G, gx = t % a.G;
      const int ci = k / pp, rem = k - ci * pp, kh = rem / a.P, kw = rem - kh * a.P;
      if (U8) {
#pragma unroll
        for (int e = 0; e < 4; ++e) ra[j][e] = pixel_norm(a, (const uint8_t*)a.x, b, ci, gy * a.P + kh, gx * a.P + kw + e);
      } else {
        ra[j] = *(const float4_t*)((const float*)a.x + (((int64_t)b * a.Cin + ci) * side + gy * a.P + kh) * side +
                                   gx * a.P + kw);
      }
      rb[j] = *(const float4_t*)((const float*)a.w + (int64_t)(n0 + row) * a.K + k);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = tid + 256 * j;
      const int row = c >> 2, off = (c & 3) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        smem[buf * BUF + row * PITCH + off + e] = ra[j][e];
        smem[buf * BUF + (BM + row) * PITCH + off + e] = rb[j][e];
      }
    }
  };

  float16_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][t][r] = 0.f;

  const int hsel = lane >> 5;
  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < kt_count; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < kt_count) load(kt + 1);
    const float* base = smem + buf * BUF;
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) {
      float af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = base[(wm * 64 + i * 32 + (lane & 31)) * PITCH + 2 * s + hsel];
#pragma unroll
      for (int t = 0; t < 2; ++t) bf[t] = base[(BM + wn * 64 + t * 32 + (lane & 31)) * PITCH + 2 * s + hsel];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[t], acc[i][t], 0, 0, 0);
    }
    if (kt + 1 < kt_count) {
      store(buf ^ 1);
      __syncthreads();
    }
  }

#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int col = n0 + wn * 64 + t * 32 + (lane & 31);
    const float bcol = a.bias ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hsel;
        if (row >= a.M) continue;
        float v = acc[i][t][r] + bcol;
        if (a.pos) v += a.pos[(int64_t)(row % gg) * a.N + col];
        ((float*)a.out)[(int64_t)row * a.N + col] = v;
      }
    }
  }
}

// fp32-accurate patch embedding on fp16 MFMA (the W4A8 engine: its first int8 quantiser sits
// right behind it).  Every fp32 operand x is split as x = hi + lo' 2^-11 with hi = fp16(x),
// lo' = fp16((x - hi) 2^11) (lo' is as large as x itself: no fp16 subnormals for small weights);
// x.w = hi_x hi_w + 2^-11 (hi_x lo'_w + lo'_x hi_w) + O(2^-22 |x w|): two accumulators, three
// v_mfma_f32_32x32x16_f16 per fragment pair instead of eight v_mfma_f32_32x32x2_f32 (x 16 the
// FLOP rate).  Same 128x128 tiles / 4 waves / LDS double buffer as conv_gemm_kernel, with hi and
// lo' planes of A and B staged side by side.
__device__ __forceinline__ void split8(const float (&v)[8], half8_t& hi, half8_t& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    hi[j] = (_Float16)v[j];
    lo[j] = (_Float16)((v[j] - (float)hi[j]) * 2048.0f);
  }
}

template <bool U8>
__global__ __launch_bounds__(256, 2) void patch_embed_x3_kernel(ConvArgs a) {
  constexpr int BM = 128, BN = 128, BK = 32;
  constexpr int PITCH = BK * 2 + 16;           // 80-byte LDS rows (conv_gemm_kernel's bank spread)
  constexpr int PLANE = 128 * PITCH;
  constexpr int BUF = 4 * PLANE;               // A hi | A lo' | B hi | B lo'
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = a.N / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (bid / tiles_n) * BM;
  const int n0 = (bid % tiles_n) * BN;
  const int kt_count = a.K / BK;
  const int gg = a.G * a.G, pp = a.P * a.P, side = a.G * a.P;
  const float* wf = (const float*)a.w;

  // staging: chunk c = tid + 256 j -> row c / 4, 8 k-values at (c % 4) * 8 (one patch row segment)
  float ra[2][8], rb[2][8];
  auto load = [&](int kt) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = tid + 256 * j;
      const int row = c >> 2, k = kt * BK + (c & 3) * 8;
      int t = m0 + row;
      t = t < a.M ? t : a.M - 1;
      const int b = t / gg, gy = (t / a.G) % a.G, gx = t % a.G;
      const int ci = k / pp, rem = k - ci * pp, kh = rem / a.P, kw = rem - kh * a.P;
      if (U8) {
#pragma unroll
        for (int e = 0; e < 8; ++e) ra[j][e] = pixel_norm(a, (const uint8_t*)a.x, b, ci, gy * a.P + kh, gx * a.P + kw + e);
      } else {
        const float4_t* src = (const float4_t*)((const float*)a.x + (((int64_t)b * a.Cin + ci) * side + gy * a.P + kh) *
                                                side + gx * a.P + kw);
        const float4_t v0 = src[0], v1 = src[1];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ra[j][e] = v0[e];
          ra[j][4 + e] = v1[e];
        }
      }
      const float4_t* ws = (const float4_t*)(wf + (int64_t)(n0 + row) * a.K + k);
      const float4_t w0 = ws[0], w1 = ws[1];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        rb[j][e] = w0[e];
        rb[j][4 + e] = w1[e];
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = tid + 256 * j;
      const int row = c >> 2, off = (c & 3) * 16;
      half8_t h, l;
      split8(ra[j], h, l);
      *(half8_t*)(smem + buf * BUF + row * PITCH + off) = h;
      *(half8_t*)(smem + buf * BUF + PLANE + row * PITCH + off) = l;
      split8(rb[j], h, l);
      *(half8_t*)(smem + buf * BUF + 2 * PLANE + row * PITCH + off) = h;
      *(half8_t*)(smem + buf * BUF + 3 * PLANE + row * PITCH + off) = l;
    }
  };

  float16_t acc[2][2], accx[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][t][r] = accx[i][t][r] = 0.f;

  const int hsel = lane >> 5;
  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < kt_count; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < kt_count) load(kt + 1);
    const char* base = smem + buf * BUF;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      half8_t ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int o = (wm * 64 + i * 32 + (lane & 31)) * PITCH + (s * 16 + 8 * hsel) * 2;
        ah[i] = *(const half8_t*)(base + o);
        al[i] = *(const half8_t*)(base + PLANE + o);
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int o = (wn * 64 + t * 32 + (lane & 31)) * PITCH + (s * 16 + 8 * hsel) * 2;
        bh[t] = *(const half8_t*)(base + 2 * PLANE + o);
        bl[t] = *(const half8_t*)(base + 3 * PLANE + o);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[t], acc[i][t], 0, 0, 0);
          accx[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[t], accx[i][t], 0, 0, 0);
          accx[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[t], accx[i][t], 0, 0, 0);
        }
    }
    if (kt + 1 < kt_count) {
      store(buf ^ 1);   // the other buffer was last read before the previous barrier
      __syncthreads();
    }
  }

#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int col = n0 + wn * 64 + t * 32 + (lane & 31);
    const float bcol = a.bias ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hsel;
        if (row >= a.M) continue;
        float v = __builtin_fmaf(accx[i][t][r], 1.0f / 2048.0f, acc[i][t][r]) + bcol;
        if (a.pos) v += a.pos[(int64_t)(row % gg) * a.N + col];
        ((float*)a.out)[(int64_t)row * a.N + col] = v;
      }
    }
  }
}

template <int MODE>
static int conv_launch(const ConvArgs& a, hipStream_t stream) {
  const int nwg = ((a.M + 127) / 128) * (a.N / 128);
  hipLaunchKernelGGL((conv_gemm_kernel<MODE>), dim3(nwg), dim3(256), 0, stream, a);
  SAMQ_LAUNCH_CHECK("conv_gemm launch");
  return SAMQ_OK;
}

}  // namespace samq

using namespace samq;

extern "C" int samq_patch_embed(const void* img, const void* weight, const float* bias, const float* pos, float* out,
                                int B, int Cin, int img_size, int patch, int N, hipStream_t stream) {
  if (B == 0) return SAMQ_OK;   // empty batch: no work, data pointers may be null
  SAMQ_REQUIRE(img && weight && out, SAMQ_ERR_INVALID, "patch_embed: null pointer");
  SAMQ_REQUIRE(B > 0 && Cin > 0 && patch > 0 && img_size % patch == 0, SAMQ_ERR_INVALID,
               "patch_embed: image size must be a multiple of the patch size");
  SAMQ_REQUIRE(patch % 8 == 0 && (Cin * patch * patch) % 32 == 0, SAMQ_ERR_UNSUPPORTED,
               "patch_embed: patch must be a multiple of 8 and Cin*patch^2 a multiple of 32");
  SAMQ_REQUIRE(N % 128 == 0, SAMQ_ERR_UNSUPPORTED, "patch_embed: embed dim must be a multiple of 128");
  SAMQ_REQUIRE(((uintptr_t)img & 15) == 0 && ((uintptr_t)weight & 15) == 0, SAMQ_ERR_INVALID,
               "patch_embed: image and weight must be 16-byte aligned");
  const int g = img_size / patch;
  ConvArgs a{img, (const _Float16*)weight, bias, pos, out, B * g * g, N, Cin * patch * patch, g, patch, Cin};
  return conv_launch<CG_PATCH>(a, stream);
}

extern "C" int samq_conv1x1_f32(const float* x, const void* weight, void* out, int64_t M, int N, int K,
                                hipStream_t stream) {
  if (M == 0) return SAMQ_OK;   // empty batch: no work, data pointers may be null
  SAMQ_REQUIRE(x && weight && out, SAMQ_ERR_INVALID, "conv1x1: null pointer");
  SAMQ_REQUIRE(M > 0 && M < (int64_t)1 << 31, SAMQ_ERR_INVALID, "conv1x1: bad M");
  SAMQ_REQUIRE(K % 32 == 0 && N % 128 == 0, SAMQ_ERR_UNSUPPORTED,
               "conv1x1: K must be a multiple of 32 and N of 128");
  SAMQ_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)weight & 15) == 0, SAMQ_ERR_INVALID,
               "conv1x1: operands must be 16-byte aligned");
  ConvArgs a{x, (const _Float16*)weight, nullptr, nullptr, out, (int)M, N, K, 1, 1, K};
  return conv_launch<CG_1X1_F32>(a, stream);
}

extern "C" int samq_conv3x3_nhwc(const void* x, const void* weight, void* out, int B, int G, int Cin, int N,
                                 hipStream_t stream) {
  if (B == 0) return SAMQ_OK;   // empty batch: no work, data pointers may be null
  SAMQ_REQUIRE(x && weight && out, SAMQ_ERR_INVALID, "conv3x3: null pointer");
  SAMQ_REQUIRE(B > 0 && G > 0, SAMQ_ERR_INVALID, "conv3x3: bad shape");
  SAMQ_REQUIRE(Cin % 32 == 0 && N % 128 == 0, SAMQ_ERR_UNSUPPORTED,
               "conv3x3: Cin must be a multiple of 32 and N of 128");
  SAMQ_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)weight & 15) == 0, SAMQ_ERR_INVALID,
               "conv3x3: operands must be 16-byte aligned");
  ConvArgs a{x, (const _Float16*)weight, nullptr, nullptr, out, B * G * G, N, 9 * Cin, G, 1, Cin};
  return conv_launch<CG_3X3>(a, stream);
}

extern "C" int samq_patch_embed_f32(const float* img, const float* weight, const float* bias, const float* pos,
                                    float* out, int B, int Cin, int img_size, int patch, int N, hipStream_t stream) {
  if (B == 0) return SAMQ_OK;   // empty batch: no work, data pointers may be null
  SAMQ_REQUIRE(img && weight && out, SAMQ_ERR_INVALID, "patch_embed_f32: null pointer");
  SAMQ_REQUIRE(B > 0 && Cin > 0 && patch > 0 && img_size % patch == 0, SAMQ_ERR_INVALID,
               "patch_embed_f32: image size must be a multiple of the patch size");
  SAMQ_REQUIRE(patch % 4 == 0 && (Cin * patch * patch) % 16 == 0, SAMQ_ERR_UNSUPPORTED,
               "patch_embed_f32: patch must be a multiple of 4 and Cin*patch^2 a multiple of 16");
  SAMQ_REQUIRE(N % 128 == 0, SAMQ_ERR_UNSUPPORTED, "patch_embed_f32: embed dim must be a multiple of 128");
  SAMQ_REQUIRE(((uintptr_t)img & 15) == 0 && ((uintptr_t)weight & 15) == 0, SAMQ_ERR_INVALID,
               "patch_embed_f32: image and weight must be 16-byte aligned");
  const int g = img_size / patch;
  ConvArgs a{img, (const _Float16*)weight, bias, pos, out, B * g * g, N, Cin * patch * patch, g, patch, Cin};
  const int nwg = ((a.M + 127) / 128) * (a.N / 128);
  if (patch % 8 == 0 && a.K % 32 == 0)   // split-fp16 MFMA form (16-byte image rows of 8 pixels)
    hipLaunchKernelGGL(patch_embed_x3_kernel<false>, dim3(nwg), dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL(patch_embed_f32_kernel<false>, dim3(nwg), dim3(256), 0, stream, a);
  SAMQ_LAUNCH_CHECK("patch_embed_f32 launch");
  return SAMQ_OK;
}

extern "C" int samq_patch_embed_u8(const uint8_t* img, int h, int w, const float* pixel_mean, const float* pixel_std,
                                   const void* weight, int weight_f32, const float* bias, const float* pos, float* out,
                                   int B, int Cin, int img_size, int patch, int N, hipStream_t stream) {
  if (B == 0) return SAMQ_OK;   // empty batch: no work, data pointers may be null
  SAMQ_REQUIRE(img && pixel_mean && pixel_std && weight && out, SAMQ_ERR_INVALID, "patch_embed_u8: null pointer");
  SAMQ_REQUIRE(B > 0 && Cin > 0 && patch > 0 && img_size % patch == 0, SAMQ_ERR_INVALID,
               "patch_embed_u8: image size must be a multiple of the patch size");
  SAMQ_REQUIRE(h > 0 && w > 0 && h <= img_size && w <= img_size, SAMQ_ERR_INVALID,
               "patch_embed_u8: the image must fit the square encoder input");
  SAMQ_REQUIRE(N % 128 == 0, SAMQ_ERR_UNSUPPORTED, "patch_embed_u8: embed dim must be a multiple of 128");
  SAMQ_REQUIRE(((uintptr_t)weight & 15) == 0, SAMQ_ERR_INVALID, "patch_embed_u8: weight must be 16-byte aligned");
  const int g = img_size / patch;
  ConvArgs a{img, (const _Float16*)weight, bias, pos, out, B * g * g, N, Cin * patch * patch, g, patch, Cin,
             pixel_mean, pixel_std, h, w};
  const int nwg = ((a.M + 127) / 128) * (a.N / 128);
  if (weight_f32) {
    SAMQ_REQUIRE(patch % 4 == 0 && (Cin * patch * patch) % 16 == 0, SAMQ_ERR_UNSUPPORTED,
                 "patch_embed_u8: patch must be a multiple of 4 and Cin*patch^2 a multiple of 16");
    if (patch % 8 == 0 && a.K % 32 == 0)
      hipLaunchKernelGGL(patch_embed_x3_kernel<true>, dim3(nwg), dim3(256), 0, stream, a);
    else
      hipLaunchKernelGGL(patch_embed_f32_kernel<true>, dim3(nwg), dim3(256), 0, stream, a);
    SAMQ_LAUNCH_CHECK("patch_embed_u8 (f32) launch");
    return SAMQ_OK;
  }
  SAMQ_REQUIRE(patch % 8 == 0 && (Cin * patch * patch) % 32 == 0, SAMQ_ERR_UNSUPPORTED,
               "patch_embed_u8: patch must be a multiple of 8 and Cin*patch^2 a multiple of 32");
  return conv_launch<CG_PATCH_U8>(a, stream);
}

// W4A16 GEMM for GPTQ-packed int4 weights on gfx950 fp16 MFMA.
//
// Replaces the reference's Triton `matmul4_kernel` + `triton_matmul4`
// (gptq_triton/quant_linear.py:231-352, 355-437):  C[M,N] = A[M,K] . W[K,N] (+bias, ...)
// with W[k,n] = s[g,n] * (q[k,n] - zp[g,n]),  q = (qweight[k/8,n] >> 4(k%8)) & 15,
// zp = ((qzeros[g,n/8] >> 4(n%8)) & 15) + 1.
//
// Numerics (deliberately NOT the reference's fp16 dequant `fp16(q*s) - fp16(zp*s)`, which
// is the dominant error of the reference path): the MFMA multiplies
// fp16 activations by the EXACT small integers (q - zp) in [-16, 15], accumulates in fp32,
// and applies the per-channel scale in the fp32 epilogue (groupsize == K).  With groups
// (groupsize < K) the integer is scaled once, in fp16, per group: fp16((q - zp) * s).
//
// Design (MI355X-first, not a translation of the Triton tiling):
//  * weights are repacked once at load (samq_w4_repack) into MFMA-fragment order: one
//    dwordx4 per lane holds the 4 k16-steps of its B column for a 64-deep K tile, with the
//    nibbles interleaved so that ((w >> 4i) & 0x000F000F) | 0x64006400 is directly the fp16
//    pair (1024+q[2i], 1024+q[2i+1]) -> 7 VALU ops unpack 8 weights, 4 v_pk_add_f16 remove
//    the zero point.  B never touches LDS: each wave streams its own fragments from L2.
//  * A is staged global->LDS with global_load_lds_dwordx4 (no VGPR round trip), double
//    buffered, XOR-swizzled on the SOURCE address (LDS image lane-linear) so the
//    ds_read_b128 fragment reads of v_mfma_f32_32x32x16_f16 are bank-conflict free.
//  * wave tiles are >=128 rows (except small fallback configs) so the in-register unpack of
//    each B word is amortised over >=4 MFMAs (VALU:MFMA issue ~1:3).
//  * fused epilogues: +bias, +bias+GELU(erf), and fp32 residual accumulate (x += y) so the
//    residual stream never takes an extra HBM round trip.
//  * XCD-aware bijective blockIdx remap: consecutive tiles (same A rows) share an L2.
#include "common.h"

#include <cstdio>

// packed-weight layout produced by samq_w4_repack (and expected by samq_w4a16_gemm)
#ifndef SAMQ_W4_LAYOUT
#define SAMQ_W4_LAYOUT 1
#endif

namespace samq {

// ------------------------------------------------------------------ repack
// packed word index ((nt * (K/64) + kb) * 64 + lane) * 4 + s   holds column n = nt*32 + (lane&31),
// k = kb*64 + 16*s + 8*(lane>>5) + {0..7}, nibble order [k0,k2,k4,k6 | k1,k3,k5,k7].
// LAYOUT 2 (v_mfma_f32_16x16x32_f16 fragments): word w of lane l in block (nt, kb) holds column
// nt*32 + 16*(w>>1) + (l&15), k = kb*64 + 32*(w&1) + 8*(l>>4) + {0..7}; same nibble interleave.
// LAYOUT 3 (int8 MFMA fragments of v_mfma_i32_32x32x32_i8, used by the W4A8 GEMM in gemm_i8.hip):
// 2-KiB blocks (nt, kb) over 128-deep K tiles, two 1-KiB pieces p; word w of lane l in piece p
// holds column nt*32 + (l&31), k = kb*128 + 32*(2p + (w>>1)) + 16*(l>>5) + 8*(w&1) + {0..7} with
// nibble order [k0,k4,k1,k5,k2,k6,k3,k7], so (w & 0x0F0F0F0F) are the bytes k0..k3 and
// ((w >> 4) & 0x0F0F0F0F) the bytes k4..k7.
template <int LAYOUT>
__global__ void w4_repack_kernel(const uint32_t* __restrict__ qweight, uint32_t* __restrict__ out,
                                 int K, int N) {
  const int64_t total = (int64_t)K * N / 8;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int s = idx & 3;
    const int lane = (idx >> 2) & 63;
    if (LAYOUT == 3) {
      const int p = (idx >> 8) & 1;
      const int64_t blk = idx >> 9;            // nt * (K/128) + kb
      const int kbs = K / 128;
      const int kb = (int)(blk % kbs);
      const int nt = (int)(blk / kbs);
      const int n = nt * 32 + (lane & 31);
      const int k0 = kb * 128 + 32 * (2 * p + (s >> 1)) + 16 * (lane >> 5) + 8 * (s & 1);
      const uint32_t w = qweight[(int64_t)(k0 >> 3) * N + n];
      uint32_t o = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        o |= ((w >> (4 * i)) & 0xFu) << (8 * i);            // q[i]   -> byte i, low nibble
        o |= ((w >> (4 * i + 16)) & 0xFu) << (8 * i + 4);   // q[i+4] -> byte i, high nibble
      }
      out[idx] = o;
      continue;
    }
    const int64_t blk = idx >> 8;             // nt * (K/64) + kb
    const int kbs = K / 64;
    const int kb = (int)(blk % kbs);
    const int nt = (int)(blk / kbs);
    const int n = LAYOUT == 2 ? nt * 32 + 16 * (s >> 1) + (lane & 15) : nt * 32 + (lane & 31);
    const int k0 = LAYOUT == 2 ? kb * 64 + 32 * (s & 1) + 8 * (lane >> 4) : kb * 64 + 16 * s + 8 * (lane >> 5);
    const uint32_t w = qweight[(int64_t)(k0 >> 3) * N + n];
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o |= ((w >> (8 * i)) & 0xFu) << (4 * i);             // q[2i]   -> bits 4i
      o |= ((w >> (8 * i + 4)) & 0xFu) << (16 + 4 * i);    // q[2i+1] -> bits 16+4i
    }
    out[idx] = o;
  }
}

// ------------------------------------------------------------------ GEMM
template <int BM, int BN, int WAVES_M, int WAVES_N, int EPI, bool GROUPED, int VAR = 1>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N)
void w4a16_gemm_kernel(const _Float16* __restrict__ A, int64_t lda,
                       const u32x4* __restrict__ Wp,
                       const _Float16* __restrict__ scales,
                       const uint32_t* __restrict__ qzeros,
                       const _Float16* __restrict__ bias,
                       void* __restrict__ Cout, int64_t ldc,
                       int M, int N, int K, int groupsize) {
  constexpr int NW = WAVES_M * WAVES_N;
  constexpr int WM = BM / WAVES_M;
  constexpr int WN = BN / WAVES_N;
  constexpr int TM = WM / 32;
  constexpr int TN = WN / 32;
  constexpr int BK = 64;
  constexpr int ROWB = BK * 2;                 // 128 bytes per A row in LDS
  constexpr int TILE_BYTES = BM * ROWB;
  constexpr int GLDS_PER_WAVE = BM / 8 / NW;   // 1 KiB (8 rows) per wave-instruction
  static_assert(TM >= 1 && TN >= 1 && GLDS_PER_WAVE >= 1, "bad tile");

  __shared__ __attribute__((aligned(16))) char smem[2 * TILE_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WAVES_N;
  const int wn = wave % WAVES_N;

  const int tiles_n = N / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tm = bid / tiles_n;
  const int tn = bid % tiles_n;
  const int m0 = tm * BM;
  const int n0 = tn * BN;
  const int kt_count = K / BK;

  // ---- A staging: this wave's global_load_lds sources (row clamp at M-1)
  const _Float16* a_src[GLDS_PER_WAVE];
  int a_dst[GLDS_PER_WAVE];
#pragma unroll
  for (int i = 0; i < GLDS_PER_WAVE; ++i) {
    const int r0 = (wave * GLDS_PER_WAVE + i) * 8;
    const int row = r0 + (lane >> 3);
    const int p = lane & 7;
    const int c = p ^ ((row >> 1) & 7);
    int gr = m0 + row;
    gr = gr < M ? gr : M - 1;
    a_src[i] = A + (int64_t)gr * lda + c * 8;
    a_dst[i] = r0 * ROWB;
  }
  auto stage_a = [&](int kt, int buf) {
#pragma unroll
    for (int i = 0; i < GLDS_PER_WAVE; ++i) {
      __builtin_amdgcn_global_load_lds((const SAMQ_GLOBAL void*)(a_src[i] + kt * BK),
                                       (SAMQ_LDS void*)(smem + buf * TILE_BYTES + a_dst[i]), 16, 0, 0);
    }
  };

  // ---- B fragments (packed): per n-tile one dwordx4 per lane per K tile
  const int ncol_tile0 = (n0 + wn * WN) / 32;
  const u32x4* b_ptr[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) b_ptr[t] = Wp + ((int64_t)(ncol_tile0 + t) * kt_count) * 64 + lane;

  // per-lane output column of each n-tile
  int col[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) col[t] = n0 + wn * WN + t * 32 + (lane & 31);

  auto load_zc = [&](int g, half2_t* zc, half2_t* sc) {
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const uint32_t zw = qzeros[(int64_t)g * (N / 8) + (col[t] >> 3)];
      const int zp = (int)((zw >> (4 * (col[t] & 7))) & 0xFu) + 1;
      const _Float16 z = (_Float16)(1024 + zp);
      zc[t] = half2_t{z, z};
      if (GROUPED) {
        const _Float16 s = scales[(int64_t)g * N + col[t]];
        sc[t] = half2_t{s, s};
      }
    }
  };

  half2_t zc[TN], sc[TN];
  load_zc(0, zc, sc);
  int cur_group = 0;

  float16_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // LDS read offsets for the A fragments of this wave (row part), k-chunk added per step
  int a_row[TM];
  int a_swz[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int rr = wm * WM + i * 32 + (lane & 31);
    a_row[i] = rr * ROWB;
    a_swz[i] = (rr >> 1) & 7;
  }
  const int hsel = lane >> 5;

  // unpack constants held in VGPRs (opaque to the compiler) so (x & M) | MAGIC fuses into one
  // v_and_or_b32 (gfx950 VOP3 takes no literal operands)
  uint32_t kMask = 0x000F000Fu, kMagic = 0x64006400u;
  if (VAR & 1) asm volatile("" : "+v"(kMask), "+v"(kMagic));

  // prologue
  stage_a(0, 0);
  u32x4 bcur[TN], bnext[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) bcur[t] = b_ptr[t][0];
  __syncthreads();

  for (int kt = 0; kt < kt_count; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < kt_count) {
      stage_a(kt + 1, buf ^ 1);
#pragma unroll
      for (int t = 0; t < TN; ++t) bnext[t] = b_ptr[t][(int64_t)(kt + 1) * 64];
    }
    if (GROUPED) {
      const int g = (kt * BK) / groupsize;
      if (g != cur_group) {
        load_zc(g, zc, sc);
        cur_group = g;
      }
    }
    const char* abase = smem + buf * TILE_BYTES;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      half8_t af[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int c = 2 * s + hsel;
        af[i] = *(const half8_t*)(abase + a_row[i] + ((c ^ a_swz[i]) << 4));
      }
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        const uint32_t w = bcur[t][s];
        half8_t bf;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t bits = ((w >> (4 * i)) & kMask) | kMagic;
          half2_t h = __builtin_bit_cast(half2_t, bits) - zc[t];
          if (GROUPED) h = h * sc[t];
          bf[2 * i] = h[0];
          bf[2 * i + 1] = h[1];
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
          acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i], bf, acc[i][t], 0, 0, 0);
      }
    }
    __syncthreads();
    if (kt + 1 < kt_count) {
#pragma unroll
      for (int t = 0; t < TN; ++t) bcur[t] = bnext[t];
    }
  }

  // ---- epilogue
  float csc[TN], cb[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    csc[t] = GROUPED ? 1.0f : (float)scales[col[t]];
    cb[t] = bias ? (float)bias[col[t]] : 0.0f;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hsel;
      if (row >= M) continue;
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        float v = acc[i][t][r] * csc[t] + cb[t];
        if (EPI == SAMQ_EPI_BIAS_GELU) v = gelu_erf(v);
        if (EPI == SAMQ_EPI_RESADD_F32) {
          float* cp = (float*)Cout + (int64_t)row * ldc + col[t];
          *cp = *cp + v;
        } else if (EPI == SAMQ_EPI_F32) {
          ((float*)Cout)[(int64_t)row * ldc + col[t]] = v;
        } else {
          ((_Float16*)Cout)[(int64_t)row * ldc + col[t]] = (_Float16)v;
        }
      }
    }
  }
}

// ------------------------------------------------------------------ GEMM v3 (3-stage LDS-DMA ring)
// Both operands reach LDS by global_load_lds: A (BM rows x 128 B, XOR-swizzled through the
// source address) and B (BN/32 packed 1-KiB fragment blocks, already in lane order); a 3-slot
// ring keeps two K tiles in flight behind counted vmcnt waits and ONE raw s_barrier per K tile
// (no vmcnt(0) drain in the loop).  Fragment reads: A ds_read_b128 (conflict-free swizzle),
// B ds_read_b128 lane-linear.
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N <= 63, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// int4 -> fp16 unpack of one packed word (8 k-values of one column, nibble order
// [k0,k2,k4,k6 | k1,k3,k5,k7]; nibble group i at bits 4i..4i+3 of both halves).  A nibble on
// mantissa bits 0..3 under the exponent of 1024 is the exact fp16 integer 1024+q; on bits 4..7
// under the exponent of 64 it is 64+q.  So groups 0 and 1 convert in place and groups 2 and 3
// after ONE shift by 8 of the word: 5 bit ops + 4 packed subtractions of (magic + zp) per 8
// weights instead of 7 + 4.  (Bits 8..15 would reach the 5-bit exponent field.)
struct W4Unpack {
  uint32_t m0, m1, g0, g1;   // masks / magics, held in VGPRs (gfx950 VOP3 takes no literal)
  __device__ void init() {
    m0 = 0x000F000Fu; m1 = 0x00F000F0u; g0 = 0x64006400u; g1 = 0x54005400u;
    asm volatile("" : "+v"(m0), "+v"(m1), "+v"(g0), "+v"(g1));
  }
};
struct W4Zero {   // (magic + zero point) splats of one column
  half2_t z1024, z64;
  __device__ void set(int zp) {
    const _Float16 a = (_Float16)(1024 + zp), b = (_Float16)(64 + zp);
    z1024 = half2_t{a, a};
    z64 = half2_t{b, b};
  }
};
__device__ __forceinline__ half8_t w4_unpack(uint32_t w, const W4Unpack& k, const W4Zero& z) {
  const uint32_t w8 = w >> 8;
  const half2_t h0 = __builtin_bit_cast(half2_t, (w & k.m0) | k.g0) - z.z1024;
  const half2_t h1 = __builtin_bit_cast(half2_t, (w & k.m1) | k.g1) - z.z64;
  const half2_t h2 = __builtin_bit_cast(half2_t, (w8 & k.m0) | k.g0) - z.z1024;
  const half2_t h3 = __builtin_bit_cast(half2_t, (w8 & k.m1) | k.g1) - z.z64;
  return half8_t{h0[0], h0[1], h1[0], h1[1], h2[0], h2[1], h3[0], h3[1]};
}
// grouped weights: the exact integers (q - zp) times the group's fp16 scale, one rounding
__device__ __forceinline__ half8_t scale8(half8_t v, half2_t s) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const half2_t h = half2_t{v[2 * i], v[2 * i + 1]} * s;
    v[2 * i] = h[0];
    v[2 * i + 1] = h[1];
  }
  return v;
}

// ---- LayerNorm-fold epilogues (SAMQ_EPI_RESADD_LNF / BIAS_LNF / GELU_LNF, include/samq.h)
struct LnfArgs {
  const float* gamma;   // producer: the next LayerNorm's weight [N]
  const float* gw;      // consumer: gamma . W [N]
  const float* bw;      // consumer: beta . W [N]
  float* stats;         // [M][N_producer / 64][2] partial sums of (x - mu_p), (x - mu_p)^2
  float* mu;            // [M] row mean of the previous LayerNorm (consumer: += delta)
  _Float16* aout;       // producer: f16 (x - mu_p) * gamma [M][N]
  float eps;
  int nblk;             // consumer: K / 64 partial-sum blocks per row
  const _Float16* bias; // consumer: the layer bias (set by the kernel)
};
constexpr bool lnf_producer(int epi) { return epi == SAMQ_EPI_RESADD_LNF; }
constexpr bool lnf_consumer(int epi) { return epi == SAMQ_EPI_BIAS_LNF || epi == SAMQ_EPI_GELU_LNF; }
constexpr bool epi_f32_out(int epi) {
  return epi == SAMQ_EPI_RESADD_F32 || epi == SAMQ_EPI_F32 || epi == SAMQ_EPI_RESADD_LNF;
}

// producer: one f32 residual row chunk (4 columns at col of row) x_new = xo + v (xo: the old
// residual, loaded ahead by the caller), its f16 fold operand and this lane's partial sums; the
// caller reduces the sums over the 16 lanes of a row
__device__ __forceinline__ void lnf_res4(const LnfArgs& L, float* C, int64_t ldc, int N, int64_t row, int col,
                                         float4_t xo, float4_t v, float m, float4_t g, float& s1, float& s2) {
  const float4_t x = xo + v;
  *(float4_t*)(C + row * ldc + col) = x;
  const float4_t d = x - m;
  *(half4_t*)(L.aout + row * N + col) = half4_t{(_Float16)(d[0] * g[0]), (_Float16)(d[1] * g[1]),
                                                (_Float16)(d[2] * g[2]), (_Float16)(d[3] * g[3])};
  s1 = (d[0] + d[1]) + (d[2] + d[3]);
  s2 = (d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]);
}
// sum over the 16 lanes of a DPP row (the xor-1, 2, 4, 8 butterfly's order: same bits)
__device__ __forceinline__ float sum16_dpp(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, true));
  return v;
}
// ... reduced over 16 lanes (one row), lane 0 of the 16 writes the block's pair
__device__ __forceinline__ void lnf_stats16(const LnfArgs& L, int N, int64_t row, int col_block, bool valid,
                                            float s1, float s2, int c4) {
  s1 = sum16_dpp(s1);
  s2 = sum16_dpp(s2);
  if (valid && c4 == 0) *(float2_t*)(L.stats + (row * (N / 64) + col_block) * 2) = float2_t{s1, s2};
}
// producer slice of R rows x 64 columns staged in LDS at ep (row pitch P floats): the old residual
// and the row means are all loaded before the first store (no store-to-load ordering per chunk)
template <int R, int P>
__device__ __forceinline__ void lnf_produce_slice(const LnfArgs& L, const float* ep, float* C, int64_t ldc, int N,
                                                  int M, int srow0, int col_base, int lane) {
  constexpr int J = R * 16 / 64;
  const int c4 = lane & 15;
  const int col = col_base + 4 * c4;
  const float4_t g = *(const float4_t*)(L.gamma + col);
  float4_t xo[J];
  float m[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    int64_t row = srow0 + 4 * j + (lane >> 4);
    row = row < M ? row : M - 1;
    xo[j] = *(const float4_t*)(C + row * ldc + col);
    m[j] = L.mu[row];
  }
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int rl = 4 * j + (lane >> 4);
    const int row = srow0 + rl;
    const float4_t v = *(const float4_t*)(ep + rl * P + 4 * c4);
    float s1 = 0.f, s2 = 0.f;
    if (row < M) lnf_res4(L, C, ldc, N, row, col, xo[j], v, m[j], g, s1, s2);
    lnf_stats16(L, N, row, col_base / 64, row < M, s1, s2, c4);
  }
}
// consumer: (delta, rstd) of the workgroup's BM rows into LDS (rowinfo[BM]), mu += delta by the
// workgroups of column tile 0.  The rows' partial sums (BM x nblk float2, contiguous) arrive by
// LDS-DMA (1 KiB pieces dealt over the NW waves, one wait), then one lane per row adds its nblk
// pairs in block order from LDS (the order of the standalone reduction: same bits).
template <int BM, int NW>
__device__ __forceinline__ void lnf_rowinfo_wg(const LnfArgs& L, float2_t* rowinfo, char* sbuf, int M, int row_base,
                                               bool col0, int wave, int lane) {
  static_assert(BM % (NW * 32) == 0 || BM <= NW * 64, "rows per wave");
  const int nfl = 2 * L.nblk;                                 // floats per row
  const int npieces = BM * nfl / 256;                         // 1 KiB pieces (BM * nblk * 8 / 1024)
  const float* base = L.stats + (int64_t)row_base * nfl;
  const int64_t lim = (int64_t)(M - row_base) * nfl - 4;      // last in-bounds 16-byte chunk
  for (int pc = wave; pc < npieces; pc += NW) {
    int64_t off = (int64_t)(pc * 64 + lane) * 4;
    off = off <= lim ? off : lim;
    __builtin_amdgcn_global_load_lds((const SAMQ_GLOBAL void*)(base + off), (SAMQ_LDS void*)(sbuf + pc * 1024), 16, 0, 0);
  }
  vm_wait<0>();
  __syncthreads();
  const float inv_k = 1.0f / (float)(L.nblk * 64);
  constexpr int RPW = BM / NW;                                // rows per wave
#pragma unroll
  for (int q = 0; q < (RPW + 63) / 64; ++q) {
    const int rl = wave * RPW + q * 64 + lane;
    if (q * 64 + lane < RPW) {
      const float2_t* sp = (const float2_t*)(sbuf + rl * nfl * 4);
      float s1 = 0.f, s2 = 0.f;
      for (int b = 0; b < L.nblk; ++b) {
        const float2_t v = sp[b];
        s1 += v.x;
        s2 += v.y;
      }
      const float delta = s1 * inv_k;
      const float var = fmaxf(s2 * inv_k - delta * delta, 0.0f);
      rowinfo[rl] = float2_t{delta, rsqrtf(var + L.eps)};
      const int64_t row = row_base + rl;
      if (col0 && row < M) L.mu[row] += delta;
    }
  }
  __syncthreads();
}
// consumer store of 8 columns: y = rstd * (v - delta * gw) + (bw + bias) (-> GELU), f16
template <int EPI>
__device__ __forceinline__ half8_t lnf_out8(float4_t v0, float4_t v1, float2_t ri, const float (&gw)[8],
                                           const float (&bb)[8]) {
  float y[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  half8_t h;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float t = __builtin_fmaf(ri.y, __builtin_fmaf(-ri.x, gw[e], y[e]), bb[e]);
    if (EPI == SAMQ_EPI_GELU_LNF) t = gelu_fast(t);
    h[e] = (_Float16)t;
  }
  return h;
}

// The same epilogue for 16x16x32 accumulators (VAR & 16 of the ping-pong kernel): lane (ql, g)
// of 16-row tile i, 32-column block t, half h holds rows 16i + 4g + r of column 32t + 16h + ql;
// staged per 16-row tile with a padded pitch (WN + 4 floats: the four lane groups' rows land
// on different banks).
template <int TM16, int TN, int EPI>
__device__ __forceinline__ void pp_epilogue16(const float4_t (&acc)[TM16][TN][2], const float (&csc)[TN][2],
                                              const float (&cb)[TN][2], char* ep_bytes, void* Cout, int64_t ldc,
                                              int M, int row_base, int col_base, int lane,
                                              const LnfArgs& L = LnfArgs{}, int N = 0,
                                              const float2_t* rowinfo = nullptr) {
  constexpr int WN = TN * 32, EP_ROWS = 16, PITCH = WN + 4;
  static_assert(!(lnf_producer(EPI) || lnf_consumer(EPI)) || WN == 64, "LN fold: 64-column wave tiles");
  float* ep = (float*)ep_bytes;
  const int ql = lane & 15, g = lane >> 4;
  float gw8[8], bb8[8];   // LNF consumer: this lane's 8 columns (fixed over the slices)
  if constexpr (lnf_consumer(EPI)) {
    const int c0 = col_base + 8 * (lane % (WN / 8));
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      gw8[e] = L.gw[c0 + e];
      bb8[e] = L.bw[c0 + e] + (L.bias ? (float)L.bias[c0 + e] : 0.0f);
    }
  }
#pragma unroll
  for (int i = 0; i < TM16; ++i) {
#pragma unroll
    for (int t = 0; t < TN; ++t)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = lnf_consumer(EPI) ? acc[i][t][h][r] * csc[t][h] : acc[i][t][h][r] * csc[t][h] + cb[t][h];
          if (EPI == SAMQ_EPI_BIAS_GELU) v = gelu_fast(v);
          ep[(4 * g + r) * PITCH + 32 * t + 16 * h + ql] = v;
        }
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the slice is in LDS (same wave reads it)
    const int srow0 = row_base + i * 16;
    if (lnf_producer(EPI)) {
      lnf_produce_slice<EP_ROWS, PITCH>(L, ep, (float*)Cout, ldc, N, M, srow0, col_base, lane);
    } else if (EPI == SAMQ_EPI_RESADD_F32 || EPI == SAMQ_EPI_F32) {
      constexpr int C4 = WN / 4;
#pragma unroll
      for (int j = 0; j < (EP_ROWS * C4 + 63) / 64; ++j) {
        const int idx = j * 64 + lane;
        if (idx < EP_ROWS * C4) {
          const int rl = idx / C4, c4 = idx % C4;
          const int row = srow0 + rl;
          const float4_t v = *(const float4_t*)(ep + rl * PITCH + 4 * c4);
          if (row < M) {
            float4_t* cp = (float4_t*)((float*)Cout + (int64_t)row * ldc + col_base + 4 * c4);
            if (EPI == SAMQ_EPI_RESADD_F32) *cp = *cp + v; else *cp = v;
          }
        }
      }
    } else if (lnf_consumer(EPI)) {
      constexpr int C8 = WN / 8;
#pragma unroll
      for (int j = 0; j < (EP_ROWS * C8 + 63) / 64; ++j) {
        const int idx = j * 64 + lane;
        if (idx < EP_ROWS * C8) {
          const int rl = idx / C8, c8 = idx % C8;
          const int row = srow0 + rl;
          const float4_t v0 = *(const float4_t*)(ep + rl * PITCH + 8 * c8);
          const float4_t v1 = *(const float4_t*)(ep + rl * PITCH + 8 * c8 + 4);
          if (row < M) {
            const float2_t ri = rowinfo[row - row_base];
            *(half8_t*)((_Float16*)Cout + (int64_t)row * ldc + col_base + 8 * c8) = lnf_out8<EPI>(v0, v1, ri, gw8, bb8);
          }
        }
      }
    } else {
      constexpr int C8 = WN / 8;
#pragma unroll
      for (int j = 0; j < (EP_ROWS * C8 + 63) / 64; ++j) {
        const int idx = j * 64 + lane;
        if (idx < EP_ROWS * C8) {
          const int rl = idx / C8, c8 = idx % C8;
          const int row = srow0 + rl;
          const float4_t v0 = *(const float4_t*)(ep + rl * PITCH + 8 * c8);
          const float4_t v1 = *(const float4_t*)(ep + rl * PITCH + 8 * c8 + 4);
          if (row < M) {
            const half8_t hv = {(_Float16)v0[0], (_Float16)v0[1], (_Float16)v0[2], (_Float16)v0[3],
                                (_Float16)v1[0], (_Float16)v1[1], (_Float16)v1[2], (_Float16)v1[3]};
            *(half8_t*)((_Float16*)Cout + (int64_t)row * ldc + col_base + 8 * c8) = hv;
          }
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);   // reads done before the next slice overwrites
  }
}

template <int BM, int BN, int WAVES_M, int WAVES_N, int EPI, bool GROUPED, int VAR = 0>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N)
void w4a16_gemm_v3(const _Float16* __restrict__ A, int64_t lda, const u32x4* __restrict__ Wp,
                   const _Float16* __restrict__ scales, const uint32_t* __restrict__ qzeros,
                   const _Float16* __restrict__ bias, void* __restrict__ Cout, int64_t ldc,
                   int M, int N, int K, int groupsize) {
  constexpr int NW = WAVES_M * WAVES_N;
  constexpr int WM = BM / WAVES_M;
  constexpr int WN = BN / WAVES_N;
  constexpr int TM = WM / 32;
  constexpr int TN = WN / 32;
  constexpr int BK = 64;
  constexpr int ROWB = BK * 2;
  constexpr int A_BYTES = BM * ROWB;
  constexpr int NA = BM / 8;                 // A pieces (1 KiB = 8 rows) per stage
  constexpr int NB = BN / 32;                // B pieces (one packed n-tile block) per stage
  constexpr int NT = NA + NB;
  constexpr int NPW = (NT + NW - 1) / NW;    // glds per wave per stage
  constexpr int STAGE = A_BYTES + NB * 1024;
  constexpr int STAGES = 3;
  static_assert(TM >= 1 && TN >= 1 && NPW <= 15, "bad tile");
  constexpr int EP_BYTES = 32 * WN * 4;                // epilogue: one 32-row slice per wave, f32
  constexpr int SMEM = STAGES * STAGE > NW * EP_BYTES ? STAGES * STAGE : NW * EP_BYTES;

  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WAVES_N;
  const int wn = wave % WAVES_N;
  const int tiles_n = N / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (bid / tiles_n) * BM;
  const int n0 = (bid % tiles_n) * BN;
  const int kt_count = K / BK;

  // ---- this wave's LDS-DMA pieces: global source (per lane) and LDS offset (wave-uniform)
  const char* src[NPW];
  int dst[NPW];
  int64_t step[NPW];   // source advance per K tile (bytes)
#pragma unroll
  for (int i = 0; i < NPW; ++i) {
    int j = wave * NPW + i;
    j = j < NT ? j : NT - 1;   // surplus slots re-issue the last piece (same bytes, same place)
    if (j < NA) {
      const int row = j * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      int gr = m0 + row;
      gr = gr < M ? gr : M - 1;
      src[i] = (const char*)(A + (int64_t)gr * lda + c * 8);
      dst[i] = j * 1024;
      step[i] = BK * 2;
    } else {
      const int nt = n0 / 32 + (j - NA);
      src[i] = (const char*)(Wp + ((int64_t)nt * kt_count) * 64 + lane);
      dst[i] = A_BYTES + (j - NA) * 1024;
      step[i] = 64 * 16;
    }
  }
  auto issue = [&](int kt, int slot) {
#pragma unroll
    for (int i = 0; i < NPW; ++i)
      __builtin_amdgcn_global_load_lds((const SAMQ_GLOBAL void*)(src[i] + kt * step[i]),
                                       (SAMQ_LDS void*)(smem + slot * STAGE + dst[i]), 16, 0, 0);
  };

  int col[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) col[t] = n0 + wn * WN + t * 32 + (lane & 31);
  W4Zero zc[TN];
  half2_t sc[TN];
  auto load_zc = [&](int g) {
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const uint32_t zw = qzeros[(int64_t)g * (N / 8) + (col[t] >> 3)];
      zc[t].set((int)((zw >> (4 * (col[t] & 7))) & 0xFu) + 1);
      if (GROUPED) {
        const _Float16 s = scales[(int64_t)g * N + col[t]];
        sc[t] = half2_t{s, s};
      }
    }
  };
  load_zc(0);
  int cur_group = 0;

  W4Unpack ku;
  ku.init();

  float16_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  int a_off[TM], a_swz[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int rr = wm * WM + i * 32 + (lane & 31);
    a_off[i] = rr * ROWB;
    a_swz[i] = (rr >> 1) & 7;
  }
  const int hsel = lane >> 5;

  issue(0, 0);
  if (kt_count > 1) issue(1, 1);
  int slot = 0;
  for (int kt = 0; kt < kt_count; ++kt) {
    if (kt + 1 < kt_count) vm_wait<NPW>(); else vm_wait<0>();
    __builtin_amdgcn_s_barrier();          // tile kt visible to all; slot (kt+2)%3 free
    if (kt + 2 < kt_count) {
      int s2 = slot + 2;
      s2 = s2 >= STAGES ? s2 - STAGES : s2;
      issue(kt + 2, s2);
    }
    if (GROUPED) {
      const int g = (kt * BK) / groupsize;
      if (g != cur_group) { load_zc(g); cur_group = g; }
    }
    const char* abase = smem + slot * STAGE;
    u32x4 bw[TN];
#pragma unroll
    for (int t = 0; t < TN; ++t) bw[t] = *(const u32x4*)(abase + A_BYTES + (wn * TN + t) * 1024 + lane * 16);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      half8_t af[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *(const half8_t*)(abase + a_off[i] + (((2 * s + hsel) ^ a_swz[i]) << 4));
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        const uint32_t w = bw[t][s];
        half8_t bf;
        if (VAR == 1) {   // TIMING-ONLY variant (wrong results): MFMA on the raw words, no unpack
          bf = __builtin_bit_cast(half8_t, bw[t]);
        } else {
          bf = w4_unpack(w, ku, zc[t]);
          if (GROUPED) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const half2_t h = half2_t{bf[2 * i], bf[2 * i + 1]} * sc[t];
              bf[2 * i] = h[0];
              bf[2 * i + 1] = h[1];
            }
          }
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i], bf, acc[i][t], 0, 0, 0);
      }
    }
    slot = slot + 1 == STAGES ? 0 : slot + 1;
  }

  // ---- epilogue: y = acc * s[n] + b[n] (-> GELU), staged through LDS per 32-row slice so the
  // global traffic is row-contiguous 16-byte vectors (f16: 8 columns / lane; f32 residual:
  // 4 columns / lane read-modify-write) instead of one 2- or 4-byte access per accumulator.
  float csc[TN], cb[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    csc[t] = GROUPED ? 1.0f : (float)scales[col[t]];
    cb[t] = bias ? (float)bias[col[t]] : 0.0f;
  }
  __syncthreads();                                      // every wave is done with the ring
  float* ep = (float*)(smem + wave * EP_BYTES);
  const int row_base = m0 + wm * WM;
  const int col_base = n0 + wn * WN;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rl = (r & 3) + 8 * (r >> 2) + 4 * hsel;   // row within the slice
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        float v = acc[i][t][r] * csc[t] + cb[t];
        if (EPI == SAMQ_EPI_BIAS_GELU) v = gelu_fast(v);
        ep[rl * WN + t * 32 + (lane & 31)] = v;
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the slice is in LDS (same wave reads it)
    if (EPI == SAMQ_EPI_RESADD_F32 || EPI == SAMQ_EPI_F32) {
      constexpr int C4 = WN / 4;                        // float4 per slice row
#pragma unroll
      for (int j = 0; j < 32 * C4 / 64; ++j) {
        const int idx = j * 64 + lane;
        const int rl = idx / C4, c4 = idx % C4;
        const int row = row_base + i * 32 + rl;
        const float4_t v = ((const float4_t*)ep)[idx];
        if (row < M) {
          float4_t* cp = (float4_t*)((float*)Cout + (int64_t)row * ldc + col_base + 4 * c4);
          if (EPI == SAMQ_EPI_RESADD_F32) *cp = *cp + v; else *cp = v;
        }
      }
    } else {
      constexpr int C8 = WN / 8;                        // 8-column chunks per slice row
#pragma unroll
      for (int j = 0; j < (32 * C8 + 63) / 64; ++j) {
        const int idx = j * 64 + lane;
        if (idx < 32 * C8) {
          const int rl = idx / C8, c8 = idx % C8;
          const int row = row_base + i * 32 + rl;
          const float4_t v0 = ((const float4_t*)ep)[2 * idx];
          const float4_t v1 = ((const float4_t*)ep)[2 * idx + 1];
          if (row < M) {
            const half8_t h = {(_Float16)v0[0], (_Float16)v0[1], (_Float16)v0[2], (_Float16)v0[3],
                               (_Float16)v1[0], (_Float16)v1[1], (_Float16)v1[2], (_Float16)v1[3]};
            *(half8_t*)((_Float16*)Cout + (int64_t)row * ldc + col_base + 8 * c8) = h;
          }
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);   // reads done before the next slice overwrites
  }
}

// ------------------------------------------------------------------ GEMM v4 (16x16x32 MFMA)
// Same 3-stage LDS-DMA ring as v3 on v_mfma_f32_16x16x32_f16 (packed LAYOUT 2).  The 16x16
// shape holds a higher clock under load than 32x32x16 at equal cycles/FLOP (MI355X_MICROARCH
// 'DVFS give-back' item 7).  A fragments: 16 rows x 16 B per lane group, XOR-swizzled.
template <int BM, int BN, int WAVES_M, int WAVES_N, int EPI, bool GROUPED>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N)
void w4a16_gemm_v4(const _Float16* __restrict__ A, int64_t lda, const u32x4* __restrict__ Wp,
                   const _Float16* __restrict__ scales, const uint32_t* __restrict__ qzeros,
                   const _Float16* __restrict__ bias, void* __restrict__ Cout, int64_t ldc,
                   int M, int N, int K, int groupsize) {
  constexpr int NW = WAVES_M * WAVES_N;
  constexpr int WM = BM / WAVES_M;
  constexpr int WN = BN / WAVES_N;
  constexpr int TM = WM / 16;                // 16-row MFMA tiles per wave
  constexpr int TB = WN / 32;                // packed 32-column blocks per wave
  constexpr int BK = 64;
  constexpr int ROWB = BK * 2;
  constexpr int A_BYTES = BM * ROWB;
  constexpr int NA = BM / 8;
  constexpr int NB = BN / 32;
  constexpr int NT = NA + NB;
  constexpr int NPW = (NT + NW - 1) / NW;
  constexpr int STAGE = A_BYTES + NB * 1024;
  constexpr int STAGES = 3;
  static_assert(TM >= 1 && TB >= 1 && NPW <= 15, "bad tile");

  __shared__ __attribute__((aligned(16))) char smem[STAGES * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WAVES_N;
  const int wn = wave % WAVES_N;
  const int ql = lane & 15;
  const int g = lane >> 4;
  const int tiles_n = N / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (bid / tiles_n) * BM;
  const int n0 = (bid % tiles_n) * BN;
  const int kt_count = K / BK;

  const char* src[NPW];
  int dst[NPW];
  int64_t step[NPW];
#pragma unroll
  for (int i = 0; i < NPW; ++i) {
    int j = wave * NPW + i;
    j = j < NT ? j : NT - 1;
    if (j < NA) {
      const int row = j * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      int gr = m0 + row;
      gr = gr < M ? gr : M - 1;
      src[i] = (const char*)(A + (int64_t)gr * lda + c * 8);
      dst[i] = j * 1024;
      step[i] = BK * 2;
    } else {
      const int nt = n0 / 32 + (j - NA);
      src[i] = (const char*)(Wp + ((int64_t)nt * kt_count) * 64 + lane);
      dst[i] = A_BYTES + (j - NA) * 1024;
      step[i] = 64 * 16;
    }
  }
  auto issue = [&](int kt, int slot) {
#pragma unroll
    for (int i = 0; i < NPW; ++i)
      __builtin_amdgcn_global_load_lds((const SAMQ_GLOBAL void*)(src[i] + kt * step[i]),
                                       (SAMQ_LDS void*)(smem + slot * STAGE + dst[i]), 16, 0, 0);
  };

  // columns of this lane: block t, half h -> n0 + wn*WN + 32t + 16h + ql
  int col[TB][2];
#pragma unroll
  for (int t = 0; t < TB; ++t)
#pragma unroll
    for (int h = 0; h < 2; ++h) col[t][h] = n0 + wn * WN + 32 * t + 16 * h + ql;
  half2_t zc[TB][2], sc[TB][2];
  auto load_zc = [&](int gi) {
#pragma unroll
    for (int t = 0; t < TB; ++t)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = col[t][h];
        const uint32_t zw = qzeros[(int64_t)gi * (N / 8) + (c >> 3)];
        const _Float16 z = (_Float16)(1024 + (int)((zw >> (4 * (c & 7))) & 0xFu) + 1);
        zc[t][h] = half2_t{z, z};
        if (GROUPED) {
          const _Float16 s = scales[(int64_t)gi * N + c];
          sc[t][h] = half2_t{s, s};
        }
      }
  };
  load_zc(0);
  int cur_group = 0;

  uint32_t kMask = 0x000F000Fu, kMagic = 0x64006400u;
  asm volatile("" : "+v"(kMask), "+v"(kMagic));

  float4_t acc[TM][TB][2];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int t = 0; t < TB; ++t)
#pragma unroll
      for (int h = 0; h < 2; ++h) acc[i][t][h] = float4_t{0.f, 0.f, 0.f, 0.f};

  int a_off[TM], a_swz[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int rr = wm * WM + i * 16 + ql;
    a_off[i] = rr * ROWB;
    a_swz[i] = (rr >> 1) & 7;
  }

  issue(0, 0);
  if (kt_count > 1) issue(1, 1);
  int slot = 0;
  for (int kt = 0; kt < kt_count; ++kt) {
    if (kt + 1 < kt_count) vm_wait<NPW>(); else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < kt_count) {
      int s2 = slot + 2;
      s2 = s2 >= STAGES ? s2 - STAGES : s2;
      issue(kt + 2, s2);
    }
    if (GROUPED) {
      const int gi = (kt * BK) / groupsize;
      if (gi != cur_group) { load_zc(gi); cur_group = gi; }
    }
    const char* abase = smem + slot * STAGE;
    u32x4 bw[TB];
#pragma unroll
    for (int t = 0; t < TB; ++t) bw[t] = *(const u32x4*)(abase + A_BYTES + (wn * TB + t) * 1024 + lane * 16);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      half8_t af[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *(const half8_t*)(abase + a_off[i] + (((4 * s + g) ^ a_swz[i]) << 4));
#pragma unroll
      for (int t = 0; t < TB; ++t) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t w = bw[t][2 * h + s];
          half8_t bf;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            half2_t hv = __builtin_bit_cast(half2_t, ((w >> (4 * q)) & kMask) | kMagic) - zc[t][h];
            if (GROUPED) hv = hv * sc[t][h];
            bf[2 * q] = hv[0];
            bf[2 * q + 1] = hv[1];
          }
#pragma unroll
          for (int i = 0; i < TM; ++i)
            acc[i][t][h] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf, acc[i][t][h], 0, 0, 0);
        }
      }
    }
    slot = slot + 1 == STAGES ? 0 : slot + 1;
  }

  // ---- epilogue (16x16 C layout: column = lane&15, row = 4*(lane>>4) + reg)
#pragma unroll
  for (int t = 0; t < TB; ++t)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = col[t][h];
      const float cs = GROUPED ? 1.0f : (float)scales[c];
      const float cb = bias ? (float)bias[c] : 0.0f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm * WM + i * 16 + 4 * g + r;
          if (row >= M) continue;
          float v = acc[i][t][h][r] * cs + cb;
          if (EPI == SAMQ_EPI_BIAS_GELU) v = gelu_fast(v);
          if (EPI == SAMQ_EPI_RESADD_F32) {
            float* cp = (float*)Cout + (int64_t)row * ldc + c;
            *cp = *cp + v;
          } else if (EPI == SAMQ_EPI_F32) {
            ((float*)Cout)[(int64_t)row * ldc + c] = v;
          } else {
            ((_Float16*)Cout)[(int64_t)row * ldc + c] = (_Float16)v;
          }
        }
    }
}

// y = acc * s[n] + b[n] (-> GELU / residual add), staged through LDS in EP_ROWS-row slices per
// wave so the global traffic is row-contiguous 16-byte vectors (v3's epilogue)
// EVAR (tuning build, timing-only): 1 = f16 outputs staged but not stored, 2 = no scale / bias / GELU
template <int TM, int TN, int EP_ROWS, int EPI, int EVAR = 0>
__device__ __forceinline__ void pp_epilogue(const float16_t (&acc)[TM][TN], const float (&csc)[TN],
                                            const float (&cb)[TN], char* ep_bytes, void* Cout, int64_t ldc,
                                            int M, int row_base, int col_base, int lane,
                                            const LnfArgs& L = LnfArgs{}, int N = 0,
                                            const float2_t* rowinfo = nullptr) {
  constexpr int WN = TN * 32;
  constexpr int NSL = 32 / EP_ROWS;
  static_assert(!(lnf_producer(EPI) || lnf_consumer(EPI)) || WN == 64, "LN fold: 64-column wave tiles");
  float* ep = (float*)ep_bytes;
  const int hsel = lane >> 5;
  constexpr bool F16SWZ = EPI == SAMQ_EPI_BIAS || EPI == SAMQ_EPI_BIAS_GELU;   // staging swizzle (below)
  if constexpr (EPI == SAMQ_EPI_SILU_MUL) {
    // gated MLP: the wave's 64 columns are one 32-column block of the gate (t = 0) and the same
    // block of the up projection (t = 1) -- samq_w4_interleave32 layout; out f16 [M, N / 2] =
    // silu(gate) * up, the 32 output columns of block (col_base / 64)
    static_assert(TN == 2 && EP_ROWS == 32, "SILU_MUL: 64-column wave tiles");
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rl = (r & 3) + 8 * (r >> 2) + 4 * hsel;
        const float gv = acc[i][0][r] * csc[0], uv = acc[i][1][r] * csc[1];
        ep[rl * 32 + (lane & 31)] = gv / (1.0f + __expf(-gv)) * uv;
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);
      const int srow0 = row_base + i * 32;
#pragma unroll
      for (int j = 0; j < 2; ++j) {   // 32 rows x 4 chunks of 8 columns
        const int idx = j * 64 + lane;
        const int rl = idx >> 2, c8 = idx & 3;
        const int row = srow0 + rl;
        const float4_t v0 = ((const float4_t*)ep)[2 * idx];
        const float4_t v1 = ((const float4_t*)ep)[2 * idx + 1];
        if (row < M) {
          const half8_t h = {(_Float16)v0[0], (_Float16)v0[1], (_Float16)v0[2], (_Float16)v0[3],
                             (_Float16)v1[0], (_Float16)v1[1], (_Float16)v1[2], (_Float16)v1[3]};
          *(half8_t*)((_Float16*)Cout + (int64_t)row * ldc + col_base / 2 + 8 * c8) = h;
        }
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);
    }
    return;
  }
  float gw8[8], bb8[8];   // LNF consumer: this lane's 8 columns (fixed over the slices)
  if constexpr (lnf_consumer(EPI)) {
    const int c0 = col_base + 8 * (lane % (WN / 8));
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      gw8[e] = L.gw[c0 + e];
      bb8[e] = L.bw[c0 + e] + (L.bias ? (float)L.bias[c0 + e] : 0.0f);
    }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int sl = 0; sl < NSL; ++sl) {
#pragma unroll
      for (int rq = 0; rq < 16 / NSL; rq += 2) {   // accumulator pairs (r, r + 1): packed fp32 math
        const int r = sl * (16 / NSL) + rq;
        const int rl = (r & 3) + 8 * (r >> 2) + 4 * hsel - sl * EP_ROWS;   // row within the slice (r + 1: rl + 1)
#pragma unroll
        for (int t = 0; t < TN; ++t) {
          float2_t v = (EVAR & 2) ? (float2_t){acc[i][t][r], acc[i][t][r + 1]}
                                  : __builtin_elementwise_fma((float2_t){acc[i][t][r], acc[i][t][r + 1]}, (float2_t)(csc[t]),
                                                              (float2_t)(lnf_consumer(EPI) ? 0.0f : cb[t]));
          if (EPI == SAMQ_EPI_BIAS_GELU && !(EVAR & 2)) v = gelu_fast2(v);
          // f16 outputs: the 4-column chunk XOR ((rl >> 1) & 1) within each 8 columns, so the two
          // 16-byte reads of a lane group's 4 rows land on distinct banks (gemm_i8.hip i8_epilogue)
          const int cs = (t * 32 + (lane & 31)) ^ (F16SWZ ? 4 * ((rl >> 1) & 1) : 0);
          ep[rl * WN + cs] = v.x;
          ep[(rl + 1) * WN + cs] = v.y;
        }
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the slice is in LDS (same wave reads it)
      const int srow0 = row_base + i * 32 + sl * EP_ROWS;
      if (lnf_producer(EPI)) {
        lnf_produce_slice<EP_ROWS, WN>(L, ep, (float*)Cout, ldc, N, M, srow0, col_base, lane);
      } else if (lnf_consumer(EPI)) {
        constexpr int C8 = WN / 8;
#pragma unroll
        for (int j = 0; j < (EP_ROWS * C8 + 63) / 64; ++j) {
          const int idx = j * 64 + lane;
          if (idx < EP_ROWS * C8) {
            const int rl = idx / C8, c8 = idx % C8;
            const int row = srow0 + rl;
            const float4_t v0 = ((const float4_t*)ep)[2 * idx];
            const float4_t v1 = ((const float4_t*)ep)[2 * idx + 1];
            if (row < M) {
              const float2_t ri = rowinfo[row - row_base];
              *(half8_t*)((_Float16*)Cout + (int64_t)row * ldc + col_base + 8 * c8) = lnf_out8<EPI>(v0, v1, ri, gw8, bb8);
            }
          }
        }
      } else if (EPI == SAMQ_EPI_RESADD_F32 || EPI == SAMQ_EPI_F32) {
        constexpr int C4 = WN / 4;
#pragma unroll
        for (int j = 0; j < (EP_ROWS * C4 + 63) / 64; ++j) {
          const int idx = j * 64 + lane;
          if (idx < EP_ROWS * C4) {
            const int rl = idx / C4, c4 = idx % C4;
            const int row = srow0 + rl;
            const float4_t v = ((const float4_t*)ep)[idx];
            if (row < M) {
              float4_t* cp = (float4_t*)((float*)Cout + (int64_t)row * ldc + col_base + 4 * c4);
              if (EPI == SAMQ_EPI_RESADD_F32) *cp = *cp + v; else *cp = v;
            }
          }
        }
      } else {
        constexpr int C8 = WN / 8;
#pragma unroll
        for (int j = 0; j < (EP_ROWS * C8 + 63) / 64; ++j) {
          const int idx = j * 64 + lane;
          if (idx < EP_ROWS * C8) {
            const int rl = idx / C8, c8 = idx % C8;
            const int row = srow0 + rl;
            const int sk = (rl >> 1) & 1;   // F16SWZ
            const float4_t v0 = ((const float4_t*)ep)[2 * idx + sk];
            const float4_t v1 = ((const float4_t*)ep)[2 * idx + (1 ^ sk)];
            if (row < M) {
              const half8_t h = {(_Float16)v0[0], (_Float16)v0[1], (_Float16)v0[2], (_Float16)v0[3],
                                 (_Float16)v1[0], (_Float16)v1[1], (_Float16)v1[2], (_Float16)v1[3]};
              if (!(EVAR & 1) || (float)h[0] == 1234.5f) *(half8_t*)((_Float16*)Cout + (int64_t)row * ldc + col_base + 8 * c8) = h;
            }
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);   // reads done before the next slice overwrites
    }
  }
}


// f16-output epilogue staged TRANSPOSED (VAR & (1 << 22), round 4): per 32-row slice the wave
// writes its 64 x 32 (column x row) f16 image -- lane (l32, hsel) packs the 4 consecutive rows of
// one column that accumulator registers 4j .. 4j+3 hold into ONE ds_write_b64 (pitch 72 B: the 16
// lanes of a write group on distinct banks) -- and reads it back row-contiguous with
// ds_read_b64_tr_b16 (T10: lane 4q+p of a 16-lane group addresses image row q = output column, 4
// output rows at 4p; lane i receives output row i, 4 columns), two reads per 16-byte store.  vs
// pp_epilogue: 8 instead of 32 LDS writes per slice and half the staged bytes (f16, not f32).
__device__ __forceinline__ half4_t ep_tr16(uint32_t addr) {
  half4_t r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}
template <int TM, int TN, int EPI>
__device__ __forceinline__ void pp_epilogue_f16t(const float16_t (&acc)[TM][TN], const float (&csc)[TN],
                                                 const float (&cb)[TN], char* ep_bytes, void* Cout, int64_t ldc,
                                                 int M, int row_base, int col_base, int lane) {
  static_assert(TN == 2, "64-column wave tiles");
  static_assert(EPI == SAMQ_EPI_BIAS || EPI == SAMQ_EPI_BIAS_GELU, "f16 outputs");
  constexpr int PITCH = 72;                              // bytes per image row (32 f16 + 8 pad)
  const int l32 = lane & 31, hsel = lane >> 5;
  const uint32_t img = (uint32_t)(uintptr_t)((const SAMQ_LDS char*)ep_bytes);
  // tr-read addresses: group g (lanes 16g..16g+15), iteration k: pair pi = 4k + g = (16-row half
  // rb = pi & 1, 8-column chunk c8 = pi >> 1); lane 4q+p: image row 8 c8 + q (+4), rows 16 rb + 4p
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3, i16 = lane & 15;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int t = 0; t < TN; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float2_t v0 = __builtin_elementwise_fma((float2_t){acc[i][t][4 * j], acc[i][t][4 * j + 1]}, (float2_t)(csc[t]),
                                                (float2_t)(cb[t]));
        float2_t v1 = __builtin_elementwise_fma((float2_t){acc[i][t][4 * j + 2], acc[i][t][4 * j + 3]},
                                                (float2_t)(csc[t]), (float2_t)(cb[t]));
        if (EPI == SAMQ_EPI_BIAS_GELU) {
          v0 = gelu_fast2(v0);
          v1 = gelu_fast2(v1);
        }
        const half2_t h0 = __builtin_convertvector(v0, half2_t), h1 = __builtin_convertvector(v1, half2_t);
        *(half4_t*)(ep_bytes + (32 * t + l32) * PITCH + (8 * j + 4 * hsel) * 2) = half4_t{h0.x, h0.y, h1.x, h1.y};
      }
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the slice image is in LDS
    const int srow0 = row_base + i * 32;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int pi = 4 * k + g, rb = pi & 1, c8 = pi >> 1;
      const uint32_t a = img + (8 * c8 + q) * PITCH + (16 * rb + 4 * pp) * 2;
      half4_t lo = ep_tr16(a), hi = ep_tr16(a + 4 * PITCH);
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(lo), "+v"(hi));
      const int row = srow0 + 16 * rb + i16;
      if (row < M)
        *(half8_t*)((_Float16*)Cout + (int64_t)row * ldc + col_base + 8 * c8) =
            half8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
  }
}

// Direct epilogue of a TRANSPOSED accumulator (VAR & 128: the MFMA is issued as W^T . A^T, so a
// lane's accumulator registers run along N): every lane holds G consecutive output columns of ONE
// row per register group and stores them straight from registers (G = 4: 8 bytes of fp16 or 16
// bytes of fp32, a 16-byte read-modify-write for the residual) -- no LDS staging round trip
// (ds_write_b32 per element + ds_read_b128 + waits in pp_epilogue).  v[q] = acc[q] * s[n] + b[n].
template <int EPI>
__device__ __forceinline__ void te_store4(const float4_t& acc, const float4_t& sc, const float4_t& bi, void* Cout,
                                          int64_t ldc, int M, int row, int col) {
  if (row >= M) return;
  float2_t v0 = __builtin_elementwise_fma((float2_t){acc[0], acc[1]}, (float2_t){sc[0], sc[1]}, (float2_t){bi[0], bi[1]});
  float2_t v1 = __builtin_elementwise_fma((float2_t){acc[2], acc[3]}, (float2_t){sc[2], sc[3]}, (float2_t){bi[2], bi[3]});
  if (EPI == SAMQ_EPI_BIAS_GELU) {
    v0 = gelu_fast2(v0);
    v1 = gelu_fast2(v1);
  }
  if (EPI == SAMQ_EPI_RESADD_F32 || EPI == SAMQ_EPI_F32) {
    float4_t* cp = (float4_t*)((float*)Cout + (int64_t)row * ldc + col);
    const float4_t v = {v0.x, v0.y, v1.x, v1.y};
    if (EPI == SAMQ_EPI_RESADD_F32) *cp = *cp + v; else *cp = v;
  } else {
    const half2_t h0 = __builtin_convertvector(v0, half2_t), h1 = __builtin_convertvector(v1, half2_t);
    *(half4_t*)((_Float16*)Cout + (int64_t)row * ldc + col) = half4_t{h0.x, h0.y, h1.x, h1.y};
  }
}

// Staged epilogue of TRANSPOSED 32x32 accumulators (VAR & 65536), f16 outputs: lane (l32, hsel) of
// tile (i, t) holds row 32 i + l32, columns 32 t + 8 j + 4 hsel .. +3 in register group j, so four
// consecutive columns convert to one 8-byte f16 group -> ONE ds_write_b64 per 4 values (the
// row-pitch 144 B keeps the 16 rows of a write group on distinct banks), then row-contiguous
// ds_read_b128 + 16-byte global stores.  The whole WM x WN wave tile is staged at once in the LDS
// the ring frees (f16: 18 KiB per wave).  vs pp_epilogue: 4x fewer LDS write instructions and half
// the staged bytes (f16 instead of f32).
template <int TM, int TN, int EPI>
__device__ __forceinline__ void te_staged_epilogue_f16(const float16_t (&acc)[TM][TN], const _Float16* __restrict__ scales,
                                                       const _Float16* __restrict__ bias, char* ep, void* Cout,
                                                       int64_t ldc, int M, int row_base, int col_base, int lane) {
  static_assert(EPI == SAMQ_EPI_BIAS || EPI == SAMQ_EPI_BIAS_GELU, "f16 outputs");
  constexpr int WN = TN * 32, PITCH = WN * 2 + 16, C8 = WN / 8;
  const int l32 = lane & 31, hsel = lane >> 5;
#pragma unroll
  for (int t = 0; t < TN; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int cl = 32 * t + 8 * j + 4 * hsel;
      const half4_t s4 = *(const half4_t*)(scales + col_base + cl);
      const half4_t b4 = bias ? *(const half4_t*)(bias + col_base + cl) : half4_t{0, 0, 0, 0};
      const float2_t sa = {(float)s4[0], (float)s4[1]}, sb = {(float)s4[2], (float)s4[3]};
      const float2_t ba = {(float)b4[0], (float)b4[1]}, bb = {(float)b4[2], (float)b4[3]};
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        float2_t v0 = __builtin_elementwise_fma((float2_t){acc[i][t][4 * j], acc[i][t][4 * j + 1]}, sa, ba);
        float2_t v1 = __builtin_elementwise_fma((float2_t){acc[i][t][4 * j + 2], acc[i][t][4 * j + 3]}, sb, bb);
        if (EPI == SAMQ_EPI_BIAS_GELU) {
          v0 = gelu_fast2(v0);
          v1 = gelu_fast2(v1);
        }
        const half2_t h0 = __builtin_convertvector(v0, half2_t), h1 = __builtin_convertvector(v1, half2_t);
        *(half4_t*)(ep + (32 * i + l32) * PITCH + cl * 2) = half4_t{h0.x, h0.y, h1.x, h1.y};
      }
    }
  __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the wave's own tile is in LDS
#pragma unroll
  for (int it = 0; it < TM * 32 * C8 / 64; ++it) {
    const int idx = it * 64 + lane;
    const int rl = idx / C8, c8 = idx % C8;
    const half8_t h = *(const half8_t*)(ep + rl * PITCH + c8 * 16);
    const int row = row_base + rl;
    if (row < M) *(half8_t*)((_Float16*)Cout + (int64_t)row * ldc + col_base + 8 * c8) = h;
  }
}

// ------------------------------------------------------------------ GEMM v6 (ping-pong, k-phases)
// As v5, but a phase is a K-PART of the tile over ALL of the wave's output tiles: phase p
// multiplies k16-steps [p*KPP, (p+1)*KPP) for TM x TN accumulators, so every phase reads its own
// A fragments (balanced LDS traffic, A registers for one k-part only) and unpacks its own slice
// of the packed B words (balanced VALU); the packed B words of the whole K tile are read in
// phase 0.  STAGES-slot ring: K tile kt+STAGES-1 is staged during tile kt (phases 1..NPH-1).
__device__ unsigned long long g_pp_stamps[8];   // timing experiments only (cfg 73)

// Tile of workgroup bid.  Default (xcd_remap): XCD x owns the x-th contiguous eighth of the
// row-major tile order, i.e. whole M-rows of tiles across ALL N tiles, so every XCD streams the
// whole packed weight (3.3 MB for lin1) through its 4 MB L2 once per round of 32 tiles -- the
// output stream evicts it in between (PMC: lin1 fetches 4.3x its algorithmic bytes).
// blocked2d (tiles_n even, tiles_m % 4 == 0, nwg % 8 == 0): XCD x owns the rectangle of M-rows
// [(x>>1) tm/4, +tm/4) x N-tiles [(x&1) tn/2, +tn/2): half of the weight per XCD stays resident
// while each A panel is read by the tn/2 concurrent tiles of its row.
__device__ __forceinline__ void xcd_tile(int bid, int tiles_m, int tiles_n, bool blocked2d, int& mt, int& nt) {
  const int nwg = tiles_m * tiles_n;
  if (blocked2d && (tiles_n & 1) == 0 && (tiles_m & 3) == 0) {
    const int x = bid & 7, k = bid >> 3, bm = tiles_m >> 2, bn = tiles_n >> 1;
    mt = (x >> 1) * bm + k / bn;
    nt = (x & 1) * bn + k % bn;
    return;
  }
  const int t = xcd_remap(bid, nwg);
  mt = t / tiles_n;
  nt = t % tiles_n;
}

// LDS budget of a ping-pong config (the kernel static_asserts its own SMEM against it).  The
// LayerNorm-fold consumer stages its workgroup's row partial sums (BM rows x K/64 float2) behind
// the epilogue slices and the (delta, rstd) table, in the LDS the ring leaves free once the main
// loop is done: LNF_KMAX is the largest consumer K that fits (samq_w4a16_gemm_lnf checks it).
template <int WAVES_M, int TM, int TN, int STAGES, int EPI, int VAR>
struct Pp2Lds {
  static constexpr int NW = 8, WM = TM * 32, WN = TN * 32, BM = WAVES_M * WM, BN = (NW / WAVES_M) * WN;
  static constexpr bool GR = (VAR & 512) != 0, M16 = (VAR & 16) != 0, GRR = GR && (VAR & (1 << 23)) != 0;
  static constexpr int GRB = GR && !GRR ? (BN * 2 / 16 + BN / 32) * 16 : 0;
  static constexpr int STAGE = BM * 128 + (BN / 32) * 1024 + GRB;
  static constexpr int EP_BYTES = M16 ? 16 * (WN + 4) * 4 : (WN > 64 ? 16 : 32) * WN * 4;
  static constexpr int RI_BYTES = (EPI == SAMQ_EPI_BIAS_LNF || EPI == SAMQ_EPI_GELU_LNF) ? BM * 8 : 0;
  static constexpr int SMEM = STAGES * STAGE > NW * EP_BYTES + RI_BYTES ? STAGES * STAGE : NW * EP_BYTES + RI_BYTES;
  static constexpr int LNF_KMAX = ((SMEM - NW * EP_BYTES - RI_BYTES) / (BM * 8)) * 64;
};

__host__ __device__ constexpr int pp2_pre(int p, int npw, int nph, int first) {   // pieces before phase p
  return p <= first ? 0 : (npw * (p - first)) / (nph - first);
}
template <int N>
__device__ __forceinline__ void vm_wait_le(int n) {   // s_waitcnt vmcnt(n) for a uniform n <= N
  if constexpr (N > 0) {
    if (n >= N) { vm_wait<N>(); return; }
    vm_wait_le<N - 1>(n);
  } else {
    vm_wait<0>();
  }
}

template <int WAVES_M, int TM, int TN, int NPH, int STAGES, int LA, int EPI, int VAR = 0>
__device__ __forceinline__
void pp2_tile(const _Float16* __restrict__ A, int64_t lda, const u32x4* __restrict__ Wp,
                    const _Float16* __restrict__ scales, const uint32_t* __restrict__ qzeros,
                    const _Float16* __restrict__ bias, void* __restrict__ Cout, int64_t ldc,
                    int M, int N, int K, int kpg, LnfArgs lnf, int bid) {
  constexpr int NW = 8;
  constexpr int WAVES_N = NW / WAVES_M;
  constexpr int WM = TM * 32, WN = TN * 32;
  constexpr int BM = WAVES_M * WM, BN = WAVES_N * WN;
  constexpr int BK = 64, ROWB = BK * 2;
  constexpr int A_BYTES = BM * ROWB;
  // VAR & 512: grouped weights (groupsize = 64 kpg < K).  The K tile that starts a group carries
  // one more LDS-DMA piece, the group row of the whole tile: BN fp16 scales (lanes 0 .. BN/8-1) and
  // BN/8 packed zero words (the next BN/32 lanes; the rest idle), GRB bytes behind the B pieces.
  // Wave 0 issues it (compile-time slot NPW - 1, in the last phase); every wave reads its columns
  // of tile kt+1's row in the MFMA half of tile kt's last phase -- after the barrier that follows
  // every wave's retire wait for tile kt+1, wave 0's included -- and converts them in tile kt+1's
  // phase 0.  The unpack scales the exact integers once in fp16, fp16((q - zp) * s) (the v3
  // kernels' semantics); the epilogue's per-channel scale is 1.
  constexpr bool GR = (VAR & 512) != 0;
  // VAR & (1 << 23) (with GR), register rows: each lane loads its own columns' group scale and zero
  // word straight into VGPRs (global loads in inline asm, so the compiler adds no wait of its own --
  // its waitcnt pass would wait vmcnt(0) on the loop-carried registers, round 3), issued in the
  // MFMA half of a group's first K tile for the NEXT group, before that phase's LDS-DMA pieces.
  // They count in the ring's vmcnt arithmetic (gl below) and a counted wait at the next group's
  // start retires them.  The ring then carries no group row: 4 slots / lookahead 3 like the
  // per-channel cfg 57, instead of 3 / 2 (4 x 40 KiB fill the 160 KiB LDS).
  constexpr bool GRR = GR && (VAR & (1 << 23)) != 0;
  // timing-only (tuning build): VAR & 1024 skips the fp16 group scaling, VAR & 2048 the group row
  constexpr bool G_NOSCALE = (VAR & 1024) != 0, G_NOROW = (VAR & 2048) != 0;
  constexpr int GLS = BN * 2 / 16, GLZ = BN / 32;   // lanes carrying scales / zero words
  static_assert(!GR || GLS + GLZ <= 64, "group row: one lane per 16 bytes");
  constexpr bool GROW = GR && !GRR;                   // the group row rides in the ring
  constexpr int GRB = GROW ? (GLS + GLZ) * 16 : 0;
  constexpr int NA = BM / 8, NB = BN / 32, NT = NA + NB + (GROW ? 1 : 0);
  constexpr int NGL = GRR ? 2 * TN * ((VAR & 16) ? 2 : 1) : 0;   // GRR: loads per lane per group
  constexpr int NPW = (NT + NW - 1) / NW;
  constexpr int STAGE = A_BYTES + NB * 1024 + GRB;
  constexpr int KPP = 4 / NPH;
  // K tile kt+LA is staged during tile kt (slot of tile kt+LA-STAGES, last read during tile kt-1
  // at the latest), its pieces issued behind the MFMA bursts: a wave's MFMA half of phase 0
  // starts after the barrier that ends every read of tile kt-1 (both groups' load halves of
  // tile kt-1's last phase lie before it, and their lgkmcnt waits precede their MFMAs), so all
  // phases may restage (WAR).  The retire wait for tile kt+1 sits in the load half of the last
  // phase, before the barrier after which the first group reads it (RAW).
  // VAR & 32: all of tile kt+LA's pieces are issued in the LOAD half of tile kt's last phase,
  // right after the retire wait for tile kt+1 and the phase's A fragment reads (the MFMA halves
  // carry no DMA issue).  WAR: that segment starts two barriers after the partner group's
  // lgkmcnt wait on its last reads of tile kt-1 (whose slot is restaged), so every read of the
  // slot has completed.
  constexpr bool DMA_LOAD = (VAR & 32) != 0;
  static_assert(!(GR && DMA_LOAD), "grouped ping-pong: DMA behind the MFMA bursts only");
  constexpr int PRE_LAST = DMA_LOAD ? 0 : pp2_pre(NPH - 1, NPW, NPH, 0);
  // VAR & 16: v_mfma_f32_16x16x32_f16 fragments (same tile, LDS bytes and unpack count; the chip
  // holds a higher clock on this shape under load, MI355X_MICROARCH.md 'DVFS give-back' item 7)
  constexpr bool M16 = (VAR & 16) != 0;
  // VAR & 65536: transposed accumulators + the LDS-staged f16 epilogue (te_staged_epilogue_f16)
  constexpr bool TES = (VAR & 65536) != 0;
  static_assert(!TES || (!M16 && !GR && (EPI == SAMQ_EPI_BIAS || EPI == SAMQ_EPI_BIAS_GELU)), "TES: f16 outputs, 32x32");
  static_assert(!TES || 8 * TM * 32 * (TN * 64 + 16) <= 163840, "TES staging");
  constexpr bool TE = (VAR & 128) != 0 || TES;   // transposed accumulators (+ direct epilogue te_store4)
  // VAR & 16384: LDS-DMA pieces spread through the MFMA burst (see the MFMA half)
  constexpr bool DMA_SPREAD = (VAR & 16384) != 0;
  static_assert(!DMA_SPREAD || !(DMA_LOAD || TE || (VAR & 2)), "DMA spread: product MFMA halves only");
  constexpr int KS32 = 2 / NPH;                  // M16: k32 steps per phase
  constexpr int EP_ROWS = WN > 64 ? 16 : 32;
  constexpr int EP_BYTES = M16 ? 16 * (WN + 4) * 4 : EP_ROWS * WN * 4;
  // LN-fold consumers: per-wave (delta, rstd) of its WM rows behind the epilogue slices
  constexpr int RI_BYTES = lnf_consumer(EPI) ? BM * 8 : 0;
  constexpr int SMEM = STAGES * STAGE > NW * EP_BYTES + RI_BYTES ? STAGES * STAGE : NW * EP_BYTES + RI_BYTES;
  static_assert(SMEM == Pp2Lds<WAVES_M, TM, TN, STAGES, EPI, VAR>::SMEM, "Pp2Lds mirrors this layout");
  static_assert(!M16 || NPH <= 2, "M16: one or two phases per K tile");
  static_assert(NPH >= 1 && 4 % NPH == 0, "phases");
  static_assert(LA >= 2 && LA < STAGES, "ring");
  static_assert((LA - 2) * (NPW + NGL) + PRE_LAST + NGL <= 63, "vmcnt");
  static_assert(!GRR || 3 * NPW <= 63, "vmcnt (group start)");
  static_assert(SMEM <= 160 * 1024, "LDS");

  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  // VAR & 4096 (and GR): the wave index -- hence piece choices and addresses -- in an SGPR
  constexpr bool RFL = GR || (VAR & 4096) != 0;
  const int wave = RFL ? __builtin_amdgcn_readfirstlane(tid >> 6) : tid >> 6;
  const int wm = wave / WAVES_N;
  const int wn = wave % WAVES_N;
  const int grp = wave >> 2;
  const int tiles_n = N / BN;
  const int tiles_m = (M + BM - 1) / BM;
  int m0, n0;
  xcd_tile(bid, tiles_m, tiles_n, (VAR & 64) != 0, m0, n0);
  m0 *= BM;
  n0 *= BN;
  const int kt_count = K / BK;

  const char* src[NPW];
  int dst[NPW];
  int step[NPW];
  // VAR & 8192 (and GR): pieces dealt j = i * 8 + wave (interleaved) instead of wave * NPW + i;
  // GR: the A / B pieces fill slots i < NPW - 1; slot NPW - 1 of wave 0 is the group row
  constexpr bool ILV = GR || (VAR & 8192) != 0;
  static_assert(!GROW || ((NA + NB) % NW == 0 && NPW == (NA + NB) / NW + 1), "group row slot");
  static_assert(!GROW || pp2_pre(NPH - 1, NPW, NPH, 0) <= NPW - 1, "group row issued in the last phase");
#pragma unroll
  for (int i = 0; i < NPW; ++i) {
    int j = ILV ? i * NW + wave : wave * NPW + i;
    j = j < NT ? j : NT - 1;
    if (GROW && i == NPW - 1) {
      if (lane < GLS) {
        src[i] = (const char*)(scales + n0 + 8 * lane);
        step[i] = N * 2;
      } else {
        const int l = lane - GLS < GLZ ? lane - GLS : 0;
        src[i] = (const char*)(qzeros + n0 / 8 + 4 * l);
        step[i] = (N / 8) * 4;
      }
      dst[i] = A_BYTES + NB * 1024;
    } else if (j < NA) {
      const int row = j * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      int gr = m0 + row;
      gr = gr < M ? gr : M - 1;
      src[i] = (const char*)(A + (int64_t)gr * lda + c * 8);
      dst[i] = j * 1024;
      step[i] = BK * 2;
    } else {
      const int nt = n0 / 32 + (j - NA);
      src[i] = (const char*)(Wp + ((int64_t)nt * kt_count) * 64 + lane);
      dst[i] = A_BYTES + (j - NA) * 1024;
      step[i] = 64 * 16;
    }
  }
  auto issue = [&](int kt, int slot, int i0, int i1) {
#pragma unroll
    for (int i = 0; i < NPW; ++i)
      if (i >= i0 && i < i1) {
        if (GROW && i == NPW - 1) {
          // wave 0, and only for a K tile that starts a group (uniform: wave is an SGPR)
          if (!G_NOROW && wave == 0 && kt % kpg == 0) {
            if (lane < GLS + GLZ)
              __builtin_amdgcn_global_load_lds((const SAMQ_GLOBAL void*)(src[i] + (int64_t)(kt / kpg) * step[i]),
                                               (SAMQ_LDS void*)(smem + slot * STAGE + dst[i]), 16, 0, 0);
          }
        } else {
          __builtin_amdgcn_global_load_lds((const SAMQ_GLOBAL void*)(src[i] + (int64_t)kt * step[i]),
                                           (SAMQ_LDS void*)(smem + slot * STAGE + dst[i]), 16, 0, 0);
        }
      }
  };
  // GR: the raw group row values of this lane's columns (read after the retire wait of their tile)
  // and the fp16 scale splats (set from them where a group starts)
  half2_t gsc[TN], gsc16[TN][2];
  uint32_t graw_s[TN][2] = {}, graw_z[TN][2] = {};
  auto gread = [&](int slot_) {
    const char* gp = smem + slot_ * STAGE + A_BYTES + NB * 1024;
#pragma unroll
    for (int t = 0; t < TN; ++t)
#pragma unroll
      for (int h = 0; h < (M16 ? 2 : 1); ++h) {
        const int cl = wn * WN + (M16 ? 32 * t + 16 * h + (lane & 15) : 32 * t + (lane & 31));
        graw_s[t][h] = *(const uint16_t*)(gp + 2 * cl);
        graw_z[t][h] = *(const uint32_t*)(gp + BN * 2 + 4 * (cl >> 3)) >> (4 * (cl & 7));
      }
  };
  // GR: LDS-DMA pieces this wave issues for K tile t (wave 0 adds the group row where a group starts)
  auto npieces = [&](int t) -> int { return GROW ? NPW - 1 + (wave == 0 && t % kpg == 0 ? 1 : 0) : NPW; };
  // GRR: the register-row loads of a group are issued in the MFMA half of the previous group's first
  // tile t0, right before K tile t0 + LA's pieces; gl(kt + j) = such loads precede tile kt + j's
  // pieces (t0 = kt + j - LA starts a group and a group follows it).  t0 % kpg from the position
  // gk of tile kt in its group: (gk + j - LA) mod kpg, at most LA - 2 additions of kpg -- not a
  // loop over t0 (that SALU chain sat in every last-phase load half: lin2, 80 K tiles, +38 %)
  auto gl = [&](int kt_, int j, int gk_) -> bool {
    if (!GRR) return false;
    const int t0 = kt_ + j - LA;
    if (t0 < 0 || t0 + kpg >= kt_count) return false;
    int r = gk_ + j - LA;
    while (r < 0) r += kpg;
    return r == 0;
  };
  auto gload = [&](int gi) {   // GRR: this lane's columns of group gi into graw_s / graw_z (no wait)
#pragma unroll
    for (int t = 0; t < TN; ++t)
#pragma unroll
      for (int h = 0; h < (M16 ? 2 : 1); ++h) {
        const int c = n0 + wn * WN + (M16 ? 32 * t + 16 * h + (lane & 15) : 32 * t + (lane & 31));
        const _Float16* sp = scales + (int64_t)gi * N + c;
        const uint32_t* zp = qzeros + (int64_t)gi * (N / 8) + (c >> 3);
        asm volatile("global_load_ushort %0, %1, off" : "+v"(graw_s[t][h]) : "v"(sp));
        asm volatile("global_load_dword %0, %1, off" : "+v"(graw_z[t][h]) : "v"(zp));
      }
  };

  int col[TN];
  W4Zero zc[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    col[t] = n0 + wn * WN + t * 32 + (lane & 31);
    const uint32_t zw = qzeros[col[t] >> 3];
    zc[t].set((int)((zw >> (4 * (col[t] & 7))) & 0xFu) + 1);
  }
  W4Unpack ku;
  ku.init();

  float16_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int hsel = lane >> 5;
  int a_off[TM], a_swz[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int rr = wm * WM + i * 32 + (lane & 31);
    a_off[i] = rr * ROWB;
    a_swz[i] = (rr >> 1) & 7;
  }

  // M16 state: 16-row tiles i, column halves h of each 32-column block t; lane (ql, g16) holds
  // column 32t + 16h + ql and k = 32 s + 8 g16 .. +7, whose packed word (layout 1: column c,
  // k chunk kb at word kb / 2 of lane c + 32 (kb & 1)) is word 2 s + (g16 >> 1) of lane
  // 16h + ql + 32 (g16 & 1) in the staged B block
  const int ql = lane & 15, g16 = lane >> 4;
  float4_t acc16[M16 ? 2 * TM : 1][TN][2];
  W4Zero zc16[TN][2];
  int a_off16[M16 ? 2 * TM : 1], a_swz16[M16 ? 2 * TM : 1];
  if constexpr (M16) {
#pragma unroll
    for (int i = 0; i < 2 * TM; ++i) {
#pragma unroll
      for (int t = 0; t < TN; ++t)
#pragma unroll
        for (int h = 0; h < 2; ++h) acc16[i][t][h] = float4_t{0.f, 0.f, 0.f, 0.f};
      const int rr = wm * WM + i * 16 + ql;
      a_off16[i] = rr * ROWB;
      a_swz16[i] = (rr >> 1) & 7;
    }
#pragma unroll
    for (int t = 0; t < TN; ++t)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = n0 + wn * WN + 32 * t + 16 * h + ql;
        zc16[t][h].set((int)((qzeros[c >> 3] >> (4 * (c & 7))) & 0xFu) + 1);
      }
  }

  // VAR & (1 << 21): the epilogue's per-channel scale / bias of this lane's columns loaded before
  // the prologue's LDS-DMA pieces (the prologue's retire wait covers them) and kept in VGPRs over
  // the main loop, instead of loaded after it, where their latency sits behind the epilogue barrier
  constexpr bool EARLY_EP = (VAR & (1 << 21)) != 0;
  static_assert(!EARLY_EP || !(GR || TE || lnf_consumer(EPI) || lnf_producer(EPI)), "early epilogue operands");
  constexpr int NEC = EARLY_EP ? (M16 ? 2 * TN : TN) : 1;
  _Float16 esc[NEC], ebi[NEC];
  if constexpr (EARLY_EP) {
#pragma unroll
    for (int e = 0; e < NEC; ++e) {
      const int c = M16 ? n0 + wn * WN + 32 * (e >> 1) + 16 * (e & 1) + (lane & 15) : col[e];
      esc[e] = scales[c];
      ebi[e] = bias ? bias[c] : (_Float16)0.0f;
    }
  }
  // VAR & 256: static priority instead of per-segment flips -- the second-dispatched half (group 1,
  // the arbitration loser) at prio 1 for the whole loop (MI355X_MICROARCH.md two-waves item 4)
  if ((VAR & 256) && grp) __builtin_amdgcn_s_setprio(1);
  // ---- prologue: K tiles 0 .. LA-1 in flight, tile 0 retired + visible; group 1 lags a barrier
  const int pro = kt_count < LA ? kt_count : LA;
  if (GRR) gload(0);   // older than every piece: the prologue's retire wait for tile 0 covers it
#pragma unroll
  for (int j = 0; j < LA; ++j)
    if (j < pro) issue(j, j, 0, NPW);
  {
    int newer = 0;
#pragma unroll
    for (int j = 1; j < LA; ++j) newer += j < pro ? npieces(j) : 0;
    vm_wait_le<(LA - 1) * NPW>(newer);
  }
  __builtin_amdgcn_s_barrier();
  if (GROW && !G_NOROW) gread(0);   // tile 0's row: wave 0's retire wait precedes the barrier above
  if (grp) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  // VAR & 4 (timing experiment): per-wave cycles of the load half, barrier 1, MFMA half, barrier 2
  unsigned long long ph[4] = {0, 0, 0, 0}, tprev = 0;
  auto stamp = [&](int k) {
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    if (tprev) ph[k] += t - tprev;
    tprev = t;
  };
  int slot = 0;
  int gk = 0;   // GR: K tiles since the current group's first
  int gidx = 0; // GR: the current group
  for (int kt = 0; kt < kt_count; ++kt) {
    const char* st = smem + slot * STAGE;
    const int ahead = kt + LA;
    const bool pf = ahead < kt_count && !(VAR & 1);   // VAR & 1: timing-only, no restaging
    const int sa = slot + LA >= STAGES ? slot + LA - STAGES : slot + LA;   // (kt + LA) % STAGES
    u32x4 bw[TN];
    uint32_t bw16[TN][2][2];
    static_for<NPH>([&](auto pc_) {   // phases: p a constant (folds the DMA piece schedule)
      constexpr int p = decltype(pc_)::value;
      // ---------------- load half
      if (p == NPH - 1 && kt + 1 < kt_count) {
        // K tile kt+1 retired: newer = whole tiles kt+2 .. kt+LA-1 + this tile's pieces so far.
        // Per-channel steady state (every later tile whole, restaging on): a compile-time count --
        // the runtime form is a ~40-SALU / 15-branch decision tree on the load half's stream
        if (!GR && pf && kt + LA < kt_count) {
          vm_wait<(LA - 2) * NPW + PRE_LAST>();
        } else if (GRR && LA == 3 && NPH > 1 && kpg == 2 && pf && kt + LA < kt_count) {
          // GRR, two K tiles per group (G = 128): of the two tiles kt - 1, kt exactly one starts a
          // group, so one set of register-row loads is newer -- a constant count, no decision tree
          vm_wait<(LA - 2) * NPW + PRE_LAST + NGL>();
        } else {
          int newer = pf ? PRE_LAST : 0;
          if (NPH > 1 && GRR && gk == 0 && kt + kpg < kt_count) newer += NGL;   // gl(ahead)   // this tile's register-row loads (phase 0)
#pragma unroll
          for (int j = 2; j < LA; ++j) newer += (kt + j < kt_count ? npieces(kt + j) : 0) + (gl(kt, j, gk) ? NGL : 0);
          vm_wait_le<(LA - 2) * (NPW + NGL) + PRE_LAST + NGL>(newer);
        }
      }
      if (GR && !G_NOROW && p == 0 && gk == 0) {   // first K tile of a group: its scale / zero splats
        if constexpr (GRR) {
          // the group's loads were issued kpg tiles ago, before the pieces of tiles kt - kpg + LA ..
          // kt + LA - 1 (those that exist); everything older has retired once at most that many
          // remain.  (kt == 0: the prologue's wait covered them.)  The empty asm re-defines the
          // registers after the wait, so nothing reading them is scheduled above it.
          if (kt > 0) {
            int left = kt_count - (kt - kpg + LA);
            left = (VAR & 1) || left < 0 ? 0 : left > kpg ? kpg : left;
            if (kpg == 2 && left == 2)
              vm_wait<2 * NPW>();
            else
              vm_wait_le<3 * NPW>(left * NPW);
          }
#pragma unroll
          for (int t = 0; t < TN; ++t)
#pragma unroll
            for (int h = 0; h < (M16 ? 2 : 1); ++h) {
              asm volatile("" : "+v"(graw_s[t][h]), "+v"(graw_z[t][h]));
              graw_s[t][h] &= 0xFFFFu;
              graw_z[t][h] >>= 4 * ((n0 + wn * WN + (M16 ? 32 * t + 16 * h + (lane & 15) : 32 * t + (lane & 31))) & 7);
            }
        }
#pragma unroll
        for (int t = 0; t < TN; ++t)
#pragma unroll
          for (int h = 0; h < (M16 ? 2 : 1); ++h) {
            // fp16 bits: 1024 + zp = 0x6400 + zp, 64 + zp = 0x5400 + 16 zp (exact), splatted
            const uint32_t zp = (graw_z[t][h] & 0xFu) + 1u;
            W4Zero z;
            z.z1024 = __builtin_bit_cast(half2_t, (0x6400u + zp) * 0x10001u);
            z.z64 = __builtin_bit_cast(half2_t, (0x5400u + 16u * zp) * 0x10001u);
            const half2_t sc2 = __builtin_bit_cast(half2_t, graw_s[t][h] * 0x10001u);
            if constexpr (M16) { zc16[t][h] = z; gsc16[t][h] = sc2; } else { zc[t] = z; gsc[t] = sc2; }
          }
      }
      if (M16 && p == 0) {
#pragma unroll
        for (int t = 0; t < TN; ++t)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const char* bp = st + A_BYTES + (wn * TN + t) * 1024 + (16 * h + ql + 32 * (g16 & 1)) * 16 + 4 * (g16 >> 1);
            bw16[t][h][0] = *(const uint32_t*)bp;         // k32 step 0
            bw16[t][h][1] = *(const uint32_t*)(bp + 8);   // k32 step 1
          }
      } else if (p == 0) {
#pragma unroll
        for (int t = 0; t < TN; ++t) bw[t] = *(const u32x4*)(st + A_BYTES + (wn * TN + t) * 1024 + lane * 16);
      }
      half8_t af16[M16 ? 2 * TM : 1][KS32], bf16[TN][2][KS32];
      if constexpr (M16) {
#pragma unroll
        for (int s = 0; s < KS32; ++s) {
          const int k32 = p * KS32 + s;
#pragma unroll
          for (int i = 0; i < 2 * TM; ++i)
            af16[i][s] = *(const half8_t*)(st + a_off16[i] + (((4 * k32 + g16) ^ a_swz16[i]) << 4));
#pragma unroll
          for (int t = 0; t < TN; ++t)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              bf16[t][h][s] = w4_unpack(bw16[t][h][k32], ku, zc16[t][h]);
              if (GR && !G_NOSCALE) bf16[t][h][s] = scale8(bf16[t][h][s], gsc16[t][h]);
            }
        }
      }
      half8_t af[TM][KPP];
      half8_t bf[TN][KPP];
      if constexpr (!M16) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int s = 0; s < KPP; ++s)
            af[i][s] = *(const half8_t*)(st + a_off[i] + (((2 * (p * KPP + s) + hsel) ^ a_swz[i]) << 4));
#pragma unroll
        for (int t = 0; t < TN; ++t)
#pragma unroll
          for (int s = 0; s < KPP; ++s) {
            bf[t][s] = w4_unpack(bw[t][p * KPP + s], ku, zc[t]);
            if (GR && !G_NOSCALE) bf[t][s] = scale8(bf[t][s], gsc[t]);
          }
      }
      if (DMA_LOAD && pf && p == NPH - 1) issue(ahead, sa, 0, NPW);
      if (VAR & 4) stamp(0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (VAR & 4) stamp(1);
      // ---------------- MFMA half
      if (!(VAR & 256)) __builtin_amdgcn_s_setprio(1);
      if constexpr (DMA_SPREAD) {
        // the phase's LDS-DMA pieces spread through the MFMA burst (one after every NMF / np
        // MFMAs) instead of after it: issued after the last MFMA they queue behind the other
        // MFMA-half waves' pieces in the TA while the MFMA pipe drains, and the partner group
        // waits at the barrier for that tail (pp2 stamps: MFMA half ~690 cycles for 512)
        constexpr int P0 = pp2_pre(p, NPW, NPH, 0), NP = pp2_pre(p + 1, NPW, NPH, 0) - P0;
        constexpr int NMF = M16 ? KS32 * 2 * TM * TN * 2 : KPP * TM * TN;
        static_for<NMF>([&](auto qc) {
          constexpr int q = decltype(qc)::value;
          if constexpr (M16) {
            constexpr int s = q / (2 * TM * TN * 2), i = (q / (TN * 2)) % (2 * TM), t = (q / 2) % TN, h = q % 2;
            acc16[i][t][h] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af16[i][s], bf16[t][h][s], acc16[i][t][h], 0, 0, 0);
          } else {
            constexpr int s = q / (TM * TN), i = (q / TN) % TM, t = q % TN;
            acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i][s], bf[t][s], acc[i][t], 0, 0, 0);
          }
          static_for<NPW>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            if constexpr (k < NP && q + 1 == ((2 * k + 1) * NMF) / (2 * NP)) {
              __builtin_amdgcn_sched_barrier(0);
              if (pf) issue(ahead, sa, P0 + k, P0 + k + 1);
              __builtin_amdgcn_sched_barrier(0);
            }
          });
        });
      } else if constexpr (M16) {
#pragma unroll
        for (int s = 0; s < KS32; ++s)
#pragma unroll
          for (int i = 0; i < 2 * TM; ++i)
#pragma unroll
            for (int t = 0; t < TN; ++t)
#pragma unroll
              for (int h = 0; h < 2; ++h)
                acc16[i][t][h] = TE ? __builtin_amdgcn_mfma_f32_16x16x32_f16(bf16[t][h][s], af16[i][s], acc16[i][t][h], 0, 0, 0)
                                    : __builtin_amdgcn_mfma_f32_16x16x32_f16(af16[i][s], bf16[t][h][s], acc16[i][t][h], 0, 0, 0);
      } else {
#pragma unroll
        for (int s = 0; s < KPP; ++s)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int t = 0; t < TN; ++t) {
              if (VAR & 2) {   // timing-only: no MFMA
                acc[i][t][0] += (float)af[i][s][0] * (float)bf[t][s][1];
              } else {
                acc[i][t] = TE ? __builtin_amdgcn_mfma_f32_32x32x16_f16(bf[t][s], af[i][s], acc[i][t], 0, 0, 0)
                               : __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i][s], bf[t][s], acc[i][t], 0, 0, 0);
              }
            }
      }
      // the next-next tile's LDS-DMA pieces behind this MFMA burst (the wave would only wait at
      // the barrier otherwise; WAR-safe in every phase: see header)
      // GRR: the next group's register rows, older than tile ahead's pieces (gl(ahead))
      if (GRR && p == 0 && gk == 0 && kt + kpg < kt_count) gload(gidx + 1);   // == gl(ahead)
      if (pf && !DMA_LOAD && !DMA_SPREAD) issue(ahead, sa, pp2_pre(p, NPW, NPH, 0), pp2_pre(p + 1, NPW, NPH, 0));
      // GR: tile kt+1 starts a group -> its row into registers (every wave's retire wait for tile
      // kt+1, wave 0's included, precedes the barrier that opened this MFMA half)
      if (GROW && !G_NOROW && p == NPH - 1 && kt + 1 < kt_count && gk + 1 == kpg)
        gread(slot + 1 == STAGES ? 0 : slot + 1);
      if (VAR & 4) stamp(2);
      if (!(VAR & 256)) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (VAR & 4) stamp(3);
    });
    slot = slot == STAGES - 1 ? 0 : slot + 1;
    if (GR) {
      gidx += gk + 1 == kpg ? 1 : 0;
      gk = gk + 1 == kpg ? 0 : gk + 1;
    }
  }
  if (!grp) __builtin_amdgcn_s_barrier();   // balance group 1's extra barrier
  if ((VAR & 4) && lane == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) atomicAdd(&g_pp_stamps[k], ph[k]);
    atomicAdd(&g_pp_stamps[4], (unsigned long long)kt_count * NPH);
  }

  if constexpr ((VAR & 32768) != 0) {   // timing-only (tuning build): no epilogue -- keeps the sums alive
    float z = 0.f;
    if constexpr (M16) {
#pragma unroll
      for (int i = 0; i < 2 * TM; ++i)
#pragma unroll
        for (int t = 0; t < TN; ++t) z += acc16[i][t][0][0] + acc16[i][t][1][3];
    } else {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int t = 0; t < TN; ++t) z += acc[i][t][0] + acc[i][t][15];
    }
    if (z == 1234.5f) ((float*)Cout)[tid] = z;
    return;
  }
  if constexpr (M16 && TE) {
    // lane (ql, g16) holds row 16 i + ql, columns 32 t + 16 h + 4 g16 .. +3 of the wave's tile
#pragma unroll
    for (int t = 0; t < TN; ++t)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = n0 + wn * WN + 32 * t + 16 * h + 4 * g16;
        const half4_t s4 = *(const half4_t*)(scales + c);
        const half4_t b4 = bias ? *(const half4_t*)(bias + c) : half4_t{0, 0, 0, 0};
        const float4_t sc = {(float)s4[0], (float)s4[1], (float)s4[2], (float)s4[3]};
        const float4_t bi = {(float)b4[0], (float)b4[1], (float)b4[2], (float)b4[3]};
#pragma unroll
        for (int i = 0; i < 2 * TM; ++i)
          te_store4<EPI>(acc16[i][t][h], sc, bi, Cout, ldc, M, m0 + wm * WM + 16 * i + ql, c);
      }
    return;
  }
  if constexpr (TES) {
    constexpr int WB = TM * 32 * (TN * 64 + 16);
    __syncthreads();   // every wave is done with the ring
    te_staged_epilogue_f16<TM, TN, EPI>(acc, scales, bias, smem + wave * WB, Cout, ldc, M, m0 + wm * WM, n0 + wn * WN,
                                        lane);
    return;
  }
  if constexpr (!M16 && TE) {
    // lane (l32, hsel) holds row 32 i + l32, columns 32 t + 8 j + 4 hsel .. +3 in register group j
#pragma unroll
    for (int t = 0; t < TN; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = n0 + wn * WN + 32 * t + 8 * j + 4 * hsel;
        const half4_t s4 = *(const half4_t*)(scales + c);
        const half4_t b4 = bias ? *(const half4_t*)(bias + c) : half4_t{0, 0, 0, 0};
        const float4_t sc = {(float)s4[0], (float)s4[1], (float)s4[2], (float)s4[3]};
        const float4_t bi = {(float)b4[0], (float)b4[1], (float)b4[2], (float)b4[3]};
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const float4_t a = {acc[i][t][4 * j], acc[i][t][4 * j + 1], acc[i][t][4 * j + 2], acc[i][t][4 * j + 3]};
          te_store4<EPI>(a, sc, bi, Cout, ldc, M, m0 + wm * WM + 32 * i + (lane & 31), c);
        }
      }
    return;
  }
  if constexpr (M16) {
    float csc16[TN][2], cb16[TN][2];
#pragma unroll
    for (int t = 0; t < TN; ++t)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = n0 + wn * WN + 32 * t + 16 * h + ql;
        csc16[t][h] = EARLY_EP ? (float)esc[EARLY_EP ? 2 * t + h : 0] : GR ? 1.0f : (float)scales[c];
        cb16[t][h] = EARLY_EP ? (float)ebi[EARLY_EP ? 2 * t + h : 0] : bias ? (float)bias[c] : 0.0f;
      }
    __syncthreads();
    float2_t* rowinfo = (float2_t*)(smem + NW * EP_BYTES) + wm * WM;
    lnf.bias = bias;
    if constexpr (lnf_consumer(EPI))
      lnf_rowinfo_wg<BM, NW>(lnf, (float2_t*)(smem + NW * EP_BYTES), smem + NW * EP_BYTES + RI_BYTES, M, m0, n0 == 0,
                             wave, lane);
    pp_epilogue16<2 * TM, TN, EPI>(acc16, csc16, cb16, smem + wave * EP_BYTES, Cout, ldc, M, m0 + wm * WM,
                                   n0 + wn * WN, lane, lnf, N, rowinfo);
    return;
  }
  float csc[TN], cb[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    csc[t] = EARLY_EP ? (float)esc[EARLY_EP ? t : 0] : GR ? 1.0f : (float)scales[col[t]];
    cb[t] = EARLY_EP ? (float)ebi[EARLY_EP ? t : 0] : bias ? (float)bias[col[t]] : 0.0f;
  }
  __syncthreads();
  float2_t* rowinfo = (float2_t*)(smem + NW * EP_BYTES) + wm * WM;
  lnf.bias = bias;
  if constexpr (lnf_consumer(EPI))
    lnf_rowinfo_wg<BM, NW>(lnf, (float2_t*)(smem + NW * EP_BYTES), smem + NW * EP_BYTES + RI_BYTES, M, m0, n0 == 0,
                           wave, lane);
  if constexpr ((VAR & (1 << 22)) != 0) {
    static_assert(EPI == SAMQ_EPI_BIAS || EPI == SAMQ_EPI_BIAS_GELU, "transposed f16 staging: f16 outputs");
    static_assert(EP_BYTES >= 64 * 72, "transposed f16 staging image");
    pp_epilogue_f16t<TM, TN, EPI>(acc, csc, cb, smem + wave * EP_BYTES, Cout, ldc, M, m0 + wm * WM, n0 + wn * WN, lane);
    return;
  }
  pp_epilogue<TM, TN, EP_ROWS, EPI, (VAR >> 17) & 3>(acc, csc, cb, smem + wave * EP_BYTES, Cout, ldc, M, m0 + wm * WM,
                                                     n0 + wn * WN, lane, lnf, N, rowinfo);
}

// The ping-pong GEMM kernel: one tile per workgroup, or (VAR & (1 << 20), persistent) a grid of at
// most one workgroup per CU looping over the tiles t = blockIdx.x, + gridDim.x, ... -- the tile's
// epilogue stores drain while the next tile's prologue DMA and first K tiles run (a one-tile
// workgroup holds its CU until its stores are acknowledged).  gridDim.x % 8 == 0 keeps every tile
// on the XCD its one-tile launch would give it (xcd_tile's t % 8 map).
template <int WAVES_M, int TM, int TN, int NPH, int STAGES, int LA, int EPI, int VAR = 0>
__global__ __launch_bounds__(512, 1)
void w4a16_gemm_pp2(const _Float16* __restrict__ A, int64_t lda, const u32x4* __restrict__ Wp,
                    const _Float16* __restrict__ scales, const uint32_t* __restrict__ qzeros,
                    const _Float16* __restrict__ bias, void* __restrict__ Cout, int64_t ldc,
                    int M, int N, int K, int kpg, LnfArgs lnf) {
  if constexpr ((VAR & (1 << 20)) != 0) {
    constexpr int BM = WAVES_M * TM * 32, BN = (8 / WAVES_M) * TN * 32;
    const int ntiles = ((M + BM - 1) / BM) * (N / BN);
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
      pp2_tile<WAVES_M, TM, TN, NPH, STAGES, LA, EPI, VAR>(A, lda, Wp, scales, qzeros, bias, Cout, ldc, M, N, K, kpg,
                                                           lnf, t);
      __syncthreads();   // the epilogue's LDS reads before the next tile's ring DMA
    }
  } else {
    pp2_tile<WAVES_M, TM, TN, NPH, STAGES, LA, EPI, VAR>(A, lda, Wp, scales, qzeros, bias, Cout, ldc, M, N, K, kpg, lnf,
                                                         blockIdx.x);
  }
}

// ------------------------------------------------------------------ dispatch
struct GemmArgs {
  const _Float16* A; int64_t lda; const u32x4* Wp; const _Float16* scales; const uint32_t* qzeros;
  const _Float16* bias; void* C; int64_t ldc; int M, N, K, groupsize;
  LnfArgs lnf;
};

template <int BM, int BN, int WMW, int WNW, int EPI, bool GR, int VAR = 1>
static int launch_cfg(const GemmArgs& a, hipStream_t st) {
  const int nwg = ((a.M + BM - 1) / BM) * (a.N / BN);
  hipLaunchKernelGGL((w4a16_gemm_kernel<BM, BN, WMW, WNW, EPI, GR, VAR>), dim3(nwg), dim3(64 * WMW * WNW), 0, st,
                     a.A, a.lda, a.Wp, a.scales, a.qzeros, a.bias, a.C, a.ldc, a.M, a.N, a.K, a.groupsize);
  SAMQ_LAUNCH_CHECK("w4a16_gemm launch");
  return SAMQ_OK;
}

template <int BM, int BN, int WMW, int WNW, int EPI, bool GR, int VAR = 0>
static int launch_v3(const GemmArgs& a, hipStream_t st) {
  const int nwg = ((a.M + BM - 1) / BM) * (a.N / BN);
  hipLaunchKernelGGL((w4a16_gemm_v3<BM, BN, WMW, WNW, EPI, GR, VAR>), dim3(nwg), dim3(64 * WMW * WNW), 0, st,
                     a.A, a.lda, a.Wp, a.scales, a.qzeros, a.bias, a.C, a.ldc, a.M, a.N, a.K, a.groupsize);
  SAMQ_LAUNCH_CHECK("w4a16_gemm_v3 launch");
  return SAMQ_OK;
}

template <int BM, int BN, int WMW, int WNW, int EPI, bool GR>
static int launch_v4(const GemmArgs& a, hipStream_t st) {
  const int nwg = ((a.M + BM - 1) / BM) * (a.N / BN);
  hipLaunchKernelGGL((w4a16_gemm_v4<BM, BN, WMW, WNW, EPI, GR>), dim3(nwg), dim3(64 * WMW * WNW), 0, st,
                     a.A, a.lda, a.Wp, a.scales, a.qzeros, a.bias, a.C, a.ldc, a.M, a.N, a.K, a.groupsize);
  SAMQ_LAUNCH_CHECK("w4a16_gemm_v4 launch");
  return SAMQ_OK;
}

// CU count of the CURRENT device, cached per device id (a process may drive several GPUs)
static int cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  if (cached[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

template <int WMW, int TM, int TN, int NPH, int STAGES, int LA, int EPI, int VAR = 0>
static int launch_pp2(const GemmArgs& a, hipStream_t st) {
  constexpr int BM = WMW * TM * 32, BN = (8 / WMW) * TN * 32;
  if (EPI == SAMQ_EPI_BIAS_LNF || EPI == SAMQ_EPI_GELU_LNF) {
    // the consumer's row partials must fit the LDS the ring frees (a grouped cfg 57
    // ring leaves room for K <= 1728 only)
    constexpr int kmax = Pp2Lds<WMW, TM, TN, STAGES, EPI, VAR>::LNF_KMAX;
    if (a.K > kmax) return fail(SAMQ_ERR_UNSUPPORTED, "w4a16_gemm_lnf: consumer K exceeds this config's LDS row-partial budget");
  }
  int nwg = ((a.M + BM - 1) / BM) * (a.N / BN);
  if ((VAR & (1 << 20)) != 0 && nwg > cu_count()) {   // persistent: <= 1 workgroup per CU, whole XCD rounds
    const int cus = cu_count() & ~7;
    nwg = cus >= 8 ? cus : cu_count();
  }
  hipLaunchKernelGGL((w4a16_gemm_pp2<WMW, TM, TN, NPH, STAGES, LA, EPI, VAR>), dim3(nwg), dim3(512), 0, st,
                     a.A, a.lda, a.Wp, a.scales, a.qzeros, a.bias, a.C, a.ldc, a.M, a.N, a.K, a.groupsize / 64, a.lnf);
  SAMQ_LAUNCH_CHECK("w4a16_gemm_pp2 launch");
  return SAMQ_OK;
}

// LayerNorm-fold epilogues: the product ping-pong configs only
template <int EPI, bool GR>
static int launch_lnf(const GemmArgs& a, int cfg, hipStream_t st) {
  if (GR) {
    if (cfg == 57) return launch_pp2<2, 4, 2, 2, 3, 2, EPI, 512>(a, st);
    if (cfg == 64) return launch_pp2<2, 4, 2, 2, 3, 2, EPI, 512 | 16>(a, st);
  } else {
    if (cfg == 57) return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 4096>(a, st);
    if (cfg == 64) return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 16 | 4096>(a, st);
  }
  return fail(SAMQ_ERR_UNSUPPORTED, "w4a16_gemm_lnf: the LayerNorm fold needs ping-pong config 57 or 64");
}

// gated-MLP epilogue: the 32x32x16 ping-pong config (57) only
template <bool GR>
static int launch_silu(const GemmArgs& a, hipStream_t st) {
  if (GR) return launch_pp2<2, 4, 2, 2, 3, 2, SAMQ_EPI_SILU_MUL, 512>(a, st);
  return launch_pp2<2, 4, 2, 2, 4, 3, SAMQ_EPI_SILU_MUL, 4096>(a, st);
}

template <int EPI, bool GR>
static int launch_epi(const GemmArgs& a, int cfg, hipStream_t st) {
  if (cfg >= 50 && cfg < 200) {   // ping-pong kernels
    if (GR) {   // grouped weights: the per-group scale / zero row rides in the ring (VAR & 512)
      switch (cfg) {
        // the group's scale / zero words prefetched into VGPRs (VAR & (1 << 23)): 4 slots, lookahead 3.
        // Selectable, not the default: measured neutral (155.6 vs 155.3 img/s), and its inline-asm
        // loads leave the compiler free to move the not-yet-filled registers before their counted wait
        case 112: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 512 | 4096 | (1 << 23)>(a, st);
        // the group row in the ring (the grouped cfg 57): 3 slots, lookahead 2 (four 40 KiB stages
        // fill the 160 KiB LDS, the group row needs 640 B more)
        case 57: case 114: return launch_pp2<2, 4, 2, 2, 3, 2, EPI, 512>(a, st);
        case 64: return launch_pp2<2, 4, 2, 2, 3, 2, EPI, 512 | 16>(a, st);   // (slower than 57 on every shape)
        // register rows (VAR & (1 << 23)): no group row in the ring -> 4 slots / lookahead 3
        case 113: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 512 | 16 | 4096 | (1 << 23)>(a, st);
#ifdef SAMQ_TUNING
        case 116: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 512 | 4096 | (1 << 23) | 1024>(a, st);   // timing-only: no group scaling
#endif
        default: return fail(SAMQ_ERR_INVALID, "w4a16_gemm: grouped weights take ping-pong configs 57 / 64 only");
      }
    }
    switch (cfg) {
      case 55: return launch_pp2<2, 4, 2, 2, 3, 2, EPI>(a, st);   // v6 256x256, 2 k-phases, 3 slots
      case 56: return launch_pp2<2, 4, 2, 2, 4, 2, EPI>(a, st);   // 4 slots, lookahead 2 (DMA in both phases)
      // 4 slots, lookahead 3; the wave index in an SGPR (VAR & 4096: uniform piece addressing,
      // -3..-6 % isolated vs the VGPR form at M = 8192, profiles/r3_gemm_rfl.log)
      case 57: case 112: case 114: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 4096>(a, st);   // (112-114: grouped forms)
      case 58: return launch_pp2<2, 4, 2, 1, 4, 2, EPI>(a, st);   // 1 phase / K tile, 4 slots, lookahead 2
      case 62: return launch_pp2<4, 2, 4, 2, 4, 3, EPI>(a, st);   // 4x2 waves (64x128 each): A read 2x, B 4x
      case 64: case 113: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 16 | 4096>(a, st);  // cfg 57 on 16x16x32 MFMA
      case 65: return launch_pp2<2, 4, 2, 2, 4, 2, EPI, 16>(a, st);  // cfg 56 on 16x16x32 MFMA
      // cfg 57 / 64 with the LDS-DMA pieces spread through the MFMA burst (VAR & 16384)
      case 100: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 4096 | 16384>(a, st);
      // cfg 57 / 64 persistent (one workgroup per CU loops over the tiles: stores drain under the
      // next tile's prologue)
      case 107: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 4096 | (1 << 20)>(a, st);
      // cfg 57 / 64 with the epilogue's scale / bias loaded before the prologue (VAR & (1 << 21))
      case 109: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 4096 | (1 << 21)>(a, st);
      // cfg 57 with the transposed f16 staging epilogue for f16 outputs; f32 outputs (RESADD_F32 /
      // F32) have no f16 staging and run cfg 57 itself
      case 111:
        if constexpr (EPI == SAMQ_EPI_BIAS || EPI == SAMQ_EPI_BIAS_GELU) return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 4096 | (1 << 22)>(a, st);
        else return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 4096>(a, st);
      case 110: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 16 | 4096 | (1 << 21)>(a, st);
      case 108: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 16 | 4096 | (1 << 20)>(a, st);
      // cfg 57 with transposed accumulators and the f16-staged epilogue (f16 outputs only)
      case 104:
        if constexpr (EPI == SAMQ_EPI_BIAS || EPI == SAMQ_EPI_BIAS_GELU) return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 4096 | 65536>(a, st);
        else return fail(SAMQ_ERR_UNSUPPORTED, "w4a16_gemm: cfg 104 has f16 epilogues (BIAS / BIAS_GELU) only");
      case 101: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 16 | 4096 | 16384>(a, st);
#ifdef SAMQ_TUNING
      // tuning build only (make tuning): untested shapes and TIMING-ONLY variants that compute
      // wrong results on purpose -- never reachable through the product library
      case 60: return launch_pp2<1, 8, 1, 2, 4, 3, EPI>(a, st);   // 1x8 waves (256x32 each): B unpacked once
      case 61: return launch_pp2<1, 8, 1, 4, 4, 3, EPI>(a, st);   // 1x8 waves, 4 k-phases
      // all LDS-DMA pieces in the last phase's load half instead of behind the MFMA bursts
      // (measured: 57 -> 66 +1-3 %, 64 -> 67 within +-2 %, in-graph no change; DESIGN dead ends)
      case 66: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 32>(a, st);
      case 67: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 48>(a, st);
      // 2-D XCD tile blocks (xcd_tile): lin1 PMC fetch 105.7 -> 92.3 MB per M = 8192 launch,
      // time unchanged isolated (121.3 vs 122.0 us) and in the graph (23.98 / 23.94 vs 23.99 ms)
      case 68: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 64>(a, st);
      case 69: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 80>(a, st);
      // transposed accumulators (W^T . A^T) stored straight from registers (te_store4), no LDS
      // staging: bit-identical, but qkv 73.5 -> 113.1 us (52) / 72.7 -> 85.9 us (53) at M = 8192 --
      // the row-scattered 8-byte stores are issue-bound; only the fp32 residual on 16x16 ties
      case 52: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 128>(a, st);
      case 53: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 144>(a, st);
      // static priority (group 1 at prio 1 for the whole loop, no per-segment flips): isolated
      // within +-2 %, in the 2-lane graph 24.41 (all 59) vs 24.39 (all 64) vs 24.48 ms (pick)
      case 54: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 256>(a, st);
      case 59: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 272>(a, st);
      case 70: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 1>(a, st);   // timing-only: cfg 57 without restaging
      // grouped timing-only (per-channel weights, grouped code path): 74 / 75 = 57g without the
      // fp16 group scaling / without the group row; 76 / 77 the same on 64g
      case 74: return launch_pp2<2, 4, 2, 2, 3, 2, EPI, 512 | 1024>(a, st);
      case 75: return launch_pp2<2, 4, 2, 2, 3, 2, EPI, 512 | 2048>(a, st);
      case 76: return launch_pp2<2, 4, 2, 2, 3, 2, EPI, 512 | 16 | 1024>(a, st);
      case 77: return launch_pp2<2, 4, 2, 2, 3, 2, EPI, 512 | 16 | 2048>(a, st);
      case 78: return launch_pp2<2, 4, 2, 2, 3, 2, EPI, 512>(a, st);        // 57g on per-channel weights
      case 79: return launch_pp2<2, 4, 2, 2, 3, 2, EPI, 512 | 16>(a, st);   // 64g on per-channel weights
      // per-channel: wave index in an SGPR (90), interleaved piece deal (91), both (92 / 93 on 16x16)
      case 90: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 4096>(a, st);
      case 91: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 8192>(a, st);
      case 92: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 4096 | 8192>(a, st);
      case 93: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 16 | 4096 | 8192>(a, st);
      case 94: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 16 | 4096>(a, st);
      case 95: return launch_pp2<2, 4, 2, 2, 4, 3, EPI>(a, st);       // round-2 cfg 57 (VGPR wave index)
      case 96: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 16>(a, st);   // round-2 cfg 64
      // 1x8 waves of 128x64: 128x512 tiles, A staged once per 512 columns (32 instead of 40 LDS-DMA
      // pieces per 256x256-equivalent of work); N % 512 == 0 (lin1)
      case 97: return launch_pp2<1, 4, 2, 2, 4, 3, EPI, 4096>(a, st);
      case 98: return launch_pp2<1, 4, 2, 2, 5, 4, EPI, 4096>(a, st);
      // timing-only: cfg 57 / 64 without the epilogue (the per-tile epilogue cost)
      case 102: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 4096 | 32768>(a, st);
      // timing-only: cfg 57 whose f16 epilogue stages but does not store (105) / skips the math (106)
      case 105: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 4096 | (1 << 17)>(a, st);
      case 106: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 4096 | (2 << 17)>(a, st);
      case 103: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 16 | 4096 | 32768>(a, st);
      case 71: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 2>(a, st);   // timing-only: cfg 57 without MFMA
      case 72: return launch_pp2<2, 4, 2, 2, 4, 3, EPI, 3>(a, st);   // timing-only: neither
      case 73: {   // timing experiment: cfg 57 with per-segment s_memtime stamps (synchronous)
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0}, h[8];
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_pp_stamps), z, sizeof(z));
        const int r = launch_pp2<2, 4, 2, 2, 4, 3, EPI, 4>(a, st);
        (void)hipStreamSynchronize(st);
        (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_pp_stamps), sizeof(h));
        const double n = (double)h[4];
        fprintf(stderr, "pp2 stamps (cycles per wave-phase): load %.0f  barrier1 %.0f  mfma %.0f  barrier2 %.0f\n",
                h[0] / n, h[1] / n, h[2] / n, h[3] / n);
        return r;
      }
#endif
      default: break;
    }
  }
  switch (cfg) {
    case 21: return launch_v3<256, 256, 2, 4, EPI, GR>(a, st);
    case 22: return launch_v3<128, 256, 2, 4, EPI, GR>(a, st);
    case 23: return launch_v3<128, 128, 2, 2, EPI, GR>(a, st);
    case 24: return launch_v3<256, 128, 2, 2, EPI, GR>(a, st);
    case 25: return launch_v3<128, 256, 1, 4, EPI, GR>(a, st);
    case 26: return launch_v3<64, 64, 2, 2, EPI, GR>(a, st);
    // 320-column tiles: ViT-H N in {1280, 3840, 5120} and M = 128*B give whole waves of tiles
    case 29: return launch_v3<128, 320, 2, 5, EPI, GR>(a, st);
    case 30: return launch_v3<256, 320, 2, 5, EPI, GR>(a, st);
    case 31: return launch_v3<128, 320, 1, 5, EPI, GR>(a, st);
    case 1: return launch_cfg<256, 256, 2, 4, EPI, GR>(a, st);
    case 2: return launch_cfg<256, 128, 2, 2, EPI, GR>(a, st);
    case 3: return launch_cfg<128, 128, 2, 2, EPI, GR>(a, st);
    case 4: return launch_cfg<64, 64, 2, 2, EPI, GR>(a, st);
    case 5: return launch_cfg<64, 32, 2, 1, EPI, GR>(a, st);
    case 6: return launch_cfg<128, 256, 1, 4, EPI, GR>(a, st);
    case 7: return launch_cfg<256, 256, 1, 8, EPI, GR>(a, st);
    case 9: return launch_cfg<128, 256, 2, 4, EPI, GR>(a, st);
#ifdef SAMQ_TUNING
    case 8: return launch_cfg<256, 128, 1, 4, EPI, GR>(a, st);
    case 11: return launch_cfg<256, 256, 2, 4, EPI, GR, 0>(a, st);   // literal-constant unpack (A/B)
    case 27: return launch_v3<128, 256, 2, 4, EPI, GR, 1>(a, st);   // timing-only: no unpack
    case 28: return launch_v3<256, 256, 2, 4, EPI, GR, 1>(a, st);   // timing-only: no unpack
    // one wave per SIMD, 128x128 / 256x64 per wave (acc in the 512-register file): 10-20 %
    // slower than the ping-pong cfg 57 on every shape (DESIGN dead ends)
    case 32: return launch_v3<256, 256, 2, 2, EPI, GR>(a, st);
    case 33: return launch_v3<256, 256, 1, 4, EPI, GR>(a, st);
    // v4 (16x16x32): needs weights repacked in LAYOUT 2 -- the caller's responsibility here
    case 41: return launch_v4<128, 256, 2, 4, EPI, GR>(a, st);
    case 42: return launch_v4<256, 256, 2, 4, EPI, GR>(a, st);
    case 43: return launch_v4<128, 128, 2, 2, EPI, GR>(a, st);
    case 44: return launch_v4<64, 64, 2, 2, EPI, GR>(a, st);
    case 45: return launch_v4<128, 256, 4, 2, EPI, GR>(a, st);
#endif
    default: return fail(SAMQ_ERR_INVALID, "w4a16_gemm: unknown tile config");
  }
}

// Measured on MI355X (tools/bench_gemm.py, ViT-H shapes at M = 16384): the 3-stage LDS-DMA
// kernel with 128x256 tiles / 64x64 wave tiles (cfg 22, 2 workgroups per CU) is the fastest or
// within 2 % of it on every projection shape and beats dense fp16 hipBLASLt on 3 of 4.
// The ping-pong v6 (cfg 57: 256x256 tiles, 4-slot ring, lookahead 3) is 5-7 % faster on the wide
// projections (qkv N=3840, lin1 N=5120 at M=16384: 1090 / 970 TF/s vs 1016 / 925); with N=1280 its
// 320 tiles leave a 25 % second round on 256 CUs, where v3's 2-workgroup/CU 128x256 stays ahead.
// 128x320 tiles (cfg 29) make exactly one round on the chip for the N=1280 projections of one
// 2-image lane (M = 8192: isolated proj 38 vs 42 us, lin2 105 vs 124 us against cfg 22,
// profiles/r1_v12_gemm_scan_m8192.log) but are the slowest per CU in steady state; see pick_cfg.
static int pick_cfg(int M, int N, bool grouped) {
  // v6 from two images up: at M = 4096 (one image) lin1 runs 63.5 us on cfg 22 vs 77.9 on v6 and
  // qkv is a tie (profiles/r1_v20_gemm_scan_m4096.log).  The N = 1280 projections (proj, lin2)
  // take v6 on 16x16x32 MFMA (cfg 64): in steady state (M = 65536, no tile-round tail) lin2 runs
  // 1161 TF/s there vs 969 on the one-round 128x320 tiles (cfg 29) that win an isolated M = 8192
  // launch, and inside the 2-lane graph -- where the other lane fills any tail -- the step drops
  // 25.66 -> 24.35 ms with bit-identical output (profiles/r2_cfg_ab.log)
  // grouped weights: the 32x32x16 ping-pong with the group rows in the ring (VAR & 512) for every
  // N (its 16x16x32 twin is 6-13 % slower on all four shapes, profiles/r3_gemm_grouped.log)
  if (N % 256 == 0 && M >= 8192) return grouped || N >= 2048 ? 57 : 64;
  if (N % 256 == 0 && M >= 1024) return 22;
  if (N % 128 == 0 && M >= 512) return 23;
  if (N % 64 == 0) return 26;
  return 5;
}

static int cfg_bn(int cfg) {
  switch (cfg) { case 1: return 256; case 2: return 128; case 3: return 128; case 4: return 64;
                 case 5: return 32; case 6: return 256; case 7: return 256; case 8: return 128;
                 case 9: return 256; case 11: return 256; case 21: return 256; case 22: return 256;
                 case 23: return 128; case 24: return 128; case 25: return 256; case 26: return 64;
                 case 27: return 256; case 28: return 256; case 29: return 320; case 30: return 320;
                 case 31: return 320; case 32: return 256; case 33: return 256; case 41: return 256; case 42: return 256;
                 case 43: return 128; case 44: return 64; case 45: return 256;
                 case 52: return 256; case 53: return 256; case 54: return 256; case 59: return 256; case 55: return 256; case 56: return 256; case 57: return 256; case 58: return 256;
                 case 60: return 256; case 61: return 256; case 62: return 256; case 64: return 256; case 65: return 256; case 68: return 256; case 69: return 256; case 66: return 256; case 67: return 256;
                 case 70: return 256; case 71: return 256; case 72: return 256; case 73: return 256;
                 case 74: case 75: case 76: case 77: case 78: case 79: return 256;
                 case 90: case 91: case 92: case 93: case 94: case 95: case 96: return 256;
                 case 97: case 98: return 512;
                 case 100: case 101: case 102: case 103: case 104: case 105: case 106: case 107: case 108: case 109: case 110: case 111: case 112: case 113: case 114: case 115: case 116: return 256;
                 default: return 0; }
}

}  // namespace samq

using namespace samq;

extern "C" size_t samq_w4_packed_words(int K, int N) { return (size_t)K * (size_t)N / 8; }

extern "C" int samq_w4_repack_layout(const int32_t* qweight, int32_t* packed, int K, int N, int layout,
                                     hipStream_t stream) {
  SAMQ_REQUIRE(qweight && packed, SAMQ_ERR_INVALID, "w4_repack: null pointer");
  SAMQ_REQUIRE(K > 0 && N > 0 && K % 64 == 0, SAMQ_ERR_INVALID, "w4_repack: K must be a positive multiple of 64");
  SAMQ_REQUIRE(N % 32 == 0, SAMQ_ERR_INVALID, "w4_repack: N must be a multiple of 32");
#ifdef SAMQ_TUNING
  SAMQ_REQUIRE(layout >= 1 && layout <= 3, SAMQ_ERR_INVALID, "w4_repack: layout must be 1, 2 or 3");
#else
  // layout 2 feeds only the tuning-build v4 kernels; the product library never consumes it
  SAMQ_REQUIRE(layout == 1 || layout == 3, SAMQ_ERR_INVALID, "w4_repack: layout must be 1 or 3");
#endif
  SAMQ_REQUIRE(layout != 3 || K % 128 == 0, SAMQ_ERR_INVALID, "w4_repack: layout 3 needs K % 128 == 0");
  const int64_t total = (int64_t)K * N / 8;
  const int blocks = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
  if (layout == 3)
    hipLaunchKernelGGL(w4_repack_kernel<3>, dim3(blocks), dim3(256), 0, stream, (const uint32_t*)qweight,
                       (uint32_t*)packed, K, N);
  else if (layout == 2)
    hipLaunchKernelGGL(w4_repack_kernel<2>, dim3(blocks), dim3(256), 0, stream, (const uint32_t*)qweight,
                       (uint32_t*)packed, K, N);
  else
    hipLaunchKernelGGL(w4_repack_kernel<1>, dim3(blocks), dim3(256), 0, stream, (const uint32_t*)qweight,
                       (uint32_t*)packed, K, N);
  SAMQ_LAUNCH_CHECK("w4_repack launch");
  return SAMQ_OK;
}

extern "C" int samq_w4_repack(const int32_t* qweight, int32_t* packed, int K, int N, hipStream_t stream) {
  return samq_w4_repack_layout(qweight, packed, K, N, SAMQ_W4_LAYOUT, stream);
}

extern "C" int samq_w4a16_gemm_cfg(const void* A, int64_t lda, const int32_t* wpacked, const void* scales,
                                   const int32_t* qzeros, const void* bias, void* C, int64_t ldc, int M, int N,
                                   int K, int groupsize, int epilogue, int cfg, hipStream_t stream) {
  if (M == 0) return SAMQ_OK;   // empty batch: no work, data pointers may be null
  SAMQ_REQUIRE(A && wpacked && scales && qzeros && C, SAMQ_ERR_INVALID, "w4a16_gemm: null pointer");
  SAMQ_REQUIRE(M >= 0 && N > 0 && K > 0, SAMQ_ERR_INVALID, "w4a16_gemm: bad shape");
  SAMQ_REQUIRE(K % 64 == 0, SAMQ_ERR_INVALID, "w4a16_gemm: K must be a multiple of 64");
  SAMQ_REQUIRE(N % 32 == 0, SAMQ_ERR_INVALID, "w4a16_gemm: N must be a multiple of 32");
  SAMQ_REQUIRE(lda >= K && lda % 8 == 0 && ((uintptr_t)A & 15) == 0, SAMQ_ERR_INVALID,
               "w4a16_gemm: A must be 16-byte aligned with lda >= K, lda % 8 == 0");
  SAMQ_REQUIRE(ldc >= N, SAMQ_ERR_INVALID, "w4a16_gemm: ldc < N");
  if (groupsize == -1) groupsize = K;
  SAMQ_REQUIRE(groupsize > 0 && (groupsize == K || groupsize % 64 == 0), SAMQ_ERR_INVALID,
               "w4a16_gemm: groupsize must be -1, K, or a multiple of 64");
  if (M == 0) return SAMQ_OK;
  // the v3 kernels (cfg 21-28) store 16-byte row vectors: C 16-byte aligned, ldc % 8 == 0
  const bool vec_ok = ((uintptr_t)C & 15) == 0 && ldc % 8 == 0;
  if (cfg <= 0) {
    cfg = pick_cfg(M, N, groupsize != -1 && groupsize != K);
    if (!vec_ok && ((cfg >= 21 && cfg <= 33) || cfg >= 50)) cfg = N % 128 == 0 ? 3 : (N % 64 == 0 ? 4 : 5);
  }
  SAMQ_REQUIRE(cfg_bn(cfg) > 0 && N % cfg_bn(cfg) == 0, SAMQ_ERR_INVALID, "w4a16_gemm: N not divisible by tile");
  SAMQ_REQUIRE(vec_ok || ((cfg < 21 || cfg > 33) && cfg < 50), SAMQ_ERR_INVALID,
               "w4a16_gemm: this tile config needs a 16-byte aligned C with ldc % 8 == 0");
  GemmArgs a{(const _Float16*)A, lda, (const u32x4*)wpacked, (const _Float16*)scales, (const uint32_t*)qzeros,
             (const _Float16*)bias, C, ldc, M, N, K, groupsize};
  const bool gr = groupsize != K;
  switch (epilogue) {
    case SAMQ_EPI_BIAS: return gr ? launch_epi<SAMQ_EPI_BIAS, true>(a, cfg, stream) : launch_epi<SAMQ_EPI_BIAS, false>(a, cfg, stream);
    case SAMQ_EPI_BIAS_GELU: return gr ? launch_epi<SAMQ_EPI_BIAS_GELU, true>(a, cfg, stream) : launch_epi<SAMQ_EPI_BIAS_GELU, false>(a, cfg, stream);
    case SAMQ_EPI_RESADD_F32: return gr ? launch_epi<SAMQ_EPI_RESADD_F32, true>(a, cfg, stream) : launch_epi<SAMQ_EPI_RESADD_F32, false>(a, cfg, stream);
    case SAMQ_EPI_F32: return gr ? launch_epi<SAMQ_EPI_F32, true>(a, cfg, stream) : launch_epi<SAMQ_EPI_F32, false>(a, cfg, stream);
    default: return fail(SAMQ_ERR_INVALID, "w4a16_gemm: unknown epilogue");
  }
}

extern "C" int samq_w4a16_gated_mlp(const void* A, int64_t lda, const int32_t* wpacked, const void* scales,
                                    const int32_t* qzeros, void* C, int64_t ldc, int M, int N2, int K, int groupsize,
                                    hipStream_t stream) {
  if (M == 0) return SAMQ_OK;   // empty batch: no work, data pointers may be null
  SAMQ_REQUIRE(A && wpacked && scales && qzeros && C, SAMQ_ERR_INVALID, "w4a16_gated_mlp: null pointer");
  SAMQ_REQUIRE(M >= 0 && N2 > 0 && K > 0 && K % 64 == 0, SAMQ_ERR_INVALID,
               "w4a16_gated_mlp: K must be a positive multiple of 64");
  SAMQ_REQUIRE(N2 % 256 == 0, SAMQ_ERR_INVALID, "w4a16_gated_mlp: 2N must be a multiple of 256");
  SAMQ_REQUIRE(lda >= K && lda % 8 == 0 && ((uintptr_t)A & 15) == 0 && ldc >= N2 / 2 && ldc % 8 == 0 &&
               ((uintptr_t)C & 15) == 0, SAMQ_ERR_INVALID, "w4a16_gated_mlp: 16-byte aligned A / C rows required");
  if (groupsize == -1) groupsize = K;
  SAMQ_REQUIRE(groupsize > 0 && (groupsize == K || groupsize % 64 == 0), SAMQ_ERR_INVALID,
               "w4a16_gated_mlp: groupsize must be -1, K, or a multiple of 64");
  if (M == 0) return SAMQ_OK;
  GemmArgs a{(const _Float16*)A, lda, (const u32x4*)wpacked, (const _Float16*)scales, (const uint32_t*)qzeros,
             nullptr, C, ldc, M, N2, K, groupsize};
  return groupsize != K ? launch_silu<true>(a, stream) : launch_silu<false>(a, stream);
}

extern "C" int samq_w4a16_gemm_lnf(const void* A, int64_t lda, const int32_t* wpacked, const void* scales,
                                   const int32_t* qzeros, const void* bias, void* C, int64_t ldc, int M, int N,
                                   int K, int groupsize, int epilogue, int cfg, const float* gamma, const float* gw,
                                   const float* bw, float* stats, float* mu, void* aout, float eps,
                                   hipStream_t stream) {
  if (M == 0) return SAMQ_OK;   // empty batch: no work, data pointers may be null
  SAMQ_REQUIRE(A && wpacked && scales && qzeros && C && stats && mu, SAMQ_ERR_INVALID, "w4a16_gemm_lnf: null pointer");
  SAMQ_REQUIRE(M >= 0 && N > 0 && K > 0 && K % 64 == 0 && N % 256 == 0, SAMQ_ERR_INVALID,
               "w4a16_gemm_lnf: K % 64 == 0 and N % 256 == 0 required");
  SAMQ_REQUIRE(lda >= K && lda % 8 == 0 && ((uintptr_t)A & 15) == 0 && ldc >= N && ldc % 8 == 0 &&
               ((uintptr_t)C & 15) == 0, SAMQ_ERR_INVALID, "w4a16_gemm_lnf: 16-byte aligned A / C rows required");
  if (groupsize == -1) groupsize = K;
  SAMQ_REQUIRE(groupsize > 0 && (groupsize == K || groupsize % 64 == 0), SAMQ_ERR_INVALID,
               "w4a16_gemm_lnf: groupsize must be -1, K, or a multiple of 64");
  const bool gr = groupsize != K;
  if (cfg <= 0) cfg = pick_cfg(M, N, gr);
  LnfArgs L{gamma, gw, bw, stats, mu, (_Float16*)aout, eps, K / 64, nullptr};
  if (epilogue == SAMQ_EPI_RESADD_LNF) {
    SAMQ_REQUIRE(gamma && aout, SAMQ_ERR_INVALID, "w4a16_gemm_lnf: the producer needs gamma and aout");
  } else if (epilogue == SAMQ_EPI_BIAS_LNF || epilogue == SAMQ_EPI_GELU_LNF) {
    SAMQ_REQUIRE(gw && bw, SAMQ_ERR_INVALID, "w4a16_gemm_lnf: the consumer needs gw and bw");
    // the workgroup's row partial sums (256 rows x K/64 pairs) are staged in the LDS the ring
    // leaves free in the epilogue: Pp2Lds::LNF_KMAX per config (launch_pp2 checks it -- K <= 3008
    // for cfg 57, 3968 for cfg 64 per-channel; 1728 / 2688 for grouped weights' 3-slot rings)
  } else {
    return fail(SAMQ_ERR_INVALID, "w4a16_gemm_lnf: epilogue must be RESADD_LNF, BIAS_LNF or GELU_LNF");
  }
  if (M == 0) return SAMQ_OK;
  GemmArgs a{(const _Float16*)A, lda, (const u32x4*)wpacked, (const _Float16*)scales, (const uint32_t*)qzeros,
             (const _Float16*)bias, C, ldc, M, N, K, groupsize, L};
  switch (epilogue) {
    case SAMQ_EPI_RESADD_LNF: return gr ? launch_lnf<SAMQ_EPI_RESADD_LNF, true>(a, cfg, stream)
                                        : launch_lnf<SAMQ_EPI_RESADD_LNF, false>(a, cfg, stream);
    case SAMQ_EPI_BIAS_LNF: return gr ? launch_lnf<SAMQ_EPI_BIAS_LNF, true>(a, cfg, stream)
                                      : launch_lnf<SAMQ_EPI_BIAS_LNF, false>(a, cfg, stream);
    default: return gr ? launch_lnf<SAMQ_EPI_GELU_LNF, true>(a, cfg, stream)
                       : launch_lnf<SAMQ_EPI_GELU_LNF, false>(a, cfg, stream);
  }
}

extern "C" int samq_w4a16_gemm(const void* A, int64_t lda, const int32_t* wpacked, const void* scales,
                               const int32_t* qzeros, const void* bias, void* C, int64_t ldc, int M, int N, int K,
                               int groupsize, int epilogue, hipStream_t stream) {
  return samq_w4a16_gemm_cfg(A, lda, wpacked, scales, qzeros, bias, C, ldc, M, N, K, groupsize, epilogue, 0, stream);
}

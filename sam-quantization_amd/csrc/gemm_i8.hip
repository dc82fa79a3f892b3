// Int8-activation GEMMs on gfx950 int8 MFMA (v_mfma_i32_32x32x32_i8):
//   W8A8: int8 per-output-channel symmetric weights x int8 per-tensor activations -- the fq_vit
//         QLinear / QConv2d compute (fq_vit/models/ptq/layers.py:160-200, 11-74) whose inputs are
//         the int8 codes of the preceding QAct (layers.py:203-242, quantizer/uniform.py:23-45);
//   W4A8: GPTQ int4 weights (gptq_triton/quant_linear.py:66-116 buffers) x int8 activations --
//         the composition "QuantLinear + fq_vit QAct on its input" (SURVEY.md §8c Oracle W4A8).
//
// C[m,n] = epilogue( float(sum_k a[m,k] * w[k,n]) * (a_scale * w_scale[n]) + bias[n] ), with the
// integer sum EXACT in int32 (the reference sums the dequantised fp32 products; both agree up to
// fp32 rounding of the final value).  W4: w = q - zp, converted to int8 in registers:
//   bytes(q) | 0x80 minus zp per byte never borrows (q in [0,15], zp in [1,16]), ^0x80 -> int8.
//
// Same machinery as the W4A16 v3 kernel (gemm_w4a16.hip): 3-slot LDS ring fed by
// global_load_lds (A rows XOR-swizzled through the source address, B pre-packed in fragment
// order), counted vmcnt waits + one s_barrier per K tile, XCD-aware tile remap, LDS-staged
// 16-byte vector epilogue.  K tile = 128 int8 = the same 128-byte A rows as the fp16 kernel.
//
// Quantising epilogues (int8 output codes, fq_vit fake quant with a TRUE division and
// round-half-to-even, clamp [-128, 127]):
//   Q8      out = q(y, out_scale)                                  (Linear -> QAct)
//   Q8_GELU out = q(GELU(y), out_scale)                            (lin1 -> GELU -> mlp.qact1)
//   Q8_RES  out = q(R * res_scale + fq(y, mid_scale), out_scale)   (proj -> qact3 -> +x -> qact2)
//           (mid_scale <= 0: no intermediate quantiser); R int8 codes, may alias C.
#include "common.h"

namespace samq {

enum { BF_W8 = 0, BF_W4 = 1 };

struct I8Epi {
  float a_scale, mid_scale, res_scale, out_scale;
  const int8_t* R;
  int64_t ldr;
  int rmod;               // > 0: residual row = output row % rmod (pos_embed codes shared by images)
  int kpg;                // grouped W4 (GRP kernels): K tiles (128) per weight group
  // W4A8 row sums (round 6): rs_in = S[m] = sum_k A[m, k] of the int8 input rows, emitted by the
  // producer of A (LN-q, the lin1 epilogue) so the zero-point ping-pong (cfg 86 / 93) does not
  // recompute it per column tile; rs_out (int8-code epilogues): S of the OUTPUT rows accumulated
  // with one int32 atomic per row and 16 x (WN / 16) codes -- the caller zeroes it first
  const int* rs_in;
  int* rs_out;
  // Q8 epilogue (round 6, the W8A8 qkv GEMM): the codes of columns >= v16_col0 (the V third) are
  // also stored as fp16 values (exact small integers) into v16 [rows, ldv] at column c - v16_col0,
  // so the attention stages V without an int8 -> fp16 conversion per key row
  _Float16* v16;
  int v16_col0;
  int64_t ldv;
};

// Implicit-GEMM A operand (AG != 0): the int8 codes are gathered from an image / feature map
// instead of an [M, K] matrix, 16 contiguous bytes per LDS-DMA lane:
//   AG_PATCH  x int8 [B, Cin, S, S] (NCHW), P = 16: A[t, (c, kh, kw)] = x[b, c, gy*16+kh, gx*16+kw]
//             (fq_vit PatchEmbed QConv2d on the image codes, fq_vit image_encoder.py PatchEmbed)
//   AG_3X3    x int8 [B, G, G, Cin] (NHWC), pad 1: A[t, (ky, kx, c)] = x[b, gy+ky-1, gx+kx-1, c], 0 outside
//             (neck QConv2d 3x3, image_encoder.py:88-104; weight codes permuted to (n, ky, kx, c))
enum { AG_ROWS = 0, AG_PATCH = 1, AG_3X3 = 2 };
struct I8Gather { int S, G, Cin; };
__device__ __attribute__((aligned(16))) int8_t g_zero_i8[16];


template <int N>
__device__ __forceinline__ void vm_wait_i8() {
  static_assert(N >= 0 && N <= 15, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ int w4_to_i8(uint32_t nib, uint32_t zpx) {
  return (int)(((nib | 0x80808080u) - zpx) ^ 0x80808080u);
}

// ------------------------------------------------------------------ W8 repack
// packed byte (((nt * (K/128) + kb) * 4 + s) * 64 + lane) * 16 + j  =  W[n][k] with
// n = nt*32 + (lane&31), k = kb*128 + 32*s + 16*(lane>>5) + j   (W row-major [N][K], i.e. the
// nn.Linear / flattened Conv2d weight layout).
__global__ void w8_repack_kernel(const int8_t* __restrict__ w, int8_t* __restrict__ out, int K, int N) {
  const int64_t units = (int64_t)K * N / 16;
  for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < units; u += (int64_t)gridDim.x * blockDim.x) {
    const int lane = u & 63;
    const int s = (u >> 6) & 3;
    const int64_t blk = u >> 8;
    const int kbs = K / 128;
    const int kb = (int)(blk % kbs), nt = (int)(blk / kbs);
    const int n = nt * 32 + (lane & 31);
    const int k = kb * 128 + 32 * s + 16 * (lane >> 5);
    *(u32x4*)(out + u * 16) = *(const u32x4*)(w + (int64_t)n * K + k);
  }
}

// y = float(acc) * (a_scale * wscale[n]) + bias[n] (-> GELU / residual / int8 quantiser), staged
// through LDS in 32-row slices per wave (ep = this wave's 32 x WN f32 slice) so the global traffic
// is row-contiguous 16-byte vectors.  Shared by the v3-style and the ping-pong int8 kernels.
// ZPS: the sums exclude the zero point (acc = sum a * q) and the epilogue subtracts zp[n] * S[m]
// (zpv = MINUS this lane's zp per column block, ssum = S of the wave's WM rows; int32-exact, on
// the full-rate 24-bit multiply: |zp| <= 16, |S| <= 128 K < 2^23)
// Grouped W4 (float accumulators, the group scales already applied): wscale == nullptr, the
// factor is a_scale alone.
// One 32-row slice i of the wave's accumulator tile (i8_epilogue runs all TM of them; the
// tile ping-pong kernel spreads them over the other group's main loop).
template <int TM, int TN, int WN, int EPI, bool ZPS = false, typename AccV = int16_t_v>
__device__ __forceinline__ void i8_epilogue_slice(int i, const AccV (&acc)[TM][TN], const int (&col)[TN],
                                                  const float* __restrict__ wscale, const float* __restrict__ bias,
                                                  const I8Epi& ep_args, float* ep, void* __restrict__ Cout,
                                                  int64_t ldc, int M, int row_base, int col_base, int lane,
                                                  const int* ssum = nullptr, const int* zpv = nullptr) {
  const int hsel = lane >> 5;
  float csc[TN], cb[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    csc[t] = wscale ? ep_args.a_scale * wscale[col[t]] : ep_args.a_scale;
    cb[t] = bias ? bias[col[t]] : 0.0f;
  }
  constexpr bool GELU = EPI == SAMQ_EPI_BIAS_GELU || EPI == SAMQ_EPI_Q8_GELU;
  const float inv_out = ep_args.out_scale > 0.f ? 1.0f / ep_args.out_scale : 0.f;   // q8_exact (common.h)
  const float inv_mid = ep_args.mid_scale > 0.f ? 1.0f / ep_args.mid_scale : 0.f;
  const float lim_out = 130.0f * ep_args.out_scale, lim_mid = 130.0f * ep_args.mid_scale;   // q8_exact2 clamps
  // staging swizzle (round 4): the readers below take 64 B (int8 path: 16 columns, 4 ds_read_b128)
  // or 32 B (f16 path: 8 columns, 2 reads) of one row per lane, and a ds_read_b128 lane group
  // spans 4 rows whose k-th 16-byte chunks sat on the same banks (PMC: 3.9 M conflict cycles per
  // W4A8 lin1 launch at M = 16384, profiles/r4_pmc_i8_pp2_m16384.txt).  Column c of slice row r is
  // stored at c ^ swz(r), swz = 4 * key: the 4-column chunk within each 16 (int8) / 8 (f16)
  // columns XOR key = (r >> 1) & 3 / & 1, so read k of the group's rows lands on distinct banks;
  // rows r, r + 1 (r even) share the key, so a lane's accumulator pair still stores with one
  // ds_write2
  constexpr bool Q8OUT = EPI == SAMQ_EPI_Q8 || EPI == SAMQ_EPI_Q8_GELU || EPI == SAMQ_EPI_Q8_RES;
  constexpr bool F16OUT = EPI == SAMQ_EPI_BIAS || EPI == SAMQ_EPI_BIAS_GELU;
  constexpr int SWZ = (Q8OUT && WN % 16 == 0) ? 1 : (F16OUT && WN % 8 == 0) ? 2 : 0;
  auto swz = [](int row) { return SWZ == 1 ? 4 * ((row >> 1) & 3) : SWZ == 2 ? 4 * ((row >> 1) & 1) : 0; };
  {
    // accumulator pairs (r, r + 1) = slice rows (rl, rl + 1): packed fp32; four rows x TN columns
    // at a time are dequantised and their GELU chains run in lockstep (gelu_r16_n: 2 TN pairs)
#pragma unroll
    for (int r0 = 0; r0 < 16; r0 += 4) {
      float2_t y[2 * TN];
#pragma unroll
      for (int r = r0; r < r0 + 4; r += 2) {
        const int rl = (r & 3) + 8 * (r >> 2) + 4 * hsel;
#pragma unroll
        for (int t = 0; t < TN; ++t) {
          auto a0 = acc[i][t][r], a1 = acc[i][t][r + 1];
          if constexpr (ZPS) {   // v_mad_i32_i24 (zpv = -zp; |S| <= 128 K < 2^23: K < 65536 checked at launch)
            a0 += __mul24(zpv[t], ssum[i * 32 + rl]);
            a1 += __mul24(zpv[t], ssum[i * 32 + rl + 1]);
          }
          y[((r - r0) / 2) * TN + t] = __builtin_elementwise_fma((float2_t){(float)a0, (float)a1}, (float2_t)(csc[t]),
                                                                 (float2_t)(cb[t]));
        }
      }
      if constexpr (GELU) gelu_r16_n<2 * TN>(y);
#pragma unroll
      for (int r = r0; r < r0 + 4; r += 2) {
        const int rl = (r & 3) + 8 * (r >> 2) + 4 * hsel;
#pragma unroll
        for (int t = 0; t < TN; ++t) {
          const float2_t v = y[((r - r0) / 2) * TN + t];
          const int cs = (t * 32 + (lane & 31)) ^ swz(rl);   // rl even: swz(rl + 1) == swz(rl)
          ep[rl * WN + cs] = v.x;
          ep[(rl + 1) * WN + cs] = v.y;
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if (EPI == SAMQ_EPI_RESADD_F32 || EPI == SAMQ_EPI_F32) {
      constexpr int C4 = WN / 4;
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
    } else if (EPI == SAMQ_EPI_BIAS || EPI == SAMQ_EPI_BIAS_GELU) {
      constexpr int C8 = WN / 8;
#pragma unroll
      for (int j = 0; j < (32 * C8 + 63) / 64; ++j) {
        const int idx = j * 64 + lane;
        if (idx < 32 * C8) {
          const int rl = idx / C8, c8 = idx % C8;
          const int row = row_base + i * 32 + rl;
          const int f4 = rl * (WN / 4) + 2 * c8, sk = swz(rl) / 4;   // float4s of the 8 columns
          const float4_t v0 = ((const float4_t*)ep)[f4 + sk];
          const float4_t v1 = ((const float4_t*)ep)[f4 + (1 ^ sk)];
          if (row < M) {
            const half8_t h = {(_Float16)v0[0], (_Float16)v0[1], (_Float16)v0[2], (_Float16)v0[3],
                               (_Float16)v1[0], (_Float16)v1[1], (_Float16)v1[2], (_Float16)v1[3]};
            *(half8_t*)((_Float16*)Cout + (int64_t)row * ldc + col_base + 8 * c8) = h;
          }
        }
      }
    } else {   // int8 codes, 16 columns per lane-store
      constexpr int C16 = WN / 16;
      static_assert(C16 >= 1 && 64 % C16 == 0, "int8 store: a row's lanes are C16 consecutive lanes");
#pragma unroll
      for (int j = 0; j < (32 * C16 + 63) / 64; ++j) {
        const int idx = j * 64 + lane;
        int rsum = 0;   // this lane's 16 codes summed (rs_out)
        if (idx < 32 * C16) {
          const int rl = idx / C16, c16 = idx % C16;
          const int row = row_base + i * 32 + rl;
          if (row < M) {
            float v[16];
            const int f4 = rl * (WN / 4) + 4 * c16, sk = swz(rl) / 4;   // float4s of the 16 columns
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float4_t f = ((const float4_t*)ep)[f4 + (e ^ sk)];
              v[4 * e] = f[0]; v[4 * e + 1] = f[1]; v[4 * e + 2] = f[2]; v[4 * e + 3] = f[3];
            }
            u32x4 res;
            if (EPI == SAMQ_EPI_Q8_RES)
              res = *(const u32x4*)(ep_args.R + (int64_t)(ep_args.rmod > 0 ? row % ep_args.rmod : row) * ep_args.ldr +
                                    col_base + 16 * c16);
            u32x4 o;
            float vq[EPI == SAMQ_EPI_Q8 ? 16 : 1];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
              float cq[4];
#pragma unroll
              for (int b = 0; b < 4; b += 2) {
                float2_t x = {v[4 * w + b], v[4 * w + b + 1]};
                if (EPI == SAMQ_EPI_Q8_RES) {
                  if (ep_args.mid_scale > 0.f) x = q8_exact2(x, ep_args.mid_scale, inv_mid, lim_mid) * ep_args.mid_scale;
                  const float2_t rv = float2_t{(float)(int8_t)((res[w] >> (8 * b)) & 0xFFu),
                                               (float)(int8_t)((res[w] >> (8 * b + 8)) & 0xFFu)} * ep_args.res_scale;
                  x = rv + x;
                }
                const float2_t q = EPI == SAMQ_EPI_Q8_GELU ? q8_recip2(x, inv_out)
                                                           : q8_exact2(x, ep_args.out_scale, inv_out, lim_out);
                cq[b] = q.x;
                cq[b + 1] = q.y;
                if constexpr (EPI == SAMQ_EPI_Q8) {
                  vq[4 * w + b] = q.x;
                  vq[4 * w + b + 1] = q.y;
                }
              }
              o[w] = q8_pack4(cq[0], cq[1], cq[2], cq[3]);
            }
            *(u32x4*)((int8_t*)Cout + (int64_t)row * ldc + col_base + 16 * c16) = o;
            if constexpr (EPI == SAMQ_EPI_Q8) {
              if (ep_args.v16 && col_base >= ep_args.v16_col0) {   // (uniform: a wave's columns are in one third)
                half8_t h0, h1;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                  h0[e] = (_Float16)vq[e];
                  h1[e] = (_Float16)vq[8 + e];
                }
                _Float16* vp = ep_args.v16 + (int64_t)row * ep_args.ldv + (col_base - ep_args.v16_col0) + 16 * c16;
                *(half8_t*)vp = h0;
                *(half8_t*)(vp + 8) = h1;
              }
            }
            if (ep_args.rs_out) {
#pragma unroll
              for (int w = 0; w < 4; ++w) rsum = __builtin_amdgcn_sdot4((int)o[w], 0x01010101, rsum, false);
            }
          }
        }
        if (ep_args.rs_out) {   // the row's C16 lanes reduce, one int32 atomic per row of the slice
#pragma unroll
          for (int off = 1; off < C16; off <<= 1) rsum += __shfl_xor(rsum, off, 64);
          const int rl = idx / C16, row = row_base + i * 32 + rl;
          if (idx < 32 * C16 && idx % C16 == 0 && row < M) atomicAdd(ep_args.rs_out + row, rsum);
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
  }
}

template <int TM, int TN, int WN, int EPI, bool ZPS = false, typename AccV = int16_t_v>
__device__ __forceinline__ void i8_epilogue(const AccV (&acc)[TM][TN], const int (&col)[TN],
                                            const float* __restrict__ wscale, const float* __restrict__ bias,
                                            const I8Epi& ep_args, float* ep, void* __restrict__ Cout, int64_t ldc,
                                            int M, int row_base, int col_base, int lane,
                                            const int* ssum = nullptr, const int* zpv = nullptr) {
#pragma unroll
  for (int i = 0; i < TM; ++i)
    i8_epilogue_slice<TM, TN, WN, EPI, ZPS, AccV>(i, acc, col, wscale, bias, ep_args, ep, Cout, ldc, M, row_base,
                                                  col_base, lane, ssum, zpv);
}

// ------------------------------------------------------------------ GEMM
// GRP (W4 only): grouped GPTQ weights, w = s[g, n] (q - zp[g, n]) with g = k / groupsize and the
// groupsize a multiple of the 128-deep K tile (ep_args.kpg tiles per group).  The int32 MFMA sums of
// one group are exact (|sum| <= 128 * 127 * 16 per tile); at each group end they are scaled by the
// group's f32 scale into f32 accumulators (one fma per element) and restarted; the zero point of
// the group is applied per byte in the unpack as for per-channel weights.  wscale is the f32
// [G, N] scale table; the next group's zero / scale words are loaded one K tile ahead, before the
// tile's LDS-DMA pieces (so the ring's counted vmcnt covers them).
template <int BM, int BN, int WAVES_M, int WAVES_N, int EPI, int BFMT, int STAGES, int AG = AG_ROWS, bool GRP = false>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N)
void i8_gemm_kernel(const int8_t* __restrict__ A, int64_t lda, const char* __restrict__ Wp,
                    const float* __restrict__ wscale, const uint32_t* __restrict__ qzeros,
                    const float* __restrict__ bias, void* __restrict__ Cout, int64_t ldc,
                    int M, int N, int K, I8Epi ep_args, I8Gather ga) {
  constexpr int NW = WAVES_M * WAVES_N;
  constexpr int WM = BM / WAVES_M;
  constexpr int WN = BN / WAVES_N;
  constexpr int TM = WM / 32;
  constexpr int TN = WN / 32;
  constexpr int BK = 128;                     // int8 k per tile = 128-byte A rows
  constexpr int ROWB = BK;
  constexpr int A_BYTES = BM * ROWB;
  constexpr int PPB = BFMT == BF_W8 ? 4 : 2;  // 1-KiB pieces per (32-column, 128-k) block
  constexpr int NA = BM / 8;
  constexpr int NB = (BN / 32) * PPB;
  constexpr int NT = NA + NB;
  constexpr int NPW = (NT + NW - 1) / NW;
  constexpr int STAGE = A_BYTES + NB * 1024;
  static_assert(TM >= 1 && TN >= 1 && NPW <= 15, "bad tile");
  static_assert(!GRP || (BFMT == BF_W4 && AG == AG_ROWS), "grouped: W4 weights, row-major A");

  __shared__ __attribute__((aligned(16))) char smem[STAGES * STAGE];

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

  const char* src[NPW];
  int dst[NPW];
  int64_t step[NPW];
  int gtok[NPW], gck[NPW];   // AG: token (b, gy, gx) and in-tile byte offset of each A piece's lane
#pragma unroll
  for (int i = 0; i < NPW; ++i) {
    int j = wave * NPW + i;
    j = j < NT ? j : NT - 1;
    if (j < NA) {
      const int row = j * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      int gr = m0 + row;
      gr = gr < M ? gr : M - 1;
      src[i] = (const char*)(A + (int64_t)gr * lda + c * 16);
      gtok[i] = gr;
      gck[i] = c * 16;
      dst[i] = j * 1024;
      step[i] = BK;
    } else {
      const int jb = j - NA;
      const int nt = n0 / 32 + jb / PPB;
      src[i] = Wp + (((int64_t)nt * kt_count) * PPB + (jb % PPB)) * 1024 + lane * 16;
      dst[i] = A_BYTES + jb * 1024;
      step[i] = PPB * 1024;
    }
  }
  auto a_gather = [&](int i, int kt) -> const char* {
    const int t = gtok[i], k = kt * BK + gck[i];
    const int gg = ga.G * ga.G;
    const int b = t / gg, rem = t - b * gg, gy = rem / ga.G, gx = rem - gy * ga.G;
    if (AG == AG_PATCH) {   // k = (c * 16 + kh) * 16 + kw, kw = 0..15 contiguous
      const int ckh = k >> 4;
      const int c = ckh >> 4, kh = ckh & 15;
      return (const char*)(A + (((int64_t)b * ga.Cin + c) * ga.S + gy * 16 + kh) * ga.S + gx * 16);
    }
    const int tap = k / ga.Cin, c0 = k - tap * ga.Cin;   // AG_3X3: k = (ky * 3 + kx) * Cin + c
    const int sy = gy + tap / 3 - 1, sx = gx + tap % 3 - 1;
    if (sy < 0 || sy >= ga.G || sx < 0 || sx >= ga.G) return (const char*)g_zero_i8;
    return (const char*)(A + (((int64_t)b * ga.G + sy) * ga.G + sx) * ga.Cin + c0);
  };
  auto issue = [&](int kt, int slot) {
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
      const char* p = src[i] + kt * step[i];
      if (AG != AG_ROWS && wave * NPW + i < NA) p = a_gather(i, kt);
      __builtin_amdgcn_global_load_lds((const SAMQ_GLOBAL void*)p, (SAMQ_LDS void*)(smem + slot * STAGE + dst[i]), 16,
                                       0, 0);
    }
  };

  int col[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) col[t] = n0 + wn * WN + t * 32 + (lane & 31);
  uint32_t zpx[TN];
  if (BFMT == BF_W4) {
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const uint32_t zw = qzeros[col[t] >> 3];
      zpx[t] = (((zw >> (4 * (col[t] & 7))) & 0xFu) + 1u) * 0x01010101u;
    }
  }

  int16_t_v acc[TM][TN];
  float16_t facc[GRP ? TM : 1][GRP ? TN : 1];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        acc[i][j][r] = 0;
        if constexpr (GRP) facc[i][j][r] = 0.f;
      }
  const int kpg = GRP ? ep_args.kpg : 1;
  float gsc[TN], nsc[TN];   // GRP: the current / next group's scales of this lane's columns
  uint32_t nzp[TN];
  if constexpr (GRP) {
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      gsc[t] = wscale[col[t]];
      nsc[t] = gsc[t];
      nzp[t] = zpx[t];
    }
  }

  int a_off[TM], a_swz[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int rr = wm * WM + i * 32 + (lane & 31);
    a_off[i] = rr * ROWB;
    a_swz[i] = (rr >> 1) & 7;
  }
  const int hsel = lane >> 5;
  uint32_t kLo = 0x0F0F0F0Fu;
  asm volatile("" : "+v"(kLo));

  issue(0, 0);
  if (STAGES > 2 && kt_count > 1) issue(1, 1);
  int slot = 0;
  for (int kt = 0; kt < kt_count; ++kt) {
    if (STAGES > 2) {
      if (kt + 1 < kt_count) vm_wait_i8<NPW>(); else vm_wait_i8<0>();
      __builtin_amdgcn_s_barrier();
      if (GRP && kt + 1 < kt_count && (kt + 1) % kpg == 0) {   // next group's zero / scale words
        const int g = (kt + 1) / kpg;
#pragma unroll
        for (int t = 0; t < TN; ++t) {
          const uint32_t zw = qzeros[(int64_t)g * (N / 8) + (col[t] >> 3)];
          nzp[t] = (((zw >> (4 * (col[t] & 7))) & 0xFu) + 1u) * 0x01010101u;
          nsc[t] = wscale[(int64_t)g * N + col[t]];
        }
      }
      if (kt + 2 < kt_count) {
        int s2 = slot + 2;
        s2 = s2 >= STAGES ? s2 - STAGES : s2;
        issue(kt + 2, s2);
      }
    } else {
      vm_wait_i8<0>();
      __builtin_amdgcn_s_barrier();            // tile kt landed; everyone is done with tile kt-1
      if (GRP && kt + 1 < kt_count && (kt + 1) % kpg == 0) {
        const int g = (kt + 1) / kpg;
#pragma unroll
        for (int t = 0; t < TN; ++t) {
          const uint32_t zw = qzeros[(int64_t)g * (N / 8) + (col[t] >> 3)];
          nzp[t] = (((zw >> (4 * (col[t] & 7))) & 0xFu) + 1u) * 0x01010101u;
          nsc[t] = wscale[(int64_t)g * N + col[t]];
        }
      }
      if (kt + 1 < kt_count) issue(kt + 1, slot ^ 1);
    }
    const char* abase = smem + slot * STAGE;
    const char* bbase = abase + A_BYTES + (wn * TN) * PPB * 1024 + lane * 16;
    u32x4 bw[TN][2];
    if (BFMT == BF_W4) {
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        bw[t][0] = *(const u32x4*)(bbase + (t * PPB + 0) * 1024);
        bw[t][1] = *(const u32x4*)(bbase + (t * PPB + 1) * 1024);
      }
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      int4_t af[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *(const int4_t*)(abase + a_off[i] + (((2 * s + hsel) ^ a_swz[i]) << 4));
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        int4_t bf;
        if (BFMT == BF_W8) {
          bf = *(const int4_t*)(bbase + (t * PPB + s) * 1024);
        } else {
          const uint32_t w0 = bw[t][s >> 1][2 * (s & 1)];
          const uint32_t w1 = bw[t][s >> 1][2 * (s & 1) + 1];
          bf[0] = w4_to_i8(w0 & kLo, zpx[t]);
          bf[1] = w4_to_i8((w0 >> 4) & kLo, zpx[t]);
          bf[2] = w4_to_i8(w1 & kLo, zpx[t]);
          bf[3] = w4_to_i8((w1 >> 4) & kLo, zpx[t]);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[i][t] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[i], bf, acc[i][t], 0, 0, 0);
      }
    }
    if (GRP && ((kt + 1) % kpg == 0 || kt + 1 == kt_count)) {   // group end: scale the exact sums in
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int t = 0; t < TN; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            facc[i][t][r] = __builtin_fmaf((float)acc[i][t][r], gsc[t], facc[i][t][r]);
            acc[i][t][r] = 0;
          }
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        zpx[t] = nzp[t];
        gsc[t] = nsc[t];
      }
    }
    if (STAGES > 2) slot = slot + 1 == STAGES ? 0 : slot + 1;
    else slot ^= 1;
  }

  // ---- epilogue (LDS-staged per 32-row slice; see gemm_w4a16.hip v3)
  static_assert(NW * 32 * WN * 4 <= STAGES * STAGE, "epilogue staging does not fit the LDS ring");
  __syncthreads();
  if constexpr (GRP)
    i8_epilogue<TM, TN, WN, EPI, false, float16_t>(facc, col, nullptr, bias, ep_args, (float*)(smem + wave * 32 * WN * 4),
                                                   Cout, ldc, M, m0 + wm * WM, n0 + wn * WN, lane);
  else
    i8_epilogue<TM, TN, WN, EPI>(acc, col, wscale, bias, ep_args, (float*)(smem + wave * 32 * WN * 4), Cout, ldc, M,
                                 m0 + wm * WM, n0 + wn * WN, lane);
}

// ------------------------------------------------------------------ W4A8 ping-pong GEMM
// The W4A16 v6 ping-pong structure (gemm_w4a16.hip w4a16_gemm_pp2) on the int8 MFMA: 256x256
// tiles, 8 waves (2 x 4, 128x64 each) in two groups one s_barrier apart, so the two waves of a SIMD
// alternate -- one issues its MFMA burst (s_setprio 1) while the other reads its A fragments and
// its B piece from LDS and unpacks int4 -> int8; the LDS-DMA pieces of K tile kt+LA are issued
// behind the MFMA bursts of tile kt.  K tile = 128 int8 (128-byte A rows, one 2-KiB layout-3 block
// per 32 columns); phase p of a K tile = k32 steps 2p, 2p+1 = B piece p, so each phase reads its own
// A fragments and unpacks its own piece.  WAR / RAW: as w4a16_gemm_pp2 (the slot restaged during
// tile kt held tile kt+LA-STAGES <= kt-1, whose last reads were consumed before the barrier that
// opens the MFMA half of tile kt's phase 0 for either group; the retire wait for tile kt+1 sits in
// the load half of the last phase, before the barrier after which the first group reads it).
__host__ __device__ constexpr int i8_pre(int p, int npw, int nph) {   // pieces issued before phase p
  return (npw * p) / nph;
}
template <int N>
__device__ __forceinline__ void i8_vm_wait_le(int n) {   // s_waitcnt vmcnt(n) for a uniform n <= N
  if constexpr (N > 0) {
    if (n >= N) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); return; }
    i8_vm_wait_le<N - 1>(n);
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// VAR & 8 (product, cfg 86): zero point by row sums -- the MFMA multiplies the raw nibbles q (an
// AND per 4 weights instead of OR / SUB / XOR on top) and the epilogue subtracts zp[n] * S[m] with
// S[m] = sum_k a[m, k] accumulated from the staged A tile by v_dot4 against ones (wave wn sums the
// 32 rows of its M block wn, 8 dot4 + 2 LDS reads per phase; the 4 waves of an M half share the
// sums through LDS at the end).  Integer-exact: identical outputs.
// VAR & 16: the phase's LDS-DMA pieces spread through the MFMA burst (one after every 16 / np
// MFMAs) instead of issued after it, where they queue in the TA behind the other MFMA-half waves'
// pieces while the MFMA pipe drains and the partner group waits at the barrier.
// VAR (tuning build only, timing experiments that compute wrong results): 1 no zero-point
// subtraction in the unpack, 2 no MFMA, 4 no restaging
template <int EPI, int STAGES, int LA, int VAR = 0>
__global__ __launch_bounds__(512, 1)
void i8_gemm_pp2(const int8_t* __restrict__ A, int64_t lda, const char* __restrict__ Wp,
                 const float* __restrict__ wscale, const uint32_t* __restrict__ qzeros,
                 const float* __restrict__ bias, void* __restrict__ Cout, int64_t ldc, int M, int N, int K,
                 I8Epi ep_args) {
  constexpr int NW = 8, WAVES_N = 4, TM = 4, TN = 2;
  constexpr int WM = TM * 32, WN = TN * 32;
  constexpr int BM = 2 * WM, BN = WAVES_N * WN;
  constexpr int BK = 128, ROWB = BK;
  constexpr int A_BYTES = BM * ROWB;
  constexpr int PPB = 2;                       // W4 layout 3: two 1-KiB pieces per (32 columns, 128 k)
  constexpr int NA = BM / 8, NB = (BN / 32) * PPB, NT = NA + NB;
  constexpr int NPW = (NT + NW - 1) / NW;
  constexpr int STAGE = A_BYTES + NB * 1024;
  constexpr int NPH = 2;
  constexpr int PRE_LAST = i8_pre(NPH - 1, NPW, NPH);
  constexpr int EP_BYTES = 32 * WN * 4;
  constexpr int SMEM = STAGES * STAGE > NW * EP_BYTES ? STAGES * STAGE : NW * EP_BYTES;
  static_assert(LA >= 2 && LA < STAGES, "ring");
  static_assert((LA - 2) * NPW + PRE_LAST <= 63 && (LA - 1) * NPW <= 63, "vmcnt");
  static_assert(SMEM <= 160 * 1024 && NW * EP_BYTES + BM * 4 <= SMEM, "LDS");

  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WAVES_N;
  const int wn = wave % WAVES_N;
  const int grp = wave >> 2;
  const int tiles_n = N / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (bid / tiles_n) * BM;
  const int n0 = (bid % tiles_n) * BN;
  const int kt_count = K / BK;

  const char* src[NPW];
  int dst[NPW];
  int step[NPW];
#pragma unroll
  for (int i = 0; i < NPW; ++i) {
    int j = wave * NPW + i;
    j = j < NT ? j : NT - 1;
    if (j < NA) {
      const int row = j * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      int gr = m0 + row;
      gr = gr < M ? gr : M - 1;
      src[i] = (const char*)(A + (int64_t)gr * lda + c * 16);
      dst[i] = j * 1024;
      step[i] = BK;
    } else {
      const int jb = j - NA;
      const int nt = n0 / 32 + jb / PPB;
      src[i] = Wp + (((int64_t)nt * kt_count) * PPB + (jb % PPB)) * 1024 + lane * 16;
      dst[i] = A_BYTES + jb * 1024;
      step[i] = PPB * 1024;
    }
  }
  auto issue = [&](int kt, int slot, int i0, int i1) {
#pragma unroll
    for (int i = 0; i < NPW; ++i)
      if (i >= i0 && i < i1)
        __builtin_amdgcn_global_load_lds((const SAMQ_GLOBAL void*)(src[i] + (int64_t)kt * step[i]),
                                         (SAMQ_LDS void*)(smem + slot * STAGE + dst[i]), 16, 0, 0);
  };

  int col[TN];
  uint32_t zpx[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    col[t] = n0 + wn * WN + t * 32 + (lane & 31);
    const uint32_t zw = qzeros[col[t] >> 3];
    zpx[t] = (((zw >> (4 * (col[t] & 7))) & 0xFu) + 1u) * 0x01010101u;
  }
  int16_t_v acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0;
  const int hsel = lane >> 5;
  int a_off[TM], a_swz[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int rr = wm * WM + i * 32 + (lane & 31);
    a_off[i] = rr * ROWB;
    a_swz[i] = (rr >> 1) & 7;
  }
  uint32_t kLo = 0x0F0F0F0Fu;
  asm volatile("" : "+v"(kLo));
  constexpr bool ZPS = (VAR & 8) != 0;
  // VAR & 64 (with ZPS): the row sums come from the producer of A (ep_args.rs_in), loaded once here
  // -- older than every LDS-DMA piece, so the ring's counted waits retire it on the way -- instead
  // of 8 v_dot4 + 2 LDS reads per wave and phase
  constexpr bool RSIN = ZPS && (VAR & 64) != 0;
  static_assert(!ZPS || TM == WAVES_N, "row sums: wave wn sums M block wn");
  const int rs_row = wm * WM + wn * 32 + (lane & 31);
  const int rs_off = rs_row * ROWB, rs_swz = (rs_row >> 1) & 7;
  int rsum = 0;
  if constexpr (RSIN) {
    const int r = m0 + rs_row;
    rsum = ep_args.rs_in[r < M ? r : M - 1];
  }

  // ---- prologue: K tiles 0 .. LA-1 in flight, tile 0 retired + visible; group 1 lags a barrier
  const int pro = kt_count < LA ? kt_count : LA;
#pragma unroll
  for (int j = 0; j < LA; ++j)
    if (j < pro) issue(j, j, 0, NPW);
  i8_vm_wait_le<(LA - 1) * NPW>((pro - 1) * NPW);
  __builtin_amdgcn_s_barrier();
  if (grp) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  int slot = 0;
  constexpr bool SPREAD = (VAR & 16) != 0;
  for (int kt = 0; kt < kt_count; ++kt) {
    const char* st = smem + slot * STAGE;
    const int ahead = kt + LA;
    const bool pf = ahead < kt_count && !(VAR & 4);
    const int sa = slot + LA >= STAGES ? slot + LA - STAGES : slot + LA;   // (kt + LA) % STAGES
    static_for<NPH>([&](auto pc_) {
      constexpr int p = decltype(pc_)::value;
      // ---------------- load half
      if (p == NPH - 1 && kt + 1 < kt_count) {
        // K tile kt+1 retired: newer = whole tiles kt+2 .. kt+LA-1 + this tile's pieces so far
        // (steady state: a compile-time count instead of the runtime SALU decision tree)
        if (pf && kt + LA < kt_count) {
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"((LA - 2) * NPW + PRE_LAST) : "memory");
        } else {
          int newer = pf ? PRE_LAST : 0;
#pragma unroll
          for (int j = 2; j < LA; ++j) newer += kt + j < kt_count ? NPW : 0;
          i8_vm_wait_le<(LA - 2) * NPW + PRE_LAST>(newer);
        }
      }
      u32x4 bw[TN];
#pragma unroll
      for (int t = 0; t < TN; ++t) bw[t] = *(const u32x4*)(st + A_BYTES + ((wn * TN + t) * PPB + p) * 1024 + lane * 16);
      int4_t af[TM][2];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          af[i][s] = *(const int4_t*)(st + a_off[i] + (((2 * (2 * p + s) + hsel) ^ a_swz[i]) << 4));
      if constexpr (ZPS && !RSIN) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int4_t x = *(const int4_t*)(st + rs_off + (((2 * (2 * p + s) + hsel) ^ rs_swz) << 4));
#pragma unroll
          for (int e = 0; e < 4; ++e) rsum = __builtin_amdgcn_sdot4(x[e], 0x01010101, rsum, false);
        }
      }
      int4_t bf[TN][2];
#pragma unroll
      for (int t = 0; t < TN; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const uint32_t w0 = bw[t][2 * s], w1 = bw[t][2 * s + 1];
          if ((VAR & 1) || ZPS) {
            bf[t][s] = int4_t{(int)(w0 & kLo), (int)((w0 >> 4) & kLo), (int)(w1 & kLo), (int)((w1 >> 4) & kLo)};
            continue;
          }
          bf[t][s][0] = w4_to_i8(w0 & kLo, zpx[t]);
          bf[t][s][1] = w4_to_i8((w0 >> 4) & kLo, zpx[t]);
          bf[t][s][2] = w4_to_i8(w1 & kLo, zpx[t]);
          bf[t][s][3] = w4_to_i8((w1 >> 4) & kLo, zpx[t]);
        }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // ---------------- MFMA half
      __builtin_amdgcn_s_setprio(1);
      if constexpr (SPREAD) {
        static_assert(!(VAR & 2), "spread: product MFMA halves only");
        constexpr int P0 = i8_pre(p, NPW, NPH), NP = i8_pre(p + 1, NPW, NPH) - P0, NMF = 2 * TM * TN;
        static_for<NMF>([&](auto qc) {
          constexpr int q = decltype(qc)::value;
          constexpr int s = q / (TM * TN), i = (q / TN) % TM, t = q % TN;
          acc[i][t] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[i][s], bf[t][s], acc[i][t], 0, 0, 0);
          static_for<NPW>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            if constexpr (k < NP && q + 1 == ((2 * k + 1) * NMF) / (2 * NP)) {
              __builtin_amdgcn_sched_barrier(0);
              if (pf) issue(ahead, sa, P0 + k, P0 + k + 1);
              __builtin_amdgcn_sched_barrier(0);
            }
          });
        });
      } else {
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int t = 0; t < TN; ++t) {
              if (VAR & 2) acc[i][t][0] += af[i][s][0] ^ bf[t][s][1];
              else acc[i][t] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[i][s], bf[t][s], acc[i][t], 0, 0, 0);
            }
        if (pf) issue(ahead, sa, i8_pre(p, NPW, NPH), i8_pre(p + 1, NPW, NPH));
      }
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    });
    slot = slot == STAGES - 1 ? 0 : slot + 1;
  }
  if (!grp) __builtin_amdgcn_s_barrier();   // balance group 1's extra barrier

  if constexpr ((VAR & 32) != 0) {   // timing-only (tuning build): no epilogue, sums kept alive
    int z = rsum;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int t = 0; t < TN; ++t) z += acc[i][t][0] + acc[i][t][15];
    if (z == 123456789) ((int*)Cout)[tid] = z;
    return;
  }
  __syncthreads();
  if constexpr (ZPS) {
    int* s_lds = (int*)(smem + NW * EP_BYTES);
    if constexpr (!RSIN) rsum += __shfl_xor(rsum, 32, 64);   // the two k halves of the row
    if (lane < 32) s_lds[rs_row] = rsum;
    __syncthreads();
    int zpv[TN];
#pragma unroll
    for (int t = 0; t < TN; ++t) zpv[t] = -(int)(zpx[t] & 0xFFu);
    i8_epilogue<TM, TN, WN, EPI, true>(acc, col, wscale, bias, ep_args, (float*)(smem + wave * EP_BYTES), Cout,
                                       ldc, M, m0 + wm * WM, n0 + wn * WN, lane, s_lds + wm * WM, zpv);
    return;
  }
  i8_epilogue<TM, TN, WN, EPI>(acc, col, wscale, bias, ep_args, (float*)(smem + wave * EP_BYTES), Cout, ldc, M,
                               m0 + wm * WM, n0 + wn * WN, lane);
}

// ------------------------------------------------------------------ W4A8 tile ping-pong GEMM (round 5)
// TUNING BUILD ONLY (cfg 99): bit-identical to cfg 86 on every epilogue (tests/test_w8a8.py with the
// tuning library), but 1.67x slower at M = 16384 (781 vs 467 us per ViT-H block,
// profiles/r5_i8_decomposition.log): one MFMA wave per SIMD that also reads its own fragments and
// issues ten LDS-DMA pieces per K step runs that step at ~20 % of the MFMA rate, and the epilogue it
// hides is smaller than what it loses.  Kept as the measured form of the verdict's option (b).
#ifdef SAMQ_TUNING
// The epilogue of one tile under the main loop of the next.  i8_gemm_pp2 alternates its two wave
// groups PHASE by phase inside one 256x256 tile, so both groups reach the epilogue together and
// the MFMA pipes idle through it (a third of the W4A8 GEMM time, profiles/r5_i8_decomposition.log:
// epilogues 158 of 472 us per ViT-H block at M = 16384).  Here the groups alternate TILE by tile:
// a workgroup owns P consecutive 256x128 tiles; group (j & 1) runs the main loop of its tile j (4
// waves, one per SIMD, 128x64 each) while the other group -- its SIMD partners -- (a) runs the
// epilogue of ITS tile j - 1 in four 32-row slices spread over tile j's K steps and (b) sums the
// int8 rows of tile j's staged A (the zero point through row sums, as cfg 86: acc = sum a * q,
// epilogue subtracts zp[n] * S[m]; integer-exact, bit-identical to cfg 86) -- so the MFMA issue of
// one wave and the VALU / store work of the other share each SIMD.  One K-step stream over the P
// tiles feeds a 3-slot LDS-DMA ring (40 KiB stages: 32 KiB A + 8 KiB layout-3 B), lookahead 2,
// issued by the main-loop group (ten 1-KiB pieces per wave per step, spread through its MFMAs);
// one barrier per K step.  vmcnt: a wave that issued pieces in the previous step and no stores
// since waits vmcnt(10) (the newest step's pieces may stay in flight), otherwise vmcnt(0).
template <int EPI>
__global__ __launch_bounds__(512, 1)
void i8_gemm_tpp(const int8_t* __restrict__ A, int64_t lda, const char* __restrict__ Wp,
                 const float* __restrict__ wscale, const uint32_t* __restrict__ qzeros,
                 const float* __restrict__ bias, void* __restrict__ Cout, int64_t ldc, int M, int N, int K,
                 I8Epi ep_args, int P) {
  constexpr int TM = 4, TN = 2, WM = 128, WN = 64, BM = 256, BN = 128, BK = 128, ROWB = BK;
  constexpr int A_BYTES = BM * ROWB, NA = BM / 8, NB = (BN / 32) * 2, NT = NA + NB, NPW = NT / 4;
  constexpr int STAGE = A_BYTES + NB * 1024, STAGES = 3, LA = 2;
  constexpr int EP_BYTES = 32 * WN * 4;
  constexpr int EP_OFF = STAGES * STAGE, RS_OFF = EP_OFF + 4 * EP_BYTES;
  constexpr int SMEM = RS_OFF + 2 * BM * 4;
  static_assert(NT % 4 == 0 && SMEM <= 160 * 1024, "tile ping-pong layout");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  int* rsl = (int*)(smem + RS_OFF);   // [2][BM] row sums of the tiles, by tile parity

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, gw = wave & 3, wm = gw >> 1, wn = gw & 1;
  const int hsel = lane >> 5;
  const int tiles_n = N / BN, tiles_m = (M + BM - 1) / BM, tiles = tiles_m * tiles_n;
  const int nwg = (tiles + P - 1) / P;
  const int t0 = xcd_remap(blockIdx.x, nwg) * P;
  const int nt = tiles - t0 < P ? tiles - t0 : P;   // tiles of this workgroup (>= 1)
  const int KT = K / BK, S = nt * KT;
  auto tile_mn = [&](int j, int& m0, int& n0) {
    const int u = t0 + j;
    m0 = (u / tiles_n) * BM;
    n0 = (u % tiles_n) * BN;
  };
  // DMA pieces of stream step q (ML group waves only): this wave's NPW 32-bit source offsets
  // (A rows or packed B blocks, both < 2^31 bytes: checked at launch) computed once per step,
  // then issued a few at a time between the MFMAs
  auto piece_offsets = [&](int q, uint32_t (&off)[NPW]) {
    const int j = q / KT, kt = q - j * KT;
    int m0, n0;
    tile_mn(j, m0, n0);
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
      const int pc = gw * NPW + i;   // uniform: A pieces for gw < 3, B for gw == 3 (NA = 32 = 3 * 10 + 2)
      if (pc < NA) {
        const int row = pc * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((row >> 1) & 7);
        int gr = m0 + row;
        gr = gr < M ? gr : M - 1;
        off[i] = (uint32_t)((int64_t)gr * lda + kt * BK + c * 16);
      } else {
        const int jb = pc - NA, nb = n0 / 32 + jb / 2;
        off[i] = (uint32_t)((((int64_t)nb * KT + kt) * 2 + (jb & 1)) * 1024 + lane * 16);
      }
    }
  };
  auto issue = [&](int q, const uint32_t (&off)[NPW], int i0, int i1) {
    char* sl = smem + (q % STAGES) * STAGE;
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
      if (i < i0 || i >= i1) continue;
      const int pc = gw * NPW + i;
      const char* src = pc < NA ? (const char*)A + off[i] : Wp + off[i];
      const int dst = pc < NA ? pc * 1024 : A_BYTES + (pc - NA) * 1024;
      __builtin_amdgcn_global_load_lds((const SAMQ_GLOBAL void*)src, (SAMQ_LDS void*)(sl + dst), 16, 0, 0);
    }
  };

  int16_t_v acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int t = 0; t < TN; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][t][r] = 0;
  int a_off[TM], a_swz[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int rr = wm * WM + i * 32 + (lane & 31);
    a_off[i] = rr * ROWB;
    a_swz[i] = (rr >> 1) & 7;
  }
  uint32_t kLo = 0x0F0F0F0Fu;
  asm volatile("" : "+v"(kLo));
  const int rs_row = gw * 64 + lane;                 // EPI role: the row of the ML tile this lane sums
  int rsum = 0;

  // prologue: group 0 runs tile 0's main loop; it stages steps 0 .. LA - 1
  if (grp == 0) {
    uint32_t off[NPW];
    piece_offsets(0, off);
    issue(0, off, 0, NPW);
    if (S > 1) {
      piece_offsets(1, off);
      issue(1, off, 0, NPW);
    }
  }
  int issued_prev = grp == 0 ? (S > 1 ? NPW : 0) : 0;   // pieces this wave issued in the previous step
  bool stores = false;                                  // global stores since this wave's last vmcnt(0)
  int epi_j = -1;                                       // the tile whose epilogue this wave owes

  for (int q = 0; q < S; ++q) {
    const int j = q / KT, kt = q - j * KT;
    const bool ml = (j & 1) == grp;
    // ---- step q's pieces landed (this wave's), then every wave's
    if (issued_prev > 0 && !stores) {
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NPW) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      stores = false;
    }
    __builtin_amdgcn_s_barrier();   // step q staged; the last step's row sums / LDS reads done
    const char* st = smem + (q % STAGES) * STAGE;
    if (ml) {
      // ---------------- main loop step: 4 k32 steps x 8 MFMAs, the next-next step's pieces spread
      if (kt == 0) {   // a new tile: the accumulators start from zero (their last epilogue slice is done)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int t = 0; t < TN; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][t][r] = 0;
      }
      const bool pf = q + LA < S;
      uint32_t poff[NPW];
      if (pf) piece_offsets(q + LA, poff);
      u32x4 bw[TN][2];
#pragma unroll
      for (int t = 0; t < TN; ++t)
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) bw[t][pp] = *(const u32x4*)(st + A_BYTES + ((wn * TN + t) * 2 + pp) * 1024 + lane * 16);
      static_for<4>([&](auto sc_) {
        constexpr int sk = decltype(sc_)::value;
        int4_t af[TM];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = *(const int4_t*)(st + a_off[i] + (((2 * sk + hsel) ^ a_swz[i]) << 4));
        int4_t bf[TN];
#pragma unroll
        for (int t = 0; t < TN; ++t) {
          const uint32_t w0 = bw[t][sk >> 1][2 * (sk & 1)], w1 = bw[t][sk >> 1][2 * (sk & 1) + 1];
          bf[t] = int4_t{(int)(w0 & kLo), (int)((w0 >> 4) & kLo), (int)(w1 & kLo), (int)((w1 >> 4) & kLo)};
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int t = 0; t < TN; ++t) {
            acc[i][t] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[i], bf[t], acc[i][t], 0, 0, 0);
          }
        // pieces of step q + LA: 2-3 behind each k32 step's MFMAs
        constexpr int I0 = (sk * NPW) / 4, I1 = ((sk + 1) * NPW) / 4;
        __builtin_amdgcn_sched_barrier(0);
        if (pf) issue(q + LA, poff, I0, I1);
        __builtin_amdgcn_sched_barrier(0);
      });
      issued_prev = pf ? NPW : 0;
      if (kt == KT - 1) epi_j = j;   // this tile's epilogue runs under the next tile's main loop
    } else {
      issued_prev = 0;
      // ---------------- row sums of the ML tile's staged A (rows 64 gw .. +63, one per lane)
      {
        const char* rp = st + rs_row * ROWB;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const int4_t x = *(const int4_t*)(rp + (((c + (rs_row >> 1)) & 7) << 4));
#pragma unroll
          for (int e = 0; e < 4; ++e) rsum = __builtin_amdgcn_sdot4(x[e], 0x01010101, rsum, false);
        }
        if (kt == KT - 1) {
          rsl[(j & 1) * BM + rs_row] = rsum;
          rsum = 0;
        }
      }
      // ---------------- epilogue slices of this wave's previous tile (needs its row sums: written
      // at that tile's last step by the other group, visible after this step's barrier)
      int sl = -1;   // the slice of the owed epilogue due at this step (slices at K steps i KT / 4)
#pragma unroll
      for (int ii = 0; ii < TM; ++ii)
        if (kt == (ii * KT) / TM) sl = ii;
      if (epi_j >= 0 && sl >= 0) {
        int m0, n0;
        tile_mn(epi_j, m0, n0);
        int col[TN], zpv[TN];
#pragma unroll
        for (int t = 0; t < TN; ++t) {
          col[t] = n0 + wn * WN + t * 32 + (lane & 31);
          const uint32_t zw = qzeros[col[t] >> 3];
          zpv[t] = -(int)(((zw >> (4 * (col[t] & 7))) & 0xFu) + 1u);
        }
        // the due slice by a uniform switch: constant register indices, the accumulators only read
        float* epw = (float*)(smem + EP_OFF + gw * EP_BYTES);
        const int* rsp = rsl + (epi_j & 1) * BM + wm * WM;
        switch (sl) {
          case 0: i8_epilogue_slice<TM, TN, WN, EPI, true>(0, acc, col, wscale, bias, ep_args, epw, Cout, ldc, M,
                                                           m0 + wm * WM, n0 + wn * WN, lane, rsp, zpv); break;
          case 1: i8_epilogue_slice<TM, TN, WN, EPI, true>(1, acc, col, wscale, bias, ep_args, epw, Cout, ldc, M,
                                                           m0 + wm * WM, n0 + wn * WN, lane, rsp, zpv); break;
          case 2: i8_epilogue_slice<TM, TN, WN, EPI, true>(2, acc, col, wscale, bias, ep_args, epw, Cout, ldc, M,
                                                           m0 + wm * WM, n0 + wn * WN, lane, rsp, zpv); break;
          default: i8_epilogue_slice<TM, TN, WN, EPI, true>(3, acc, col, wscale, bias, ep_args, epw, Cout, ldc, M,
                                                            m0 + wm * WM, n0 + wn * WN, lane, rsp, zpv); break;
        }
        stores = true;
        if (sl == TM - 1) epi_j = -1;   // done; the accumulators restart at the next main-loop tile
      }
    }
  }
  // ---- tail: the last tile's epilogue (its group ran its main loop last; the row sums were written
  // at the last step by the other group)
  __syncthreads();
  if (epi_j >= 0) {
    int m0, n0;
    tile_mn(epi_j, m0, n0);
    int col[TN], zpv[TN];
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      col[t] = n0 + wn * WN + t * 32 + (lane & 31);
      const uint32_t zw = qzeros[col[t] >> 3];
      zpv[t] = -(int)(((zw >> (4 * (col[t] & 7))) & 0xFu) + 1u);
    }
    i8_epilogue<TM, TN, WN, EPI, true>(acc, col, wscale, bias, ep_args, (float*)(smem + EP_OFF + gw * EP_BYTES), Cout,
                                       ldc, M, m0 + wm * WM, n0 + wn * WN, lane, rsl + (epi_j & 1) * BM + wm * WM, zpv);
  }
}
#endif  // SAMQ_TUNING

struct I8Args {
  const int8_t* A; int64_t lda; const char* Wp; const float* wscale; const uint32_t* qzeros;
  const float* bias; void* C; int64_t ldc; int M, N, K; I8Epi ep; I8Gather ga;
};

template <int BM, int BN, int WMW, int WNW, int EPI, int BF, int ST, int AG = AG_ROWS, bool GRP = false>
static int launch_i8(const I8Args& a, hipStream_t st) {
  const int nwg = ((a.M + BM - 1) / BM) * (a.N / BN);
  hipLaunchKernelGGL((i8_gemm_kernel<BM, BN, WMW, WNW, EPI, BF, ST, AG, GRP>), dim3(nwg), dim3(64 * WMW * WNW), 0, st,
                     a.A, a.lda, a.Wp, a.wscale, a.qzeros, a.bias, a.C, a.ldc, a.M, a.N, a.K, a.ep, a.ga);
  SAMQ_LAUNCH_CHECK("i8_gemm launch");
  return SAMQ_OK;
}

#ifdef SAMQ_TUNING
template <int EPI>
static int launch_i8_tpp(const I8Args& a, hipStream_t st) {
  SAMQ_REQUIRE(a.K < 65536 && a.K / 128 >= 4, SAMQ_ERR_UNSUPPORTED,
               "w4a8_gemm: the tile ping-pong needs 512 <= K < 65536 (four epilogue slices per tile's K steps)");
  SAMQ_REQUIRE((int64_t)a.M * a.lda < (int64_t)1 << 31 && (int64_t)a.K * a.N / 2 < (int64_t)1 << 31, SAMQ_ERR_UNSUPPORTED,
               "w4a8_gemm: the tile ping-pong addresses A and the weights with 31-bit offsets");
  const int tiles = ((a.M + 255) / 256) * (a.N / 128);
  const int P = tiles >= 4 * 256 ? 4 : 2;   // tiles per workgroup (even: both groups run main loops)
  const int nwg = (tiles + P - 1) / P;
  hipLaunchKernelGGL((i8_gemm_tpp<EPI>), dim3(nwg), dim3(512), 0, st, a.A, a.lda, a.Wp, a.wscale, a.qzeros, a.bias,
                     a.C, a.ldc, a.M, a.N, a.K, a.ep, P);
  SAMQ_LAUNCH_CHECK("i8_gemm_tpp launch");
  return SAMQ_OK;
}
#endif

template <int EPI, int STAGES, int LA, int VAR = 0>
static int launch_i8_pp2(const I8Args& a, hipStream_t st) {
  if constexpr ((VAR & 8) != 0)   // row sums on the 24-bit multiply (i8_epilogue ZPS)
    SAMQ_REQUIRE(a.K < 65536, SAMQ_ERR_UNSUPPORTED, "w4a8_gemm: the row-sum zero-point path needs K < 65536");
  const int nwg = ((a.M + 255) / 256) * (a.N / 256);
  hipLaunchKernelGGL((i8_gemm_pp2<EPI, STAGES, LA, VAR>), dim3(nwg), dim3(512), 0, st, a.A, a.lda, a.Wp, a.wscale,
                     a.qzeros, a.bias, a.C, a.ldc, a.M, a.N, a.K, a.ep);
  SAMQ_LAUNCH_CHECK("i8_gemm_pp2 launch");
  return SAMQ_OK;
}

// tile configs: 81 256x256 (W4: 3 stages; W8: 2), 82 128x256, 83 128x128, 84 64x64, 87 128x64,
// 88 64x128, 89 64x64 on 2 stages;
// 85 the W4 ping-pong kernel (256x256, 3-slot ring, lookahead 2)
template <int EPI, int BF>
static int launch_i8_cfg(const I8Args& a, int cfg, hipStream_t st) {
  switch (cfg) {
    case 85:
      if constexpr (BF == BF_W4) return launch_i8_pp2<EPI, 3, 2>(a, st);
      else return fail(SAMQ_ERR_INVALID, "i8_gemm: cfg 85 is the W4 ping-pong kernel");
    case 86:
      if constexpr (BF == BF_W4)
        return a.ep.rs_in ? launch_i8_pp2<EPI, 3, 2, 8 | 64>(a, st) : launch_i8_pp2<EPI, 3, 2, 8>(a, st);
      else return fail(SAMQ_ERR_INVALID, "i8_gemm: cfg 86 is the W4 ping-pong kernel");
    case 93:   // cfg 86 with the LDS-DMA pieces spread through the MFMA bursts
      if constexpr (BF == BF_W4)
        return a.ep.rs_in ? launch_i8_pp2<EPI, 3, 2, 8 | 16 | 64>(a, st) : launch_i8_pp2<EPI, 3, 2, 8 | 16>(a, st);
      else return fail(SAMQ_ERR_INVALID, "i8_gemm: cfg 93 is the W4 ping-pong kernel");
#ifdef SAMQ_TUNING
    case 99:   // tile ping-pong: one group's epilogue under the other group's main loop (correct, slower)
      if constexpr (BF == BF_W4) return launch_i8_tpp<EPI>(a, st);
      else return fail(SAMQ_ERR_INVALID, "i8_gemm: cfg 99 is a W4 kernel");
    case 94:   // timing-only: cfg 86 without its epilogue
      if constexpr (BF == BF_W4) return launch_i8_pp2<EPI, 3, 2, 8 | 32>(a, st);
      return fail(SAMQ_ERR_INVALID, "i8_gemm: W4 only");
    case 95: case 96: case 97:   // timing-only (wrong results): no zero point / no MFMA / no restaging
      if constexpr (BF == BF_W4) {
        if (cfg == 95) return launch_i8_pp2<EPI, 3, 2, 1>(a, st);
        if (cfg == 96) return launch_i8_pp2<EPI, 3, 2, 2>(a, st);
        return launch_i8_pp2<EPI, 3, 2, 4>(a, st);
      }
      return fail(SAMQ_ERR_INVALID, "i8_gemm: W4 only");
#endif
    case 81:
      if constexpr (BF == BF_W4) return launch_i8<256, 256, 2, 4, EPI, BF, 3>(a, st);
      else return launch_i8<256, 256, 2, 4, EPI, BF, 2>(a, st);
    case 82: return launch_i8<128, 256, 2, 4, EPI, BF, 3>(a, st);
    case 83: return launch_i8<128, 128, 2, 2, EPI, BF, 3>(a, st);
    case 84: return launch_i8<64, 64, 2, 2, EPI, BF, 3>(a, st);
    case 87: return launch_i8<128, 64, 2, 2, EPI, BF, 3>(a, st);
    case 88: return launch_i8<64, 128, 2, 2, EPI, BF, 3>(a, st);
    case 89: return launch_i8<64, 64, 2, 2, EPI, BF, 2>(a, st);
    case 90: return launch_i8<64, 128, 2, 2, EPI, BF, 2>(a, st);
    case 91: return launch_i8<32, 64, 1, 2, EPI, BF, 2>(a, st);
    case 92: return launch_i8<64, 32, 2, 1, EPI, BF, 2>(a, st);
    // round 6: bigger tiles on a 2-stage ring for the L2-bound vit_b B = 1 shapes (each 64x64 tile
    // re-reads its A and B panels from L2: 128x128 halves those bytes per output)
    case 180: return launch_i8<128, 128, 2, 2, EPI, BF, 2>(a, st);   // 64 KiB: two workgroups per CU
    case 181: return launch_i8<128, 64, 2, 2, EPI, BF, 2>(a, st);    // 48 KiB
    case 182: return launch_i8<128, 128, 2, 4, EPI, BF, 2>(a, st);   // 8 waves of 64x32
    default: return fail(SAMQ_ERR_INVALID, "i8_gemm: unknown tile config");
  }
}

static int i8_cfg_bn(int cfg) {
  switch (cfg) { case 81: case 82: case 85: case 86: case 93: case 94: case 95: case 96: case 97: return 256; case 83: case 88: case 90: case 99: case 180: case 182: return 128; case 84: case 87: case 89: case 91: case 181: return 64;
    case 92: return 32; default: return 0; }
}

static int i8_pick_cfg(int M, int N, int bfmt) {
  // W4 at ViT-H sizes: 256x256 tiles for all four projections.  In steady state (tools/bench_i8.py
  // --m 65536: no tile-round tail) they are the fastest per CU on every shape (lin2 1717 TOPS vs
  // 1602 on 128x128, proj 857 vs 833), and inside the 2-lane W4A8 graph -- the other lane fills
  // tails -- proj / lin2 on them take the step 40.06 -> 38.29 ms, bit-identical
  // (tools/bench_cfg_ab_w4a8.py, profiles/r2_cfg_ab_w4a8.log); the round-1 pick of 128x128 for
  // N = 1280 came from isolated M = 16384 launches (profiles/r1_v11_i8_scan.log).
  // Round 2: the ping-pong kernel for those 256x256 tiles, zero point through row sums (cfg 86): in
  // the 2-lane W4A8 graph (interleaved A/B, tools/bench_cfg_ab_w4a8.py) 37.64 vs 38.33 ms for cfg
  // 81 and 38.34 for cfg 85 (its plain-unpack form; steady state 1710 vs 1760 us per block for 81),
  // bit-identical
  if (bfmt == BF_W4 && M >= 8192) {
    if (N % 256 == 0) return 86;
    if (N % 128 == 0) return 83;
  }
  const int64_t t256 = (int64_t)((M + 127) / 128) * (N / 256);
  // W8 below two rounds of 128x256 tiles (fq_vit vit_b at B=1, M = 4096): 64x64 tiles fill the
  // chip — per block 77 vs 88-90 us (tools/bench_i8.py --w8-vitb, profiles/r1_v17_w8_scan.log).
  // Round 3: on a 2-stage ring (32 KiB LDS, five workgroups per CU instead of three) the W8A8
  // graph takes 1.8325 vs 1.8610 ms per image, bit-identical; 128x64 / 64x128 tiles were slower
  // (tools/bench_cfg_ab_w8a8.py, profiles/r3_w8_cfg_ab.log).
  // Round 5: the wide outputs (qkv N = 2304, lin1 N = 3072 at vit_b) on 64x128 tiles, 2 stages
  // (cfg 90): in the W8A8 graph 1.7067 vs 1.7568 ms per image, bit-identical; proj / lin2 (N = 768)
  // stay on 64x64 (all four on 64x128: 1.7335; profiles/r5_w8_cfg_ab_64x128.log)
  if (bfmt == BF_W8 && t256 < 512 && N % 128 == 0 && N > 1024) return 90;
  if (bfmt == BF_W8 && t256 < 512 && N % 64 == 0) return 89;
  if (N % 256 == 0 && t256 >= 512) return 82;
  if (N % 128 == 0 && M >= 256) return 83;
  return 84;
}

// grouped W4 (ep.kpg K tiles per group): the v3-style kernel with f32 group accumulators beside the
// int32 ones -- wave tiles of at most 64x64 (the pair of accumulator sets must fit the registers)
template <int EPI>
static int launch_i8_grouped(const I8Args& a, int cfg, hipStream_t st) {
  switch (cfg) {
    case 83: return launch_i8<128, 128, 2, 2, EPI, BF_W4, 3, AG_ROWS, true>(a, st);
    case 84: return launch_i8<64, 64, 2, 2, EPI, BF_W4, 3, AG_ROWS, true>(a, st);
    case 87: return launch_i8<128, 64, 2, 2, EPI, BF_W4, 3, AG_ROWS, true>(a, st);
    case 88: return launch_i8<64, 128, 2, 2, EPI, BF_W4, 3, AG_ROWS, true>(a, st);
    default: return fail(SAMQ_ERR_INVALID, "w4a8_gemm: grouped weights take tile configs 83 / 84 / 87 / 88");
  }
}

static int i8_dispatch_grouped(const I8Args& a, int epi, int cfg, hipStream_t st) {
  switch (epi) {
    case SAMQ_EPI_BIAS: return launch_i8_grouped<SAMQ_EPI_BIAS>(a, cfg, st);
    case SAMQ_EPI_BIAS_GELU: return launch_i8_grouped<SAMQ_EPI_BIAS_GELU>(a, cfg, st);
    case SAMQ_EPI_RESADD_F32: return launch_i8_grouped<SAMQ_EPI_RESADD_F32>(a, cfg, st);
    case SAMQ_EPI_F32: return launch_i8_grouped<SAMQ_EPI_F32>(a, cfg, st);
    case SAMQ_EPI_Q8: return launch_i8_grouped<SAMQ_EPI_Q8>(a, cfg, st);
    case SAMQ_EPI_Q8_GELU: return launch_i8_grouped<SAMQ_EPI_Q8_GELU>(a, cfg, st);
    default: return fail(SAMQ_ERR_INVALID, "w4a8_gemm: unknown epilogue for grouped weights");
  }
}

static int i8_dispatch(const I8Args& a, int bfmt, int epi, int cfg, hipStream_t st) {
#define I8_EPI(E) \
  case E: return bfmt == BF_W8 ? launch_i8_cfg<E, BF_W8>(a, cfg, st) : launch_i8_cfg<E, BF_W4>(a, cfg, st)
  switch (epi) {
    I8_EPI(SAMQ_EPI_BIAS);
    I8_EPI(SAMQ_EPI_BIAS_GELU);
    I8_EPI(SAMQ_EPI_RESADD_F32);
    I8_EPI(SAMQ_EPI_F32);
    I8_EPI(SAMQ_EPI_Q8);
    I8_EPI(SAMQ_EPI_Q8_GELU);
    I8_EPI(SAMQ_EPI_Q8_RES);
    default: return fail(SAMQ_ERR_INVALID, "i8_gemm: unknown epilogue");
  }
#undef I8_EPI
}

}  // namespace samq

using namespace samq;

extern "C" int samq_w8_repack(const int8_t* w, int8_t* packed, int K, int N, hipStream_t stream) {
  SAMQ_REQUIRE(w && packed, SAMQ_ERR_INVALID, "w8_repack: null pointer");
  SAMQ_REQUIRE(K > 0 && K % 128 == 0, SAMQ_ERR_INVALID, "w8_repack: K must be a positive multiple of 128");
  SAMQ_REQUIRE(N > 0 && N % 32 == 0, SAMQ_ERR_INVALID, "w8_repack: N must be a multiple of 32");
  SAMQ_REQUIRE(((uintptr_t)w & 15) == 0 && ((uintptr_t)packed & 15) == 0, SAMQ_ERR_INVALID,
               "w8_repack: pointers must be 16-byte aligned");
  const int64_t units = (int64_t)K * N / 16;
  const int blocks = (int)((units + 255) / 256 < 8192 ? (units + 255) / 256 : 8192);
  hipLaunchKernelGGL(w8_repack_kernel, dim3(blocks), dim3(256), 0, stream, w, packed, K, N);
  SAMQ_LAUNCH_CHECK("w8_repack launch");
  return SAMQ_OK;
}

extern "C" int samq_i8_gemm_cfg(const int8_t* A, int64_t lda, int bfmt, const void* wpacked, const float* wscale,
                                const int32_t* qzeros, const float* bias, void* C, int64_t ldc, const int8_t* R,
                                int64_t ldr, int M, int N, int K, int epilogue, float a_scale, float mid_scale,
                                float res_scale, float out_scale, int cfg, hipStream_t stream) {
  if (M == 0) return SAMQ_OK;   // empty batch: no work, data pointers may be null
  SAMQ_REQUIRE(A && wpacked && wscale && C, SAMQ_ERR_INVALID, "i8_gemm: null pointer");
  SAMQ_REQUIRE(bfmt == BF_W8 || bfmt == BF_W4, SAMQ_ERR_INVALID, "i8_gemm: unknown weight format");
  SAMQ_REQUIRE(bfmt == BF_W8 || qzeros, SAMQ_ERR_INVALID, "i8_gemm: W4 needs qzeros");
  SAMQ_REQUIRE(M >= 0 && N > 0 && K > 0 && K % 128 == 0, SAMQ_ERR_INVALID, "i8_gemm: K must be a multiple of 128");
  SAMQ_REQUIRE(N % 64 == 0, SAMQ_ERR_INVALID, "i8_gemm: N must be a multiple of 64");
  SAMQ_REQUIRE(lda >= K && lda % 16 == 0 && ((uintptr_t)A & 15) == 0, SAMQ_ERR_INVALID,
               "i8_gemm: A must be 16-byte aligned with lda >= K, lda % 16 == 0");
  SAMQ_REQUIRE(ldc >= N && ((uintptr_t)C & 15) == 0, SAMQ_ERR_INVALID, "i8_gemm: C must be 16-byte aligned, ldc >= N");
  const bool q8 = epilogue == SAMQ_EPI_Q8 || epilogue == SAMQ_EPI_Q8_GELU || epilogue == SAMQ_EPI_Q8_RES;
  const bool f32 = epilogue == SAMQ_EPI_RESADD_F32 || epilogue == SAMQ_EPI_F32;
  SAMQ_REQUIRE(ldc % (q8 ? 16 : (f32 ? 4 : 8)) == 0, SAMQ_ERR_INVALID, "i8_gemm: ldc breaks 16-byte row alignment");
  SAMQ_REQUIRE(!q8 || out_scale > 0.f, SAMQ_ERR_INVALID, "i8_gemm: quantising epilogue needs out_scale > 0");
  SAMQ_REQUIRE(epilogue != SAMQ_EPI_Q8_RES || (R && ldr % 16 == 0 && ((uintptr_t)R & 15) == 0), SAMQ_ERR_INVALID,
               "i8_gemm: Q8_RES needs a 16-byte aligned residual R with ldr % 16 == 0");
  if (M == 0) return SAMQ_OK;
  if (cfg <= 0) cfg = i8_pick_cfg(M, N, bfmt);
  SAMQ_REQUIRE(i8_cfg_bn(cfg) > 0 && N % i8_cfg_bn(cfg) == 0, SAMQ_ERR_INVALID, "i8_gemm: N not divisible by tile");
  I8Args a{A, lda, (const char*)wpacked, wscale, (const uint32_t*)qzeros, bias, C, ldc, M, N, K,
           I8Epi{a_scale, mid_scale, res_scale, out_scale, R, ldr, 0}, I8Gather{0, 0, 0}};
  return i8_dispatch(a, bfmt, epilogue, cfg, stream);
}

extern "C" int samq_w8a8_conv_gemm(const int8_t* x, int mode, int B, int Cin, int side, const int8_t* wpacked,
                                   const float* wscale, const float* bias, void* C, const int8_t* R, int rmod,
                                   int N, int epilogue, float a_scale, float mid_scale, float res_scale,
                                   float out_scale, hipStream_t stream) {
  if (B == 0) return SAMQ_OK;   // empty batch: no work, data pointers may be null
  SAMQ_REQUIRE(x && wpacked && wscale && C, SAMQ_ERR_INVALID, "w8a8_conv_gemm: null pointer");
  SAMQ_REQUIRE(mode == AG_PATCH || mode == AG_3X3, SAMQ_ERR_INVALID, "w8a8_conv_gemm: mode must be 1 (patch) or 2 (3x3)");
  SAMQ_REQUIRE(epilogue == SAMQ_EPI_Q8 || epilogue == SAMQ_EPI_Q8_RES, SAMQ_ERR_UNSUPPORTED,
               "w8a8_conv_gemm: epilogue must be Q8 or Q8_RES");
  SAMQ_REQUIRE(B > 0 && Cin > 0 && side > 0 && N > 0 && N % 64 == 0, SAMQ_ERR_INVALID, "w8a8_conv_gemm: bad shape");
  SAMQ_REQUIRE(out_scale > 0.f, SAMQ_ERR_INVALID, "w8a8_conv_gemm: needs out_scale > 0");
  SAMQ_REQUIRE(epilogue != SAMQ_EPI_Q8_RES || (R && ((uintptr_t)R & 15) == 0), SAMQ_ERR_INVALID,
               "w8a8_conv_gemm: Q8_RES needs a 16-byte aligned residual");
  SAMQ_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)C & 15) == 0, SAMQ_ERR_INVALID,
               "w8a8_conv_gemm: operands must be 16-byte aligned");
  int G, K;
  if (mode == AG_PATCH) {
    SAMQ_REQUIRE(side % 16 == 0 && (Cin * 256) % 128 == 0, SAMQ_ERR_UNSUPPORTED,
                 "w8a8_conv_gemm: patch mode is the 16x16 / stride 16 PatchEmbed");
    G = side / 16;
    K = Cin * 256;
  } else {
    SAMQ_REQUIRE(Cin % 128 == 0, SAMQ_ERR_UNSUPPORTED, "w8a8_conv_gemm: 3x3 mode needs Cin % 128 == 0");
    G = side;
    K = 9 * Cin;
  }
  const int M = B * G * G;
  I8Args a{x, K, (const char*)wpacked, wscale, nullptr, bias, C, N, M, N, K,
           I8Epi{a_scale, mid_scale, res_scale, out_scale, R, N, rmod}, I8Gather{side, G, Cin}};
  if (epilogue == SAMQ_EPI_Q8)
    return mode == AG_PATCH ? launch_i8<64, 64, 2, 2, SAMQ_EPI_Q8, BF_W8, 3, AG_PATCH>(a, stream)
                            : launch_i8<64, 64, 2, 2, SAMQ_EPI_Q8, BF_W8, 3, AG_3X3>(a, stream);
  return mode == AG_PATCH ? launch_i8<64, 64, 2, 2, SAMQ_EPI_Q8_RES, BF_W8, 3, AG_PATCH>(a, stream)
                          : launch_i8<64, 64, 2, 2, SAMQ_EPI_Q8_RES, BF_W8, 3, AG_3X3>(a, stream);
}

extern "C" int samq_w8a8_gemm(const int8_t* A, int64_t lda, const int8_t* wpacked, const float* wscale,
                              const float* bias, void* C, int64_t ldc, const int8_t* R, int64_t ldr, int M, int N,
                              int K, int epilogue, float a_scale, float mid_scale, float res_scale, float out_scale,
                              hipStream_t stream) {
  return samq_i8_gemm_cfg(A, lda, BF_W8, wpacked, wscale, nullptr, bias, C, ldc, R, ldr, M, N, K, epilogue, a_scale,
                          mid_scale, res_scale, out_scale, 0, stream);
}

extern "C" int samq_w4a8_gemm_cfg(const int8_t* A, int64_t lda, const int32_t* wpacked, const float* wscale,
                                  const int32_t* qzeros, const float* bias, void* C, int64_t ldc, int M, int N,
                                  int K, int groupsize, int epilogue, float a_scale, float out_scale, int cfg,
                                  hipStream_t stream) {
  SAMQ_REQUIRE(epilogue != SAMQ_EPI_Q8_RES, SAMQ_ERR_INVALID, "w4a8_gemm: Q8_RES is a W8A8 epilogue");
  if (groupsize == -1 || groupsize == K)
    return samq_i8_gemm_cfg(A, lda, BF_W4, wpacked, wscale, qzeros, bias, C, ldc, nullptr, 0, M, N, K, epilogue,
                            a_scale, 0.f, 0.f, out_scale, cfg, stream);
  // grouped weights (gptq_triton/quant_linear.py:324-335: per-group scale / zero rows)
  if (M == 0) return SAMQ_OK;   // empty batch: no work, data pointers may be null
  SAMQ_REQUIRE(A && wpacked && wscale && qzeros && C, SAMQ_ERR_INVALID, "w4a8_gemm: null pointer");
  SAMQ_REQUIRE(M >= 0 && N > 0 && K > 0 && K % 128 == 0 && N % 64 == 0, SAMQ_ERR_INVALID,
               "w4a8_gemm: K % 128 == 0 and N % 64 == 0 required");
  SAMQ_REQUIRE(groupsize > 0 && groupsize % 128 == 0, SAMQ_ERR_UNSUPPORTED,
               "w4a8_gemm: grouped weights need a groupsize that is a multiple of 128 (the int8 K tile)");
  SAMQ_REQUIRE(lda >= K && lda % 16 == 0 && ((uintptr_t)A & 15) == 0, SAMQ_ERR_INVALID,
               "w4a8_gemm: A must be 16-byte aligned with lda >= K, lda % 16 == 0");
  const bool q8 = epilogue == SAMQ_EPI_Q8 || epilogue == SAMQ_EPI_Q8_GELU;
  const bool f32 = epilogue == SAMQ_EPI_RESADD_F32 || epilogue == SAMQ_EPI_F32;
  SAMQ_REQUIRE(ldc >= N && ((uintptr_t)C & 15) == 0 && ldc % (q8 ? 16 : (f32 ? 4 : 8)) == 0, SAMQ_ERR_INVALID,
               "w4a8_gemm: C must be 16-byte aligned rows, ldc >= N");
  SAMQ_REQUIRE(!q8 || out_scale > 0.f, SAMQ_ERR_INVALID, "w4a8_gemm: quantising epilogue needs out_scale > 0");
  if (M == 0) return SAMQ_OK;
  if (cfg <= 0) cfg = N % 128 == 0 && M >= 1024 ? 83 : 84;
  SAMQ_REQUIRE(i8_cfg_bn(cfg) > 0 && N % i8_cfg_bn(cfg) == 0, SAMQ_ERR_INVALID, "w4a8_gemm: N not divisible by tile");
  I8Args a{A, lda, (const char*)wpacked, wscale, (const uint32_t*)qzeros, bias, C, ldc, M, N, K,
           I8Epi{a_scale, 0.f, 0.f, out_scale, nullptr, 0, 0, groupsize / 128}, I8Gather{0, 0, 0}};
  return i8_dispatch_grouped(a, epilogue, cfg, stream);
}

extern "C" int samq_w8a8_gemm_v16(const int8_t* A, int64_t lda, const int8_t* wpacked, const float* wscale,
                                  const float* bias, int8_t* C, int64_t ldc, int M, int N, int K, float a_scale,
                                  float out_scale, void* v16, int v_col0, int64_t ldv, int cfg, hipStream_t stream) {
  if (M == 0) return SAMQ_OK;   // empty batch: no work, data pointers may be null
  SAMQ_REQUIRE(A && wpacked && wscale && C && v16, SAMQ_ERR_INVALID, "w8a8_gemm_v16: null pointer");
  SAMQ_REQUIRE(M > 0 && N > 0 && K > 0 && K % 128 == 0 && N % 64 == 0, SAMQ_ERR_INVALID,
               "w8a8_gemm_v16: K % 128 == 0 and N % 64 == 0 required");
  SAMQ_REQUIRE(lda >= K && lda % 16 == 0 && ((uintptr_t)A & 15) == 0 && ldc >= N && ldc % 16 == 0 &&
               ((uintptr_t)C & 15) == 0, SAMQ_ERR_INVALID, "w8a8_gemm_v16: 16-byte aligned rows required");
  SAMQ_REQUIRE(out_scale > 0.f, SAMQ_ERR_INVALID, "w8a8_gemm_v16: needs out_scale > 0");
  if (cfg <= 0) cfg = i8_pick_cfg(M, N, BF_W8);
  const int bn = i8_cfg_bn(cfg);
  SAMQ_REQUIRE(bn > 0 && N % bn == 0, SAMQ_ERR_INVALID, "w8a8_gemm_v16: N not divisible by tile");
  SAMQ_REQUIRE(v_col0 >= 0 && v_col0 < N && v_col0 % 64 == 0 && ldv >= N - v_col0 && ldv % 8 == 0 &&
               ((uintptr_t)v16 & 15) == 0, SAMQ_ERR_INVALID,
               "w8a8_gemm_v16: v_col0 must be a multiple of 64 inside N; v16 rows 16-byte aligned, ldv >= N - v_col0");
  I8Args a{A, lda, (const char*)wpacked, wscale, nullptr, bias, C, ldc, M, N, K,
           I8Epi{a_scale, 0.f, 0.f, out_scale, nullptr, 0, 0, 0, nullptr, nullptr, (_Float16*)v16, v_col0, ldv},
           I8Gather{0, 0, 0}};
  return launch_i8_cfg<SAMQ_EPI_Q8, BF_W8>(a, cfg, stream);
}

extern "C" int samq_w4a8_gemm_rs(const int8_t* A, int64_t lda, const int32_t* wpacked, const float* wscale,
                                 const int32_t* qzeros, const float* bias, void* C, int64_t ldc, int M, int N, int K,
                                 int epilogue, float a_scale, float out_scale, const int32_t* rowsum_in,
                                 int32_t* rowsum_out, int cfg, hipStream_t stream) {
  if (M == 0) return SAMQ_OK;   // empty batch: no work, data pointers may be null
  SAMQ_REQUIRE(epilogue != SAMQ_EPI_Q8_RES, SAMQ_ERR_INVALID, "w4a8_gemm_rs: Q8_RES is a W8A8 epilogue");
  SAMQ_REQUIRE(!rowsum_out || epilogue == SAMQ_EPI_Q8 || epilogue == SAMQ_EPI_Q8_GELU, SAMQ_ERR_INVALID,
               "w4a8_gemm_rs: rowsum_out needs an int8-code epilogue (Q8 / Q8_GELU)");
  SAMQ_REQUIRE(M < (1 << 30) && (!rowsum_in || K < 65536), SAMQ_ERR_UNSUPPORTED,
               "w4a8_gemm_rs: row sums need K < 65536");
  SAMQ_REQUIRE(A && wpacked && wscale && qzeros && C, SAMQ_ERR_INVALID, "w4a8_gemm_rs: null pointer");
  SAMQ_REQUIRE(lda >= K && lda % 16 == 0 && ((uintptr_t)A & 15) == 0, SAMQ_ERR_INVALID,
               "w4a8_gemm_rs: A must be 16-byte aligned with lda >= K, lda % 16 == 0");
  SAMQ_REQUIRE(M > 0 && N > 0 && K > 0 && K % 128 == 0 && N % 64 == 0, SAMQ_ERR_INVALID,
               "w4a8_gemm_rs: K % 128 == 0 and N % 64 == 0 required");
  const bool q8 = epilogue == SAMQ_EPI_Q8 || epilogue == SAMQ_EPI_Q8_GELU;
  const bool f32 = epilogue == SAMQ_EPI_RESADD_F32 || epilogue == SAMQ_EPI_F32;
  SAMQ_REQUIRE(ldc >= N && ((uintptr_t)C & 15) == 0 && ldc % (q8 ? 16 : (f32 ? 4 : 8)) == 0, SAMQ_ERR_INVALID,
               "w4a8_gemm_rs: C must be 16-byte aligned rows, ldc >= N");
  SAMQ_REQUIRE(!q8 || out_scale > 0.f, SAMQ_ERR_INVALID, "w4a8_gemm_rs: quantising epilogue needs out_scale > 0");
  if (cfg <= 0) cfg = i8_pick_cfg(M, N, BF_W4);
  SAMQ_REQUIRE(i8_cfg_bn(cfg) > 0 && N % i8_cfg_bn(cfg) == 0, SAMQ_ERR_INVALID, "w4a8_gemm_rs: N not divisible by tile");
  I8Args a{A, lda, (const char*)wpacked, wscale, (const uint32_t*)qzeros, bias, C, ldc, M, N, K,
           I8Epi{a_scale, 0.f, 0.f, out_scale, nullptr, 0, 0, 0, rowsum_in, rowsum_out}, I8Gather{0, 0, 0}};
  return i8_dispatch(a, BF_W4, epilogue, cfg, stream);
}

extern "C" int samq_w4a8_gemm(const int8_t* A, int64_t lda, const int32_t* wpacked, const float* wscale,
                              const int32_t* qzeros, const float* bias, void* C, int64_t ldc, int M, int N, int K,
                              int groupsize, int epilogue, float a_scale, float out_scale, hipStream_t stream) {
  return samq_w4a8_gemm_cfg(A, lda, wpacked, wscale, qzeros, bias, C, ldc, M, N, K, groupsize, epilogue, a_scale,
                            out_scale, 0, stream);
}

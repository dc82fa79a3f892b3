// Windowed / global multi-head attention with in-kernel decomposed relative-position bias.
//
// Replaces QuantAttention's attention part (gptq_triton/fused_attention.py:107-149): the two
// torch.matmul rel-pos products (add_decomposed_rel_pos :46-80), the `torch.full(+inf)` output
// init and the Triton flash kernel `_fwd_kernel1` (:159-309) -- and, in the windowed blocks,
// the window_partition / window_unpartition copies (image_encoder.py:195-202, 282-333): tokens
// are read from / written to the natural [B, H, W, C] layout, padded window tokens are
// synthesised in-kernel (their q/k/v equal the qkv bias).
//
// Structure (gfx950, wave64, v_mfma_f32_16x16x32_f16, 7-8 waves per workgroup = 2 waves/SIMD):
//  * work unit = (window or image, head, block of query tiles); a query tile is 16 queries of
//    ONE grid row (rows padded to SP = 16 / 32 / 64 slots), so a tile has one query row qh;
//  * keys are consumed one GRID ROW at a time (SP slots).  For key row kh the scores are
//        s[q, kw] = q.k * scale + TH[q, kh] + TW[q, kw]
//    TW[q, kw] = q . Rw[qh - kw + S - 1] is identical for every key row: it is computed once per
//    query tile by MFMA directly in the score-tile register layout and fed as the C input of
//    every Q.K^T; TH[q, kh] = q . Rh[qh - kh + S - 1] is constant along the row, so it is folded
//    into the running max instead of being added per score.  (Both tables are indexed by the
//    query ROW qh: reference quirk 1.)
//  * scores are computed transposed (S^T = K . Q^T): each lane owns one query, row reductions are
//    in-register + 2 cross-lane steps; P feeds O^T += V^T . P^T as the B operand with a permuted
//    k order that V^T supplies through ds_read_b64_tr_b16 from the row-major V tile;
//  * K / V rows reach LDS by global_load_lds (no VGPR round trip): windows (S <= 16) are staged
//    whole before the loop (no barrier inside it); global attention streams key rows through a
//    3-deep LDS ring with counted vmcnt and one raw s_barrier per row;
//  * online softmax in the exp2 domain with f32 statistics; the O rescale is skipped when no
//    query of the wave raised its max (alpha == 1 exactly, bit-identical results).
#include "common.h"

namespace samq {

constexpr float LOG2E = 1.4426950408889634f;

__device__ __attribute__((aligned(16))) _Float16 g_zero16[8];   // zero source for pad slots

struct AttnParams {
  const _Float16* qkv;      // token stride tok_stride (elements); q at h*D, k at C+h*D, v at 2C+h*D
  const _Float16* qkv_bias; // [3C] or null
  const _Float16* relh;     // table [2S-1][D] f16  | precomputed [B'*heads][S][S][S] f16
  const _Float16* relw;
  _Float16* out;            // token stride C
  int64_t tok_stride;
  int C, heads;
  int S;                    // window side (windowed) or grid side (global)
  int H, W;                 // image token grid
  int nwx, upi;             // windows per row, windows per image
  float scale;              // sm_scale
};

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N <= 15, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ds_read_b64_tr_b16 through inline asm: the intrinsic form carries no alias information, so the
// compiler treats it as possibly reading the in-flight LDS-DMA ring and drains vmcnt(0) before it
// (killing the K/V prefetch).  The asm form is invisible to that analysis; the caller waits
// lgkmcnt itself (lds_wait below, which also orders the MFMAs after the wait).
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)((const SAMQ_LDS char*)p);
}
__device__ __forceinline__ half4_t ds_read_tr16(uint32_t addr) {
  half4_t r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}

__device__ __forceinline__ float max3f(float a, float b, float c) {
  // NOT inline asm: the hazard recognizer does not pad an asm VALU read of a fresh MFMA result,
  // which then reads stale accumulator lanes at random (nondeterministic scores).
  return fmaxf(fmaxf(a, b), c);
}

template <int D, int SP, int QT, int NW, bool RESIDENT, bool PRECOMP, int RS = 16, int SC = 0>
__global__ __launch_bounds__(64 * NW, 1) void rel_attention_kernel(AttnParams p) {
  constexpr int KT = SP / 16;                  // key tiles per key row
  constexpr int DT = D / 16;                   // output d tiles
  constexpr int KS = (D + 31) / 32;            // k32 steps of Q.K^T (D=80 -> 3, last half-zero)
  constexpr int D8 = D / 8;                    // 16-byte chunks per token
  constexpr int ROWB = SP * D * 2;             // bytes of one key row (K or V) in LDS
  // RESIDENT: the keys of the whole (<= RS x RS) grid packed with row pitch S, plus 16 - S slack
  // keys so the 16-slot tile of the last row stays in bounds (slots >= S are masked)
  constexpr int RKEYS = RS * RS + 16 - RS;
  constexpr int UNIT_CHUNKS = RESIDENT ? 2 * RKEYS * D8 : 2 * SP * D8;
  constexpr int NI = (UNIT_CHUNKS + 64 * NW - 1) / (64 * NW);   // glds per wave per unit
  constexpr int BUFB = NI * NW * 1024;
  constexpr int NBUF = RESIDENT ? 1 : 3;
  constexpr int TH_ROWS = RESIDENT ? 16 : SP;   // >= 16: the TH tile writes 16 rows
  constexpr int TH_BYTES = NW * QT * TH_ROWS * 16 * 4;
  static_assert(D == 64 || D == 80, "head dim");
  static_assert(!RESIDENT || SP == 16, "resident mode holds <= 16 rows of 16 slots");

  __shared__ __attribute__((aligned(16))) char smem[NBUF * BUFB + TH_BYTES];
  float* th_lds = (float*)(smem + NBUF * BUFB);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int ql = lane & 15;
  const int g = lane >> 4;
  const int head = blockIdx.y;
  const int unit = blockIdx.z;
  const int S = SC ? SC : p.S;   // grid side, compile-time where the dispatcher knows it
  const int b = unit / p.upi;
  const int wi = unit % p.upi;
  const int Y0 = (wi / p.nwx) * S;
  const int X0 = (wi % p.nwx) * S;
  const int C = p.C;
  const float qscale = p.scale * LOG2E;

  // 0 = real token, 1 = window pad (q/k/v = bias), 2 = slot beyond the row (masked / unused)
  auto tok_kind = [&](int y, int x) -> int {
    if (x >= S || y >= S) return 2;
    return (Y0 + y < p.H && X0 + x < p.W) ? 0 : 1;
  };
  auto tok_ptr = [&](int y, int x) -> const _Float16* {
    return p.qkv + (((int64_t)b * p.H + (Y0 + y)) * p.W + (X0 + x)) * p.tok_stride;
  };

  // ---------------------------------------------------------------- K/V staging (LDS-DMA)
  // chunk c of a unit -> LDS byte c*16; unit layout [K|V][key][D] (STREAM: one row of SP slots;
  // RESIDENT: key r*S + x of the whole grid)
  // per-lane sources for key row 0 (STREAM) / the whole grid (RESIDENT); a STREAM row kh is the
  // same pattern kh grid rows further down, so the loop only adds kh * rowstride
  const _Float16* src0[NI];
  bool adv[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int c = (wave * NI + i) * 64 + lane;
    const _Float16* src = g_zero16;
    bool real = false;
    if (c < UNIT_CHUNKS) {
      constexpr int HALF = UNIT_CHUNKS / 2;
      const bool isv = c >= HALF;
      const int cc = isv ? c - HALF : c;
      const int key = cc / D8, d8 = cc % D8;
      const int r = RESIDENT ? key / S : 0;
      const int slot = RESIDENT ? key % S : key;
      const int kind = r < S ? tok_kind(r, slot) : 2;
      const int off = (isv ? 2 * C : C) + head * D + d8 * 8;
      if (kind == 0) { src = tok_ptr(r, slot) + off; real = true; }
      else if (kind == 1 && p.qkv_bias) src = p.qkv_bias + off;
    }
    src0[i] = src;
    adv[i] = real && !RESIDENT;
  }
  const int64_t rowstride = (int64_t)p.W * p.tok_stride;
  auto issue = [&](int row0, int buf) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const _Float16* src = adv[i] ? src0[i] + row0 * rowstride : src0[i];
      __builtin_amdgcn_global_load_lds((const SAMQ_GLOBAL void*)src,
                                       (SAMQ_LDS void*)(smem + buf * BUFB + (wave * NI + i) * 1024), 16, 0, 0);
    }
  };

  // start the K/V traffic first, it overlaps the Q / rel-pos prologue
  issue(0, 0);
  if (!RESIDENT && S > 1) issue(1, 1);

  // ---------------------------------------------------------------- Q fragments (scaled)
  const bool kin3 = 64 + 8 * g < D;   // this lane group holds real d in the last k-step
  half8_t qf[QT][KS];
  int qrow[QT], qcol0[QT];
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    const int qi = (blockIdx.x * NW + wave) * QT + t;
    qrow[t] = qi / KT;
    qcol0[t] = (qi % KT) * 16;
    const int kind = tok_kind(qrow[t], qcol0[t] + ql);
    const _Float16* src = nullptr;
    if (kind == 0) src = tok_ptr(qrow[t], qcol0[t] + ql) + head * D;
    else if (kind == 1 && p.qkv_bias) src = p.qkv_bias + head * D;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      half8_t v = {};
      if (src && (s < 2 || kin3)) v = *(const half8_t*)(src + 32 * s + 8 * g);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (_Float16)((float)v[j] * qscale);
      qf[t][s] = v;
    }
  }

  // ---------------------------------------------------------------- rel-pos terms
  float4_t tw[QT][KT];
  const float inv_scale = 1.0f / p.scale;  // (Qs . R) / scale = log2e * (q . R)
  float* th_w = th_lds + wave * (QT * TH_ROWS * 16);
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    const int qh = qrow[t] < S ? qrow[t] : S - 1;
    if (!PRECOMP) {
#pragma unroll
      for (int which = 0; which < 2; ++which) {
        const _Float16* tab = which ? p.relw : p.relh;
#pragma unroll
        for (int kt = 0; kt < KT; ++kt) {
          int r = qh - (kt * 16 + ql) + S - 1;     // table row of this lane's A-operand row
          r = r < 0 ? 0 : r;
          const _Float16* rp = tab + (int64_t)r * D;
          float4_t a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            half8_t ra = {};
            if (s < 2 || kin3) ra = *(const half8_t*)(rp + 32 * s + 8 * g);
            a = __builtin_amdgcn_mfma_f32_16x16x32_f16(ra, qf[t][s], a, 0, 0, 0);
          }
          a = a * inv_scale;
          if (which) {
            tw[t][kt] = a;
          } else {
#pragma unroll
            for (int r2 = 0; r2 < 4; ++r2) th_w[(t * TH_ROWS + kt * 16 + 4 * g + r2) * 16 + ql] = a[r2];
          }
        }
      }
    } else {
      // precomputed bias tensors [B'*heads][S][S][S]: rel_h[.., qh, qw, kh], rel_w[.., qh, qw, kw]
      const int qw = qcol0[t] + ql;
      const bool ok = qw < S && qrow[t] < S;
      const int64_t base = ((((int64_t)unit * p.heads + head) * S + qh) * S + (ok ? qw : 0)) * S;
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
#pragma unroll
        for (int r2 = 0; r2 < 4; ++r2) {
          const int kk = kt * 16 + 4 * g + r2;
          const bool kin = ok && kk < S;
          tw[t][kt][r2] = kin ? (float)p.relw[base + kk] * LOG2E : 0.f;
          th_w[(t * TH_ROWS + kk) * 16 + ql] = kin ? (float)p.relh[base + kk] * LOG2E : 0.f;
        }
      }
    }
  }

  float m[QT], l[QT];
  float4_t o[QT][DT];
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    m[t] = -INFINITY;
    l[t] = 0.f;
#pragma unroll
    for (int d = 0; d < DT; ++d) o[t][d] = float4_t{0.f, 0.f, 0.f, 0.f};
  }
  const bool mask_slots = S < SP;
  const int trow = ql >> 2;            // ds_read_b64_tr_b16: lane 4q+p of a 16-lane group reads
  const int tcol = 4 * (ql & 3);       // block row q, columns 4p..4p+3; receives column (lane&15)

  if (RESIDENT) {
    wait_vmcnt<0>();
    __syncthreads();   // K/V of the whole window + TH visible
  } else {
    __syncthreads();   // TH visible (the K/V ring is ordered by counted vmcnt + s_barrier below)
  }

  for (int kh = 0; kh < S; ++kh) {
    const char* kb;
    if (RESIDENT) {
      kb = smem + kh * S * (D * 2);
    } else {
      if (kh + 1 < S) wait_vmcnt<NI>(); else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();   // row kh landed for every wave; row kh-1 fully consumed
      if (kh + 2 < S) issue(kh + 2, (kh + 2) % 3);
      kb = smem + (kh % 3) * BUFB;
    }
    const char* vb = kb + (RESIDENT ? (UNIT_CHUNKS / 2) * 16 : ROWB);

    // ---- scores S^T = K . Q^T (+ TW as the C input)
    float4_t sc[QT][KT];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      const char* krow = kb + (kt * 16 + ql) * (D * 2);
      half8_t kf[KS];
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        kf[s] = half8_t{};
        if (s < 2 || kin3) kf[s] = *(const half8_t*)(krow + (32 * s + 8 * g) * 2);
      }
#pragma unroll
      for (int t = 0; t < QT; ++t) {
        float4_t a = tw[t][kt];
#pragma unroll
        for (int s = 0; s < KS; ++s) a = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[s], qf[t][s], a, 0, 0, 0);
        sc[t][kt] = a;
      }
    }

    // ---- online softmax (exp2 domain); TH[q, kh] is constant along the row
    half8_t pb[QT][(SP + 31) / 32];
    half4_t pb16[QT];
    bool any_rescale = false;
    float alpha[QT];
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      if (mask_slots) {
#pragma unroll
        for (int kt = 0; kt < KT; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (kt * 16 + 4 * g + r >= S) sc[t][kt][r] = -INFINITY;
      }
      float mx = max3f(sc[t][0][0], sc[t][0][1], sc[t][0][2]);
      mx = max3f(mx, sc[t][0][3], mx);
#pragma unroll
      for (int kt = 1; kt < KT; ++kt) {
        mx = max3f(mx, sc[t][kt][0], sc[t][kt][1]);
        mx = max3f(mx, sc[t][kt][2], sc[t][kt][3]);
      }
      mx = max3f(mx, __shfl_xor(mx, 16, 64), __shfl_xor(mx, 32, 64));
      mx = max3f(mx, __shfl_xor(mx, 16, 64), mx);
      const float th = th_w[(t * TH_ROWS + kh) * 16 + ql];
      const float mnew = fmaxf(m[t], mx + th);
      alpha[t] = __builtin_amdgcn_exp2f(m[t] - mnew);
      any_rescale |= mnew != m[t];
      m[t] = mnew;
      const float corr = mnew - th;
      float rs = 0.f;
#pragma unroll
      for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __builtin_amdgcn_exp2f(sc[t][kt][r] - corr);
          sc[t][kt][r] = e;
          rs += e;
        }
      l[t] = l[t] * alpha[t] + rs;
      if (SP == 16) {
        pb16[t] = half4_t{(_Float16)sc[t][0][0], (_Float16)sc[t][0][1], (_Float16)sc[t][0][2], (_Float16)sc[t][0][3]};
      } else {
#pragma unroll
        for (int s = 0; s < SP / 32; ++s) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            pb[t][s][r] = (_Float16)sc[t][2 * s][r];
            pb[t][s][4 + r] = (_Float16)sc[t][2 * s + 1][r];
          }
        }
      }
    }
    if (__any(any_rescale)) {
#pragma unroll
      for (int t = 0; t < QT; ++t)
#pragma unroll
        for (int d = 0; d < DT; ++d) o[t][d] = o[t][d] * alpha[t];
    }

    // ---- O^T += V^T . P^T  (V^T fragments by hardware-transposed LDS reads of row-major V)
#pragma unroll
    for (int d = 0; d < DT; ++d) {
      if constexpr (SP == 16) {
        const char* a0 = vb + ((4 * g + trow) * D + d * 16 + tcol) * 2;
        const half4_t va = __builtin_bit_cast(
            half4_t, __builtin_amdgcn_ds_read_tr16_b64_v4i16((SAMQ_LDS short4_t*)(a0)));
#pragma unroll
        for (int t = 0; t < QT; ++t) o[t][d] = __builtin_amdgcn_mfma_f32_16x16x16f16(va, pb16[t], o[t][d], 0, 0, 0);
      } else {
        constexpr int NS = SP / 32;
        half4_t lo[NS], hi[NS];
        const uint32_t vaddr = lds_addr(vb + ((4 * g + trow) * D + d * 16 + tcol) * 2);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          lo[s] = ds_read_tr16(vaddr + (32 * s) * D * 2);
          hi[s] = ds_read_tr16(vaddr + (32 * s + 16) * D * 2);
        }
        if constexpr (NS == 2) {
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(lo[0]), "+v"(hi[0]), "+v"(lo[1]), "+v"(hi[1]));
        } else {
#pragma unroll
          for (int s = 0; s < NS; ++s) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(lo[s]), "+v"(hi[s]));
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const half8_t va = {lo[s][0], lo[s][1], lo[s][2], lo[s][3], hi[s][0], hi[s][1], hi[s][2], hi[s][3]};
#pragma unroll
          for (int t = 0; t < QT; ++t) o[t][d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va, pb[t][s], o[t][d], 0, 0, 0);
        }
      }
    }
  }

  // ---------------------------------------------------------------- normalise + store
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    float lt = l[t];
    lt += __shfl_xor(lt, 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    const int x = qcol0[t] + ql;
    if (tok_kind(qrow[t], x) != 0) continue;
    const float inv = 1.0f / lt;
    _Float16* dst = p.out + (((int64_t)b * p.H + (Y0 + qrow[t])) * p.W + (X0 + x)) * C + head * D;
#pragma unroll
    for (int d = 0; d < DT; ++d) {
      half4_t v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = (_Float16)(o[t][d][r] * inv);
      *(half4_t*)(dst + d * 16 + 4 * g) = v;
    }
  }
}

template <int D, int SP, int QT, int NW, bool RES, bool PRE, int RS = 16, int SC = 0>
static int launch_attn(const AttnParams& p, int units, hipStream_t stream) {
  const int tiles = p.S * (SP / 16);
  const int qblocks = (tiles + NW * QT - 1) / (NW * QT);
  hipLaunchKernelGGL((rel_attention_kernel<D, SP, QT, NW, RES, PRE, RS, SC>), dim3(qblocks, p.heads, units),
                     dim3(64 * NW), 0, stream, p);
  SAMQ_LAUNCH_CHECK("rel_attention launch");
  return SAMQ_OK;
}

template <bool PRE>
static int dispatch_attn(const AttnParams& p, int hd, int units, hipStream_t stream) {
  const int S = p.S;
  if (S <= 16) {  // whole window / small grid resident in LDS; one query tile per grid row
    if (S == 14)
      return hd == 80 ? launch_attn<80, 16, 2, 7, true, PRE, 14, 14>(p, units, stream)
                      : launch_attn<64, 16, 2, 7, true, PRE, 14, 14>(p, units, stream);
    return hd == 80 ? launch_attn<80, 16, 2, 8, true, PRE>(p, units, stream)
                    : launch_attn<64, 16, 2, 8, true, PRE>(p, units, stream);
  } else if (S == 32) {
    return hd == 80 ? launch_attn<80, 32, 2, 8, false, PRE, 16, 32>(p, units, stream)
                    : launch_attn<64, 32, 2, 8, false, PRE, 16, 32>(p, units, stream);
  } else {
    return hd == 80 ? launch_attn<80, 64, 2, 8, false, PRE, 16, 64>(p, units, stream)
                    : launch_attn<64, 64, 2, 8, false, PRE, 16, 64>(p, units, stream);
  }
}

}  // namespace samq

using namespace samq;

extern "C" int samq_rel_attention(const void* qkv, const void* qkv_bias, const void* rel_pos_h, const void* rel_pos_w,
                                  void* out, int B, int H, int W, int heads, int hd, int window, float sm_scale,
                                  hipStream_t stream) {
  SAMQ_REQUIRE(qkv && rel_pos_h && rel_pos_w && out, SAMQ_ERR_INVALID, "rel_attention: null pointer");
  SAMQ_REQUIRE(hd == 64 || hd == 80, SAMQ_ERR_UNSUPPORTED, "rel_attention: head_dim must be 64 or 80");
  SAMQ_REQUIRE(B > 0 && H > 0 && W > 0 && heads > 0, SAMQ_ERR_INVALID, "rel_attention: bad shape");
  AttnParams p{};
  p.qkv = (const _Float16*)qkv;
  p.qkv_bias = (const _Float16*)qkv_bias;
  p.relh = (const _Float16*)rel_pos_h;
  p.relw = (const _Float16*)rel_pos_w;
  p.out = (_Float16*)out;
  p.C = heads * hd;
  p.tok_stride = 3 * (int64_t)p.C;
  p.heads = heads;
  p.H = H;
  p.W = W;
  p.scale = sm_scale;
  int units;
  if (window > 0) {
    SAMQ_REQUIRE(window <= 16, SAMQ_ERR_UNSUPPORTED, "rel_attention: window must be <= 16");
    p.S = window;
    const int nwy = (H + window - 1) / window, nwx = (W + window - 1) / window;
    p.nwx = nwx;
    p.upi = nwy * nwx;
    units = B * p.upi;
  } else {
    SAMQ_REQUIRE(H == W, SAMQ_ERR_UNSUPPORTED, "rel_attention: global attention needs H == W");
    SAMQ_REQUIRE(H <= 16 || H == 32 || H == 64, SAMQ_ERR_UNSUPPORTED,
                 "rel_attention: global grid side must be <= 16, 32 or 64");
    p.S = H;
    p.nwx = 1;
    p.upi = 1;
    units = B;
  }
  SAMQ_REQUIRE(units <= 65535, SAMQ_ERR_INVALID, "rel_attention: too many windows*batch");
  return dispatch_attn<false>(p, hd, units, stream);
}

extern "C" int samq_attention_relbias(const void* inp, const void* rel_h, const void* rel_w, void* out, int B, int S,
                                      int heads, int hd, float sm_scale, hipStream_t stream) {
  SAMQ_REQUIRE(inp && rel_h && rel_w && out, SAMQ_ERR_INVALID, "attention_relbias: null pointer");
  SAMQ_REQUIRE(hd == 64 || hd == 80, SAMQ_ERR_UNSUPPORTED, "attention_relbias: head_dim must be 64 or 80");
  SAMQ_REQUIRE(B > 0 && B <= 65535 && heads > 0, SAMQ_ERR_INVALID, "attention_relbias: bad shape");
  SAMQ_REQUIRE(S <= 16 || S == 32 || S == 64, SAMQ_ERR_UNSUPPORTED,
               "attention_relbias: grid side must be <= 16, 32 or 64");
  AttnParams p{};
  p.qkv = (const _Float16*)inp;
  p.qkv_bias = nullptr;
  p.relh = (const _Float16*)rel_h;
  p.relw = (const _Float16*)rel_w;
  p.out = (_Float16*)out;
  p.C = heads * hd;
  p.tok_stride = 3 * (int64_t)p.C;
  p.heads = heads;
  p.S = S;
  p.H = S;
  p.W = S;
  p.nwx = 1;
  p.upi = 1;
  p.scale = sm_scale;
  return dispatch_attn<true>(p, hd, B, stream);
}

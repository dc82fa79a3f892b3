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

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <string>
#include <type_traits>
#include <vector>

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
  int nqb, units;           // streaming path with a 1-D XCD-ordered grid: query blocks, units
  int dbg;                  // tuning build only: timing experiments (0 in the product)
  float out_scale, out_inv; // > 0: out holds int8 codes q8(fp16(o), out_scale) (W4A8 proj QAct)
};

// Store 4 output channels at element offset off of the [B, H, W, C] output: fp16, or (W4A8) the
// int8 codes of the proj input QAct applied to the f32 attention output itself (round 4: no fp16
// rounding in between -- the W4A8 oracle quantises its f32 attention; the fp16 round trip moved
// ~127 * 2^-11 code units at the top of the range, the dominant share of the stage's one-code
// flips).
__device__ __forceinline__ void attn_store4(const AttnParams& p, int64_t off, float4_t o) {
  if (p.out_scale > 0.f) {
    const float lim = 130.0f * p.out_scale;
    const float2_t c01 = q8_exact2(float2_t{o[0], o[1]}, p.out_scale, p.out_inv, lim);
    const float2_t c23 = q8_exact2(float2_t{o[2], o[3]}, p.out_scale, p.out_inv, lim);
    *(uint32_t*)((int8_t*)p.out + off) = q8_pack4(c01.x, c01.y, c23.x, c23.y);
  } else {
    *(half4_t*)(p.out + off) = half4_t{(_Float16)o[0], (_Float16)o[1], (_Float16)o[2], (_Float16)o[3]};
  }
}

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

template <int OFF>   // same, with the instruction's 16-bit immediate offset (no VGPR per address)
__device__ __forceinline__ half4_t ds_read_tr16_off(uint32_t addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset");
  half4_t r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
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
  // XCD-aware order for the streaming (global) path: the grid is 1-D and the query blocks of one
  // (image, head) all land on one XCD (workgroups are dealt round-robin over the 8 XCDs), so that
  // XCD's L2 serves their shared K/V stream instead of every XCD fetching every head's keys
  int qblk = blockIdx.x, head = blockIdx.y, unit = blockIdx.z;
  // p.nqb > 0 only on the 1-D launch (launch_attn sets it there); a 3-D launch whose y / z
  // extents happen to be 1 (heads * units == 1) keeps blockIdx as is
  if (!RESIDENT && p.nqb > 0) {
    const int nqb = p.nqb, pairs = p.heads * p.units;
    const int xcd = blockIdx.x & 7, k = blockIdx.x >> 3;
    const int pair = xcd * (pairs >> 3) + k / nqb;
    qblk = k % nqb;
    head = pair % p.heads;
    unit = pair / p.heads;
  }
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
    const int qi = (qblk * NW + wave) * QT + t;
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

  // SP >= 32: the softmax denominator is accumulated by the P.V MFMAs themselves (one more
  // 16x16x32 against an all-ones A operand per 32 keys, rescaled with O) instead of one VALU add
  // per score plus the cross-lane reduction -- the softmax VALU is what bounds this kernel.
  constexpr bool MSUM = SP >= 32;
  float m[QT], l[QT];
  float4_t o[QT][DT], lacc[QT];
  const half8_t ones = {1, 1, 1, 1, 1, 1, 1, 1};
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    m[t] = -INFINITY;
    l[t] = 0.f;
    lacc[t] = float4_t{0.f, 0.f, 0.f, 0.f};
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

  // ---- per key row: scores (QK), online softmax, O += P.V -- as lambdas so the streaming loop
  // can software-pipeline them (see below)
  using PB = half8_t[QT][(SP + 31) / 32];
  auto qk = [&](const char* kb, float4_t (&sc)[QT][KT]) {
      // ---- scores S^T = K . Q^T (+ TW as the C input)
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        const char* krow = kb + (kt * 16 + ql) * (D * 2);
        half8_t kf[KS];
        // unconditional: lanes past D in the last k-step read the next key's bytes (finite K/V
        // data of the LDS image) against zero Q dims -- no v_mov zero-fill per fragment
#pragma unroll
        for (int s = 0; s < KS; ++s) kf[s] = *(const half8_t*)(krow + (32 * s + 8 * g) * 2);
#pragma unroll
        for (int t = 0; t < QT; ++t) {
          float4_t a = tw[t][kt];
#pragma unroll
          for (int s = 0; s < KS; ++s) a = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[s], qf[t][s], a, 0, 0, 0);
          sc[t][kt] = a;
        }
      }

  };
  auto soft = [&](int kh, float4_t (&sc)[QT][KT], PB& pb, half4_t (&pb16)[QT]) {
    // ---- online softmax (exp2 domain); TH[q, kh] is constant along the row
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
      float mx;
      if constexpr (KT == 1) {
        mx = max3f(sc[t][0][0], sc[t][0][1], fmaxf(sc[t][0][2], sc[t][0][3]));
      } else {   // two max3 chains (no canonicalising v_max of a lone fmaxf)
        mx = max3f(sc[t][0][0], sc[t][0][1], sc[t][0][2]);
        float my = max3f(sc[t][1][0], sc[t][1][1], sc[t][1][2]);
        mx = max3f(mx, sc[t][0][3], sc[t][1][3]);
#pragma unroll
        for (int kt = 2; kt < KT; kt += 2) {
          mx = max3f(mx, sc[t][kt][0], sc[t][kt][1]);
          my = max3f(my, sc[t][kt + 1][0], sc[t][kt + 1][1]);
          mx = max3f(mx, sc[t][kt][2], sc[t][kt][3]);
          my = max3f(my, sc[t][kt + 1][2], sc[t][kt + 1][3]);
        }
        mx = fmaxf(mx, my);
      }
      mx = max_rows4(mx);
      const float th = th_w[(t * TH_ROWS + kh) * 16 + ql];
      // lazy rescale: the exp2 offset m only moves when the row max exceeds it by > 8 (P <= 2^8,
      // far inside fp16; O and l carry the same offset, so O / l is unchanged) -- most key rows
      // then skip the O rescale, whose packed multiplies beside the MFMAs bound this loop
      const float mrow = mx + th;
      const bool up = mrow > m[t] + 8.0f;
      const float mnew = up ? mrow : m[t];
      alpha[t] = up ? __builtin_amdgcn_exp2f(m[t] - mnew) : 1.0f;
      any_rescale |= up;
      m[t] = mnew;
      const float corr = mnew - th;
      float rs = 0.f;
#pragma unroll
      for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __builtin_amdgcn_exp2f(sc[t][kt][r] - corr);
          sc[t][kt][r] = e;
          if (!MSUM) rs += e;
        }
      if (!MSUM) l[t] = l[t] * alpha[t] + rs;
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
#pragma unroll
      for (int t = 0; t < QT; ++t)
        if (MSUM) lacc[t] = lacc[t] * alpha[t];
    }

  };
  auto pv = [&](const char* vb, PB& pb, half4_t (&pb16)[QT]) {
    // ---- O^T += V^T . P^T  (V^T fragments by hardware-transposed LDS reads of row-major V)
    // one base address per key row, the (d, s) offsets as the instruction's immediate
    const uint32_t vbase = lds_addr(vb + ((4 * g + trow) * D + tcol) * 2);
    static_for<DT>([&](auto dc_) {
      constexpr int d = decltype(dc_)::value;
      if constexpr (SP == 16) {
        half4_t va = ds_read_tr16_off<(d * 16) * 2>(vbase);
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(va));
#pragma unroll
        for (int t = 0; t < QT; ++t) o[t][d] = __builtin_amdgcn_mfma_f32_16x16x16f16(va, pb16[t], o[t][d], 0, 0, 0);
      } else {
        constexpr int NS = SP / 32;
        half4_t lo[NS], hi[NS];
        static_for<NS>([&](auto sc_) {
          constexpr int s_ = decltype(sc_)::value;
          lo[s_] = ds_read_tr16_off<((32 * s_) * D + d * 16) * 2>(vbase);
          hi[s_] = ds_read_tr16_off<((32 * s_ + 16) * D + d * 16) * 2>(vbase);
        });
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
    });
    if constexpr (MSUM) {
      constexpr int NS = SP / 32;
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int t = 0; t < QT; ++t) lacc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ones, pb[t][s], lacc[t], 0, 0, 0);
    }
  };

  if (RESIDENT) {
    for (int kh = 0; kh < S; ++kh) {
      const char* kb = smem + kh * S * (D * 2);
      float4_t sc[QT][KT];
      PB pb;
      half4_t pb16[QT];
      qk(kb, sc);
      soft(kh, sc, pb, pb16);
      pv(kb + (UNIT_CHUNKS / 2) * 16, pb, pb16);
    }
  } else {
    // Streaming (global) attention, software-pipelined by one key row: the Q.K^T MFMAs of row
    // kh+1 are issued ahead of the softmax of row kh (independent registers), so the MFMA tail
    // drains under the first softmax VALU work (with the MFMA row sums: 507 -> 474 us at ViT-H
    // B=4; forcing a finer MFMA/VALU interleave with sched_group_barrier spills, and the
    // softmax's max -> reduce -> exp chain leaves little to interleave).  Ring: row r in slot
    // r % 3; at the top of iteration kh row kh+1 is retired (nothing newer in flight) and, after
    // the barrier that also ends every read of row kh-1, row kh+2 is staged into row kh-1's slot.
    float4_t scA[QT][KT], scB[QT][KT];
    PB pb;
    half4_t pb16[QT];
    if (S > 1) wait_vmcnt<NI>(); else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();   // row 0 landed for every wave
    qk(smem, scA);
    auto step = [&](int kh, float4_t (&cur)[QT][KT], float4_t (&nxt)[QT][KT]) {
      if (kh + 1 < S) {
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();   // row kh+1 landed for every wave; row kh-1 fully consumed
        if (kh + 2 < S) issue(kh + 2, (kh + 2) % 3);
        qk(smem + ((kh + 1) % 3) * BUFB, nxt);
      }
      soft(kh, cur, pb, pb16);
      pv(smem + (kh % 3) * BUFB + ROWB, pb, pb16);
    };
    for (int kh = 0; kh < S; kh += 2) {   // S is even on this path (32 or 64)
      step(kh, scA, scB);
      step(kh + 1, scB, scA);
    }
  }

  // ---------------------------------------------------------------- normalise + store
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    float lt = l[t];
    if (MSUM) {
      lt = lacc[t][0];
    } else {
      lt += __shfl_xor(lt, 16, 64);
      lt += __shfl_xor(lt, 32, 64);
    }
    const int x = qcol0[t] + ql;
    if (tok_kind(qrow[t], x) != 0) continue;
    const float inv = 1.0f / lt;
    const int64_t dst = (((int64_t)b * p.H + (Y0 + qrow[t])) * p.W + (X0 + x)) * C + head * D;
#pragma unroll
    for (int d = 0; d < DT; ++d) attn_store4(p, dst + d * 16 + 4 * g, o[t][d] * inv);
  }
}

// ------------------------------------------------------------------ windowed attention (14 x 14)
// The 14x14-window blocks (28 of 32 in ViT-H).  One (window, head) item per 4-wave workgroup, TWO
// workgroups per CU (LDS < 80 KiB, <= 256 VGPRs): the partner workgroup runs out of phase, so
// one's HBM wait, softmax VALU and MFMA runs overlap the other's (no barrier couples them), and the
// hardware deals the 800 items of a 2-image ViT-H launch dynamically over the 512 slots.
//  * LDS image of an item: per key row kh (16 key slots; slots 14, 15 duplicate slot 13 and are
//    masked) NPC 1-KiB pieces, each written by ONE global_load_lds_dwordx4 whose lanes pick their
//    own sources:  K piece s: position l = (g, ql) holds key ql, dims 32 s + 8 g  -- read back by
//    lane l itself (ds_read_b128 at l * 16: the A operand of k-step s, conflict-free);  V piece:
//    position (g8, slot ^ 8 (g8 & 1)) holds key slot, dims 32 dblk + 8 g8 -- the XOR spreads the
//    ds_read_b64_tr_b16 reads of V^T over all 64 banks.  (D = 80: K dims 64..79 and V dims 64..79
//    share one piece; lanes of k-step 2 past dim 79 read V bytes against zero Q dims.)
//    Sources are one 64-bit add per piece (row stride); window pad tokens (past the image) read
//    the qkv bias, as the reference's zero-padded tokens do after the qkv Linear.
//  * query rows in passes of two 16-slot tiles per wave (rows 2w, 2w+1 then 8+2w, 9+2w); per tile
//    TW[q, kw] = q . Rw[qh - kw + 13] and TH[q, kh] = q . Rh[qh - kh + 13] (both indexed by the
//    query ROW qh: reference quirk 1) come out of 2 x KS MFMAs in the score layout; TW is the C
//    input of every key row's Q.K^T, TH[q, kh] is added to it per row (lane-local after one LDS
//    exchange; TH is rounded to fp16 as the reference's rel_h is);
//  * S^T = K.Q^T per key row (16 x 16 tile, each lane owns one query), one exact softmax over the
//    window's keys in the exp2 domain, O^T += V^T.P^T two key rows per MFMA with P^T in the score
//    registers' own k order, the row sum as one more MFMA against ones.
// pieces of the window kernel
// UNSC (round 4): Q enters the MFMAs unscaled (exact fp16 qkv values) and the scores stay in
// unscaled units S_u = q.k + (q.Rw + fp16(q.Rh)) / scale, the sm scale and log2e applied inside the
// softmax's exp2 argument (one fma per score, as the subtraction it replaces): no fp16 rounding of
// q * scale * log2e (a 2^-12 relative error on every score), and TH rounded to fp16 where the
// reference rounds rel_h (q . Rh, unscaled)
// PHL (round 4, the W4A8 int8-code store): P enters P.V as fp16 hi + lo (P - hi, |P - hi - lo| ~
// 2^-22 |P|, attention_q8.hip's split) -- two MFMAs per P.V step and for the row sums -- so the
// output carries fp32-level error instead of fp16 P's 2^-12, before the proj QAct's quantiser
template <int D, bool UNSC = false, bool PHL = false>
struct Win {
  static constexpr int S = 14, QT = 2;
  static constexpr int KS = D == 80 ? 3 : 2;            // k32 steps of Q.K^T
  static constexpr int DT = D / 16;                     // output d tiles
  static constexpr int NPC = D == 80 ? 5 : 4;           // 1-KiB pieces per key row
  static constexpr int ROWB = NPC * 1024;
  static constexpr int KVB = S * ROWB;                  // one item's K/V image
  static constexpr int V0 = (NPC - 2) * 1024;           // V dims 0..31 piece (dims 32..63 follow)
  static constexpr int TAB = (2 * S - 1) * D;           // elements per rel-pos table
  static constexpr int TABB = ((2 * TAB * 2 + 1023) / 1024) * 1024;   // both tables, whole pieces
  static_assert(D == 64 || D == 80, "head dim");

  struct Geo { const _Float16* tok0; int b, Y0, X0, head, nrow, ncol; };

  __device__ static __forceinline__ Geo geo(const AttnParams& p, int item) {
    Geo o;
    const int unit = item / p.heads;
    o.head = item - unit * p.heads;
    o.b = unit / p.upi;
    const int wi = unit - o.b * p.upi;
    const int wy = wi / p.nwx;
    o.Y0 = wy * S;
    o.X0 = (wi - wy * p.nwx) * S;
    o.nrow = p.H - o.Y0 < S ? p.H - o.Y0 : S;           // rows / columns inside the image
    o.ncol = p.W - o.X0 < S ? p.W - o.X0 : S;
    o.tok0 = p.qkv + (((int64_t)o.b * p.H + o.Y0) * p.W + o.X0) * p.tok_stride;
    return o;
  }

  // both rel-pos tables -> LDS, pieces i0, i0 + istep, ... (one wave's share)
  __device__ static __forceinline__ void issue_tables(const AttnParams& p, char* tab, int lane, int i0, int istep) {
    for (int i = i0; i < TABB / 1024; i += istep) {
      const int c = i * 64 + lane;                       // 16-byte chunk of [relh | relw]
      const int tc = c < TAB / 8 ? c : c - TAB / 8;
      const _Float16* src = c < 2 * (TAB / 8) ? (c < TAB / 8 ? p.relh : p.relw) + 8 * tc : g_zero16;
      __builtin_amdgcn_global_load_lds((const SAMQ_GLOBAL void*)src, (SAMQ_LDS void*)(tab + i * 1024), 16, 0, 0);
    }
  }

  // key rows kh0, kh0 + khstep, ... of one item -> its LDS image (one global_load_lds per piece)
  __device__ static __forceinline__ void issue_rows(const AttnParams& p, const Geo& G, char* kv, int lane, int kh0,
                                                    int khstep) {
    const int ql = lane & 15, g = lane >> 4;
    const int64_t ts = p.tok_stride, rowstride = (int64_t)p.W * ts;
    const _Float16* src[NPC];
    int64_t step[NPC];
    const _Float16* pad[NPC];
#pragma unroll
    for (int j = 0; j < NPC; ++j) {
      int col, ch;
      if (j < KS - (D == 80 ? 1 : 0) || (D == 80 && j == 2 && lane < 32)) {   // K: (g, ql)
        col = ql;
        ch = p.C + G.head * D + 32 * j + 8 * g;
      } else {                                                                // V: (g8, slot ^ 8 (g8 & 1))
        const bool comb = D == 80 && j == 2;             // upper half of the shared K/V piece
        const int g8 = comb ? g - 2 : g;
        const int dblk = comb ? 2 : j - (NPC - 2);
        col = ql ^ (8 * (g8 & 1));
        ch = 2 * p.C + G.head * D + 32 * dblk + 8 * g8;
      }
      col = col < S - 1 ? col : S - 1;
      pad[j] = p.qkv_bias ? p.qkv_bias + ch : g_zero16;
      const bool real = col < G.ncol;
      src[j] = real ? G.tok0 + (int64_t)col * ts + ch + kh0 * rowstride : pad[j];
      step[j] = real ? khstep * rowstride : 0;
    }
    for (int kh = kh0; kh < S; kh += khstep) {
      const bool rowreal = kh < G.nrow;
#pragma unroll
      for (int j = 0; j < NPC; ++j) {
        __builtin_amdgcn_global_load_lds((const SAMQ_GLOBAL void*)(rowreal ? src[j] : pad[j]),
                                         (SAMQ_LDS void*)(kv + kh * ROWB + j * 1024), 16, 0, 0);
        src[j] += step[j];
      }
    }
  }

  // raw Q of one tile (query row r, slots ql; dims 32 s + 8 g; zero past D and for slots 14, 15)
  __device__ static __forceinline__ void load_q(const AttnParams& p, const Geo& G, int r, int lane, half8_t (&q)[KS]) {
    const int ql = lane & 15, g = lane >> 4;
    const bool inwin = ql < S && r < S;
    const bool real = inwin && r < G.nrow && ql < G.ncol;
    const _Float16* base = real ? G.tok0 + ((int64_t)r * p.W + ql) * p.tok_stride + G.head * D
                                : ((inwin && p.qkv_bias) ? p.qkv_bias + G.head * D : nullptr);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const _Float16* a = (base && 32 * s + 8 * g < D) ? base + 32 * s + 8 * g : g_zero16;
      asm volatile("" : "+v"(a));
      q[s] = *(const SAMQ_GLOBAL half8_t*)a;
    }
  }

  // query rows row0, row0 + 1 of one item: rel-pos terms, S^T = K.Q^T + TW + TH, exact softmax,
  // O^T = V^T.P^T, normalise, store.  after_qk() runs once the scores are in registers (the
  // caller's prefetch of the next tiles' Q goes there: qraw is dead by then).
  template <typename F>
  __device__ static __forceinline__ void tiles(const AttnParams& p, const Geo& G, const char* kv, const char* tab,
                                               half8_t (&qraw)[QT][KS], int row0, int lane, F&& after_qk) {
    const int ql = lane & 15, g = lane >> 4;
    const float qscale = p.scale * LOG2E;
    const float inv_scale = 1.0f / p.scale;              // (Qs . R) / scale = log2e * (q . R)
    const _Float16* tabh = (const _Float16*)tab;
    // ---- rel-pos table fragments (A operands: row i = key column / key row) from the LDS copy
    half8_t relh[QT][KS], relw[QT][KS];
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      int idx = row0 + t - ql + S - 1;
      idx = idx < 0 ? 0 : idx;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        int dd = 32 * s + 8 * g;
        dd = dd < D ? dd : dd - 16;                      // k-step-2 lanes past D: any in-bounds row bytes
        relh[t][s] = *(const half8_t*)(tabh + idx * D + dd);
        relw[t][s] = *(const half8_t*)(tabh + TAB + idx * D + dd);
      }
    }
    // ---- Q scale (fp16(q * scale * log2e), the reference's rounding; UNSC: unscaled) and rel-pos terms
    half8_t qf[QT][KS];
    float4_t tw[QT];
    half8_t th[QT][2];
#pragma unroll
    for (int t = 0; t < QT; ++t) {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        half8_t v = qraw[t][s];
        if constexpr (!UNSC) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (_Float16)__builtin_fmaf((float)v[j], qscale, 0.0f);
        }
        qf[t][s] = v;
      }
      float4_t a = {0.f, 0.f, 0.f, 0.f}, c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        a = __builtin_amdgcn_mfma_f32_16x16x32_f16(relw[t][s], qf[t][s], a, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(relh[t][s], qf[t][s], c, 0, 0, 0);
      }
      a = a * inv_scale;                 // UNSC: (q . Rw) / scale; else log2e q . Rw
      if constexpr (!UNSC) c = c * inv_scale;   // UNSC: q . Rh, rounded below like rel_h
      if (g == 3) { a[2] = -INFINITY; a[3] = -INFINITY; }   // key slots 14, 15
      tw[t] = a;
      // lane (g, ql) holds TH[kh = 4g..4g+3][query ql]; gather kh 0..15 of its query from the
      // lanes (g', ql) (fp16, as the reference rounds rel_h)
      union { half4_t h; uint32_t u[2]; } mine;
      mine.h = half4_t{(_Float16)c[0], (_Float16)c[1], (_Float16)c[2], (_Float16)c[3]};
      union { half8_t h[2]; uint32_t u[8]; } all;
#pragma unroll
      for (int gg = 0; gg < 4; ++gg)
#pragma unroll
        for (int w = 0; w < 2; ++w) all.u[2 * gg + w] = (uint32_t)__shfl((int)mine.u[w], ql + 16 * gg, 64);
      th[t][0] = all.h[0];
      th[t][1] = all.h[1];
    }

    // ---- scores S^T = K.Q^T + TW + TH for all key rows (next row's K fragments in flight)
    float4_t sc[QT][S];
    half8_t kf[2][KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) kf[0][s] = *(const half8_t*)(kv + s * 1024 + lane * 16);
#pragma unroll
    for (int kh = 0; kh < S; ++kh) {
      if (kh + 1 < S) {
#pragma unroll
        for (int s = 0; s < KS; ++s) kf[(kh + 1) & 1][s] = *(const half8_t*)(kv + (kh + 1) * ROWB + s * 1024 + lane * 16);
      }
#pragma unroll
      for (int t = 0; t < QT; ++t) {
        const float h = UNSC ? (float)th[t][kh >> 3][kh & 7] * inv_scale : (float)th[t][kh >> 3][kh & 7];
        float4_t a = tw[t] + h;
#pragma unroll
        for (int s = 0; s < KS; ++s) a = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[kh & 1][s], qf[t][s], a, 0, 0, 0);
        sc[t][kh] = a;
      }
      __builtin_amdgcn_sched_barrier(0);   // no hoisting of later rows' C inputs (register pressure)
    }
    after_qk();

    // ---- exact softmax over the window (exp2 domain)
    half8_t pb[QT][S / 2];
    half8_t pl[PHL ? QT : 1][PHL ? S / 2 : 1];   // PHL: the lo parts
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      // two independent max3 chains (no canonicalising v_max of a lone fmaxf)
      float mx = max3f(sc[t][0][0], sc[t][0][1], sc[t][0][2]);
      float my = max3f(sc[t][1][0], sc[t][1][1], sc[t][1][2]);
      mx = max3f(mx, sc[t][0][3], sc[t][1][3]);
#pragma unroll
      for (int kh = 2; kh < S; kh += 2) {
        mx = max3f(mx, sc[t][kh][0], sc[t][kh][1]);
        my = max3f(my, sc[t][kh + 1][0], sc[t][kh + 1][1]);
        mx = max3f(mx, sc[t][kh][2], sc[t][kh][3]);
        my = max3f(my, sc[t][kh + 1][2], sc[t][kh + 1][3]);
      }
      mx = fmaxf(mx, my);
      mx = max_rows4(mx);
      if constexpr (UNSC && PHL) {
        const float nmx = -mx * qscale;
#pragma unroll
        for (int pr = 0; pr < S / 2; ++pr)
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[t][2 * pr + (r >> 2)][r & 3], qscale, nmx));
            const _Float16 hi = (_Float16)e;
            pb[t][pr][r] = hi;
            pl[PHL ? t : 0][PHL ? pr : 0][r] = (_Float16)(e - (float)hi);
          }
      } else if constexpr (UNSC) {   // P = exp2((S_u - max) * scale * log2e) as one fma per score
        const float nmx = -mx * qscale;
#pragma unroll
        for (int pr = 0; pr < S / 2; ++pr)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            pb[t][pr][r] = (_Float16)__builtin_amdgcn_exp2f(__builtin_fmaf(sc[t][2 * pr][r], qscale, nmx));
            pb[t][pr][4 + r] = (_Float16)__builtin_amdgcn_exp2f(__builtin_fmaf(sc[t][2 * pr + 1][r], qscale, nmx));
          }
      } else {
#pragma unroll
        for (int pr = 0; pr < S / 2; ++pr)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            pb[t][pr][r] = (_Float16)__builtin_amdgcn_exp2f(sc[t][2 * pr][r] - mx);
            pb[t][pr][4 + r] = (_Float16)__builtin_amdgcn_exp2f(sc[t][2 * pr + 1][r] - mx);
          }
      }
    }

    // ---- O^T = V^T . P^T (two key rows per MFMA), l = ones . P^T
    // V^T fragment address of this lane (ds_read_b64_tr_b16: lane 4q+p of a group reads key slot
    // 4g + q, dims 4p..4p+3 of the tile's 16; the V pieces' XOR layout)
    const int tq = ql >> 2, tp = ql & 3;
    const int vslot = 4 * g + tq;
    const uint32_t vlane = lds_addr(kv) + (((tp >> 1) * 16 + (vslot ^ (8 * (tp >> 1)))) * 16 + (tp & 1) * 8);
    const half8_t ones = {1, 1, 1, 1, 1, 1, 1, 1};
    float4_t o[QT][DT], lsum[QT];   // first written by the pr = 0 MFMAs (zero C operand)
    const float4_t zero4 = {0.f, 0.f, 0.f, 0.f};
    half4_t vlo[2][DT], vhi[2][DT];
    // V^T fragments of key rows (2 pr, 2 pr + 1) for all d tiles (immediate offsets from two bases)
    auto vread = [&](auto prc, half4_t (&lo)[DT], half4_t (&hi)[DT]) {
      constexpr int PR = decltype(prc)::value;
      constexpr int HB = PR >= 4 ? 32768 : 0;
      const uint32_t base = vlane + HB;
      static_for<DT>([&](auto dc) {
        constexpr int d = decltype(dc)::value;
        constexpr int VO = d < 4 ? V0 + (d >> 1) * 1024 + (d & 1) * 512 : 2 * 1024 + 512;
        lo[d] = ds_read_tr16_off<(2 * PR) * ROWB + VO - HB>(base);
        hi[d] = ds_read_tr16_off<(2 * PR + 1) * ROWB + VO - HB>(base);
      });
    };
    vread(std::integral_constant<int, 0>{}, vlo[0], vhi[0]);
    static_for<S / 2>([&](auto prc) {
      constexpr int pr = decltype(prc)::value;
      constexpr int cb = pr & 1;
      if constexpr (pr + 1 < S / 2) vread(std::integral_constant<int, pr + 1>{}, vlo[cb ^ 1], vhi[cb ^ 1]);
      // this pair's fragments landed (the next pair's 2*DT reads may still be in flight)
      if constexpr (DT == 5) {
        if (pr + 1 < S / 2)
          asm volatile("s_waitcnt lgkmcnt(10)" : "+v"(vlo[cb][0]), "+v"(vlo[cb][1]), "+v"(vlo[cb][2]), "+v"(vlo[cb][3]),
                       "+v"(vlo[cb][4]), "+v"(vhi[cb][0]), "+v"(vhi[cb][1]), "+v"(vhi[cb][2]), "+v"(vhi[cb][3]), "+v"(vhi[cb][4]));
        else
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vlo[cb][0]), "+v"(vlo[cb][1]), "+v"(vlo[cb][2]), "+v"(vlo[cb][3]),
                       "+v"(vlo[cb][4]), "+v"(vhi[cb][0]), "+v"(vhi[cb][1]), "+v"(vhi[cb][2]), "+v"(vhi[cb][3]), "+v"(vhi[cb][4]));
      } else {
        if (pr + 1 < S / 2)
          asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(vlo[cb][0]), "+v"(vlo[cb][1]), "+v"(vlo[cb][2]), "+v"(vlo[cb][3]),
                       "+v"(vhi[cb][0]), "+v"(vhi[cb][1]), "+v"(vhi[cb][2]), "+v"(vhi[cb][3]));
        else
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vlo[cb][0]), "+v"(vlo[cb][1]), "+v"(vlo[cb][2]), "+v"(vlo[cb][3]),
                       "+v"(vhi[cb][0]), "+v"(vhi[cb][1]), "+v"(vhi[cb][2]), "+v"(vhi[cb][3]));
      }
#pragma unroll
      for (int d = 0; d < DT; ++d) {
        const half8_t va = {vlo[cb][d][0], vlo[cb][d][1], vlo[cb][d][2], vlo[cb][d][3],
                            vhi[cb][d][0], vhi[cb][d][1], vhi[cb][d][2], vhi[cb][d][3]};
#pragma unroll
        for (int t = 0; t < QT; ++t) {
          o[t][d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va, pb[t][pr], pr ? o[t][d] : zero4, 0, 0, 0);
          if constexpr (PHL) o[t][d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va, pl[t][pr], o[t][d], 0, 0, 0);
        }
      }
#pragma unroll
      for (int t = 0; t < QT; ++t) {
        lsum[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ones, pb[t][pr], pr ? lsum[t] : zero4, 0, 0, 0);
        if constexpr (PHL) lsum[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ones, pl[t][pr], lsum[t], 0, 0, 0);
      }
    });

    // ---- normalise + store (token-major [B, H, W, C])
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      const int r = row0 + t;
      if (r >= G.nrow || ql >= G.ncol) continue;
      const float inv = __builtin_amdgcn_rcpf(lsum[t][0]);
      const int64_t dst = (((int64_t)G.b * p.H + (G.Y0 + r)) * p.W + (G.X0 + ql)) * p.C + G.head * D;
#pragma unroll
      for (int d = 0; d < DT; ++d) attn_store4(p, dst + d * 16 + 4 * g, o[t][d] * inv);
    }
  }
};

// One item per 4-wave workgroup, two workgroups per CU (rows 2w, 2w+1 then 8+2w, 9+2w).  (A
// persistent form -- one 8-wave workgroup per CU, wave 7 streaming the next item's K/V into a second
// buffer while waves 0..6 compute -- measured 37.9 vs 37.0 us per 2-image ViT-H launch.)
template <int D, bool UNSC = false, bool PHL = false>
__global__ __launch_bounds__(256, 2) void win_attention_kernel(AttnParams p, int items) {
  using W = Win<D, UNSC, PHL>;
  static_assert(W::KVB + W::TABB <= 80 * 1024, "two workgroups per CU");
  __shared__ __attribute__((aligned(16))) char smem[W::KVB + W::TABB];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // consecutive items (the heads of one window: K/V cache lines shared across head slices) on one XCD
  const int item = xcd_remap(blockIdx.x, gridDim.x);
  if (item >= items) return;
  const typename W::Geo G = W::geo(p, item);
  char* tab = smem + W::KVB;
  W::issue_tables(p, tab, lane, wave, 4);
  W::issue_rows(p, G, smem, lane, wave, 4);
  half8_t qraw[W::QT][W::KS];
#pragma unroll
  for (int t = 0; t < W::QT; ++t) W::load_q(p, G, 2 * wave + t, lane, qraw[t]);
  wait_vmcnt<0>();
  __syncthreads();   // the item's K/V image and the tables are complete
  const int npass = 8 + 2 * wave < W::S ? 2 : 1;
  for (int pass = 0; pass < npass; ++pass) {
    const int row0 = 8 * pass + 2 * wave;
    W::tiles(p, G, smem, tab, qraw, row0, lane, [&] {
      if (pass + 1 < npass) {
#pragma unroll
        for (int t = 0; t < W::QT; ++t) W::load_q(p, G, row0 + 8 + t, lane, qraw[t]);
      }
    });
  }
}

// ------------------------------------------------------------------ global attention, 32x32 MFMA
// ViT-H global blocks (64 x 64 grid, head dim 80) on v_mfma_f32_32x32x16_f16: the 32x32 form
// issues half the MFMA instructions per FLOP of 16x16x32 (each holds the SIMD's vector issue for
// 8 of its 32 cycles, MI355X_MICROARCH.md constants) and D = 80 is 5 k16-steps, no padding.
//  * a wave owns one query tile of 32 queries of ONE grid row qh (so the width table row
//    qh - kw + 63 is one A operand for the whole tile: reference quirk 1 keeps both tables on qh);
//    8 waves = 4 grid rows per workgroup, 16 workgroups per (image, head), one workgroup per CU;
//  * key row kh (64 keys) = two 32-key tiles: S^T = K.Q^T + TW (5 MFMAs each, TW[kt] = log2e q.Rw
//    as the C input, computed once per tile by the same MFMA form); TH[q, kh] = log2e q.Rh, fp16-
//    rounded like the reference's rel_h, kept per wave in LDS and folded into the running max;
//  * a lane holds 32 scores of ONE query (its partner lane ^ 32 the other 32): the row max is
//    in-register + one cross-lane step; lazy exp2 offset (moves only past +8); P stays in the
//    score registers' order, which IS the B operand of O^T += V^T . P^T (k-slot 8h + j <-> key
//    16u + 4h + j (j < 4) / 16u + 8 + 4h + j - 4);
//  * V^T fragments by ds_read_b64_tr_b16 from 4-key x 32-dim chunks (256 contiguous bytes per
//    read group: conflict-free); d-block 2 covers dims 64..95, its rows 80..95 read as 1.0 (a
//    ones region per ring slot, ONESL below) so the same MFMAs produce the softmax row sums (no
//    extra MFMA, no VALU sum);
//  * K pieces lane-linear (lane l of piece (kt, s) = key 32 kt + l % 32, dims 16 s + 8 (l / 32):
//    the A fragment read is ds_read_b128 at l * 16); key rows stream through a 5-slot LDS ring
//    (20 KiB of K / V per row, LDS-DMA, 20 pieces over 8 waves), two barriers per key row (the
//    two-group ping-pong below), the next row's Q.K^T MFMAs issued ahead of the current row's
//    softmax.
__device__ __forceinline__ float16_t mfma32(half8_t a, half8_t b, float16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

#ifdef SAMQ_TUNING
__device__ unsigned long long g_attn_stamps[8];   // timing experiments (tuning build)
__device__ unsigned long long g_attn_wgt[4096 * 6];   // DBG & 8: per-workgroup timeline
#endif
template <int DBG>
__device__ __forceinline__ void wg_mark(unsigned long long (&t)[6], int k) {
  if constexpr ((DBG & 8) != 0) {
    t[k] = __builtin_amdgcn_s_memrealtime();
    if (k == 1 || k == 2) t[k + 3] = __builtin_amdgcn_s_memtime();
  }
}

// DBG (tuning build only): & 1 per-wave s_memtime stamps of the four loop segments; & 2 no exp2,
// & 4 no MFMAs (timing-only variants, wrong results); & 8 per-workgroup timeline (realtime at
// entry / loop start / loop end / exit + shader clock over the loop); & 16 the round-3 softmax (offset subtracted
// in the softmax segment instead of folded into the Q.K^T C input, COFF below)
template <int DBG>
__global__ __launch_bounds__(512, 1) void glob80_attention_kernel(AttnParams p) {
  constexpr int D = 80, S = 64, KS = 5;
  constexpr int NSLOT = 5;                        // key-row ring slots
  // ONESL (round 4; DBG & 512 = the round-3 layout): V of a key row as dims 0..63 (16 key quads x
  // 512 B) | dims 64..79 (16 quads x 128 B) | 128 B pad | 2 KiB of fp16 ones written once per slot,
  // so the lanes of d-block 2 that hold rows 80..95 (the softmax row sums) read 1.0 from LDS at
  // their own base (+2176: the other 32 banks) instead of masking 4 dwords per P.V step.  Round 3:
  // 16 key quads x (256 + 256 + 128 B) interleaved, rows 80..95 forced to 1.0 in registers.
  constexpr bool ONESL = (DBG & 512) == 0;
  constexpr int VB = 10 * 1024;                   // V dims 0..63 (ONESL) / all of V
  constexpr int V2B = 18 * 1024;                  // ONESL: V dims 64..79
  constexpr int ONESB = V2B + 2048 + 128;         // ONESL: the ones (+2176 from V2B)
  constexpr int ROWB = ONESL ? ONESB + 2048 : 20 * 1024;   // one key row's ring slot
  constexpr int THB = 64 * 32 * 2;                // per wave: fp16 TH[kh][q]
  __shared__ __attribute__((aligned(16))) char smem[NSLOT * ROWB + 8 * THB];
  static_assert(NSLOT * ROWB + 8 * THB <= 160 * 1024, "LDS");
  constexpr bool DBG_NOEXP = (DBG & 2) != 0, DBG_NOMFMA = (DBG & 4) != 0;
  // COFF (round 4): the next row's TH and softmax offset enter its Q.K^T as part of the C input
  // (C = TW + (TH[kh] - offset), a per-lane scalar added in the MFMA segment), so the softmax
  // segment -- the longer of the two -- runs exp2 straight on the scores (32 fewer v_sub per row):
  // 204.1 vs 209.6 us per 2-image launch, outputs within 3e-5 (profiles/r4_i.attn.log)
  constexpr bool COFF = (DBG & 16) == 0;
  // round 4 loop variants (tuning A/B): & 32 the next row's K fragment reads issued at the start of
  // the VALU segment; & 64 the first P.V step's V^T fragments read at the end of the VALU segment;
  // & 128 without PFENCE
  constexpr bool KEARLY = (DBG & 32) != 0, VPRE = (DBG & 64) != 0, PFENCE = (DBG & 128) == 0;
  // & 256: CMFMA -- the per-row C offset (TH - offset) enters Q.K^T as one more MFMA k-step (ones x
  // [hi; lo] of the offset, |c - hi - lo| <= 2^-22 |c|) instead of 32 adds to the C input
  constexpr bool CMFMA = (DBG & 256) != 0 && COFF;
  // & 1024: G1DMA -- group 1 alone issues all 20 pieces of row kh+4, 5 per wave, in its VALU
  // segment of row kh (after its exp2s; the LDS-DMA issue is cheap among VALU, dear inside an MFMA
  // burst, MI355X_MICROARCH.md constants); group 0's MFMA segments carry no DMA
  constexpr bool G1DMA = (DBG & 1024) != 0;
  // & 2048: STATPRIO -- group 1 (the younger half) at s_setprio 1 for the whole loop, no
  // per-segment priority flips (MI355X_MICROARCH.md "Two waves per SIMD" item 4)
  constexpr bool STATPRIO = (DBG & 2048) != 0;
  // & 4096: QKDMA -- the row's LDS-DMA pieces issued between the Q.K^T MFMAs (no LDS reads in
  // flight there) instead of ahead of the P.V step's V^T reads
  constexpr bool QKDMA = (DBG & 4096) != 0;

  _Float16* th_lds = (_Float16*)(smem + NSLOT * ROWB);
  unsigned long long wgt[6] = {0, 0, 0, 0, 0, 0};
  wg_mark<DBG>(wgt, 0);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2;                       // waves w, w + 4 share a SIMD
  const int l32 = lane & 31, h = lane >> 5;
  // XCD-aware 1-D grid: the 16 query blocks of one (image, head) on one XCD (shared K/V in its L2)
  const int nqb = p.nqb, pairs = p.heads * p.units;
  const int xcd = blockIdx.x & 7, kk = blockIdx.x >> 3;
  const int pair = xcd * (pairs >> 3) + kk / nqb;
  const int qblk = kk % nqb;
  const int head = pair % p.heads;
  const int b = pair / p.heads;
  const int C = p.C;
  const int qh = 4 * qblk + (wave >> 1);           // this wave's query grid row
  const int qw0 = 32 * (wave & 1);
  const _Float16* img = p.qkv + (int64_t)b * S * S * p.tok_stride;

  // ---- K / V staging: 20 pieces per key row; wave w issues pieces w, w + 8 (, w + 16 for w < 4)
  // (G1DMA: group 1's wave 4 + u issues pieces u, u + 4, .., u + 16)
  constexpr int NI = G1DMA ? 5 : 3;
  const int npc = G1DMA ? (grp ? 5 : 0) : (wave < 4 ? 3 : 2);
  const _Float16* src0[NI];
  int dst[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int v = G1DMA ? (wave & 3) + 4 * i : wave + 8 * i;
    int key, dim;
    if (v < 10) {                                  // K piece (kt, s): lane-linear A fragments
      key = 32 * (v / 5) + l32;
      dim = C + 16 * (v % 5) + 8 * h;
    } else if (ONESL) {                            // V: dims 0..63 (pieces 10..17), 64..79 (18, 19)
      const int gl = 64 * (v - 10) + lane;
      if (v < 18) {                                // 16 key quads x (256 + 256 B)
        const int kq = gl >> 5, w = gl & 31;
        key = 4 * kq + ((w & 15) >> 2);
        dim = 2 * C + 32 * (w >> 4) + 8 * (w & 3);
      } else {                                     // 16 key quads x 128 B
        const int g2 = gl - 512, kq = g2 >> 3, w = g2 & 7;
        key = 4 * kq + (w >> 1);
        dim = 2 * C + 64 + 8 * (w & 1);
      }
      key = key < S ? key : S - 1;
    } else {                                       // V: 16 key-quads x (256 + 256 + 128 bytes)
      const int gl = 64 * (v - 10) + lane;
      const int kq = gl / 40, w = gl % 40;
      if (w < 16)      { key = 4 * kq + (w >> 2);        dim = 2 * C + 8 * (w & 3); }
      else if (w < 32) { key = 4 * kq + ((w - 16) >> 2); dim = 2 * C + 32 + 8 * (w & 3); }
      else             { key = 4 * kq + ((w - 32) >> 1); dim = 2 * C + 64 + 8 * (w & 1); }
      key = key < S ? key : S - 1;
    }
    src0[i] = img + (int64_t)key * p.tok_stride + head * D + dim;
    dst[i] = v * 1024;
  }
  const int64_t rowstride = (int64_t)S * p.tok_stride;
  auto issue_one = [&](int kh, int slot, int i) {
    if (i < npc)
      __builtin_amdgcn_global_load_lds((const SAMQ_GLOBAL void*)(src0[i] + kh * rowstride),
                                       (SAMQ_LDS void*)(smem + slot * ROWB + dst[i]), 16, 0, 0);
  };
  auto issue = [&](int kh, int slot) {
#pragma unroll
    for (int i = 0; i < NI; ++i) issue_one(kh, slot, i);
  };
#pragma unroll
  for (int r = 0; r < NSLOT - 1; ++r) issue(r, r);

  // ---- Q^T fragments (B operand): lane = query qw0 + l32, dims 16 s + 8 h (fp16(q * scale * log2e))
  const float qscale = p.scale * LOG2E;
  half8_t qf[KS];
  {
    const _Float16* qp = img + ((int64_t)qh * S + qw0 + l32) * p.tok_stride + head * D + 8 * h;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      half8_t v = *(const half8_t*)(qp + 16 * s);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (_Float16)__builtin_fmaf((float)v[j], qscale, 0.0f);
      qf[s] = v;
    }
  }
  // ---- rel-pos terms: TW[kt] (score layout, the C input) and TH -> LDS (fp16, per wave)
  const float inv_scale = 1.0f / p.scale;
  float16_t tw[2];
  _Float16* thw = th_lds + wave * (64 * 32);
#pragma unroll
  for (int which = 0; which < 2; ++which) {
    const _Float16* tab = which ? p.relw : p.relh;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const int r = qh - (32 * kt + l32) + S - 1;   // table row of this lane's A row (key column / key row)
      const _Float16* rp = tab + (int64_t)r * D + 8 * h;
      float16_t a = {};
#pragma unroll
      for (int s = 0; s < KS; ++s) a = mfma32(*(const half8_t*)(rp + 16 * s), qf[s], a);
      a = a * inv_scale;
      if (which) {
        tw[kt] = a;
      } else {
#pragma unroll
        for (int r2 = 0; r2 < 16; ++r2) {
          const int kh = 32 * kt + 8 * (r2 >> 2) + 4 * h + (r2 & 3);
          thw[kh * 32 + l32] = (_Float16)a[r2];
        }
      }
    }
  }

  // ---- V^T fragment addresses (ds_read_b64_tr_b16): lane 4q + p of its 16-lane group reads
  // key 4 kq + q, dims 16 g16 + 4p .. of the chunk; d-block 2 lanes g16 = 1 (dims 80..95) read
  // the slot's ones (ONESL; the round-3 layout read the g16 = 0 bytes and forced 1.0 in pv)
  const int i16 = lane & 15, g16 = (lane >> 4) & 1;
  const int tq = i16 >> 2, tp = i16 & 3;
  constexpr int QB = ONESL ? 512 : 640, QB2 = ONESL ? 128 : 640;   // bytes per key quad (dims 0..63 / 64..79)
  const uint32_t vb01 = lds_addr(smem + VB) + h * QB + tq * 64 + g16 * 32 + tp * 8;
  const uint32_t vb2 = ONESL ? lds_addr(smem + V2B) + h * QB2 + tq * 32 + tp * 8 + g16 * (ONESB - V2B)
                             : lds_addr(smem + VB) + h * 640 + 512 + tq * 32 + tp * 8;
  const uint32_t ones_or = g16 ? 0x3C003C00u : 0u, ones_and = g16 ? 0u : 0xFFFFFFFFu;
  if constexpr (ONESL) {   // the ones of every ring slot (read only after the barrier below)
    const u32x4 one4 = {0x3C003C00u, 0x3C003C00u, 0x3C003C00u, 0x3C003C00u};
    for (int i = tid; i < NSLOT * 128; i += 512)
      *(u32x4*)(smem + (i >> 7) * ROWB + ONESB + (i & 127) * 16) = one4;
  }

  float16_t o[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) o[d] = float16_t{};
  float m = -INFINITY;
  float16_t sc[2];
  half8_t pb[2][2];

  half8_t kf[2][KS];
  auto kread = [&](const char* kb) {   // K fragments of a key row (A operands, lane-linear pieces)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int s = 0; s < KS; ++s) kf[kt][s] = *(const half8_t*)(kb + (kt * 5 + s) * 1024 + lane * 16);
  };
  float coff = 0.f;   // COFF: TH of the next row minus the offset baked into its scores
  // CMFMA operands: A = ones in k-slots 0, 1 (lanes h = 0), B = [hi; lo] of coff in the same slots
  const half8_t ones01 = h ? half8_t{} : half8_t{1, 1, 0, 0, 0, 0, 0, 0};
  half8_t cq = {};
  auto set_cq = [&] {
    const _Float16 hi = (_Float16)coff;
    const _Float16 lo = (_Float16)(coff - (float)hi);
    cq = h ? half8_t{} : half8_t{hi, lo, 0, 0, 0, 0, 0, 0};
  };
  // dma(i): QKDMA's piece issue after the i-th Q.K^T MFMA (i = 0..9; pieces at i = 1, 4, 7)
  auto qk_d = [&](auto&& dma) {   // S^T = K . Q^T + TW (COFF: + coff) for the two 32-key tiles of a key row
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      float16_t a = tw[kt];
      if constexpr (CMFMA) a = mfma32(ones01, cq, a);
      else if constexpr (COFF) a = a + coff;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        if (DBG_NOMFMA) a[s] += (float)kf[kt][s][0] * (float)qf[s][0];
        else a = mfma32(kf[kt][s], qf[s], a);
        dma(KS * kt + s);
      }
      sc[kt] = a;
    }
  };
  auto qk = [&]() { qk_d([](int) {}); };
  // Online softmax (exp2 domain), lane = one query, 32 of its 64 keys.  P is computed with the
  // offset m of the PREVIOUS rows, so the exp2s do not wait for this row's max (whose reduction +
  // cross-lane step + compare is a serial chain): the max runs beside them and only decides
  //  * m moves by > 8 (lazy offset): applied after this row's P.V, before the next row's P
  //    (O *= exp2(m - m_new) there; P and O of this row share the old offset);
  //  * this row's P could exceed 2^15 (fp16 range): rare slow path, O rescaled and P recomputed
  //    with the new offset now (always taken for row 0, m = -inf).
  float th_cur = (float)thw[l32];   // TH of row 0
  float m_pend = -INFINITY;
  bool pend = false;
  // COFF: moff = the offset baked into the current row's scores (m after the pending move, 0 for
  // row 0 whose m is -inf); the scores are then s + TH - moff and P = exp2(score)
  float moff = 0.f;
  if constexpr (COFF) coff = th_cur;
  if constexpr (CMFMA) set_cq();
  auto softmax_coff = [&](int kh) {
    if (__any(pend)) {   // last row's deferred offset move (moff already includes it)
      const float alpha = pend ? __builtin_amdgcn_exp2f(m - m_pend) : 1.0f;
      m = pend ? m_pend : m;
#pragma unroll
      for (int d = 0; d < 3; ++d) o[d] = o[d] * alpha;
      pend = false;
    }
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) pb[kt][u][j] = (_Float16)__builtin_amdgcn_exp2f(sc[kt][8 * u + j]);
    // PFENCE: keep the fast-path exp2s ahead of the max chain (the compiler otherwise sinks them
    // into the not-unsafe branch, behind the serial max3 / permlane / compare chain)
    if constexpr (PFENCE) asm volatile("" : "+v"(pb[0][0]), "+v"(pb[0][1]), "+v"(pb[1][0]), "+v"(pb[1][1]));
    float mx = max3f(sc[0][0], sc[0][1], sc[0][2]);
    float my = max3f(sc[1][0], sc[1][1], sc[1][2]);
#pragma unroll
    for (int r = 3; r + 1 < 16; r += 2) {
      mx = max3f(mx, sc[0][r], sc[0][r + 1]);
      my = max3f(my, sc[1][r], sc[1][r + 1]);
    }
    mx = max3f(mx, my, fmaxf(sc[0][15], sc[1][15]));
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(int, mx), __builtin_bit_cast(int, mx),
                                                       false, false);
      mx = fmaxf(__builtin_bit_cast(float, (int)sw[0]), __builtin_bit_cast(float, (int)sw[1]));
    }
    const float mrow = mx + moff;
    const bool unsafe = !(mrow <= m + 15.0f);   // (m = -inf: unsafe)
    if (__any(unsafe)) {
      const float mnew = unsafe ? mrow : m;
      const float alpha = unsafe ? __builtin_amdgcn_exp2f(m - mnew) : 1.0f;
      m = mnew;
#pragma unroll
      for (int d = 0; d < 3; ++d) o[d] = o[d] * alpha;
      const float delta = m - moff;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int j = 0; j < 8; ++j) pb[kt][u][j] = (_Float16)__builtin_amdgcn_exp2f(sc[kt][8 * u + j] - delta);
    }
    pend = mrow > m + 8.0f;
    m_pend = mrow;
    if (kh + 1 < S) {
      th_cur = (float)thw[(kh + 1) * 32 + l32];
      moff = pend ? m_pend : m;
      coff = th_cur - moff;
      if constexpr (CMFMA) set_cq();
    }
  };
  auto softmax = [&](int kh) {
    if constexpr (COFF) return softmax_coff(kh);
    if (__any(pend)) {   // last row's deferred offset move
      const float alpha = pend ? __builtin_amdgcn_exp2f(m - m_pend) : 1.0f;
      m = pend ? m_pend : m;
#pragma unroll
      for (int d = 0; d < 3; ++d) o[d] = o[d] * alpha;
      pend = false;
    }
    float corr = m - th_cur;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) pb[kt][u][j] = (_Float16)(DBG_NOEXP ? sc[kt][8 * u + j] - corr
                                                                   : __builtin_amdgcn_exp2f(sc[kt][8 * u + j] - corr));
    float mx = max3f(sc[0][0], sc[0][1], sc[0][2]);
    float my = max3f(sc[1][0], sc[1][1], sc[1][2]);
#pragma unroll
    for (int r = 3; r + 1 < 16; r += 2) {
      mx = max3f(mx, sc[0][r], sc[0][r + 1]);
      my = max3f(my, sc[1][r], sc[1][r + 1]);
    }
    mx = max3f(mx, my, fmaxf(sc[0][15], sc[1][15]));
    {   // lane ^ 32 (the query's other 32 keys): one VALU permlane swap instead of an LDS bpermute
        // (v_permlane32_swap of mx with itself: result 0 holds mx[l & 31], result 1 mx[32 + (l & 31)])
      const auto sw = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(int, mx), __builtin_bit_cast(int, mx),
                                                       false, false);
      mx = fmaxf(__builtin_bit_cast(float, (int)sw[0]), __builtin_bit_cast(float, (int)sw[1]));
    }
    const float mrow = mx + th_cur;
    const bool unsafe = !(mrow <= m + 15.0f);   // (m = -inf: unsafe)
    if (__any(unsafe)) {
      const float mnew = unsafe ? mrow : m;
      const float alpha = unsafe ? __builtin_amdgcn_exp2f(m - mnew) : 1.0f;
      m = mnew;
#pragma unroll
      for (int d = 0; d < 3; ++d) o[d] = o[d] * alpha;
      corr = m - th_cur;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int j = 0; j < 8; ++j) pb[kt][u][j] = (_Float16)__builtin_amdgcn_exp2f(sc[kt][8 * u + j] - corr);
    }
    pend = mrow > m + 8.0f;
    m_pend = mrow;
    if (kh + 1 < S) th_cur = (float)thw[(kh + 1) * 32 + l32];
  };
  // V^T fragments of k16-step t = (kt, u): six ds_read_b64_tr_b16 (lo / hi key quads x 3 d-blocks)
  auto vread = [&](auto tc, uint32_t rb, half4_t (&lo)[3], half4_t (&hi)[3]) {
    constexpr int t = decltype(tc)::value;
    constexpr int KQ = 8 * (t >> 1) + 4 * (t & 1);   // key quad of slot j < 4 (+h); j >= 4: +2
    lo[0] = ds_read_tr16_off<KQ * QB>(vb01 + rb);
    hi[0] = ds_read_tr16_off<(KQ + 2) * QB>(vb01 + rb);
    lo[1] = ds_read_tr16_off<KQ * QB + 256>(vb01 + rb);
    hi[1] = ds_read_tr16_off<(KQ + 2) * QB + 256>(vb01 + rb);
    lo[2] = ds_read_tr16_off<KQ * QB2>(vb2 + rb);
    hi[2] = ds_read_tr16_off<(KQ + 2) * QB2>(vb2 + rb);
  };
  half4_t vlo0[3], vhi0[3];   // VPRE: the t = 0 fragments, read in the VALU segment
  auto pv = [&](int slot) {   // O^T += V^T . P^T: 4 k16-steps x 3 d-blocks, next step's reads in flight
    const uint32_t rb = slot * ROWB;
    half4_t lo[2][3], hi[2][3];
    if constexpr (VPRE) {
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        lo[0][d] = vlo0[d];
        hi[0][d] = vhi0[d];
      }
    } else {
      vread(std::integral_constant<int, 0>{}, rb, lo[0], hi[0]);
    }
    static_for<4>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      constexpr int cb = t & 1;
      if constexpr (t + 1 < 4) {
        vread(std::integral_constant<int, t + 1>{}, rb, lo[cb ^ 1], hi[cb ^ 1]);
        asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(lo[cb][0]), "+v"(hi[cb][0]), "+v"(lo[cb][1]), "+v"(hi[cb][1]),
                     "+v"(lo[cb][2]), "+v"(hi[cb][2]));
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(lo[cb][0]), "+v"(hi[cb][0]), "+v"(lo[cb][1]), "+v"(hi[cb][1]),
                     "+v"(lo[cb][2]), "+v"(hi[cb][2]));
      }
      if constexpr (!ONESL) {   // d-block 2, dims 80..95 -> 1.0 (row sums)
        union { half4_t v; uint32_t w[2]; } a, c;
        a.v = lo[cb][2];
        c.v = hi[cb][2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          a.w[e] = (a.w[e] & ones_and) | ones_or;
          c.w[e] = (c.w[e] & ones_and) | ones_or;
        }
        lo[cb][2] = a.v;
        hi[cb][2] = c.v;
      }
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const half8_t va = {lo[cb][d][0], lo[cb][d][1], lo[cb][d][2], lo[cb][d][3],
                            hi[cb][d][0], hi[cb][d][1], hi[cb][d][2], hi[cb][d][3]};
        if (DBG_NOMFMA) o[d][0] += (float)va[0] * (float)pb[t >> 1][t & 1][0];
        else o[d] = mfma32(va, pb[t >> 1][t & 1], o[d]);
      }
    });
  };

  // ---- key-row loop as a two-group ping-pong (MI355X_MICROARCH.md "Two waves per SIMD"): per
  // key row a VALU segment (softmax of row kh + the K fragment reads of row kh+1) and an MFMA
  // segment (P.V of row kh, Q.K^T of row kh+1), one barrier apart; waves 4..7 (group 1) run one
  // barrier behind waves 0..3, so each SIMD pairs one wave's softmax with its partner's MFMAs.
  // Barrier n: group 0's VALU segment of row kh lies between barriers 2kh-1 and 2kh, its MFMA
  // segment between 2kh and 2kh+1; group 1's one barrier later.  Ring of 5 slots, row r in slot
  // r % 5:
  //  * row kh+4 is staged at the start of the MFMA segment of row kh into row kh-1's slot, whose
  //    last reads (group 1's P.V of row kh-1) ended at that segment's opening barrier;
  //  * row r is first read by group 0's VALU segment of row r-1 (after barrier 2r-3), so every
  //    wave retires its pieces of row r before barrier 2r-3: group 0 at the end of its MFMA
  //    segment of row r-2, group 1 at the end of its VALU segment of row r-2.
  // The asm fences pin the softmax results and K fragments to their segment (the compiler would
  // otherwise sink the exp2s past the barrier into the MFMA segment).
  wait_vmcnt<0>();
  __syncthreads();   // rows 0..3 landed; TH visible
  kread(smem);
  qk();
  if (grp) __builtin_amdgcn_s_barrier();
  wg_mark<DBG>(wgt, 1);
  unsigned long long ph[4] = {0, 0, 0, 0}, tprev = 0;
  auto stamp = [&](int k) {
    if constexpr ((DBG & 1) != 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (tprev) ph[k] += t - tprev;
      tprev = t;
    }
  };
  // segment fences: empty volatile asm that "redefines" the registers crossing a barrier, so the
  // compiler can neither hoist the next row's softmax into the MFMA segment nor sink either
  // segment's work across its barrier
  auto fence_sc = [&] {
    asm volatile("" : "+v"(sc[0]), "+v"(sc[1]), "+v"(o[0]), "+v"(o[1]), "+v"(o[2]) :: "memory");
  };
  auto fence_pk = [&] {
    asm volatile("" : "+v"(pb[0][0]), "+v"(pb[0][1]), "+v"(pb[1][0]), "+v"(pb[1][1]), "+v"(kf[0][0]),
                 "+v"(kf[0][1]), "+v"(kf[0][2]), "+v"(kf[0][3]), "+v"(kf[0][4]) :: "memory");
    asm volatile("" : "+v"(kf[1][0]), "+v"(kf[1][1]), "+v"(kf[1][2]), "+v"(kf[1][3]), "+v"(kf[1][4]),
                 "+v"(o[0]), "+v"(o[1]), "+v"(o[2]) :: "memory");
    if constexpr (CMFMA) asm volatile("" : "+v"(cq));
  };
  // ring slots as rotating wave-uniform counters (no per-row modulo); constant vmcnt counts per
  // group: group 0 (waves 0..3) issues 3 pieces per row, group 1 two
  static_assert(NI == (G1DMA ? 5 : 3), "vmcnt counts below: 3 / 2 pieces per row for group 0 / 1 (G1DMA: 0 / 5)");
  int j = 0;   // kh % NSLOT
  if constexpr (STATPRIO) {
    if (grp) __builtin_amdgcn_s_setprio(1);
  }
  for (int kh = 0; kh < S; ++kh) {
    const int j1 = j == NSLOT - 1 ? 0 : j + 1, j4 = j == 0 ? NSLOT - 1 : j - 1;
    stamp(3);
    fence_sc();
    if constexpr (KEARLY) {
      if (kh + 1 < S) kread(smem + j1 * ROWB);
    }
    softmax(kh);
    if constexpr (G1DMA) {   // row kh+4 into row kh-1's slot: every P.V of row kh-1 ended at barrier 2kh
      if (grp && kh + 4 < S) issue(kh + 4, j4);
    }
    if constexpr (!KEARLY) {
      if (kh + 1 < S) kread(smem + j1 * ROWB);
    }
    if constexpr (VPRE) vread(std::integral_constant<int, 0>{}, j * ROWB, vlo0, vhi0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    fence_pk();
    if constexpr (VPRE)
      asm volatile("" : "+v"(vlo0[0]), "+v"(vlo0[1]), "+v"(vlo0[2]), "+v"(vhi0[0]), "+v"(vhi0[1]), "+v"(vhi0[2]));
    if constexpr (G1DMA) {
      if (grp && kh + 2 < S) {   // row kh+2 (rows kh+3, kh+4 newer), read by group 0 after barrier 2kh+1
        if (kh + 4 < S) wait_vmcnt<10>();
        else if (kh + 3 < S) wait_vmcnt<5>();
        else wait_vmcnt<0>();
      }
    } else if (grp && kh + 2 < S) {   // row kh+2 (row kh+3 newer)
      if (kh + 3 < S) wait_vmcnt<2>();
      else wait_vmcnt<0>();
    }
    stamp(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    stamp(1);
    fence_pk();
    if constexpr (!STATPRIO) __builtin_amdgcn_s_setprio(1);
    if (!G1DMA && !QKDMA && kh + 4 < S) issue(kh + 4, j4);
    pv(j);
    if constexpr (QKDMA) {
      const bool pf = kh + 4 < S;
      if (kh + 1 < S) {
        qk_d([&](int q) {
          if (pf && (q == 1 || q == 4 || q == 7)) {
            __builtin_amdgcn_sched_barrier(0);
            issue_one(kh + 4, j4, q / 3);
            __builtin_amdgcn_sched_barrier(0);
          }
        });
      } else if (pf) {
        issue(kh + 4, j4);
      }
    } else if (kh + 1 < S) {
      qk();
    }
    fence_sc();
    if constexpr (!STATPRIO) __builtin_amdgcn_s_setprio(0);
    if (!G1DMA && !grp && kh + 2 < S) {   // row kh+2 (rows kh+3, kh+4 newer)
      if (kh + 4 < S) wait_vmcnt<6>();
      else if (kh + 3 < S) wait_vmcnt<3>();
      else wait_vmcnt<0>();
    }
    stamp(2);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    j = j1;
  }
#ifdef SAMQ_TUNING
  if ((DBG & 1) && lane == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) atomicAdd(&g_attn_stamps[k + (grp ? 4 : 0)], ph[k]);
  }
#endif
  if constexpr (STATPRIO) __builtin_amdgcn_s_setprio(0);
  if (!grp) __builtin_amdgcn_s_barrier();   // balance group 1's extra barrier
  wg_mark<DBG>(wgt, 2);

  // ---- normalise + store: lane = query (qh, qw0 + l32), dims 32 db + 8 c + 4 h .. + 3
  const float inv = 1.0f / o[2][8];
  const int64_t dst_tok = (((int64_t)b * p.H + qh) * p.W + qw0 + l32) * C + head * D;
#pragma unroll
  for (int db = 0; db < 3; ++db)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (db == 2 && c >= 2) continue;
      const float4_t v = {o[db][4 * c], o[db][4 * c + 1], o[db][4 * c + 2], o[db][4 * c + 3]};
      attn_store4(p, dst_tok + 32 * db + 8 * c + 4 * h, v * inv);
    }
#ifdef SAMQ_TUNING
  if constexpr ((DBG & 8) != 0) {
    wg_mark<DBG>(wgt, 3);
    if (tid == 0) {
#pragma unroll
      for (int k = 0; k < 6; ++k) g_attn_wgt[blockIdx.x * 6 + k] = wgt[k];
    }
  }
#endif
}

static int launch_glob80(const AttnParams& p, int units, hipStream_t stream) {
  AttnParams q = p;
  q.nqb = 16;
  q.units = units;
#ifdef SAMQ_TUNING
  const char* e = getenv("SAMQ_ATTN_DBG");
  q.dbg = e ? atoi(e) : 0;
  if (q.dbg & 1) {
    unsigned long long z[8] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_attn_stamps), z, sizeof(z));
  }
#endif
#ifdef SAMQ_TUNING
  switch (q.dbg) {
    case 1: hipLaunchKernelGGL(glob80_attention_kernel<1>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 2: hipLaunchKernelGGL(glob80_attention_kernel<2>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 4: hipLaunchKernelGGL(glob80_attention_kernel<4>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 6: hipLaunchKernelGGL(glob80_attention_kernel<6>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 8: hipLaunchKernelGGL(glob80_attention_kernel<8>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 4096: hipLaunchKernelGGL(glob80_attention_kernel<4096>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 4097: hipLaunchKernelGGL(glob80_attention_kernel<4097>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 2048: hipLaunchKernelGGL(glob80_attention_kernel<2048>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 2304: hipLaunchKernelGGL(glob80_attention_kernel<2304>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 257: hipLaunchKernelGGL(glob80_attention_kernel<257>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 1024: hipLaunchKernelGGL(glob80_attention_kernel<1024>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 1280: hipLaunchKernelGGL(glob80_attention_kernel<1280>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 1025: hipLaunchKernelGGL(glob80_attention_kernel<1025>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 1032: hipLaunchKernelGGL(glob80_attention_kernel<1032>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 512: hipLaunchKernelGGL(glob80_attention_kernel<512>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 256: hipLaunchKernelGGL(glob80_attention_kernel<256>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 288: hipLaunchKernelGGL(glob80_attention_kernel<288>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 320: hipLaunchKernelGGL(glob80_attention_kernel<320>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 32: hipLaunchKernelGGL(glob80_attention_kernel<32>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 64: hipLaunchKernelGGL(glob80_attention_kernel<64>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 96: hipLaunchKernelGGL(glob80_attention_kernel<96>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 128: hipLaunchKernelGGL(glob80_attention_kernel<128>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 160: hipLaunchKernelGGL(glob80_attention_kernel<160>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 224: hipLaunchKernelGGL(glob80_attention_kernel<224>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 16: hipLaunchKernelGGL(glob80_attention_kernel<16>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    case 17: hipLaunchKernelGGL(glob80_attention_kernel<17>, dim3(16 * p.heads * units), dim3(512), 0, stream, q); break;
    default: hipLaunchKernelGGL(glob80_attention_kernel<0>, dim3(16 * p.heads * units), dim3(512), 0, stream, q);
  }
#else
  hipLaunchKernelGGL(glob80_attention_kernel<0>, dim3(16 * p.heads * units), dim3(512), 0, stream, q);
#endif
  SAMQ_LAUNCH_CHECK("glob80_attention launch");
#ifdef SAMQ_TUNING
  if (q.dbg & 1) {
    unsigned long long hst[8];
    (void)hipStreamSynchronize(stream);
    (void)hipMemcpyFromSymbol(hst, HIP_SYMBOL(g_attn_stamps), sizeof(hst));
    const double n = 16.0 * p.heads * units * 4 * 64;   // waves per group x rows
    fprintf(stderr, "glob80 stamps (cycles per wave-row): grp0 V %.0f bar %.0f M %.0f bar %.0f | grp1 V %.0f bar "
            "%.0f M %.0f bar %.0f\n", hst[0] / n, hst[1] / n, hst[2] / n, hst[3] / n, hst[4] / n, hst[5] / n,
            hst[6] / n, hst[7] / n);
  }
  if (q.dbg & 8) {   // per-workgroup timeline (realtime ticks = 10 ns)
    const int nwg = 16 * p.heads * units;
    std::vector<unsigned long long> t((size_t)nwg * 6);
    (void)hipStreamSynchronize(stream);
    (void)hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_attn_wgt), t.size() * 8);
    unsigned long long t0 = ~0ull, t3 = 0;
    for (int i = 0; i < nwg; ++i) { t0 = std::min(t0, t[i * 6]); t3 = std::max(t3, t[i * 6 + 3]); }
    std::vector<double> st, pro, lp, epi, clk, fin;
    for (int i = 0; i < nwg; ++i) {
      const unsigned long long* w = &t[i * 6];
      st.push_back((w[0] - t0) * 0.01); pro.push_back((w[1] - w[0]) * 0.01); lp.push_back((w[2] - w[1]) * 0.01);
      epi.push_back((w[3] - w[2]) * 0.01); fin.push_back((w[3] - t0) * 0.01);
      clk.push_back(w[2] > w[1] ? (double)(w[5] - w[4]) / ((w[2] - w[1]) * 10.0) : 0.0);
    }
    auto q5 = [](std::vector<double> v) {
      std::sort(v.begin(), v.end());
      const size_t n = v.size();
      char b[160];
      snprintf(b, sizeof(b), "min %.2f p25 %.2f med %.2f p75 %.2f max %.2f", v[0], v[n / 4], v[n / 2], v[3 * n / 4], v[n - 1]);
      return std::string(b);
    };
    fprintf(stderr, "glob80 timeline: span %.2f us over %d workgroups\n  start(us) %s\n  prologue(us) %s\n  loop(us) %s\n"
            "  epilogue(us) %s\n  finish(us) %s\n  loop clock(GHz) %s\n", (t3 - t0) * 0.01, nwg, q5(st).c_str(),
            q5(pro).c_str(), q5(lp).c_str(), q5(epi).c_str(), q5(fin).c_str(), q5(clk).c_str());
  }
#endif
  return SAMQ_OK;
}

template <int D>
static int launch_win(const AttnParams& p, int units, hipStream_t stream) {
  const int items = units * p.heads;
#ifdef SAMQ_TUNING
  // tuning A/B: 2 = the round-3 scaled-Q form (Win !UNSC); 4 = hi + lo P for either output
  const char* e = getenv("SAMQ_ATTN_WIN");
  if (e && (atoi(e) == 2 || atoi(e) == 4)) {
    if (atoi(e) == 2) hipLaunchKernelGGL((win_attention_kernel<D, false>), dim3(items), dim3(256), 0, stream, p, items);
    else hipLaunchKernelGGL((win_attention_kernel<D, true, true>), dim3(items), dim3(256), 0, stream, p, items);
    SAMQ_LAUNCH_CHECK("win_attention launch");
    return SAMQ_OK;
  }
#endif
  // unscaled Q (UNSC): 35.6 vs 36.2 us per ViT-H 2-image launch, fp16 output 1.59e-3 vs 1.95e-3
  // max-abs from the fp32 oracle, W4A8 store codes off by one 1.7e-3 vs 2.5e-3 (profiles/r4_m.win.log).
  // The W4A8 int8-code store (round 5): P as fp16 hi + lo (PHL), the output at
  // fp32-level error before the proj QAct's quantiser -- window-stage codes off by one 1.21-1.33e-3
  // instead of 2.05-2.24e-3, for two MFMAs per P.V step (int8-store launch 45.4 vs 35.5 us, W4A8
  // step -1.4 %, profiles/r5_w4a8_window_phl.log)
  if (p.out_scale > 0.f)
    hipLaunchKernelGGL((win_attention_kernel<D, true, true>), dim3(items), dim3(256), 0, stream, p, items);
  else
    hipLaunchKernelGGL((win_attention_kernel<D, true>), dim3(items), dim3(256), 0, stream, p, items);
  SAMQ_LAUNCH_CHECK("win_attention launch");
  return SAMQ_OK;
}

template <int D, int SP, int QT, int NW, bool RES, bool PRE, int RS = 16, int SC = 0>
static int launch_attn(const AttnParams& p, int units, hipStream_t stream) {
  const int tiles = p.S * (SP / 16);
  const int qblocks = (tiles + NW * QT - 1) / (NW * QT);
  if (!RES && (p.heads * units) % 8 == 0) {   // 1-D grid, XCD-aware (see the kernel)
    AttnParams q = p;
    q.nqb = qblocks;
    q.units = units;
    hipLaunchKernelGGL((rel_attention_kernel<D, SP, QT, NW, RES, PRE, RS, SC>), dim3(qblocks * p.heads * units),
                       dim3(64 * NW), 0, stream, q);
  } else {
    hipLaunchKernelGGL((rel_attention_kernel<D, SP, QT, NW, RES, PRE, RS, SC>), dim3(qblocks, p.heads, units),
                       dim3(64 * NW), 0, stream, p);
  }
  SAMQ_LAUNCH_CHECK("rel_attention launch");
  return SAMQ_OK;
}

template <bool PRE>
static int dispatch_attn(const AttnParams& p, int hd, int units, hipStream_t stream) {
  const int S = p.S;
  if (!PRE && S == 14)   // SAM's window size: two-workgroups-per-CU window kernel
    return hd == 80 ? launch_win<80>(p, units, stream) : launch_win<64>(p, units, stream);
  // ViT-H global blocks: the 32x32-MFMA kernel (needs heads * units % 8 == 0 for its XCD order)
  if (!PRE && S == 64 && hd == 80 && (p.heads * units) % 8 == 0 && p.H == 64 && p.W == 64)
    return launch_glob80(p, units, stream);
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

static int rel_attention_impl(const void* qkv, const void* qkv_bias, const void* rel_pos_h, const void* rel_pos_w,
                              void* out, int B, int H, int W, int heads, int hd, int window, float sm_scale,
                              float out_scale, hipStream_t stream) {
  if (B == 0) return SAMQ_OK;   // empty batch: no work, data pointers may be null
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
  p.out_scale = out_scale;
  p.out_inv = out_scale > 0.f ? 1.0f / out_scale : 0.f;
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

extern "C" int samq_rel_attention(const void* qkv, const void* qkv_bias, const void* rel_pos_h, const void* rel_pos_w,
                                  void* out, int B, int H, int W, int heads, int hd, int window, float sm_scale,
                                  hipStream_t stream) {
  return rel_attention_impl(qkv, qkv_bias, rel_pos_h, rel_pos_w, out, B, H, W, heads, hd, window, sm_scale, 0.f,
                            stream);
}

extern "C" int samq_rel_attention_q(const void* qkv, const void* qkv_bias, const void* rel_pos_h,
                                    const void* rel_pos_w, int8_t* out, int B, int H, int W, int heads, int hd,
                                    int window, float sm_scale, float out_scale, hipStream_t stream) {
  SAMQ_REQUIRE(out_scale > 0.f, SAMQ_ERR_INVALID, "rel_attention_q: out_scale must be > 0");
  SAMQ_REQUIRE(((uintptr_t)out & 3) == 0, SAMQ_ERR_INVALID, "rel_attention_q: out must be 4-byte aligned");
  return rel_attention_impl(qkv, qkv_bias, rel_pos_h, rel_pos_w, out, B, H, W, heads, hd, window, sm_scale,
                            out_scale, stream);
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

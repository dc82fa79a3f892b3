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
  int nqb, units;           // streaming path with a 1-D XCD-ordered grid: query blocks, units
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
  // XCD-aware order for the streaming (global) path: the grid is 1-D and the query blocks of one
  // (image, head) all land on one XCD (workgroups are dealt round-robin over the 8 XCDs), so that
  // XCD's L2 serves their shared K/V stream instead of every XCD fetching every head's keys
  int qblk = blockIdx.x, head = blockIdx.y, unit = blockIdx.z;
  if (!RESIDENT && gridDim.y == 1 && gridDim.z == 1) {
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

// ------------------------------------------------------------------ windowed attention, persistent
// The 14x14-window blocks (28 of 32 in ViT-H) as a persistent kernel: one workgroup per CU walks
// its share of the (window, head) items with the NEXT item's K/V already streaming into the
// second LDS buffer (LDS-DMA) and its Q into registers while the current item computes, so the
// HBM stream and the MFMA/VALU work overlap inside one CU.  Per item, everything is local to
// the window and the VALU work per score is cut to max3/sub/exp/cvt:
//  * the whole score s[q,k] = q.k*scale + TH[q,kh] + TW[q,kw] (log2 domain) comes out of the
//    MFMAs: S^T = K'.Q'^T on 16x16x32 with TW as the C input, and TH carried by 16 extra
//    contraction dims -- K' rows get a one-hot of their key row (DMA'd from a constant table
//    next to the K data), Q' rows get TH[q, 0..15] in fp16 (the reference also rounds rel_h to
//    fp16, fused_attention.py:46-80); for D = 80 these are the zero-padded dims 80..95 of the
//    third k-step, so TH costs no MFMA at all;
//  * one exact softmax over the window's 196 keys (no online rescale); the two masked slots of
//    each 16-slot key row are -inf in the C input;
//  * O^T += V^T . P^T on 16x16x32 with two key rows per MFMA (k order [row 2p: 4g..4g+3 |
//    row 2p+1: 4g..4g+3], the score registers' own layout; V^T by ds_read_b64_tr_b16), and the
//    softmax denominator as one more MFMA against an all-ones A operand (sum of the same fp16
//    P that multiplies V);
//  * the rel-pos tables (shared by every window and head) sit in LDS for the whole kernel.
// Items are numbered so the 32 workgroups of one XCD take the 16 heads of the same two windows
// at a time (the cache lines shared by adjacent heads' K/V slices then land in one L2).
struct OneHot16 { uint16_t v[16 * 16]; };
constexpr OneHot16 make_onehot16() {
  OneHot16 o{};
  for (int r = 0; r < 16; ++r) o.v[r * 16 + r] = 0x3C00;   // fp16 1.0 on the diagonal
  return o;
}
__device__ __attribute__((aligned(16))) OneHot16 g_onehot16 = make_onehot16();

template <int D>
__global__ __launch_bounds__(64 * 7, 1) void win_attention_kernel(AttnParams p, int items) {
  constexpr int S = 14, NW = 7, QT = 2;
  constexpr int KS = 3;                         // k32 steps of Q'.K'^T: D + 16 TH dims <= 96
  constexpr int DT = D / 16;
  constexpr int D8 = D / 8;
  constexpr int KCH = D8 + 2;                   // 16-byte chunks per K' row (data + one-hot)
  constexpr int KROW = KCH * 16;                // K' row pitch (bytes)
  constexpr int GTH = (D - 64) / 8;             // first lane group holding TH dims in k-step 2
  constexpr int RKEYS = S * S + 16 - S;         // 196 keys + slack for the last row's 16-slot tile
  constexpr int KC = RKEYS * KCH, VC = RKEYS * D8;
  constexpr int NI = (KC + VC + 64 * NW - 1) / (64 * NW);
  constexpr int BUFB = NI * NW * 1024;
  constexpr int TAB = (2 * S - 1) * D;          // elements per rel-pos table
  constexpr int TABP = TAB + 32;                // + slack: k-step-2 reads past the last row
  constexpr int TH16_BYTES = NW * QT * 16 * 32;
  constexpr int SMEM = 2 * TABP * 2 + TH16_BYTES + 2 * BUFB;
  static_assert(SMEM <= 160 * 1024, "LDS");
  static_assert(D == 64 || D == 80, "head dim");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  _Float16* tab_h = (_Float16*)smem;
  _Float16* tab_w = tab_h + TABP;
  char* th16 = smem + 2 * TABP * 2;
  char* bufs = th16 + TH16_BYTES;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int ql = lane & 15;
  const int g = lane >> 4;
  const int C = p.C;
  const int64_t ts = p.tok_stride;
  const float qscale = p.scale * LOG2E;
  const bool qin2 = 64 + 8 * g < D;             // lane holds real q dims in k-step 2
  const bool thl = g == GTH || g == GTH + 1;    // lane holds TH dims in k-step 2

  // rel-pos tables -> LDS (once per workgroup); the slack is zeroed
  for (int i = tid; i < 2 * TABP / 8; i += 64 * NW) {
    const int which = i >= TABP / 8;
    const int j = which ? i - TABP / 8 : i;
    half8_t v = {};
    if (8 * j < TAB) v = *(const half8_t*)((which ? p.relw : p.relh) + 8 * j);
    *(half8_t*)((which ? tab_w : tab_h) + 8 * j) = v;
  }

  // logical item -> (unit, head); workgroups of one XCD share windows (see header)
  const int nxcd_wg = gridDim.x >> 3;           // grid is a multiple of 8
  auto item_of = [&](int it) -> int {
    const int b = blockIdx.x;
    return it * gridDim.x + (b & 7) * nxcd_wg + (b >> 3);
  };
  struct Geo { int b, Y0, X0, head; bool edge; };
  auto geo = [&](int item) -> Geo {
    const int unit = item / p.heads;
    Geo o;
    o.head = item - unit * p.heads;
    o.b = unit / p.upi;
    const int wi = unit - o.b * p.upi;
    o.Y0 = (wi / p.nwx) * S;
    o.X0 = (wi % p.nwx) * S;
    o.edge = o.Y0 + S > p.H || o.X0 + S > p.W;
    return o;
  };

  // ---- per-lane DMA chunk table (item-invariant): offset of the chunk relative to the item's
  // first token (elements) for token chunks, or into g_onehot16; kind in the top bits
  // (0 token K/V data, 1 one-hot, 2 zero).  Edge windows re-derive (row, slot) on a slow path.
  uint32_t chunk[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int c = (wave * NI + i) * 64 + lane;
    const bool isv = c >= KC;
    const int cc = isv ? c - KC : c;
    const int per = isv ? D8 : KCH;
    const int key = cc / per, d8 = cc - (cc / per) * per;
    const int r = key / S, slot = key - (key / S) * S;
    uint32_t e;
    if (c >= KC + VC) e = 2u << 30;
    else if (!isv && d8 >= D8) e = (1u << 30) | (uint32_t)((r < S ? r : 15) * 16 + 8 * (d8 - D8));
    else if (r >= S) e = 2u << 30;
    else e = (uint32_t)((r * p.W + slot) * ts + (isv ? 2 * C : C) + d8 * 8);
    chunk[i] = e;
  }
  auto issue = [&](const Geo& q, int buf) {
    const _Float16* tok0 = p.qkv + (((int64_t)q.b * p.H + q.Y0) * p.W + q.X0) * ts + q.head * D;
    const _Float16* onehot = (const _Float16*)&g_onehot16;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      uint32_t e = chunk[i];
      asm volatile("" : "+v"(e));   // no loop-invariant 64-bit pointers hoisted out of the item loop
      const uint32_t kind = e >> 30, off = e & 0x3FFFFFFFu;
      const _Float16* src = kind == 0 ? tok0 + off : (kind == 1 ? onehot + off : g_zero16);
      if (q.edge && kind == 0) {   // pad token of an edge window: its K/V = the qkv bias
        const int c = (wave * NI + i) * 64 + lane;
        const bool isv = c >= KC;
        const int cc = isv ? c - KC : c;
        const int per = isv ? D8 : KCH;
        const int key = cc / per, d8 = cc - (cc / per) * per;
        const int r = key / S, slot = key - (key / S) * S;
        if (q.Y0 + r >= p.H || q.X0 + slot >= p.W)
          src = p.qkv_bias ? p.qkv_bias + (isv ? 2 * C : C) + q.head * D + d8 * 8 : g_zero16;
      }
      __builtin_amdgcn_global_load_lds((const SAMQ_GLOBAL void*)src,
                                       (SAMQ_LDS void*)(bufs + buf * BUFB + (wave * NI + i) * 1024), 16, 0, 0);
    }
  };
  // Q of this wave's tiles (query row wave*QT + t, slots ql) -> registers, unscaled; every lane
  // issues every load (zero source for absent data) so the vmcnt count is wave-uniform
  auto load_q = [&](const Geo& q, half8_t (&qv)[QT][KS]) {
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      const int qr = wave * QT + t;
      const bool inwin = qr < S && ql < S;
      const bool real = inwin && q.Y0 + qr < p.H && q.X0 + ql < p.W;
      const int64_t tok = ((int64_t)q.b * p.H + (q.Y0 + qr)) * p.W + (q.X0 + ql);
      const _Float16* pad = (inwin && p.qkv_bias) ? p.qkv_bias + q.head * D : nullptr;
      const _Float16* src = real ? p.qkv + tok * ts + q.head * D : pad;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const _Float16* a = (src && (s < 2 || qin2)) ? src + 32 * s + 8 * g : g_zero16;
        asm volatile("" : "+v"(a));   // opaque: keeps the compiler from splitting the loads by source
        qv[t][s] = *(const SAMQ_GLOBAL half8_t*)a;
      }
    }
  };

  int it = 0;
  int item = item_of(0);
  if (item >= items) return;
  Geo cur = geo(item);
  half8_t qn[QT][KS];
  issue(cur, 0);
  load_q(cur, qn);

  const int trow = ql >> 2;            // ds_read_b64_tr_b16 addressing (see rel_attention_kernel)
  const int tcol = 4 * (ql & 3);
  char* th_w = th16 + wave * (QT * 16 * 32);
  const half8_t ones = {1, 1, 1, 1, 1, 1, 1, 1};
  int buf = 0;

  for (;;) {
    wait_vmcnt<0>();
    __syncthreads();   // item's K/V + Q landed and visible; the other buffer is free (all waves past it)
    half8_t qf[QT][KS];
#pragma unroll
    for (int t = 0; t < QT; ++t)
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        half8_t v = qn[t][s];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (_Float16)((float)v[j] * qscale);
        qf[t][s] = v;
      }
    const int nitem = item_of(it + 1);
    const bool has_next = nitem < items;
    Geo nxt = cur;
    if (has_next) {
      nxt = geo(nitem);
      issue(nxt, buf ^ 1);
      load_q(nxt, qn);
    }

    // ---- rel-pos terms: TW -> C input (slots >= S masked to -inf); TH -> the Q' extra dims
    float4_t tw[QT];
    const float inv_scale = 1.0f / p.scale;    // (Qs . R) / scale = log2e * (q . R)
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      const int qr = wave * QT + t;
      const int qh = qr < S ? qr : S - 1;
      int r = qh - ql + S - 1;
      r = r < 0 ? 0 : r;
      float4_t th, tww;
#pragma unroll
      for (int which = 0; which < 2; ++which) {
        const _Float16* rp = (which ? tab_w : tab_h) + r * D;
        float4_t a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s)   // k-step 2 of lanes without q dims multiplies zeros
          a = __builtin_amdgcn_mfma_f32_16x16x32_f16(*(const half8_t*)(rp + 32 * s + 8 * g), qf[t][s], a, 0, 0, 0);
        a = a * inv_scale;
        if (which) tww = a; else th = a;
      }
      if (g == 3) { tww[2] = -INFINITY; tww[3] = -INFINITY; }   // key slots 14, 15
      tw[t] = tww;
      // lane (g, ql) holds TH[kh = 4g..4g+3][ql]; lanes of groups GTH, GTH+1 need kh 0..7 / 8..15
      *(half4_t*)(th_w + (t * 16 + ql) * 32 + 8 * g) =
          half4_t{(_Float16)th[0], (_Float16)th[1], (_Float16)th[2], (_Float16)th[3]};
      const half8_t thv = *(const half8_t*)(th_w + (t * 16 + ql) * 32 + 16 * (g - GTH > 0 ? 1 : 0));
      half8_t q2 = qin2 ? qf[t][2] : half8_t{};
      qf[t][2] = thl ? thv : q2;
    }

    const char* kb = bufs + buf * BUFB;
    const char* vb = kb + KC * 16;

    // ---- scores S^T = K'.Q'^T + TW for all key rows
    float4_t sc[QT][S];
#pragma unroll
    for (int kh = 0; kh < S; ++kh) {
      half8_t kf[KS];
#pragma unroll
      for (int s = 0; s < KS; ++s) kf[s] = *(const half8_t*)(kb + (kh * S + ql) * KROW + (32 * s + 8 * g) * 2);
#pragma unroll
      for (int t = 0; t < QT; ++t) {
        float4_t a = tw[t];
#pragma unroll
        for (int s = 0; s < KS; ++s) a = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[s], qf[t][s], a, 0, 0, 0);
        sc[t][kh] = a;
      }
      __builtin_amdgcn_sched_barrier(0);   // keep the K' loads of row kh next to their MFMAs
    }

    // ---- exact softmax over the window (exp2 domain)
    half8_t pb[QT][S / 2];
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      float mx = max3f(sc[t][0][0], sc[t][0][1], sc[t][0][2]);
      mx = max3f(mx, sc[t][0][3], sc[t][1][0]);
      mx = max3f(mx, sc[t][1][1], sc[t][1][2]);
      mx = fmaxf(mx, sc[t][1][3]);
#pragma unroll
      for (int kh = 2; kh < S; ++kh) {
        mx = max3f(mx, sc[t][kh][0], sc[t][kh][1]);
        mx = max3f(mx, sc[t][kh][2], sc[t][kh][3]);
      }
      mx = max3f(mx, __shfl_xor(mx, 16, 64), __shfl_xor(mx, 32, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
#pragma unroll
      for (int pr = 0; pr < S / 2; ++pr)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pb[t][pr][r] = (_Float16)__builtin_amdgcn_exp2f(sc[t][2 * pr][r] - mx);
          pb[t][pr][4 + r] = (_Float16)__builtin_amdgcn_exp2f(sc[t][2 * pr + 1][r] - mx);
        }
    }

    // ---- O^T = V^T . P^T (two key rows per MFMA; V^T fragments of the next pair in flight),
    // l = ones . P^T
    float4_t o[QT][DT], lsum[QT];
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      lsum[t] = float4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int d = 0; d < DT; ++d) o[t][d] = float4_t{0.f, 0.f, 0.f, 0.f};
    }
    const uint32_t vaddr = lds_addr(vb + ((4 * g + trow) * D + tcol) * 2);
    half4_t vlo[2][DT], vhi[2][DT];
#pragma unroll
    for (int d = 0; d < DT; ++d) {
      vlo[0][d] = ds_read_tr16(vaddr + d * 32);
      vhi[0][d] = ds_read_tr16(vaddr + S * D * 2 + d * 32);
    }
#pragma unroll
    for (int pr = 0; pr < S / 2; ++pr) {
      const int cb = pr & 1;
      if (pr + 1 < S / 2) {
#pragma unroll
        for (int d = 0; d < DT; ++d) {
          vlo[cb ^ 1][d] = ds_read_tr16(vaddr + (2 * pr + 2) * S * D * 2 + d * 32);
          vhi[cb ^ 1][d] = ds_read_tr16(vaddr + (2 * pr + 3) * S * D * 2 + d * 32);
        }
      }
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
        for (int t = 0; t < QT; ++t) o[t][d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va, pb[t][pr], o[t][d], 0, 0, 0);
      }
#pragma unroll
      for (int t = 0; t < QT; ++t) lsum[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ones, pb[t][pr], lsum[t], 0, 0, 0);
    }

    // ---- normalise + store (token-major [B, H, W, C])
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      const int qr = wave * QT + t;
      if (qr >= S || ql >= S || cur.Y0 + qr >= p.H || cur.X0 + ql >= p.W) continue;
      const float inv = 1.0f / lsum[t][0];
      _Float16* dst = p.out + (((int64_t)cur.b * p.H + (cur.Y0 + qr)) * p.W + (cur.X0 + ql)) * C + cur.head * D;
#pragma unroll
      for (int d = 0; d < DT; ++d) {
        half4_t v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (_Float16)(o[t][d][r] * inv);
        *(half4_t*)(dst + d * 16 + 4 * g) = v;
      }
    }

    if (!has_next) break;
    ++it;
    item = nitem;
    cur = nxt;
    buf ^= 1;
  }
}

template <int D>
static int launch_win(const AttnParams& p, int units, hipStream_t stream) {
  const int items = units * p.heads;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  int grid = cus < items ? cus : items;
  grid = (grid + 7) & ~7;   // multiple of 8 (XCD-aware item numbering); surplus workgroups exit
  hipLaunchKernelGGL((win_attention_kernel<D>), dim3(grid), dim3(64 * 7), 0, stream, p, items);
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
  if (!PRE && S == 14)   // SAM's window size: persistent double-buffered kernel
    return hd == 80 ? launch_win<80>(p, units, stream) : launch_win<64>(p, units, stream);
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

// Windowed / global multi-head attention with in-kernel decomposed relative-position bias.
//
// Replaces QuantAttention's attention part (gptq_triton/fused_attention.py:107-149): the two
// torch.matmul rel-pos products (add_decomposed_rel_pos :46-80), the `torch.full(+inf)` output
// init and the Triton flash kernel `_fwd_kernel1` (:159-309) -- and, in the windowed blocks,
// the window_partition / window_unpartition copies (image_encoder.py:195-202, 282-333): tokens
// are read from / written to the natural [B, H, W, C] layout, padded window tokens are
// synthesised in-kernel (their q/k/v equal the qkv bias).
//
// Structure (gfx950, wave64, v_mfma_f32_16x16x{32,16}_f16):
//  * work unit = (window or image, head, block of query tiles); a query tile is 16 queries of
//    ONE grid row (grid rows are padded to SP = 16 or 64 slots), so every tile has a single
//    query row index qh;
//  * keys are consumed one GRID ROW at a time (SP slots): the scores of a key row are
//        s[q, kw] = q.k * scale + TH[q, kh] + TW[q, kw]
//    where TW[q, kw] = q . Rw[qh - kw + S - 1] is the SAME for every key row, so it is computed
//    once per query tile by MFMA straight into the score-tile register layout and used as the
//    initial accumulator of every Q.K^T; TH[q, kh] = q . Rh[qh - kh + S - 1] is one scalar per
//    (query, key row) kept in LDS.  (Both tables index the query ROW qh: reference quirk 1.)
//  * scores are computed transposed (S^T = K . Q^T) so each lane owns one query and softmax
//    row reductions are in-register + 2 cross-lane steps; P feeds P.V as the B operand with a
//    permuted k order that V^T (staged transposed in LDS) reads with two ds_read_b64;
//  * online softmax in exp2 domain, f32 statistics, f16 MFMA operands, f32 accumulation;
//  * K / V^T key rows are register-prefetched and double-buffered in LDS (1 barrier / row).
#include "common.h"

namespace samq {

constexpr float LOG2E = 1.4426950408889634f;

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

template <int D, int SP, int QT, bool PRECOMP>
__global__ __launch_bounds__(256) void rel_attention_kernel(AttnParams p) {
  constexpr int KT = SP / 16;            // key tiles per key row
  constexpr int DT = D / 16;             // d tiles
  constexpr int DP = D + 8;              // K row pitch (halfs) in LDS
  constexpr int VP = SP + 4;             // V^T row pitch (halfs)
  constexpr int K_BYTES = SP * DP * 2;
  constexpr int V_BYTES = D * VP * 2;
  constexpr int BUF_BYTES = K_BYTES + V_BYTES;
  constexpr int TH_BYTES = 4 * QT * SP * 16 * 4;
  constexpr int D8 = D / 8;
  constexpr int NCHUNK = 2 * SP * D8;
  constexpr int CH = (NCHUNK + 255) / 256;
  static_assert(D == 64 || D == 80, "head dim");
  static_assert(SP == 16 || SP == 32 || SP == 64, "row pad");

  __shared__ __attribute__((aligned(16))) char smem[2 * BUF_BYTES + TH_BYTES];
  float* th_lds = (float*)(smem + 2 * BUF_BYTES);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int ql = lane & 15;
  const int g = lane >> 4;
  const int head = blockIdx.y;
  const int unit = blockIdx.z;
  const int S = p.S;
  const int b = unit / p.upi;
  const int wi = unit % p.upi;
  const int Y0 = (wi / p.nwx) * S;
  const int X0 = (wi % p.nwx) * S;
  const int C = p.C;
  const float qscale = p.scale * LOG2E;

  // token helpers: 0 = real, 1 = window pad (bias), 2 = slot pad (masked / unused)
  auto tok_kind = [&](int y, int x) -> int {
    if (x >= S || y >= S) return 2;
    return (Y0 + y < p.H && X0 + x < p.W) ? 0 : 1;
  };
  auto tok_ptr = [&](int y, int x) -> const _Float16* {
    return p.qkv + (((int64_t)b * p.H + (Y0 + y)) * p.W + (X0 + x)) * p.tok_stride;
  };

  // ---------------------------------------------------------------- Q fragments (scaled)
  // D = 80 is covered by three 16x16x32 k-steps; lanes of the third step with d >= D hold 0.
  constexpr int KS = (D + 31) / 32;
  const bool kin3 = 64 + 8 * g < D;   // lane group holds real d in the last k-step
  half8_t qf[QT][KS];
  int qrow[QT], qcol0[QT];
  bool qvalid[QT];
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    const int qi = (blockIdx.x * 4 + wave) * QT + t;
    qrow[t] = qi / KT;
    qcol0[t] = (qi % KT) * 16;
    const int kind = tok_kind(qrow[t], qcol0[t] + ql);
    qvalid[t] = kind != 2;
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
  float* th_w = th_lds + wave * (QT * SP * 16);
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    const int qh = qrow[t] < S ? qrow[t] : S - 1;
    if (!PRECOMP) {
#pragma unroll
      for (int which = 0; which < 2; ++which) {
        const _Float16* tab = which ? p.relw : p.relh;
#pragma unroll
        for (int kt = 0; kt < KT; ++kt) {
          const int kk = kt * 16 + ql;                 // table row for the A operand
          int r = qh - kk + S - 1;
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
            for (int r2 = 0; r2 < 4; ++r2) th_w[(t * SP + kt * 16 + 4 * g + r2) * 16 + ql] = a[r2];
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
          th_w[(t * SP + kk) * 16 + ql] = kin ? (float)p.relh[base + kk] * LOG2E : 0.f;
        }
      }
    }
  }

  // ---------------------------------------------------------------- K/V staging
  uint4 stg[CH];
  auto load_row = [&](int kh) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = tid + 256 * i;
      uint4 v = {0u, 0u, 0u, 0u};
      if (c < NCHUNK) {
        const bool isv = c >= SP * D8;
        const int cc = isv ? c - SP * D8 : c;
        const int x = cc / D8, d8 = cc % D8;
        const int kind = tok_kind(kh, x);
        const int off = (isv ? 2 * C : C) + head * D + d8 * 8;
        if (kind == 0) v = *(const uint4*)(tok_ptr(kh, x) + off);
        else if (kind == 1 && p.qkv_bias) v = *(const uint4*)(p.qkv_bias + off);
      }
      stg[i] = v;
    }
  };
  auto store_row = [&](int buf) {
    char* base = smem + buf * BUF_BYTES;
    _Float16* vt = (_Float16*)(base + K_BYTES);
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = tid + 256 * i;
      if (c < NCHUNK) {
        const bool isv = c >= SP * D8;
        const int cc = isv ? c - SP * D8 : c;
        const int x = cc / D8, d8 = cc % D8;
        if (!isv) {
          *(uint4*)(base + (x * DP + d8 * 8) * 2) = stg[i];
        } else {
          const half8_t h = __builtin_bit_cast(half8_t, stg[i]);
#pragma unroll
          for (int j = 0; j < 8; ++j) vt[(d8 * 8 + j) * VP + x] = h[j];
        }
      }
    }
  };

  float m[QT], l[QT];
  float4_t o[QT][DT];
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    m[t] = -INFINITY;
    l[t] = 0.f;
#pragma unroll
    for (int d = 0; d < DT; ++d) o[t][d] = float4_t{0.f, 0.f, 0.f, 0.f};
  }

  load_row(0);
  store_row(0);
  __syncthreads();

  for (int kh = 0; kh < S; ++kh) {
    const int buf = kh & 1;
    if (kh + 1 < S) load_row(kh + 1);
    const char* kb = smem + buf * BUF_BYTES;
    const _Float16* vt = (const _Float16*)(kb + K_BYTES);

    // ---- scores S^T (per key tile, per query tile)
    float4_t sc[QT][KT];
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      const float thv = th_w[(t * SP + kh) * 16 + ql];
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) sc[t][kt] = tw[t][kt] + thv;
    }
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      const char* krow = kb + ((kt * 16 + ql) * DP) * 2;
      const half8_t k0 = *(const half8_t*)(krow + (8 * g) * 2);
      const half8_t k1 = *(const half8_t*)(krow + (32 + 8 * g) * 2);
      half8_t k2 = {};
      if (D == 80 && kin3) k2 = *(const half8_t*)(krow + (64 + 8 * g) * 2);
#pragma unroll
      for (int t = 0; t < QT; ++t) {
        sc[t][kt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(k0, qf[t][0], sc[t][kt], 0, 0, 0);
        sc[t][kt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(k1, qf[t][1], sc[t][kt], 0, 0, 0);
        if (D == 80) sc[t][kt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(k2, qf[t][KS - 1], sc[t][kt], 0, 0, 0);
      }
    }

    // ---- online softmax (exp2 domain)
    half8_t pb[QT][(SP + 31) / 32];
    half4_t pb16[QT];
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      if (SP > 14) {  // mask padded key slots (only when S < SP)
#pragma unroll
        for (int kt = 0; kt < KT; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (kt * 16 + 4 * g + r >= S) sc[t][kt][r] = -INFINITY;
      }
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, sc[t][kt][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = fmaxf(m[t], mx);
      const float alpha = __builtin_amdgcn_exp2f(m[t] - mnew);
      m[t] = mnew;
      float rs = 0.f;
#pragma unroll
      for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __builtin_amdgcn_exp2f(sc[t][kt][r] - mnew);
          sc[t][kt][r] = e;
          rs += e;
        }
      l[t] = l[t] * alpha + rs;
#pragma unroll
      for (int d = 0; d < DT; ++d) o[t][d] = o[t][d] * alpha;
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

    // ---- O^T += V^T . P^T
#pragma unroll
    for (int d = 0; d < DT; ++d) {
      const _Float16* vrow = vt + (d * 16 + ql) * VP;
      if (SP == 16) {
        const half4_t va = *(const half4_t*)(vrow + 4 * g);
#pragma unroll
        for (int t = 0; t < QT; ++t) o[t][d] = __builtin_amdgcn_mfma_f32_16x16x16f16(va, pb16[t], o[t][d], 0, 0, 0);
      } else {
#pragma unroll
        for (int s = 0; s < SP / 32; ++s) {
          const half4_t lo = *(const half4_t*)(vrow + 32 * s + 4 * g);
          const half4_t hi = *(const half4_t*)(vrow + 32 * s + 16 + 4 * g);
          const half8_t va = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
          for (int t = 0; t < QT; ++t) o[t][d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va, pb[t][s], o[t][d], 0, 0, 0);
        }
      }
    }

    if (kh + 1 < S) store_row(buf ^ 1);
    __syncthreads();
  }

  // ---------------------------------------------------------------- normalise + store
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    float lt = l[t];
    lt += __shfl_xor(lt, 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    const int x = qcol0[t] + ql;
    if (!qvalid[t] || tok_kind(qrow[t], x) != 0) continue;
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

template <int D, int SP, int QT, bool PRE>
static int launch_attn(const AttnParams& p, int units, hipStream_t stream) {
  const int tiles = p.S * (SP / 16);
  const int qblocks = (tiles + 4 * QT - 1) / (4 * QT);
  hipLaunchKernelGGL((rel_attention_kernel<D, SP, QT, PRE>), dim3(qblocks, p.heads, units), dim3(256), 0, stream, p);
  SAMQ_LAUNCH_CHECK("rel_attention launch");
  return SAMQ_OK;
}

template <bool PRE>
static int dispatch_attn(const AttnParams& p, int hd, int units, hipStream_t stream) {
  const int S = p.S;
  if (S <= 16) {
    return hd == 80 ? launch_attn<80, 16, 4, PRE>(p, units, stream) : launch_attn<64, 16, 4, PRE>(p, units, stream);
  } else if (S == 32) {
    return hd == 80 ? launch_attn<80, 32, 2, PRE>(p, units, stream) : launch_attn<64, 32, 2, PRE>(p, units, stream);
  } else {
    return hd == 80 ? launch_attn<80, 64, 2, PRE>(p, units, stream) : launch_attn<64, 64, 2, PRE>(p, units, stream);
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
    SAMQ_REQUIRE(H == 16 || H == 32 || H == 64 || H < 16, SAMQ_ERR_UNSUPPORTED,
                 "rel_attention: global grid side must be < 16, 16, 32 or 64");
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

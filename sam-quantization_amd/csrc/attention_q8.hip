// W8A8 (fq_vit) attention with decomposed relative position on int8 q/k/v codes, gfx950.
//
// Replaces fq_vit's quant-mode Attention.forward (fq_vit/models/sam/image_encoder.py:437-478):
//   qkv   = qact1(qkv(x))                       -> int8 codes, per-tensor scale s_qkv (input)
//   attn  = qact_attn1((q * scale) @ k^T)       -> quantised with s_a1
//   attn  = use_rel_pos_qact(attn + rel_h + rel_w)   (add_decomposed_rel_pos, quirk-1 rel_w
//           indexed by the query ROW, image_encoder.py:402)          -> quantised with s_a2
//   attn  = softmax(attn)                       (QIntSoftmax = F.softmax, layers.py:379)
//   o     = qact2(attn @ v)                     -> int8 codes with s_out (output, proj input)
// together with window_partition / window_unpartition (padded tokens are keys/values whose qkv is
// the fake-quantised qkv bias, exactly as the reference's zero-padded LayerNorm output projects).
//
// Arithmetic (all exact or fp32, SURVEY.md §8c Oracle F):
//   * q.k on v_mfma_i32_16x16x64_i8: exact int32; value = int * (s_qkv * scale * s_qkv);
//   * rel_h / rel_w: fp32 dot products of the fake-quant q (code * s_qkv) with the f32 tables;
//   * the two score quantisers use a true division and round-half-to-even (uniform.py:31-36);
//   * softmax in fp32 (online, exp of x - max as the reference), P.V on fp16 MFMA with P split
//     hi + lo (both fp16; |P - hi - lo| ~ 2^-22 |P|) and the exact int8 V codes as fp16.
// Layout: S^T = K.Q^T per 16-key block (lane = one query, 4 keys), so P^T feeds the P.V MFMA's B
// operand from the same registers; V^T is staged in LDS as fp16 [d][key].
//
// Grid: (images * windows, heads, query tiles of 16*NWQ).  RESIDENT (windows, S*S <= 256 keys):
// all keys staged once; otherwise 64-key chunks double-buffered through LDS.
#include "common.h"

namespace samq {

struct AttnQ8Params {
  const int8_t* qkv;        // [B, H, W, 3, heads, 64] codes
  const float* qkv_bias;    // [3 * C] f32 or null (pad tokens)
  const float* relh;        // [2S-1, 64] f32
  const float* relw;        // [2S-1, 64] f32
  int8_t* out;              // [B, H, W, C] codes
  int B, H, W, heads, C, S, window, nwh, nww, L;
  const _Float16* v16;      // optional [B, H, W, C] fp16 copy of the V codes (samq_w8a8_gemm_v16)
  int row0;                 // row range (round 6, samq_rel_attention_q8_rows): global -- first query grid
                            // row (grid z = rows); windows -- first window row (nwh = the range's rows)
  float qk_scale, s_qkv, s_a1, s_a2, s_out;
  float inv_a1, inv_a2, k2;   // 1/s_a1, 1/s_a2, s_a2*log2(e)
};

typedef int int4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float aq8(float v, float s) {
  return q8_exact(v, s, 1.0f / s);   // s is a kernel argument: the reciprocal is hoisted
}

constexpr int QD = 64;       // head dim (vit_b)

__device__ __forceinline__ float q8max3(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }
constexpr int KPITCH = 80;   // K row pitch in LDS (bytes) of the generic kernel (the row64 / window kernels use 96)

// ROW64: global attention over a 64-wide grid -- a 64-key chunk is exactly one key row, so the
// height term is one value per chunk and the width term a fixed per-lane set (registers).
template <bool RESIDENT, int NWQ, int KC, int MAXS, bool ROW64 = false>
__global__ __launch_bounds__(64 * NWQ) void rel_attention_q8_kernel(AttnQ8Params p) {
  constexpr int NBUF = RESIDENT ? 1 : 2;
  constexpr int VTP = KC + 8;                    // V^T row pitch (halves)
  __shared__ __attribute__((aligned(16))) int8_t k_lds[NBUF][KC * KPITCH];
  __shared__ __attribute__((aligned(16))) _Float16 vt_lds[NBUF][QD * VTP];
  __shared__ __attribute__((aligned(16))) int8_t q_lds[NWQ][16 * KPITCH];
  __shared__ float rh_lds[NWQ][16 * (MAXS + 1)];
  __shared__ float rw_lds[NWQ][16 * (MAXS + 1)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int g = lane >> 4;
  const int ql = lane & 15;
  const int S = p.S, L = p.L, C = p.C;
  const int head = blockIdx.y;
  int b, wy = 0, wx = 0;
  if (p.window > 0) {
    const int per = p.nwh * p.nww;
    b = blockIdx.x / per;
    wy = p.row0 + (blockIdx.x % per) / p.nww;
    wx = blockIdx.x % p.nww;
  } else {
    b = blockIdx.x;
  }
  const float invS = 1.0f / (float)S;

  // local token index -> (row, col) in the window / grid and validity in the image
  auto tok = [&](int t, int& ty, int& tx) {
    ty = (int)(((float)t + 0.5f) * invS);
    tx = t - ty * S;
  };
  auto tok_ptr = [&](int ty, int tx, bool& inimg) -> const int8_t* {
    const int y = wy * S + ty, x = wx * S + tx;
    inimg = y < p.H && x < p.W;
    return p.qkv + (((int64_t)b * p.H + y) * p.W + x) * (3 * C);
  };

  // ---- stage keys [c0, c0 + KC) of K (codes) and V^T (fp16) into buffer buf
  auto stage = [&](int c0, int buf) {
    for (int u = tid; u < KC * 4; u += 64 * NWQ) {
      const int key = u % KC, part = u / KC;
      const int kk = c0 + key;
      u32x4 kc = {0u, 0u, 0u, 0u}, vc = {0u, 0u, 0u, 0u};
      if (kk < L) {
        int ty, tx;
        tok(kk, ty, tx);
        bool inimg;
        const int8_t* tp = tok_ptr(ty, tx, inimg);
        if (inimg) {
          kc = *(const u32x4*)(tp + C + head * QD + part * 16);
          vc = *(const u32x4*)(tp + 2 * C + head * QD + part * 16);
        } else if (p.qkv_bias) {
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int kq = (int)aq8(p.qkv_bias[C + head * QD + part * 16 + e], p.s_qkv);
            const int vq = (int)aq8(p.qkv_bias[2 * C + head * QD + part * 16 + e], p.s_qkv);
            kc[e >> 2] |= ((uint32_t)kq & 0xFFu) << (8 * (e & 3));
            vc[e >> 2] |= ((uint32_t)vq & 0xFFu) << (8 * (e & 3));
          }
        }
      }
      *(u32x4*)(&k_lds[buf][key * KPITCH + part * 16]) = kc;
#pragma unroll
      for (int e = 0; e < 16; ++e)
        vt_lds[buf][(part * 16 + e) * VTP + key] = (_Float16)(float)(int8_t)((vc[e >> 2] >> (8 * (e & 3))) & 0xFFu);
    }
  };

  // ---- this wave's 16 queries: codes (B operand of S^T = K.Q^T) and the rel-pos terms
  const int q0 = blockIdx.z * (16 * NWQ) + wave * 16;
  const int qt = q0 + ql;
  int qy = 0, qx = 0;
  bool q_ok = false;
  int4v qfrag = {0, 0, 0, 0};
  if (qt < L) {
    tok(qt, qy, qx);
    bool inimg;
    const int8_t* tp = tok_ptr(qy, qx, inimg);
    q_ok = inimg;
    if (inimg) {
      qfrag = *(const int4v*)(tp + head * QD + g * 16);
    } else if (p.qkv_bias) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int qq = (int)aq8(p.qkv_bias[head * QD + g * 16 + e], p.s_qkv);
        qfrag[e >> 2] |= (qq & 0xFF) << (8 * (e & 3));
      }
    }
  }
  *(int4v*)(&q_lds[wave][ql * KPITCH + g * 16]) = qfrag;
  __builtin_amdgcn_s_waitcnt(0xC07F);
  {
    // rel_h[q][kh] = sum_d (code_q[d] * s_qkv) * Rh[qy - kh + S - 1][d];  rel_w likewise with Rw and
    // the same ROW index qy (quirk 1).  16 lanes share one table row.
    const int pairs = 16 * S;
    for (int pi = lane; pi < pairs; pi += 64) {
      const int qi = pi & 15, kk = pi >> 4;
      const int qtt = q0 + qi;
      int ty = 0, tx = 0;
      if (qtt < L) tok(qtt, ty, tx);
      const int ridx = ty - kk + S - 1;
      const float* th = p.relh + (int64_t)ridx * QD;
      const float* tw = p.relw + (int64_t)ridx * QD;
      float ah = 0.f, aw = 0.f;
#pragma unroll 1
      for (int d4 = 0; d4 < QD / 16; ++d4) {
        const u32x4 cw = *(const u32x4*)(&q_lds[wave][qi * KPITCH + d4 * 16]);
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) {
          const float4_t h4 = *(const float4_t*)(th + d4 * 16 + e4 * 4);
          const float4_t w4 = *(const float4_t*)(tw + d4 * 16 + e4 * 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float qf = (float)(int8_t)((cw[e4] >> (8 * e)) & 0xFFu) * p.s_qkv;
            ah = fmaf(qf, h4[e], ah);
            aw = fmaf(qf, w4[e], aw);
          }
        }
      }
      rh_lds[wave][qi * (MAXS + 1) + kk] = ah;
      rw_lds[wave][qi * (MAXS + 1) + kk] = aw;
    }
  }

  const int nchunks = (L + 63) / 64;
  float m = -INFINITY, lsum = 0.f;
  float4_t acc[QD / 16];
#pragma unroll
  for (int t = 0; t < QD / 16; ++t) acc[t] = float4_t{0.f, 0.f, 0.f, 0.f};
  const float* rhq = &rh_lds[wave][ql * (MAXS + 1)];
  const float* rwq = &rw_lds[wave][ql * (MAXS + 1)];
  float rwr[4][4];
  if constexpr (ROW64) {
    __builtin_amdgcn_s_waitcnt(0xC07F);   // this wave's rel terms are in LDS
#pragma unroll
    for (int bb = 0; bb < 4; ++bb)
#pragma unroll
      for (int i = 0; i < 4; ++i) rwr[bb][i] = rwq[bb * 16 + 4 * g + i];
  }
  // Score quantisers by reciprocal multiply: the pre-quantisation values already differ from the
  // reference's by fp32 summation order, so a correctly rounded division buys no parity here
  // (stage-level code agreement is tested, test_w8a8_stage_local_parity).
  const float inv1 = p.inv_a1, inv2 = p.inv_a2, sa1 = p.s_a1;

  if (RESIDENT) {
    for (int c0 = 0; c0 < L; c0 += KC) stage(c0, 0);   // KC >= L: one pass
  } else {
    stage(0, 0);
  }
  __syncthreads();

  for (int ch = 0; ch < nchunks; ++ch) {
    const int buf = RESIDENT ? 0 : (ch & 1);
    const int koff = RESIDENT ? ch * 64 : 0;             // key offset inside the staged buffer
    if (!RESIDENT && ch + 1 < nchunks) stage((ch + 1) * 64, buf ^ 1);
    // ---- S^T block scores
    float c2[4][4];
    float cmax = -INFINITY;
    float rh_row = 0.f;
    if constexpr (ROW64) rh_row = rhq[ch];
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
      const int4v kf = *(const int4v*)(&k_lds[buf][(koff + bb * 16 + ql) * KPITCH + g * 16]);
      const int4v z = {0, 0, 0, 0};
      const int4v st = __builtin_amdgcn_mfma_i32_16x16x64_i8(kf, qfrag, z, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float c;
        if constexpr (ROW64) {
          const float v = (float)st[i] * p.qk_scale;
          const float v1 = fminf(fmaxf(__builtin_rintf(v * inv1), -128.f), 127.f) * sa1;
          const float t = (v1 + rh_row) + rwr[bb][i];
          c = fminf(fmaxf(__builtin_rintf(t * inv2), -128.f), 127.f);
        } else {
          const int key = ch * 64 + bb * 16 + 4 * g + i;
          c = -INFINITY;
          if (key < L) {
            int kh, kw;
            tok(key, kh, kw);
            const float v = (float)st[i] * p.qk_scale;
            const float v1 = fminf(fmaxf(__builtin_rintf(v * inv1), -128.f), 127.f) * sa1;
            const float t = (v1 + rhq[kh]) + rwq[kw];
            c = fminf(fmaxf(__builtin_rintf(t * inv2), -128.f), 127.f);
          }
        }
        c2[bb][i] = c;
        cmax = fmaxf(cmax, c);
      }
    }
    cmax = max_rows4(cmax);
    if (cmax > m) {
      const float alpha = m == -INFINITY ? 0.f : exp2f((m - cmax) * p.k2);
      lsum *= alpha;
#pragma unroll
      for (int t = 0; t < QD / 16; ++t) acc[t] = acc[t] * alpha;
      m = cmax;
    }
    float (&pr)[4][4] = c2;   // probabilities overwrite the score codes in place
    // exp(s_a2 * (c - m)) with c, m integer codes (exact difference); exp2 of a pre-scaled
    // argument is within a few ulps of the reference's exp(x - max x)
#pragma unroll
    for (int bb = 0; bb < 4; ++bb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float pv = c2[bb][i] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f((c2[bb][i] - m) * p.k2);
        pr[bb][i] = pv;
        lsum += pv;
      }
    // ---- O^T += V^T . P^T  (two 32-key steps, P split hi + lo)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      half8_t bhi, blo;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float pv = pr[2 * s2 + (j >> 2)][j & 3];
        const _Float16 h = (_Float16)pv;
        bhi[j] = h;
        blo[j] = (_Float16)(pv - (float)h);
      }
#pragma unroll
      for (int t = 0; t < QD / 16; ++t) {
        const _Float16* vr = &vt_lds[buf][(t * 16 + ql) * VTP + koff + 32 * s2 + 4 * g];
        const half4_t a0 = *(const half4_t*)vr;
        const half4_t a1 = *(const half4_t*)(vr + 16);
        const half8_t af = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bhi, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, blo, acc[t], 0, 0, 0);
      }
    }
    if (!RESIDENT) __syncthreads();   // chunk ch+1 staged; everyone done reading buffer buf
  }

  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  if (q_ok) {
    int8_t* op = p.out + (((int64_t)b * p.H + (wy * S + qy)) * p.W + (wx * S + qx)) * C + head * QD;
#pragma unroll
    for (int t = 0; t < QD / 16; ++t) {
      uint32_t w = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float o = acc[t][i] / lsum * p.s_qkv;
        w |= ((uint32_t)(int)aq8(o, p.s_out) & 0xFFu) << (8 * i);
      }
      *(uint32_t*)(op + t * 16 + 4 * g) = w;
    }
  }
}


// rel_h / rel_w for the 16 queries of a wave that share the query grid row qy, by MFMA:
// rel[kk][q] = s_qkv * sum_d code_q[d] * R[qy - kk + side - 1][d], for the 16 key rows / columns
// kk = 16 bb + m of block bb (A operand row m = the table row of kk; B = the int8 query codes,
// exact in fp16); the f32 tables enter as fp16 hi + lo pairs (|R - hi - lo| <= 2^-22 |R|), so the
// sums carry fp32-level error like a scalar fp32 dot product (whose order differs from the
// reference's anyway).  Lane (ql, g) receives rel[16 bb + 4 g + i][query ql], i = 0..3.
__device__ __forceinline__ void q8_rel_block(const AttnQ8Params& p, const int8_t* qcodes_lane, int qy, int side,
                                             int bb, int lane, float4_t& rh4, float4_t& rw4) {
  const int ql = lane & 15, g = lane >> 4;
  int r = qy - (16 * bb + ql) + side - 1;      // table row of this lane's A row (kk = 16 bb + ql)
  r = r < 0 ? 0 : (r > 2 * side - 2 ? 2 * side - 2 : r);   // rows past the window: any valid row (masked)
  rh4 = float4_t{0.f, 0.f, 0.f, 0.f};
  rw4 = float4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < QD / 32; ++s) {
    const uint2 cw = *(const uint2*)(qcodes_lane + 32 * s + 8 * g);   // codes of query ql, dims 32s+8g..+7
    half8_t qb;
#pragma unroll
    for (int e = 0; e < 8; ++e) qb[e] = (_Float16)(float)(int8_t)((((e < 4) ? cw.x : cw.y) >> (8 * (e & 3))) & 0xFFu);
#pragma unroll
    for (int tab = 0; tab < 2; ++tab) {
      const float* src = (tab ? p.relw : p.relh) + (int64_t)r * QD + 32 * s + 8 * g;
      const float4_t x0 = *(const float4_t*)src, x1 = *(const float4_t*)(src + 4);
      half8_t hi, lo;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float x = e < 4 ? x0[e] : x1[e - 4];
        hi[e] = (_Float16)x;
        lo[e] = (_Float16)(x - (float)hi[e]);
      }
      float4_t& d = tab ? rw4 : rh4;
      d = __builtin_amdgcn_mfma_f32_16x16x32_f16(hi, qb, d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_16x16x32_f16(lo, qb, d, 0, 0, 0);
    }
  }
  rh4 = rh4 * p.s_qkv;
  rw4 = rw4 * p.s_qkv;
}

// ------------------------------------------------------------------ global, 64 x 64 grid (vit_b)
// The global blocks of the W8A8 vit_b encoder (4096 keys).  A workgroup = one query grid row
// (64 queries, 4 waves x 16); key row kh is chunk kh (64 keys): its K codes (int8) and V codes
// (converted once to fp16, row-major) go through a 2-deep LDS ring with 16-byte stores, the next
// chunk's global loads in flight under the current chunk's math.  Per chunk and wave:
//   S^T = K.Q^T on 4 x v_mfma_i32_16x16x64_i8 (exact int32; lane = query ql, keys 16bb+4g+i);
//   c = q8(q8(st * s_qkv^2 * scale, s_a1) * s_a1 + rel_h[kh] + rel_w[kw], s_a2): the two score
//       quantisers (reciprocal multiply, round-half-even, clamp) of fq_vit image_encoder.py:455-470
//       (rel_w indexed by the query ROW, quirk 1).  NOT bit-exact: the second argument is
//       evaluated as fma(code1, s_a1/s_a2, (rel_h + rel_w)/s_a2) -- pre-scaled terms in another
//       addition order than the reference's (code1*s_a1 + rel_h + rel_w)/s_a2 -- so a code can move
//       by one at a .5 tie; test_w8a8_stage_local_parity bounds that (all codes within +-1, at
//       most 1e-4 of them off by one);
//   online softmax on the integer codes, p = exp2(c * k2 - m * k2) (one fma + exp2);
//   O^T += V^T.P^T on 16x16x32 f16 MFMAs with P split hi + lo (|P - hi - lo| ~ 2^-22 |P|), V^T
//       fragments by ds_read_b64_tr_b16 from the row-major fp16 V; the softmax denominators come
//       from the same MFMAs against an all-ones operand (fp32 sums of the same hi + lo).
// Softmax numerator table (round 4): the score codes are integers and the lazy offset m is one of
// them, so P = exp2((c - m) k2) takes at most 256 + lazy distinct values, d = c - m in [-255, lazyc].
// Entry 256 + d holds P split as fp16 hi (low half) + lo (high half) -- the operands the P.V MFMAs
// take -- and entry 0 is P = 0 (a masked key: index max(int(-inf) + 256 - m, 0)), so a score costs
// one LDS read and half a v_perm instead of fma + exp2 + three conversions + a subtraction.
// P = exp2(fl(d k2)) (the table) vs exp2(fl(c k2 - fl(m k2))) (the direct form): last-bit
// differences of fp32 P, below the 2^-22 of the hi + lo split.
constexpr int PTAB = 512;
__device__ __forceinline__ int q8_ptab_lazy(float k2) {   // lazy offset threshold in codes
  return (int)fminf(floorf(8.0f / k2), 255.0f);
}
template <int NT>
__device__ __forceinline__ void q8_ptab_fill(uint32_t* ptab, float k2, int lazyc, int tid) {
  for (int i = tid; i <= 256 + lazyc; i += NT) {
    const float pv = i == 0 ? 0.0f : __builtin_amdgcn_exp2f((float)(i - 256) * k2);
    const _Float16 h = (_Float16)pv, l = (_Float16)(pv - (float)h);
    ptab[i] = (uint32_t)__builtin_bit_cast(uint16_t, h) | ((uint32_t)__builtin_bit_cast(uint16_t, l) << 16);
  }
}
// The window kernel's table (round 6): entry 528 + d holds P(d) for d = c - m in [-255, lazyc], entries
// 0 .. 272 hold 0 -- the masked slots carry the biased code MAG - 400, whose entry -400 - m + 528 is
// at most 256 for any offset m >= -128 -- so every score, masked or not, is one lookup
constexpr int PTABW_BASE = 528, PTABW = PTABW_BASE + 256;
template <int NT>
__device__ __forceinline__ void q8_ptabw_fill(uint32_t* ptab, float k2, int lazyc, int tid) {
  for (int i = tid; i <= PTABW_BASE + lazyc; i += NT) {
    const float pv = i < PTABW_BASE - 255 ? 0.0f : __builtin_amdgcn_exp2f((float)(i - PTABW_BASE) * k2);
    const _Float16 h = (_Float16)pv, l = (_Float16)(pv - (float)h);
    ptab[i] = (uint32_t)__builtin_bit_cast(uint16_t, h) | ((uint32_t)__builtin_bit_cast(uint16_t, l) << 16);
  }
}
// P^T fragments (hi, lo) of 8 scores from their table words (v_perm: two per pair of scores)
__device__ __forceinline__ void q8_ptab_unpack(const uint32_t (&w)[8], half8_t& bhi, half8_t& blo) {
  uint32_t hi[4], lo[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    hi[j] = __builtin_amdgcn_perm(w[2 * j + 1], w[2 * j], 0x05040100u);
    lo[j] = __builtin_amdgcn_perm(w[2 * j + 1], w[2 * j], 0x07060302u);
  }
  bhi = __builtin_bit_cast(half8_t, hi);
  blo = __builtin_bit_cast(half8_t, lo);
}

// V16 (round 6): V staged from the producer's fp16 copy (p.v16, two 16-byte pieces per thread and
// key row, no int8 -> fp16 conversion: 28 of the loop's 252 VALU per wave and key row).  Score codes
// (round 6): the second quantiser rounds by adding 1.5 * 2^23 (exact round-half-even for |x| < 2^22)
// and clamps in that biased form, so a code's P-table address is one v_lshl_add of its bits -- no
// float -> int conversion per score.
// LDS pitches (round 6, second pass): K rows at 96 bytes -- the ds_read_b128 fragment reads are then
// conflict-free in all four lane groups (at 80 bytes three lane pairs of every group shared a bank) --
// and V rows at 80 halves, which takes the tr reads of key quads 0 / 7 off the same banks (72 made
// every tr read 2-way); the query staging of the prologue aliases V buffer 1 (unused until the first
// key row's store, after the prologue barrier), so three workgroups still fit a CU.  Kernel 120.3 ->
// 118.5 us per vit_b launch, bit-identical (profiles/r6_w8a8_row64_variants.log; that log also holds
// the measured-slower speculative P-table reads and the LDS-free direct-from-L2 prototype).
template <int NWQ, bool V16 = false>
__global__ __launch_bounds__(64 * NWQ, 3) void rel_attention_q8_row64_kernel(AttnQ8Params p) {
  constexpr int G = 64, KC = 64;
  constexpr int KP = 96;                         // K row pitch (bytes)
  constexpr int VP = QD + 16;                    // V row pitch (halves)
  constexpr int NT = 64 * NWQ;
  constexpr int UNITS = KC * 4;                  // 16-byte pieces of one chunk's K (and of its V)
  static_assert(UNITS % NT == 0, "staging");
  constexpr int UPT = UNITS / NT;
  __shared__ __attribute__((aligned(16))) int8_t k_lds[2][KC * KP];
  __shared__ __attribute__((aligned(16))) _Float16 v_lds[2][KC * VP];
  int8_t(*q_lds)[16 * KP] = (int8_t(*)[16 * KP])(void*)&v_lds[1][0];   // prologue only
  static_assert(NWQ * 16 * KP <= KC * VP * 2, "query staging inside V buffer 1");
  __shared__ float rh_lds[NWQ][16 * (G + 1)];
  __shared__ uint32_t ptab[PTAB];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int g = lane >> 4;
  const int ql = lane & 15;
  const int C = p.C;
  const int head = blockIdx.y;
  const int b = blockIdx.x;
  const int qy = p.row0 + blockIdx.z;           // query grid row of this workgroup
  const int lazyc = q8_ptab_lazy(p.k2);
  q8_ptab_fill<NT>(ptab, p.k2, lazyc, tid);     // visible after the first barrier below
  const int qx = wave * 16 + ql;
  const int64_t ts = 3 * (int64_t)C;
  const int8_t* img = p.qkv + (int64_t)b * G * G * ts;

  // ---- K / V staging: piece u = key * 4 + part (16 bytes of dims 16 part .. +15).  Two register
  // sets: chunk ch + 2 is loaded while chunk ch is computed and chunk ch + 1 (loaded one chunk
  // earlier) is stored -- two chunks of math to cover each load's latency
  u32x4 kreg[2][UPT], vreg[2][V16 ? 2 * UPT : UPT];
  const _Float16* v16img = V16 ? p.v16 + (int64_t)b * G * G * C : nullptr;
  auto load = [&](int kh, int r) {
#pragma unroll
    for (int j = 0; j < UPT; ++j) {
      const int u = tid + j * NT, key = u >> 2, part = u & 3;
      const int8_t* tp = img + ((int64_t)kh * G + key) * ts + head * QD + part * 16;
      kreg[r][j] = *(const u32x4*)(tp + C);
      if constexpr (V16) {
        const _Float16* vp = v16img + ((int64_t)kh * G + key) * C + head * QD + part * 16;
        vreg[r][2 * j] = *(const u32x4*)vp;
        vreg[r][2 * j + 1] = *(const u32x4*)(vp + 8);
      } else {
        vreg[r][j] = *(const u32x4*)(tp + 2 * C);
      }
    }
  };
  auto store = [&](int buf, int r) {
#pragma unroll
    for (int j = 0; j < UPT; ++j) {
      const int u = tid + j * NT, key = u >> 2, part = u & 3;
      *(u32x4*)(&k_lds[buf][key * KP + part * 16]) = kreg[r][j];
      if constexpr (V16) {
        *(u32x4*)(&v_lds[buf][key * VP + part * 16]) = vreg[r][2 * j];
        *(u32x4*)(&v_lds[buf][key * VP + part * 16 + 8]) = vreg[r][2 * j + 1];
      } else {
        half8_t h0, h1;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          h0[e] = (_Float16)(float)(int8_t)((vreg[r][j][e >> 2] >> (8 * (e & 3))) & 0xFFu);
          h1[e] = (_Float16)(float)(int8_t)((vreg[r][j][2 + (e >> 2)] >> (8 * (e & 3))) & 0xFFu);
        }
        *(half8_t*)(&v_lds[buf][key * VP + part * 16]) = h0;
        *(half8_t*)(&v_lds[buf][key * VP + part * 16 + 8]) = h1;
      }
    }
  };
  load(0, 0);
  load(1, 1);

  // ---- this wave's 16 queries (codes) and their rel-pos terms: fp32 dot products of the
  // fake-quant q with the f32 tables (rows qy - k + 63 for both, quirk 1).  Lane (g, ql) computes
  // the terms of query ql at k = 16 bb + 4 g + i: rel_w straight into the registers the score loop
  // reads, rel_h into LDS (one value per key row per chunk); no rel_w table in LDS, so three
  // workgroups fit a CU (the 768 workgroups of a vit_b launch are then all resident at once).
  const int4v qfrag = *(const int4v*)(img + ((int64_t)qy * G + qx) * ts + head * QD + g * 16);
  *(int4v*)(&q_lds[wave][ql * KP + g * 16]) = qfrag;
  __builtin_amdgcn_s_waitcnt(0xC07F);
  float rwr[4][4];
#pragma unroll
  for (int bb = 0; bb < 4; ++bb) {
    float4_t rh4, rw4;
    q8_rel_block(p, &q_lds[wave][ql * KP], qy, G, bb, lane, rh4, rw4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      rh_lds[wave][ql * (G + 1) + 16 * bb + 4 * g + i] = rh4[i];
      rwr[bb][i] = rw4[i];
    }
  }
  store(0, 0);
  __syncthreads();   // chunk 0 staged; the rel_h rows visible
  const float* rhq = &rh_lds[wave][ql * (G + 1)];

  // second quantiser argument (v1 + rel_h + rel_w) / s_a2 as fma(code1, s_a1 / s_a2, (rel_h + rel_w) /
  // s_a2): 8 instead of 10 VALU per score (reciprocal-multiply quantisers: see rel_attention_q8_kernel)
  const float c1 = p.qk_scale * p.inv_a1, inv2 = p.inv_a2, k2 = p.k2, k12 = p.s_a1 * p.inv_a2;
#pragma unroll
  for (int bb = 0; bb < 4; ++bb)
#pragma unroll
    for (int i = 0; i < 4; ++i) rwr[bb][i] *= inv2;
  // lazy softmax offset: m moves only when a code exceeds it by more than lazyc = 8 / k2 codes
  // (P <= 2^8, far inside fp16; O and l carry the same offset) -- most chunks then skip the O / l
  // rescale; P comes from the table (ptab, d = c - m <= lazyc)
  const float lazy = (float)lazyc;
  const int trow = ql >> 2, tcol = 4 * (ql & 3);
  const half8_t ones = {1, 1, 1, 1, 1, 1, 1, 1};
  // score codes in the biased form y = MAG + c (MAG = 1.5 * 2^23: the add rounds half-even, the
  // bits of y are MAGB + c); m is kept in the same form
  constexpr float MAG = 12582912.0f;
  constexpr int MAGB = 0x4B400000;
  float m = -INFINITY;
  // LDS byte address of the P-table entry of code y: (bits(y) << 2) + tbase, tbase = ptab + 4 (256 -
  // m_code - MAGB) (mod 2^32)
  uint32_t tbase = 0;
  const uint32_t ptab_addr = (uint32_t)(uintptr_t)(SAMQ_LDS void*)ptab;
  float4_t acc[QD / 16], lacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < QD / 16; ++t) acc[t] = float4_t{0.f, 0.f, 0.f, 0.f};

#pragma unroll 2
  for (int ch = 0; ch < G; ++ch) {
    const int buf = ch & 1;
    load(ch + 2 < G ? ch + 2 : G - 1, buf);      // register set of chunk ch (stored one chunk ago);
                                                // unconditional (clamped) so the waits stay counted
    // ---- scores -> two quantisers -> integer codes, biased (y = MAG + c)
    const float rh_row = rhq[ch] * inv2;
    float c[4][4];
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
      const int4v kf = *(const int4v*)(&k_lds[buf][(bb * 16 + ql) * KP + g * 16]);
      const int4v z = {0, 0, 0, 0};
      const int4v st = __builtin_amdgcn_mfma_i32_16x16x64_i8(kf, qfrag, z, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float q1 = __builtin_amdgcn_fmed3f(__builtin_rintf((float)st[i] * c1), -128.f, 127.f);
        c[bb][i] = __builtin_amdgcn_fmed3f(fmaf(q1, k12, rh_row + rwr[bb][i]) + MAG, MAG - 128.f, MAG + 127.f);
      }
    }
    float cmax = q8max3(c[0][0], c[0][1], c[0][2]);
    cmax = q8max3(cmax, c[0][3], c[1][0]);
    cmax = q8max3(cmax, c[1][1], c[1][2]);
    cmax = q8max3(cmax, c[1][3], c[2][0]);
    cmax = q8max3(cmax, c[2][1], c[2][2]);
    cmax = q8max3(cmax, c[2][3], c[3][0]);
    cmax = q8max3(cmax, c[3][1], c[3][2]);
    cmax = fmaxf(cmax, c[3][3]);
    cmax = max_rows4(cmax);
    if (cmax > m + lazy) {   // per query column: move the offset, rescale O and l
      const float alpha = m == -INFINITY ? 0.f : __builtin_amdgcn_exp2f((m - cmax) * k2);
#pragma unroll
      for (int t = 0; t < QD / 16; ++t) acc[t] = acc[t] * alpha;
      lacc = lacc * alpha;
      m = cmax;
      tbase = ptab_addr + 4u * (uint32_t)(256 - (__builtin_bit_cast(int, cmax) - MAGB) - MAGB);
    }
    // ---- P (hi + lo fp16, from the table) and O^T += V^T.P^T, l += ones.P^T, two 32-key steps
    uint32_t pw[2][8];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t a = ((uint32_t)__builtin_bit_cast(int, c[j >> 2][j & 3]) << 2) + tbase;
      pw[j >> 3][j & 7] = *(const SAMQ_LDS uint32_t*)(uintptr_t)a;
    }
    const _Float16* vb = &v_lds[buf][0];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      half8_t bhi, blo;
      q8_ptab_unpack(pw[s2], bhi, blo);
#pragma unroll
      for (int t = 0; t < QD / 16; ++t) {
        const _Float16* a0 = vb + (32 * s2 + 4 * g + trow) * VP + t * 16 + tcol;
        const half4_t lo = __builtin_bit_cast(half4_t, __builtin_amdgcn_ds_read_tr16_b64_v4i16((SAMQ_LDS short4_t*)a0));
        const half4_t hi = __builtin_bit_cast(
            half4_t, __builtin_amdgcn_ds_read_tr16_b64_v4i16((SAMQ_LDS short4_t*)(a0 + 16 * VP)));
        const half8_t af = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bhi, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, blo, acc[t], 0, 0, 0);
      }
      lacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ones, bhi, lacc, 0, 0, 0);
      lacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ones, blo, lacc, 0, 0, 0);
    }
    store(buf ^ 1, buf ^ 1);                    // chunk ch + 1 (register set (ch + 1) & 1; the last is a dummy); the other
    __syncthreads();                            // buffer was last read before the previous barrier
  }

  const float lsum = lacc[0];
  int8_t* op = p.out + (((int64_t)b * G + qy) * G + qx) * C + head * QD;
#pragma unroll
  for (int t = 0; t < QD / 16; ++t) {
    uint32_t w = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float o = acc[t][i] / lsum * p.s_qkv;
      w |= ((uint32_t)(int)aq8(o, p.s_out) & 0xFFu) << (8 * i);
    }
    *(uint32_t*)(op + t * 16 + 4 * g) = w;
  }
}

// ------------------------------------------------------------------ windows (S <= 16), key rows of 16 slots
// The windowed blocks of the W8A8 encoder (14 x 14 windows).  A workgroup = one (window, head), one
// wave per query row (16 slots, query (wave, ql), slots ql >= S idle), so the rel-pos terms of a
// wave are one MFMA block (q8_rel_block).  The keys are staged once with key
// (kh, kw) in slot 16 kh + kw (slots kw >= S zero and masked), so a 16-key block is exactly one key
// row: the height term is one value per block and the width term a fixed per-lane set (kw = 4 g + i,
// registers) -- per score no index decode and no table reads, unlike the generic path above.
// Scores, quantisers, softmax and P.V (hi + lo fp16, tr-read V, MFMA row sums) as the row64 kernel.
// NWQ < SW (round 5): a workgroup takes NWQ of the window's SW query rows (blockIdx.z = which NWQ),
// each staging the whole window's K / V: 14 x 14 windows of vit_b at B = 1 are 300 (window, head)
// items on 256 CUs, so 44 CUs ran two whole items one after the other; as 600 half-items of 7 waves
// the load spreads as ~2.3 half-items per CU.
template <int SW, int NWQ = SW>
// two workgroups per CU: LDS <= 80 KiB and (HIP's second bound = waves per SIMD) <= 512 / (waves / 2) VGPRs
__global__ __launch_bounds__(64 * NWQ, (2 * NWQ + 3) / 4) void rel_attention_q8_win_kernel(AttnQ8Params p) {
  constexpr int SLOTS = 16 * SW, KP = 96, VP = QD + 16;   // conflict-free pitches: see the row64 kernel
  static_assert(SW % NWQ == 0, "query rows split evenly");
  constexpr int NCH = (SW + 3) / 4;                        // chunks of up to 4 key rows (64 slots)
  static_assert(SW <= 16, "one window per workgroup");
  __shared__ __attribute__((aligned(16))) int8_t k_lds[SLOTS * KP];
  __shared__ __attribute__((aligned(16))) _Float16 v_lds[SLOTS * VP];
  __shared__ __attribute__((aligned(16))) int8_t q_lds[NWQ][16 * KP];
  __shared__ float rh_lds[NWQ][16 * (SW + 1)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int g = lane >> 4;
  const int ql = lane & 15;
  const int C = p.C;
  const int head = blockIdx.y;
  const int per = p.nwh * p.nww;
  const int b = blockIdx.x / per;
  const int wy = p.row0 + (blockIdx.x % per) / p.nww;
  const int wx = blockIdx.x % p.nww;
  auto tok_ptr = [&](int ty, int tx, bool& inimg) -> const int8_t* {
    const int y = wy * SW + ty, x = wx * SW + tx;
    inimg = y < p.H && x < p.W;
    return p.qkv + (((int64_t)b * p.H + y) * p.W + x) * (3 * C);
  };

  // ---- stage K codes and V (fp16, row-major) of every key slot; pad tokens = q8(qkv bias)
  for (int u = tid; u < SLOTS * 4; u += 64 * NWQ) {
    const int slot = u >> 2, part = u & 3;
    const int kh = slot >> 4, kw = slot & 15;
    u32x4 kc = {0u, 0u, 0u, 0u}, vc = {0u, 0u, 0u, 0u};
    if (kh < SW && kw < SW) {
      bool inimg;
      const int8_t* tp = tok_ptr(kh, kw, inimg);
      if (inimg) {
        kc = *(const u32x4*)(tp + C + head * QD + part * 16);
        vc = *(const u32x4*)(tp + 2 * C + head * QD + part * 16);
      } else if (p.qkv_bias) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int kq = (int)aq8(p.qkv_bias[C + head * QD + part * 16 + e], p.s_qkv);
          const int vq = (int)aq8(p.qkv_bias[2 * C + head * QD + part * 16 + e], p.s_qkv);
          kc[e >> 2] |= ((uint32_t)kq & 0xFFu) << (8 * (e & 3));
          vc[e >> 2] |= ((uint32_t)vq & 0xFFu) << (8 * (e & 3));
        }
      }
    }
    *(u32x4*)(&k_lds[slot * KP + part * 16]) = kc;
    half8_t h0, h1;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      h0[e] = (_Float16)(float)(int8_t)((vc[e >> 2] >> (8 * (e & 3))) & 0xFFu);
      h1[e] = (_Float16)(float)(int8_t)((vc[2 + (e >> 2)] >> (8 * (e & 3))) & 0xFFu);
    }
    *(half8_t*)(&v_lds[slot * VP + part * 16]) = h0;
    *(half8_t*)(&v_lds[slot * VP + part * 16 + 8]) = h1;
  }

  // ---- this wave's query row qy = wave (queries qx = ql < S) and its rel-pos terms (MFMA, rows
  // qy - k + S - 1 for both tables: quirk 1); rel_w for kw = 4 g + i into registers
  const bool q_in = ql < SW;
  const int qy = blockIdx.z * NWQ + wave, qx = q_in ? ql : 0;
  bool q_ok = false;
  int4v qfrag = {0, 0, 0, 0};
  if (q_in) {
    const int8_t* tp = tok_ptr(qy, qx, q_ok);
    if (q_ok) {
      qfrag = *(const int4v*)(tp + head * QD + g * 16);
    } else if (p.qkv_bias) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int qq = (int)aq8(p.qkv_bias[head * QD + g * 16 + e], p.s_qkv);
        qfrag[e >> 2] |= (qq & 0xFF) << (8 * (e & 3));
      }
    }
  }
  *(int4v*)(&q_lds[wave][ql * KP + g * 16]) = qfrag;
  __builtin_amdgcn_s_waitcnt(0xC07F);
  float rwr[4];
  {
    float4_t rh4, rw4;
    q8_rel_block(p, &q_lds[wave][ql * KP], qy, SW, 0, lane, rh4, rw4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      rwr[i] = rw4[i];
      if (4 * g + i < SW) rh_lds[wave][ql * (SW + 1) + 4 * g + i] = rh4[i];
    }
  }
  __syncthreads();   // K / V staged; this wave's rel_h rows visible; q_lds read for the last time
  // the P table (q8_ptab_fill) in q_lds's bytes: the two workgroups per CU leave no room for it
  static_assert(sizeof(q_lds) >= PTABW * 4, "P table alias");
  uint32_t* ptab = (uint32_t*)&q_lds[0][0];
  const int lazyc = q8_ptab_lazy(p.k2);
  q8_ptabw_fill<64 * NWQ>(ptab, p.k2, lazyc, tid);
  __syncthreads();
  const float* rhq = &rh_lds[wave][ql * (SW + 1)];

  const float c1 = p.qk_scale * p.inv_a1, inv2 = p.inv_a2, k2 = p.k2, k12 = p.s_a1 * p.inv_a2;
#pragma unroll
  for (int i = 0; i < 4; ++i) rwr[i] *= inv2;   // see the row64 kernel
  const float lazy = (float)lazyc;
  // biased score codes y = MAG + c as in the row64 kernel; masked slots MAG - 400 (table above)
  constexpr float MAG = 12582912.0f, MASKC = MAG - 400.f;
  constexpr int MAGB = 0x4B400000;
  uint32_t tbase = 0;
  const uint32_t ptab_addr = (uint32_t)(uintptr_t)(SAMQ_LDS void*)ptab;
  const int trow = ql >> 2, tcol = 4 * (ql & 3);
  const half8_t ones = {1, 1, 1, 1, 1, 1, 1, 1};
  float m = -INFINITY;
  float4_t acc[QD / 16], lacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < QD / 16; ++t) acc[t] = float4_t{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    constexpr int dummy = 0;
    (void)dummy;
    const int nb = SW - 4 * ch < 4 ? SW - 4 * ch : 4;   // key rows in this chunk (compile-time after unroll)
    float c[4][4];
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
      if (bb >= nb) {
#pragma unroll
        for (int i = 0; i < 4; ++i) c[bb][i] = MASKC;
        continue;
      }
      const int kh = 4 * ch + bb;
      const float rh_row = rhq[kh] * inv2;
      const int4v kf = *(const int4v*)(&k_lds[(kh * 16 + ql) * KP + g * 16]);
      const int4v z = {0, 0, 0, 0};
      const int4v st = __builtin_amdgcn_mfma_i32_16x16x64_i8(kf, qfrag, z, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float q1 = __builtin_amdgcn_fmed3f(__builtin_rintf((float)st[i] * c1), -128.f, 127.f);
        const float cq = __builtin_amdgcn_fmed3f(fmaf(q1, k12, rh_row + rwr[i]) + MAG, MAG - 128.f, MAG + 127.f);
        c[bb][i] = 4 * g + i < SW ? cq : MASKC;
      }
    }
    float cmax = q8max3(c[0][0], c[0][1], c[0][2]);
    cmax = q8max3(cmax, c[0][3], c[1][0]);
    cmax = q8max3(cmax, c[1][1], c[1][2]);
    cmax = q8max3(cmax, c[1][3], c[2][0]);
    cmax = q8max3(cmax, c[2][1], c[2][2]);
    cmax = q8max3(cmax, c[2][3], c[3][0]);
    cmax = q8max3(cmax, c[3][1], c[3][2]);
    cmax = fmaxf(cmax, c[3][3]);
    cmax = max_rows4(cmax);
    if (cmax > m + lazy) {
      const float alpha = m == -INFINITY ? 0.f : __builtin_amdgcn_exp2f((m - cmax) * k2);
#pragma unroll
      for (int t = 0; t < QD / 16; ++t) acc[t] = acc[t] * alpha;
      lacc = lacc * alpha;
      m = cmax;
      tbase = ptab_addr + 4u * (uint32_t)(PTABW_BASE - (__builtin_bit_cast(int, cmax) - MAGB) - MAGB);
    }
    const _Float16* vb = &v_lds[(ch * 64) * VP];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      if (2 * s2 >= nb) continue;   // both key rows of this k32 step are past the window
      half8_t bhi, blo;
      uint32_t pw[8];   // masked keys (MASKC): an entry below 273, P = 0
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t a = ((uint32_t)__builtin_bit_cast(int, c[2 * s2 + (j >> 2)][j & 3]) << 2) + tbase;
        pw[j] = *(const SAMQ_LDS uint32_t*)(uintptr_t)a;
      }
      q8_ptab_unpack(pw, bhi, blo);
#pragma unroll
      for (int t = 0; t < QD / 16; ++t) {
        const _Float16* a0 = vb + (32 * s2 + 4 * g + trow) * VP + t * 16 + tcol;
        const half4_t lo = __builtin_bit_cast(half4_t, __builtin_amdgcn_ds_read_tr16_b64_v4i16((SAMQ_LDS short4_t*)a0));
        const half4_t hi = __builtin_bit_cast(
            half4_t, __builtin_amdgcn_ds_read_tr16_b64_v4i16((SAMQ_LDS short4_t*)(a0 + 16 * VP)));
        const half8_t af = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bhi, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, blo, acc[t], 0, 0, 0);
      }
      lacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ones, bhi, lacc, 0, 0, 0);
      lacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ones, blo, lacc, 0, 0, 0);
    }
  }

  if (q_ok) {
    const float lsum = lacc[0];
    int8_t* op = p.out + (((int64_t)b * p.H + (wy * SW + qy)) * p.W + (wx * SW + qx)) * C + head * QD;
#pragma unroll
    for (int t = 0; t < QD / 16; ++t) {
      uint32_t w = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float o = acc[t][i] / lsum * p.s_qkv;
        w |= ((uint32_t)(int)aq8(o, p.s_out) & 0xFFu) << (8 * i);
      }
      *(uint32_t*)(op + t * 16 + 4 * g) = w;
    }
  }
}

}  // namespace samq

using namespace samq;

extern "C" int samq_rel_attention_q8_rows(const int8_t* qkv, const float* qkv_bias, const float* rel_pos_h,
                                          const float* rel_pos_w, int8_t* out, int B, int H, int W, int heads,
                                          int hd, int window, float sm_scale, float s_qkv, float s_a1, float s_a2,
                                          float s_out, int row0, int rows, const void* v16, hipStream_t stream) {
  if (B == 0) return SAMQ_OK;   // empty batch: no work, data pointers may be null
  SAMQ_REQUIRE(qkv && rel_pos_h && rel_pos_w && out, SAMQ_ERR_INVALID, "rel_attention_q8: null pointer");
  SAMQ_REQUIRE(hd == QD, SAMQ_ERR_UNSUPPORTED, "rel_attention_q8: head_dim must be 64");
  SAMQ_REQUIRE(B > 0 && H > 0 && W > 0 && heads > 0, SAMQ_ERR_INVALID, "rel_attention_q8: bad shape");
  SAMQ_REQUIRE(s_qkv > 0.f && s_a1 > 0.f && s_a2 > 0.f && s_out > 0.f, SAMQ_ERR_INVALID,
               "rel_attention_q8: scales must be > 0");
  SAMQ_REQUIRE(((uintptr_t)qkv & 15) == 0 && ((uintptr_t)out & 3) == 0, SAMQ_ERR_INVALID,
               "rel_attention_q8: qkv must be 16-byte aligned");
  if (rows < 0) { row0 = 0; rows = H; }   // the whole grid
  SAMQ_REQUIRE(row0 >= 0 && rows > 0 && row0 + rows <= H, SAMQ_ERR_INVALID, "rel_attention_q8: bad row range");
  SAMQ_REQUIRE(window > 0 ? (row0 % window == 0 && (rows % window == 0 || row0 + rows == H))
                          : (rows == H || H == 64), SAMQ_ERR_UNSUPPORTED,
               "rel_attention_q8: a row range must cover whole windows (global: the 64 x 64 grid only)");
  SAMQ_REQUIRE(((uintptr_t)v16 & 15) == 0, SAMQ_ERR_INVALID, "rel_attention_q8: v16 must be 16-byte aligned");
  AttnQ8Params p{};
  p.qkv = qkv; p.qkv_bias = qkv_bias; p.relh = rel_pos_h; p.relw = rel_pos_w; p.out = out;
  p.v16 = (const _Float16*)v16;
  p.B = B; p.H = H; p.W = W; p.heads = heads; p.C = heads * hd;
  // (q * scale) . k with q = c_q * s_qkv, k = c_k * s_qkv  (fq_vit image_encoder.py:455)
  p.qk_scale = (s_qkv * sm_scale) * s_qkv;
  p.s_qkv = s_qkv; p.s_a1 = s_a1; p.s_a2 = s_a2; p.s_out = s_out;
  p.inv_a1 = 1.0f / s_a1; p.inv_a2 = 1.0f / s_a2; p.k2 = s_a2 * 1.4426950408889634f;
  if (window > 0) {
    SAMQ_REQUIRE(window <= 16, SAMQ_ERR_UNSUPPORTED, "rel_attention_q8: window must be <= 16");
    p.S = window; p.window = window;
    p.nwh = (rows + window - 1) / window; p.nww = (W + window - 1) / window;
    p.row0 = row0 / window;
    p.L = window * window;
    const dim3 grid(B * p.nwh * p.nww, heads, 1);
    if (window == 14) {   // SAM's 14 x 14 windows: key and query rows of 16 slots, half a window per workgroup
      const dim3 grid2(B * p.nwh * p.nww, heads, 2);
      hipLaunchKernelGGL((rel_attention_q8_win_kernel<14, 7>), grid2, dim3(64 * 7), 0, stream, p);
    }
    else if (p.L <= 13 * 16)
      hipLaunchKernelGGL((rel_attention_q8_kernel<true, 13, 256, 16>), grid, dim3(64 * 13), 0, stream, p);
    else
      hipLaunchKernelGGL((rel_attention_q8_kernel<true, 16, 256, 16>), grid, dim3(64 * 16), 0, stream, p);
  } else {
    SAMQ_REQUIRE(H == W && H <= 64, SAMQ_ERR_UNSUPPORTED, "rel_attention_q8: global attention needs H == W <= 64");
    p.S = H; p.window = 0; p.nwh = p.nww = 1; p.L = H * W;
    constexpr int NWQ = 4;
    const dim3 grid(B, heads, (p.L + 16 * NWQ - 1) / (16 * NWQ));
    p.row0 = row0;
    if (H == 64)   // one grid row of queries per workgroup (16 * NWQ == 64)
    {
      if (v16) hipLaunchKernelGGL((rel_attention_q8_row64_kernel<NWQ, true>), dim3(B, heads, rows), dim3(64 * NWQ), 0, stream, p);
      else hipLaunchKernelGGL((rel_attention_q8_row64_kernel<NWQ>), dim3(B, heads, rows), dim3(64 * NWQ), 0, stream, p);
    }
    else
      hipLaunchKernelGGL((rel_attention_q8_kernel<false, NWQ, 64, 64, false>), grid, dim3(64 * NWQ), 0, stream, p);
  }
  SAMQ_LAUNCH_CHECK("rel_attention_q8 launch");
  return SAMQ_OK;
}

extern "C" int samq_rel_attention_q8(const int8_t* qkv, const float* qkv_bias, const float* rel_pos_h,
                                     const float* rel_pos_w, int8_t* out, int B, int H, int W, int heads, int hd,
                                     int window, float sm_scale, float s_qkv, float s_a1, float s_a2, float s_out,
                                     hipStream_t stream) {
  return samq_rel_attention_q8_rows(qkv, qkv_bias, rel_pos_h, rel_pos_w, out, B, H, W, heads, hd, window, sm_scale,
                                    s_qkv, s_a1, s_a2, s_out, 0, -1, nullptr, stream);
}

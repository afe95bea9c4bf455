// Fused multi-head attention BACKWARD (flash-style, recompute from the saved log-sum-exp) for the
// Cellpose-SAM ViT-L/8 training step (reference fine-tunes Cellpose-SAM,
// apps/cellpose-finetuning/main.py:1278-1713) including the gradient of SAM's decomposed
// relative-position bias (logit += rel_h[q, key_row] + rel_w[q, key_col]).  The N x N probability /
// score-gradient matrices never exist in HBM.
//
// Two kernels, both head_dim 64, bf16 operands, fp32 accumulation on v_mfma_f32_32x32x16_bf16:
//
//  * dq kernel (query-major, the forward's "swapped" shape): a lane owns one query column of
//    S^T = K Q^T and dP^T = V dO^T, recomputes P^T from the saved LSE, forms dS^T = P^T (dP^T - delta)
//    in registers and accumulates dQ^T += K^T dS^T with dS^T (converted to bf16) as the MFMA B operand
//    and K^T read transposed out of LDS (ds_read_b64_tr_b16).  Because a 32-key block of the 32-wide
//    SAM grid is exactly one grid row, drel_h[q, row] is a lane-local sum (+ one lane^32 exchange) and
//    drel_w[q, col] accumulates in 16 registers per lane across all key blocks -- no atomics.  It also
//    writes delta = rowsum(dO * O) for the key-major kernel.
//  * dkv kernel (key-major): a lane owns one KEY column of S = Q K^T and dP = dO V^T (its K and V
//    rows sit in registers for the whole kernel); the query tiles stream through LDS.  dV^T += dO^T P
//    and dK^T += Q^T dS with P / dS straight from the accumulators, dO^T / Q^T read transposed.
//
// Tiles are XOR-swizzled per 16-byte chunk (v_off: conflict-free transposed reads), and the next
// tile's global loads are register-staged while the current tile's MFMAs run.  Block ids are
// XCD-remapped so the blocks that stream the same (batch, head) K/V or Q/dO rows share an L2.
#include "common.h"

namespace {

constexpr int HD = 64;   // head dim
constexpr int TT = 64;   // streamed rows per LDS tile (keys in the dq kernel, queries in the dkv kernel)
constexpr float LOG2E = 1.4426950408889634f;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) short s16x4;

struct BwdArgs {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  long long s_tok, s_head, s_batch;  // element strides shared by q, k, v (packed qkv)
  const bf16_t* o;
  const bf16_t* dout;
  long long o_tok, o_head, o_batch;  // strides shared by o, dout and dq
  const float* lse;                  // [B*H, N] natural-log sum-exp of the logits (forward)
  float* delta;                      // [B*H, N] rowsum(dO * O), written by the dq kernel
  const float* relh;                 // [B*H, N, Hg] or null
  const float* relw;                 // [B*H, N, 32]
  int Hg;
  float* dq;                         // fp32, o strides (unscaled by nothing: final dQ)
  float* drelh;                      // [B*H, N, Hg]
  float* drelw;                      // [B*H, N, 32]
  bf16_t* dk;
  bf16_t* dv;
  long long d_tok, d_head, d_batch;  // strides shared by dk and dv
  int B, H, N;
  float scale;
  int blocks_per_bh;
  int write_delta;  // dq blocks store delta (two-launch path); the fused path gets it from attn_delta_kernel
};

__device__ __forceinline__ uint32_t cvt_pk_bf16(float lo, float hi) {
  uint32_t r;
  asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}

// chunk swizzles (16-byte chunks, 8 per 128-byte row); same layouts as attention.hip
__device__ __forceinline__ int k_off(int row, int ch) { return row * HD + ((ch ^ ((row >> 1) & 7)) << 3); }
__device__ __forceinline__ int v_off(int row, int ch) { return row * HD + ((ch ^ (((row >> 1) & 1) << 2)) << 3); }

// Transposed A operand X^T [32 head dims (db) x 16 rows (rb*32 + 16 st ...)] of a v_off-laid tile;
// the k order matches the B operand built from an accumulator by pack_b() below.
__device__ __forceinline__ bf16x8 read_tr(const bf16_t* X, int lane, int rb, int st, int db) {
  const int h = lane >> 5;
  const int g1 = (lane >> 4) & 1;
  const int qq = (lane & 15) >> 2, pp = lane & 3;
  const int ch = db * 4 + 2 * g1 + (pp >> 1);
  const int row0 = rb * 32 + 16 * st + 4 * h + qq;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(X + v_off(row0, ch) + 4 * (pp & 1)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(X + v_off(row0 + 8, ch) + 4 * (pp & 1)));
  bf16x8 f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return f;
}

// accumulator rows 16 st .. 16 st + 15 of a 32x32 block -> bf16 B operand (k = those rows)
__device__ __forceinline__ bf16x8 pack_b(const f32x16& s, int st) {
  u32x4 w;
  w[0] = cvt_pk_bf16(s[8 * st + 0], s[8 * st + 1]);
  w[1] = cvt_pk_bf16(s[8 * st + 2], s[8 * st + 3]);
  w[2] = cvt_pk_bf16(s[8 * st + 4], s[8 * st + 5]);
  w[3] = cvt_pk_bf16(s[8 * st + 6], s[8 * st + 7]);
  return *reinterpret_cast<bf16x8*>(&w);
}

__device__ __forceinline__ bf16x8 load_frag(const bf16_t* p, bool ok) {
  u32x4 r = ok ? *reinterpret_cast<const u32x4*>(p) : (u32x4){0u, 0u, 0u, 0u};
  return *reinterpret_cast<bf16x8*>(&r);
}

// ------------------------------------------------------------------ dQ (+ drel, delta)
template <int NW, int BIAS>
__device__ __forceinline__ void dq_body(const BwdArgs& a, int logical) {
  constexpr int NT = NW * 64;
  constexpr int CHUNKS = 2 * TT * (HD / 8);
  constexpr int CPT = (CHUNKS + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) bf16_t Ks[TT * HD];  // v_off: row reads + transposed reads
  __shared__ __attribute__((aligned(16))) bf16_t Vs[TT * HD];  // k_off: row reads

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, ql = lane & 31;
  const int bh = logical / a.blocks_per_bh, qb = logical % a.blocks_per_bh;
  const int b = bh / a.H, hh = bh % a.H;
  const int qi = qb * NW * 32 + wave * 32 + ql;
  const bool qv = qi < a.N;
  const int qc = min(qi, a.N - 1);

  const long long kvoff = (long long)b * a.s_batch + (long long)hh * a.s_head;
  const long long ooff = (long long)b * a.o_batch + (long long)hh * a.o_head + (long long)qc * a.o_tok;
  const bf16_t* kbase = a.k + kvoff;
  const bf16_t* vbase = a.v + kvoff;

  bf16x8 qf[4], df[4];
  float dl = 0.f;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    qf[ks] = load_frag(a.q + kvoff + (long long)qc * a.s_tok + ks * 16 + h * 8, qv);
    df[ks] = load_frag(a.dout + ooff + ks * 16 + h * 8, qv);
    const bf16x8 of = load_frag(a.o + ooff + ks * 16 + h * 8, qv);
#pragma unroll
    for (int j = 0; j < 8; ++j) dl += bf2f((uint16_t)df[ks][j]) * bf2f((uint16_t)of[j]);
  }
  dl += __shfl_xor(dl, 32, 64);
  if (qv && h == 0 && a.write_delta) a.delta[(long long)bh * a.N + qi] = dl;
  const float lse2 = qv ? a.lse[(long long)bh * a.N + qi] * LOG2E : 0.f;
  const float c2 = a.scale * LOG2E;

  const float* rh = nullptr;
  float rwr[16], drw[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) { rwr[i] = 0.f; drw[i] = 0.f; }
  if (BIAS) {
    rh = a.relh + ((long long)bh * a.N + qc) * a.Hg;
    const float* rw = a.relw + ((long long)bh * a.N + qc) * 32;
#pragma unroll
    for (int i = 0; i < 16; ++i) rwr[i] = rw[8 * (i >> 2) + 4 * h + (i & 3)] * LOG2E;
  }

  f32x16 dqa[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) { dqa[0][i] = 0.f; dqa[1][i] = 0.f; }

  const int ntiles = (a.N + TT - 1) / TT;
  u32x4 stage[CPT];
  auto issue = [&](int t) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + i * NT;
      u32x4 r = (u32x4){0u, 0u, 0u, 0u};
      if (c < CHUNKS) {
        const int isv = c >= CHUNKS / 2;
        const int cc = c - isv * (CHUNKS / 2);
        const int row = cc >> 3, ch = cc & 7;
        const int key = t * TT + row;
        if (key < a.N) r = *reinterpret_cast<const u32x4*>((isv ? vbase : kbase) + (long long)key * a.s_tok + ch * 8);
      }
      stage[i] = r;
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + i * NT;
      if (c < CHUNKS) {
        const int isv = c >= CHUNKS / 2;
        const int cc = c - isv * (CHUNKS / 2);
        const int row = cc >> 3, ch = cc & 7;
        if (isv)
          *reinterpret_cast<u32x4*>(Vs + k_off(row, ch)) = stage[i];
        else
          *reinterpret_cast<u32x4*>(Ks + v_off(row, ch)) = stage[i];
      }
    }
  };

  issue(0);
  for (int t = 0; t < ntiles; ++t) {
    __syncthreads();
    commit();
    __syncthreads();
    if (t + 1 < ntiles) issue(t + 1);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      f32x16 s, dp;
#pragma unroll
      for (int i = 0; i < 16; ++i) { s[i] = 0.f; dp[i] = 0.f; }
      const int row = kb * 32 + ql;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + v_off(row, 2 * ks + h));
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], s, 0, 0, 0);
        const bf16x8 vf = *reinterpret_cast<const bf16x8*>(Vs + k_off(row, 2 * ks + h));
        dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, df[ks], dp, 0, 0, 0);
      }
      const int krow = 2 * t + kb;  // grid row of this 32-key block (BIAS: Wg == 32)
      const float rhv = BIAS ? rh[min(krow, a.Hg - 1)] * LOG2E : 0.f;
      float dsum = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = t * TT + kb * 32 + 8 * (i >> 2) + 4 * h + (i & 3);
        const float x = s[i] * c2 + (BIAS ? rhv + rwr[i] : 0.f);
        const float p = (key < a.N && qv) ? __builtin_amdgcn_exp2f(x - lse2) : 0.f;
        const float ds = p * (dp[i] - dl);
        s[i] = ds;
        dsum += ds;
        drw[i] += ds;
      }
      if (BIAS) {
        dsum += __shfl_xor(dsum, 32, 64);
        if (qv && h == 0 && krow < a.Hg) a.drelh[((long long)bh * a.N + qi) * a.Hg + krow] = dsum;
      }
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf16x8 pf = pack_b(s, st);
#pragma unroll
        for (int db = 0; db < 2; ++db)
          dqa[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(read_tr(Ks, lane, kb, st, db), pf, dqa[db], 0, 0, 0);
      }
    }
  }

  if (qv) {
    float* dqr = a.dq + (long long)b * a.o_batch + (long long)hh * a.o_head + (long long)qi * a.o_tok;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float4 w;
        w.x = dqa[db][4 * g + 0] * a.scale;
        w.y = dqa[db][4 * g + 1] * a.scale;
        w.z = dqa[db][4 * g + 2] * a.scale;
        w.w = dqa[db][4 * g + 3] * a.scale;
        *reinterpret_cast<float4*>(dqr + db * 32 + 8 * g + 4 * h) = w;
      }
    if (BIAS) {
      float* dw = a.drelw + ((long long)bh * a.N + qi) * 32;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float4 w;
        w.x = drw[4 * g + 0]; w.y = drw[4 * g + 1]; w.z = drw[4 * g + 2]; w.w = drw[4 * g + 3];
        *reinterpret_cast<float4*>(dw + 8 * g + 4 * h) = w;
      }
    }
  }
}

// ------------------------------------------------------------------ dK, dV
template <int NW, int BIAS>
__device__ __forceinline__ void dkv_body(const BwdArgs& a, int logical) {
  constexpr int NT = NW * 64;
  constexpr int QCH = 2 * TT * (HD / 8);       // Q + dO tile chunks (bf16 x 8)
  constexpr int WCH = BIAS ? TT * 32 / 4 : 0;   // rel_w tile chunks (fp32 x 4)
  constexpr int HCH = BIAS ? TT : 0;             // rel_h: the block's NW grid rows, one chunk per query
  constexpr int SCH = TT / 4 * 2;               // lse2 + delta chunks
  constexpr int CHUNKS = QCH + WCH + HCH + SCH;
  constexpr int CPT = (CHUNKS + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) bf16_t Qs[TT * HD];
  __shared__ __attribute__((aligned(16))) bf16_t Ds[TT * HD];
  __shared__ __attribute__((aligned(16))) float Ws[BIAS ? TT * 32 : 4];
  __shared__ __attribute__((aligned(16))) float Hs[BIAS ? TT * 4 : 4];
  __shared__ __attribute__((aligned(16))) float L2s[TT];
  __shared__ __attribute__((aligned(16))) float DLs[TT];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, kl = lane & 31;
  const int bh = logical / a.blocks_per_bh, kblk = logical % a.blocks_per_bh;
  const int b = bh / a.H, hh = bh % a.H;
  const int k0 = kblk * NW * 32 + wave * 32;
  const int kj = k0 + kl;
  const bool kv = kj < a.N;
  const int kc = min(kj, a.N - 1);
  // BIAS: this wave's 32 keys are one grid row (Wg == 32), row kblk * NW + wave; key col = kl

  const long long kvoff = (long long)b * a.s_batch + (long long)hh * a.s_head;
  const bf16_t* qbase = a.q + kvoff;
  const bf16_t* dbase = a.dout + (long long)b * a.o_batch + (long long)hh * a.o_head;
  const float* lrow = a.lse + (long long)bh * a.N;
  const float* drow = a.delta + (long long)bh * a.N;

  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    kf[ks] = load_frag(a.k + kvoff + (long long)kc * a.s_tok + ks * 16 + h * 8, kv);
    vf[ks] = load_frag(a.v + kvoff + (long long)kc * a.s_tok + ks * 16 + h * 8, kv);
  }
  const float c2 = a.scale * LOG2E;

  f32x16 dva[2], dka[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) { dva[0][i] = 0.f; dva[1][i] = 0.f; dka[0][i] = 0.f; dka[1][i] = 0.f; }

  const int ntiles = (a.N + TT - 1) / TT;
  u32x4 stage[CPT];
  auto issue = [&](int t) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + i * NT;
      u32x4 r = (u32x4){0u, 0u, 0u, 0u};
      if (c < QCH) {
        const int isd = c >= QCH / 2;
        const int cc = c - isd * (QCH / 2);
        const int row = cc >> 3, ch = cc & 7;
        const int qq = t * TT + row;
        if (qq < a.N)
          r = *reinterpret_cast<const u32x4*>(isd ? dbase + (long long)qq * a.o_tok + ch * 8
                                                  : qbase + (long long)qq * a.s_tok + ch * 8);
      } else if (c < QCH + WCH) {  // rel_w, pre-scaled to log2 units
        const int cc = c - QCH;
        const int row = cc >> 3, c4 = cc & 7;
        const int qq = t * TT + row;
        if (qq < a.N) {
          const float4 f = *reinterpret_cast<const float4*>(a.relw + ((long long)bh * a.N + qq) * 32 + c4 * 4);
          r[0] = __float_as_uint(f.x * LOG2E); r[1] = __float_as_uint(f.y * LOG2E);
          r[2] = __float_as_uint(f.z * LOG2E); r[3] = __float_as_uint(f.w * LOG2E);
        }
      } else if (c < QCH + WCH + HCH) {  // rel_h of the block's grid rows minus the row's LSE (log2)
        const int qq = t * TT + (c - QCH - WCH);
        if (qq < a.N) {
          const float* hr = a.relh + ((long long)bh * a.N + qq) * a.Hg;
          const float l2 = lrow[qq] * LOG2E;
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const int gr = kblk * NW + w;
            r[w] = __float_as_uint(((w < NW && gr < a.Hg) ? hr[gr] * LOG2E : 0.f) - l2);
          }
        } else {  // padded query: P = 0
          r[0] = r[1] = r[2] = r[3] = __float_as_uint(-INFINITY);
        }
      } else if (c < CHUNKS) {
        const int cc = c - QCH - WCH - HCH;
        const int isd = cc >= TT / 4;
        const int q4 = (cc - isd * (TT / 4)) * 4;
        float f[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int qq = t * TT + q4 + j;
          // lse of a padded query = +inf -> P = 0; delta 0
          f[j] = qq < a.N ? (isd ? drow[qq] : lrow[qq] * LOG2E) : (isd ? 0.f : INFINITY);
        }
        r[0] = __float_as_uint(f[0]); r[1] = __float_as_uint(f[1]);
        r[2] = __float_as_uint(f[2]); r[3] = __float_as_uint(f[3]);
      }
      stage[i] = r;
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + i * NT;
      if (c < QCH) {
        const int isd = c >= QCH / 2;
        const int cc = c - isd * (QCH / 2);
        const int row = cc >> 3, ch = cc & 7;
        *reinterpret_cast<u32x4*>((isd ? Ds : Qs) + v_off(row, ch)) = stage[i];
      } else if (c < QCH + WCH) {
        const int cc = c - QCH;
        *reinterpret_cast<u32x4*>(Ws + cc * 4) = stage[i];
      } else if (c < QCH + WCH + HCH) {
        const int cc = c - QCH - WCH;
        *reinterpret_cast<u32x4*>(Hs + cc * 4) = stage[i];
      } else if (c < CHUNKS) {
        const int cc = c - QCH - WCH - HCH;
        const int isd = cc >= TT / 4;
        const int q4 = (cc - isd * (TT / 4)) * 4;
        *reinterpret_cast<u32x4*>((isd ? DLs : L2s) + q4) = stage[i];
      }
    }
  };

  issue(0);
  for (int t = 0; t < ntiles; ++t) {
    __syncthreads();
    commit();
    __syncthreads();
    if (t + 1 < ntiles) issue(t + 1);
#pragma unroll 1  // one 32-query half at a time: keeps dkv<4, 1> at 254 VGPRs without spills
    for (int qb = 0; qb < 2; ++qb) {
      f32x16 s, dp;
#pragma unroll
      for (int i = 0; i < 16; ++i) { s[i] = 0.f; dp[i] = 0.f; }
      const int row = qb * 32 + kl;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bf16x8 qa = *reinterpret_cast<const bf16x8*>(Qs + v_off(row, 2 * ks + h));
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kf[ks], s, 0, 0, 0);
        const bf16x8 da = *reinterpret_cast<const bf16x8*>(Ds + v_off(row, 2 * ks + h));
        dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, vf[ks], dp, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qr = qb * 32 + 8 * (i >> 2) + 4 * h + (i & 3);  // query row in the tile
        // BIAS: Hs holds rel_h * log2e - lse * log2e, Ws rel_w * log2e (folded at staging time)
        const float x = BIAS ? s[i] * c2 + (Hs[qr * 4 + wave] + Ws[qr * 32 + kl]) : s[i] * c2 - L2s[qr];
        const float p = kv ? __builtin_amdgcn_exp2f(x) : 0.f;
        s[i] = p;
        dp[i] = p * (dp[i] - DLs[qr]);
      }
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf16x8 pf = pack_b(s, st);
        const bf16x8 dsf = pack_b(dp, st);
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          dva[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(read_tr(Ds, lane, qb, st, db), pf, dva[db], 0, 0, 0);
          dka[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(read_tr(Qs, lane, qb, st, db), dsf, dka[db], 0, 0, 0);
        }
      }
    }
  }

  if (kv) {
    const long long doff = (long long)b * a.d_batch + (long long)hh * a.d_head + (long long)kj * a.d_tok;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u32x2 wv, wk;
        wv[0] = cvt_pk_bf16(dva[db][4 * g + 0], dva[db][4 * g + 1]);
        wv[1] = cvt_pk_bf16(dva[db][4 * g + 2], dva[db][4 * g + 3]);
        wk[0] = cvt_pk_bf16(dka[db][4 * g + 0] * a.scale, dka[db][4 * g + 1] * a.scale);
        wk[1] = cvt_pk_bf16(dka[db][4 * g + 2] * a.scale, dka[db][4 * g + 3] * a.scale);
        *reinterpret_cast<u32x2*>(a.dv + doff + db * 32 + 8 * g + 4 * h) = wv;
        *reinterpret_cast<u32x2*>(a.dk + doff + db * 32 + 8 * g + 4 * h) = wk;
      }
  }
}

// 4-wave blocks are register-capped to 256 VGPRs so TWO waves share each SIMD (the unconstrained
// build took 264 / 376 VGPRs -> one wave per SIMD, SQ_WAIT_ANY ~65 % of wave cycles in dkv).
#define BE_ATTN_BWD_WPE __attribute__((amdgpu_waves_per_eu(NW == 4 ? 2 : 1, NW == 4 ? 2 : 1)))

template <int NW, int BIAS>
__global__ __launch_bounds__(NW * 64) BE_ATTN_BWD_WPE void attn_bwd_dq_kernel(BwdArgs a) {
  dq_body<NW, BIAS>(a, xcd_remap(blockIdx.x, a.blocks_per_bh * a.B * a.H));
}

template <int NW, int BIAS>
__global__ __launch_bounds__(NW * 64) BE_ATTN_BWD_WPE void attn_bwd_dkv_kernel(BwdArgs a) {
  dkv_body<NW, BIAS>(a, xcd_remap(blockIdx.x, a.blocks_per_bh * a.B * a.H));
}

// Small grids (batch 1: 16 heads x 1024 tokens = 256 + 256 two-wave blocks): the dq and dkv blocks
// run as ONE launch (blocks [0, n) dq, [n, 2n) dkv) so both halves fill the 1024 SIMDs together;
// delta = rowsum(dO * O) comes from attn_delta_kernel first.
template <int NW, int BIAS>
__global__ __launch_bounds__(NW * 64) BE_ATTN_BWD_WPE void attn_bwd_fused_kernel(BwdArgs a) {
  const int n = a.blocks_per_bh * a.B * a.H;
  if ((int)blockIdx.x < n)
    dq_body<NW, BIAS>(a, xcd_remap(blockIdx.x, n));
  else
    dkv_body<NW, BIAS>(a, xcd_remap(blockIdx.x - n, n));
}

// delta[bh, q] = sum_c dO[b, q, h, c] O[b, q, h, c]: 8 lanes per row, 16-byte loads
__global__ __launch_bounds__(256) void attn_delta_kernel(BwdArgs a) {
  const long long row = (long long)blockIdx.x * 32 + (threadIdx.x >> 3);
  const int part = threadIdx.x & 7;
  const long long rows = (long long)a.B * a.H * a.N;
  float acc = 0.f;
  if (row < rows) {
    const int bh = (int)(row / a.N), q = (int)(row % a.N);
    const int b = bh / a.H, hh = bh % a.H;
    const long long off = (long long)b * a.o_batch + (long long)hh * a.o_head + (long long)q * a.o_tok + part * 8;
    const bf16x8 d = *reinterpret_cast<const bf16x8*>(a.dout + off);
    const bf16x8 o = *reinterpret_cast<const bf16x8*>(a.o + off);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += bf2f((uint16_t)d[j]) * bf2f((uint16_t)o[j]);
  }
  acc += __shfl_xor(acc, 1, 64);
  acc += __shfl_xor(acc, 2, 64);
  acc += __shfl_xor(acc, 4, 64);
  if (row < rows && part == 0) a.delta[row] = acc;
}

template <int NW>
void launch_fused(BwdArgs a, hipStream_t s) {
  a.blocks_per_bh = (a.N + NW * 32 - 1) / (NW * 32);
  const long long rows = (long long)a.B * a.H * a.N;
  hipLaunchKernelGGL(attn_delta_kernel, dim3((unsigned)((rows + 31) / 32)), dim3(256), 0, s, a);
  a.write_delta = 0;
  const int grid = 2 * a.blocks_per_bh * a.B * a.H;
  if (a.relh)
    hipLaunchKernelGGL((attn_bwd_fused_kernel<NW, 1>), dim3(grid), dim3(NW * 64), 0, s, a);
  else
    hipLaunchKernelGGL((attn_bwd_fused_kernel<NW, 0>), dim3(grid), dim3(NW * 64), 0, s, a);
}

template <int NW>
void launch_dq(BwdArgs a, hipStream_t s) {
  a.blocks_per_bh = (a.N + NW * 32 - 1) / (NW * 32);
  const int grid = a.blocks_per_bh * a.B * a.H;
  if (a.relh)
    hipLaunchKernelGGL((attn_bwd_dq_kernel<NW, 1>), dim3(grid), dim3(NW * 64), 0, s, a);
  else
    hipLaunchKernelGGL((attn_bwd_dq_kernel<NW, 0>), dim3(grid), dim3(NW * 64), 0, s, a);
}

template <int NW>
void launch_dkv(BwdArgs a, hipStream_t s) {
  a.blocks_per_bh = (a.N + NW * 32 - 1) / (NW * 32);
  const int grid = a.blocks_per_bh * a.B * a.H;
  if (a.relh)
    hipLaunchKernelGGL((attn_bwd_dkv_kernel<NW, 1>), dim3(grid), dim3(NW * 64), 0, s, a);
  else
    hipLaunchKernelGGL((attn_bwd_dkv_kernel<NW, 0>), dim3(grid), dim3(NW * 64), 0, s, a);
}

}  // namespace

extern "C" {

// q/k/v: bf16 with shared element strides (packed qkv); o/dout: bf16 and dq: fp32 with the o strides;
// lse: [B*H, N] from the forward; delta: [B*H, N] fp32 scratch; rel-pos (optional): relh [B*H, N, Hg],
// relw [B*H, N, 32] in, drelh / drelw out (same shapes; the SAM grid must be 32 wide);
// dk/dv: bf16 with their own shared strides (e.g. slots of a packed dqkv buffer).  head_dim 64.
// nw: waves (x 32 rows) per block for both kernels; 0 = pick from the grid size.
int be_attn_bwd(const void* q, const void* k, const void* v, long long s_tok, long long s_head, long long s_batch,
                const void* o, const void* dout, long long o_tok, long long o_head, long long o_batch,
                const float* lse, float* delta, const float* relh, const float* relw, int Hg, int Wg, float* dq,
                float* drelh, float* drelw, void* dk, void* dv, long long d_tok, long long d_head, long long d_batch,
                int B, int H, int N, int head_dim, float scale, int nw, hipStream_t stream) {
  if (head_dim != HD) return -1;
  if (N <= 0 || B <= 0 || H <= 0) return 0;
  if ((relh == nullptr) != (relw == nullptr)) return -2;
  if (relh && (Wg != 32 || Hg <= 0 || Hg * Wg != N || !drelh || !drelw)) return -3;
  BwdArgs a;
  a.q = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v;
  a.s_tok = s_tok; a.s_head = s_head; a.s_batch = s_batch;
  a.o = (const bf16_t*)o; a.dout = (const bf16_t*)dout;
  a.o_tok = o_tok; a.o_head = o_head; a.o_batch = o_batch;
  a.lse = lse; a.delta = delta; a.relh = relh; a.relw = relw; a.Hg = Hg;
  a.dq = dq; a.drelh = drelh; a.drelw = drelw;
  a.dk = (bf16_t*)dk; a.dv = (bf16_t*)dv; a.d_tok = d_tok; a.d_head = d_head; a.d_batch = d_batch;
  a.B = B; a.H = H; a.N = N; a.scale = scale; a.write_delta = 1;
  // fill the 256 CUs: 4 waves per block when that still gives >= 512 blocks, else 2
  const int blocks4 = ((N + 127) / 128) * B * H;
  if (nw == 0) nw = blocks4 >= 512 ? 4 : 2;
  if (blocks4 < 512) {  // small grid: dq + dkv blocks in one launch (see attn_bwd_fused_kernel)
    switch (nw) {
      case 2: launch_fused<2>(a, stream); break;
      case 4: launch_fused<4>(a, stream); break;
      default: return -4;
    }
    return BE_CHECK_LAUNCH();
  }
  switch (nw) {
    case 2: launch_dq<2>(a, stream); break;
    case 4: launch_dq<4>(a, stream); break;
    default: return -4;
  }
  int rc = BE_CHECK_LAUNCH();
  if (rc) return rc;
  switch (nw) {
    case 2: launch_dkv<2>(a, stream); break;
    case 4: launch_dkv<4>(a, stream); break;
  }
  return BE_CHECK_LAUNCH();
}

}  // extern "C"

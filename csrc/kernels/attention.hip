// Fused multi-head attention forward (flash-style) for the ViT encoders: DINOv2 ViT-B/14
// (cell-image-search embedder, SURVEY.md §2.5 K17, reference apps/cell-image-search/embedder.py:59-95)
// and the Cellpose-SAM ViT-L/8 encoder (K8, reference apps/cellpose-finetuning/main.py:126-127),
// including SAM's decomposed relative-position bias (attn += rel_h[q, key_row] + rel_w[q, key_col]),
// so the N x N score matrix never exists in HBM.
//
// CDNA4 design (head_dim 64, bf16 in/out, fp32 online softmax):
//  * v_mfma_f32_32x32x16_bf16 with the *keys on the rows* ("swapped" S^T = K Q^T): a lane owns one
//    query column and 16 of every 32 keys, so the row max / row sum is lane-local plus one exchange
//    with lane^32, and the S^T accumulator converted to bf16 IS the B operand of O^T = V^T P^T
//    (cdna_hip_programming.md §3 "accumulator tile as the next MFMA's operand") — P never touches LDS.
//  * V^T fragments come from ds_read_b64_tr_b16 transposed reads of a row-major V tile; K and V LDS
//    tiles are XOR-swizzled per 16-byte chunk (conflict-free transposed reads, spread b128 row reads).
//  * K/V tiles of 64 keys are register-staged: the next tile's global loads are in flight while the
//    current tile's MFMAs run (T14 "issue early / write late") and land in the second of two LDS
//    images, so each tile costs one barrier.
//  * block = NW waves x 32 queries of one (batch, head); the linear block id is XCD-remapped so the
//    blocks sharing a (batch, head)'s K/V stream run on one XCD's L2.
#include <cstdlib>

#include "common.h"

namespace {

constexpr int HD = 64;    // head dim
constexpr int KT = 64;    // keys per tile
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) short s16x4;

struct AttnArgs {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  long long s_tok, s_head, s_batch;  // element strides shared by q, k, v
  bf16_t* o;
  long long o_tok, o_head, o_batch;
  float* lse;          // optional [B, H, N] natural-log sum-exp of the scaled (+bias) scores
  const float* relh;   // optional [B*H, N, Hg]
  const float* relw;   // optional [B*H, N, Wg]
  int Hg, Wg;
  int B, H, N;
  float scale;
  int qblocks;         // ceil(N / (32 * NW))
  uint8_t* oq;         // optional MX-fp8 output instead of o: e4m3 with o's strides (bytes) ...
  uint8_t* os;         // ... + E8M0 scales [B * N, H * 2] (one per 32 head dims), the block-scaled
                       // input of the next fp8 GEMM (gemm_fp8.hip, XS) with no quantisation pass
};

__device__ __forceinline__ uint32_t cvt_pk_bf16(float lo, float hi) {
  uint32_t r;
  asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}

// chunk swizzles (16-byte chunks, 8 per 128-byte row)
__device__ __forceinline__ int k_off(int row, int ch) { return row * HD + ((ch ^ ((row >> 1) & 7)) << 3); }
__device__ __forceinline__ int v_off(int row, int ch) { return row * HD + ((ch ^ (((row >> 1) & 1) << 2)) << 3); }

// BIAS: 0 none, 1 generic decomposed rel-pos (per-key gathers), 2 the SAM 32-wide grid: a 32-key
// block is exactly one grid row, so a lane's 16 key columns are fixed (rel_w in registers) and the
// row term is one value per block.
//
// Per-tile VALU budget (the loop is VALU-issue bound at head_dim 64: 16 MFMAs of 32 cycles vs 32
// scores per lane): the rel_w term and the score scale are one FMA per score, the rel_h term is
// applied to the two block maxima and to the exponent offsets instead of to every score, the
// key-range mask runs only on a ragged last tile, and the O / l rescale is skipped (wave-uniform
// branch) when no query's running maximum grew -- exact, alpha would be 1.  K/V tiles are double
// buffered in LDS: one barrier per tile, the next tile's global loads in flight under the MFMAs and
// written to the other buffer after them.
template <int NW, int BIAS>
__global__ __launch_bounds__(NW * 64) void attn_fwd_kernel(AttnArgs a) {
  constexpr int NT = NW * 64;
  constexpr int CHUNKS = 2 * KT * (HD / 8);        // K + V tile, 16-byte chunks
  constexpr int CPT = (CHUNKS + NT - 1) / NT;      // chunks per thread
  __shared__ __attribute__((aligned(16))) bf16_t Ks[2][KT * HD];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[2][KT * HD];
  constexpr float LOG2E = 1.4426950408889634f;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int h = lane >> 5;
  const int ql = lane & 31;
  const int total = a.qblocks * a.B * a.H;
  const int logical = xcd_remap(blockIdx.x, total);
  const int bh = logical / a.qblocks;
  const int qb = logical % a.qblocks;
  const int b = bh / a.H, hh = bh % a.H;
  const int q0 = qb * NW * 32 + wave * 32;
  const int qi = q0 + ql;                 // this lane's query
  const int qc = min(qi, a.N - 1);        // clamped for loads

  const bf16_t* qbase = a.q + (long long)b * a.s_batch + (long long)hh * a.s_head;
  const bf16_t* kbase = a.k + (long long)b * a.s_batch + (long long)hh * a.s_head;
  const bf16_t* vbase = a.v + (long long)b * a.s_batch + (long long)hh * a.s_head;

  const int ntiles = (a.N + KT - 1) / KT;
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
        const int key = t * KT + row;
        if (key < a.N) {
          const bf16_t* src = (isv ? vbase : kbase) + (long long)key * a.s_tok + ch * 8;
          r = *reinterpret_cast<const u32x4*>(src);
        }
      }
      stage[i] = r;
    }
  };
  auto commit = [&](int buf) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + i * NT;
      if (c < CHUNKS) {
        const int isv = c >= CHUNKS / 2;
        const int cc = c - isv * (CHUNKS / 2);
        const int row = cc >> 3, ch = cc & 7;
        if (isv)
          *reinterpret_cast<u32x4*>(&Vs[buf][v_off(row, ch)]) = stage[i];
        else
          *reinterpret_cast<u32x4*>(&Ks[buf][k_off(row, ch)]) = stage[i];
      }
    }
  };
  issue(0);

  // Q^T fragments (B operand of S^T = K Q^T): 4 k-steps of 16 head dims.
  bf16x8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    u32x4 r = *reinterpret_cast<const u32x4*>(qbase + (long long)qc * a.s_tok + ks * 16 + h * 8);
    if (qi >= a.N) r = (u32x4){0u, 0u, 0u, 0u};
    qf[ks] = *reinterpret_cast<bf16x8*>(&r);
  }
  const float c2 = a.scale * LOG2E;  // scores -> log2 domain
  const float* rh = nullptr;
  const float* rw = nullptr;
  float rwr[16];
  if (BIAS) {
    rh = a.relh + ((long long)bh * a.N + qc) * a.Hg;
    rw = a.relw + ((long long)bh * a.N + qc) * a.Wg;
  }
  float rh_cur[2] = {0.f, 0.f};
  if (BIAS == 2) {
#pragma unroll
    for (int i = 0; i < 16; ++i) rwr[i] = rw[8 * (i >> 2) + 4 * h + (i & 3)] * LOG2E;
    rh_cur[0] = rh[0];
    rh_cur[1] = rh[min(1, a.Hg - 1)];
  }

  f32x16 oacc[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) { oacc[0][i] = 0.f; oacc[1][i] = 0.f; }
  float m = -INFINITY, l = 0.f;
  const f32x16 zero16 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

  commit(0);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntiles) issue(t + 1);
    float rh_next[2] = {0.f, 0.f};
    if (BIAS == 2) {  // the next tile's row terms (clamped), in flight under this tile's work
      rh_next[0] = rh[min(2 * t + 2, a.Hg - 1)];
      rh_next[1] = rh[min(2 * t + 3, a.Hg - 1)];
    }
    const bf16_t* Kc = Ks[cur];
    const bf16_t* Vc = Vs[cur];

    // ---- S^T = K Q^T for the two 32-key blocks: all 8 K fragments requested before the MFMAs
    // so the reads' latency is paid once per tile, not once per MFMA
    bf16x8 kf[2][4];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        kf[kb][ks] = *reinterpret_cast<const bf16x8*>(Kc + k_off(kb * 32 + ql, 2 * ks + h));
    __builtin_amdgcn_sched_barrier(0);
    f32x16 s[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[kb][0], qf[0], zero16, 0, 0, 0);
#pragma unroll
      for (int ks = 1; ks < 4; ++ks) s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[kb][ks], qf[ks], s[kb], 0, 0, 0);
    }
    // ---- online softmax (lane = query; keys: kb*32 + 8(i>>2) + 4h + (i&3)), log2 domain
    float rhv[2] = {0.f, 0.f};
    if (BIAS == 2) {
      rhv[0] = rh_cur[0] * LOG2E;
      rhv[1] = rh_cur[1] * LOG2E;
    }
    float mt = -INFINITY;
    const bool ragged = (t + 1) * KT > a.N;  // wave-uniform
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      float mk = -INFINITY;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float x;
        if (BIAS == 2) {
          x = __builtin_fmaf(s[kb][i], c2, rwr[i]);
        } else if (BIAS == 1) {
          const int key = t * KT + kb * 32 + 8 * (i >> 2) + 4 * h + (i & 3);
          const int kc = min(key, a.N - 1);
          const int kh = kc / a.Wg, kw = kc - kh * a.Wg;
          x = __builtin_fmaf(s[kb][i], c2, (rh[kh] + rw[kw]) * LOG2E);
        } else {
          x = s[kb][i] * c2;
        }
        s[kb][i] = x;
      }
      if (ragged) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = t * KT + kb * 32 + 8 * (i >> 2) + 4 * h + (i & 3);
          s[kb][i] = key < a.N ? s[kb][i] : -INFINITY;
        }
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) mk = fmaxf(mk, s[kb][i]);
      mt = fmaxf(mt, mk + rhv[kb]);
    }
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    if (__any(mt > m)) {  // some query's maximum grew: rescale (others get alpha = 1 exactly)
      const float mn = fmaxf(m, mt);
      const float alpha = (m == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(m - mn);
      m = mn;
      l *= alpha;
#pragma unroll
      for (int i = 0; i < 16; ++i) { oacc[0][i] *= alpha; oacc[1][i] *= alpha; }
    }
    float rs = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const float off = m - rhv[kb];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = __builtin_amdgcn_exp2f(s[kb][i] - off);
        s[kb][i] = p;
        rs += p;
      }
    }
    l += rs;

    // ---- O^T += V^T P^T
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        u32x4 pw;
        pw[0] = cvt_pk_bf16(s[kb][8 * st + 0], s[kb][8 * st + 1]);
        pw[1] = cvt_pk_bf16(s[kb][8 * st + 2], s[kb][8 * st + 3]);
        pw[2] = cvt_pk_bf16(s[kb][8 * st + 4], s[kb][8 * st + 5]);
        pw[3] = cvt_pk_bf16(s[kb][8 * st + 6], s[kb][8 * st + 7]);
        const bf16x8 pf = *reinterpret_cast<bf16x8*>(&pw);
        const int g1 = (lane >> 4) & 1;
        const int qq = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          const int ch = db * 4 + 2 * g1 + (pp >> 1);
          const int row0 = kb * 32 + 16 * st + 4 * h + qq;
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(Vc + v_off(row0, ch) + 4 * (pp & 1)));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(Vc + v_off(row0 + 8, ch) + 4 * (pp & 1)));
          bf16x8 vf;
          vf[0] = lo[0]; vf[1] = lo[1]; vf[2] = lo[2]; vf[3] = lo[3];
          vf[4] = hi[0]; vf[5] = hi[1]; vf[6] = hi[2]; vf[7] = hi[3];
          oacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, oacc[db], 0, 0, 0);
        }
      }
    if (t + 1 < ntiles) commit(cur ^ 1);
    rh_cur[0] = rh_next[0];
    rh_cur[1] = rh_next[1];
    __syncthreads();
  }

  // ---- epilogue: O = O^T / l  (lane = query, d = db*32 + 8(i>>2) + 4h + (i&3))
  const float lt = l + __shfl_xor(l, 32, 64);
  if (a.oq) {  // MX-fp8: block db = head dims [32 db, +32) = this lane's 16 values + the partner lane's
    const float inv = 1.f / lt;
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      float amax = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) amax = fmaxf(amax, fabsf(oacc[db][i] * inv));
      amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
      // smallest power of two 2^e with amax / 2^e <= 448 (E8M0 byte e + 127), as gemm_fp8.hip EPI 2
      int e = amax > 0.f ? (int)ceilf(__log2f(amax * (1.f / 448.f))) : -127;
      if (e > 0 && amax * __builtin_ldexpf(1.f, -e) > 448.f) ++e;
      e = max(-127, min(127, e));
      const float sc = inv * __builtin_ldexpf(1.f, -e);
      if (qi < a.N) {
        uint8_t* oqb = a.oq + (long long)b * a.o_batch + (long long)hh * a.o_head + (long long)qi * a.o_tok + db * 32;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          int w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(oacc[db][4 * g + 0] * sc, -448.f), 448.f),
                                                  fminf(fmaxf(oacc[db][4 * g + 1] * sc, -448.f), 448.f), 0, false);
          w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(oacc[db][4 * g + 2] * sc, -448.f), 448.f),
                                              fminf(fmaxf(oacc[db][4 * g + 3] * sc, -448.f), 448.f), w, true);
          *reinterpret_cast<uint32_t*>(oqb + 8 * g + 4 * h) = (uint32_t)w;
        }
        if (h == 0) a.os[((long long)b * a.N + qi) * (2 * a.H) + 2 * hh + db] = (uint8_t)(e + 127);
      }
    }
    if (qi < a.N && a.lse && h == 0) a.lse[(long long)bh * a.N + qi] = (m + __log2f(lt)) * 0.6931471805599453f;
    return;
  }
  if (qi < a.N) {
    const float inv = 1.f / lt;
    bf16_t* ob = a.o + (long long)b * a.o_batch + (long long)hh * a.o_head + (long long)qi * a.o_tok;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u32x2 w;
        w[0] = cvt_pk_bf16(oacc[db][4 * g + 0] * inv, oacc[db][4 * g + 1] * inv);
        w[1] = cvt_pk_bf16(oacc[db][4 * g + 2] * inv, oacc[db][4 * g + 3] * inv);
        *reinterpret_cast<u32x2*>(ob + db * 32 + 8 * g + 4 * h) = w;
      }
    if (a.lse && h == 0) a.lse[(long long)bh * a.N + qi] = (m + __log2f(lt)) * 0.6931471805599453f;
  }
}

template <int NW>
int launch_nw(AttnArgs a, hipStream_t s) {
  a.qblocks = (a.N + NW * 32 - 1) / (NW * 32);
  const int grid = a.qblocks * a.B * a.H;
  if (a.relh && a.Wg == 32)
    hipLaunchKernelGGL((attn_fwd_kernel<NW, 2>), dim3(grid), dim3(NW * 64), 0, s, a);
  else if (a.relh)
    hipLaunchKernelGGL((attn_fwd_kernel<NW, 1>), dim3(grid), dim3(NW * 64), 0, s, a);
  else
    hipLaunchKernelGGL((attn_fwd_kernel<NW, 0>), dim3(grid), dim3(NW * 64), 0, s, a);
  return BE_CHECK_LAUNCH();
}

// nw = 0 picks the waves per block (2, 3 or 4 x 32 queries) that least overpads N.  BE_ATTN_NW pins
// it (A/B).  Filling the CUs at CPSAM batch 1 (16 heads x 1024 queries = 128 four-wave blocks) with
// 256 two-wave blocks measured slower: 26.5 vs 23.5 us per layer (profiles/r04/cpsam/attn_nw_ab.txt).
static int g_attn_nw = [] {
  const char* e = getenv("BE_ATTN_NW");
  return e ? atoi(e) : 0;
}();

int attn_dispatch(AttnArgs a, int nw, hipStream_t stream) {
  const int N = a.N;
  if (nw == 0) nw = g_attn_nw;
  if (nw == 0) {
    const int slices = (N + 31) / 32;
    int best = 4, waste = 1 << 30;
    for (int c : {4, 3, 2}) {
      const int w = ((slices + c - 1) / c) * c - slices;
      if (w < waste) { waste = w; best = c; }
    }
    nw = best;
  }
  switch (nw) {
    case 2: return launch_nw<2>(a, stream);
    case 3: return launch_nw<3>(a, stream);
    case 4: return launch_nw<4>(a, stream);
    case 8: return launch_nw<8>(a, stream);
  }
  return -4;
}

}  // namespace

extern "C" {

// q/k/v: bf16 with element strides (token, head, batch) shared by the three (e.g. a packed
// [B, N, 3, H, 64] qkv buffer); o: bf16 with its own strides.  head_dim must be 64.
// nw = 0 picks the waves per block (2, 3 or 4 x 32 queries) that least overpads N.
// be_attn_fwd with an MX-fp8 output: oq e4m3 [B, N, H, 64] contiguous + os E8M0 [B * N, H * 2].
int be_attn_fwd_mx(const void* q, const void* k, const void* v, long long s_tok, long long s_head, long long s_batch,
                   void* oq, void* os, int B, int H, int N, int head_dim, float scale, hipStream_t stream) {
  if (head_dim != HD) return -1;
  if (N <= 0 || B <= 0 || H <= 0) return 0;
  if (!oq || !os) return -2;
  AttnArgs a;
  a.q = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v;
  a.s_tok = s_tok; a.s_head = s_head; a.s_batch = s_batch;
  a.o = nullptr; a.o_tok = (long long)H * HD; a.o_head = HD; a.o_batch = (long long)N * H * HD;
  a.lse = nullptr; a.relh = nullptr; a.relw = nullptr; a.Hg = 0; a.Wg = 0;
  a.B = B; a.H = H; a.N = N; a.scale = scale;
  a.oq = (uint8_t*)oq; a.os = (uint8_t*)os;
  return attn_dispatch(a, 0, stream);
}

int be_attn_fwd(const void* q, const void* k, const void* v, long long s_tok, long long s_head, long long s_batch,
                void* o, long long o_tok, long long o_head, long long o_batch, float* lse, const float* relh,
                const float* relw, int Hg, int Wg, int B, int H, int N, int head_dim, float scale, int nw,
                hipStream_t stream) {
  if (head_dim != HD) return -1;
  if (N <= 0 || B <= 0 || H <= 0) return 0;
  if ((relh == nullptr) != (relw == nullptr)) return -2;
  if (relh && (Hg <= 0 || Wg <= 0 || Hg * Wg != N)) return -3;
  AttnArgs a;
  a.q = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v;
  a.s_tok = s_tok; a.s_head = s_head; a.s_batch = s_batch;
  a.o = (bf16_t*)o; a.o_tok = o_tok; a.o_head = o_head; a.o_batch = o_batch;
  a.lse = lse; a.relh = relh; a.relw = relw; a.Hg = Hg; a.Wg = Wg;
  a.B = B; a.H = H; a.N = N; a.scale = scale;
  a.oq = nullptr; a.os = nullptr;
  return attn_dispatch(a, nw, stream);
}

}  // extern "C"

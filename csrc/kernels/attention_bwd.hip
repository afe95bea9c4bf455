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
// Tiles are XOR-swizzled per 16-byte chunk (v_off: conflict-free transposed reads) and stream
// HBM -> LDS by LDS-DMA two tiles ahead of the MFMAs (three LDS stages, counted vmcnt across raw
// barriers).  Block ids are XCD-remapped so the blocks that stream the same (batch, head) K/V or
// Q/dO rows share an L2.
#include "common.h"

namespace {

constexpr int HD = 64;   // head dim
constexpr int TT = 64;   // streamed rows per LDS tile (keys in the dq kernel, queries in the dkv kernel)
constexpr float LOG2E = 1.4426950408889634f;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) uint8_t lds_u8;

// s_waitcnt immediate waiting for vmcnt <= n only (gfx9 encoding, as in gemm_fp8.hip)
constexpr int waitcnt_vm(int n) { return (n & 0xf) | (0x7 << 4) | (0xf << 8) | ((n >> 4) << 14); }

// HBM -> LDS DMA (global_load_lds_dword / _dwordx4) in inline asm.  Through the builtin the compiler
// treats every later ds_read of the (single) LDS array as aliasing the newest DMA and puts a
// vmcnt(0) in front of it, which drains the prefetch this pipeline keeps in flight; these waits are
// explicit below.  lds is the wave-uniform LDS byte address of lane 0's destination (lane i writes
// at lds + i * size); M0 is saved and restored around the instruction.
template <int SIZE>
__device__ __forceinline__ void glds(const void* src, uint32_t lds) {
  unsigned keep;
  lds = __builtin_amdgcn_readfirstlane(lds);
  if constexpr (SIZE == 16)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(size_t)(lds_u8*)(p);
}

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

// chunk swizzles (16-byte chunks, 8 per 128-byte row).  k_off: conflict-free 16-row b128 row reads.
// v_off, for tiles read BOTH as rows (b128, 16 lanes = 16 rows at one chunk) and transposed
// (read_tr: 4 rows x 4 chunks per 32 lanes): with m = row >> 1, bit 2 of the XOR is m & 1 (rows r and
// r + 2 of a transposed group land in different 4-chunk halves) and bits 0-1 are m >> 1, so the 8
// even (odd) rows of a 16-row group get 8 distinct chunk slots.  (attention.hip's v_off, XOR 4 (m & 1)
// only, is 4-way conflicted on row reads: SQ_LDS_BANK_CONFLICT in profiles/r03/cpsam/attn_pmc.md.)
__device__ __forceinline__ int k_off(int row, int ch) { return row * HD + ((ch ^ ((row >> 1) & 7)) << 3); }
__device__ __forceinline__ int v_swz(int row) { return (((row >> 1) & 1) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int v_off(int row, int ch) { return row * HD + ((ch ^ v_swz(row)) << 3); }

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

// LDS bytes per block (three pipeline stages).  dq: K | V tile + the tile's two rel_h grid rows per
// query.  dkv: see dkv_body.
template <int NW, int BIAS>
constexpr int dq_lds() {
  return 3 * (2 * TT * HD * 2 + (BIAS ? NW * 64 * 4 : 0));
}
template <int NW, int BIAS>
constexpr int dkv_lds() {
  return 3 * (2 * TT * HD * 2 + (BIAS ? TT * 32 * 4 + NW * TT * 4 : 0) + 2 * TT * 4);
}

// ------------------------------------------------------------------ dQ (+ drel, delta)
// The K / V tiles go HBM -> LDS by global_load_lds through three stages (the dkv pipeline below);
// the tile's two rel_h grid rows per query ride along as one dword DMA per wave, so the loop has no
// register loads left (an in-loop global load would make the compiler drain the DMAs with vmcnt(0)).
template <int NW, int BIAS>
__device__ __forceinline__ void dq_body(const BwdArgs& a, int logical, uint8_t* smem) {
  constexpr int TB = TT * HD * 2;
  constexpr int OFF_R = 2 * TB;  // rel_h: [wave][kb][32 queries]
  constexpr int STAGE = OFF_R + (BIAS ? NW * 64 * 4 : 0);
  constexpr int LOADS = 16 / NW + (BIAS ? 1 : 0);  // DMA instructions per wave and tile
  static_assert(3 * STAGE <= dq_lds<NW, BIAS>(), "LDS size");

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
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

  const float* rhq = BIAS ? a.relh + ((long long)bh * a.N + qc) * a.Hg : nullptr;
  float rwr[16], drw[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) { rwr[i] = 0.f; drw[i] = 0.f; }
  if (BIAS) {
    const float* rw = a.relw + ((long long)bh * a.N + qc) * 32;
#pragma unroll
    for (int i = 0; i < 16; ++i) rwr[i] = rw[8 * (i >> 2) + 4 * h + (i & 3)] * LOG2E;
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));  // register loads land before the (compiler-invisible) DMAs

  f32x16 dqa[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) { dqa[0][i] = 0.f; dqa[1][i] = 0.f; }

  const int ntiles = (a.N + TT - 1) / TT;
  auto issue = [&](int t) {
    uint8_t* st = smem + (t % 3) * STAGE;
#pragma unroll
    for (int j = 0; j < 16 / NW; ++j) {
      const int g = j * NW + wave;  // wave-uniform: 1 KiB = 8 key rows of K (g < 8) or V
      const int row = (g & 7) * 8 + (lane >> 3);
      const int key = min(t * TT + row, a.N - 1);  // padded keys: any finite row, P = 0 below
      // source chunk = the swizzle's inverse at the lane-linear LDS slot (both are involutions)
      const int ch = g < 8 ? (lane & 7) ^ v_swz(row) : (lane & 7) ^ ((row >> 1) & 7);
      const bf16_t* src = (g < 8 ? kbase : vbase) + (long long)key * a.s_tok + ch * 8;
      glds<16>(src, lds_addr(st + (g < 8 ? 0 : TB) + (g & 7) * 1024));
    }
    if (BIAS)  // lanes 0-31: grid row 2t, 32-63: row 2t+1, of this wave's 32 queries
      glds<4>(rhq + min(2 * t + h, a.Hg - 1), lds_addr(st + OFF_R + wave * 256));
  };

  issue(0);
  if (ntiles > 1) issue(1);
  for (int t = 0; t < ntiles; ++t) {
    // tile t landed (tile t+1 may stay in flight).  The drel_h stores of earlier tiles also count in
    // vmcnt; waiting for <= LOADS outstanding is safe whatever order they retire in.
    if (t + 1 < ntiles)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LOADS) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + 2 < ntiles) issue(t + 2);
    const uint8_t* st = smem + (t % 3) * STAGE;
    const bf16_t* Ks = reinterpret_cast<const bf16_t*>(st);
    const bf16_t* Vs = reinterpret_cast<const bf16_t*>(st + TB);
    const float* Rh = reinterpret_cast<const float*>(st + OFF_R) + wave * 64;
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
      const float rhv = BIAS ? Rh[kb * 32 + ql] * LOG2E : 0.f;
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
      for (int st2 = 0; st2 < 2; ++st2) {
        const bf16x8 pf = pack_b(s, st2);
#pragma unroll
        for (int db = 0; db < 2; ++db)
          dqa[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(read_tr(Ks, lane, kb, st2, db), pf, dqa[db], 0, 0, 0);
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
// The query tiles go HBM -> LDS with global_load_lds (no staging VGPRs, no ds_write pass) through
// THREE LDS stages: tile t+2's DMA is issued right after the barrier that opens tile t and stays in
// flight across the next barrier (counted vmcnt, raw s_barrier).  The register-staged version of
// this kernel waited for tile t+1's loads at the top of every tile: SQ_WAIT_ANY 62 % of its wave
// cycles; with the DMA pipeline 25 % and 0.58x the wave cycles (profiles/r03/cpsam/attn_pmc.md).
// The LDS image is raw: rel_w / rel_h / lse stay in natural-log units and are combined at read time.
// Stage = Q 8K | dO 8K | rel_w 8K | rel_h NW x 256 B | lse 256 B | delta 256 B; three stages of the
// 4-wave bias kernel = 76.5 KiB: two blocks per CU.
template <int NW, int BIAS>
__device__ __forceinline__ void dkv_body(const BwdArgs& a, int logical, uint8_t* smem) {
  constexpr int QB = TT * HD * 2;
  constexpr int WB = BIAS ? TT * 32 * 4 : 0;
  constexpr int HB = BIAS ? NW * TT * 4 : 0;
  constexpr int OFF_D = QB, OFF_W = 2 * QB, OFF_H = OFF_W + WB, OFF_L = OFF_H + HB, OFF_DL = OFF_L + TT * 4;
  constexpr int STAGE = OFF_DL + TT * 4;
  constexpr int GROUPS = BIAS ? 24 : 16;  // 1 KiB wave-instructions: Q 8, dO 8, rel_w 8
  static_assert(GROUPS % NW == 0, "row groups must split evenly over waves");
  // per-wave DMA instructions per tile: GROUPS / NW (+ one rel_h row, + lse / delta on waves 0 / 1);
  // the counted wait uses the smallest count (a wave with more waits a little longer, never too short)
  constexpr int LOADS_MIN = GROUPS / NW + (BIAS ? 1 : 0) + (NW > 2 ? 0 : 1);
  static_assert(3 * STAGE <= dkv_lds<NW, BIAS>(), "LDS size");

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  (void)tid;
  const int h = lane >> 5, kl = lane & 31;
  const int bh = logical / a.blocks_per_bh, kblk = logical % a.blocks_per_bh;
  const int b = bh / a.H, hh = bh % a.H;
  const int kj = kblk * NW * 32 + wave * 32 + kl;
  const bool kv = kj < a.N;
  const int kc = min(kj, a.N - 1);

  const long long kvoff = (long long)b * a.s_batch + (long long)hh * a.s_head;
  const bf16_t* qbase = a.q + kvoff;
  const bf16_t* dbase = a.dout + (long long)b * a.o_batch + (long long)hh * a.o_head;
  const float* lrow = a.lse + (long long)bh * a.N;
  const float* drow = a.delta + (long long)bh * a.N;
  const float* hbase = BIAS ? a.relh + (long long)bh * a.N * a.Hg + min(kblk * NW + wave, a.Hg - 1) : nullptr;
  const float* wbase = BIAS ? a.relw + (long long)bh * a.N * 32 : nullptr;

  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    kf[ks] = load_frag(a.k + kvoff + (long long)kc * a.s_tok + ks * 16 + h * 8, kv);
    vf[ks] = load_frag(a.v + kvoff + (long long)kc * a.s_tok + ks * 16 + h * 8, kv);
  }
  // K / V rows land before the DMA pipeline starts: the compiler does not see the asm DMAs, and a
  // first use of kf / vf inside the loop would make it wait vmcnt(0) there on every tile
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
  const float c2 = a.scale * LOG2E;

  f32x16 dva[2], dka[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) { dva[0][i] = 0.f; dva[1][i] = 0.f; dka[0][i] = 0.f; dka[1][i] = 0.f; }

  const int ntiles = (a.N + TT - 1) / TT;
  auto issue = [&](int t) {
    uint8_t* st = smem + (t % 3) * STAGE;
    const int q0 = t * TT;
#pragma unroll
    for (int j = 0; j < GROUPS / NW; ++j) {
      const int g = j * NW + wave;  // wave-uniform
      const int row = (g & 7) * 8 + (lane >> 3);
      const int qc = min(q0 + row, a.N - 1);  // padded queries: any finite row, P = 0 below
      const void* src;
      if (!BIAS || g < 16) {  // Q / dO rows, v_off swizzle applied on the source chunk (involution)
        const int ch = (lane & 7) ^ v_swz(row);
        src = g < 8 ? (const void*)(qbase + (long long)qc * a.s_tok + ch * 8)
                    : (const void*)(dbase + (long long)qc * a.o_tok + ch * 8);
      } else {
        src = (const void*)(wbase + (long long)qc * 32 + (lane & 7) * 4);
      }
      const int off = g < 8 ? 0 : (g < 16 ? OFF_D : OFF_W);
      glds<16>(src, lds_addr(st + off + (g & 7) * 1024));
    }
    const int qc = min(q0 + lane, a.N - 1);
    if (BIAS)
      glds<4>(hbase + (long long)qc * a.Hg, lds_addr(st + OFF_H + wave * TT * 4));
    if (wave < 2)
      glds<4>((wave == 0 ? lrow : drow) + qc, lds_addr(st + (wave == 0 ? OFF_L : OFF_DL)));
  };

  issue(0);
  if (ntiles > 1) issue(1);
  for (int t = 0; t < ntiles; ++t) {
    // tile t landed; tile t+1 stays in flight
    if (t + 1 < ntiles)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LOADS_MIN) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's part of tile t is in LDS; every wave is done with t-1
    if (t + 2 < ntiles) issue(t + 2);  // into tile t-1's stage
    const uint8_t* st = smem + (t % 3) * STAGE;
    const bf16_t* Qc = reinterpret_cast<const bf16_t*>(st);
    const bf16_t* Dc = reinterpret_cast<const bf16_t*>(st + OFF_D);
    const float* Wc = reinterpret_cast<const float*>(st + OFF_W);
    const float* Hc = reinterpret_cast<const float*>(st + OFF_H) + wave * TT;
    const float* Lc = reinterpret_cast<const float*>(st + OFF_L);
    const float* DLc = reinterpret_cast<const float*>(st + OFF_DL);
    const int qlim = a.N - t * TT;  // queries >= qlim in this tile are padding
#pragma unroll 1
    for (int qb = 0; qb < 2; ++qb) {
      f32x16 s, dp;
#pragma unroll
      for (int i = 0; i < 16; ++i) { s[i] = 0.f; dp[i] = 0.f; }
      // LDS reads of this lane's 16 queries' lse / delta / rel_h / rel_w, all issued ahead of the
      // S / dP MFMAs (sched_barrier) so their latency hides under the matrix work
      float4 lv[4], dlv[4], hv[4];
      float wv[16];
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int qr0 = qb * 32 + 8 * g4 + 4 * h;
        lv[g4] = *reinterpret_cast<const float4*>(Lc + qr0);
        dlv[g4] = *reinterpret_cast<const float4*>(DLc + qr0);
        hv[g4] = BIAS ? *reinterpret_cast<const float4*>(Hc + qr0) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int j = 0; j < 4; ++j) wv[4 * g4 + j] = BIAS ? Wc[(qr0 + j) * 32 + kl] : 0.f;
      }
      const int row = qb * 32 + kl;
      bf16x8 qa[4], da[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        qa[ks] = *reinterpret_cast<const bf16x8*>(Qc + v_off(row, 2 * ks + h));
        da[ks] = *reinterpret_cast<const bf16x8*>(Dc + v_off(row, 2 * ks + h));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa[ks], kf[ks], s, 0, 0, 0);
        dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da[ks], vf[ks], dp, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int g4 = i >> 2, j = i & 3;
        const int qr = qb * 32 + 8 * g4 + 4 * h + j;
        const float l = j == 0 ? lv[g4].x : j == 1 ? lv[g4].y : j == 2 ? lv[g4].z : lv[g4].w;
        const float d = j == 0 ? dlv[g4].x : j == 1 ? dlv[g4].y : j == 2 ? dlv[g4].z : dlv[g4].w;
        const float hr = j == 0 ? hv[g4].x : j == 1 ? hv[g4].y : j == 2 ? hv[g4].z : hv[g4].w;
        const float bz = ((BIAS ? hr + wv[i] : 0.f) - l) * LOG2E;
        const float p = (kv && qr < qlim) ? __builtin_amdgcn_exp2f(__builtin_fmaf(s[i], c2, bz)) : 0.f;
        s[i] = p;
        dp[i] = p * (dp[i] - d);
      }
#pragma unroll
      for (int st2 = 0; st2 < 2; ++st2) {
        const bf16x8 pf = pack_b(s, st2);
        const bf16x8 dsf = pack_b(dp, st2);
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          dva[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(read_tr(Dc, lane, qb, st2, db), pf, dva[db], 0, 0, 0);
          dka[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(read_tr(Qc, lane, qb, st2, db), dsf, dka[db], 0, 0, 0);
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
  __shared__ __attribute__((aligned(16))) uint8_t smem[dq_lds<NW, BIAS>()];  // the only LDS object
  dq_body<NW, BIAS>(a, xcd_remap(blockIdx.x, a.blocks_per_bh * a.B * a.H), smem);
}

template <int NW, int BIAS>
__global__ __launch_bounds__(NW * 64) BE_ATTN_BWD_WPE void attn_bwd_dkv_kernel(BwdArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[dkv_lds<NW, BIAS>()];
  dkv_body<NW, BIAS>(a, xcd_remap(blockIdx.x, a.blocks_per_bh * a.B * a.H), smem);
}

// Small grids (batch 1: 16 heads x 1024 tokens = 256 + 256 two-wave blocks): the dq and dkv blocks
// run as ONE launch (blocks [0, n) dq, [n, 2n) dkv) so both halves fill the 1024 SIMDs together;
// delta = rowsum(dO * O) comes from attn_delta_kernel first.  One LDS array serves either body.
template <int NW, int BIAS>
__global__ __launch_bounds__(NW * 64) BE_ATTN_BWD_WPE void attn_bwd_fused_kernel(BwdArgs a) {
  constexpr int L = dq_lds<NW, BIAS>() > dkv_lds<NW, BIAS>() ? dq_lds<NW, BIAS>() : dkv_lds<NW, BIAS>();
  __shared__ __attribute__((aligned(16))) uint8_t smem[L];
  const int n = a.blocks_per_bh * a.B * a.H;
  if ((int)blockIdx.x < n) {
    dq_body<NW, BIAS>(a, xcd_remap(blockIdx.x, n), smem);
  } else {
    dkv_body<NW, BIAS>(a, xcd_remap(blockIdx.x - n, n), smem);
  }
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

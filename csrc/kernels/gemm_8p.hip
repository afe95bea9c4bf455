// 256 x 256 bf16 GEMM on two staggered wave groups ("8-phase" ping-pong) for the Cellpose-SAM
// ViT-L linear layers (reference training step apps/cellpose-finetuning/main.py:
// 1483-1546, inference :4966-5144):
//
//   NT  C[M][N] = A[M][K] . B[N][K]^T (+ bias) (+ residual | GELU)       forward, x W^T
//
// Why a second kernel beside gemm_mt.hip: gemm_mt runs ONE wave per SIMD (4 waves, 128 x 128
// accumulators each), so a wave waiting on a barrier or on its next fragments leaves its SIMD's
// matrix core idle; its counters showed MFMA-busy 0.91-1.40 per wave-cycle against hipBLASLt's
// 1.9-2.5 (profiles/r05/pmc/gemm_mt_vs_hipblaslt_fwd_b8.txt).  Here every SIMD holds two waves, one
// from each group, and the groups run one barrier apart, so while one wave issues its 16 MFMAs the
// other issues its LDS fragment reads and its share of the next tiles' LDS-DMA
// (cdna_hip_programming.md §5 "The 256² 8-phase template").
//
// MI355X design:
//  * 512 threads = 8 waves as 2 (M) x 4 (N); a wave owns 128 x 64 outputs = 8 x 4 fragments of
//    v_mfma_f32_16x16x32_bf16 (128 fp32 accumulators), the block 256 x 256.
//  * K in 64-deep tiles, two LDS buffers of 64 KiB (A image 256 rows x 128 B, B image likewise).  A
//    tile is consumed in 4 phases, one C quadrant each (64 x 32 x K64 = 16 MFMAs):
//      phase 1 (m0, n0)  reads A[m0] (8 ds_read_b128) + B[n0] (4)   DMA: A[m1] of tile t+1
//      phase 2 (m0, n1)  reads B[n1] (4)
//      phase 3 (m1, n1)  reads A[m1] (8)                            DMA: A[m0], B[n0] of tile t+2
//      phase 4 (m1, n0)  (B[n0] still in registers)                 DMA: B[n1] of tile t+2; vmcnt(6)
//    Each operand image is stored as two PARTS (the m0 / m1 rows of both wave rows, the n0 / n1
//    columns of all four wave columns), so a part dies as soon as every wave has read it and the
//    next-but-one tile's DMA refills it: a load gets 1-1.5 tiles (4-6 phases) of MFMAs to land, with
//    only two buffers.  The WAR / RAW distances assume the one-barrier stagger: a part is refilled
//    >= 2 barriers after the lagging group's last read of it, and every wave's counted vmcnt sits
//    before the barrier that precedes the first read of what it waits for (derivation in
//    gemm_8p_notes below).
//  * Phase = [fragment reads, DMA issue] s_barrier, lgkmcnt(0), s_setprio(1), 16 MFMAs, s_setprio(0),
//    s_barrier; group 1 (waves 4-7) enters the loop one s_barrier late and group 0 leaves one late,
//    so on every SIMD one wave's MFMAs overlap the other's reads.
//  * LDS images: 128-byte rows, 16-byte chunk c of row r at c ^ ((r >> 1) & 7) (gemm_mt's measured
//    conflict-free swizzle); the DMA destination stays lane-linear, the swizzle lives in the per-lane
//    source address (§5.4 rule 21).
//  * XCD-aware block order (T1): the N tiles of one M row are consecutive logical blocks on one XCD,
//    so the A rows they share are read once into that XCD's L2.
//
// Status (round 6, profiles/r06/gemm/): correct (tests/test_gemm_8p.py), but NOT a default.  On the
// Cellpose-SAM forward shapes it trails hipBLASLt by 15-35 % (8192x3072x1024: 70.2 vs 58.2 us;
// 8192x4096x1024: 78.9 vs 59.2; 4096^3: 1,276 vs 1,466 TF/s) and gemm_mt on the N = 1024 shapes
// (128 blocks on 256 CUs).  A persistent variant (one block per CU, cross-tile DMA cursors, the
// epilogue inside the K loop overlapping the other group's MFMAs) measured no better than one block
// per tile (gemm_8p_persistent_s2.jsonl; source kept as gemm_8p_persistent_variant.hip.txt).
//
// gemm_8p_notes (barrier instances numbered within tile t; group 0 passes instance 2p-1 before its
// phase-p MFMAs and 2p after them, group 1 one instance later):
//  - part X read in phase p is dead once group 1's phase-p MFMAs started (lgkmcnt(0) after instance
//    2p): instance 2p + 1 at the latest.  A[m0], B[n0]: read phase 1 -> refilled in phase 3 (group 0
//    issues after instance 4); B[n1]: phase 2 -> phase 4 (after 6); A[m1]: phase 3 -> next tile's
//    phase 1 (after 8).
//  - tile t+1 is read from instance 8 on (group 0's next phase-1 reads); its last DMA (A[m1], issued
//    in tile t's phase 1) is retired by the vmcnt(6) every wave executes before its phase-4 first
//    barrier (instance 7 / 8): the 6 younger DMAs are tile t+2's A[m0], B[n0], B[n1].
#include "common.h"

namespace {

typedef __attribute__((address_space(3))) void lds_void;

constexpr int BK = 64, NT8 = 512;
constexpr int IMG = 256 * 128;       // one operand image per buffer (bytes)
constexpr int BUF = 2 * IMG;         // A + B
constexpr int LDS8 = 2 * BUF;        // two buffers: 128 KiB

enum { E_NONE = 0, E_BIAS = 1, E_BIAS_GELU = 2, E_BIAS_RES = 6 };

constexpr int vm_imm(int n) { return (n & 0xf) | (0x7 << 4) | (0xf << 8) | ((n >> 4) << 14); }
template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt(vm_imm(N));
}
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xf | (0x7 << 4) | (0x3 << 14)); }
__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }

struct GArgs8 {
  const bf16_t* A;   // [M][lda] K-contiguous
  const bf16_t* B;   // [N][ldb] K-contiguous
  bf16_t* C;         // [M][ldc]
  bf16_t* C2;        // E_BIAS_GELU: gelu(C)
  const void* bias;  // [N] fp32 or bf16
  const bf16_t* aux; // E_BIAS_RES: residual [M][ldc]
  int bias_bf16;
  int M, N, K, lda, ldb, ldc;
  int tiles_n, tiles, nkt;
};

template <int EPI>
__global__ __launch_bounds__(NT8, 1) void gemm_8p_kernel(GArgs8 a) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;  // group = wr
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = lid / a.tiles_n, tn = lid - (lid / a.tiles_n) * a.tiles_n;
  const int m0 = tm * 256, n0 = tn * 256;
  const int nkt = a.nkt;

  // ---- DMA sources: part p of an image = LDS rows p*128 .. p*128+127, 16 wave-instructions of
  // 8 rows; this wave issues instructions i = 0, 1 -> LDS block b = i * 8 + wave.
  // A part p, LDS row R' (0..127) = wr' * 64 + j  <-  tile row wr' * 128 + p * 64 + j
  // B part p, LDS row R' = wc' * 32 + j           <-  tile col wc' * 64 + p * 32 + j
  const int lr = lane >> 3, pc = lane & 7;
  uint32_t aoff[2][2], boff[2][2];  // [part][i] element offsets (k0 = 0)
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int Rp = (i * 8 + wave) * 8 + lr;  // row within the part
      const int R = p * 128 + Rp;              // LDS row (swizzle key)
      const int c = pc ^ ((R >> 1) & 7);       // logical chunk this lane fetches
      int m = m0 + (Rp >> 6) * 128 + p * 64 + (Rp & 63);
      m = m < a.M ? m : a.M - 1;
      int n = n0 + (Rp >> 5) * 64 + p * 32 + (Rp & 31);
      n = n < a.N ? n : a.N - 1;
      aoff[p][i] = (uint32_t)m * (uint32_t)a.lda + c * 8;
      boff[p][i] = (uint32_t)n * (uint32_t)a.ldb + c * 8;
    }
  // DMA of part p of operand X (0 = A, 1 = B) of K-tile t into buffer t & 1; tiles past the end
  // re-read the last one into a dead part, so every phase issues a fixed count (exact vmcnt)
  auto dma = [&](int X, int p, int t) {
    const int k0 = (t < nkt ? t : nkt - 1) * BK;
    unsigned char* dst = smem + (t & 1) * BUF + X * IMG + p * (IMG / 2);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bf16_t* src = X == 0 ? a.A + aoff[p][i] + k0 : a.B + boff[p][i] + k0;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(dst + (i * 8 + wave) * 1024), 16, 0, 0);
    }
  };

  // ---- fragment reads: row tile of 16 at LDS row R0 + (lane & 15), k chunk ks * 4 + (lane >> 4)
  const int frow = lane & 15, fch = lane >> 4, fsw = (frow >> 1) & 7;
  const int rb0 = frow * 128 + ((fch ^ fsw) << 4), rb1 = frow * 128 + (((4 + fch) ^ fsw) << 4);
  // A quadrant mq: LDS rows mq*128 + wr*64 + i*16 (i < 4); B quadrant nq: nq*128 + wc*32 + jj*16
  auto read_a = [&](int t, int mq, bf16x8 (&fa)[4][2]) {
    const unsigned char* s = smem + (t & 1) * BUF + (mq * 128 + wr * 64) * 128;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fa[i][0] = *reinterpret_cast<const bf16x8*>(s + i * 16 * 128 + rb0);
      fa[i][1] = *reinterpret_cast<const bf16x8*>(s + i * 16 * 128 + rb1);
    }
  };
  auto read_b = [&](int t, int nq, bf16x8 (&fb)[2][2]) {
    const unsigned char* s = smem + (t & 1) * BUF + IMG + (nq * 128 + wc * 32) * 128;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      fb[j][0] = *reinterpret_cast<const bf16x8*>(s + j * 16 * 128 + rb0);
      fb[j][1] = *reinterpret_cast<const bf16x8*>(s + j * 16 * 128 + rb1);
    }
  };

  f32x4 acc[4][8];  // [n fragment (nq*2 + jj)][m fragment (mq*4 + i)]
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = (f32x4){0.f, 0.f, 0.f, 0.f};

  bf16x8 fa[4][2], fb0[2][2], fb1[2][2];
  auto mma = [&](int mq, int nq, const bf16x8 (&fb)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[nq * 2 + j][mq * 4 + i] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][ks], fa[i][ks], acc[nq * 2 + j][mq * 4 + i], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // ---- prologue: tile 0 whole, tile 1 without A[m1] (issued in tile 0's phase 1)
  dma(0, 0, 0); dma(0, 1, 0); dma(1, 0, 0); dma(1, 1, 0);
  dma(0, 0, 1); dma(1, 0, 1); dma(1, 1, 1);
  wait_vm<6>();
  bar();
  if (wr == 1) bar();  // the stagger: group 1 runs one barrier behind group 0

  for (int t = 0; t < nkt; ++t) {
    // phase 1: quadrant (m0, n0)
    read_a(t, 0, fa);
    read_b(t, 0, fb0);
    dma(0, 1, t + 1);
    bar();
    wait_lgkm0();
    __builtin_amdgcn_sched_barrier(0);
    mma(0, 0, fb0);
    bar();
    // phase 2: (m0, n1)
    read_b(t, 1, fb1);
    bar();
    wait_lgkm0();
    __builtin_amdgcn_sched_barrier(0);
    mma(0, 1, fb1);
    bar();
    // phase 3: (m1, n1)
    read_a(t, 1, fa);
    dma(0, 0, t + 2);
    dma(1, 0, t + 2);
    bar();
    wait_lgkm0();
    __builtin_amdgcn_sched_barrier(0);
    mma(1, 1, fb1);
    bar();
    // phase 4: (m1, n0); tile t+1 must be whole before the next phase-1 reads
    dma(1, 1, t + 2);
    wait_vm<6>();
    bar();
    __builtin_amdgcn_sched_barrier(0);
    mma(1, 0, fb0);
    bar();
  }
  if (wr == 0) bar();  // balance the stagger
  wait_vm<0>();        // trailing re-read DMAs land before the block exits

  // ---- epilogue: acc[j][i] lane -> row m0 + wr*128 + i*16 + (lane & 15), cols n0 + wc*64 + j*16 + 4*(lane >> 4)
  const int nq4 = 4 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wc * 64 + j * 16 + nq4;
    const bool nok = n < a.N;  // N % 4 == 0 (host-checked)
    float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (EPI == E_BIAS || EPI == E_BIAS_GELU || EPI == E_BIAS_RES) {
      if (nok && a.bias) {
        if (a.bias_bf16) {
          const u32x2 w = *reinterpret_cast<const u32x2*>((const bf16_t*)a.bias + n);
          bv = make_float4(lo_bf(w[0]), hi_bf(w[0]), lo_bf(w[1]), hi_bf(w[1]));
        } else {
          bv = *reinterpret_cast<const float4*>((const float*)a.bias + n);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + wr * 128 + i * 16 + frow;
      if (!nok || m >= a.M) continue;
      const long long o = (long long)m * a.ldc + n;
      f32x4 v = acc[j][i];
      v[0] += bv.x; v[1] += bv.y; v[2] += bv.z; v[3] += bv.w;
      if constexpr (EPI == E_BIAS_RES) {
        const u32x2 r = *reinterpret_cast<const u32x2*>(a.aux + o);
        v[0] += lo_bf(r[0]); v[1] += hi_bf(r[0]); v[2] += lo_bf(r[1]); v[3] += hi_bf(r[1]);
      }
      u32x2 st;
      st[0] = pack2bf(v[0], v[1]);
      st[1] = pack2bf(v[2], v[3]);
      if (EPI != E_BIAS_GELU || a.C) *reinterpret_cast<u32x2*>(a.C + o) = st;
      if constexpr (EPI == E_BIAS_GELU) {
        u32x2 gt;
        gt[0] = pack2bf(gelu_erf(lo_bf(st[0])), gelu_erf(hi_bf(st[0])));
        gt[1] = pack2bf(gelu_erf(lo_bf(st[1])), gelu_erf(hi_bf(st[1])));
        *reinterpret_cast<u32x2*>(a.C2 + o) = gt;
      }
    }
  }
}

template <int EPI>
int launch_8p(GArgs8 a, hipStream_t s) {
  static bool attr[BE_MAX_DEV] = {};
  if (!attr[be_cur_dev()]) {
    if (hipFuncSetAttribute((const void*)gemm_8p_kernel<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS8) !=
        hipSuccess)
      return -30;
    attr[be_cur_dev()] = true;
  }
  a.tiles_n = (a.N + 255) / 256;
  const long long tiles = (long long)((a.M + 255) / 256) * a.tiles_n;
  if (tiles >= (1LL << 31)) return -31;
  a.tiles = (int)tiles;
  hipLaunchKernelGGL((gemm_8p_kernel<EPI>), dim3((unsigned)tiles), dim3(NT8), LDS8, s, a);
  return BE_CHECK_LAUNCH();
}

}  // namespace

extern "C" {

// C[M][N] (bf16) = A[M][K] . B[N][K]^T with epilogue epi: 0 none, 1 + bias, 2 + bias with
// C2 = gelu(C) (C may be null: gelu only), 6 + bias + residual aux[M][ldc].  K % 64 == 0, N % 4 == 0,
// lda / ldb % 8 == 0, and every element offset of A / B below 2^32.
int be_gemm_8p(const void* A, const void* B, void* C, void* C2, const void* bias, int bias_bf16, const void* aux, int M,
               int N, int K, int lda, int ldb, int ldc, int epi, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (K % BK || N % 4 || lda % 8 || ldb % 8 || ldc % 4) return -40;
  if ((unsigned long long)M * lda >= (1ULL << 32) || (unsigned long long)N * ldb >= (1ULL << 32)) return -44;
  if (epi == E_BIAS_GELU && !C2) return -41;
  if (epi == E_BIAS_RES && !aux) return -41;
  if (epi != E_BIAS_GELU && !C) return -41;
  GArgs8 a = {};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = (bf16_t*)C; a.C2 = (bf16_t*)C2; a.bias = bias;
  a.bias_bf16 = bias_bf16; a.aux = (const bf16_t*)aux;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.nkt = K / BK;
  switch (epi) {
    case E_NONE: return launch_8p<E_NONE>(a, s);
    case E_BIAS: return launch_8p<E_BIAS>(a, s);
    case E_BIAS_GELU: return launch_8p<E_BIAS_GELU>(a, s);
    case E_BIAS_RES: return launch_8p<E_BIAS_RES>(a, s);
  }
  return -42;
}

}  // extern "C"

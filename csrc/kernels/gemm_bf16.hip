// bf16 GEMM with fused epilogues for the Cellpose-SAM (ViT-L/8) training step (SURVEY.md §2.5 K8:
// "bf16/fp8 MFMA GEMMs, fused LayerNorm, GELU ..."), replacing the vendor GEMMs of
// train/cpsam_engine.py.  The reference trains this model through cellpose 4.0.7 + PyTorch
// (apps/cellpose-finetuning/main.py:1483-1546, fp32 semantics :1350-1358; kept by fp32 master
// weights and fp32 accumulation here).
//
//   C[m][n] = sum_k A(m, k) B(n, k)          A: [M][K] (TA 0) or [K][M] (TA 1)
//                                             B: [N][K] (TB 0) or [K][N] (TB 1)
//   linear  y = x W^T (+ b)    TA 0, TB 0      x [M][K], W [N][K]
//   dgrad   y = dy W           TA 0, TB 1      W [K][N] read as stored (no transposed copy)
//   wgrad   dW = dy^T x        TA 1, TB 1      fp32 out, split-K over the token dimension
//
// Epilogues: bias; bias + GELU with the pre-activation kept (MLP lin1: f and gelu(f) from one GEMM);
// GELU backward times the accumulator with the lin1 bias gradient reduced in the same pass (lin2
// dgrad: df = gelu'(f) * (dm W2), db = sum_rows df); fp32 weight-gradient slabs.
//
// MI355X design (cdna_hip_programming.md §5 "glds vs register staging", T1, T2, T10):
//  * block = BM x BN (256 x 128 on 8 waves, or 128 x 128 on 4 waves), wave tile 64 x 64 =
//    4 x 4 v_mfma_f32_16x16x32_bf16 tiles (64 fp32 accumulators); the MFMA's A operand is the N side
//    so each lane ends with 4 consecutive output columns of one row (8-/16-byte stores).
//  * BK = 64, THREE LDS stages filled by LDS-DMA (global_load_lds_dwordx4): the tile kt+2 DMA is in
//    flight across the barrier (raw s_barrier + counted vmcnt, never __syncthreads in the loop),
//    one barrier per K tile.
//  * K-contiguous operand tiles ([rows][64] bf16, 128-byte rows): 16-byte chunk c of row r sits at
//    c ^ ((r >> 1) & 7) -> every ds_read_b128 fragment read hits 16 distinct bank slots (exhaustive
//    check over the four lane groups and both K steps).  M/N-contiguous tiles ([64][cols]): read
//    transposed with ds_read_b64_tr_b16, chunk c of row k at c ^ 2 ((k & 3) | ((k >> 1) & 4)) ->
//    the 8 rows a 32-lane half reads get 8 distinct slot pairs.  Both swizzles live in the per-lane
//    DMA SOURCE address (the DMA destination is lane-linear).
//  * XCD-aware block order (T1): consecutive logical blocks share the A row panel; a split-K
//    group's slices are consecutive too.
#include <cstdlib>

#include "common.h"

namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int BK = 64;

// s_waitcnt immediate waiting for vmcnt <= n only (gfx9 encoding: vmcnt[3:0] | expcnt 7 | lgkmcnt 15 | vmcnt[5:4])
constexpr int vm_wait(int n) { return (n & 0xf) | (0x7 << 4) | (0xf << 8) | ((n >> 4) << 14); }

enum { E_NONE = 0, E_BIAS = 1, E_BIAS_GELU = 2, E_DGELU = 3, E_F32 = 4 };

struct GArgs {
  const bf16_t* A;
  const bf16_t* B;
  void* C;             // bf16 [M][ldc] (E_F32: fp32; split-K: slabs [split][M][ldc])
  bf16_t* C2;          // E_BIAS_GELU: gelu(f) [M][ldc]
  const float* bias;   // [N]
  const bf16_t* aux;   // E_DGELU: f [M][ldc]
  float* dbias;        // E_DGELU: += sum over rows of the output (fp32, pre-zeroed)
  int M, N, K, lda, ldb, ldc;
  int tiles_n, tiles, split, kchunk;
};

__device__ __forceinline__ int kswz(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int tswz(int k) { return 2 * ((k & 3) | ((k >> 1) & 4)); }

// DMA of a K-contiguous [R][64] tile (rows r0.., k0..) of a row-major [rows][ld] matrix.
template <int R, int NW>
__device__ __forceinline__ void dma_k(const bf16_t* __restrict__ g, int ld, int r0, int rmax, int k0, unsigned char* dst,
                                      int wave, int lane) {
#pragma unroll
  for (int j = 0; j < R / 8 / NW; ++j) {
    const int i = j * NW + wave;
    const int row = i * 8 + (lane >> 3);
    const int c = (lane & 7) ^ kswz(row);
    int gr = r0 + row;
    gr = gr < rmax ? gr : rmax - 1;  // ragged edge: any valid row, masked at the store
    __builtin_amdgcn_global_load_lds((const void*)(g + (long long)gr * ld + k0 + c * 8), (lds_void*)(dst + i * 1024),
                                     16, 0, 0);
  }
}

// DMA of an M/N-contiguous [64][C] tile (k rows k0.., columns c0..) of a row-major [K][ld] matrix.
template <int C, int NW>
__device__ __forceinline__ void dma_t(const bf16_t* __restrict__ g, int ld, int c0, int k0, unsigned char* dst, int wave,
                                      int lane) {
  constexpr int CPR = C / 8;        // 16-byte chunks per row
  constexpr int RPI = 64 / CPR;     // rows per 1 KiB DMA
#pragma unroll
  for (int j = 0; j < BK / RPI / NW; ++j) {
    const int i = j * NW + wave;
    const int row = i * RPI + lane / CPR;
    const int c = (lane % CPR) ^ tswz(row);
    __builtin_amdgcn_global_load_lds((const void*)(g + (long long)(k0 + row) * ld + c0 + c * 8),
                                     (lds_void*)(dst + i * 1024), 16, 0, 0);
  }
}

// 16x16x32 fragment (row r0 + (lane & 15), k-step ks) of a K-contiguous tile
__device__ __forceinline__ bf16x8 frag_k(const unsigned char* t, int r0, int ks, int lane) {
  const int row = r0 + (lane & 15);
  const int c = ks * 4 + (lane >> 4);
  return *reinterpret_cast<const bf16x8*>(t + row * 128 + ((c ^ kswz(row)) << 4));
}

// 16x16x32 fragment (column c0 + (lane & 15), k-step ks) of an M/N-contiguous [64][C] tile
template <int C>
__device__ __forceinline__ bf16x8 frag_t(const unsigned char* t, int c0, int ks, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int k = ks * 32 + g * 8 + q;
  const int ch = (c0 >> 3) + (p >> 1);
  const unsigned char* a0 = t + k * (C * 2) + ((ch ^ tswz(k)) << 4) + 8 * (p & 1);
  const unsigned char* a1 = t + (k + 4) * (C * 2) + ((ch ^ tswz(k + 4)) << 4) + 8 * (p & 1);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
  bf16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return v;
}

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_erf_grad(float x) {
  return 0.5f * (1.f + erff(x * 0.70710678118654752f)) + x * 0.3989422804014327f * __expf(-0.5f * x * x);
}

// wave tile = 16 FM (rows) x 16 FN (columns); block = WM x WN waves
template <int TA, int TB, int WM, int WN, int FM, int FN, int EPI>
__global__ __launch_bounds__(WM * WN * 64, 1) void gemm_bf16_kernel(GArgs a) {
  constexpr int NW = WM * WN;
  constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
  constexpr int ABYTES = BM * BK * 2, BBYTES = BN * BK * 2, SBYTES = ABYTES + BBYTES;
  constexpr int LOADS = BM / 8 / NW + BN / 8 / NW;  // DMAs per wave per stage (either layout)
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int sp = lid % a.split;
  const int tile = lid / a.split;
  const int tm = tile / a.tiles_n, tn = tile % a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kb = sp * a.kchunk;
  const int nk = min(a.kchunk, a.K - kb) / BK;

  auto stage = [&](int kt, unsigned char* buf) {
    const int k0 = kb + kt * BK;
    if constexpr (TA == 0) dma_k<BM, NW>(a.A, a.lda, m0, a.M, k0, buf, wave, lane);
    else dma_t<BM, NW>(a.A, a.lda, m0, k0, buf, wave, lane);
    if constexpr (TB == 0) dma_k<BN, NW>(a.B, a.ldb, n0, a.N, k0, buf + ABYTES, wave, lane);
    else dma_t<BN, NW>(a.B, a.ldb, n0, k0, buf + ABYTES, wave, lane);
  };

  f32x4 acc[FN][FM];  // [n frag][m frag]
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  stage(0, smem);
  if (nk > 1) stage(1, smem + SBYTES);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) __builtin_amdgcn_s_waitcnt(vm_wait(LOADS));  // tile kt landed, kt+1 in flight
    else __builtin_amdgcn_s_waitcnt(vm_wait(0));
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();  // every wave's DMA of kt is in; every wave is done reading kt-1
    __builtin_amdgcn_sched_barrier(0);  // no LDS read of tile kt is scheduled above the barrier
    if (kt + 2 < nk) stage(kt + 2, smem + ((kt + 2) % 3) * SBYTES);
    const unsigned char* ta = smem + (kt % 3) * SBYTES;
    const unsigned char* tb = ta + ABYTES;
    // both K-steps' fragments are read up front (two register sets): the MFMAs of step 0 run
    // while step 1's reads are in flight
    bf16x8 af[2][FM], bf[2][FN];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        if constexpr (TA == 0) af[ks][j] = frag_k(ta, wm * 16 * FM + j * 16, ks, lane);
        else af[ks][j] = frag_t<BM>(ta, wm * 16 * FM + j * 16, ks, lane);
      }
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        if constexpr (TB == 0) bf[ks][i] = frag_k(tb, wn * 16 * FN + i * 16, ks, lane);
        else bf[ks][i] = frag_t<BN>(tb, wn * 16 * FN + i * 16, ks, lane);
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[ks][i], af[ks][j], acc[i][j], 0, 0, 0);
  }

  // ---- epilogue: acc[i][j] lane -> row m = m0 + wm*64 + j*16 + (lane & 15),
  //                                  cols n = n0 + wn*64 + i*16 + 4*(lane >> 4) + 0..3
  const int ml = lane & 15, nq = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int n = n0 + wn * 16 * FN + i * 16 + nq;
    const bool nok = n < a.N;  // N % 4 == 0 (host-checked): a lane's 4 columns are all in or all out
    float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (EPI == E_BIAS || EPI == E_BIAS_GELU)
      if (nok && a.bias) bv = *reinterpret_cast<const float4*>(a.bias + n);
    float dsum[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = m0 + wm * 16 * FM + j * 16 + ml;
      const bool ok = nok && m < a.M;
      const long long o = (long long)m * a.ldc + n;
      f32x4 v = acc[i][j];
      if constexpr (EPI == E_F32) {
        if (ok) {
          float* c = reinterpret_cast<float*>(a.C) + (long long)sp * a.M * a.ldc + o;
          *reinterpret_cast<float4*>(c) = make_float4(v[0], v[1], v[2], v[3]);
        }
      } else if constexpr (EPI == E_DGELU) {
        u32x2 fr = ok ? *reinterpret_cast<const u32x2*>(a.aux + o) : (u32x2){0u, 0u};
        const float f0 = lo_bf(fr[0]), f1 = hi_bf(fr[0]), f2 = lo_bf(fr[1]), f3 = hi_bf(fr[1]);
        u32x2 st;
        st[0] = pack2bf(v[0] * gelu_erf_grad(f0), v[1] * gelu_erf_grad(f1));
        st[1] = pack2bf(v[2] * gelu_erf_grad(f2), v[3] * gelu_erf_grad(f3));
        if (ok) {
          *reinterpret_cast<u32x2*>(reinterpret_cast<bf16_t*>(a.C) + o) = st;
          dsum[0] += lo_bf(st[0]); dsum[1] += hi_bf(st[0]); dsum[2] += lo_bf(st[1]); dsum[3] += hi_bf(st[1]);
        }
      } else {
        v[0] += bv.x; v[1] += bv.y; v[2] += bv.z; v[3] += bv.w;
        u32x2 st;
        st[0] = pack2bf(v[0], v[1]);
        st[1] = pack2bf(v[2], v[3]);
        if (ok) {
          *reinterpret_cast<u32x2*>(reinterpret_cast<bf16_t*>(a.C) + o) = st;
          if constexpr (EPI == E_BIAS_GELU) {
            // gelu of the bf16-rounded pre-activation, the value the backward reads back
            u32x2 gt;
            gt[0] = pack2bf(gelu_erf(lo_bf(st[0])), gelu_erf(hi_bf(st[0])));
            gt[1] = pack2bf(gelu_erf(lo_bf(st[1])), gelu_erf(hi_bf(st[1])));
            *reinterpret_cast<u32x2*>(a.C2 + o) = gt;
          }
        }
      }
    }
    if constexpr (EPI == E_DGELU) {
      // column sums over this wave's 64 rows: the 16 lanes of a lane group share the columns
#pragma unroll
      for (int c = 0; c < 4; ++c) {
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) dsum[c] += __shfl_xor(dsum[c], off, 64);
      }
      if (ml == 0 && nok && a.dbias) {
#pragma unroll
        for (int c = 0; c < 4; ++c) atomicAdd(a.dbias + n + c, dsum[c]);
      }
    }
  }
}

__global__ __launch_bounds__(256) void slab_sum_kernel(const float* __restrict__ s, float* __restrict__ out, int split,
                                                       long long n4) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 acc = reinterpret_cast<const float4*>(s)[i];
    for (int k = 1; k < split; ++k) {
      const float4 v = reinterpret_cast<const float4*>(s + (long long)k * n4 * 4)[i];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    reinterpret_cast<float4*>(out)[i] = acc;
  }
}

template <int TA, int TB, int WM, int WN, int FM, int FN, int EPI>
int launch_gemm(GArgs a, hipStream_t s) {
  constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
  constexpr size_t LDS = 3 * (size_t)(BM + BN) * BK * 2;
  static bool attr[BE_MAX_DEV] = {};
  if (!attr[be_cur_dev()]) {
    if (hipFuncSetAttribute((const void*)gemm_bf16_kernel<TA, TB, WM, WN, FM, FN, EPI>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS) != hipSuccess)
      return -30;
    attr[be_cur_dev()] = true;
  }
  if ((TA == 1 && a.M % BM) || (TB == 1 && a.N % BN)) return -31;  // transposed tiles are read whole
  a.tiles_n = (a.N + BN - 1) / BN;
  a.tiles = ((a.M + BM - 1) / BM) * a.tiles_n;
  const long long nblk = (long long)a.tiles * a.split;
  hipLaunchKernelGGL((gemm_bf16_kernel<TA, TB, WM, WN, FM, FN, EPI>), dim3((unsigned)nblk), dim3(WM * WN * 64), LDS, s,
                     a);
  return BE_CHECK_LAUNCH();
}

}  // namespace

extern "C" {

// C = op(A) op(B)^T with a fused epilogue; see the header.  ta/tb: 0 = K-contiguous, 1 = M/N-contiguous.
// epi: 0 none, 1 bias, 2 bias + GELU (C = f, C2 = gelu(f)), 3 GELU backward (aux = f, dbias += column
// sums), 4 fp32 out.  cfg: 0 = 256 x 128 tile on 8 waves, 1 = 128 x 128 on 4 waves, 2 = 256 x 128 on 4
// waves (128 x 64 each), 3 = 128 x 256 on 4 waves (64 x 128 each).  split > 1 (fp32
// out only): K is split into `split` slices summed through `ws` (split * M * ldc floats).
int be_gemm_bf16(const void* A, const void* B, void* C, void* C2, const float* bias, const void* aux, float* dbias,
                 void* ws, long long ws_bytes, int M, int N, int K, int lda, int ldb, int ldc, int ta, int tb, int epi,
                 int cfg, int split, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (K % BK || N % 4 || lda % 8 || ldb % 8 || ldc % 4) return -40;
  if (split < 1 || K % (split * BK)) return -41;
  if (split > 1 && (epi != E_F32 || !ws || ws_bytes < (long long)split * M * ldc * 4)) return -42;
  GArgs a;
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = split > 1 ? ws : C; a.C2 = (bf16_t*)C2; a.bias = bias;
  a.aux = (const bf16_t*)aux; a.dbias = dbias;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.split = split; a.kchunk = K / split;
  int r = -43;
#define BE_GEMM_CFG(TA, TB, EPI)                                                                         \
  switch (cfg) {                                                                                         \
    case 0: r = launch_gemm<TA, TB, 4, 2, 4, 4, EPI>(a, s); break;  /* 256 x 128, 8 waves of 64 x 64 */  \
    case 1: r = launch_gemm<TA, TB, 2, 2, 4, 4, EPI>(a, s); break;  /* 128 x 128, 4 waves of 64 x 64 */  \
    case 2: r = launch_gemm<TA, TB, 2, 2, 8, 4, EPI>(a, s); break;  /* 256 x 128, 4 waves of 128 x 64 */ \
    case 3: r = launch_gemm<TA, TB, 2, 2, 4, 8, EPI>(a, s); break;  /* 128 x 256, 4 waves of 64 x 128 */ \
  }
  if (ta == 0 && tb == 0 && epi == E_NONE) { BE_GEMM_CFG(0, 0, E_NONE) }
  else if (ta == 0 && tb == 0 && epi == E_BIAS) { BE_GEMM_CFG(0, 0, E_BIAS) }
  else if (ta == 0 && tb == 0 && epi == E_BIAS_GELU) { BE_GEMM_CFG(0, 0, E_BIAS_GELU) }
  else if (ta == 0 && tb == 1 && epi == E_NONE) { BE_GEMM_CFG(0, 1, E_NONE) }
  else if (ta == 0 && tb == 1 && epi == E_DGELU) { BE_GEMM_CFG(0, 1, E_DGELU) }
  else if (ta == 1 && tb == 1 && epi == E_F32) { BE_GEMM_CFG(1, 1, E_F32) }
  else if (ta == 0 && tb == 0 && epi == E_F32) { BE_GEMM_CFG(0, 0, E_F32) }
#undef BE_GEMM_CFG
  if (r != 0 || split == 1) return r;
  const long long n4 = (long long)M * ldc / 4;
  int blocks = (int)((n4 + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(slab_sum_kernel, dim3(blocks), dim3(256), 0, s, (const float*)ws, (float*)C, split, n4);
  return BE_CHECK_LAUNCH();
}

}  // extern "C"

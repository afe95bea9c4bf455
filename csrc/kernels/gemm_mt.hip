// Macro-tile bf16 GEMM for the Cellpose-SAM linear layers (reference step
// apps/cellpose-finetuning/main.py:1483-1546, inference :4966-5144): one kernel family, one main loop,
// for every GEMM of the ViT-L training step and forward pass:
//
//   NT  C[M][N] = A[M][K] . B[N][K]^T          forward (x W^T), epilogues: bias, bias + GELU (pre-
//                                                activation kept), bias + residual
//   NN  C[M][N] = A[M][K] . B[K][N]            data gradient (dy W, W as stored), epilogue: GELU
//                                                backward gelu'(f) * (.) with the bias gradient
//   TN  C[M][N] = A[K][M]^T . B[K][N]  (fp32)  weight gradient (dy^T x over the tokens), written in
//                                                fp32 straight into the flat gradient buffer; split-K
//                                                slices reduced in the same launch by the last arriver
//
// MI355X design (cdna_hip_programming.md §5; MI355X_MICROARCH.md §LDS, §Register files):
//  * 4 waves (one per SIMD, __launch_bounds__(256, 1)), each owning a large output tile of
//    16FM x 16FN (up to 128 x 128: 256 fp32 accumulators), so every ds_read_b128 feeds FM or FN
//    MFMAs (0.25 LDS reads per v_mfma_f32_16x16x32_bf16 at 128 x 128) and one wave's MFMAs issue
//    back to back with the next k-step's fragment reads interleaved.
//  * K is consumed in 64-deep tiles staged by global_load_lds (16 B per lane) into full 128-byte
//    LDS rows: every DMA wave-instruction moves 8 whole 128-byte lines (the fragment-shaped 64-byte
//    row loads of the older kernels cost TA time, §5 "Projection GEMM" item 3).  NST stages, one
//    counted vmcnt + raw s_barrier per tile, placed in the middle of the last k-step's MFMAs: after
//    it the tile's stage is refilled with tile t + NST and the next tile's first fragment reads
//    issue under the remaining MFMAs.
//  * K-contiguous operands: row r, 16-byte chunk c stored at chunk c ^ ((r >> 1) & 7): the 16
//    lanes of each ds_read_b128 lane group ({0-3,12-15,20-27}, ...) hit 16 distinct bank slots.  The
//    swizzle lives in the per-lane DMA source address (the DMA destination is lane-linear).
//  * M/N-contiguous operands (the data gradient's W, both weight-gradient operands): [64 k][BN]
//    images read with ds_read_b64_tr_b16 (T10); chunk c of k-row k at c ^ tswz(k), conflict-free.
//  * XCD-aware block order (T1), a tile's split-K slices adjacent (same XCD: the reducer reads
//    slabs written on its own L2).
#include "common.h"

namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int BK = 64;

constexpr int vm_imm(int n) { return (n & 0xf) | (0x7 << 4) | (0xf << 8) | ((n >> 4) << 14); }

__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {
#define BE_VM_CASE(k) \
  case k: __builtin_amdgcn_s_waitcnt(vm_imm(k)); break;
    BE_VM_CASE(1) BE_VM_CASE(2) BE_VM_CASE(3) BE_VM_CASE(4) BE_VM_CASE(5) BE_VM_CASE(6) BE_VM_CASE(7)
    BE_VM_CASE(8) BE_VM_CASE(10) BE_VM_CASE(12) BE_VM_CASE(14) BE_VM_CASE(16) BE_VM_CASE(20) BE_VM_CASE(24)
    BE_VM_CASE(28) BE_VM_CASE(32) BE_VM_CASE(36) BE_VM_CASE(40) BE_VM_CASE(48)
#undef BE_VM_CASE
    default: __builtin_amdgcn_s_waitcnt(vm_imm(0)); break;
  }
}

template <int N>
__device__ __forceinline__ void wait_vm_c() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt(vm_imm(N));
}

// lgkmcnt(0), vmcnt / expcnt untouched
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xf | (0x7 << 4) | (0x3 << 14)); }

__device__ __forceinline__ int tswz(int k) { return 2 * ((k & 3) | ((k >> 1) & 4)); }

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_erf_grad(float x) {
  return 0.5f * (1.f + erff(x * 0.70710678118654752f)) + x * 0.3989422804014327f * __expf(-0.5f * x * x);
}

// 16x16x32 operand fragment (column c0 + (lane & 15), k 0..31) of a [32 k][C] image, transposed read
template <int C>
__device__ __forceinline__ bf16x8 frag_t(const unsigned char* t, int c0, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int k = g * 8 + q;
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

enum { E_NONE = 0, E_BIAS = 1, E_BIAS_GELU = 2, E_DGELU = 4, E_F32 = 5, E_BIAS_RES = 6, E_CONV = 7 };

struct MArgs {
  const bf16_t* A;      // TA 0: [M][lda] (K-contiguous); TA 1: [K][lda] (M-contiguous)
  const bf16_t* B;      // TB 0: [N][ldb] (K-contiguous); TB 1: [K][ldb] (N-contiguous)
  bf16_t* C;            // bf16 [M][ldc]
  bf16_t* C2;           // E_BIAS_GELU: gelu(C)
  const void* bias;     // [N], fp32 or bf16 (bias_bf16)
  const bf16_t* aux;    // E_DGELU: pre-activation f [M][ldc]; E_BIAS_RES: residual [M][ldc]
  float* dbias;         // E_DGELU: += column sums of C (fp32, pre-zeroed)
  float* Cf;            // E_F32: fp32 [M][ldc]
  float* ws;            // E_F32, split > 1: fp32 slabs [tiles * split][BM * BN]
  int* cnt;             // E_F32, split > 1: per-tile arrival counters (zero between calls)
  long long ws_bytes;
  int bias_bf16;
  int M, N, K, lda, ldb, ldc;
  int tiles_n, nkt, split;
  // TA 2 (implicit 3x3x3 conv): A = x NDHWC [M voxels][cin], K = 27 taps x cin (tap-major, padded to
  // 64 with the zero page), zero padding at the volume faces
  const bf16_t* zero;
  int D, H, W, cin, relu;
};

template <int WM, int WN, int FM, int FN, int NST, int EPI, int TA, int TB>
__global__ __launch_bounds__(64 * WM * WN) void gemm_mt_kernel(MArgs a) {
  constexpr int NW = WM * WN;                 // waves
  constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
  constexpr int ABY = BM * 128, STB = (BM + BN) * 128;
  constexpr int GA = BM / (8 * NW), GB = BN / (8 * NW), G = GA + GB;  // DMA wave-instructions per thread per tile
  constexpr int FH = FN / 2;                  // B fragments before the mid-tile barrier
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "whole DMA rounds");
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WN, wc = wave % WN;
  const int lid0 = xcd_remap(blockIdx.x, gridDim.x);
  const int sp = lid0 % a.split, tile = lid0 / a.split;
  const int tm = tile / a.tiles_n, tn = tile - (tile / a.tiles_n) * a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kt0 = (int)((long long)a.nkt * sp / a.split);
  const int nkt = (int)((long long)a.nkt * (sp + 1) / a.split) - kt0;

  // ---- per-thread DMA source (fixed over K except the k offset)
  // K-contiguous operand: wave-instruction i covers rows (4 i + wave) * 8 + lane / 8, 128 B each
  const int lr = lane >> 3;
  const int swzc = (lane & 7) ^ ((wave * 4 + (lr >> 1)) & 7);  // logical chunk this lane fetches
  // TA 2: this thread's DMA rows as output voxels (index, z, y, x), decoded once; z = -1: past M
  int vox[TA == 2 ? GA : 1], vz[TA == 2 ? GA : 1], vy[TA == 2 ? GA : 1], vx[TA == 2 ? GA : 1];
  if constexpr (TA == 2) {
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const int r = m0 + (i * NW + wave) * 8 + lr;
      const int rr = r < a.M ? r : a.M - 1;
      int q = rr / a.W;
      vx[i] = rr - q * a.W;
      const int q2 = q / a.H;
      vy[i] = q - q2 * a.H;
      vz[i] = r < a.M ? q2 - (q2 / a.D) * a.D : -1;
      vox[i] = rr;
    }
  }
  auto stage = [&](int t) {
    unsigned char* st = smem + (t % NST) * STB;
    // past the slice's end the DMA re-reads its last tile into a stage nothing reads any more: every
    // tile then issues exactly G DMAs and every wait below is a compile-time count
    const int k0 = (kt0 + (t < nkt ? t : nkt - 1)) * BK;
    if constexpr (TA == 0) {
#pragma unroll
      for (int i = 0; i < GA; ++i) {
        int r = m0 + (i * NW + wave) * 8 + lr;
        r = r < a.M ? r : a.M - 1;
        __builtin_amdgcn_global_load_lds((const void*)(a.A + (long long)r * a.lda + k0 + swzc * 8),
                                         (lds_void*)(st + (i * NW + wave) * 1024), 16, 0, 0);
      }
    } else if constexpr (TA == 2) {
      // this lane's 8-channel chunk of K: one tap (cin % 8 == 0), a whole-voxel shift of the row
      const int kg = k0 + swzc * 8;
      const int tap = kg / a.cin, ch = kg - tap * a.cin;
      const int dz = tap / 9 - 1, dy = (tap / 3) % 3 - 1, dx = tap % 3 - 1;
      const int off = (dz * a.H + dy) * a.W + dx;
#pragma unroll
      for (int i = 0; i < GA; ++i) {
        const bool ok = tap < 27 && vz[i] >= 0 && (unsigned)(vz[i] + dz) < (unsigned)a.D &&
                        (unsigned)(vy[i] + dy) < (unsigned)a.H && (unsigned)(vx[i] + dx) < (unsigned)a.W;
        const bf16_t* src = ok ? a.A + (long long)(vox[i] + off) * a.cin + ch : a.zero;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(st + (i * NW + wave) * 1024), 16, 0, 0);
      }
    } else {
      constexpr int CPR = BM / 8, RPI = 64 / CPR;
#pragma unroll
      for (int i = 0; i < GA; ++i) {
        const int blk = i * NW + wave;
        const int kr = blk * RPI + lane / CPR;
        const int c = (lane % CPR) ^ tswz(kr);
        // a partial last M tile (M % 8 == 0): chunks past M re-read the row's last chunk (their
        // output rows are never stored)
        int col = m0 + c * 8;
        col = col < a.M ? col : a.M - 8;
        __builtin_amdgcn_global_load_lds((const void*)(a.A + (long long)(k0 + kr) * a.lda + col),
                                         (lds_void*)(st + blk * 1024), 16, 0, 0);
      }
    }
    if constexpr (TB == 0) {
#pragma unroll
      for (int i = 0; i < GB; ++i) {
        int r = n0 + (i * NW + wave) * 8 + lr;
        r = r < a.N ? r : a.N - 1;
        __builtin_amdgcn_global_load_lds((const void*)(a.B + (long long)r * a.ldb + k0 + swzc * 8),
                                         (lds_void*)(st + ABY + (i * NW + wave) * 1024), 16, 0, 0);
      }
    } else {
      constexpr int CPR = BN / 8, RPI = 64 / CPR;
#pragma unroll
      for (int i = 0; i < GB; ++i) {
        const int blk = i * NW + wave;
        const int kr = blk * RPI + lane / CPR;
        const int c = (lane % CPR) ^ tswz(kr);
        int col = n0 + c * 8;
        col = col < a.N ? col : a.N - 8;
        __builtin_amdgcn_global_load_lds((const void*)(a.B + (long long)(k0 + kr) * a.ldb + col),
                                         (lds_void*)(st + ABY + blk * 1024), 16, 0, 0);
      }
    }
  };

  // ---- fragment reads of k-step ks (0 / 1) of the tile in stage t % NST
  const int frow = lane & 15, fch = lane >> 4, fsw = (frow >> 1) & 7;
  auto read_a = [&](int t, int ks, bf16x8* fa) {
    const unsigned char* st = smem + (t % NST) * STB;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      if constexpr (TA != 1) {
        const int r = wr * 16 * FM + i * 16 + frow;
        fa[i] = *reinterpret_cast<const bf16x8*>(st + r * 128 + (((ks * 4 + fch) ^ fsw) << 4));
      } else {
        fa[i] = frag_t<BM>(st + ks * 32 * BM * 2, wr * 16 * FM + i * 16, lane);
      }
    }
  };
  auto read_b = [&](int t, int ks, bf16x8* fb) {
    const unsigned char* st = smem + (t % NST) * STB + ABY;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      if constexpr (TB == 0) {
        const int r = wc * 16 * FN + j * 16 + frow;
        fb[j] = *reinterpret_cast<const bf16x8*>(st + r * 128 + (((ks * 4 + fch) ^ fsw) << 4));
      } else {
        fb[j] = frag_t<BN>(st + ks * 32 * BN * 2, wc * 16 * FN + j * 16, lane);
      }
    }
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int i = 0; i < FM; ++i) acc[j][i] = (f32x4){0.f, 0.f, 0.f, 0.f};

  bf16x8 fa0[FM], fb0[FN], fa1[FM], fb1[FN];

  // ---- prologue: tiles 0 .. NST-1 in flight, tile 0 landed everywhere
#pragma unroll
  for (int t = 0; t < NST; ++t) stage(t);
  wait_vm_c<G * (NST - 1)>();
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  read_b(0, 0, fb0);
  read_a(0, 0, fa0);
  wait_lgkm0();  // (as at the end of each iteration: nothing pending across the loop header)

  // ---- main loop: no branches inside (a branch here splits the accumulators over two register
  // sets joined by v_accvgpr copies); the last tile is peeled
  for (int t = 0; t < nkt - 1; ++t) {
    // tile t - 1's stage: every wave retired its reads of it before the barrier just passed
    read_b(t, 1, fb1);
    read_a(t, 1, fa1);
    __builtin_amdgcn_sched_barrier(0);  // the k-step-1 reads issue ahead of the k-step-0 MFMAs
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int i = 0; i < FM; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[j], fa0[i], acc[j][i], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < FH; ++j)
#pragma unroll
      for (int i = 0; i < FM; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[j], fa1[i], acc[j][i], 0, 0, 0);
    // this wave's DMAs of tile t + 1 landed, its reads of tile t retired: then the barrier
    __builtin_amdgcn_sched_barrier(0);
    wait_lgkm0();
    wait_vm_c<G * (NST - 2)>();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // every wave's reads of tile t retired before the barrier: its stage takes tile t + NST now, a
    // whole tile of MFMAs before that tile's wait (issued at the top of the tile it would leave only
    // half of one)
    stage(t + NST);
    read_b(t + 1, 0, fb0);
    read_a(t + 1, 0, fa0);
#pragma unroll
    for (int j = FH; j < FN; ++j)
#pragma unroll
      for (int i = 0; i < FM; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[j], fa1[i], acc[j][i], 0, 0, 0);
    // retire the next tile's k-step-0 reads here, so the back edge carries no pending LDS reads and
    // the compiler does not wait for the next k-step-1 reads before the first MFMA
    __builtin_amdgcn_sched_barrier(0);
    wait_lgkm0();
    __builtin_amdgcn_sched_barrier(0);
  }
  {
    const int t = nkt - 1;
    read_b(t, 1, fb1);
    read_a(t, 1, fa1);
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int i = 0; i < FM; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[j], fa0[i], acc[j][i], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int i = 0; i < FM; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[j], fa1[i], acc[j][i], 0, 0, 0);
  }
  wait_vm_c<0>();  // the trailing re-read DMAs land before the block exits or reuses its LDS

  // ---- epilogue: acc[j][i] lane -> row m0 + wr*16FM + i*16 + (lane & 15),
  //                                  cols n0 + wc*16FN + j*16 + 4*(lane >> 4) + 0..3
  const int nq = 4 * (lane >> 4);
  if constexpr (EPI == E_F32) {
    if (a.split > 1) {
      // split-K: fp32 slab in register-native order, then the last arriving slice of this tile sums
      // the others into its registers (release / acquire at agent scope, cdna_hip_programming.md
      // §5 "Projection GEMM at M = 256" item 2)
      float* slab = a.ws + ((long long)tile * a.split + sp) * (BM * BN);
      const int wbase = wave * (FM * FN * 256);
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int i = 0; i < FM; ++i)
          *reinterpret_cast<f32x4*>(slab + wbase + ((j * FM + i) * 64 + lane) * 4) = acc[j][i];
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      int* flag = reinterpret_cast<int*>(smem);
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int prev = __hip_atomic_fetch_add(a.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = prev == a.split - 1;
        if (last) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __hip_atomic_store(a.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        flag[0] = last;
      }
      __syncthreads();
      if (!flag[0]) return;
      for (int s = 0; s < a.split; ++s) {
        if (s == sp) continue;
        const float* o = a.ws + ((long long)tile * a.split + s) * (BM * BN) + wbase;
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int i = 0; i < FM; ++i) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(o + ((j * FM + i) * 64 + lane) * 4);
            acc[j][i] += v;
          }
      }
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wc * 16 * FN + j * 16 + nq;
      if (n >= a.N) continue;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int m = m0 + wr * 16 * FM + i * 16 + frow;
        if (m >= a.M) continue;
        const f32x4 v = acc[j][i];
        *reinterpret_cast<float4*>(a.Cf + (long long)m * a.ldc + n) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
    return;
  }

#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wc * 16 * FN + j * 16 + nq;
    const bool nok = n < a.N;  // N % 4 == 0 (host-checked)
    float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (EPI == E_BIAS || EPI == E_BIAS_GELU || EPI == E_BIAS_RES || EPI == E_CONV) {
      if (nok && a.bias) {
        if (a.bias_bf16) {
          const u32x2 w = *reinterpret_cast<const u32x2*>((const bf16_t*)a.bias + n);
          bv = make_float4(lo_bf(w[0]), hi_bf(w[0]), lo_bf(w[1]), hi_bf(w[1]));
        } else {
          bv = *reinterpret_cast<const float4*>((const float*)a.bias + n);
        }
      }
    }
    float dsum[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = m0 + wr * 16 * FM + i * 16 + frow;
      if (!nok || m >= a.M) continue;
      const long long o = (long long)m * a.ldc + n;
      f32x4 v = acc[j][i];
      if constexpr (EPI == E_DGELU) {
        const u32x2 fr = *reinterpret_cast<const u32x2*>(a.aux + o);
        u32x2 st;
        st[0] = pack2bf(v[0] * gelu_erf_grad(lo_bf(fr[0])), v[1] * gelu_erf_grad(hi_bf(fr[0])));
        st[1] = pack2bf(v[2] * gelu_erf_grad(lo_bf(fr[1])), v[3] * gelu_erf_grad(hi_bf(fr[1])));
        *reinterpret_cast<u32x2*>(a.C + o) = st;
        dsum[0] += lo_bf(st[0]); dsum[1] += hi_bf(st[0]); dsum[2] += lo_bf(st[1]); dsum[3] += hi_bf(st[1]);
        continue;
      }
      v[0] += bv.x; v[1] += bv.y; v[2] += bv.z; v[3] += bv.w;
      if constexpr (EPI == E_BIAS_RES) {
        const u32x2 r = *reinterpret_cast<const u32x2*>(a.aux + o);
        v[0] += lo_bf(r[0]); v[1] += hi_bf(r[0]); v[2] += lo_bf(r[1]); v[3] += hi_bf(r[1]);
      }
      u32x2 st;
      st[0] = pack2bf(v[0], v[1]);
      st[1] = pack2bf(v[2], v[3]);
      if constexpr (EPI == E_CONV) {
        if (a.relu) {
          st[0] = relu_bf16x2(st[0]);
          st[1] = relu_bf16x2(st[1]);
        }
      }
      if (EPI != E_BIAS_GELU || a.C) *reinterpret_cast<u32x2*>(a.C + o) = st;  // inference: gelu only
      if constexpr (EPI == E_BIAS_GELU) {
        u32x2 gt;
        gt[0] = pack2bf(gelu_erf(lo_bf(st[0])), gelu_erf(hi_bf(st[0])));
        gt[1] = pack2bf(gelu_erf(lo_bf(st[1])), gelu_erf(hi_bf(st[1])));
        *reinterpret_cast<u32x2*>(a.C2 + o) = gt;
      }
    }
    if constexpr (EPI == E_DGELU) {
      // column sums over this wave's rows: the 16 lanes of a lane group share the columns
#pragma unroll
      for (int c = 0; c < 4; ++c) {
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) dsum[c] += __shfl_xor(dsum[c], off, 64);
      }
      if (frow == 0 && nok && a.dbias) {
#pragma unroll
        for (int c = 0; c < 4; ++c) atomicAdd(a.dbias + n + c, dsum[c]);
      }
    }
  }
}

template <int WM, int WN, int FM, int FN, int NST, int EPI, int TA, int TB>
int launch_mt(MArgs a, hipStream_t s) {
  constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
  constexpr int LDS = NST * (BM + BN) * 128;
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static bool attr[BE_MAX_DEV] = {};
  if (!attr[be_cur_dev()]) {
    if (hipFuncSetAttribute((const void*)gemm_mt_kernel<WM, WN, FM, FN, NST, EPI, TA, TB>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, LDS) != hipSuccess)
      return -30;
    attr[be_cur_dev()] = true;
  }
  // M/N-contiguous images: [64][BM | BN] k-row tiles of whole 16-byte chunks, power-of-two widths
  static_assert((TA == 0 || (BM & (BM - 1)) == 0) && (TB == 0 || (BN & (BN - 1)) == 0), "swizzled k-row tiles");
  if ((TA == 1 && a.M % 8) || (TB == 1 && a.N % 8)) return -33;
  a.tiles_n = (a.N + BN - 1) / BN;
  const long long tiles = (long long)((a.M + BM - 1) / BM) * a.tiles_n;
  const long long nblk = tiles * a.split;
  if (nblk >= (1LL << 31)) return -31;
  if (a.split > a.nkt) return -34;
  if (a.split > 1 && a.ws_bytes < nblk * BM * BN * 4) return -35;  // fp32 slab per (tile, slice)
  hipLaunchKernelGGL((gemm_mt_kernel<WM, WN, FM, FN, NST, EPI, TA, TB>), dim3((unsigned)nblk), dim3(64 * WM * WN), LDS,
                     s, a);
  return BE_CHECK_LAUNCH();
}

// tile configurations: (WM x WN waves of 16FM x 16FN, NST LDS stages of (BM + BN) x 128 B)
//   0: 256 x 256, 8 waves of 128 x 64, 2 stages (128 KiB)   1: 256 x 192, 8 waves of 64 x 96, 2 (112 KiB)
//   2: 256 x 128, 4 waves of 128 x 64, 3 stages (144 KiB)   3: 128 x 256, 4 waves of 64 x 128, 3 (144 KiB)
//   4: 128 x 128, 4 waves of 64 x 64, 4 stages (128 KiB)
template <int EPI, int TA, int TB>
int launch_cfg(MArgs a, int cfg, hipStream_t s) {
  switch (cfg) {
    case 0: return launch_mt<2, 4, 8, 4, 2, EPI, TA, TB>(a, s);
    case 2: return launch_mt<2, 2, 8, 4, 3, EPI, TA, TB>(a, s);
    case 3: return launch_mt<2, 2, 4, 8, 3, EPI, TA, TB>(a, s);
    case 4: return launch_mt<2, 2, 4, 4, 4, EPI, TA, TB>(a, s);
    case 1:
      if constexpr (TB == 0 && TA == 0) return launch_mt<4, 2, 4, 6, 2, EPI, TA, TB>(a, s);
      return -32;
  }
  return -32;
}

// implicit 3x3x3 conv tiles (narrow Cout): 5 = 256 x 32, 6 = 256 x 64 (4 waves of 64 x 32 / 64 x 64),
// 4 = 128 x 128, 2 = 256 x 128
int launch_conv(MArgs a, int cfg, hipStream_t s) {
  switch (cfg) {
    case 5: return launch_mt<4, 1, 4, 2, 4, E_CONV, 2, 0>(a, s);
    case 6: return launch_mt<4, 1, 4, 4, 3, E_CONV, 2, 0>(a, s);
    case 4: return launch_mt<2, 2, 4, 4, 4, E_CONV, 2, 0>(a, s);
    case 2: return launch_mt<2, 2, 8, 4, 3, E_CONV, 2, 0>(a, s);
  }
  return -32;
}

const bf16_t* conv_zero_page() { return be_zero_page(1, 4096); }

}  // namespace

extern "C" {

// bf16 GEMM family (see the file comment).  ta / tb: operand layouts (0 = K-contiguous rows, 1 =
// K-major [K][M | N]).  epi: 0 none, 1 + bias, 2 + bias with C2 = gelu(C), 4 GELU backward
// C = gelu'(aux) * (A B) with dbias += column sums, 5 fp32 out into Cf (split-K slices reduced
// in-launch through ws / cnt), 6 + bias + residual aux.  cfg: tile configuration (launch_cfg).
int be_gemm_mt(const void* A, const void* B, void* C, void* C2, const void* bias, int bias_bf16, const void* aux,
               float* dbias, float* Cf, float* ws, long long ws_bytes, int* cnt, int M, int N, int K, int lda,
               int ldb, int ldc, int ta, int tb, int epi, int cfg, int split, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (K % BK || N % 4 || lda % 8 || ldb % 8 || ldc % 4) return -40;
  if (epi == E_BIAS_GELU && !C2) return -41;
  if ((epi == E_DGELU || epi == E_BIAS_RES) && !aux) return -41;
  if (epi == E_F32 && !Cf) return -41;
  if (epi != E_F32 && epi != E_BIAS_GELU && !C) return -41;
  if (split < 1 || (split > 1 && epi != E_F32)) return -42;
  MArgs a = {};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = (bf16_t*)C; a.C2 = (bf16_t*)C2; a.bias = bias;
  a.bias_bf16 = bias_bf16; a.aux = (const bf16_t*)aux; a.dbias = dbias; a.Cf = Cf; a.ws = ws; a.cnt = cnt;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.nkt = K / BK; a.split = split;
  if (split > 1 && (!ws || !cnt)) return -43;
  a.ws_bytes = ws_bytes;
#ifdef GMT_PROBE  // build-time register probe of one configuration
  return launch_mt<GMT_PROBE, E_NONE, 0, 0>(a, s);
#else
  if (ta == 0 && tb == 0) {
    switch (epi) {
      case E_NONE: return launch_cfg<E_NONE, 0, 0>(a, cfg, s);
      case E_BIAS: return launch_cfg<E_BIAS, 0, 0>(a, cfg, s);
      case E_BIAS_GELU: return launch_cfg<E_BIAS_GELU, 0, 0>(a, cfg, s);
      case E_BIAS_RES: return launch_cfg<E_BIAS_RES, 0, 0>(a, cfg, s);
    }
  } else if (ta == 0 && tb == 1) {
    switch (epi) {
      case E_NONE: return launch_cfg<E_NONE, 0, 1>(a, cfg, s);
      case E_DGELU: return launch_cfg<E_DGELU, 0, 1>(a, cfg, s);
    }
  } else if (ta == 1 && tb == 1) {
    if (epi == E_F32) return launch_cfg<E_F32, 1, 1>(a, cfg, s);
  }
  return -42;
#endif
}

// 3x3x3 / stride 1 / zero-pad 1 conv of x NDHWC bf16 [N][D][H][W][cin] (cin % 8 == 0) with w bf16
// [cout][kpad] (k = tap * cin + c, tap = 9 dz + 3 dy + dx, zero past 27 cin; kpad % 64 == 0):
// out NDHWC [N][D][H][W][cout] = relu?(conv + bias[cout] (fp32)).  One launch over the whole batch,
// fp32 accumulation across all 27 taps.  cfg: 5 / 6 / 4 / 2 (launch_conv).
int be_conv3d_mt(const void* x, const void* w, const float* bias, void* out, int N, int D, int H, int W, int cin,
                 int cout, int kpad, int relu, int cfg, hipStream_t s) {
  if (cin % 8 || cout % 4 || kpad % BK || kpad < 27 * cin || kpad - 27 * cin >= BK) return -10;
  const long long M = (long long)N * D * H * W;
  if (M >= (1LL << 31) || M * cin >= (1LL << 40)) return -11;
  MArgs a = {};
  a.A = (const bf16_t*)x; a.B = (const bf16_t*)w; a.C = (bf16_t*)out; a.bias = bias; a.bias_bf16 = 0;
  a.M = (int)M; a.N = cout; a.K = kpad; a.lda = cin; a.ldb = kpad; a.ldc = cout; a.nkt = kpad / BK; a.split = 1;
  a.zero = conv_zero_page();
  if (!a.zero) return -13;
  a.D = D; a.H = H; a.W = W; a.cin = cin; a.relu = relu;
  return launch_conv(a, cfg, s);
}

}  // extern "C"

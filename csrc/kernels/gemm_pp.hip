// Ping-pong bf16 GEMM: 8 waves in two staggered groups over a 4-slot LDS-DMA ring of K-halves.
// Serves two hot paths with one main loop:
//   * GEMM   C[M][N] = A[M][K] B[N][K]^T (+ bias, + GELU with the pre-activation kept) -- the
//     large-M linear layers of the Cellpose-SAM training step (reference step
//     apps/cellpose-finetuning/main.py:1483-1546);
//   * CONV3  the deep 3x3 convolutions of the Cellpose CPnet as an implicit GEMM
//     over NHWC pixels: M = N*H*W output pixels, K = 9 taps x Cin, B = weights [Cout][3][3][Cin].
//     The A rows of a K-half are the tile's pixels shifted by the tap offset; a lane whose shifted
//     pixel falls outside its image points its DMA at a zero page (the conv's zero padding), so
//     the input stays in its plain NHWC layout.  The epilogue is the CPnet one: + bias + residual
//     (+ ReLU), and optionally the consumer's BN + ReLU (+ style shift) on the bf16 result.
//
// MI355X design (cdna_hip_programming.md §5 "The 256² 8-phase template", T2-T5):
//  * block = BM x BN on 8 waves (wave tile 16 FM x 16 FN: 128 x 64 or 64 x 64), one block per CU.
//  * K is consumed in K-halves of 32: a K-half is two PHASES (the wave's top and bottom row
//    halves), 16 or 8 v_mfma_f32_16x16x32_bf16 each.  A phase = fragment reads + its share of the
//    DMA prefetch, raw s_barrier, the MFMA cluster (s_setprio 1), raw s_barrier.
//  * the two wave groups (waves 0-3, 4-7: one of each per SIMD) run one barrier apart, so on every
//    SIMD one wave issues MFMAs while its partner reads LDS and issues DMA.
//  * LDS = 4 slots x (BM + BN) x 64 B, filled by global_load_lds three K-halves ahead; part 0 of
//    a K-half (B + the A top half) is staged in the phase after the slot's previous top-half
//    reads retired, part 1 (the A bottom half) one phase later, and each wave waits with a
//    counted vmcnt (never 0 in the loop) one phase before the first read of a K-half.
//  * 64-byte LDS rows, 16-byte chunk c of row r at c ^ g((r >> 2) & 3), g = {0, 2, 3, 1}: every
//    ds_read_b128 lane group (4 x 16 lanes: {0-3, 12-15, 20-27}, ...) hits 16 distinct bank slots.
//    The swizzle lives in the per-lane DMA source address (the DMA destination is lane-linear).
//  * XCD-aware block order (T1); N tiles of one M panel are consecutive.
#include "common.h"

namespace {

typedef __attribute__((address_space(3))) void lds_void;

constexpr int KH = 32;      // K-half depth
constexpr int NSLOT = 4;    // LDS ring slots
constexpr int DPRE = 3;     // K-halves staged ahead

constexpr int vm_imm(int n) { return (n & 0xf) | (0x7 << 4) | (0xf << 8) | ((n >> 4) << 14); }

__device__ __forceinline__ void wait_vm_dyn(int n) {
  switch (n) {
#define BE_VM_CASE(k) \
  case k: __builtin_amdgcn_s_waitcnt(vm_imm(k)); break;
    BE_VM_CASE(1) BE_VM_CASE(2) BE_VM_CASE(3) BE_VM_CASE(4) BE_VM_CASE(5) BE_VM_CASE(6) BE_VM_CASE(7)
    BE_VM_CASE(8) BE_VM_CASE(9) BE_VM_CASE(10) BE_VM_CASE(11) BE_VM_CASE(12)
#undef BE_VM_CASE
    default: __builtin_amdgcn_s_waitcnt(vm_imm(0)); break;
  }
}

__device__ __forceinline__ int swz(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_erf_grad(float x) {
  return 0.5f * (1.f + erff(x * 0.70710678118654752f)) + x * 0.3989422804014327f * __expf(-0.5f * x * x);
}

// N-contiguous B ([K][N] in memory, the dgrad's W as stored): the slot's B region is [32 k][BN] bf16,
// read transposed with ds_read_b64_tr_b16; 16-byte chunk c of k-row k sits at c ^ tswz(k) (the 8
// k-rows a 32-lane half reads land on 8 distinct slot pairs).
__device__ __forceinline__ int tswz(int k) { return 2 * ((k & 3) | ((k >> 1) & 4)); }

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// 16x16x32 fragment (column c0 + (lane & 15), k 0..31) of a [32][C] k-row tile
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

enum { P_NONE = 0, P_BIAS = 1, P_BIAS_GELU = 2, P_CONV = 3, P_DGELU = 4, P_F32 = 5 };

struct PArgs {
  const bf16_t* A;     // GEMM: [M][lda]; CONV: x NHWC [M][Cin]
  const bf16_t* B;     // [N][ldb] (CONV: [Cout][9 * Cin])
  bf16_t* C;           // [M][ldc] (CONV: out, may be null)
  bf16_t* C2;          // P_BIAS_GELU: gelu(f)
  const float* bias;   // [N]
  const bf16_t* aux;   // P_DGELU: f [M][ldc]
  float* dbias;        // P_DGELU: += column sums of the output (fp32, pre-zeroed)
  const bf16_t* res;   // CONV: residual [M][ldc]
  bf16_t* aout;        // CONV: relu?(out * as + at)
  const float* as;     // [N]
  const float* at;     // [N] or [images][at_ns]
  const bf16_t* zero;  // CONV: zero page
  int at_ns, arelu, post_relu;
  int M, N, K, lda, ldb, ldc;
  int H, W, HW, cpt;   // CONV geometry; cpt = Cin / 32 (K-halves per tap)
  float* Cf;           // P_F32: fp32 [M][ldc] (split > 1: slabs [split][M][ldc])
  int tiles_n, nkh, split, kchunk;
};

template <int WM, int WN, int FM, int FN, int EPI, int TA, int TB>
__global__ __launch_bounds__(512, 1) void gemm_pp_kernel(PArgs a) {
  static_assert(WM * WN == 8, "8 waves");
  constexpr bool CONV = EPI == P_CONV;
  constexpr int HF = FM / 2;            // fragments per row half
  constexpr int HR = 16 * HF;           // rows per wave per half
  constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
  constexpr int ABYTES = BM * 64, SLOT = (BM + BN) * 64;
  constexpr int GA = BM / 256, GB = BN / 128, G = 2 * GA + GB;  // DMAs per thread: A half, B, K-half
  static_assert(BM % 256 == 0 && BN % 128 == 0, "whole DMA rounds");
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2;  // waves w and w + 4 share a SIMD
  const int wr = wave / WN, wn = wave % WN;
  const int lid0 = xcd_remap(blockIdx.x, gridDim.x);
  const int sp = lid0 % a.split, lid = lid0 / a.split;  // a tile's K slices run back to back
  const int tm = lid / a.tiles_n, tn = lid % a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nkh = a.nkh;
  const int kbase = sp * a.kchunk;

  // ---- this thread's DMA rows (fixed over K): A rows of both halves, B rows
  const int lr = wave * 16 + (lane >> 2);           // row within a 128-row DMA round
  const int lch = lane & 3;                          // LDS chunk position
  int arow[2][GA], ay[2][GA], ax[2][GA];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const int R = i * 128 + lr;                    // row within the half: [wr][HR]
      const int trow = (R / HR) * 2 * HR + h * HR + (R % HR);
      int m = m0 + trow;
      if (CONV) {
        if (m < a.M) {
          const int img = m / a.HW, rem = m - img * a.HW;
          ay[h][i] = rem / a.W;
          ax[h][i] = rem - ay[h][i] * a.W;
        } else {
          ay[h][i] = -4;  // every tap reads the zero page
          ax[h][i] = 0;
        }
      }
      arow[h][i] = m < a.M ? m : a.M - 1;
    }
  int brow[GB];
#pragma unroll
  for (int i = 0; i < GB; ++i) {
    const int n = n0 + i * 128 + lr;
    brow[i] = n < a.N ? n : a.N - 1;
  }

  auto stage = [&](int J, int part) {
    unsigned char* slot = smem + (J & (NSLOT - 1)) * SLOT;
    const int k0 = kbase + J * KH;
    if (part == 0) {
      if constexpr (TB == 0) {
#pragma unroll
        for (int i = 0; i < GB; ++i) {
          const int R = i * 128 + lr;
          const int c = lch ^ swz(R);
          __builtin_amdgcn_global_load_lds((const void*)(a.B + (long long)brow[i] * a.ldb + k0 + c * 8),
                                           (lds_void*)(slot + ABYTES + (i * 128 + wave * 16) * 64), 16, 0, 0);
        }
      } else {
        constexpr int CPR = BN / 8, RPI = 64 / CPR;  // 16-byte chunks per k-row, k-rows per 1 KiB DMA
#pragma unroll
        for (int i = 0; i < GB; ++i) {
          const int blk = i * 8 + wave;              // 1 KiB DMA block of the [32][BN] region
          const int kr = blk * RPI + lane / CPR;
          const int c = (lane % CPR) ^ tswz(kr);
          __builtin_amdgcn_global_load_lds((const void*)(a.B + (long long)(k0 + kr) * a.ldb + n0 + c * 8),
                                           (lds_void*)(slot + ABYTES + blk * 1024), 16, 0, 0);
        }
      }
    }
    int dy = 0, dx = 0, c0 = k0;
    if (CONV) {
      const int t = J / a.cpt;
      c0 = (J - t * a.cpt) * KH;
      dy = t / 3 - 1;
      dx = t - (t / 3) * 3 - 1;
    }
    if constexpr (TA == 1) {
      // M-contiguous A ([K][M], the wgrad's dy): half `part` is [32 k][BM/2 cols], cols [wr][HR]
      constexpr int CPR = BM / 16, RPI = 64 / CPR;
#pragma unroll
      for (int i = 0; i < GA; ++i) {
        const int blk = i * 8 + wave;
        const int kr = blk * RPI + lane / CPR;
        const int cl = 8 * ((lane % CPR) ^ tswz(kr));  // logical column of this lane's chunk
        const int m = (cl / HR) * 2 * HR + part * HR + (cl % HR);
        __builtin_amdgcn_global_load_lds((const void*)(a.A + (long long)(k0 + kr) * a.lda + m0 + m),
                                         (lds_void*)(slot + part * (32 * BM) + blk * 1024), 16, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const int R = part * (BM / 2) + i * 128 + lr;
      const int c = lch ^ swz(R);
      const bf16_t* src;
      if (CONV) {
        const int yy = ay[part][i] + dy, xx = ax[part][i] + dx;
        src = ((unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W)
                  ? a.A + (long long)(arow[part][i] + dy * a.W + dx) * a.lda + c0 + c * 8
                  : a.zero + c * 8;
      } else {
        src = a.A + (long long)arow[part][i] * a.lda + k0 + c * 8;
      }
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (lds_void*)(slot + (part * (BM / 2) + i * 128 + wave * 16) * 64), 16, 0, 0);
    }
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // ---- prologue: K-halves 0 .. DPRE-1 in flight, K-half 0 landed everywhere
  for (int J = 0; J < DPRE && J < nkh; ++J) {
    stage(J, 0);
    stage(J, 1);
  }
  wait_vm_dyn(G * min(DPRE - 1, nkh - 1));
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if (grp == 1) __builtin_amdgcn_s_barrier();  // the stagger: group 1 runs one barrier behind
  __builtin_amdgcn_sched_barrier(0);

  const int frow = lane & 15, fch = lane >> 4;
  bf16x8 af[HF], bfr[FN];
  for (int J = 0; J < nkh; ++J) {
    const unsigned char* slot = smem + (J & (NSLOT - 1)) * SLOT;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      // fragment reads of this phase
#pragma unroll
      for (int jj = 0; jj < HF; ++jj) {
        if constexpr (TA == 0) {
          const int R = s * (BM / 2) + wr * HR + jj * 16 + frow;
          af[jj] = *reinterpret_cast<const bf16x8*>(slot + R * 64 + ((fch ^ swz(R)) << 4));
        } else {
          af[jj] = frag_t<BM / 2>(slot + s * (32 * BM), wr * HR + jj * 16, lane);
        }
      }
      if (s == 0) {
#pragma unroll
        for (int i = 0; i < FN; ++i) {
          if constexpr (TB == 0) {
            const int R = wn * 16 * FN + i * 16 + frow;
            bfr[i] = *reinterpret_cast<const bf16x8*>(slot + ABYTES + R * 64 + ((fch ^ swz(R)) << 4));
          } else {
            bfr[i] = frag_t<BN>(slot + ABYTES, wn * 16 * FN + i * 16, lane);
          }
        }
      }
      // prefetch share: part s of K-half J + DPRE (its slot's part-s regions were last read a
      // phase ago by the lagging group, and those reads retired before the barrier just passed)
      if (J + DPRE < nkh) stage(J + DPRE, s);
      // one phase before K-half J+1 is first read: this wave's DMAs of it have landed
      if (s == 1 && J + 1 < nkh) wait_vm_dyn(G * min(DPRE - 1, nkh - 2 - J));
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int jj = 0; jj < HF; ++jj)
          acc[i][s * HF + jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[i], af[jj], acc[i][s * HF + jj], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();  // balance the stagger

  // ---- epilogue: acc[i][j] lane -> row wr*2HR + (j / HF)*HR + (j % HF)*16 + (lane & 15),
  //                                  cols wn*16FN + i*16 + 4*(lane >> 4) + 0..3
  const int nq = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int n = n0 + wn * 16 * FN + i * 16 + nq;
    const bool nok = n < a.N;  // N % 4 == 0 (host-checked)
    float4 bv = make_float4(0.f, 0.f, 0.f, 0.f), sv = make_float4(1.f, 1.f, 1.f, 1.f);
    if (nok && a.bias) bv = *reinterpret_cast<const float4*>(a.bias + n);
    if (CONV && nok && a.as) sv = *reinterpret_cast<const float4*>(a.as + n);
    float dsum[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = m0 + wr * 2 * HR + (j / HF) * HR + (j % HF) * 16 + frow;
      if (!nok || m >= a.M) continue;
      const long long o = (long long)m * a.ldc + n;
      f32x4 v = acc[i][j];
      if constexpr (EPI == P_F32) {
        *reinterpret_cast<float4*>(a.Cf + (long long)sp * a.M * a.ldc + o) = make_float4(v[0], v[1], v[2], v[3]);
        continue;
      }
      if constexpr (EPI == P_DGELU) {
        const u32x2 fr = *reinterpret_cast<const u32x2*>(a.aux + o);
        u32x2 st;
        st[0] = pack2bf(v[0] * gelu_erf_grad(lo_bf(fr[0])), v[1] * gelu_erf_grad(hi_bf(fr[0])));
        st[1] = pack2bf(v[2] * gelu_erf_grad(lo_bf(fr[1])), v[3] * gelu_erf_grad(hi_bf(fr[1])));
        *reinterpret_cast<u32x2*>(a.C + o) = st;
        dsum[0] += lo_bf(st[0]); dsum[1] += hi_bf(st[0]); dsum[2] += lo_bf(st[1]); dsum[3] += hi_bf(st[1]);
        continue;
      }
      v[0] += bv.x; v[1] += bv.y; v[2] += bv.z; v[3] += bv.w;
      if (CONV && a.res) {
        const u32x2 r = *reinterpret_cast<const u32x2*>(a.res + o);
        v[0] += lo_bf(r[0]); v[1] += hi_bf(r[0]); v[2] += lo_bf(r[1]); v[3] += hi_bf(r[1]);
      }
      u32x2 st;
      st[0] = pack2bf(v[0], v[1]);
      st[1] = pack2bf(v[2], v[3]);
      if (CONV && a.post_relu) {
        st[0] = relu_bf16x2(st[0]);
        st[1] = relu_bf16x2(st[1]);
      }
      if (a.C) *reinterpret_cast<u32x2*>(a.C + o) = st;
      if constexpr (EPI == P_BIAS_GELU) {
        u32x2 gt;
        gt[0] = pack2bf(gelu_erf(lo_bf(st[0])), gelu_erf(hi_bf(st[0])));
        gt[1] = pack2bf(gelu_erf(lo_bf(st[1])), gelu_erf(hi_bf(st[1])));
        *reinterpret_cast<u32x2*>(a.C2 + o) = gt;
      }
      if constexpr (CONV) {
        if (a.aout) {
          float4 tv = make_float4(0.f, 0.f, 0.f, 0.f);
          if (a.at) tv = *reinterpret_cast<const float4*>(a.at + (long long)(m / a.HW) * a.at_ns + n);
          u32x2 q;
          q[0] = pack2bf(fmaf(lo_bf(st[0]), sv.x, tv.x), fmaf(hi_bf(st[0]), sv.y, tv.y));
          q[1] = pack2bf(fmaf(lo_bf(st[1]), sv.z, tv.z), fmaf(hi_bf(st[1]), sv.w, tv.w));
          if (a.arelu) {
            q[0] = relu_bf16x2(q[0]);
            q[1] = relu_bf16x2(q[1]);
          }
          *reinterpret_cast<u32x2*>(a.aout + o) = q;
        }
      }
    }
    if constexpr (EPI == P_DGELU) {
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

template <int WM, int WN, int FM, int FN, int EPI, int TA, int TB>
int launch_pp(PArgs a, hipStream_t s) {
  constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
  constexpr int LDS = NSLOT * (BM + BN) * 64;
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static bool attr[BE_MAX_DEV] = {};
  if (!attr[be_cur_dev()]) {
    if (hipFuncSetAttribute((const void*)gemm_pp_kernel<WM, WN, FM, FN, EPI, TA, TB>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, LDS) != hipSuccess)
      return -30;
    attr[be_cur_dev()] = true;
  }
  if ((TB == 1 && a.N % BN) || (TA == 1 && a.M % BM)) return -33;  // k-row tiles are read whole
  a.tiles_n = (a.N + BN - 1) / BN;
  const long long nblk = (long long)((a.M + BM - 1) / BM) * a.tiles_n * a.split;
  if (nblk >= (1LL << 31)) return -31;
  hipLaunchKernelGGL((gemm_pp_kernel<WM, WN, FM, FN, EPI, TA, TB>), dim3((unsigned)nblk), dim3(512), LDS, s, a);
  return BE_CHECK_LAUNCH();
}

template <int EPI, int TB = 0, int TA = 0>
int launch_cfg(PArgs a, int cfg, hipStream_t s) {
  switch (cfg) {
    case 0: return launch_pp<2, 4, 8, 4, EPI, TA, TB>(a, s);  // 256 x 256, waves 128 x 64
    case 1: return launch_pp<4, 2, 8, 4, EPI, TA, TB>(a, s);  // 512 x 128, waves 128 x 64
    case 2: return launch_pp<4, 2, 4, 4, EPI, TA, TB>(a, s);  // 256 x 128, waves 64 x 64
  }
  return -32;
}

__global__ __launch_bounds__(256) void pp_slab_sum_kernel(const float* __restrict__ s, float* __restrict__ out, int split,
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

const bf16_t* zero_page() { return be_zero_page(2, 4096); }

}  // namespace

extern "C" {

// C = A op(B) with A [M][K] K-contiguous and B [N][K] (tb 0) or [K][N] (tb 1, the dgrad's W as
// stored).  epi 0 none, 1 + bias, 2 + bias and C2 = gelu(C) (tb 0), 4 GELU backward
// C = gelu'(aux) * (A B) with dbias += column sums (tb 1).  cfg: 0 = 256 x 256 tiles, 1 = 512 x 128,
// 2 = 256 x 128.
int be_gemm_pp(const void* A, const void* B, void* C, void* C2, const float* bias, const void* aux, float* dbias, int M,
               int N, int K, int lda, int ldb, int ldc, int tb, int epi, int cfg, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (K % KH || N % 4 || lda % 8 || ldb % 8 || ldc % 4) return -40;
  if (epi == P_BIAS_GELU && !C2) return -41;
  if (epi == P_DGELU && !aux) return -41;
  PArgs a = {};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = (bf16_t*)C; a.C2 = (bf16_t*)C2; a.bias = bias;
  a.aux = (const bf16_t*)aux; a.dbias = dbias;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.nkh = K / KH;
  a.split = 1; a.kchunk = K;
  if (tb == 0) {
    switch (epi) {
      case P_NONE: return launch_cfg<P_NONE>(a, cfg, s);
      case P_BIAS: return launch_cfg<P_BIAS>(a, cfg, s);
      case P_BIAS_GELU: return launch_cfg<P_BIAS_GELU>(a, cfg, s);
    }
  } else {
    switch (epi) {
      case P_NONE: return launch_cfg<P_NONE, 1>(a, cfg, s);
      case P_DGELU: return launch_cfg<P_DGELU, 1>(a, cfg, s);
    }
  }
  return -42;
}

// 3x3 / pad 1 conv of x NHWC bf16 [N][H][W][Cin] with w bf16 [Cout][3][3][Cin]:
//   out  = conv(x) + bias (+ res) (relu if post_relu)                  (bf16, optional)
//   aout = relu?(out * as[c] + at[n][c])                                (bf16, optional)
int be_conv3_pp(const void* x, const void* w, const float* bias, const void* res, void* out, void* aout,
                const float* as, const float* at, int at_ns, int arelu, int post_relu, int N, int H, int W, int Cin,
                int Cout, int cfg, hipStream_t s) {
  if (Cin % KH || Cout % 4 || (long long)N * H * W >= (1LL << 31)) return -10;
  if (!out && !aout) return -11;
  PArgs a = {};
  a.A = (const bf16_t*)x; a.B = (const bf16_t*)w; a.C = (bf16_t*)out; a.bias = bias; a.res = (const bf16_t*)res;
  a.aout = (bf16_t*)aout; a.as = as; a.at = at; a.at_ns = at_ns; a.arelu = arelu; a.post_relu = post_relu;
  a.zero = zero_page();
  if (!a.zero) return -13;
  a.M = N * H * W; a.N = Cout; a.K = 9 * Cin; a.lda = Cin; a.ldb = 9 * Cin; a.ldc = Cout;
  a.H = H; a.W = W; a.HW = H * W; a.cpt = Cin / KH; a.nkh = 9 * Cin / KH;
  a.split = 1; a.kchunk = a.K;
  return launch_cfg<P_CONV>(a, cfg, s);
}

// Weight gradient out (fp32 [M][ldc]) = A^T B over K tokens with A [K][M] (dy) and B [K][N] (x), both
// read as stored (transposed in LDS).  split > 1: K is cut into `split` slices written as fp32 slabs
// into ws (split * M * ldc floats) and summed by a second pass.  M % BM == 0 and N % BN == 0.
int be_wgrad_pp(const void* A, const void* B, float* out, void* ws, long long ws_bytes, int M, int N, int K, int lda,
                int ldb, int ldc, int cfg, int split, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (N % 4 || lda % 8 || ldb % 8 || ldc % 4) return -40;
  if (split < 1 || K % (split * KH)) return -41;
  if (split > 1 && (!ws || ws_bytes < (long long)split * M * ldc * 4)) return -42;
  PArgs a = {};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.Cf = split > 1 ? (float*)ws : out;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.split = split; a.kchunk = K / split; a.nkh = a.kchunk / KH;
  const int r = launch_cfg<P_F32, 1, 1>(a, cfg, s);
  if (r != 0 || split == 1) return r;
  const long long n4 = (long long)M * ldc / 4;
  int blocks = (int)((n4 + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(pp_slab_sum_kernel, dim3(blocks), dim3(256), 0, s, (const float*)ws, out, split, n4);
  return BE_CHECK_LAUNCH();
}

}  // extern "C"

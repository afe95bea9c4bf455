// FP8 (OCP e4m3fn) GEMM on the CDNA4 block-scaled MFMA, for the ViT linear layers of the
// cell-image-search embedder (DINOv2 ViT-B/14, reference apps/cell-image-search/embedder.py:35-57,
// SURVEY.md §2.5 K8; BASELINE.json config "ViT-B embedding extraction, CDNA4 fp8 MFMA").
//
//   Y[M,N] (bf16) = epi( (Xq[M,K] . Wq[N,K]^T) * sx[m] * sw[n] + bias[n] )
//
// * Xq: activations quantised per row (token) with sx[m] = amax_k|x[m,k]| / 448 by
//   be_quant_fp8_rows below; Wq: weights quantised per output channel once at load time.
// * The matrix core is v_mfma_scale_f32_16x16x128_f8f6f4 with e4m3 operands and unit E8M0 block
//   scales (0x7f = 2^0): K = 128 per instruction at twice the bf16 MFMA rate.  The per-row /
//   per-column dequantisation scales are applied once in the fp32 epilogue, not per k-block.
// * Tiles: 128x128 (4 waves), 256x128 / 128x256 (8 waves, 64x64 per wave = 4x4 MFMA tiles) or
//   256x256 (8 waves, 128x64 per wave), K-step 128; chosen by shape so the grid fills 256 CUs while
//   the bigger tiles halve the L2->LDS bytes per FLOP.  Both operands are staged HBM -> LDS with global_load_lds_dwordx4 (no VGPR
//   round trip) into two LDS buffers; the LDS image is linear per wave-instruction and the 16-byte
//   chunk index of each 128-byte row is XOR-swizzled (frag_swz: conflict-free ds_read_b128) on the SOURCE address and on
//   the ds_read address (cdna_hip_programming.md §5.4 rule 21), so the 16 rows a fragment read
//   touches fall on distinct bank groups.
// * The next K-tile's DMA stays in flight across the barrier (raw s_barrier + counted vmcnt),
//   overlapping the current tile's 16 MFMAs per wave.
// * The MFMA's "A" operand is the weight tile and "B" the activation tile, so the accumulator of
//   each lane holds 4 consecutive output channels of one token: the epilogue writes 8-byte packed
//   bf16 runs along N (the row-major output's contiguous axis).
// * Block -> tile mapping is XCD-aware (common.h xcd_remap): consecutive tiles of one M-panel run
//   on one XCD and share its L2 copy of the activation panel.
// * MX-fp8 activations (XS): E8M0 scales per row and 32-wide K block go into the MFMA's scale
//   operand; each K step's [rows][4] scale bytes ride along with the tile (dword LDS-DMA) and are read
//   after the barrier like a fragment.  Producers: this kernel's EPI 2 (fc1: GELU + block
//   quantisation) and the attention epilogue (attention.hip, oq / os) for proj.
// * Nothing in the main loop waits on an ordinary global load: the epilogue operands (channel
//   scales, bias, row scales) are loaded before the K loop (or all at once at its end for the
//   256x256 tile) behind one unconditional wait, so no store waits for another round trip.
// * Default GEMM of Fp8Linear (ops/fp8.py); tile choice: pick_cfg.
#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(8))) int i32x8;

constexpr int BK = 128;                         // k-bytes (= e4m3 elements) per K-step
constexpr int E8M0_ONE = 0x7f7f7f7f;            // block scale 2^0 in every byte

typedef __attribute__((address_space(3))) void lds_void;

// s_waitcnt immediate (gfx9 encoding) waiting for vmcnt <= n only: vmcnt[3:0] | expcnt[6:4]=7 |
// lgkmcnt[11:8]=15 | vmcnt[5:4] at [15:14].
constexpr int waitcnt_vm(int n) { return (n & 0xf) | (0x7 << 4) | (0xf << 8) | ((n >> 4) << 14); }

// XOR applied to the 16-byte chunk index of tile row `row`.  A ds_read_b128 of read_frag serves
// four 16-lane groups, each = rows {0-3,12-15} at chunk c plus rows {4-11} at chunk c+2 (or the
// mirror); two 128-byte rows share one 256-byte bank row, so the slot of (row, c) is
// 8*(row&1) + (c ^ swz).  swz = row & 7 maps rows 4-11 onto the slots of rows 0-3/12-15 (every group
// 2-way: SQ_LDS_BANK_CONFLICT = 4 cycles per read, measured); swz = (row >> 1) & 5 puts all 16
// lanes of every group on distinct slots (exhaustive check over the four groups, both halves).
__device__ __forceinline__ int frag_swz(int row) { return (row >> 1) & 5; }

// Stage one R x 128-byte tile (rows r0.., k-bytes k0..) of a [rows, ld] fp8 matrix into LDS.
// Each wave-instruction writes 8 rows (1 KiB, lane-linear); row groups go round-robin over waves.
template <int R, int NW>
__device__ __forceinline__ void stage_tile(const uint8_t* __restrict__ g, long long ld, int r0, int rmax, int k0,
                                           uint8_t* lds_tile, int wave, int lane) {
  const int rin = lane >> 3;
#pragma unroll
  for (int j = 0; j < R / 8 / NW; ++j) {
    const int grp = j * NW + wave;
    const int chunk = (lane & 7) ^ frag_swz(grp * 8 + rin);  // inverse swizzle on the source (involution)
    int gr = r0 + grp * 8 + rin;
    gr = gr < rmax ? gr : rmax - 1;  // clamp ragged edges to a valid row; results are masked at store
    const uint8_t* src = g + (long long)gr * ld + k0 + chunk * 16;
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(lds_tile + grp * 1024), 16, 0, 0);
  }
}

// Fragment of a 16x128 (rows x k-bytes) slab for v_mfma_scale_f32_16x16x128_f8f6f4: lane l holds row
// (l & 15) as two swizzled 16-byte chunks.  FP8_KLAYOUT 0: k-bytes [32 (l>>4), +32); 1: [16 (l>>4), +16)
// and [64 + 16 (l>>4), +16).  Any layout shared by A and B gives the same plain GEMM; with block
// scales the instruction's own K order decides which elements a 32-block scale covers
// (tools/mx_scale_probe.py).
#ifndef FP8_KLAYOUT
#define FP8_KLAYOUT 1  // the instruction's own K order: a 32-block scale covers memory K [32b, 32b+32) (mx_scale_probe)
#endif
__device__ __forceinline__ i32x8 read_frag(const uint8_t* lds_tile, int row, int lane) {
  const int c0 = FP8_KLAYOUT ? (lane >> 4) : 2 * (lane >> 4);
  const int c1 = FP8_KLAYOUT ? c0 + 4 : c0 + 1;
  const int sw = frag_swz(row);
  const uint8_t* base = lds_tile + row * 128;
  const u32x4 lo = *reinterpret_cast<const u32x4*>(base + ((c0 ^ sw) << 4));
  const u32x4 hi = *reinterpret_cast<const u32x4*>(base + ((c1 ^ sw) << 4));
  i32x8 f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return f;
}

// GELU(x) = x * Phi(x) with a branch-free erf (Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7, far below
// the bf16 output's 2^-9 relative step): one v_rcp, one v_exp and a handful of FMAs, where the
// library erff takes range branches that diverge inside a wave.
__device__ __forceinline__ float gelu_erf(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float erf_z = 1.f - p * __expf(-z * z);  // erf(|x| / sqrt 2)
  const float phi = 0.5f + 0.5f * copysignf(erf_z, x);
  return x * phi;
}

// Block tile BM x BN = (WAVES_M * 16 * TM) x (WAVES_N * 16 * TN); each wave owns TM x TN MFMA tiles.
// PRIO: s_setprio(1) around the MFMA cluster (cdna_hip_programming.md T5).
// EPI 0: scale + bias -> bf16, 1: + GELU(erf) -> bf16, 2: + GELU -> MX-fp8 (e4m3 + one E8M0 scale per
// 32 consecutive outputs of a row, written to Yq / Ys): the next GEMM consumes it with XS = true.
// XS: X carries E8M0 block scales (one per row and 32-element K block, Xs [M, K/32]) that go into the
// MFMA's scale operand (scale_b: the lane's row / K block is exactly its fragment's 32 bytes), instead
// of a per-row fp32 scale in the epilogue.
template <int TM, int TN, int WAVES_M, int WAVES_N, int EPI, bool PRIO = false, bool XS = false>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void gemm_fp8_kernel(
    const uint8_t* __restrict__ X, const uint8_t* __restrict__ W, const float* __restrict__ sx,
    const float* __restrict__ sw, const float* __restrict__ bias, bf16_t* __restrict__ Y, int M, int N, int K,
    int tiles_n, const uint8_t* __restrict__ Xs = nullptr, uint8_t* __restrict__ Yq = nullptr,
    uint8_t* __restrict__ Ys = nullptr) {
  constexpr int NW = WAVES_M * WAVES_N;
  constexpr int BM = WAVES_M * 16 * TM, BN = WAVES_N * 16 * TN;
  constexpr int XB = BM * BK, BUF = (BM + BN) * BK;
  constexpr int LOADS = (BM + BN) / 8 / NW;  // glds per thread per K-step
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "row groups must split evenly over waves");
  // XS: one dword (a row's 4 E8M0 bytes of the K step) per lane; every wave issues XSL DMAs so the
  // counted waits stay uniform; lanes past BM reload rows modulo BM into a spare tail (harmless)
  constexpr int XSL = XS ? (BM + 64 * NW - 1) / (64 * NW) : 0;
  constexpr int SCB = XSL * NW * 64 * 4;            // LDS bytes per K step of scales
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * BUF + 2 * SCB];  // the only LDS object (rule 4a)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
  const int wm = (wave / WAVES_N) * 16 * TM, wn = (wave % WAVES_N) * 16 * TN;

  f32x4 acc[TN][TM];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Epilogue operands (per-channel scales, bias, per-token scales) loaded once, before the K loop:
  // they are in registers when the epilogue runs, so its stores never sit behind a load.  (Loaded
  // inside the epilogue, every 8-byte store was followed by the next column's scale load and an
  // s_waitcnt vmcnt(0) that also waited for the store's write acknowledgement: TM x TN serial
  // store + load round trips per tile.)
  // The 256x256 tile (TM * TN = 32) has no registers to spare across its K loop: it loads them all
  // together at the start of the epilogue instead (one exposed round trip, not TM x TN).
  constexpr bool EARLY_EPI_LOADS = TM * TN <= 16;
  float4 swv[TN], bvv[TN];
  float sxv[TM];
  auto load_epi = [&]() {
#pragma unroll
    for (int a = 0; a < TN; ++a) {
      const int n = min(n0 + wn + a * 16 + 4 * (lane >> 4), N - 4);
      swv[a] = *reinterpret_cast<const float4*>(sw + n);
      bvv[a] = bias ? *reinterpret_cast<const float4*>(bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int b = 0; b < TM; ++b) sxv[b] = XS ? 1.f : sx[min(m0 + wm + b * 16 + (lane & 15), M - 1)];
  };
  if constexpr (EARLY_EPI_LOADS) load_epi();

  const int nk = K / BK;
  const int kb32 = K / 32;
  // XS: the X block scales of each K step ride along with its tile: dword LDS-DMAs stage the BM
  // rows x 4 E8M0 bytes next to the tile, and each lane reads its (row, 32-block)
  // byte after the barrier like a fragment.  (Held in registers, the scales loaded for step kt+1
  // had to be copied into the set step kt+2 reads, and that copy compiled to an s_waitcnt
  // vmcnt(0) that drained the next tile's DMA every K step.)
  auto stage_xs = [&](int kt, uint8_t* dst) {
    if constexpr (XS) {
#pragma unroll
      for (int i = 0; i < XSL; ++i) {
        const int r = ((i * NW + wave) * 64 + lane) % BM;  // row whose 4 scale bytes this lane moves
        const int m = min(m0 + r, M - 1);
        __builtin_amdgcn_global_load_lds((const void*)(Xs + (long long)m * kb32 + kt * 4),
                                         (lds_void*)(dst + (i * NW + wave) * 256), 4, 0, 0);
      }
    }
  };
  stage_tile<BM, NW>(X, K, m0, M, 0, smem, wave, lane);
  stage_tile<BN, NW>(W, K, n0, N, 0, smem + XB, wave, lane);
  stage_xs(0, smem + 2 * BUF);
  for (int kt = 0; kt < nk; ++kt) {
    const uint8_t* buf = smem + (kt & 1) * BUF;
    if (kt + 1 < nk) {
      uint8_t* nxt = smem + ((kt + 1) & 1) * BUF;
      stage_tile<BM, NW>(X, K, m0, M, (kt + 1) * BK, nxt, wave, lane);
      stage_tile<BN, NW>(W, K, n0, N, (kt + 1) * BK, nxt + XB, wave, lane);
      stage_xs(kt + 1, smem + 2 * BUF + ((kt + 1) & 1) * SCB);
      __builtin_amdgcn_s_waitcnt(waitcnt_vm(LOADS + XSL));  // step kt landed; step kt+1 stays in flight
    } else {
      __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
    }
    __builtin_amdgcn_s_barrier();
    const uint8_t* xt = buf;
    const uint8_t* wt = buf + XB;
    int xsc[XS ? TM : 1];
    if constexpr (XS) {
      const uint8_t* sc = smem + 2 * BUF + (kt & 1) * SCB;
#pragma unroll
      for (int b = 0; b < TM; ++b) xsc[b] = sc[(wm + b * 16 + (lane & 15)) * 4 + (lane >> 4)];
    }
    i32x8 bx[TM];
#pragma unroll
    for (int b = 0; b < TM; ++b) bx[b] = read_frag(xt, wm + b * 16 + (lane & 15), lane);
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int a = 0; a < TN; ++a) {
      const i32x8 aw = read_frag(wt, wn + a * 16 + (lane & 15), lane);
#pragma unroll
      for (int b = 0; b < TM; ++b)
        acc[a][b] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(aw, bx[b], acc[a][b], 0, 0, 0, E8M0_ONE, 0,
                                                                     XS ? xsc[b] : E8M0_ONE);
    }
    if (PRIO) __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // WAR: the next iteration restages the buffer read here
  }
  // One unconditional wait for the hoisted epilogue operands: a wait the compiler places inside the
  // guarded (m < M, n < N) store blocks does not carry across their joins, so it would re-wait
  // (vmcnt(0), i.e. for every earlier store's acknowledgement too) before each of them.
  if constexpr (!EARLY_EPI_LOADS) load_epi();
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
  if constexpr (EPI == 2) {
    // GELU -> MX-fp8: a 32-output block of row m is tiles a, a+1 (16 columns each) x the 4 lane
    // groups sharing lane & 15 x 4 values; amax over it = lane-local max of 8 + two xor shuffles.
    static_assert(TN % 2 == 0, "MX blocks pair 16-column tiles");
#pragma unroll
    for (int b = 0; b < TM; ++b) {
      const int m = m0 + wm + b * 16 + (lane & 15);
      const float s_m = sxv[b];
#pragma unroll
      for (int a = 0; a < TN; a += 2) {
        float v[2][4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float4 sv = swv[a + h], bv = bvv[a + h];
          v[h][0] = gelu_erf(acc[a + h][b][0] * s_m * sv.x + bv.x);
          v[h][1] = gelu_erf(acc[a + h][b][1] * s_m * sv.y + bv.y);
          v[h][2] = gelu_erf(acc[a + h][b][2] * s_m * sv.z + bv.z);
          v[h][3] = gelu_erf(acc[a + h][b][3] * s_m * sv.w + bv.w);
        }
        float amax = 0.f;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int i = 0; i < 4; ++i) amax = fmaxf(amax, fabsf(v[h][i]));
        amax = fmaxf(amax, __shfl_xor(amax, 16, 64));
        amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
        // smallest power of two 2^e with amax / 2^e <= 448 (E8M0 byte e + 127)
        int e = amax > 0.f ? (int)ceilf(__log2f(amax * (1.f / 448.f))) : -127;
        if (e > 0 && amax * __builtin_ldexpf(1.f, -e) > 448.f) ++e;  // log2 rounding guard
        e = max(-127, min(127, e));
        const float inv = __builtin_ldexpf(1.f, -e);
        const int nb = n0 + wn + a * 16;  // first column of the 32-block
        if (m < M && nb < N) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            int w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[h][0] * inv, -448.f), 448.f),
                                                    fminf(fmaxf(v[h][1] * inv, -448.f), 448.f), 0, false);
            w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[h][2] * inv, -448.f), 448.f),
                                                fminf(fmaxf(v[h][3] * inv, -448.f), 448.f), w, true);
            *reinterpret_cast<uint32_t*>(Yq + (long long)m * N + nb + h * 16 + 4 * (lane >> 4)) = (uint32_t)w;
          }
          if ((lane >> 4) == 0) Ys[(long long)m * (N / 32) + nb / 32] = (uint8_t)(e + 127);
        }
      }
    }
    return;
  }

  // epilogue: acc[a][b][i] = C[m = wm + 16b + (lane&15)][n = wn + 16a + 4(lane>>4) + i]
#pragma unroll
  for (int b = 0; b < TM; ++b) {
    const int m = m0 + wm + b * 16 + (lane & 15);
    if (m >= M) continue;
    const float s_m = sxv[b];
#pragma unroll
    for (int a = 0; a < TN; ++a) {
      const int n = n0 + wn + a * 16 + 4 * (lane >> 4);
      if (n >= N) continue;
      const float4 sv = swv[a], bv = bvv[a];
      float v0 = acc[a][b][0] * s_m * sv.x + bv.x;
      float v1 = acc[a][b][1] * s_m * sv.y + bv.y;
      float v2 = acc[a][b][2] * s_m * sv.z + bv.z;
      float v3 = acc[a][b][3] * s_m * sv.w + bv.w;
      if (EPI == 1) { v0 = gelu_erf(v0); v1 = gelu_erf(v1); v2 = gelu_erf(v2); v3 = gelu_erf(v3); }
      u32x2 o;
      o[0] = pack2bf(v0, v1);
      o[1] = pack2bf(v2, v3);
      *reinterpret_cast<u32x2*>(Y + (long long)m * N + n) = o;
    }
  }
}

template <int TM, int TN, int WAVES_M, int WAVES_N, bool PRIO = false>
int launch_gemm(const void* xq, const void* wq, const float* sx, const float* sw, const float* bias, void* y, int M,
                int N, int K, int epi, hipStream_t s) {
  constexpr int BM = WAVES_M * 16 * TM, BN = WAVES_N * 16 * TN;
  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const dim3 grid((unsigned)(tiles_m * tiles_n)), block(64 * WAVES_M * WAVES_N);
  if (epi == 1)
    hipLaunchKernelGGL((gemm_fp8_kernel<TM, TN, WAVES_M, WAVES_N, 1, PRIO>), grid, block, 0, s, (const uint8_t*)xq,
                       (const uint8_t*)wq, sx, sw, bias, (bf16_t*)y, M, N, K, tiles_n);
  else
    hipLaunchKernelGGL((gemm_fp8_kernel<TM, TN, WAVES_M, WAVES_N, 0, PRIO>), grid, block, 0, s, (const uint8_t*)xq,
                       (const uint8_t*)wq, sx, sw, bias, (bf16_t*)y, M, N, K, tiles_n);
  return BE_CHECK_LAUNCH();
}

// Per-row dynamic quantisation bf16 -> e4m3fn: scale[m] = max(amax_k |x[m,k]|, tiny) / 448.
// One wave per row; the row stays in registers between the amax and the conversion.  GELU: apply the
// exact (erf) GELU first — the MLP's fc1 output becomes fc2's fp8 input in one pass over HBM.
template <int NV, bool GELU>
__global__ __launch_bounds__(256) void quant_rows_kernel(const bf16_t* __restrict__ x, uint8_t* __restrict__ q,
                                                         float* __restrict__ scale, long long rows, int K) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const bf16_t* xr = x + row * K;
  u32x4 v[NV];
  float amax = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < K) {
      v[k] = *reinterpret_cast<const u32x4*>(xr + c);
      if (GELU) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[k][j] = pack2bf(gelu_erf(lo_bf(v[k][j])), gelu_erf(hi_bf(v[k][j])));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) amax = fmaxf(amax, fmaxf(fabsf(lo_bf(v[k][j])), fabsf(hi_bf(v[k][j]))));
    }
  }
  amax = wave_max(amax);
  const float s = fmaxf(amax, 1e-12f) * (1.f / 448.f);
  const float inv = 448.f / fmaxf(amax, 1e-12f);
  if (lane == 0) scale[row] = s;
  uint8_t* qr = q + row * K;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < K) {
      u32x2 o;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        int w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(lo_bf(v[k][2 * h]) * inv, -448.f), 448.f),
                                                fminf(fmaxf(hi_bf(v[k][2 * h]) * inv, -448.f), 448.f), 0, false);
        w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(lo_bf(v[k][2 * h + 1]) * inv, -448.f), 448.f),
                                            fminf(fmaxf(hi_bf(v[k][2 * h + 1]) * inv, -448.f), 448.f), w, true);
        o[h] = (uint32_t)w;
      }
      *reinterpret_cast<u32x2*>(qr + c) = o;
    }
  }
}

}  // namespace

extern "C" {

// Tile by shape, measured on the ViT-B/14 batch-64 shapes (profiles/r03/fp8/fp8_bench_s23.jsonl, per-config
// TF/s): 256x256 for long K (fc2: 1552 vs 1393 TF/s for 128x128, even at 195 tiles on 256 CUs) and for
// narrow N (proj: 851 vs 826) as long as the grid is at least half full; otherwise 128x128 on 8
// waves, 64x32 per wave with the GELU epilogue (fc1: 986 vs 962), 32x64 without (qkv: 1023 vs 1018).
static int pick_cfg(int M, int N, int K, int epi) {
  const long long t256 = (long long)((M + 255) / 256) * ((N + 255) / 256);
  if ((K >= 2048 || N <= 1024) && t256 >= 128) return 4;
  return epi == 0 ? 6 : 5;
}

// Y[M,N] bf16 = epi(Xq[M,K] e4m3 . Wq[N,K]^T e4m3 * sx[M] * sw[N] + bias[N]); epi 0 = none, 1 = GELU.
// K % 128 == 0, N % 4 == 0; any M.  cfg selects the block tile (0 = by shape):
//   1: 128x128 (4 waves, 64x64 each)   2: 256x128 (8 waves)   3: 128x256 (8 waves)
//   4: 256x256 (8 waves, 128x64 each)  5 / 6: 128x128 on 8 waves (64x32 / 32x64 each).  The 128x128 tiles raise
//   the wave priority around their MFMA
//   cluster (+0-13 %, profiles/r02/fp8_gemm_bench_r02.md); on 256x256 that costs 6 %.
int be_gemm_fp8(const void* xq, const void* wq, const float* sx, const float* sw, const float* bias, void* y, int M,
                int N, int K, int epi, int cfg, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0 || K % BK != 0 || N % 4 != 0) return -1;
  if (cfg == 0) cfg = pick_cfg(M, N, K, epi);
  switch (cfg) {
    case 1: return launch_gemm<4, 4, 2, 2, true>(xq, wq, sx, sw, bias, y, M, N, K, epi, s);
    case 2: return launch_gemm<4, 4, 4, 2>(xq, wq, sx, sw, bias, y, M, N, K, epi, s);
    case 3: return launch_gemm<4, 4, 2, 4>(xq, wq, sx, sw, bias, y, M, N, K, epi, s);
    case 4: return launch_gemm<8, 4, 2, 4>(xq, wq, sx, sw, bias, y, M, N, K, epi, s);
    // 128x128 tiles on 8 waves (64x32 / 32x64 per wave): 4 waves per SIMD at 2 blocks/CU
    case 5: return launch_gemm<4, 2, 2, 4, true>(xq, wq, sx, sw, bias, y, M, N, K, epi, s);
    case 6: return launch_gemm<2, 4, 4, 2, true>(xq, wq, sx, sw, bias, y, M, N, K, epi, s);
    default: return -2;
  }
}

// MX-fp8 variants of be_gemm_fp8 (tile by shape: pick_cfg):
//   xs != null: X carries E8M0 block scales xs [M, K/32] (sx unused); else per-row fp32 sx.
//   epi 0 / 1: y bf16 [M, N] (GELU for 1);  epi 2: GELU -> yq e4m3 [M, N] + ys E8M0 [M, N/32] (N % 32 == 0).
int be_gemm_fp8_mx(const void* xq, const float* sx, const void* xs, const void* wq, const float* sw,
                   const float* bias, void* y, void* yq, void* ys, int M, int N, int K, int epi, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0 || K % BK != 0 || N % 4 != 0) return -1;
  if (epi == 2 && (N % 32 != 0 || !yq || !ys)) return -3;
  if (epi != 2 && !y) return -3;
  if (!xs && !sx) return -4;
  const int cfg = pick_cfg(M, N, K, epi);
  const uint8_t* X = (const uint8_t*)xq;
  const uint8_t* Wt = (const uint8_t*)wq;
  const uint8_t* Xs = (const uint8_t*)xs;
  bf16_t* Y = (bf16_t*)y;
  uint8_t* Yq = (uint8_t*)yq;
  uint8_t* Ys = (uint8_t*)ys;
#define MXL(TM, TN, WM, WN, PR, EP, XSV)                                                                     \
  {                                                                                                          \
    constexpr int BM = WM * 16 * TM, BN = WN * 16 * TN;                                                      \
    const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;                                      \
    hipLaunchKernelGGL((gemm_fp8_kernel<TM, TN, WM, WN, EP, PR, XSV>), dim3((unsigned)(tiles_m * tiles_n)),   \
                       dim3(64 * WM * WN), 0, s, X, Wt, sx, sw, bias, Y, M, N, K, tiles_n, Xs, Yq, Ys);      \
  }
#define MXE(TM, TN, WM, WN, PR, XSV) \
  if (epi == 2) MXL(TM, TN, WM, WN, PR, 2, XSV) else if (epi == 1) MXL(TM, TN, WM, WN, PR, 1, XSV) else MXL(TM, TN, WM, WN, PR, 0, XSV)
  // block-scaled X: the scales come from LDS per K step (stage_xs), so the 256x256 tile takes them too
  if (cfg == 4) {
    if (xs) MXE(8, 4, 2, 4, false, true) else MXE(8, 4, 2, 4, false, false)
  } else if (cfg == 5) {
    if (xs) MXE(4, 2, 2, 4, true, true) else MXE(4, 2, 2, 4, true, false)
  } else {
    if (xs) MXE(2, 4, 4, 2, true, true) else MXE(2, 4, 4, 2, true, false)
  }
#undef MXE
#undef MXL
  return BE_CHECK_LAUNCH();
}

// x bf16 [rows, K] -> q e4m3fn [rows, K] + scale float [rows]; K % 8 == 0, K <= 4096.
// gelu != 0: quantise GELU(x) (bf16-rounded, like a bf16 GELU pass) instead of x.
int be_quant_fp8_rows(const void* x, void* q, float* scale, long long rows, int K, int gelu, hipStream_t s) {
  if (K % 8 != 0 || K > 64 * 8 * 8) return -1;
  const int nv = (K / 8 + 63) / 64;
  const dim3 grid((unsigned)((rows + 3) / 4)), block(256);
#define QR(NV)                                                                                                 \
  case NV:                                                                                                     \
    if (gelu)                                                                                                  \
      hipLaunchKernelGGL((quant_rows_kernel<NV, true>), grid, block, 0, s, (const bf16_t*)x, (uint8_t*)q, scale, \
                         rows, K);                                                                             \
    else                                                                                                       \
      hipLaunchKernelGGL((quant_rows_kernel<NV, false>), grid, block, 0, s, (const bf16_t*)x, (uint8_t*)q,       \
                         scale, rows, K);                                                                      \
    break;
  switch (nv) {
    QR(1) QR(2) QR(3) QR(4) QR(5) QR(6) QR(7) QR(8)
    default: return -1;
  }
#undef QR
  return BE_CHECK_LAUNCH();
}

}  // extern "C"

// Training kernels for the fused pre-activation conv family (Cellpose CPnet fwd/bwd on MFMA).
//
// SURVEY.md §2.5 K1/K8/K12 + §7.2 step 7: the reference fine-tunes through PyTorch autograd inside
// the cellpose package (apps/cellpose-finetuning/main.py:1483-1546: net(x) -> _loss_fn_seg ->
// backward -> AdamW).  Here the CPnet unit  out = conv_k( relu?( BN_train( T(x) [+ x2] [+ f[n]] ) ) )
// [+ bias] [+ residual]  gets hand-written backward kernels:
//
//   be_bn_stats          per-(n,c) sum / sum-of-squares of v = T(x) [+ x2]; the LAST block (atomic
//                        ticket) finalises the batch statistics into the conv prologue's affine
//                        (scale[c], shift[n,c]) for one or two BN units sharing the input, and
//                        updates the running statistics — one launch per BN input.
//   be_conv_wgrad        dW[co, tap, ci] = sum_{n,p} dOut[n,p,co] * act(n, p+tap, ci): implicit GEMM on
//                        v_mfma_f32_16x16x32_bf16 with K = pixels.  Both operands are staged in their
//                        natural NHWC layout and read K-major with ds_read_b64_tr_b16 (gfx950
//                        transposed LDS read, cdna_hip_programming.md T10) — no transposes in VALU.
//                        The activation is recomputed from the saved pre-BN input in the halo loader
//                        (pool / upsample / skip add / BN affine / ReLU in registers), exactly as the
//                        forward kernel does, so activations are never materialised.  dbias rides
//                        along as one extra MFMA against an all-ones B fragment.  Split-K over pixel
//                        tiles writes fp32 partials; be_conv_wgrad_reduce sums them into the torch
//                        [Cout, Cin, k, k] gradient layout of the flat fp32 grad buffer.
//   be_bn_bwd_reduce     per-(n,c) sum(dy) and sum(dy * xhat) (dy = dAct masked by the ReLU); last
//                        block finalises dgamma / dbeta, the per-channel backward coefficients and the
//                        style-feature gradient dfeat[n, c].
//   be_bn_bwd_apply      du = sum_k s_k dy_k + B0[c] + B1[c] * xhat, routed through T^T (max-pool
//                        argmax scatter / nearest-upsample 2x2 gather) into dx, and into dx2 (skip).
//   be_pack_conv_weights fp32 master -> bf16 packed forward weights and flipped/transposed dgrad
//                        weights for every conv in one launch (descriptor table).
//
// The data gradient (dgrad) of a stride-1 'same' conv is itself a forward conv of dOut with the
// spatially flipped, in/out-transposed weights, so it runs on be_conv2d_nhwc unchanged.
#include "common.h"
#include <cstdlib>

namespace {

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// Two transposed LDS reads -> one 16x16x32 MFMA fragment (8 K-values of one M/N index per lane).
__device__ __forceinline__ bf16x8 tr_frag(const bf16_t* p0, const bf16_t* p1) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1));
  bf16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return v;
}

__device__ __forceinline__ float ld_acq(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Raw 8-channel input of the (transformed) tensor at output-resolution pixel (gy, gx):
// INMODE 0 identity, 1 nearest-upsample x2 (source (gy/2, gx/2)), 2 max-pool 2x2.
template <int INMODE>
__device__ __forceinline__ u32x4 load_t8(const bf16_t* __restrict__ x, int n, int gy, int gx, int Hs, int Ws, int C,
                                         int c) {
  if (INMODE == 0) return *reinterpret_cast<const u32x4*>(x + (((size_t)n * Hs + gy) * Ws + gx) * C + c);
  if (INMODE == 1) return *reinterpret_cast<const u32x4*>(x + (((size_t)n * Hs + (gy >> 1)) * Ws + (gx >> 1)) * C + c);
  const bf16_t* base = x + (((size_t)n * Hs + 2 * gy) * Ws + 2 * gx) * C + c;
  const u32x4 r0 = *reinterpret_cast<const u32x4*>(base);
  const u32x4 r1 = *reinterpret_cast<const u32x4*>(base + C);
  const u32x4 q0 = *reinterpret_cast<const u32x4*>(base + (size_t)Ws * C);
  const u32x4 q1 = *reinterpret_cast<const u32x4*>(base + (size_t)Ws * C + C);
  u32x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float lo = fmaxf(fmaxf(lo_bf(r0[j]), lo_bf(r1[j])), fmaxf(lo_bf(q0[j]), lo_bf(q1[j])));
    const float hi = fmaxf(fmaxf(hi_bf(r0[j]), hi_bf(r1[j])), fmaxf(hi_bf(q0[j]), hi_bf(q1[j])));
    r[j] = (__float_as_uint(lo) >> 16) | (__float_as_uint(hi) & 0xffff0000u);
  }
  return r;
}

__device__ __forceinline__ void unpack8(const u32x4 r, float (&v)[8]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[2 * j] = lo_bf(r[j]); v[2 * j + 1] = hi_bf(r[j]); }
}

__device__ __forceinline__ void ld8(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// ============================================================================================
// Weight-gradient kernel
// ============================================================================================

struct WgArgs {
  const bf16_t* x;      // pre-transform input [N, Hs, Ws, Cin]
  const bf16_t* x2;     // optional skip [N, H, W, Cin]
  const float* pscale;  // [N?, Cin] (null = 1; row stride pscale_ns, GroupNorm: Cin)
  const float* pshift;  // [N?, Cin] (null = 0)
  const bf16_t* dy;     // dOut [N, H, W, Cy] (Cy % 8 == 0)
  float* ws;            // partials [splits][cout_valid][Cin][KS*KS] (torch weight layout per split)
  float* wsb;           // optional dbias partials [splits][cout_valid]
  int N, H, W, Hs, Ws, Cin, Cy, cout_valid;
  int pshift_ns, pscale_ns, relu;
  int tiles_x, tiles_y, ntiles, splits;
};

template <int KS, int CK, int TCO, int INMODE, bool X2, int WCO, int WCI>
struct WCfg {
  static constexpr int TH = 4, TW = 32;
  static constexpr int NCO = TCO / 16;
  static constexpr int NCI = CK >= 16 ? CK / 16 : 1;
  static constexpr int NWV = (NCO / WCO) * (NCI / WCI);
  static constexpr int NT = NWV * 64;
  static constexpr int HH = TH + KS - 1, HWW = TW + KS - 1, HP = HH * HWW;
  // pixel strides (elements): (stride/2) % 64 is an odd multiple of 8 dwords, so the 8 consecutive
  // pixel rows one 32-lane half reads with ds_read_b64_tr_b16 cover all 64 banks once.
  static constexpr int SX = CK == 8 ? 16 : CK + 16;
  static constexpr int SY = TCO == 16 ? 16 : TCO + 16;
  static constexpr int CG = CK / 8;
  static constexpr int HU = HP * CG, HUPT = (HU + NT - 1) / NT;
  static constexpr int YG = TCO / 8, YU = TH * TW * YG, YUPT = (YU + NT - 1) / NT;
  static constexpr int NTAP = KS * KS;
  static constexpr int LDS_X = HP * SX, LDS_Y = TH * TW * SY;
  static constexpr size_t LDS = (size_t)(LDS_X + LDS_Y) * sizeof(bf16_t);
  static_assert(NCO % WCO == 0 && NCI % WCI == 0, "wave tiling");
  static_assert(NT % CG == 0, "fixed halo channel group per thread");
  static_assert(((SX / 2) % 16) == 8 && ((SY / 2) % 16) == 8, "conflict-free transposed reads");
};

template <typename C, int KS, int CK, int INMODE, bool X2>
__device__ __forceinline__ void wg_issue(const WgArgs& a, int t, int ci0, int co0, int tid, u32x4 (&xr)[C::HUPT],
                                         u32x4 (&x2r)[X2 ? C::HUPT : 1], u32x4 (&yr)[C::YUPT]) {
  const int per_img = a.tiles_x * a.tiles_y;
  const int n = t / per_img, rem = t % per_img;
  const int ty0 = (rem / a.tiles_x) * C::TH, tx0 = (rem % a.tiles_x) * C::TW;
#pragma unroll
  for (int i = 0; i < C::HUPT; ++i) {
    const int u = tid + i * C::NT;
    u32x4 r = (u32x4){0u, 0u, 0u, 0u}, r2 = r;
    if (u < C::HU) {
      const int pix = u / C::CG, cg = u % C::CG;
      const int gy = ty0 + pix / C::HWW - KS / 2, gx = tx0 + pix % C::HWW - KS / 2;
      if (gy >= 0 && gy < a.H && gx >= 0 && gx < a.W) {
        r = load_t8<INMODE>(a.x, n, gy, gx, a.Hs, a.Ws, a.Cin, ci0 + cg * 8);
        if (X2) r2 = *reinterpret_cast<const u32x4*>(a.x2 + (((size_t)n * a.H + gy) * a.W + gx) * a.Cin + ci0 + cg * 8);
      }
    }
    xr[i] = r;
    if (X2) x2r[i] = r2;
  }
#pragma unroll
  for (int i = 0; i < C::YUPT; ++i) {
    const int u = tid + i * C::NT;
    u32x4 r = (u32x4){0u, 0u, 0u, 0u};
    if (u < C::YU) {
      const int pix = u / C::YG, cg = u % C::YG;
      const int gy = ty0 + pix / C::TW, gx = tx0 + pix % C::TW;
      const int c = co0 + cg * 8;
      if (gy < a.H && gx < a.W && c < a.Cy)
        r = *reinterpret_cast<const u32x4*>(a.dy + (((size_t)n * a.H + gy) * a.W + gx) * a.Cy + c);
    }
    yr[i] = r;
  }
}

template <typename C, int KS, int CK, bool X2>
__device__ __forceinline__ void wg_commit(const WgArgs& a, int t, int ci0, int tid, const u32x4 (&xr)[C::HUPT],
                                          const u32x4 (&x2r)[X2 ? C::HUPT : 1], const u32x4 (&yr)[C::YUPT],
                                          bf16_t* xs, bf16_t* ys) {
  const int per_img = a.tiles_x * a.tiles_y;
  const int n = t / per_img, rem = t % per_img;
  const int ty0 = (rem / a.tiles_x) * C::TH, tx0 = (rem % a.tiles_x) * C::TW;
  // a thread's halo channel group is fixed (NT % CG == 0): its 8 affine pairs are loaded once per tile
  float sc[8], sh[8];
  {
    const int c = ci0 + (tid % C::CG) * 8;
    if (a.pscale) ld8(a.pscale + (size_t)n * a.pscale_ns + c, sc);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) sc[j] = 1.f;
    }
    if (a.pshift) ld8(a.pshift + (size_t)n * a.pshift_ns + c, sh);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) sh[j] = 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < C::HUPT; ++i) {
    const int u = tid + i * C::NT;
    if (u >= C::HU) continue;
    const int pix = u / C::CG, cg = u % C::CG;
    const int gy = ty0 + pix / C::HWW - KS / 2, gx = tx0 + pix % C::HWW - KS / 2;
    u32x4 packed = (u32x4){0u, 0u, 0u, 0u};
    if (gy >= 0 && gy < a.H && gx >= 0 && gx < a.W) {  // zero padding applies after the activation
      float v[8];
      unpack8(xr[i], v);
      if (X2) {
        float w[8];
        unpack8(x2r[i], w);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += w[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fmaf(v[j], sc[j], sh[j]);
#pragma unroll
      for (int j = 0; j < 4; ++j) packed[j] = pack2bf(v[2 * j], v[2 * j + 1]);
      if (a.relu) {
#pragma unroll
        for (int j = 0; j < 4; ++j) packed[j] = relu_bf16x2(packed[j]);
      }
    }
    *reinterpret_cast<u32x4*>(xs + pix * C::SX + cg * 8) = packed;
    if (CK == 8) *reinterpret_cast<u32x4*>(xs + pix * C::SX + 8) = (u32x4){0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (int i = 0; i < C::YUPT; ++i) {
    const int u = tid + i * C::NT;
    if (u >= C::YU) continue;
    const int pix = u / C::YG, cg = u % C::YG;
    *reinterpret_cast<u32x4*>(ys + pix * C::SY + cg * 8) = yr[i];
  }
}

template <int KS, int CK, int TCO, int INMODE, bool X2, int WCO, int WCI>
__global__ __launch_bounds__(((TCO / 16) / WCO) * ((CK >= 16 ? CK / 16 : 1) / WCI) * 64) void conv_wgrad_kernel(WgArgs a) {
  using C = WCfg<KS, CK, TCO, INMODE, X2, WCO, WCI>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* xs = reinterpret_cast<bf16_t*>(smem);
  bf16_t* ys = xs + C::LDS_X;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int split = blockIdx.x;
  const int ci0 = blockIdx.y * CK;
  const int co0 = blockIdx.z * TCO;
  const int wco = wave % (C::NCO / WCO), wci = wave / (C::NCO / WCO);
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int t0 = (int)(((long long)split * a.ntiles) / a.splits);
  const int t1 = (int)(((long long)(split + 1) * a.ntiles) / a.splits);

  f32x4 acc[WCO][WCI][C::NTAP];
  f32x4 accb[WCO];
#pragma unroll
  for (int i = 0; i < WCO; ++i) {
    accb[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < WCI; ++j)
#pragma unroll
      for (int tp = 0; tp < C::NTAP; ++tp) acc[i][j][tp] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (short)0x3f80;
  const bool do_bias = a.wsb != nullptr && blockIdx.y == 0 && wci == 0;

  u32x4 xr[C::HUPT], x2r[X2 ? C::HUPT : 1], yr[C::YUPT];
  if (t0 < t1) wg_issue<C, KS, CK, INMODE, X2>(a, t0, ci0, co0, tid, xr, x2r, yr);
  for (int t = t0; t < t1; ++t) {
    __syncthreads();  // previous tile's fragment reads are done
    wg_commit<C, KS, CK, X2>(a, t, ci0, tid, xr, x2r, yr, xs, ys);
    __syncthreads();
    if (t + 1 < t1) wg_issue<C, KS, CK, INMODE, X2>(a, t + 1, ci0, co0, tid, xr, x2r, yr);
#pragma unroll
    for (int r = 0; r < C::TH; ++r) {
      // K permutation inside the 32-pixel chunk: lane group g owns pixels 4g..4g+3 and 16+4g..16+4g+3
      // (same for A and B), so each tr-read's 32-lane half touches 8 consecutive pixel rows.
      const int k0 = 4 * g + q, k1 = 16 + 4 * g + q;
      bf16x8 af[WCO];
#pragma unroll
      for (int i = 0; i < WCO; ++i) {
        const int cb = (wco * WCO + i) * 16 + 4 * p;
        af[i] = tr_frag(ys + (r * C::TW + k0) * C::SY + cb, ys + (r * C::TW + k1) * C::SY + cb);
      }
#pragma unroll
      for (int tp = 0; tp < C::NTAP; ++tp) {
        const int dy = tp / KS, dx = tp % KS;
#pragma unroll
        for (int j = 0; j < WCI; ++j) {
          const int cb = (wci * WCI + j) * 16 + 4 * p;
          const bf16x8 bf = tr_frag(xs + ((r + dy) * C::HWW + k0 + dx) * C::SX + cb,
                                    xs + ((r + dy) * C::HWW + k1 + dx) * C::SX + cb);
#pragma unroll
          for (int i = 0; i < WCO; ++i)
            acc[i][j][tp] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf, acc[i][j][tp], 0, 0, 0);
        }
      }
      if (do_bias) {
#pragma unroll
        for (int i = 0; i < WCO; ++i) accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], ones, accb[i], 0, 0, 0);
      }
    }
  }
  // partials: C/D layout col = lane & 15 (ci), row = 4 * (lane >> 4) + e (co)
  const int ci_l = lane & 15;
#pragma unroll
  for (int i = 0; i < WCO; ++i) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int co = co0 + (wco * WCO + i) * 16 + 4 * g + e;
      if (co >= a.cout_valid) continue;
#pragma unroll
      for (int j = 0; j < WCI; ++j) {
        const int ci = ci0 + (wci * WCI + j) * 16 + ci_l;
        if (ci >= a.Cin || (CK == 8 && ci_l >= 8)) continue;
#pragma unroll
        for (int tp = 0; tp < C::NTAP; ++tp)
          a.ws[(((size_t)split * a.cout_valid + co) * a.Cin + ci) * C::NTAP + tp] = acc[i][j][tp][e];
      }
      if (do_bias && ci_l == 0) a.wsb[(size_t)split * a.cout_valid + co] = accb[i][e];
    }
  }
}

template <int KS, int CK, int TCO, int INMODE, bool X2, int WCO, int WCI>
int wgrad_launch(WgArgs a, hipStream_t s) {
  using C = WCfg<KS, CK, TCO, INMODE, X2, WCO, WCI>;
  dim3 grid(a.splits, a.Cin / CK, (a.Cy + TCO - 1) / TCO);
  hipLaunchKernelGGL((conv_wgrad_kernel<KS, CK, TCO, INMODE, X2, WCO, WCI>), grid, dim3(C::NT), C::LDS, s, a);
  return BE_CHECK_LAUNCH();
}

template <int KS, int CK, int TCO, int INMODE, bool X2>
int wgrad_wco(WgArgs a, hipStream_t s) {
  if constexpr (TCO >= 64) return wgrad_launch<KS, CK, TCO, INMODE, X2, 2, 1>(a, s);
  else return wgrad_launch<KS, CK, TCO, INMODE, X2, 1, 1>(a, s);
}

template <int KS, int CK, int TCO>
int wgrad_mode(int inmode, bool x2, WgArgs a, hipStream_t s) {
  if (x2) {
    if (inmode != 0) return -2;
    return wgrad_wco<KS, CK, TCO, 0, true>(a, s);
  }
  switch (inmode) {
    case 0: return wgrad_wco<KS, CK, TCO, 0, false>(a, s);
    case 1: return wgrad_wco<KS, CK, TCO, 1, false>(a, s);
    case 2: return wgrad_wco<KS, CK, TCO, 2, false>(a, s);
  }
  return -2;
}

template <int KS, int CK>
int wgrad_tco(int tco, int inmode, bool x2, WgArgs a, hipStream_t s) {
  switch (tco) {
    case 16: return wgrad_mode<KS, CK, 16>(inmode, x2, a, s);
    case 32: return wgrad_mode<KS, CK, 32>(inmode, x2, a, s);
    case 64: return wgrad_mode<KS, CK, 64>(inmode, x2, a, s);
  }
  return -3;
}

// Tunables (environment overrides read once, for sweeps): BE_WG_REDUCE_THREADS = threads of the wgrad
// split reduction, BE_BN_BLOCKS = target blocks of the BN statistics / reduction kernels.
static int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
}

// Sum the split-K partials into the (pre-zeroed) torch-layout gradient.  The partials already use the
// weight layout [co][ci][tap], so thread t owns element t: every split's slab is read coalesced and the
// final atomicAdd of a wave covers 256 contiguous bytes.  Grid.y splits the split dimension into
// chunks (sized by the host so that ~256k threads run), each chunk adding its sum atomically.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ ws, const float* __restrict__ wsb,
                                                           int splits, int cout, int ntap, int cin_ld, int cin,
                                                           float* __restrict__ dw, float* __restrict__ db) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int nw = cout * cin_ld * ntap;
  const int spc = (splits + gridDim.y - 1) / gridDim.y;
  const int s0 = blockIdx.y * spc, s1 = min(splits, s0 + spc);
  if (e < nw) {
    const int tp = e % ntap, ci = (e / ntap) % cin_ld, co = e / (ntap * cin_ld);
    if (ci >= cin) return;
    float acc = 0.f;
#pragma unroll 8
    for (int k = s0; k < s1; ++k) acc += ws[(size_t)k * nw + e];
    atomicAdd(dw + ((size_t)co * cin + ci) * ntap + tp, acc);
  } else if (db != nullptr && e < nw + cout) {
    const int co = e - nw;
    float acc = 0.f;
    for (int k = s0; k < s1; ++k) acc += wsb[(size_t)k * cout + co];
    atomicAdd(db + co, acc);
  }
}

// ============================================================================================
// BatchNorm (train) statistics + finalise
// ============================================================================================

struct BnUnits {
  const float* gamma[2];
  const float* beta[2];
  float* scale[2];     // [C] (BatchNorm) or [N, C] (GroupNorm)
  float* shift[2];     // [N, C]
  float* run_mean[2];  // optional
  float* run_var[2];
  int relu[2];
  const bf16_t* dact[2];  // backward: dAct of each unit [N, H, W, C]
  float* dgamma[2];       // backward: parameter grads (c < c_valid)
  float* dbeta[2];
};

struct BnArgs {
  const bf16_t* x;   // [N, Hs, Ws, C]
  const bf16_t* x2;  // optional [N, H, W, C]
  const float* feat; // optional [N, C] (style feature added before the BN)
  int N, Hs, Ws, H, W, C, c_valid, inmode, nunits;
  int groups;        // 0: BatchNorm (batch statistics per channel); G > 0: GroupNorm, G groups per image
  int cns;           // per-image stride of the coefficient arrays: 0 (BN) or C (GN)
  float eps, momentum;
  float* stat;       // workspace: sum[N*C], sq[N*C], mean[CC], rstd[CC], then bwd: sdy[2][N*C], sdyx[2][N*C], B0[CC],
                     // B1[CC] with CC = C (BN) or N*C (GN: per-image group values broadcast to the channels)
  unsigned* ticket;  // zeroed counters: [0] fwd, [1] bwd
  BnUnits u;
  float* dfeat;      // backward: [N, C]
  int per_block;     // pixels per block
  float* scratch;    // per-block partials [N][nb][NACC][C] (shared scratch, plain stores)
  int nb;            // blocks per image of the partial kernel
};

__device__ __forceinline__ float* st_sum(const BnArgs& a) { return a.stat; }
__device__ __forceinline__ float* st_sq(const BnArgs& a) { return a.stat + (size_t)a.N * a.C; }
__device__ __forceinline__ float* st_mean(const BnArgs& a) { return a.stat + (size_t)2 * a.N * a.C; }
__device__ __forceinline__ size_t st_cc(const BnArgs& a) { return a.cns ? (size_t)a.N * a.C : (size_t)a.C; }
__device__ __forceinline__ float* st_rstd(const BnArgs& a) { return st_mean(a) + st_cc(a); }
__device__ __forceinline__ float* st_sdy(const BnArgs& a, int k) { return st_rstd(a) + st_cc(a) + (size_t)k * 2 * a.N * a.C; }
__device__ __forceinline__ float* st_sdyx(const BnArgs& a, int k) { return st_sdy(a, k) + (size_t)a.N * a.C; }
__device__ __forceinline__ float* st_b0(const BnArgs& a) { return st_rstd(a) + st_cc(a) + (size_t)4 * a.N * a.C; }
__device__ __forceinline__ float* st_b1(const BnArgs& a) { return st_b0(a) + st_cc(a); }

// v = T(x) [+ x2] at output pixel pix (row-major over H x W) for channels c..c+7
template <int INMODE, bool X2>
__device__ __forceinline__ void load_v8(const BnArgs& a, int n, int pix, int c, float (&v)[8]) {
  const int gy = pix / a.W, gx = pix % a.W;
  unpack8(load_t8<INMODE>(a.x, n, gy, gx, a.Hs, a.Ws, a.C, c), v);
  if (X2) {
    float w[8];
    unpack8(*reinterpret_cast<const u32x4*>(a.x2 + (((size_t)n * a.H + gy) * a.W + gx) * a.C + c), w);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += w[j];
  }
}

// Block-level reduction of per-thread 8-channel partials (NACC arrays) -> this block's slot of the
// partial scratch.  Lanes l and l ^ o (o a multiple of C/8) hold the same channel group, so a shuffle
// butterfly over those offsets reduces a wave; the 4 waves meet in LDS ([4][NACC][256]: C <= 256).
// Plain stores to a per-block slot: same-address atomics from every block serialised in one L2
// channel (measured ~50 ns per block).
template <int NACC>
__device__ __forceinline__ void block_reduce_store(const BnArgs& a, int n, float (&acc)[NACC][8]) {
  __shared__ float red[4][NACC][256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, C8 = a.C / 8;
  for (int o = C8; o < 64; o <<= 1) {
#pragma unroll
    for (int k = 0; k < NACC; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[k][j] += __shfl_xor(acc[k][j], o, 64);
  }
  if (lane < C8) {
#pragma unroll
    for (int k = 0; k < NACC; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[wave][k][lane * 8 + j] = acc[k][j];
  }
  __syncthreads();
  float* slot = a.scratch + ((size_t)n * a.nb + blockIdx.x) * NACC * a.C;
  for (int c = tid; c < a.C; c += 256) {
#pragma unroll
    for (int k = 0; k < NACC; ++k) slot[k * a.C + c] = red[0][k][c] + red[1][k][c] + red[2][k][c] + red[3][k][c];
  }
}

// Sum image n's nb block partials into dst[k][n*C + c] (block per image; 256 / C lane groups).
template <int NACC>
__device__ __forceinline__ void image_reduce(const BnArgs& a, int n, float* const* dst) {
  __shared__ float red2[NACC][256];
  const int tid = threadIdx.x, G = 256 / a.C, c = tid % a.C, g = tid / a.C;
  float s[NACC];
#pragma unroll
  for (int k = 0; k < NACC; ++k) s[k] = 0.f;
  const float* base = a.scratch + (size_t)n * a.nb * NACC * a.C;
#pragma unroll 8
  for (int b = g; b < a.nb; b += G) {
#pragma unroll
    for (int k = 0; k < NACC; ++k) s[k] += base[((size_t)b * NACC + k) * a.C + c];
  }
#pragma unroll
  for (int k = 0; k < NACC; ++k) red2[k][tid] = s[k];
  __syncthreads();
  if (g == 0) {
#pragma unroll
    for (int k = 0; k < NACC; ++k) {
      float t = 0.f;
      for (int q = 0; q < G; ++q) t += red2[k][q * a.C + c];
      dst[k][(size_t)n * a.C + c] = t;
    }
  }
}

__device__ __forceinline__ bool last_block(unsigned* ticket) {
  __shared__ bool is_last;
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned total = gridDim.x * gridDim.y;
    is_last = atomicAdd(ticket, 1u) == total - 1;
  }
  __syncthreads();
  if (is_last) __threadfence();
  return is_last;
}

template <int INMODE, bool X2>
__global__ __launch_bounds__(256) void bn_stats_kernel(BnArgs a) {
  const int n = blockIdx.y, tid = threadIdx.x;
  const int C8 = a.C / 8, PL = 256 / C8, cg = tid % C8, pl = tid / C8;
  const int HW = a.H * a.W;
  const int p0 = blockIdx.x * a.per_block, p1 = min(HW, p0 + a.per_block);
  float acc[2][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { acc[0][j] = 0.f; acc[1][j] = 0.f; }
  if (pl < PL) {
#pragma unroll 4
    for (int pix = p0 + pl; pix < p1; pix += PL) {
      float v[8];
      load_v8<INMODE, X2>(a, n, pix, cg * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) { acc[0][j] += v[j]; acc[1][j] = fmaf(v[j], v[j], acc[1][j]); }
    }
  }
  block_reduce_store<2>(a, n, acc);
}

// Grid = N blocks: per-image sums, then the last block finalises batch mean / var over N*H*W of
// u = v + feat[n] into the conv-prologue affine of every unit.
__global__ __launch_bounds__(256) void bn_stats_fin_kernel(BnArgs a) {
  const int tid = threadIdx.x, HW = a.H * a.W;
  float* dst[2] = {st_sum(a), st_sq(a)};
  image_reduce<2>(a, blockIdx.x, dst);
  if (!last_block(a.ticket)) return;
  const float cnt = (float)a.N * (float)HW;
  for (int c = tid; c < a.C; c += 256) {
    float s1 = 0.f, q = 0.f;
#pragma unroll 8
    for (int m = 0; m < a.N; ++m) {
      const float s = ld_acq(st_sum(a) + (size_t)m * a.C + c), sq = ld_acq(st_sq(a) + (size_t)m * a.C + c);
      const float f = a.feat ? a.feat[(size_t)m * a.C + c] : 0.f;
      s1 += s + (float)HW * f;
      q += sq + 2.f * f * s + (float)HW * f * f;
    }
    const bool valid = c < a.c_valid;
    const float mean = s1 / cnt;
    const float var = fmaxf(q / cnt - mean * mean, 0.f);
    const float rstd = valid ? 1.f / sqrtf(var + a.eps) : 0.f;
    st_mean(a)[c] = valid ? mean : 0.f;
    st_rstd(a)[c] = rstd;
    for (int k = 0; k < a.nunits; ++k) {
      const float sc = valid ? a.u.gamma[k][c] * rstd : 0.f;
      const float be = valid ? a.u.beta[k][c] : 0.f;
      a.u.scale[k][c] = sc;
  #pragma unroll 8
    for (int m = 0; m < a.N; ++m) {
        const float f = a.feat ? a.feat[(size_t)m * a.C + c] : 0.f;
        a.u.shift[k][(size_t)m * a.C + c] = valid ? (f - mean) * sc + be : 0.f;
      }
      if (valid && a.u.run_mean[k]) {
        a.u.run_mean[k][c] = (1.f - a.momentum) * a.u.run_mean[k][c] + a.momentum * mean;
        a.u.run_var[k][c] = (1.f - a.momentum) * a.u.run_var[k][c] + a.momentum * var * cnt / fmaxf(cnt - 1.f, 1.f);
      }
    }
  }
}

// ---- backward reduce: sum(dy_k), sum(dy_k * xhat) per (n, c); last block -> coefficients
template <int INMODE, bool X2, int NU>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(BnArgs a) {
  const int n = blockIdx.y, tid = threadIdx.x;
  const int C8 = a.C / 8, PL = 256 / C8, cg = tid % C8, pl = tid / C8;
  const int HW = a.H * a.W;
  const int p0 = blockIdx.x * a.per_block, p1 = min(HW, p0 + a.per_block);
  const int c0 = cg * 8;
  float acc[2 * NU][8];
#pragma unroll
  for (int k = 0; k < 2 * NU; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
  if (pl < PL) {
    float mean[8], rstd[8], f[8], sc[NU][8], sh[NU][8];
    const size_t cr = (size_t)n * a.cns + c0;  // coefficient row (per image for GroupNorm)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mean[j] = st_mean(a)[cr + j];
      rstd[j] = st_rstd(a)[cr + j];
      f[j] = a.feat ? a.feat[(size_t)n * a.C + c0 + j] : 0.f;
#pragma unroll
      for (int k = 0; k < NU; ++k) {
        sc[k][j] = a.u.scale[k][cr + j];
        sh[k][j] = a.u.shift[k][(size_t)n * a.C + c0 + j];
      }
    }
#pragma unroll 2
    for (int pix = p0 + pl; pix < p1; pix += PL) {
      float v[8];
      load_v8<INMODE, X2>(a, n, pix, c0, v);
#pragma unroll
      for (int k = 0; k < NU; ++k) {
        float d[8];
        unpack8(*reinterpret_cast<const u32x4*>(a.u.dact[k] + ((size_t)n * HW + pix) * a.C + c0), d);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float dyv = d[j];
          if (a.u.relu[k] && fmaf(v[j], sc[k][j], sh[k][j]) <= 0.f) dyv = 0.f;
          const float xh = (v[j] + f[j] - mean[j]) * rstd[j];
          acc[2 * k][j] += dyv;
          acc[2 * k + 1][j] = fmaf(dyv, xh, acc[2 * k + 1][j]);
        }
      }
    }
  }
  block_reduce_store<2 * NU>(a, n, acc);
}

template <int NU>
__global__ __launch_bounds__(256) void bn_bwd_fin_kernel(BnArgs a) {
  const int tid = threadIdx.x, HW = a.H * a.W;
  float* dst[2 * NU];
#pragma unroll
  for (int k = 0; k < NU; ++k) { dst[2 * k] = st_sdy(a, k); dst[2 * k + 1] = st_sdyx(a, k); }
  image_reduce<2 * NU>(a, blockIdx.x, dst);
  if (!last_block(a.ticket + 1)) return;
  const float cnt = (float)a.N * (float)HW;
  for (int c = tid; c < a.C; c += 256) {
    const bool valid = c < a.c_valid;
    float b0 = 0.f, b1 = 0.f;
    for (int k = 0; k < NU; ++k) {
      float sdy = 0.f, sdyx = 0.f;
  #pragma unroll 8
    for (int m = 0; m < a.N; ++m) {
        sdy += ld_acq(st_sdy(a, k) + (size_t)m * a.C + c);
        sdyx += ld_acq(st_sdyx(a, k) + (size_t)m * a.C + c);
      }
      const float s = a.u.scale[k][c];
      b0 -= s * sdy / cnt;
      b1 -= s * sdyx / cnt;
      if (valid) {
        if (a.u.dgamma[k]) a.u.dgamma[k][c] = sdyx;
        if (a.u.dbeta[k]) a.u.dbeta[k][c] = sdy;
      }
    }
    st_b0(a)[c] = b0;
    st_b1(a)[c] = b1;
    if (a.dfeat) {  // dfeat[n, c] = sum_hw du = s * sum_hw dy + HW * B0 + B1 * sum_hw xhat   (NU == 1)
      const float mean = st_mean(a)[c], rstd = st_rstd(a)[c], s = a.u.scale[0][c];
  #pragma unroll 8
    for (int m = 0; m < a.N; ++m) {
        const float f = a.feat ? a.feat[(size_t)m * a.C + c] : 0.f;
        const float sx = (ld_acq(st_sum(a) + (size_t)m * a.C + c) + (float)HW * (f - mean)) * rstd;
        const float sdy = ld_acq(st_sdy(a, 0) + (size_t)m * a.C + c);
        a.dfeat[(size_t)m * a.C + c] = valid ? s * sdy + (float)HW * b0 + b1 * sx : 0.f;
      }
    }
  }
}

// ---- GroupNorm finalise (forward): image n's per-channel sums -> per-(image, group) mean / rstd over
// H*W*(c_valid/G) values of u = v + feat[n]; the conv-prologue affine becomes per image:
// scale[n, c] = gamma[c] * rstd[n, g(c)], shift[n, c] = (feat[n, c] - mean[n, g]) * scale[n, c] + beta[c].
// One block per image (no cross-image dependency, so no last-block ticket).
__global__ __launch_bounds__(256) void gn_stats_fin_kernel(BnArgs a) {
  const int n = blockIdx.x, tid = threadIdx.x, HW = a.H * a.W;
  float* dst[2] = {st_sum(a), st_sq(a)};
  image_reduce<2>(a, n, dst);
  __syncthreads();
  __threadfence_block();
  const int G = a.groups, cg = a.c_valid / G;
  const float cnt = (float)HW * (float)cg;
  __shared__ float gm[256], gr[256];
  for (int g = tid; g < G; g += 256) {
    float s1 = 0.f, q = 0.f;
    for (int c = g * cg; c < (g + 1) * cg; ++c) {
      const float s = st_sum(a)[(size_t)n * a.C + c], sq = st_sq(a)[(size_t)n * a.C + c];
      const float f = a.feat ? a.feat[(size_t)n * a.C + c] : 0.f;
      s1 += s + (float)HW * f;
      q += sq + 2.f * f * s + (float)HW * f * f;
    }
    const float mean = s1 / cnt;
    gm[g] = mean;
    gr[g] = 1.f / sqrtf(fmaxf(q / cnt - mean * mean, 0.f) + a.eps);
  }
  __syncthreads();
  for (int c = tid; c < a.C; c += 256) {
    const bool valid = c < a.c_valid;
    const int g = valid ? c / cg : 0;
    const float mean = valid ? gm[g] : 0.f, rstd = valid ? gr[g] : 0.f;
    const size_t i = (size_t)n * a.C + c;
    st_mean(a)[i] = mean;
    st_rstd(a)[i] = rstd;
    const float f = a.feat ? a.feat[i] : 0.f;
    for (int k = 0; k < a.nunits; ++k) {
      const float sc = valid ? a.u.gamma[k][c] * rstd : 0.f;
      a.u.scale[k][i] = sc;
      a.u.shift[k][i] = valid ? (f - mean) * sc + a.u.beta[k][c] : 0.f;
    }
  }
}

// ---- GroupNorm finalise (backward): per (image, group) B0 = -sum_{c in g} scale*sum(dy) / M,
// B1 = -sum scale*sum(dy*xhat) / M (M = H*W*c_valid/G), summed over the units; dgamma / dbeta sum
// over images (last block); dfeat per (image, channel).
template <int NU>
__global__ __launch_bounds__(256) void gn_bwd_fin_kernel(BnArgs a) {
  const int n = blockIdx.x, tid = threadIdx.x, HW = a.H * a.W;
  float* dst[2 * NU];
#pragma unroll
  for (int k = 0; k < NU; ++k) { dst[2 * k] = st_sdy(a, k); dst[2 * k + 1] = st_sdyx(a, k); }
  image_reduce<2 * NU>(a, n, dst);
  __syncthreads();
  __threadfence_block();
  const int G = a.groups, cg = a.c_valid / G;
  const float M = (float)HW * (float)cg;
  __shared__ float gb0[256], gb1[256];
  for (int g = tid; g < G; g += 256) {
    float b0 = 0.f, b1 = 0.f;
    for (int k = 0; k < NU; ++k)
      for (int c = g * cg; c < (g + 1) * cg; ++c) {
        const size_t i = (size_t)n * a.C + c;
        const float s = a.u.scale[k][i];
        b0 -= s * st_sdy(a, k)[i] / M;
        b1 -= s * st_sdyx(a, k)[i] / M;
      }
    gb0[g] = b0;
    gb1[g] = b1;
  }
  __syncthreads();
  for (int c = tid; c < a.C; c += 256) {
    const bool valid = c < a.c_valid;
    const size_t i = (size_t)n * a.C + c;
    const float b0 = valid ? gb0[c / cg] : 0.f, b1 = valid ? gb1[c / cg] : 0.f;
    st_b0(a)[i] = b0;
    st_b1(a)[i] = b1;
    if (a.dfeat) {
      const float f = a.feat ? a.feat[i] : 0.f;
      const float sx = (st_sum(a)[i] + (float)HW * (f - st_mean(a)[i])) * st_rstd(a)[i];
      a.dfeat[i] = valid ? a.u.scale[0][i] * st_sdy(a, 0)[i] + (float)HW * b0 + b1 * sx : 0.f;
    }
  }
  if (!last_block(a.ticket + 1)) return;
  for (int c = tid; c < a.c_valid; c += 256) {
    for (int k = 0; k < NU; ++k) {
      float sdy = 0.f, sdyx = 0.f;
      for (int m = 0; m < a.N; ++m) {
        sdy += ld_acq(st_sdy(a, k) + (size_t)m * a.C + c);
        sdyx += ld_acq(st_sdyx(a, k) + (size_t)m * a.C + c);
      }
      if (a.u.dgamma[k]) a.u.dgamma[k][c] = sdyx;
      if (a.u.dbeta[k]) a.u.dbeta[k][c] = sdy;
    }
  }
}

// ---- backward apply: du at every post-transform pixel, routed into dx (T^T) and dx2
struct ApplyOut {
  bf16_t* dx;   // [N, Hs, Ws, C] or null
  bf16_t* dx2;  // [N, H, W, C] or null
  int dx_acc, dx2_acc;
};

__device__ __forceinline__ void store8(bf16_t* p, const float (&v)[8], bool acc) {
  float w[8];
  if (acc) {
    unpack8(*reinterpret_cast<const u32x4*>(p), w);
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] += v[j];
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = v[j];
  }
  u32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = pack2bf(w[2 * j], w[2 * j + 1]);
  *reinterpret_cast<u32x4*>(p) = o;
}

// Per-thread backward coefficients of its 8 channels (a thread's channel group never changes in the
// grid-stride loop: the stride is a multiple of C/8); per-image shift / feature rows are reloaded when
// the image index changes.
template <int NU>
struct Coef {
  float mean[8], rstd[8], b0[8], b1[8], sc[NU][8], sh[NU][8], f[8];
  int n;
  __device__ void coefs(const BnArgs& a, size_t cr) {
    ld8(st_mean(a) + cr, mean);
    ld8(st_rstd(a) + cr, rstd);
    ld8(st_b0(a) + cr, b0);
    ld8(st_b1(a) + cr, b1);
#pragma unroll
    for (int k = 0; k < NU; ++k) ld8(a.u.scale[k] + cr, sc[k]);
  }
  __device__ void init(const BnArgs& a, int c0) {
    n = -1;
    if (!a.cns) coefs(a, c0);  // BatchNorm: one coefficient row for the whole batch
  }
  __device__ void image(const BnArgs& a, int nn, int c0) {
    if (nn == n) return;
    n = nn;
    if (a.cns) coefs(a, (size_t)nn * a.cns + c0);
#pragma unroll
    for (int k = 0; k < NU; ++k) ld8(a.u.shift[k] + (size_t)nn * a.C + c0, sh[k]);
    if (a.feat) {
      ld8(a.feat + (size_t)nn * a.C + c0, f);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = 0.f;
    }
  }
};

template <int NU>
__device__ __forceinline__ void du8(const BnArgs& a, const Coef<NU>& cf, size_t opix, const float (&v)[8], int c0,
                                    float (&du)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) du[j] = fmaf(cf.b1[j], (v[j] + cf.f[j] - cf.mean[j]) * cf.rstd[j], cf.b0[j]);
#pragma unroll
  for (int k = 0; k < NU; ++k) {
    float d[8];
    unpack8(*reinterpret_cast<const u32x4*>(a.u.dact[k] + opix * a.C + c0), d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool on = !a.u.relu[k] || fmaf(v[j], cf.sc[k][j], cf.sh[k][j]) > 0.f;
      du[j] = on ? fmaf(cf.sc[k][j], d[j], du[j]) : du[j];
    }
  }
}

template <int INMODE, bool X2, int NU>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(BnArgs a, ApplyOut o) {
  const int C8 = a.C / 8;
  // INMODE 1 (up2): one thread per SOURCE pixel x 8 channels (gathers its 2x2 children);
  // otherwise one thread per output pixel x 8 channels.
  const int PH = INMODE == 1 ? a.Hs : a.H, PW = INMODE == 1 ? a.Ws : a.W;
  const long long total = (long long)a.N * PH * PW * C8;
  Coef<NU> cf;
  cf.init(a, (int)(threadIdx.x % C8) * 8);
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int cg = (int)(i % C8);
    const long long pp = i / C8;
    const int px = (int)(pp % PW), py = (int)((pp / PW) % PH), n = (int)(pp / ((long long)PW * PH));
    const int c0 = cg * 8;
    cf.image(a, n, c0);
    if (INMODE == 1) {
      float src[8], acc[8];
      unpack8(*reinterpret_cast<const u32x4*>(a.x + (((size_t)n * a.Hs + py) * a.Ws + px) * a.C + c0), src);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
      for (int ch = 0; ch < 4; ++ch) {
        const int oy = 2 * py + (ch >> 1), ox = 2 * px + (ch & 1);
        const size_t opix = ((size_t)n * a.H + oy) * a.W + ox;
        float v[8], du[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = src[j];
        if (X2) {
          float w[8];
          unpack8(*reinterpret_cast<const u32x4*>(a.x2 + opix * a.C + c0), w);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] += w[j];
        }
        du8<NU>(a, cf, opix, v, c0, du);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += du[j];
        if (X2 && o.dx2) store8(o.dx2 + opix * a.C + c0, du, o.dx2_acc);
      }
      if (o.dx) store8(o.dx + (((size_t)n * a.Hs + py) * a.Ws + px) * a.C + c0, acc, o.dx_acc);
    } else {
      const size_t opix = ((size_t)n * a.H + py) * a.W + px;
      float v[8], du[8];
      int am[8];
      if (INMODE == 2) {
        const bf16_t* base = a.x + (((size_t)n * a.Hs + 2 * py) * a.Ws + 2 * px) * a.C + c0;
        float s[4][8];
        unpack8(*reinterpret_cast<const u32x4*>(base), s[0]);
        unpack8(*reinterpret_cast<const u32x4*>(base + a.C), s[1]);
        unpack8(*reinterpret_cast<const u32x4*>(base + (size_t)a.Ws * a.C), s[2]);
        unpack8(*reinterpret_cast<const u32x4*>(base + (size_t)a.Ws * a.C + a.C), s[3]);
#pragma unroll
        for (int j = 0; j < 8; ++j) {  // first maximum in (0,0),(0,1),(1,0),(1,1) order
          float m = s[0][j];
          int k = 0;
#pragma unroll
          for (int e = 1; e < 4; ++e)
            if (s[e][j] > m) { m = s[e][j]; k = e; }
          v[j] = m;
          am[j] = k;
        }
      } else {
        unpack8(*reinterpret_cast<const u32x4*>(a.x + opix * a.C + c0), v);
      }
      if (X2) {
        float w[8];
        unpack8(*reinterpret_cast<const u32x4*>(a.x2 + opix * a.C + c0), w);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += w[j];
      }
      du8<NU>(a, cf, opix, v, c0, du);
      if (X2 && o.dx2) store8(o.dx2 + opix * a.C + c0, du, o.dx2_acc);
      if (o.dx) {
        if (INMODE == 2) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float g[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) g[j] = am[j] == e ? du[j] : 0.f;
            const int sy = 2 * py + (e >> 1), sx = 2 * px + (e & 1);
            store8(o.dx + (((size_t)n * a.Hs + sy) * a.Ws + sx) * a.C + c0, g, o.dx_acc);
          }
        } else {
          store8(o.dx + opix * a.C + c0, du, o.dx_acc);
        }
      }
    }
  }
}

template <int INMODE, bool X2>
int bn_dispatch_x2(int which, BnArgs a, ApplyOut o, hipStream_t s) {
  const int HW = a.H * a.W;
  const int nb = a.nb;
  dim3 grid(nb, a.N);
  if (which == 0) {
    hipLaunchKernelGGL((bn_stats_kernel<INMODE, X2>), grid, dim3(256), 0, s, a);
    if (a.groups) hipLaunchKernelGGL(gn_stats_fin_kernel, dim3(a.N), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(bn_stats_fin_kernel, dim3(a.N), dim3(256), 0, s, a);
  } else if (which == 1) {
    if (a.nunits == 2) {
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<INMODE, X2, 2>), grid, dim3(256), 0, s, a);
      if (a.groups) hipLaunchKernelGGL(gn_bwd_fin_kernel<2>, dim3(a.N), dim3(256), 0, s, a);
      else hipLaunchKernelGGL(bn_bwd_fin_kernel<2>, dim3(a.N), dim3(256), 0, s, a);
    } else {
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<INMODE, X2, 1>), grid, dim3(256), 0, s, a);
      if (a.groups) hipLaunchKernelGGL(gn_bwd_fin_kernel<1>, dim3(a.N), dim3(256), 0, s, a);
      else hipLaunchKernelGGL(bn_bwd_fin_kernel<1>, dim3(a.N), dim3(256), 0, s, a);
    }
  } else {
    const int PH = INMODE == 1 ? a.Hs : a.H, PW = INMODE == 1 ? a.Ws : a.W;
    const long long total = (long long)a.N * PH * PW * (a.C / 8);
    const int blocks = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
    if (a.nunits == 2) hipLaunchKernelGGL((bn_bwd_apply_kernel<INMODE, X2, 2>), dim3(blocks), dim3(256), 0, s, a, o);
    else hipLaunchKernelGGL((bn_bwd_apply_kernel<INMODE, X2, 1>), dim3(blocks), dim3(256), 0, s, a, o);
  }
  return BE_CHECK_LAUNCH();
}

int bn_dispatch(int which, BnArgs a, ApplyOut o, hipStream_t s) {
  if (a.C % 8 || a.C > 256 || 64 % (a.C / 8) || a.nunits < 1 || a.nunits > 2) return -1;
  if (a.groups && (a.groups > 256 || a.c_valid % a.groups)) return -3;
  const bool x2 = a.x2 != nullptr;
  switch (a.inmode) {
    case 0: return x2 ? bn_dispatch_x2<0, true>(which, a, o, s) : bn_dispatch_x2<0, false>(which, a, o, s);
    case 1: return x2 ? bn_dispatch_x2<1, true>(which, a, o, s) : bn_dispatch_x2<1, false>(which, a, o, s);
    case 2: return x2 ? bn_dispatch_x2<2, true>(which, a, o, s) : bn_dispatch_x2<2, false>(which, a, o, s);
  }
  return -2;
}

// ============================================================================================
// Weight packing (fp32 master -> bf16 MFMA layouts), all convs in one launch
// ============================================================================================

struct PackDesc {
  int src_off;   // element offset of W [cout, cin, ks, ks] in the flat fp32 master
  int dst_off;   // element offset in the bf16 arena
  int cout, cin, ks;
  int rows_pad;  // packed rows (cout_pad forward / cin_pad' dgrad)
  int in_pad;    // packed input channels (cin_pad forward / cout' dgrad)
  int ck, kp;
  int transpose; // 1 = dgrad layout: rows = cin, inputs = cout, taps flipped
};

__global__ __launch_bounds__(256) void pack_weights_kernel(const PackDesc* __restrict__ descs,
                                                           const float* __restrict__ flat, bf16_t* __restrict__ out) {
  const PackDesc d = descs[blockIdx.y];
  const int nchunk = d.in_pad / d.ck;
  const int total = d.rows_pad * nchunk * d.kp;
  const int kk = d.ks * d.ks;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int k = i % d.kp;
    const int ch = (i / d.kp) % nchunk;
    const int r = i / (d.kp * nchunk);
    float v = 0.f;
    if (k < kk * d.ck) {
      const int tap = k / d.ck, c = ch * d.ck + k % d.ck;
      if (!d.transpose) {
        if (r < d.cout && c < d.cin) v = flat[d.src_off + (r * d.cin + c) * kk + tap];
      } else {  // W'[ci][co][tap'] = W[co][ci][kk-1-tap']
        if (r < d.cin && c < d.cout) v = flat[d.src_off + (c * d.cin + r) * kk + (kk - 1 - tap)];
      }
    }
    out[d.dst_off + i] = f2bf(v);
  }
}

}  // namespace

extern "C" {

// Weight gradient (+ optional bias gradient) of one fused conv unit.  ws/wsb: fp32 partial workspace
// sized [splits][cout_valid][ks*ks][Cin] / [splits][cout_valid]; dw: [cout_valid, cin_valid, ks, ks].
int be_conv_wgrad(const void* x, const void* x2, const float* pscale, const float* pshift, int pshift_ns, int pscale_ns,
                  int relu,
                  const void* dy, float* ws, float* wsb, float* dw, float* db, int N, int H, int W, int Hs, int Ws,
                  int Cin, int cin_valid, int Cy, int cout_valid, int ks, int inmode, int splits, hipStream_t s) {
  if (Cin != 8 && Cin % 32) return -1;
  if (Cy % 8 || cout_valid > Cy || splits < 1) return -1;
  WgArgs a;
  a.x = (const bf16_t*)x; a.x2 = (const bf16_t*)x2; a.pscale = pscale; a.pshift = pshift;
  a.dy = (const bf16_t*)dy; a.ws = ws; a.wsb = db ? wsb : nullptr;
  a.N = N; a.H = H; a.W = W; a.Hs = Hs; a.Ws = Ws; a.Cin = Cin; a.Cy = Cy; a.cout_valid = cout_valid;
  a.pshift_ns = pshift_ns; a.pscale_ns = pscale_ns; a.relu = relu;
  a.tiles_x = (W + 31) / 32; a.tiles_y = (H + 3) / 4;
  a.ntiles = N * a.tiles_x * a.tiles_y;
  a.splits = splits < a.ntiles ? splits : a.ntiles;
  const int tco = Cy <= 16 ? 16 : (Cy <= 32 ? 32 : 64);
  int rc;
  if (ks == 3) rc = Cin == 8 ? wgrad_tco<3, 8>(tco, inmode, x2 != nullptr, a, s) : wgrad_tco<3, 32>(tco, inmode, x2 != nullptr, a, s);
  else if (ks == 1) rc = Cin == 8 ? wgrad_tco<1, 8>(tco, inmode, x2 != nullptr, a, s) : wgrad_tco<1, 32>(tco, inmode, x2 != nullptr, a, s);
  else return -4;
  if (rc) return rc;
  // dw / db must be zero on entry (the engine zeroes the flat gradient buffer once per step)
  const int ne = cout_valid * ks * ks * Cin + (db ? cout_valid : 0);
  static const int target = env_int("BE_WG_REDUCE_THREADS", 262144);
  int nch = (target + ne - 1) / ne;
  nch = nch < 1 ? 1 : (nch > 64 ? 64 : nch);
  nch = nch > a.splits ? a.splits : nch;
  dim3 rgrid((ne + 255) / 256, nch);
  hipLaunchKernelGGL(wgrad_reduce_kernel, rgrid, dim3(256), 0, s, ws, a.wsb, a.splits, cout_valid, ks * ks, Cin,
                     cin_valid, dw, db);
  return BE_CHECK_LAUNCH();
}

// which: 0 = forward statistics + finalise, 1 = backward reduce + finalise, 2 = backward apply.
// Pointer arrays hold up to two BN units sharing the same input (proj + conv_0 of a res block).
// groups = 0: BatchNorm (train-mode batch statistics); groups = G: GroupNorm with G groups of the
// c_valid channels per image (scale / shift / stat coefficient arrays are then per image: [N, C]).
int be_bn_train(int which, const void* x, const void* x2, const float* feat, int N, int Hs, int Ws, int H, int W, int C,
                int c_valid, int inmode, int nunits, float eps, float momentum, int groups, float* stat,
                unsigned* ticket,
                const float* gamma0, const float* beta0, float* scale0, float* shift0, float* rm0, float* rv0, int relu0,
                const void* dact0, float* dgamma0, float* dbeta0,
                const float* gamma1, const float* beta1, float* scale1, float* shift1, float* rm1, float* rv1, int relu1,
                const void* dact1, float* dgamma1, float* dbeta1,
                float* dfeat, void* dx, int dx_acc, void* dx2, int dx2_acc, float* scratch, int scratch_floats,
                hipStream_t s) {
  BnArgs a;
  a.x = (const bf16_t*)x; a.x2 = (const bf16_t*)x2; a.feat = feat;
  a.N = N; a.Hs = Hs; a.Ws = Ws; a.H = H; a.W = W; a.C = C; a.c_valid = c_valid; a.inmode = inmode;
  a.nunits = nunits; a.eps = eps; a.momentum = momentum; a.stat = stat; a.ticket = ticket;
  a.groups = groups; a.cns = groups ? C : 0;
  a.u.gamma[0] = gamma0; a.u.beta[0] = beta0; a.u.scale[0] = scale0; a.u.shift[0] = shift0;
  a.u.run_mean[0] = rm0; a.u.run_var[0] = rv0; a.u.relu[0] = relu0; a.u.dact[0] = (const bf16_t*)dact0;
  a.u.dgamma[0] = dgamma0; a.u.dbeta[0] = dbeta0;
  a.u.gamma[1] = gamma1; a.u.beta[1] = beta1; a.u.scale[1] = scale1; a.u.shift[1] = shift1;
  a.u.run_mean[1] = rm1; a.u.run_var[1] = rv1; a.u.relu[1] = relu1; a.u.dact[1] = (const bf16_t*)dact1;
  a.u.dgamma[1] = dgamma1; a.u.dbeta[1] = dbeta1;
  a.dfeat = dfeat;
  // ~4 blocks per CU over the whole tensor, at least 64 pixels per block
  const long long HW = (long long)H * W;
  static const int bn_blocks = env_int("BE_BN_BLOCKS", 512);
  const long long want = (bn_blocks + N - 1) / N;
  long long pb = (HW + want - 1) / want;
  pb = pb < 256 ? 256 : pb;
  // the partial scratch holds N * nb * NACC * C floats (NACC <= 4)
  long long nb = (HW + pb - 1) / pb;
  const long long cap = scratch_floats / ((long long)N * 4 * C);
  if (cap < 1) return -5;
  if (nb > cap) {
    nb = cap;
    pb = (HW + nb - 1) / nb;
  }
  a.per_block = (int)pb;
  a.nb = (int)((HW + pb - 1) / pb);
  a.scratch = scratch;
  ApplyOut o;
  o.dx = (bf16_t*)dx; o.dx2 = (bf16_t*)dx2; o.dx_acc = dx_acc; o.dx2_acc = dx2_acc;
  return bn_dispatch(which, a, o, s);
}

// descs: device array of `n` PackDesc (10 int32 each); one launch packs every conv.
int be_pack_conv_weights(const void* descs, int n, int max_elems, const float* flat, void* out, hipStream_t s) {
  if (n <= 0) return 0;
  int bx = (max_elems + 255) / 256;
  bx = bx < 1 ? 1 : (bx > 256 ? 256 : bx);
  hipLaunchKernelGGL(pack_weights_kernel, dim3(bx, n), dim3(256), 0, s, (const PackDesc*)descs, flat, (bf16_t*)out);
  return BE_CHECK_LAUNCH();
}

}  // extern "C"

// Fused pre-activation conv2d for the Cellpose U-Net family (and generic BioImage.IO U-Nets).
//
//   out = conv_{KSxKS}( act( inxform(x) [+ x2] ) ) [+ bias] [+ residual]
//   act(v) = relu?( v * scale[c] + shift[n, c] )          (eval BatchNorm / style shift folded)
//   inxform = identity | nearest-upsample x2 | maxpool 2x2  (fused into the halo loader)
//
// This is the hot op of Cellpose CPnet "batchconv" / "batchconvstyle" / "resdown" / "resup"
// blocks.  The reference reaches the same math through cellpose's
// nn.Sequential(BatchNorm2d, ReLU, Conv2d) modules (EXT, called from
// apps/model-runner/runtime_deployment.py:206-210 via cellpose==3.1.1.2).
//
// MI355X design:
//  * NHWC bf16 activations, implicit GEMM on v_mfma_f32_16x16x32_bf16 with the *weights as the A
//    operand* (rows = output channels) and pixels as B, so each lane ends with 4 consecutive
//    output channels of one pixel -> 8-byte stores in NHWC and 64-byte rows in NCHW heads.
//  * one workgroup = NW waves = a (2*NW)x32 output pixel tile x TCO output channels; the input
//    halo ((2NW+KS-1) x (32+KS-1) x CK channels) is staged through LDS once per Cin chunk with the
//    pre-activation (BN affine, style shift, skip add, ReLU, pool/upsample) applied in registers
//    on the way in, so the activated tensor never exists in HBM.
//  * software pipeline across Cin chunks: the global loads of chunk c+1 (halo + packed weights)
//    are issued into registers right after chunk c is committed to LDS, so they are in flight
//    while the MFMAs of chunk c run (register staging, "issue early / write late").
//  * K ordering inside a chunk is tap-major / channel-minor (k = tap*CK + c), so a 16-byte
//    B fragment is 8 contiguous channels of one shifted pixel; small-Cin layers (Cin=8) pack 4
//    taps into one 32-deep MFMA step instead of padding channels to 32.
//  * LDS layouts are bank-conflict-free for ds_read_b128 (lane groups {0-3,12-15,20-27},
//    {4-11,16-19,28-31}, ...; MI355X_MICROARCH.md §LDS): a fragment read is 16 rows (pixels or
//    output channels) x 4 K-chunks of 16 B, and a row stride of 8 (mod 64) dwords + 16 B chunks
//    maps every lane group onto 64 distinct banks for ANY row offset (halo shift dy, dx) — so the
//    layout stays linear (pixel stride CK+16 bf16, weight stride KPL+16) and the compiler folds
//    the tap offsets into ds_read immediates instead of holding ~50 swizzled addresses in VGPRs.
//    The previous +8 padding measured ~4 conflict cycles per LDS instruction
//    (SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS; profiles/conv_pmc_swizzled.txt shows 0 after the fix).
#include <cstdlib>

#include "common.h"

// Tuning experiments only (tools/build_native.py --variant): 1 = no halo loads, 2 = no output
// stores, 3 = no MFMAs.  0 in every shipped build.
#ifndef CONV_EXP
#define CONV_EXP 0
#endif
#ifndef CONV_SCHED_BARRIER
#define CONV_SCHED_BARRIER 1  // per-K-step scheduling fence: deep 3x3 layers 6.03 -> 5.78 ms/step (profiles/r03/conv_deep_ab.md)
#endif
// Output-channel-major block order for the one-tile-per-block kernel: the Cout/TCO blocks of one
// pixel tile are consecutive block ids, so the second..last of them find the tile's halo in L2
// instead of re-reading it from HBM once per output-channel tile.
#ifndef CONV_RES_PREFETCH
#define CONV_RES_PREFETCH 0  // 1: +32 VGPRs on a kernel already at the 256 cap -> 131 spills (not used)
#endif
#ifndef CONV_CO_MAJOR
#define CONV_CO_MAJOR 0
#endif

namespace {

constexpr int TW = 32;  // output tile cols (two 16-pixel MFMA column tiles)

struct ConvArgs {
  const bf16_t* x;       // [N, Hs, Ws, Cin]
  const bf16_t* x2;      // optional [N, H, W, Cin] added before the affine
  const float* pscale;   // optional [N?, Cin] (row stride pscale_ns: 0 => shared over batch; GroupNorm: Cin)
  const float* pshift;   // optional [N?, Cin]  (row stride pshift_ns: 0 => shared over batch)
  const bf16_t* w;       // packed [Cout_pad][nchunk][KP]
  const float* bias;     // optional [Cout]
  const bf16_t* res;     // optional residual [N, H, W, Cout]
  void* out;             // bf16 NHWC [N,H,W,Cout] or f32 NCHW [N,cout_valid,H,W]
  int N, H, W, Hs, Ws, Cin, Cout, cout_valid;
  int nchunk, KP;
  int pshift_ns, pscale_ns;
  int prelu;           // bit 0: ReLU on the (affine) input; bit 1: ReLU on the output (after bias/residual)
  int out_f32_nchw;
  int tiles_x, tiles_y;
  int persist_blocks;  // 0 = auto
  int cot;             // output-channel blocks (block order 2)
  int order;           // conv2d_nhwc_kernel block order: 0 tile-major, 2 XCD-grouped co-major (1-D grid)
  // optional post-activation of the stored value (the NEXT conv's pre-activation, applied by this
  // producer): v = bf16(v) * qscale[co] + qshift[n * qshift_ns + co], then the prelu bit-1 ReLU
  const float* qscale;
  const float* qshift;
  int qshift_ns;
  // INMODE 3 (3x3x3 conv as ONE 2-D launch over the N * zD slices): the K axis stacks the three
  // depth taps, stacked channel dz * zC + c = channel c of slice z + dz - 1 (zero outside the volume)
  // INMODE 4 (conv of a channel concatenation, the U-Net decoder's cat([skip, up])): channels
  // [0, zC) come from x ([N, H, W, zC]), channels [zC, Cin) from x2 ([N, H, W, Cin - zC])
  // INMODE 5 (INMODE 3 over a concatenation, the 3-D decoder): stacked channel dz * zC + c is
  // channel c of slice z + dz - 1 of x ([.., zA]) for c < zA, else channel c - zA of x2 ([.., zC - zA])
  int zD, zC, zA;
};

// Block order of the one-block-per-tile kernel.  Tile-major (grid x = tile, y = cout block) sends
// the cot blocks that read one input halo through the GPU ~`tiles` blocks apart: by the time the
// second one runs, the halo has left the XCD's 4 MiB L2 and comes back from the Infinity Cache
// (the deep 3x3 layers moved ~2.2 GB per 32-image batch through L2 -> LDS at ~7 TB/s).  Order 2
// numbers blocks so that each XCD works through a contiguous range of (tile, cout block) pairs,
// cout block fastest: a tile's cot blocks run back to back on one XCD and share its L2 copy of the
// halo, and the layer's weights stay L2-resident on every XCD.  BE_CONV_ORDER overrides (A/B).
static int conv_block_order() {
  static int o = [] {
    const char* e = getenv("BE_CONV_ORDER");
    return e ? atoi(e) : 2;
  }();
  return o;
}

template <int KS, int CK, int TCO, int INMODE, bool X2, int NW>
struct Cfg {
  static constexpr int NT = NW * 64;
  static constexpr int TH = 2 * NW;
  static constexpr int HH = TH + KS - 1;
  static constexpr int HW_ = TW + KS - 1;
  // dwords/pixel = 8 (mod 16) for CK = 16 / 32 / 64 (CK = 16 needs no pad: 8 dwords); CK = 8: 12
  static constexpr int PSTR = CK == 8 ? 24 : (CK == 16 ? 16 : CK + 16);
  static constexpr int KSTEPS = (KS * KS * CK + 31) / 32;
  static constexpr int KPL = KSTEPS * 32;
  static constexpr int WSTR = KPL + 16;
  static constexpr int CG = CK / 8;
  static constexpr int NCT = TCO / 16;
  static constexpr int HU = HH * HW_ * CG;
  static constexpr int HUPT = (HU + NT - 1) / NT;
  static constexpr int WU = TCO * KPL / 8;
  static constexpr int WUPT = (WU + NT - 1) / NT;
  static_assert(NT % CG == 0, "a thread's halo channel group must not change across units");
  static_assert((WSTR / 2) % 16 == 8, "weight row stride must be 8 (mod 16) dwords");
  static_assert(CK == 8 || (PSTR / 2) % 16 == 8, "pixel stride must be 8 (mod 16) dwords");
  // Output staging (coalesced 16-byte stores): each wave's 2 x 32 pixels x TCO bf16, placed over
  // the halo region once the MFMAs are done with it.  Chunk swizzle shift: see stage_off().
  static constexpr int OUT_WAVE = 2 * TW * TCO;  // bf16 elements per wave
  static constexpr int OSH = TCO == 16 ? 2 : (TCO == 32 ? 1 : 0);
  static constexpr int HREG = HH * HW_ * PSTR > NW * OUT_WAVE ? HH * HW_ * PSTR : NW * OUT_WAVE;
  static constexpr size_t LDS = (size_t)(HREG + TCO * WSTR) * sizeof(bf16_t);
};

template <typename C>
__device__ __forceinline__ int hoff(int pix, int cg) { return pix * C::PSTR + cg * 8; }
__device__ __forceinline__ int woff(int wstr, int r, int kc) { return r * wstr + kc * 8; }

// Issue the global loads of one Cin chunk into registers (halo raw values + packed weights).
template <typename C, int KS, int INMODE, bool X2>
__device__ __forceinline__ void issue_chunk(const ConvArgs& a, int n, int ty0, int tx0, int co0, int ch, int tid,
                                            u32x4 (&hraw)[C::HUPT], u32x4 (&h2raw)[X2 ? C::HUPT : 1],
                                            u32x4 (&wraw)[C::WUPT], float4 (&aff)[4], bool with_weights) {
  const int c0 = ch * (C::CG * 8);
  {  // this thread's 8 channels are the same for every halo unit (NT % CG == 0): prefetch the affine
    const int c = c0 + (tid % C::CG) * 8;
    if (a.pscale) {
      const float* sc = a.pscale + (size_t)n * a.pscale_ns + c;
      aff[0] = *reinterpret_cast<const float4*>(sc);
      aff[1] = *reinterpret_cast<const float4*>(sc + 4);
    }
    if (a.pshift) {
      const float* sr = a.pshift + (size_t)n * a.pshift_ns + c;
      aff[2] = *reinterpret_cast<const float4*>(sr);
      aff[3] = *reinterpret_cast<const float4*>(sr + 4);
    }
  }
#pragma unroll
  for (int i = 0; i < C::HUPT; ++i) {
    const int u = tid + i * C::NT;
    u32x4 r = (u32x4){0u, 0u, 0u, 0u};
    u32x4 r2 = (u32x4){0u, 0u, 0u, 0u};
    if (CONV_EXP != 1 && u < C::HU) {
      const int pix = u / C::CG, cg = u % C::CG;
      const int gy = ty0 + pix / C::HW_ - KS / 2, gx = tx0 + pix % C::HW_ - KS / 2;
      if (gy >= 0 && gy < a.H && gx >= 0 && gx < a.W) {
        const int c = c0 + cg * 8;
        if (INMODE == 0) {
          r = *reinterpret_cast<const u32x4*>(a.x + (((size_t)n * a.Hs + gy) * a.Ws + gx) * a.Cin + c);
        } else if (INMODE == 3) {
          const int dz = c / a.zC - 1, cz = c - (dz + 1) * a.zC;  // zC % CK == 0: one slice per chunk
          const int zz = n % a.zD + dz;
          if (zz >= 0 && zz < a.zD)
            r = *reinterpret_cast<const u32x4*>(a.x + (((size_t)(n + dz) * a.Hs + gy) * a.Ws + gx) * a.zC + cz);
        } else if (INMODE == 5) {
          const int dz = c / a.zC - 1, cz = c - (dz + 1) * a.zC;
          const int zz = n % a.zD + dz;
          if (zz >= 0 && zz < a.zD) {
            const size_t pix = ((size_t)(n + dz) * a.Hs + gy) * a.Ws + gx;
            if (cz < a.zA)
              r = *reinterpret_cast<const u32x4*>(a.x + pix * a.zA + cz);
            else
              r = *reinterpret_cast<const u32x4*>(a.x2 + pix * (a.zC - a.zA) + (cz - a.zA));
          }
        } else if (INMODE == 4) {  // zC % 8 == 0 (host-checked): an 8-channel group never straddles the seam
          if (c < a.zC)
            r = *reinterpret_cast<const u32x4*>(a.x + (((size_t)n * a.H + gy) * a.W + gx) * a.zC + c);
          else
            r = *reinterpret_cast<const u32x4*>(a.x2 + (((size_t)n * a.H + gy) * a.W + gx) * (a.Cin - a.zC) + (c - a.zC));
        } else if (INMODE == 6) {  // INMODE 4 with x2 still in the 2x2 transposed conv's sub-pixel layout
          if (c < a.zC) {
            r = *reinterpret_cast<const u32x4*>(a.x + (((size_t)n * a.H + gy) * a.W + gx) * a.zC + c);
          } else {
            const int cb = a.Cin - a.zC, sub = (gy & 1) * 2 + (gx & 1);
            r = *reinterpret_cast<const u32x4*>(
                a.x2 + (((size_t)n * (a.H >> 1) + (gy >> 1)) * (a.W >> 1) + (gx >> 1)) * (4 * cb) + sub * cb + (c - a.zC));
          }
        } else if (INMODE == 1) {
          r = *reinterpret_cast<const u32x4*>(a.x + (((size_t)n * a.Hs + (gy >> 1)) * a.Ws + (gx >> 1)) * a.Cin + c);
        } else {
          const bf16_t* base = a.x + (((size_t)n * a.Hs + 2 * gy) * a.Ws + 2 * gx) * a.Cin + c;
          const u32x4 r0 = *reinterpret_cast<const u32x4*>(base);
          const u32x4 r1 = *reinterpret_cast<const u32x4*>(base + a.Cin);
          const u32x4 q0 = *reinterpret_cast<const u32x4*>(base + (size_t)a.Ws * a.Cin);
          const u32x4 q1 = *reinterpret_cast<const u32x4*>(base + (size_t)a.Ws * a.Cin + a.Cin);
#pragma unroll
          for (int j = 0; j < 4; ++j) {  // max of bf16 values is exact in bf16
            const float lo = fmaxf(fmaxf(lo_bf(r0[j]), lo_bf(r1[j])), fmaxf(lo_bf(q0[j]), lo_bf(q1[j])));
            const float hi = fmaxf(fmaxf(hi_bf(r0[j]), hi_bf(r1[j])), fmaxf(hi_bf(q0[j]), hi_bf(q1[j])));
            r[j] = (__float_as_uint(lo) >> 16) | (__float_as_uint(hi) & 0xffff0000u);
          }
        }
        if (X2) r2 = *reinterpret_cast<const u32x4*>(a.x2 + (((size_t)n * a.H + gy) * a.W + gx) * a.Cin + c);
      }
    }
    if (CONV_EXP == 1) r = (u32x4){(uint32_t)u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u};
    hraw[i] = r;
    if (X2) h2raw[i] = r2;
  }
  if (!with_weights) return;
#pragma unroll
  for (int i = 0; i < C::WUPT; ++i) {
    const int u = tid + i * C::NT;
    if (u < C::WU) {
      const int r = u / (C::KPL / 8), k8 = u % (C::KPL / 8);
      wraw[i] = *reinterpret_cast<const u32x4*>(a.w + ((size_t)(co0 + r) * a.nchunk + ch) * a.KP + k8 * 8);
    }
  }
}

// Apply the pre-activation to the staged registers and write the chunk into LDS.
template <typename C, int KS, bool X2>
__device__ __forceinline__ void commit_chunk(const ConvArgs& a, int ty0, int tx0, int tid,
                                             const u32x4 (&hraw)[C::HUPT], const u32x4 (&h2raw)[X2 ? C::HUPT : 1],
                                             const u32x4 (&wraw)[C::WUPT], const float4 (&aff)[4], bf16_t* hl, bf16_t* wl,
                                             bool with_weights) {
  const float sc[8] = {aff[0].x, aff[0].y, aff[0].z, aff[0].w, aff[1].x, aff[1].y, aff[1].z, aff[1].w};
  const float sh[8] = {aff[2].x, aff[2].y, aff[2].z, aff[2].w, aff[3].x, aff[3].y, aff[3].z, aff[3].w};
#pragma unroll
  for (int i = 0; i < C::HUPT; ++i) {
    const int u = tid + i * C::NT;
    if (u >= C::HU) continue;
    const int pix = u / C::CG, cg = u % C::CG;
    const int gy = ty0 + pix / C::HW_ - KS / 2, gx = tx0 + pix % C::HW_ - KS / 2;
    u32x4 packed = (u32x4){0u, 0u, 0u, 0u};
    if (gy >= 0 && gy < a.H && gx >= 0 && gx < a.W) {  // conv zero-padding applies AFTER the activation
      float v[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[2 * j] = lo_bf(hraw[i][j]); v[2 * j + 1] = hi_bf(hraw[i][j]); }
      if (X2) {
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[2 * j] += lo_bf(h2raw[i][j]); v[2 * j + 1] += hi_bf(h2raw[i][j]); }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fmaf(v[j], sc[j], sh[j]);
#pragma unroll
      for (int j = 0; j < 4; ++j) packed[j] = pack2bf(v[2 * j], v[2 * j + 1]);
      if (a.prelu & 1) {  // ReLU commutes with the (monotone, sign-preserving) bf16 rounding
#pragma unroll
        for (int j = 0; j < 4; ++j) packed[j] = relu_bf16x2(packed[j]);
      }
    }
    *reinterpret_cast<u32x4*>(hl + hoff<C>(pix, cg)) = packed;
  }
  if (!with_weights) return;
#pragma unroll
  for (int i = 0; i < C::WUPT; ++i) {
    const int u = tid + i * C::NT;
    if (u < C::WU) {
      const int r = u / (C::KPL / 8), k8 = u % (C::KPL / 8);
      *reinterpret_cast<u32x4*>(wl + woff(C::WSTR, r, k8)) = wraw[i];
    }
  }
}

// K loop of one staged chunk.  Fragments of step ks+1 are read while the MFMAs of step ks run
// (explicit register double buffer); the scheduling barrier keeps the compiler from hoisting every
// step's ds_reads to the top, which cost ~100 VGPRs (and the occupancy) in the fully unrolled loop.
template <typename C, int KS>
__device__ __forceinline__ void load_frags(int ks, const bf16_t* hl, const bf16_t* wl, int wave, int lrow, int kq,
                                           bf16x8 (&af)[C::NCT], bf16x8 (&bfr)[4]) {
  const int g = ks * 4 + kq;
  int tap = g / C::CG;
  const int cg = g % C::CG;
  if (tap >= KS * KS) tap = 0;  // zero-weight K padding: read any finite data
  const int dy = tap / KS, dx = tap % KS;
#pragma unroll
  for (int ct = 0; ct < C::NCT; ++ct)
    af[ct] = *reinterpret_cast<const bf16x8*>(wl + woff(C::WSTR, ct * 16 + lrow, ks * 4 + kq));
#pragma unroll
  for (int pt = 0; pt < 4; ++pt) {
    const int py = 2 * wave + (pt >> 1);
    const int px = (pt & 1) * 16 + lrow;
    bfr[pt] = *reinterpret_cast<const bf16x8*>(hl + hoff<C>((py + dy) * C::HW_ + (px + dx), cg));
  }
}

template <typename C, int KS>
__device__ __forceinline__ void mma_chunk(f32x4 (&acc)[C::NCT][4], const bf16_t* hl, const bf16_t* wl, int wave,
                                          int lrow, int kq) {
  bf16x8 af[2][C::NCT], bfr[2][4];
  load_frags<C, KS>(0, hl, wl, wave, lrow, kq, af[0], bfr[0]);
#pragma unroll
  for (int ks = 0; ks < C::KSTEPS; ++ks) {
    const int cur = ks & 1;
    if (ks + 1 < C::KSTEPS) load_frags<C, KS>(ks + 1, hl, wl, wave, lrow, kq, af[cur ^ 1], bfr[cur ^ 1]);
#pragma unroll
    for (int ct = 0; ct < C::NCT; ++ct)
#pragma unroll
      for (int pt = 0; pt < 4; ++pt)
        if constexpr (CONV_EXP == 3) {
          acc[ct][pt][0] += __builtin_bit_cast(float, (int)(af[cur][ct][0] ^ bfr[cur][pt][1]));
        } else {
          acc[ct][pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[cur][ct], bfr[cur][pt], acc[ct][pt], 0, 0, 0);
        }
#if CONV_SCHED_BARRIER
    __builtin_amdgcn_sched_barrier(0);
#endif
  }
}

template <typename C>
__device__ __forceinline__ void load_bias(const ConvArgs& a, int co0, int kq, float4 (&bias)[C::NCT]) {
#pragma unroll
  for (int ct = 0; ct < C::NCT; ++ct) {
    const int co = co0 + ct * 16 + kq * 4;
    bias[ct] = (a.bias && !a.out_f32_nchw && co < a.Cout) ? *reinterpret_cast<const float4*>(a.bias + co)
                                                          : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// All global loads (residual) are issued before the first store: out may alias nothing, but the
// compiler cannot know that, and a load->wait->store chain per fragment serialises 8-16 memory
// latencies per tile (measured: ~45% of wave cycles in SQ_WAIT_ANY before this ordering).
// Staging layout: pixel-major, TCO bf16 per pixel, 16-byte chunks XOR-swizzled by pixel bits so
// both the 8-byte fragment writes (16 pixels x one channel quad per lane group: 2-way at most) and
// the 16-byte row reads (conflict-free) spread over the banks.
template <typename C>
__device__ __forceinline__ int stage_off(int p, int co) {
  constexpr int CPP = C::NCT * 2;  // 16-byte chunks per pixel
  return p * (C::NCT * 16) + ((co >> 3) ^ ((p >> C::OSH) & (CPP - 1))) * 8 + (co & 7);
}

template <typename C>
__device__ __forceinline__ void load_res_regs(const ConvArgs& a, int n, int ty0, int tx0, int co0, int wave, int lrow,
                                              int kq, u32x2 (&rv)[4][C::NCT]) {
#pragma unroll
  for (int pt = 0; pt < 4; ++pt) {
    const int py = ty0 + 2 * wave + (pt >> 1);
    const int px = tx0 + (pt & 1) * 16 + lrow;
    const bool ok = a.res && py < a.H && px < a.W;
    const size_t pix = ((size_t)n * a.H + py) * a.W + px;
#pragma unroll
    for (int ct = 0; ct < C::NCT; ++ct) {
      const int co = co0 + ct * 16 + kq * 4;
      rv[pt][ct] = (ok && co < a.Cout) ? *reinterpret_cast<const u32x2*>(a.res + pix * a.Cout + co) : (u32x2){0u, 0u};
    }
  }
}

// Post-activation (producer-side pre-activation of the consumer): the affine acts on the
// bf16-rounded value, exactly as if the consumer re-read this tensor and applied it itself.
__device__ __forceinline__ void post_affine(const ConvArgs& a, int n, int co, float& v0, float& v1, float& v2,
                                            float& v3) {
  if (!a.qscale && !a.qshift) return;
  const float4 qs = a.qscale ? *reinterpret_cast<const float4*>(a.qscale + co) : make_float4(1.f, 1.f, 1.f, 1.f);
  const float4 qt = a.qshift ? *reinterpret_cast<const float4*>(a.qshift + (size_t)n * a.qshift_ns + co)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
  const uint32_t p0 = pack2bf(v0, v1), p1 = pack2bf(v2, v3);
  v0 = fmaf(lo_bf(p0), qs.x, qt.x);
  v1 = fmaf(hi_bf(p0), qs.y, qt.y);
  v2 = fmaf(lo_bf(p1), qs.z, qt.z);
  v3 = fmaf(hi_bf(p1), qs.w, qt.w);
}

// rvp: residual registers loaded earlier (load_res_regs), or null to load them here
template <typename C>
__device__ __forceinline__ void epilogue(const ConvArgs& a, f32x4 (&acc)[C::NCT][4], const float4 (&bias)[C::NCT],
                                         int n, int ty0, int tx0, int co0, int wave, int lrow, int kq,
                                         bf16_t* stage, const u32x2 (*rvp)[C::NCT] = nullptr) {
  if (a.out_f32_nchw) {
#pragma unroll
    for (int pt = 0; pt < 4; ++pt) {
      const int py = ty0 + 2 * wave + (pt >> 1);
      const int px = tx0 + (pt & 1) * 16 + lrow;
      if (py >= a.H || px >= a.W) continue;
      float* o = reinterpret_cast<float*>(a.out);
#pragma unroll
      for (int ct = 0; ct < C::NCT; ++ct) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = co0 + ct * 16 + kq * 4 + i;
          if (c < a.cout_valid) {
            float r = acc[ct][pt][i] + (a.bias ? a.bias[c] : 0.f);
            if (a.prelu & 2) r = fmaxf(r, 0.f);
            o[(((size_t)n * a.cout_valid + c) * a.H + py) * a.W + px] = r;
          }
        }
      }
    }
    return;
  }
  u32x2 rv[4][C::NCT];
  if (rvp) {
#pragma unroll
    for (int pt = 0; pt < 4; ++pt)
#pragma unroll
      for (int ct = 0; ct < C::NCT; ++ct) rv[pt][ct] = rvp[pt][ct];
  } else if (a.res) {
    load_res_regs<C>(a, n, ty0, tx0, co0, wave, lrow, kq, rv);
  } else {
#pragma unroll
    for (int pt = 0; pt < 4; ++pt)
#pragma unroll
      for (int ct = 0; ct < C::NCT; ++ct) rv[pt][ct] = (u32x2){0u, 0u};
  }
  const bool post = a.prelu & 2;
  if (stage != nullptr) {  // Cout % 8 == 0: stage the wave's 2x32xTCO tile, then full-row 16-byte stores
    bf16_t* ws = stage + wave * C::OUT_WAVE;
#pragma unroll
    for (int pt = 0; pt < 4; ++pt) {
      const int p = (pt >> 1) * TW + (pt & 1) * 16 + lrow;
#pragma unroll
      for (int ct = 0; ct < C::NCT; ++ct) {
        const int col = ct * 16 + kq * 4;
        float v0 = acc[ct][pt][0] + bias[ct].x + lo_bf(rv[pt][ct][0]);
        float v1 = acc[ct][pt][1] + bias[ct].y + hi_bf(rv[pt][ct][0]);
        float v2 = acc[ct][pt][2] + bias[ct].z + lo_bf(rv[pt][ct][1]);
        float v3 = acc[ct][pt][3] + bias[ct].w + hi_bf(rv[pt][ct][1]);
        if (co0 + col < a.Cout) post_affine(a, n, co0 + col, v0, v1, v2, v3);
        u32x2 st;
        st[0] = pack2bf(v0, v1);
        st[1] = pack2bf(v2, v3);
        if (post) {
          st[0] = relu_bf16x2(st[0]);
          st[1] = relu_bf16x2(st[1]);
        }
        *reinterpret_cast<u32x2*>(ws + stage_off<C>(p, col)) = st;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    constexpr int CPP = C::NCT * 2;
    const int lane = lrow + 16 * kq;
#pragma unroll
    for (int it = 0; it < 2 * TW * CPP / 64; ++it) {
      const int q = it * 64 + lane;
      const int p = q / CPP, c = q % CPP;
      const int py = ty0 + 2 * wave + p / TW, px = tx0 + p % TW;
      const int co = co0 + c * 8;
      const u32x4 v = *reinterpret_cast<const u32x4*>(ws + stage_off<C>(p, c * 8));
      if (py < a.H && px < a.W && co < a.Cout)
        *reinterpret_cast<u32x4*>(reinterpret_cast<bf16_t*>(a.out) + (((size_t)n * a.H + py) * a.W + px) * a.Cout + co) = v;
    }
    return;
  }
#pragma unroll
  for (int pt = 0; pt < 4; ++pt) {
    const int py = ty0 + 2 * wave + (pt >> 1);
    const int px = tx0 + (pt & 1) * 16 + lrow;
    if (py >= a.H || px >= a.W) continue;
    const size_t pix = ((size_t)n * a.H + py) * a.W + px;
#pragma unroll
    for (int ct = 0; ct < C::NCT; ++ct) {
      const int co = co0 + ct * 16 + kq * 4;
      if (co >= a.Cout) continue;
      float v0 = acc[ct][pt][0] + bias[ct].x + lo_bf(rv[pt][ct][0]);
      float v1 = acc[ct][pt][1] + bias[ct].y + hi_bf(rv[pt][ct][0]);
      float v2 = acc[ct][pt][2] + bias[ct].z + lo_bf(rv[pt][ct][1]);
      float v3 = acc[ct][pt][3] + bias[ct].w + hi_bf(rv[pt][ct][1]);
      post_affine(a, n, co, v0, v1, v2, v3);
      u32x2 st;
      st[0] = pack2bf(v0, v1);
      st[1] = pack2bf(v2, v3);
      if (post) {
        st[0] = relu_bf16x2(st[0]);
        st[1] = relu_bf16x2(st[1]);
      }
      if (CONV_EXP != 2 || a.cout_valid == -12345)
        *reinterpret_cast<u32x2*>(reinterpret_cast<bf16_t*>(a.out) + pix * a.Cout + co) = st;
    }
  }
}

// Persistent over pixel tiles: block b handles tiles b, b + gridDim.x, ...; the (tile, chunk)
// stages form one software pipeline, so the next tile's halo loads overlap this tile's MFMAs and
// its epilogue stores.  Single-chunk layers keep their weights resident in LDS for all tiles.
template <int KS, int CK, int TCO, int INMODE, bool X2, int NW>
#ifndef CONV_PERSIST_WPE
#define CONV_PERSIST_WPE 2
#endif
__global__ __launch_bounds__(NW * 64, CONV_PERSIST_WPE) void conv2d_nhwc_persist(ConvArgs a) {
  using C = Cfg<KS, CK, TCO, INMODE, X2, NW>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* hl = reinterpret_cast<bf16_t*>(smem);
  bf16_t* wl = hl + C::HREG;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int lrow = lane & 15;
  const int kq = lane >> 4;
  const int tiles_per_img = a.tiles_x * a.tiles_y;
  const int total = a.N * tiles_per_img;
  const int co0 = blockIdx.y * TCO;
  const bool resident_w = a.nchunk == 1;
  const bool staged = !a.out_f32_nchw && (a.Cout & 7) == 0;

  int tile = blockIdx.x;
  if (tile >= total) return;
  int n = tile / tiles_per_img;
  int ty0 = ((tile % tiles_per_img) / a.tiles_x) * C::TH;
  int tx0 = ((tile % tiles_per_img) % a.tiles_x) * TW;
  int ch = 0;

  f32x4 acc[C::NCT][4];
#pragma unroll
  for (int i = 0; i < C::NCT; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  u32x4 hraw[C::HUPT];
  u32x4 h2raw[X2 ? C::HUPT : 1];
  u32x4 wraw[C::WUPT];
  float4 aff[4] = {make_float4(1.f, 1.f, 1.f, 1.f), make_float4(1.f, 1.f, 1.f, 1.f), make_float4(0.f, 0.f, 0.f, 0.f),
                   make_float4(0.f, 0.f, 0.f, 0.f)};
  float4 bias[C::NCT];
  load_bias<C>(a, co0, kq, bias);
  issue_chunk<C, KS, INMODE, X2>(a, n, ty0, tx0, co0, 0, tid, hraw, h2raw, wraw, aff, true);
  bool first = true;
  for (;;) {
    if (!first) __syncthreads();  // MFMAs of the previous stage finished reading LDS
    commit_chunk<C, KS, X2>(a, ty0, tx0, tid, hraw, h2raw, wraw, aff, hl, wl, first || !resident_w);
    __syncthreads();
    first = false;
    // next stage (chunk ch+1 of this tile, or chunk 0 of the next tile)
    int nch = ch + 1, ntile = tile;
    if (nch == a.nchunk) { nch = 0; ntile += gridDim.x; }
    // TCO=64 tiles keep 64 accumulator registers live; crossing tiles in the same block would
    // spill, so only the <=32-channel layers (latency-bound, 1 chunk) run persistent.
    const bool more = ntile < total;
    int nn = n, nty0 = ty0, ntx0 = tx0;
    if (more) {
      nn = ntile / tiles_per_img;
      nty0 = ((ntile % tiles_per_img) / a.tiles_x) * C::TH;
      ntx0 = ((ntile % tiles_per_img) % a.tiles_x) * TW;
      issue_chunk<C, KS, INMODE, X2>(a, nn, nty0, ntx0, co0, nch, tid, hraw, h2raw, wraw, aff, !resident_w);
    }
    mma_chunk<C, KS>(acc, hl, wl, wave, lrow, kq);
    if (ch == a.nchunk - 1) {
      bf16_t* stage = nullptr;
      if (staged) {
        __syncthreads();  // every wave is done reading the halo the staging area overlays
        stage = hl;
      }
      epilogue<C>(a, acc, bias, n, ty0, tx0, co0, wave, lrow, kq, stage);
#pragma unroll
      for (int i = 0; i < C::NCT; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    if (!more) break;
    tile = ntile; ch = nch; n = nn; ty0 = nty0; tx0 = ntx0;
  }
}

// One block per pixel tile (no cross-tile pipeline): the 64-output-channel variants need all
// their registers for accumulators + the chunk prefetch, and their multi-chunk K loop already
// overlaps loads with MFMAs.
template <int KS, int CK, int TCO, int INMODE, bool X2, int NW>
#ifndef CONV_KERNEL_WPE
#define CONV_KERNEL_WPE 2
#endif
__global__ __launch_bounds__(NW * 64, X2 ? 1 : CONV_KERNEL_WPE) void conv2d_nhwc_kernel(ConvArgs a) {
  using C = Cfg<KS, CK, TCO, INMODE, X2, NW>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* hl = reinterpret_cast<bf16_t*>(smem);
  bf16_t* wl = hl + C::HREG;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int lrow = lane & 15;
  const int kq = lane >> 4;
  const int tiles_per_img = a.tiles_x * a.tiles_y;
  int tile, cob;
  if (a.order == 2) {
    const int lid = xcd_remap(blockIdx.x, gridDim.x);
    tile = lid / a.cot;
    cob = lid % a.cot;
  } else {
    tile = CONV_CO_MAJOR ? blockIdx.y : blockIdx.x;
    cob = CONV_CO_MAJOR ? blockIdx.x : blockIdx.y;
  }
  const int n = tile / tiles_per_img;
  const int ty0 = ((tile % tiles_per_img) / a.tiles_x) * C::TH;
  const int tx0 = ((tile % tiles_per_img) % a.tiles_x) * TW;
  const int co0 = cob * TCO;
  f32x4 acc[C::NCT][4];
#pragma unroll
  for (int i = 0; i < C::NCT; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  u32x4 hraw[C::HUPT];
  u32x4 h2raw[X2 ? C::HUPT : 1];
  u32x4 wraw[C::WUPT];
  float4 aff[4] = {make_float4(1.f, 1.f, 1.f, 1.f), make_float4(1.f, 1.f, 1.f, 1.f), make_float4(0.f, 0.f, 0.f, 0.f),
                   make_float4(0.f, 0.f, 0.f, 0.f)};
  issue_chunk<C, KS, INMODE, X2>(a, n, ty0, tx0, co0, 0, tid, hraw, h2raw, wraw, aff, true);
  // residual operand fetched at tile start: its latency hides behind the K loop (the registers are
  // free -- occupancy here is set by LDS, two blocks per CU); it was exposed at the epilogue
  u32x2 rv[4][C::NCT];
  if (CONV_RES_PREFETCH) load_res_regs<C>(a, n, ty0, tx0, co0, wave, lrow, kq, rv);
  for (int ch = 0; ch < a.nchunk; ++ch) {
    if (ch > 0) __syncthreads();
    commit_chunk<C, KS, X2>(a, ty0, tx0, tid, hraw, h2raw, wraw, aff, hl, wl, true);
    __syncthreads();
    if (ch + 1 < a.nchunk)
      issue_chunk<C, KS, INMODE, X2>(a, n, ty0, tx0, co0, ch + 1, tid, hraw, h2raw, wraw, aff, true);
    mma_chunk<C, KS>(acc, hl, wl, wave, lrow, kq);
  }
  float4 bias[C::NCT];
  load_bias<C>(a, co0, kq, bias);
  bf16_t* stage = nullptr;
  if (!a.out_f32_nchw && (a.Cout & 7) == 0) {
    __syncthreads();
    stage = hl;
  }
  epilogue<C>(a, acc, bias, n, ty0, tx0, co0, wave, lrow, kq, stage, CONV_RES_PREFETCH ? rv : nullptr);
}

template <int KS, int CK, int TCO, int INMODE, bool X2, int NW>
int launch(ConvArgs a, hipStream_t s) {
  using C = Cfg<KS, CK, TCO, INMODE, X2, NW>;
  a.tiles_x = (a.W + TW - 1) / TW;
  a.tiles_y = (a.H + C::TH - 1) / C::TH;
  const int tiles = a.N * a.tiles_x * a.tiles_y;
  const int cot = (a.Cout + TCO - 1) / TCO;
  // persistent blocks: ~4 resident workgroups per CU across the cout tiles (256 CUs)
  if constexpr (TCO > 32) {  // non-persistent variant: one block per tile
    a.cot = cot;
    a.order = conv_block_order();
    if (a.order == 2 && (long long)tiles * cot < (1LL << 31)) {
      hipLaunchKernelGGL((conv2d_nhwc_kernel<KS, CK, TCO, INMODE, X2, NW>), dim3((unsigned)(tiles * cot)), dim3(C::NT),
                         C::LDS, s, a);
      return BE_CHECK_LAUNCH();
    }
    a.order = 0;
    if (CONV_CO_MAJOR && tiles > 65535) return -13;
    hipLaunchKernelGGL((conv2d_nhwc_kernel<KS, CK, TCO, INMODE, X2, NW>), CONV_CO_MAJOR ? dim3(cot, tiles) : dim3(tiles, cot),
                       dim3(C::NT), C::LDS, s, a);
    return BE_CHECK_LAUNCH();
  } else {
  int gx = (256 * 4 * (NW == 4 ? 2 : 1)) / cot;
  if (a.persist_blocks > 0) gx = a.persist_blocks;
  if (gx < 1) gx = 1;
  if (gx > tiles) gx = tiles;
  hipLaunchKernelGGL((conv2d_nhwc_persist<KS, CK, TCO, INMODE, X2, NW>), dim3(gx, cot), dim3(C::NT), C::LDS, s, a);
  return BE_CHECK_LAUNCH();
  }
}

template <int KS, int CK, int TCO, int INMODE, bool X2>
int dispatch_nw(int nw, const ConvArgs& a, hipStream_t s) {
  if (nw == 8) return launch<KS, CK, TCO, INMODE, X2, 8>(a, s);
  return launch<KS, CK, TCO, INMODE, X2, 4>(a, s);
}

template <int KS, int CK, int TCO>
int dispatch_mode(int inmode, bool x2, int nw, const ConvArgs& a, hipStream_t s) {
  if (x2) {
    if (inmode != 0) return -3;
    return dispatch_nw<KS, CK, TCO, 0, true>(nw, a, s);
  }
  switch (inmode) {
    case 0: return dispatch_nw<KS, CK, TCO, 0, false>(nw, a, s);
    case 1: return dispatch_nw<KS, CK, TCO, 1, false>(nw, a, s);
    case 2: return dispatch_nw<KS, CK, TCO, 2, false>(nw, a, s);
  }
  return -1;
}

template <int KS, int CK>
int dispatch_tco(int tco, int inmode, bool x2, int nw, const ConvArgs& a, hipStream_t s) {
  switch (tco) {
    case 16: return dispatch_mode<KS, CK, 16>(inmode, x2, nw, a, s);
    case 32: return dispatch_mode<KS, CK, 32>(inmode, x2, nw, a, s);
    case 64: return dispatch_mode<KS, CK, 64>(inmode, x2, nw, a, s);
  }
  return -2;
}

}  // namespace

template <int CK, int MODE>
int dispatch_concat(int tco, int nw, const ConvArgs& a, hipStream_t s) {
  switch (tco) {
    case 16: return dispatch_nw<3, CK, 16, MODE, false>(nw, a, s);
    case 32: return dispatch_nw<3, CK, 32, MODE, false>(nw, a, s);
    case 64: return dispatch_nw<3, CK, 64, MODE, false>(nw, a, s);
  }
  return -2;
}

template <int CK, int MODE = 3>
int dispatch_ztaps(int tco, int nw, const ConvArgs& a, hipStream_t s) {
  switch (tco) {
    case 16: return dispatch_nw<3, CK, 16, MODE, false>(nw, a, s);
    case 32: return dispatch_nw<3, CK, 32, MODE, false>(nw, a, s);
    case 64: return dispatch_nw<3, CK, 64, MODE, false>(nw, a, s);
  }
  return -2;
}

static int g_persist_blocks = 0;  // tuning override (0 = heuristic)

extern "C" {

int be_conv2d_set_persist(int blocks) {
  g_persist_blocks = blocks;
  return 0;
}

// Returns the K chunk length (padded) the packed weight layout must use for (ks, ck).
int be_conv2d_packed_kp(int ks, int ck) { return ((ks * ks * ck + 31) / 32) * 32; }

int be_conv2d_nhwc(const void* x, const void* x2, const float* pscale, const float* pshift, int pshift_ns, int pscale_ns,
                   int prelu, const void* w, const float* bias, const void* res, void* out, int N, int H, int W,
                   int Hs, int Ws, int Cin, int Cout, int cout_valid, int ks, int ck, int tco, int inmode,
                   int out_f32_nchw, int nw, const float* qscale, const float* qshift, int qshift_ns,
                   hipStream_t stream) {
  if (Cin % ck != 0 || Cout % 4 != 0) return -10;
  if ((qscale || qshift) && out_f32_nchw) return -14;
  if (!(ks == 1 || ks == 3)) return -11;
  ConvArgs a;
  a.x = (const bf16_t*)x; a.x2 = (const bf16_t*)x2; a.pscale = pscale; a.pshift = pshift;
  a.pshift_ns = pshift_ns; a.pscale_ns = pscale_ns; a.prelu = prelu; a.w = (const bf16_t*)w; a.bias = bias;
  a.res = (const bf16_t*)res; a.out = out;
  a.N = N; a.H = H; a.W = W; a.Hs = Hs; a.Ws = Ws; a.Cin = Cin; a.Cout = Cout; a.cout_valid = cout_valid;
  a.nchunk = Cin / ck; a.KP = be_conv2d_packed_kp(ks, ck);
  a.out_f32_nchw = out_f32_nchw;
  a.persist_blocks = g_persist_blocks;
  a.qscale = qscale; a.qshift = qshift; a.qshift_ns = qshift_ns;
  const bool x2p = x2 != nullptr;
  if (ks == 3) {
    if (ck == 8) return dispatch_tco<3, 8>(tco, inmode, x2p, nw, a, stream);
    if (ck == 32) return dispatch_tco<3, 32>(tco, inmode, x2p, nw, a, stream);
  } else {
    if (ck == 8) return dispatch_tco<1, 8>(tco, inmode, x2p, nw, a, stream);
    if (ck == 32) return dispatch_tco<1, 32>(tco, inmode, x2p, nw, a, stream);
    if (ck == 64) return dispatch_tco<1, 64>(tco, inmode, x2p, nw, a, stream);
  }
  return -12;
}

// 3x3x3 / stride 1 / zero-pad 1 conv of x NDHWC bf16 [N][D][H][W][zC] as ONE launch of the 2-D
// LDS-staged kernel over the N * D slices, K = 3 depth taps x zC stacked channels x 9 in-plane taps
// (w: the 2-D packed layout of W'[co][dz * zC + c][ky][kx] = W[co][c][dz][ky][kx]); fp32 accumulation
// over all 27 taps, one bf16 rounding, bias (+ ReLU) in the epilogue.  The halo of every slice tap
// is staged in LDS once per output tile, so the narrow layers of a 3-D U-Net read each input voxel
// ~3x from L2 instead of 27x (the implicit-GEMM gather of be_conv3d_mt).
int be_conv3d_ztaps(const void* x, const void* w, const float* bias, void* out, int N, int D, int H, int W, int zC,
                    int Cout, int ck, int tco, int relu, int nw, hipStream_t stream) {
  if (zC % ck != 0 || Cout % 4 != 0 || (ck != 8 && ck != 16 && ck != 32)) return -10;
  ConvArgs a = {};
  a.x = (const bf16_t*)x; a.w = (const bf16_t*)w; a.bias = bias; a.out = out;
  a.N = N * D; a.H = H; a.W = W; a.Hs = H; a.Ws = W; a.Cin = 3 * zC; a.Cout = Cout; a.cout_valid = Cout;
  a.nchunk = 3 * zC / ck; a.KP = be_conv2d_packed_kp(3, ck);
  a.prelu = relu ? 2 : 0;
  a.persist_blocks = g_persist_blocks;
  a.zD = D; a.zC = zC;
  if (ck == 16) return dispatch_ztaps<16>(tco, nw, a, stream);  // the 16-channel 3-D U-Net layers
  return ck == 8 ? dispatch_ztaps<8>(tco, nw, a, stream) : dispatch_ztaps<32>(tco, nw, a, stream);
}

// be_conv3d_ztaps over the channel concatenation [xa (Ca channels), xb (Cb)] of two NDHWC bf16 volumes
// of one shape (INMODE 5): the 3-D U-Net decoder's torch.cat([skip, up]) is never materialised.
// w: the z-tap stacked packed layout for zC = Ca + Cb input channels.
int be_conv3d_ztaps_concat(const void* xa, const void* xb, const void* w, const float* bias, void* out, int N, int D,
                           int H, int W, int Ca, int Cb, int Cout, int ck, int tco, int relu, int nw, hipStream_t stream) {
  const int zC = Ca + Cb;
  if (Ca % 8 != 0 || Cb % 8 != 0 || zC % ck != 0 || Cout % 4 != 0 || (ck != 8 && ck != 32)) return -10;
  ConvArgs a = {};
  a.x = (const bf16_t*)xa; a.x2 = (const bf16_t*)xb; a.w = (const bf16_t*)w; a.bias = bias; a.out = out;
  a.N = N * D; a.H = H; a.W = W; a.Hs = H; a.Ws = W; a.Cin = 3 * zC; a.Cout = Cout; a.cout_valid = Cout;
  a.nchunk = 3 * zC / ck; a.KP = be_conv2d_packed_kp(3, ck);
  a.prelu = relu ? 2 : 0;
  a.persist_blocks = g_persist_blocks;
  a.zD = D; a.zC = zC; a.zA = Ca;
  return ck == 8 ? dispatch_ztaps<8, 5>(tco, nw, a, stream) : dispatch_ztaps<32, 5>(tco, nw, a, stream);
}

// 3x3 / stride 1 / zero-pad 1 conv of the channel concatenation [xa (Ca channels), xb (Cb)] of two
// NHWC bf16 tensors of one spatial shape, without materialising it: the halo loader picks the source
// per 8-channel group (INMODE 4).  The U-Net decoder's torch.cat([skip, up]) copy (~22 % of the 2-D EM
// line's inference kernel time, profiles/r06/em2d/) disappears.  w: the packed layout of the conv over
// Ca + Cb input channels; bias (+ ReLU) in the epilogue.
// xb_d2s = 1: xb is [N, H/2, W/2, 4 * Cb] with channel (2 dy + dx) * Cb + c = channel c of pixel
// (2y + dy, 2x + dx) -- the 1x1 MFMA conv half of ConvTranspose2d(k=2, s=2), read before its
// depth-to-space shuffle (INMODE 6; H, W even).
int be_conv2d_concat(const void* xa, const void* xb, const void* w, const float* bias, void* out, int N, int H, int W,
                     int Ca, int Cb, int Cout, int ck, int tco, int relu, int nw, int xb_d2s, hipStream_t stream) {
  if (Ca % 8 != 0 || Cb % 8 != 0 || (Ca + Cb) % ck != 0 || Cout % 4 != 0 || (ck != 8 && ck != 32)) return -10;
  if (xb_d2s && ((H | W) & 1)) return -11;
  ConvArgs a = {};
  a.x = (const bf16_t*)xa; a.x2 = (const bf16_t*)xb; a.w = (const bf16_t*)w; a.bias = bias; a.out = out;
  a.N = N; a.H = H; a.W = W; a.Hs = H; a.Ws = W; a.Cin = Ca + Cb; a.Cout = Cout; a.cout_valid = Cout;
  a.nchunk = (Ca + Cb) / ck; a.KP = be_conv2d_packed_kp(3, ck);
  a.prelu = relu ? 2 : 0;
  a.persist_blocks = g_persist_blocks;
  a.zC = Ca;
  if (xb_d2s) return ck == 8 ? dispatch_concat<8, 6>(tco, nw, a, stream) : dispatch_concat<32, 6>(tco, nw, a, stream);
  return ck == 8 ? dispatch_concat<8, 4>(tco, nw, a, stream) : dispatch_concat<32, 4>(tco, nw, a, stream);
}

}  // extern "C"

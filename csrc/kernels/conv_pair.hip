// Fused residual half-block of the Cellpose CPnet: two pre-activation 3x3 convs in ONE kernel, the
// intermediate feature map never leaves LDS.
//
//   h   = relu( (convA( actA(inxform(x)) ) [+ x2]) * sB[c] + tB[n, c] )                tile + 1-px halo, LDS
//   out = convB(h) + bias [+ projP( actP(x) )] [+ res | + up2(res)]                     bf16 NHWC
//   actA(v) = relu(v * sA[c] + tA[n, c]),  actP(v) = v * sP[c] + tP[c]                  (eval BN / style folded)
//
// convA's bias is folded into tB on the host (tB' = tB + sB * biasA) and the projection's bias into
// `bias`, so the kernel never reads them.
//
// One CPnet residual block is two of these: resdown = {proj+c0+c1, c2+c3(+x1)}, resup =
// {c0+c1 (+skip, +up2(proj)), c2+c3(+x1)} (cellpose `resdown`/`resup`, reached by the reference
// through cellpose==3.1.1.2, apps/model-runner/runtime_deployment.py:19).  The
// per-layer kernel (conv2d_nhwc.hip) writes every intermediate to HBM and re-reads it; at the
// 32/64-channel levels (224^2 / 112^2 tiles) those layers are memory bound, so keeping h on chip
// removes most of their HBM traffic (profiles/r02/conv_roofline.md: 11.6 of 18.5 ms were there).
//
// MI355X design:
//  * 512-thread workgroup, one per CU (LDS 113-137 KB), persistent over a CONTIGUOUS range of
//    16x32 output tiles so neighbouring tiles (shared halo rows) run back to back on one CU / L2.
//  * stage A computes h on the 18x34 tile+halo region (612 px = 39 MFMA pixel tiles in linear
//    pixel order, 5 per wave) from a 20x36 input halo staged in LDS with actA applied on the way
//    in; its epilogue applies actB (+ skip add) and writes h as bf16 over the (dead) input halo.
//  * stage B is the 16x32 x CM implicit GEMM over h (tap-major K, chunks of 32 channels); the 1x1
//    projection is one extra K step into the SAME accumulators (K concatenation); then residual +
//    bias and a staged, 16-byte-coalesced NHWC store.
//  * v_mfma_f32_16x16x32_bf16 with the weights as the A operand: each lane ends with 4 consecutive
//    output channels of one pixel (8-byte LDS writes of h, 8-byte residual reads).
//  * CM = 32: every weight panel stays resident in LDS for the whole launch; CM = 64: one weight
//    chunk buffer, the next chunk's weights and the next A chunk's halo are prefetched into
//    registers while the current chunk's MFMAs run ("issue early, write late").
//  * pixel strides are 8 (mod 16) dwords, so ds_read_b128 fragment reads are conflict-free for any
//    tap offset (same rule as conv2d_nhwc.hip).
#include <cstdlib>

#include "common.h"

namespace {

struct PairArgs {
  const bf16_t* x;   // [N, Hs, Ws, Cin]
  const bf16_t* x2;  // [N, H, W, CM] skip added to convA's output (X2)
  const float* sa; const float* ta; int ta_ns;  // actA: scale [Cin], shift [Cin] (ns 0) or [N, ns]
  const float* sb; const float* tb; int tb_ns;  // actB (convA bias folded into tb)
  const float* sp; const float* tp;             // actP (projection), shared
  const bf16_t* wa;                             // [CM][NCA][KPA]
  const bf16_t* wb;                             // [CM][CM/32][288]
  const bf16_t* wp;                             // [CM][1][32]
  const float* bias;                            // [CM] convB bias (+ projection bias)
  const bf16_t* res;                            // [N, H, W, CM] or [N, H/2, W/2, CM] (RES = 2)
  bf16_t* out;                                  // [N, H, W, CM]
  // HEAD (final up half-block only): the network's output conv fused into the epilogue,
  //   y = Wh relu(bf16(out) * sH + tH) + bH  -> fp32 NCHW [N, nh, H, W]; `out` is never written
  const float* sh; const float* th;             // [CM] head pre-activation (eval BN folded)
  const bf16_t* wh;                             // [16][32] bf16, k order permuted to the accumulator layout
  const float* bh;                              // [16] head bias (zero padded)
  float* hout;                                  // [N, nh, H, W]
  int nh;
  int N, H, W, Hs, Ws, Cin;
  int tiles_x, tiles_y;
  // diagnostics (STAMP instantiations only): per-workgroup cycles of wave 0 in each tile phase,
  // [grid][8] = {halo commit, stage-A MFMA, stage-A epilogue, stage-B MFMA, output epilogue, -, -, tiles}
  unsigned long long* stamps;
};

// The one-group kernel and its helpers, once per tile geometry (conv_pair_onegroup.inc).
namespace g32 {
constexpr int TW = 32, TH = 16, NW = 8;
#include "conv_pair_onegroup.inc"
}  // namespace g32
namespace g12 {
constexpr int TW = 16, TH = 12, NW = 4;
#include "conv_pair_onegroup.inc"
}  // namespace g12
using namespace g32;  // the ping-pong kernel and the launchers below use the 16 x 32 geometry

unsigned long long* g_pair_stamps = nullptr;  // diagnostics: be_conv_pair_set_stamps
int g_pair_stamps_cap = 0;                    // workgroups the stamp buffer holds

// A/B of the CM = 64 builds (see conv_pair_kernel's VAR): BE_PAIR_LATE_EPI (default 1) -> bit 0,
// BE_PAIR_ROLL (default 1) -> bit 1, BE_PAIR_EARLY_AFF (default 1) -> bit 2.  LATE: -0.5..-2.2 % cycles
// per tile on the three CM = 64 pairs, +0.4 % headline; ROLL on top: stage A -8..-23 %, tiles
// -2.6..-6.2 %, +0.3 % headline; EARLY on top: halo commit -2..-9 %, tiles -1.1..-2.4 %, +0.4 %
// headline; two alternating runs each (profiles/r04/conv/pair_{late_epi,roll,early_aff}_ab.txt).
static int g_pair_var = [] {
  const char* l = getenv("BE_PAIR_LATE_EPI");
  const char* r = getenv("BE_PAIR_ROLL");
  const char* e = getenv("BE_PAIR_EARLY_AFF");
  const char* p = getenv("BE_PAIR_EPIA");
  const char* q = getenv("BE_PAIR_SEPS");
  const char* te = getenv("BE_PAIR_TOPEPI");
  return ((l ? atoi(l) : 1) ? 1 : 0) | ((r ? atoi(r) : 1) ? 2 : 0) | ((e ? atoi(e) : 1) ? 4 : 0) |
         ((p && atoi(p)) ? 8 : 0) | ((q && atoi(q)) ? 16 : 0) | ((te && atoi(te)) ? 32 : 0);
}();

template <int CK, int CM, int INMODE, bool X2, bool PROJ, int RES, int NCA, bool HEAD, bool STAMP, int VAR>
int launch_pair_l(PairArgs a, int g, hipStream_t s) {
  using C = PC<CK, CM, INMODE, X2, PROJ, RES, NCA>;
  constexpr bool seps = (VAR & 16) != 0 && C::RESW && !HEAD;
  constexpr size_t lds = C::LDS + (seps ? (size_t)C::R_OUT * sizeof(bf16_t) : 0);
  static_assert(lds <= 160 * 1024, "LDS budget (separate output staging)");
  static bool attr_set[BE_MAX_DEV] = {};
  if (!attr_set[be_cur_dev()]) {
    hipFuncSetAttribute(
        reinterpret_cast<const void*>(&conv_pair_kernel<CK, CM, INMODE, X2, PROJ, RES, NCA, HEAD, STAMP, VAR>),
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set[be_cur_dev()] = true;
  }
  hipLaunchKernelGGL((conv_pair_kernel<CK, CM, INMODE, X2, PROJ, RES, NCA, HEAD, STAMP, VAR>), dim3(g), dim3(NT), lds, s,
                     a);
  return BE_CHECK_LAUNCH();
}

template <int CK, int CM, int INMODE, bool X2, bool PROJ, int RES, int NCA, bool HEAD = false, bool STAMP = false>
int launch_pair_k(PairArgs a, int g, hipStream_t s) {
  if constexpr (CM == 32 && CK == 32 && !HEAD) {  // level-0 half-blocks: the SEPS bit applies
    if (g_pair_var & 16) {
      if constexpr (NCA == 1)
        if (g_pair_var & 32) return launch_pair_l<CK, CM, INMODE, X2, PROJ, RES, NCA, HEAD, STAMP, 48>(a, g, s);
      return launch_pair_l<CK, CM, INMODE, X2, PROJ, RES, NCA, HEAD, STAMP, 16>(a, g, s);
    }
  }
  if constexpr (CM == 32 && NCA == 1) {  // the TOPEPI bit (see conv_pair_kernel's LATEEPI)
    if (g_pair_var & 32) return launch_pair_l<CK, CM, INMODE, X2, PROJ, RES, NCA, HEAD, STAMP, 32>(a, g, s);
  }
  if constexpr (CM == 64 && RES != 0) {
    switch (g_pair_var & 15) {
      case 1: return launch_pair_l<CK, CM, INMODE, X2, PROJ, RES, NCA, HEAD, STAMP, 1>(a, g, s);
      case 2: return launch_pair_l<CK, CM, INMODE, X2, PROJ, RES, NCA, HEAD, STAMP, 2>(a, g, s);
      case 3: return launch_pair_l<CK, CM, INMODE, X2, PROJ, RES, NCA, HEAD, STAMP, 3>(a, g, s);
      case 5: return launch_pair_l<CK, CM, INMODE, X2, PROJ, RES, NCA, HEAD, STAMP, 5>(a, g, s);
      case 7: return launch_pair_l<CK, CM, INMODE, X2, PROJ, RES, NCA, HEAD, STAMP, 7>(a, g, s);
      case 15: return launch_pair_l<CK, CM, INMODE, X2, PROJ, RES, NCA, HEAD, STAMP, 15>(a, g, s);
      default: break;
    }
  }
  return launch_pair_l<CK, CM, INMODE, X2, PROJ, RES, NCA, HEAD, STAMP, 0>(a, g, s);
}

template <int CK, int CM, int INMODE, bool X2, bool PROJ, int RES, int NCA, bool HEAD = false>
int launch_pair(PairArgs a, int grid_cap, hipStream_t s) {
  a.tiles_x = (a.W + TW - 1) / TW;
  a.tiles_y = (a.H + TH - 1) / TH;
  const int tiles = a.N * a.tiles_x * a.tiles_y;
  int g = grid_cap > 0 ? grid_cap : 256;  // one 512-thread workgroup per CU
  if (g > tiles) g = tiles;
  if (g < 1) return 0;
  a.stamps = nullptr;
  // phase-stamped build of the level-0/1 half-blocks (tools/pair_phase_profile.py); the buffer must
  // hold [grid][8] words
  if constexpr (!HEAD && !PROJ && CK == 32) {
    if (g_pair_stamps != nullptr) {
      if (g > g_pair_stamps_cap) return -30;
      a.stamps = g_pair_stamps;
      return launch_pair_k<CK, CM, INMODE, X2, PROJ, RES, NCA, HEAD, true>(a, g, s);
    }
  }
  return launch_pair_k<CK, CM, INMODE, X2, PROJ, RES, NCA, HEAD, false>(a, g, s);
}

// =====================================================================================================
// Ping-pong level-0 half-block (CK = CM = 32, NCA = 1, full-resolution input, + x residual): the
// resdown / resup c2 + c3 pairs at 224^2, and the final one with the output head fused (HEAD).
//
// The one-group kernel above runs every phase of a tile on all 8 waves between workgroup barriers,
// so the MFMA pipe idles through the VALU / LDS-store phases (halo activation, the two epilogues):
// ~65 % of a tile (tools/pair_phase_profile.py, profiles/r04/conv/pair_phases.jsonl).  Here the 8
// waves are TWO GROUPS of 4 (waves w and w + 4 share a SIMD) that own alternate tiles of the
// workgroup's range, each in its own LDS region, and run ONE PHASE APART on the same barriers: while
// one group's wave issues MFMAs on a SIMD, the other group's wave on that SIMD runs a VALU phase.
//
//   phases per tile (each ends at a workgroup barrier):
//     P1 commit   input halo registers -> actA -> LDS image               VALU + ds_write
//     P2 stage A  h-region implicit GEMM (10 pixel tiles x 2 ct per wave)  MFMA   (s_setprio 1)
//     P3 epi A    actB -> h (bf16) over the input image                    VALU + ds_write
//     P4 stage B  output implicit GEMM (8 pixel tiles x 2 ct per wave)     MFMA   (s_setprio 1);
//                 issues this tile's residual first
//     P5 epi B    issues the group's next halo; bias + residual -> staged
//                 16-byte stores (or the head)                               VALU + stores
//   group 1 starts one barrier late, so the slots pair (P2,P1) (P3,P2) (P4,P3) (P5,P4) (P1,P5).
//
// LDS: 2 group regions of 45 KiB (the 20 x 36 input image; h and the output staging overlay it) +
// both weight panels (38 KiB) = 128 KiB.  The fp32-accumulated regions hold 64-byte pixels with NO
// padding (the one-group kernel pads to 96 B; two 69 KiB images would not fit) and an XOR swizzle
// of the 16-byte chunk c, chosen by search over the ds_read_b128 lane groups so that every
// 16-pixel fragment read is conflict-free at every tap offset:
//     input image  c ^ 2 * (((x >> 2) ^ y) & 1)   (x, y in the 36-wide halo; edge tiles 2-way)
//     h, staging   c ^ ((x >> 1) & 3)             (ds_write_b64 of the epilogues 2-way)
// Both depend on the lane and on the parity of the tap row only, so every fragment address is a
// per-lane base + a compile-time ds_read offset (no per-read VALU).
#ifndef PP_VAR
#define PP_VAR 1  // tuning variants (tools/build_native.py --variant ... --vflags=-DPP_VAR=n)
#endif
#ifndef PP_GW
#define PP_GW 4  // waves per group (4: one per SIMD, 8: two per SIMD, 128 VGPRs)
#endif
namespace ppk {
constexpr int GW = PP_GW, GT = GW * 64;  // waves / threads per group
constexpr int NTP = 2 * GT;              // threads per workgroup
constexpr int RPW = TH / GW;             // stage-B output rows per wave
constexpr int IN_B = IPIX * 64;         // 46080
constexpr int H_B = RPIX * 64;          // 39168
constexpr int OUTW_B = RPW * TW * 64;   // one wave's RPW x 32 output pixels
constexpr int RB = IN_B;                // one group's region
constexpr int WSTR = 9 * 32 + 16;       // 304: weight row stride (elements; 8 (mod 16) dwords)
constexpr int W_B = 32 * WSTR * 2;      // one conv's panel, bytes
constexpr int APT = 40 / GW, BPT = 32 / GW;  // pixel tiles per wave: stage A (39 in 40 slots), stage B
constexpr int TLAST0 = GW * (APT - 1);        // stage-A tile index of a wave's last slot, minus gw
constexpr int HU = IPIX * 4;            // 16-byte halo units per tile
constexpr int HUPT = (HU + GT - 1) / GT;
static_assert(H_B <= RB && GW * OUTW_B <= RB, "ping-pong region overlays");
static_assert(APT * GW >= RPT && (APT - 1) * GW <= 2 * RH && BPT * GW * 16 == TH * TW, "tile maps");
static_assert(GW == 4 || GW == 8, "group size");
}  // namespace ppk

struct PPHalo {
  u32x4 h[ppk::HUPT];
  float4 aff[4];  // actA scale / shift of this thread's 8 channels ((gt & 3) * 8 ..)
};

__device__ __forceinline__ int pp_in_off(int pi, int c) {  // byte offset of chunk c of input-image pixel pi
  const int y = pi / IW, x = pi - y * IW;
  return pi * 64 + ((c ^ ((((x >> 2) ^ y) & 1) << 1)) << 4);
}

template <int INMODE, int CIN, bool INT = false>
__device__ __forceinline__ void pp_issue_halo(const PairArgs& a, TileXY t, int ch, int gt, PPHalo& hr) {
  const int c = ch * 32 + (gt & 3) * 8;  // a thread's chunk is the same for every unit (GT % 4 == 0)
  hr.aff[0] = *reinterpret_cast<const float4*>(a.sa + c);
  hr.aff[1] = *reinterpret_cast<const float4*>(a.sa + c + 4);
  const float* tr = a.ta + (size_t)t.n * a.ta_ns + c;
  hr.aff[2] = *reinterpret_cast<const float4*>(tr);
  hr.aff[3] = *reinterpret_cast<const float4*>(tr + 4);
#pragma unroll
  for (int i = 0; i < ppk::HUPT; ++i) {  // clamped, unconditional (exact vmcnt counts; see issue_halo)
    const int pi = min(gt + i * ppk::GT, ppk::HU - 1) >> 2;
    const int y = pi / IW, x = pi - y * IW;
    const int gy = INT ? t.ty0 - 2 + y : min(max(t.ty0 - 2 + y, 0), a.H - 1);
    const int gx = INT ? t.tx0 - 2 + x : min(max(t.tx0 - 2 + x, 0), a.W - 1);
    if constexpr (INMODE == 0)
      hr.h[i] = *reinterpret_cast<const u32x4*>(a.x + (((size_t)t.n * a.Hs + gy) * a.Ws + gx) * CIN + c);
    else  // nearest 2x upsampling of the half-resolution input
      hr.h[i] = *reinterpret_cast<const u32x4*>(a.x + (((size_t)t.n * a.Hs + (gy >> 1)) * a.Ws + (gx >> 1)) * CIN + c);
  }
}

// INT: the tile's whole 20 x 36 halo lies inside the image (most tiles): no bounds tests
__device__ __forceinline__ bool pp_interior(const PairArgs& a, TileXY t) {
  return t.ty0 >= 2 && t.ty0 + TH + 2 <= a.H && t.tx0 >= 2 && t.tx0 + TW + 2 <= a.W;
}

template <bool INT>
__device__ __forceinline__ void pp_commit(const PairArgs& a, TileXY t, int gt, const PPHalo& hr, unsigned char* rin) {
  float sc[8], sh[8];
  unpack_aff(hr.aff, sc, sh);
  const int c = gt & 3;
#pragma unroll
  for (int i = 0; i < ppk::HUPT; ++i) {
    const int u = gt + i * ppk::GT;
    if (u >= ppk::HU) continue;
    const int pi = u >> 2;
    const int y = pi / IW, x = pi - y * IW;
    const int gy = t.ty0 - 2 + y, gx = t.tx0 - 2 + x;
    u32x4 pk = (u32x4){0u, 0u, 0u, 0u};
    if (INT || (gy >= 0 && gy < a.H && gx >= 0 && gx < a.W)) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        pk[j] = relu_bf16x2(pack2bf(fmaf(lo_bf(hr.h[i][j]), sc[2 * j], sh[2 * j]),
                                    fmaf(hi_bf(hr.h[i][j]), sc[2 * j + 1], sh[2 * j + 1])));
    }
    *reinterpret_cast<u32x4*>(rin + pi * 64 + ((c ^ ((((x >> 2) ^ y) & 1) << 1)) << 4)) = pk;
  }
}

// stage A: wave gw's row tiles j = 0..8 are region row (gw >> 1) + 2j, columns (gw & 1) * 16 + lrow;
// j = 9 is edge / padding tile gw + 36 (columns 32, 33 of rows 8 gw ..)
__device__ __forceinline__ void pp_mma_a(f32x4 (&acc)[2][ppk::APT], const unsigned char* rin, const bf16_t* wa, int gw,
                                         int lrow, int kq) {
  const int par = (gw >> 1) & 1;
  const int b0 = ((gw >> 1) * IW + (gw & 1) * 16 + lrow) * 64;
  int A0[3][2];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx)
#pragma unroll
    for (int pr = 0; pr < 2; ++pr)
      A0[dx][pr] = b0 + dx * 64 + ((kq ^ (((((lrow + dx) >> 2) ^ par ^ pr) & 1) << 1)) << 4);
  // the wave's last slot: a row tile (8-wave groups, gw < 4) or an edge / padding tile
  int L[3][2];
  const int tl = gw + ppk::TLAST0;  // wave-uniform
  if (tl < 2 * RH) {
    const int ryl = tl >> 1, rxl = (tl & 1) * 16 + lrow;
#pragma unroll
    for (int dx = 0; dx < 3; ++dx)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
        L[dx][pr] = (ryl * IW + rxl + dx) * 64 + ((kq ^ (((((lrow + dx) >> 2) ^ ryl ^ pr) & 1) << 1)) << 4);
  } else {
    int ry9 = (tl - 2 * RH) * 8 + (lrow >> 1), rx9 = 32 + (lrow & 1);
    if (ry9 >= RH) { ry9 = 0; rx9 = 0; }  // padding lanes: valid data, never stored
#pragma unroll
    for (int dx = 0; dx < 3; ++dx)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
        L[dx][pr] = (ry9 * IW + rx9 + dx) * 64 + ((kq ^ ((((ry9 & 1) ^ pr) & 1) << 1)) << 4);
  }
  auto frags = [&](int ks, bf16x8 (&af)[2], bf16x8 (&bf)[ppk::APT]) {
    const int dy = ks / 3, dx = ks % 3;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
      af[ct] = *reinterpret_cast<const bf16x8*>(wa + (ct * 16 + lrow) * ppk::WSTR + ks * 32 + kq * 8);
#pragma unroll
    for (int j = 0; j < ppk::APT - 1; ++j)
      bf[j] = *reinterpret_cast<const bf16x8*>(rin + A0[dx][dy & 1] + j * (ppk::GW / 2) * IW * 64 + dy * IW * 64);
    bf[ppk::APT - 1] = *reinterpret_cast<const bf16x8*>(rin + L[dx][dy & 1] + dy * IW * 64);
  };
  // one pixel-fragment set, rolling reload: each pixel fragment of K-step ks + 1 is read right after
  // its last MFMA of step ks (80 accumulator VGPRs leave no room for a second set); the two weight
  // fragments of ks + 1 are read at the top of step ks into a second pair (read after the last
  // pixel tile they would be waited on two MFMAs later)
  bf16x8 af[2], afn[2], bf[ppk::APT];
  frags(0, af, bf);
#pragma unroll
  for (int ks = 0; ks < 9; ++ks) {
    const bool more = ks + 1 < 9;
    const int kn = more ? ks + 1 : ks, dy = kn / 3, dx = kn % 3;
#pragma unroll
    for (int j = 0; j < ppk::APT; ++j) {
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        acc[ct][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ct], bf[j], acc[ct][j], 0, 0, 0);
        if (j == 0 && more)
          afn[ct] = *reinterpret_cast<const bf16x8*>(wa + (ct * 16 + lrow) * ppk::WSTR + kn * 32 + kq * 8);
      }
      if (more) {
        if (j < ppk::APT - 1)
          bf[j] = *reinterpret_cast<const bf16x8*>(rin + A0[dx][dy & 1] + j * (ppk::GW / 2) * IW * 64 + dy * IW * 64);
        else
          bf[j] = *reinterpret_cast<const bf16x8*>(rin + L[dx][dy & 1] + dy * IW * 64);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (more) {
      af[0] = afn[0];
      af[1] = afn[1];
    }
  }
}

// X2: the skip operand of stage A's output (resup: convA(x) + skip) at this lane's h pixels
struct PPSkip {
  u32x2 xv[ppk::APT][2];
};

// the h pixel (ry, rx) of a wave's last stage-A slot: a row tile (8-wave groups, gw < 4) or an
// edge / padding tile; false for padding lanes
__device__ __forceinline__ bool pp_last(int gw, int lrow, int& ry, int& rx) {
  const int tl = gw + ppk::TLAST0;
  if (tl < 2 * RH) {
    ry = tl >> 1;
    rx = (tl & 1) * 16 + lrow;
    return true;
  }
  ry = (tl - 2 * RH) * 8 + (lrow >> 1);
  rx = 32 + (lrow & 1);
  return ry < RH;
}

__device__ __forceinline__ void pp_issue_skip(const PairArgs& a, TileXY t, int gw, int lrow, int kq, PPSkip& sk) {
#pragma unroll
  for (int j = 0; j < ppk::APT; ++j) {
    int ry, rx;
    if (j < ppk::APT - 1) {
      ry = (gw >> 1) + (ppk::GW / 2) * j;
      rx = (gw & 1) * 16 + lrow;
    } else {
      pp_last(gw, lrow, ry, rx);
    }
    // clamped, unconditional: pp_epi_a stores zero outside the image and nothing for padding lanes
    const int gy = min(max(t.ty0 - 1 + ry, 0), a.H - 1), gx = min(max(t.tx0 - 1 + rx, 0), a.W - 1);
    const bf16_t* xp = a.x2 + (((size_t)t.n * a.H + gy) * a.W + gx) * 32 + kq * 4;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) sk.xv[j][ct] = *reinterpret_cast<const u32x2*>(xp + ct * 16);
  }
}

// actB(+ skip) -> h (bf16) in the region, zero outside the image; h pixel (ry, rx) of the 18 x 34 region
template <bool X2, bool INT>
__device__ __forceinline__ void pp_epi_a(const PairArgs& a, TileXY t, const f32x4 (&acc)[2][ppk::APT],
                                         unsigned char* rh, const float4 (&s)[2], const float4 (&sh)[2],
                                         const PPSkip& sk, int gw, int lrow, int kq) {
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    const int hc = ((2 * ct) | (kq >> 1));
    const int hw = (((gw >> 1) * RW + (gw & 1) * 16 + lrow) * 64) + ((hc ^ ((lrow >> 1) & 3)) << 4) + (kq & 1) * 8;
#pragma unroll
    for (int j = 0; j < ppk::APT; ++j) {
      int ry, rx, off;
      if (j < ppk::APT - 1) {
        ry = (gw >> 1) + (ppk::GW / 2) * j;
        rx = (gw & 1) * 16 + lrow;
        off = hw + j * (ppk::GW / 2) * RW * 64;
      } else {
        if (!pp_last(gw, lrow, ry, rx)) continue;
        off = (ry * RW + rx) * 64 + ((hc ^ ((rx >> 1) & 3)) << 4) + (kq & 1) * 8;
      }
      const int gy = t.ty0 - 1 + ry, gx = t.tx0 - 1 + rx;
      float v0 = acc[ct][j][0], v1 = acc[ct][j][1], v2 = acc[ct][j][2], v3 = acc[ct][j][3];
      if constexpr (X2) {
        u32x2 xv = sk.xv[j][ct];
        asm volatile("" : "+v"(xv));  // unpacked here, not next to its load (see pp_epi_b)
        v0 += lo_bf(xv[0]); v1 += hi_bf(xv[0]); v2 += lo_bf(xv[1]); v3 += hi_bf(xv[1]);
      }
      u32x2 st = (u32x2){0u, 0u};
      if (INT || (gy >= 0 && gy < a.H && gx >= 0 && gx < a.W)) {
        st[0] = relu_bf16x2(pack2bf(fmaf(v0, s[ct].x, sh[ct].x), fmaf(v1, s[ct].y, sh[ct].y)));
        st[1] = relu_bf16x2(pack2bf(fmaf(v2, s[ct].z, sh[ct].z), fmaf(v3, s[ct].w, sh[ct].w)));
      }
      *reinterpret_cast<u32x2*>(rh + off) = st;
    }
  }
}

// stage B: wave gw owns output rows RPW gw .. RPW gw + RPW - 1; pixel tile pt = row (pt >> 1), half (pt & 1)
__device__ __forceinline__ void pp_mma_b(f32x4 (&acc)[2][ppk::BPT], const unsigned char* rh, const bf16_t* wb, int gw,
                                         int lrow, int kq) {
  int B0[3];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) B0[dx] = ((ppk::RPW * gw) * RW + lrow + dx) * 64 + ((kq ^ (((lrow + dx) >> 1) & 3)) << 4);
  auto frags = [&](int ks, bf16x8 (&af)[2], bf16x8 (&bf)[ppk::BPT]) {
    const int dy = ks / 3, dx = ks % 3;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
      af[ct] = *reinterpret_cast<const bf16x8*>(wb + (ct * 16 + lrow) * ppk::WSTR + ks * 32 + kq * 8);
#pragma unroll
    for (int pt = 0; pt < ppk::BPT; ++pt)
      bf[pt] = *reinterpret_cast<const bf16x8*>(rh + B0[dx] + ((pt >> 1) + dy) * RW * 64 + (pt & 1) * 16 * 64);
  };
  bf16x8 af[2], afn[2], bf[ppk::BPT];  // rolling reload, weight pair read a step ahead (as pp_mma_a)
  frags(0, af, bf);
#pragma unroll
  for (int ks = 0; ks < 9; ++ks) {
    const bool more = ks + 1 < 9;
    const int kn = more ? ks + 1 : ks, dy = kn / 3, dx = kn % 3;
#pragma unroll
    for (int pt = 0; pt < ppk::BPT; ++pt) {
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        acc[ct][pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ct], bf[pt], acc[ct][pt], 0, 0, 0);
        if (pt == 0 && more)
          afn[ct] = *reinterpret_cast<const bf16x8*>(wb + (ct * 16 + lrow) * ppk::WSTR + kn * 32 + kq * 8);
      }
      if (more) bf[pt] = *reinterpret_cast<const bf16x8*>(rh + B0[dx] + ((pt >> 1) + dy) * RW * 64 + (pt & 1) * 16 * 64);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (more) {
      af[0] = afn[0];
      af[1] = afn[1];
    }
  }
}

struct PPRes {
  u32x2 rv[ppk::BPT][2];
  float4 bias[2];
};

template <int RES>
__device__ __forceinline__ void pp_issue_res(const PairArgs& a, TileXY t, int gw, int lrow, int kq, PPRes& r) {
#pragma unroll
  for (int pt = 0; pt < ppk::BPT; ++pt) {
    if constexpr (RES == 0) {  // the stem: its residual is the in-kernel projection
      r.rv[pt][0] = r.rv[pt][1] = (u32x2){0u, 0u};
      continue;
    }
    const int py = min(t.ty0 + ppk::RPW * gw + (pt >> 1), a.H - 1), px = min(t.tx0 + (pt & 1) * 16 + lrow, a.W - 1);
    const bf16_t* rp = RES == 1 ? a.res + (((size_t)t.n * a.H + py) * a.W + px) * 32 + kq * 4
                                : a.res + (((size_t)t.n * (a.H >> 1) + (py >> 1)) * (a.W >> 1) + (px >> 1)) * 32 + kq * 4;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) r.rv[pt][ct] = *reinterpret_cast<const u32x2*>(rp + ct * 16);
  }
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) r.bias[ct] = *reinterpret_cast<const float4*>(a.bias + ct * 16 + kq * 4);
}

// bias + residual -> wave-private staging (swizzled like h) -> 16-byte coalesced NHWC stores
template <int RES>
__device__ __forceinline__ void pp_epi_b(const PairArgs& a, TileXY t, const f32x4 (&acc)[2][ppk::BPT], const PPRes& r,
                                         unsigned char* ws, int gw, int lrow, int kq, bool act) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      a.out + (size_t)t.n * a.H * a.W * 32, (short)0, a.H * a.W * 64, 0x00020000);
  if constexpr (PP_VAR & 16) {
    // direct: 8-byte buffer stores from the accumulator layout (lane = 4 channels of one pixel; a
    // 16-lane row covers 16 pixels x 8 B, the four kq rows and the two ct halves fill each pixel's
    // 64 B in L2), no LDS staging round trip; 16 stores (PP_NST)
#pragma unroll
    for (int pt = 0; pt < ppk::BPT; ++pt) {
      const int py = t.ty0 + ppk::RPW * gw + (pt >> 1), px = t.tx0 + (pt & 1) * 16 + lrow;
      const bool ok = act && py < a.H && px < a.W;
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        u32x2 rv = r.rv[pt][ct];
        asm volatile("" : "+v"(rv));
        u32x2 st;
        st[0] = pack2bf(acc[ct][pt][0] + r.bias[ct].x + lo_bf(rv[0]), acc[ct][pt][1] + r.bias[ct].y + hi_bf(rv[0]));
        st[1] = pack2bf(acc[ct][pt][2] + r.bias[ct].z + lo_bf(rv[1]), acc[ct][pt][3] + r.bias[ct].w + hi_bf(rv[1]));
        const int off = ok ? ((py * a.W + px) * 32 + ct * 16 + kq * 4) * 2 : 0x7ffffff0;
        __builtin_amdgcn_raw_buffer_store_b64(st, rs, off, 0, 0);
      }
    }
    return;
  }
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    const int ow = lrow * 64 + ((((2 * ct) | (kq >> 1)) ^ ((lrow >> 1) & 3)) << 4) + (kq & 1) * 8;
#pragma unroll
    for (int pt = 0; pt < ppk::BPT; ++pt) {
      u32x2 rv = r.rv[pt][ct];
      if constexpr (RES != 0) asm volatile("" : "+v"(rv));  // keeps the bf16 unpacking here, not hoisted next to the loads in P4
      u32x2 st;
      st[0] = pack2bf(acc[ct][pt][0] + r.bias[ct].x + lo_bf(rv[0]), acc[ct][pt][1] + r.bias[ct].y + hi_bf(rv[0]));
      st[1] = pack2bf(acc[ct][pt][2] + r.bias[ct].z + lo_bf(rv[1]), acc[ct][pt][3] + r.bias[ct].w + hi_bf(rv[1]));
      *reinterpret_cast<u32x2*>(ws + ow + ((pt >> 1) * 32 + (pt & 1) * 16) * 64) = st;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int lane = lrow + 16 * kq;
  const int rd = (lane >> 2) * 64 + (((lane & 3) ^ ((lane >> 3) & 3)) << 4);
  // Buffer stores through a per-image descriptor: a pixel outside the image (or a tile that is not
  // this group's) gets an out-of-range offset and the range check drops it, so exactly PP_EPI_STORES
  // stores are issued on every path and the next P1's halo wait can be a counted vmcnt.  One unit in
  // flight at a time (the next halo's registers are live through this phase).
  const int py0 = t.ty0 + ppk::RPW * gw, px0 = t.tx0 + (lane >> 2);
#pragma unroll
  for (int it = 0; it < 2 * ppk::RPW; ++it) {
    const int py = py0 + (it >> 1), px = px0 + (it & 1) * 16;
    const u32x4 v = *reinterpret_cast<const u32x4*>(ws + rd + it * 1024);
    const int off = (act && py < a.H && px < a.W) ? ((py * a.W + px) * 32 + (lane & 3) * 8) * 2 : 0x7ffffff0;
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// HEAD: out = bf16(acc + bias + res), then the output layer (see epi_head) straight from registers
__device__ __forceinline__ void pp_epi_head(const PairArgs& a, TileXY t, const f32x4 (&acc)[2][ppk::BPT], const PPRes& r,
                                            const HeadRegs& hr, int gw, int lrow, int kq, bool act) {
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      a.hout + (size_t)t.n * a.nh * a.H * a.W, (short)0, a.nh * a.H * a.W * 4, 0x00020000);
#pragma unroll
  for (int pt = 0; pt < ppk::BPT; ++pt) {
    u32x4 bw;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      u32x2 rv = r.rv[pt][ct];
      asm volatile("" : "+v"(rv));  // see pp_epi_b
      const float4 bias = r.bias[ct];
      const uint32_t o0 = pack2bf(acc[ct][pt][0] + bias.x + lo_bf(rv[0]), acc[ct][pt][1] + bias.y + hi_bf(rv[0]));
      const uint32_t o1 = pack2bf(acc[ct][pt][2] + bias.z + lo_bf(rv[1]), acc[ct][pt][3] + bias.w + hi_bf(rv[1]));
      bw[2 * ct] = relu_bf16x2(pack2bf(fmaf(lo_bf(o0), hr.s[ct].x, hr.t[ct].x), fmaf(hi_bf(o0), hr.s[ct].y, hr.t[ct].y)));
      bw[2 * ct + 1] = relu_bf16x2(pack2bf(fmaf(lo_bf(o1), hr.s[ct].z, hr.t[ct].z), fmaf(hi_bf(o1), hr.s[ct].w, hr.t[ct].w)));
    }
    const f32x4 y = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hr.w, *reinterpret_cast<const bf16x8*>(&bw), zero, 0, 0, 0);
    const int py = t.ty0 + ppk::RPW * gw + (pt >> 1), px = t.tx0 + (pt & 1) * 16 + lrow;
    const bool ok = act && py < a.H && px < a.W;
    const float bb[4] = {hr.b.x, hr.b.y, hr.b.z, hr.b.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // unconditional buffer stores, out-of-range offsets dropped (see pp_epi_b)
      const int co = kq * 4 + i;
      const int off = (ok && co < a.nh) ? ((co * a.H + py) * a.W + px) * 4 : 0x7ffffff0;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(y[i] + bb[i]), rs, off, 0, 0);
    }
  }
}

// ---- stem (Cin = 8 + the 1x1 projection) on the ping-pong kernel -------------------------------
// In: the 20 x 36 halo of actA(x) at 8 channels per pixel, padded to 24 elements (48 B: sixteen
// consecutive pixels hit 16 distinct 16-byte slots); P: actP(x) at the 16 x 32 centre pixels,
// unpadded 16-byte pixels (a fragment read is 256 contiguous bytes), read by stage B's projection K
// step; h and the output staging as the 32-channel path.  Total 122 KiB: the same ~32 KiB of a CU's
// LDS stays free for the mask-stage kernels that run beside the network (the first build padded P
// to 48 B, took 154 KiB and slowed the pipelined headline although the stem call itself was faster).
namespace pps {
constexpr int PST = 24;                      // In pixel stride (elements)
constexpr int PSP = 8;                       // P pixel stride (elements)
constexpr int KPA = 96, WSTRA = KPA + 16;    // stage-A K: 9 taps x 8 channels, 4 taps per 32-deep step
constexpr int WSTRP = 48;                    // projection weight row stride
constexpr int IN_B = IPIX * PST * 2;         // 34560
constexpr int P_B = TH * TW * PSP * 2;       // 8192
constexpr int R_B = ppk::H_B > IN_B ? ppk::H_B : IN_B;  // In / h / output staging overlay
constexpr int RB = R_B + P_B;                // one group's region
constexpr int WA_B = 32 * WSTRA * 2, WB_B = 32 * ppk::WSTR * 2, WP_B = 32 * WSTRP * 2;
constexpr int LDS = 2 * RB + WA_B + WB_B + WP_B;
constexpr int HUPT = (IPIX + ppk::GT - 1) / ppk::GT;  // one 16-byte unit (8 channels) per pixel
static_assert(LDS <= 128 * 1024 && ppk::GW * ppk::OUTW_B <= R_B, "stem ping-pong LDS budget");
}  // namespace pps

struct PPHalo8 {
  u32x4 h[pps::HUPT];
  float4 aff[4], paff[4];
};

template <bool INT = false>
__device__ __forceinline__ void pp8_issue_halo(const PairArgs& a, TileXY t, int gt, PPHalo8& hr) {
  hr.aff[0] = *reinterpret_cast<const float4*>(a.sa);
  hr.aff[1] = *reinterpret_cast<const float4*>(a.sa + 4);
  const float* tr = a.ta + (size_t)t.n * a.ta_ns;
  hr.aff[2] = *reinterpret_cast<const float4*>(tr);
  hr.aff[3] = *reinterpret_cast<const float4*>(tr + 4);
  hr.paff[0] = *reinterpret_cast<const float4*>(a.sp);
  hr.paff[1] = *reinterpret_cast<const float4*>(a.sp + 4);
  hr.paff[2] = *reinterpret_cast<const float4*>(a.tp);
  hr.paff[3] = *reinterpret_cast<const float4*>(a.tp + 4);
#pragma unroll
  for (int i = 0; i < pps::HUPT; ++i) {  // clamped, unconditional (exact vmcnt counts)
    const int pi = min(gt + i * ppk::GT, IPIX - 1);
    const int y = pi / IW, x = pi - y * IW;
    const int gy = INT ? t.ty0 - 2 + y : min(max(t.ty0 - 2 + y, 0), a.H - 1);
    const int gx = INT ? t.tx0 - 2 + x : min(max(t.tx0 - 2 + x, 0), a.W - 1);
    hr.h[i] = *reinterpret_cast<const u32x4*>(a.x + (((size_t)t.n * a.Hs + gy) * a.Ws + gx) * 8);
  }
}

template <bool INT>
__device__ __forceinline__ void pp8_commit(const PairArgs& a, TileXY t, int gt, const PPHalo8& hr, unsigned char* rin,
                                           unsigned char* preg) {
  float sc[8], sh[8], ps[8], pt[8];
  unpack_aff(hr.aff, sc, sh);
  unpack_aff(hr.paff, ps, pt);
#pragma unroll
  for (int i = 0; i < pps::HUPT; ++i) {
    const int pi = gt + i * ppk::GT;
    if (pi >= IPIX) continue;
    const int iy = pi / IW, ix = pi - iy * IW;
    const int gy = t.ty0 - 2 + iy, gx = t.tx0 - 2 + ix;
    const bool in = INT || (gy >= 0 && gy < a.H && gx >= 0 && gx < a.W);
    float v[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[2 * j] = lo_bf(hr.h[i][j]); v[2 * j + 1] = hi_bf(hr.h[i][j]); }
    u32x4 pk = (u32x4){0u, 0u, 0u, 0u};
    if (in) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        pk[j] = relu_bf16x2(pack2bf(fmaf(v[2 * j], sc[2 * j], sh[2 * j]), fmaf(v[2 * j + 1], sc[2 * j + 1], sh[2 * j + 1])));
    }
    *reinterpret_cast<u32x4*>(rin + pi * pps::PST * 2) = pk;
    if (iy >= 2 && iy < TH + 2 && ix >= 2 && ix < TW + 2) {
      u32x4 pp = (u32x4){0u, 0u, 0u, 0u};
      if (in) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          pp[j] = pack2bf(fmaf(v[2 * j], ps[2 * j], pt[2 * j]), fmaf(v[2 * j + 1], ps[2 * j + 1], pt[2 * j + 1]));
      }
      *reinterpret_cast<u32x4*>(preg + ((iy - 2) * TW + (ix - 2)) * pps::PSP * 2) = pp;
    }
  }
}

// stage A of the stem: 3 K steps of 4 taps x 8 channels (lane kq: tap 4 ks + kq; taps >= 9 have zero
// weights and read the tap-0 pixel)
__device__ __forceinline__ void pp8_mma_a(f32x4 (&acc)[2][ppk::APT], const unsigned char* rin, const bf16_t* wa, int gw,
                                          int lrow, int kq) {
  int toff[3];
#pragma unroll
  for (int ks = 0; ks < 3; ++ks) {
    int tap = ks * 4 + kq;
    if (tap >= 9) tap = 0;
    toff[ks] = ((tap / 3) * IW + tap % 3) * pps::PST * 2;
  }
  const int b0 = ((gw >> 1) * IW + (gw & 1) * 16 + lrow) * pps::PST * 2;
  int ryl, rxl;
  if (!pp_last(gw, lrow, ryl, rxl)) { ryl = 0; rxl = 0; }
  const int bl = (ryl * IW + rxl) * pps::PST * 2;
#pragma unroll
  for (int ks = 0; ks < 3; ++ks) {
    bf16x8 af[2], bf[ppk::APT];
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
      af[ct] = *reinterpret_cast<const bf16x8*>(wa + (ct * 16 + lrow) * pps::WSTRA + ks * 32 + kq * 8);
#pragma unroll
    for (int j = 0; j < ppk::APT - 1; ++j)
      bf[j] = *reinterpret_cast<const bf16x8*>(rin + b0 + toff[ks] + j * (ppk::GW / 2) * IW * pps::PST * 2);
    bf[ppk::APT - 1] = *reinterpret_cast<const bf16x8*>(rin + bl + toff[ks]);
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int j = 0; j < ppk::APT; ++j)
        acc[ct][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ct], bf[j], acc[ct][j], 0, 0, 0);
  }
}

// the stem's 1x1 projection as one more K step into stage B's accumulators (k >= 8: zero weights)
__device__ __forceinline__ void pp8_mma_p(f32x4 (&acc)[2][ppk::BPT], const unsigned char* preg, const bf16_t* wp, int gw,
                                          int lrow, int kq) {
  bf16x8 af[2], bf[ppk::BPT];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) af[ct] = *reinterpret_cast<const bf16x8*>(wp + (ct * 16 + lrow) * pps::WSTRP + kq * 8);
#pragma unroll
  for (int pt = 0; pt < ppk::BPT; ++pt) {
    const int oy = ppk::RPW * gw + (pt >> 1), ox = (pt & 1) * 16 + lrow;
    bf[pt] = *reinterpret_cast<const bf16x8*>(preg + (oy * TW + ox) * pps::PSP * 2);
  }
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int pt = 0; pt < ppk::BPT; ++pt)
      acc[ct][pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ct], bf[pt], acc[ct][pt], 0, 0, 0);
}

template <bool STEM> struct PPHaloOf { using T = PPHalo; };
template <> struct PPHaloOf<true> { using T = PPHalo8; };

// NCA input chunks of 32 channels (Cin = 32 NCA), INMODE 0 (full resolution) or 1 (nearest 2x up),
// X2: + skip operand on stage A's output, RES 1 (full) or 2 (up2 of a half-resolution map).
// STEM: Cin = 8 with the 1x1 projection as the residual (NCA 1, INMODE 0, RES 0; regions pps::).
template <int NCA, int INMODE, bool X2, int RES, bool HEAD, bool STEM = false, bool STAMP = false>
__global__ __launch_bounds__(ppk::NTP, ppk::GW == 4 ? 2 : 4) void conv_pair_pp_kernel(PairArgs a) {
  static_assert(!STEM || (NCA == 1 && INMODE == 0 && !X2 && RES == 0 && !HEAD), "stem configuration");
  constexpr int CIN = 32 * NCA;
  constexpr int RB = STEM ? pps::RB : ppk::RB;
  // STAMP (diagnostics, tools/pp_phase_profile.py): wave 0 of each group accumulates s_memtime
  // cycles of every phase's own work and of its wait at the closing barrier, [grid][2 groups][16]
  unsigned long long ph_work[7] = {0, 0, 0, 0, 0, 0, 0}, ph_wait[7] = {0, 0, 0, 0, 0, 0, 0};
  unsigned long long tstamp = STAMP ? __builtin_amdgcn_s_memtime() : 0;
  auto pre = [&](int i) {
    if constexpr (STAMP) {
      const unsigned long long tn = __builtin_amdgcn_s_memtime();
      ph_work[i] += tn - tstamp;
      tstamp = tn;
    }
  };
  auto post = [&](int i) {
    if constexpr (STAMP) {
      const unsigned long long tn = __builtin_amdgcn_s_memtime();
      ph_wait[i] += tn - tstamp;
      tstamp = tn;
    }
  };
  // buffer stores per P5 (counted wait in P1)
  constexpr int NST = HEAD ? 4 * ppk::BPT : ((PP_VAR & 16) ? 2 * ppk::BPT : 2 * ppk::RPW);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid0 = threadIdx.x;
  const int total = a.N * a.tiles_x * a.tiles_y;
  const int t0 = (int)(((long long)blockIdx.x * total) / gridDim.x);
  const int t1 = (int)(((long long)(blockIdx.x + 1) * total) / gridDim.x);
  if (t0 >= t1) return;  // workgroup-uniform
  bf16_t* wl = reinterpret_cast<bf16_t*>(smem + 2 * RB);
  const bf16_t* wb = wl + (STEM ? 32 * pps::WSTRA : NCA * 32 * ppk::WSTR);
  const bf16_t* wp = wb + 32 * ppk::WSTR;  // STEM: the projection panel [32][48]
  if constexpr (STEM) {  // [32][96] stage A, [32][288] stage B, [32][32] projection
    for (int u = tid0; u < 32 * (12 + 36 + 4); u += ppk::NTP) {
      const int r = u / 52, q = u % 52;
      const bf16_t* src;
      bf16_t* dst;
      if (q < 12) { src = a.wa + (size_t)r * 96 + q * 8; dst = wl + r * pps::WSTRA + q * 8; }
      else if (q < 48) { src = a.wb + (size_t)r * 288 + (q - 12) * 8; dst = const_cast<bf16_t*>(wb) + r * ppk::WSTR + (q - 12) * 8; }
      else { src = a.wp + (size_t)r * 32 + (q - 48) * 8; dst = const_cast<bf16_t*>(wp) + r * pps::WSTRP + (q - 48) * 8; }
      *reinterpret_cast<u32x4*>(dst) = *reinterpret_cast<const u32x4*>(src);
    }
  } else {
    // NCA stage-A panels then the stage-B panel, [32 rows][304] each (from the packed [Cout][NCA][288]
    // and [Cout][1][288] layouts)
    for (int u = tid0; u < (NCA + 1) * 32 * 36; u += ppk::NTP) {
      const int pnl = u / (32 * 36), q = u % (32 * 36), r = q / 36, k8 = q % 36;
      const bf16_t* src = pnl < NCA ? a.wa + ((size_t)r * NCA + pnl) * 288 + k8 * 8 : a.wb + (size_t)r * 288 + k8 * 8;
      *reinterpret_cast<u32x4*>(wl + pnl * 32 * ppk::WSTR + r * ppk::WSTR + k8 * 8) = *reinterpret_cast<const u32x4*>(src);
    }
  }
  // wave-uniform values in SGPRs (readfirstlane): the group / wave-in-group branches stay scalar
  const int grp = __builtin_amdgcn_readfirstlane(tid0 / ppk::GT);  // waves 0..GW-1 | GW..2GW-1 (w, w + GW share a SIMD)
  const int gt0 = tid0 & (ppk::GT - 1);
  unsigned char* reg = smem + grp * RB;
  HeadRegs hr;
  if constexpr (HEAD) load_head(a, tid0 & 15, (tid0 & 63) >> 4, hr);
  typename PPHaloOf<STEM>::T halo;
  // chunk 0 of a tile's input halo -> registers
  auto issue0 = [&](TileXY nx, int gtv) {
    if constexpr (STEM) {
      if (pp_interior(a, nx)) pp8_issue_halo<true>(a, nx, gtv, halo);
      else pp8_issue_halo<false>(a, nx, gtv, halo);
    } else {
      if (pp_interior(a, nx)) pp_issue_halo<INMODE, CIN, true>(a, nx, 0, gtv, halo);
      else pp_issue_halo<INMODE, CIN>(a, nx, 0, gtv, halo);
    }
  };
  if constexpr (STEM) pp8_issue_halo<false>(a, tile_xy(a, min(t0 + grp, t1 - 1)), gt0, halo);
  else pp_issue_halo<INMODE, CIN>(a, tile_xy(a, min(t0 + grp, t1 - 1)), 0, gt0, halo);
  __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xf << 8));  // vmcnt(0): see the counted wait in P1
  __syncthreads();  // weights resident
  if (grp == 1) __builtin_amdgcn_s_barrier();  // the stagger: group 1 runs one phase behind
  const int iters = (t1 - t0 + 1) >> 1;
  for (int k = 0; k < iters; ++k) {
    int gt = gt0;
    asm volatile("" : "+v"(gt));  // per-iteration opaque copy (see conv_pair_kernel)
    const int gw = __builtin_amdgcn_readfirstlane(gt >> 6), lane = gt & 63, lrow = lane & 15, kq = lane >> 4;
    const int t = t0 + 2 * k + grp;
    // A group without a tile in the last iteration (odd range) recomputes the range's last tile and
    // stores nothing: every phase runs unconditionally (no divergent-looking branches around the
    // big register sets, which the allocator handled badly), only the global stores are predicated.
    const bool act = t < t1;
    const TileXY cur = tile_xy(a, act ? t : t1 - 1);
    const bool inner = pp_interior(a, cur);  // tile-uniform: bounds-free commit / epilogue A
    f32x4 acc_a[2][ppk::APT];
    float4 sb[2], tb[2];
    PPSkip sk;
#pragma unroll
    for (int c = 0; c < NCA; ++c) {
      // P1: input chunk c -> activated image.  For c = 0 in flight: the halo (issued in P4), then
      // exactly the previous P5's NST buffer stores; the counted wait retires the halo only (the
      // builtin, so the compiler's own wait tracking sees it and adds no vmcnt(0) behind the stores).
      constexpr int NW = (PP_VAR & 2) ? 0 : NST;
      if (c == 0) __builtin_amdgcn_s_waitcnt((NW & 0xf) | (0x7 << 4) | (0xf << 8) | ((NW >> 4) << 14));
      int gc = gt0;
      asm volatile("" : "+v"(gc));  // per chunk: the unit addresses are recomputed, not kept across P2
      if constexpr (STEM) {
        if (inner) pp8_commit<true>(a, cur, gc, halo, reg, reg + pps::R_B);
        else pp8_commit<false>(a, cur, gc, halo, reg, reg + pps::R_B);
      } else {
        if (inner) pp_commit<true>(a, cur, gc, halo, reg);
        else pp_commit<false>(a, cur, gc, halo, reg);
      }
      pre(2 * c);
      __syncthreads();
      post(2 * c);
      // P2: stage A over chunk c (the next chunk's halo, or the epilogue operands, in flight)
      if constexpr (!STEM) {
        if (c + 1 < NCA) {
          if (inner) pp_issue_halo<INMODE, CIN, true>(a, cur, c + 1, gt, halo);
          else pp_issue_halo<INMODE, CIN>(a, cur, c + 1, gt, halo);
        }
      }
      if (c == NCA - 1) {
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          sb[ct] = *reinterpret_cast<const float4*>(a.sb + ct * 16 + kq * 4);
          tb[ct] = *reinterpret_cast<const float4*>(a.tb + (size_t)cur.n * a.tb_ns + ct * 16 + kq * 4);
        }
        if constexpr (X2) pp_issue_skip(a, cur, gw, lrow, kq, sk);
      }
      if (c == 0) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < ppk::APT; ++j) acc_a[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      }
      if constexpr (!(PP_VAR & 4)) __builtin_amdgcn_s_setprio(1);
      if constexpr (STEM) pp8_mma_a(acc_a, reg, wl, gw, lrow, kq);
      else pp_mma_a(acc_a, reg, wl + c * 32 * ppk::WSTR, gw, lrow, kq);
      if constexpr (!(PP_VAR & 4)) __builtin_amdgcn_s_setprio(0);
      pre(2 * c + 1);
      __syncthreads();
      post(2 * c + 1);
    }
    // P3: epilogue A -> h
    int g3 = gt0;
    asm volatile("" : "+v"(g3));
    if (inner) pp_epi_a<X2, true>(a, cur, acc_a, reg, sb, tb, sk, gw, g3 & 15, (g3 & 63) >> 4);
    else pp_epi_a<X2, false>(a, cur, acc_a, reg, sb, tb, sk, gw, g3 & 15, (g3 & 63) >> 4);
    PPRes res;
    if constexpr (PP_VAR & 1) pp_issue_res<RES>(a, cur, gw, g3 & 15, (g3 & 63) >> 4, res);
    if constexpr (PP_VAR & 8) issue0(tile_xy(a, min(t + 2, t1 - 1)), g3);  // two slots ahead of its commit
    pre(2 * NCA);
    __syncthreads();
    post(2 * NCA);
    // P4: stage B; this tile's residual first, the group's next halo behind the MFMAs (its registers
    // are free once the fragments are; it is needed two phases later).  Fresh opaque lane index:
    // the P4 / P5 addresses are computed here, not hoisted into P1 and kept (spilled) across.
    int g4 = gt0;
    asm volatile("" : "+v"(g4));
    const int lrow4 = g4 & 15, kq4 = (g4 & 63) >> 4;
    f32x4 acc_b[2][ppk::BPT];
    if constexpr (!(PP_VAR & 1)) pp_issue_res<RES>(a, cur, gw, lrow4, kq4, res);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < ppk::BPT; ++j) acc_b[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if constexpr (!(PP_VAR & 4)) __builtin_amdgcn_s_setprio(1);
    pp_mma_b(acc_b, reg, wb, gw, lrow4, kq4);
    if constexpr (STEM) pp8_mma_p(acc_b, reg + pps::R_B, wp, gw, lrow4, kq4);
    if constexpr (!(PP_VAR & 4)) __builtin_amdgcn_s_setprio(0);
    pre(2 * NCA + 1);
    __syncthreads();
    post(2 * NCA + 1);
    // P5: the group's next halo (issued here, not behind the stage-B MFMAs: the issue of 16 wide
    // loads stalled the MFMA phase, the longest slot; it is needed at the next phase), then the
    // output epilogue (its staging overlays h: every wave of the group is past stage B)
    int g5 = gt0;
    asm volatile("" : "+v"(g5));
    const int lrow5 = g5 & 15, kq5 = (g5 & 63) >> 4;
    auto next_halo = [&]() { issue0(tile_xy(a, min(t + 2, t1 - 1)), g5); };
    if constexpr (!(PP_VAR & 10)) next_halo();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (HEAD) pp_epi_head(a, cur, acc_b, res, hr, gw, lrow5, kq5, act);
    else pp_epi_b<RES>(a, cur, acc_b, res, reg + gw * ppk::OUTW_B, gw, lrow5, kq5, act);
    if constexpr (PP_VAR & 2) next_halo();
    pre(2 * NCA + 2);
    __syncthreads();
    post(2 * NCA + 2);
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();  // balance the stagger
  if constexpr (STAMP) {
    if ((tid0 & (ppk::GT - 1)) < 16) {  // wave 0 of each group: lane k stores slot k (lane-indexed vector store)
      const int k = tid0 & 15;
      unsigned long long v = 0;
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        if (k == i) v = ph_work[i];
        if (k == 8 + i) v = ph_wait[i];
      }
      if (k == 15) v = (unsigned long long)iters;
      a.stamps[((size_t)blockIdx.x * 2 + grp) * 16 + k] = v;
    }
  }
}

unsigned long long* g_pp_stamps = nullptr;  // diagnostics: be_conv_pair_pp_set_stamps
int g_pp_stamps_cap = 0;

template <int NCA, int INMODE, bool X2, int RES, bool HEAD, bool STEM = false>
int launch_pair_pp(PairArgs a, int grid_cap, hipStream_t s) {
  constexpr int lds = STEM ? pps::LDS : 2 * ppk::RB + (NCA + 1) * ppk::W_B;
  static_assert(lds <= 160 * 1024, "ping-pong LDS budget");
  a.tiles_x = (a.W + TW - 1) / TW;
  a.tiles_y = (a.H + TH - 1) / TH;
  const int tiles = a.N * a.tiles_x * a.tiles_y;
  int g = grid_cap > 0 ? grid_cap : 256;
  if (g > tiles) g = tiles;
  if (g < 1) return 0;
  a.stamps = nullptr;
  static bool attr_set[BE_MAX_DEV] = {};
  if (!attr_set[be_cur_dev()]) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_pair_pp_kernel<NCA, INMODE, X2, RES, HEAD, STEM>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr_set[be_cur_dev()] = true;
  }
  if (g_pp_stamps != nullptr) {
    if (g > g_pp_stamps_cap) return -30;
    a.stamps = g_pp_stamps;
    static bool attr_st[BE_MAX_DEV] = {};
    if (!attr_st[be_cur_dev()]) {
      hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_pair_pp_kernel<NCA, INMODE, X2, RES, HEAD, STEM, true>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      attr_st[be_cur_dev()] = true;
    }
    hipLaunchKernelGGL((conv_pair_pp_kernel<NCA, INMODE, X2, RES, HEAD, STEM, true>), dim3(g), dim3(ppk::NTP), lds, s, a);
    return BE_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL((conv_pair_pp_kernel<NCA, INMODE, X2, RES, HEAD, STEM>), dim3(g), dim3(ppk::NTP), lds, s, a);
  return BE_CHECK_LAUNCH();
}
}  // namespace

// tuning override (0 = one workgroup per CU); BE_PAIR_GRID sets it for A/B runs
static int g_pair_grid = [] {
  const char* e = getenv("BE_PAIR_GRID");
  return e ? atoi(e) : 0;
}();

// BE_PAIR_PP (default 1): the level-0 32 -> 32 half-blocks (+ the head) on the ping-pong kernel
static int g_pair_pp = [] {
  const char* e = getenv("BE_PAIR_PP");
  return e ? atoi(e) : 1;
}();

// BE_PAIR_G12 (A/B): the level-1 (CM = 64) half-blocks on the 12 x 16-tile geometry -- 4 waves and
// <= 79 KB of LDS per workgroup, so two workgroups share each CU and one's halo / epilogue phases run
// beside the other's MFMAs (the one-group 16 x 32 kernel leaves the MFMA pipe idle through them:
// profiles/r04/conv/pair_phases.jsonl).  BE_PAIR_G12_GRID: workgroups (default 512).
static int g_pair_g12 = [] {
  const char* e = getenv("BE_PAIR_G12");
  return e ? atoi(e) : 0;
}();
static int g_pair_g12_grid = [] {
  const char* e = getenv("BE_PAIR_G12_GRID");
  return e ? atoi(e) : 512;
}();

template <int CK, int CM, int INMODE, bool X2, int RES, int NCA>
int launch_pair12(PairArgs a, hipStream_t s) {
  using C = g12::PC<CK, CM, INMODE, X2, false, RES, NCA>;
  constexpr size_t lds = C::LDS;
  static_assert(2 * lds <= 160 * 1024, "two workgroups per CU");
  a.tiles_x = (a.W + g12::TW - 1) / g12::TW;
  a.tiles_y = (a.H + g12::TH - 1) / g12::TH;
  const int tiles = a.N * a.tiles_x * a.tiles_y;
  int g = g_pair_g12_grid > 0 ? g_pair_g12_grid : 512;
  if (g > tiles) g = tiles;
  if (g < 1) return 0;
  a.stamps = nullptr;
  constexpr auto kern = &g12::conv_pair_kernel<CK, CM, INMODE, X2, false, RES, NCA, false, false, 7>;
  static bool attr_set[BE_MAX_DEV] = {};
  if (!attr_set[be_cur_dev()]) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set[be_cur_dev()] = true;
  }
  hipLaunchKernelGGL(kern, dim3(g), dim3(g12::NT), lds, s, a);
  return BE_CHECK_LAUNCH();
}

// BE_PAIR_PP_STEM (default 1): the stem (8 -> 32 + projection) on the ping-pong kernel as well
static int g_pair_pp_stem = [] {
  const char* e = getenv("BE_PAIR_PP_STEM");
  return e ? atoi(e) : 1;
}();

// The ping-pong kernel pays off when each workgroup has tiles for both groups: with fewer than two
// tiles per workgroup (batch-1 latency calls) the second group would only recompute a dummy tile,
// so those calls keep the one-group kernel.
static bool pp_ok(const PairArgs& a, int grid_cap) {
  if (!g_pair_pp || g_pair_stamps != nullptr) return false;
  const long long tiles = (long long)a.N * ((a.W + TW - 1) / TW) * ((a.H + TH - 1) / TH);
  const int g = grid_cap > 0 ? grid_cap : 256;
  return tiles >= 2LL * g;
}

extern "C" {

int be_conv_pair_set_grid(int blocks) {
  g_pair_grid = blocks;
  return 0;
}

// Diagnostics: route the level-0/1 half-blocks (not the stem / head) to the phase-stamped build,
// which writes [workgroup][8] cycle counts into `buf` (device, >= cap_workgroups * 64 bytes);
// nullptr switches back.  Not for production launches (the stamps cost ~1 % of the kernel).
int be_conv_pair_set_stamps(void* buf, int cap_workgroups) {
  g_pair_stamps = static_cast<unsigned long long*>(buf);
  g_pair_stamps_cap = buf ? cap_workgroups : 0;
  return 0;
}

// Diagnostics: the ping-pong half-blocks write [workgroup][group][16] u64 phase stamps into `buf`
// (work cycles of phase i at slot i, barrier-wait cycles at 8 + i, iterations at 15); nullptr
// switches back.  Not for production launches.
int be_conv_pair_pp_set_stamps(void* buf, int cap_workgroups) {
  g_pp_stamps = static_cast<unsigned long long*>(buf);
  g_pp_stamps_cap = buf ? cap_workgroups : 0;
  return 0;
}

// LDS bytes of one configuration (tests / tooling); -1 = unsupported configuration.
int be_conv_pair_lds(int cin, int cm, int inmode, int x2, int proj, int res) {
  (void)inmode; (void)x2; (void)res;
  if (cm == 32 && cin == 8 && proj) return (int)PC<8, 32, 0, false, true, 0, 1>::LDS;
  if (cm == 32 && cin == 32) return (int)PC<32, 32, 0, false, false, 1, 1>::LDS;
  if (cm == 32 && cin == 64) return (int)PC<32, 32, 1, true, false, 2, 2>::LDS;
  if (cm == 64) return (int)PC<32, 64, 0, false, false, 1, 2>::LDS;
  return -1;
}

// Supported (cin, cm, inmode, x2, proj, res) configurations = the CPnet levels 0/1 half-blocks:
//   (8,32,none,0,1,0)  stem: proj + c0 + c1          (32,32,none,0,0,full) c2 + c3 + x1 (down and up)
//   (32,64,pool2,0,0,full) level-1 c0 + c1 + proj    (64,64,none,0,0,full) level-1 c2 + c3 + x1
//   (128,64,up2,1,0,up2)  up level-1 c0 + c1 + skip + up2(proj)
//   (64,32,up2,1,0,up2)   up level-0 c0 + c1 + skip + up2(proj)
int be_conv_pair(const void* x, const void* x2, const float* sa, const float* ta, int ta_ns, const float* sb,
                 const float* tb, int tb_ns, const float* sp, const float* tp, const void* wa, const void* wb,
                 const void* wp, const float* bias, const void* res, void* out, int N, int H, int W, int Hs, int Ws,
                 int Cin, int CM, int inmode, int proj, int resmode, hipStream_t stream) {
  PairArgs a;
  a.x = (const bf16_t*)x; a.x2 = (const bf16_t*)x2;
  a.sa = sa; a.ta = ta; a.ta_ns = ta_ns; a.sb = sb; a.tb = tb; a.tb_ns = tb_ns; a.sp = sp; a.tp = tp;
  a.wa = (const bf16_t*)wa; a.wb = (const bf16_t*)wb; a.wp = (const bf16_t*)wp; a.bias = bias;
  a.res = (const bf16_t*)res; a.out = (bf16_t*)out;
  a.N = N; a.H = H; a.W = W; a.Hs = Hs; a.Ws = Ws; a.Cin = Cin;
  a.sh = a.th = a.bh = nullptr; a.wh = nullptr; a.hout = nullptr; a.nh = 0;
  const bool hx2 = x2 != nullptr;
  if (!sa || !ta || !sb || !tb || !wa || !wb || !bias || !out || !x) return -20;
  if ((resmode != 0) != (res != nullptr)) return -21;
  if (proj && (!sp || !tp || !wp)) return -22;
  const int g = g_pair_grid;
  if (CM == 32 && Cin == 8 && inmode == 0 && !hx2 && proj && resmode == 0) {
    if (g_pair_pp_stem && pp_ok(a, g) && Hs == H && Ws == W)
      return launch_pair_pp<1, 0, false, 0, false, true>(a, g, stream);
    return launch_pair<8, 32, 0, false, true, 0, 1>(a, g, stream);
  }
  if (CM == 32 && Cin == 32 && inmode == 0 && !hx2 && !proj && resmode == 1) {
    if (pp_ok(a, g) && Hs == H && Ws == W) return launch_pair_pp<1, 0, false, 1, false>(a, g, stream);
    return launch_pair<32, 32, 0, false, false, 1, 1>(a, g, stream);
  }
  if (CM == 32 && Cin == 64 && inmode == 1 && hx2 && !proj && resmode == 2) {
    if (pp_ok(a, g) && 2 * Hs == H && 2 * Ws == W)
      return launch_pair_pp<2, 1, true, 2, false>(a, g, stream);
    return launch_pair<32, 32, 1, true, false, 2, 2>(a, g, stream);
  }
  if (CM == 64 && Cin == 32 && inmode == 2 && !hx2 && !proj && resmode == 1)
    return g_pair_g12 ? launch_pair12<32, 64, 2, false, 1, 1>(a, stream) : launch_pair<32, 64, 2, false, false, 1, 1>(a, g, stream);
  if (CM == 64 && Cin == 64 && inmode == 0 && !hx2 && !proj && resmode == 1)
    return g_pair_g12 ? launch_pair12<32, 64, 0, false, 1, 2>(a, stream) : launch_pair<32, 64, 0, false, false, 1, 2>(a, g, stream);
  if (CM == 64 && Cin == 128 && inmode == 1 && hx2 && !proj && resmode == 2)
    return g_pair_g12 ? launch_pair12<32, 64, 1, true, 2, 4>(a, stream) : launch_pair<32, 64, 1, true, false, 2, 4>(a, g, stream);
  return -23;
}

// The final up half-block (32 -> 32 channels, + x1) with the network's output layer fused into its
// epilogue (see epi_head): writes hout fp32 NCHW [N, nh, H, W] (nh <= 16), never `out`.
int be_conv_pair_head(const void* x, const float* sa, const float* ta, int ta_ns, const float* sb, const float* tb,
                      int tb_ns, const void* wa, const void* wb, const float* bias, const void* res, const float* sh,
                      const float* th, const void* wh, const float* bh, float* hout, int nh, int N, int H, int W,
                      hipStream_t stream) {
  if (!x || !sa || !ta || !sb || !tb || !wa || !wb || !bias || !res || !sh || !th || !wh || !bh || !hout) return -20;
  if (nh < 1 || nh > 16) return -24;
  PairArgs a;
  a.x = (const bf16_t*)x; a.x2 = nullptr;
  a.sa = sa; a.ta = ta; a.ta_ns = ta_ns; a.sb = sb; a.tb = tb; a.tb_ns = tb_ns; a.sp = nullptr; a.tp = nullptr;
  a.wa = (const bf16_t*)wa; a.wb = (const bf16_t*)wb; a.wp = nullptr; a.bias = bias;
  a.res = (const bf16_t*)res; a.out = nullptr;
  a.sh = sh; a.th = th; a.wh = (const bf16_t*)wh; a.bh = bh; a.hout = hout; a.nh = nh;
  a.N = N; a.H = H; a.W = W; a.Hs = H; a.Ws = W; a.Cin = 32;
  if (pp_ok(a, g_pair_grid)) return launch_pair_pp<1, 0, false, 1, true>(a, g_pair_grid, stream);
  return launch_pair<32, 32, 0, false, false, 1, 1, true>(a, g_pair_grid, stream);
}

}  // extern "C"

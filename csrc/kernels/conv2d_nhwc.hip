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
//  * one workgroup = 4 waves = an 8x32 output pixel tile x TCO output channels; the input halo
//    ((8+KS-1) x (32+KS-1) x CK channels) is staged through LDS once per Cin chunk with the
//    pre-activation (BN affine, style shift, skip add, ReLU, pool/upsample) applied in registers
//    on the way in, so the activated tensor never exists in HBM.
//  * K ordering inside a chunk is tap-major / channel-minor (k = tap*CK + c), so a 16-byte
//    B fragment is 8 contiguous channels of one shifted pixel; small-Cin layers (Cin=8) pack 4
//    taps into one 32-deep MFMA step instead of padding channels to 32.
//  * pixel stride in LDS is padded by 16 B to break the power-of-two bank pattern of ds_read_b128.
#include "common.h"

namespace {

constexpr int TH = 8;    // output tile rows
constexpr int TW = 32;   // output tile cols
constexpr int NT = 256;  // threads / block (4 waves)

struct ConvArgs {
  const bf16_t* x;       // [N, Hs, Ws, Cin]
  const bf16_t* x2;      // optional [N, H, W, Cin] added before the affine
  const float* pscale;   // optional [Cin]
  const float* pshift;   // optional [N?, Cin]  (row stride pshift_ns: 0 => shared over batch)
  const bf16_t* w;       // packed [Cout_pad][nchunk][KP]
  const float* bias;     // optional [Cout]
  const bf16_t* res;     // optional residual [N, H, W, Cout]
  void* out;             // bf16 NHWC [N,H,W,Cout] or f32 NCHW [N,cout_valid,H,W]
  int N, H, W, Hs, Ws, Cin, Cout, cout_valid;
  int nchunk, KP;
  int pshift_ns;
  int prelu;
  int out_f32_nchw;
  int tiles_x, tiles_y;
};

template <int KS, int CK, int TCO, int INMODE>
__global__ __launch_bounds__(NT, 2) void conv2d_nhwc_kernel(ConvArgs a) {
  constexpr int HH = TH + KS - 1;
  constexpr int HW_ = TW + KS - 1;
  constexpr int PSTR = CK + 8;                    // elements per pixel in LDS (16 B pad)
  constexpr int KSTEPS = (KS * KS * CK + 31) / 32;
  constexpr int KPL = KSTEPS * 32;
  constexpr int WSTR = KPL + 8;                   // elements per cout row in LDS
  constexpr int CG = CK / 8;                      // 8-channel groups per pixel
  constexpr int NCT = TCO / 16;

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* hl = reinterpret_cast<bf16_t*>(smem);
  bf16_t* wl = hl + HH * HW_ * PSTR;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;

  int bid = blockIdx.x;
  const int tiles_per_img = a.tiles_x * a.tiles_y;
  const int n = bid / tiles_per_img;
  const int t = bid % tiles_per_img;
  const int ty0 = (t / a.tiles_x) * TH;
  const int tx0 = (t % a.tiles_x) * TW;
  const int co0 = blockIdx.y * TCO;

  f32x4 acc[NCT][4];
#pragma unroll
  for (int i = 0; i < NCT; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const float* shift_row = a.pshift ? a.pshift + (size_t)n * a.pshift_ns : nullptr;

  for (int ch = 0; ch < a.nchunk; ++ch) {
    const int c0 = ch * CK;
    // ---- stage activated input halo into LDS ----
    for (int u = tid; u < HH * HW_ * CG; u += NT) {
      const int pix = u / CG, cg = u % CG;
      const int hy = pix / HW_, hx = pix % HW_;
      const int gy = ty0 + hy - KS / 2, gx = tx0 + hx - KS / 2;
      u32x4 packed = (u32x4){0u, 0u, 0u, 0u};
      if (gy >= 0 && gy < a.H && gx >= 0 && gx < a.W) {
        const int c = c0 + cg * 8;
        float v[8];
        if (INMODE == 0) {
          const u32x4 r = *reinterpret_cast<const u32x4*>(a.x + (((size_t)n * a.Hs + gy) * a.Ws + gx) * a.Cin + c);
#pragma unroll
          for (int j = 0; j < 4; ++j) { v[2 * j] = lo_bf(r[j]); v[2 * j + 1] = hi_bf(r[j]); }
        } else if (INMODE == 1) {  // nearest upsample x2: source is half resolution
          const u32x4 r = *reinterpret_cast<const u32x4*>(a.x + (((size_t)n * a.Hs + (gy >> 1)) * a.Ws + (gx >> 1)) * a.Cin + c);
#pragma unroll
          for (int j = 0; j < 4; ++j) { v[2 * j] = lo_bf(r[j]); v[2 * j + 1] = hi_bf(r[j]); }
        } else {  // maxpool 2x2: source is double resolution
          const bf16_t* base = a.x + (((size_t)n * a.Hs + 2 * gy) * a.Ws + 2 * gx) * a.Cin + c;
          const u32x4 r0 = *reinterpret_cast<const u32x4*>(base);
          const u32x4 r1 = *reinterpret_cast<const u32x4*>(base + a.Cin);
          const u32x4 r2 = *reinterpret_cast<const u32x4*>(base + (size_t)a.Ws * a.Cin);
          const u32x4 r3 = *reinterpret_cast<const u32x4*>(base + (size_t)a.Ws * a.Cin + a.Cin);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[2 * j] = fmaxf(fmaxf(lo_bf(r0[j]), lo_bf(r1[j])), fmaxf(lo_bf(r2[j]), lo_bf(r3[j])));
            v[2 * j + 1] = fmaxf(fmaxf(hi_bf(r0[j]), hi_bf(r1[j])), fmaxf(hi_bf(r2[j]), hi_bf(r3[j])));
          }
        }
        if (a.x2) {
          const u32x4 r = *reinterpret_cast<const u32x4*>(a.x2 + (((size_t)n * a.H + gy) * a.W + gx) * a.Cin + c);
#pragma unroll
          for (int j = 0; j < 4; ++j) { v[2 * j] += lo_bf(r[j]); v[2 * j + 1] += hi_bf(r[j]); }
        }
        if (a.pscale) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = v[j] * a.pscale[c + j] + (shift_row ? shift_row[c + j] : 0.f);
        } else if (shift_row) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] += shift_row[c + j];
        }
        if (a.prelu) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) packed[j] = pack2bf(v[2 * j], v[2 * j + 1]);
      }
      *reinterpret_cast<u32x4*>(hl + pix * PSTR + cg * 8) = packed;
    }
    // ---- stage packed weights for this chunk ----
    {
      constexpr int WU = TCO * KPL / 8;
      for (int u = tid; u < WU; u += NT) {
        const int r = u / (KPL / 8), k8 = u % (KPL / 8);
        const u32x4 wv = *reinterpret_cast<const u32x4*>(a.w + ((size_t)(co0 + r) * a.nchunk + ch) * a.KP + k8 * 8);
        *reinterpret_cast<u32x4*>(wl + r * WSTR + k8 * 8) = wv;
      }
    }
    __syncthreads();

    // ---- MFMA main loop over the chunk's K ----
    const int lrow = lane & 15;
    const int kq = lane >> 4;
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      const int g = ks * 4 + kq;
      int tap = g / CG;
      const int cg = g % CG;
      if (tap >= KS * KS) tap = 0;  // zero-weight K padding: read any finite data
      const int dy = tap / KS, dx = tap % KS;
      bf16x8 af[NCT];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
        af[ct] = *reinterpret_cast<const bf16x8*>(wl + (ct * 16 + lrow) * WSTR + ks * 32 + kq * 8);
      bf16x8 bfr[4];
#pragma unroll
      for (int pt = 0; pt < 4; ++pt) {
        const int py = 2 * wave + (pt >> 1);
        const int px = (pt & 1) * 16 + lrow;
        bfr[pt] = *reinterpret_cast<const bf16x8*>(hl + ((py + dy) * HW_ + (px + dx)) * PSTR + cg * 8);
      }
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
        for (int pt = 0; pt < 4; ++pt)
          acc[ct][pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ct], bfr[pt], acc[ct][pt], 0, 0, 0);
    }
    __syncthreads();
  }

  // ---- epilogue: bias, residual, store ----
  const int lrow = lane & 15;
  const int kq = lane >> 4;
#pragma unroll
  for (int pt = 0; pt < 4; ++pt) {
    const int py = ty0 + 2 * wave + (pt >> 1);
    const int px = tx0 + (pt & 1) * 16 + lrow;
    if (py >= a.H || px >= a.W) continue;
    const size_t pix = ((size_t)n * a.H + py) * a.W + px;
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      const int co = co0 + ct * 16 + kq * 4;
      float v0 = acc[ct][pt][0], v1 = acc[ct][pt][1], v2 = acc[ct][pt][2], v3 = acc[ct][pt][3];
      if (a.out_f32_nchw) {
        float* o = reinterpret_cast<float*>(a.out);
        const float vv[4] = {v0, v1, v2, v3};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = co + i;
          if (c < a.cout_valid) {
            float r = vv[i] + (a.bias ? a.bias[c] : 0.f);
            o[(((size_t)n * a.cout_valid + c) * a.H + py) * a.W + px] = r;
          }
        }
      } else {
        if (co >= a.Cout) continue;
        if (a.bias) { v0 += a.bias[co]; v1 += a.bias[co + 1]; v2 += a.bias[co + 2]; v3 += a.bias[co + 3]; }
        if (a.res) {
          const u32x2 r = *reinterpret_cast<const u32x2*>(a.res + pix * a.Cout + co);
          v0 += lo_bf(r[0]); v1 += hi_bf(r[0]); v2 += lo_bf(r[1]); v3 += hi_bf(r[1]);
        }
        u32x2 st;
        st[0] = pack2bf(v0, v1);
        st[1] = pack2bf(v2, v3);
        *reinterpret_cast<u32x2*>(reinterpret_cast<bf16_t*>(a.out) + pix * a.Cout + co) = st;
      }
    }
  }
}

template <int KS, int CK, int TCO, int INMODE>
int launch(const ConvArgs& a, hipStream_t s) {
  constexpr int HH = TH + KS - 1, HW_ = TW + KS - 1, PSTR = CK + 8;
  constexpr int KSTEPS = (KS * KS * CK + 31) / 32, WSTR = KSTEPS * 32 + 8;
  const size_t lds = (size_t)(HH * HW_ * PSTR + TCO * WSTR) * sizeof(bf16_t);
  dim3 grid(a.N * a.tiles_x * a.tiles_y, (a.Cout + TCO - 1) / TCO);
  hipLaunchKernelGGL((conv2d_nhwc_kernel<KS, CK, TCO, INMODE>), grid, dim3(NT), lds, s, a);
  return BE_CHECK_LAUNCH();
}

template <int KS, int CK, int TCO>
int dispatch_inmode(int inmode, const ConvArgs& a, hipStream_t s) {
  switch (inmode) {
    case 0: return launch<KS, CK, TCO, 0>(a, s);
    case 1: return launch<KS, CK, TCO, 1>(a, s);
    case 2: return launch<KS, CK, TCO, 2>(a, s);
  }
  return -1;
}

template <int KS, int CK>
int dispatch_tco(int tco, int inmode, const ConvArgs& a, hipStream_t s) {
  switch (tco) {
    case 16: return dispatch_inmode<KS, CK, 16>(inmode, a, s);
    case 32: return dispatch_inmode<KS, CK, 32>(inmode, a, s);
    case 64: return dispatch_inmode<KS, CK, 64>(inmode, a, s);
  }
  return -2;
}

}  // namespace

extern "C" {

// Returns the K chunk length (padded) the packed weight layout must use for (ks, ck).
int be_conv2d_packed_kp(int ks, int ck) { return ((ks * ks * ck + 31) / 32) * 32; }

int be_conv2d_nhwc(const void* x, const void* x2, const float* pscale, const float* pshift, int pshift_ns,
                   int prelu, const void* w, const float* bias, const void* res, void* out, int N, int H, int W,
                   int Hs, int Ws, int Cin, int Cout, int cout_valid, int ks, int ck, int tco, int inmode,
                   int out_f32_nchw, hipStream_t stream) {
  if (Cin % ck != 0 || Cout % 4 != 0) return -10;
  if (!(ks == 1 || ks == 3)) return -11;
  ConvArgs a;
  a.x = (const bf16_t*)x; a.x2 = (const bf16_t*)x2; a.pscale = pscale; a.pshift = pshift;
  a.pshift_ns = pshift_ns; a.prelu = prelu; a.w = (const bf16_t*)w; a.bias = bias;
  a.res = (const bf16_t*)res; a.out = out;
  a.N = N; a.H = H; a.W = W; a.Hs = Hs; a.Ws = Ws; a.Cin = Cin; a.Cout = Cout; a.cout_valid = cout_valid;
  a.nchunk = Cin / ck; a.KP = be_conv2d_packed_kp(ks, ck);
  a.out_f32_nchw = out_f32_nchw;
  a.tiles_x = (W + TW - 1) / TW; a.tiles_y = (H + TH - 1) / TH;
  if (ks == 3) {
    if (ck == 8) return dispatch_tco<3, 8>(tco, inmode, a, stream);
    if (ck == 32) return dispatch_tco<3, 32>(tco, inmode, a, stream);
  } else {
    if (ck == 8) return dispatch_tco<1, 8>(tco, inmode, a, stream);
    if (ck == 32) return dispatch_tco<1, 32>(tco, inmode, a, stream);
  }
  return -12;
}

}  // extern "C"

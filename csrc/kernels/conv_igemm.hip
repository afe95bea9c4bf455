// 3x3 conv as an implicit GEMM over LINEAR pixel tiles, for the deep layers of the Cellpose CPnet
// (3x3, Cin = Cout = 128 / 256 at 56^2 / 28^2, and the 64-channel layers at 112^2).
//
//   out  = conv3x3(x) + bias [+ res]                      (bf16 NHWC, optional)
//   aout = relu?( out * as[c] + at[n, c] )                (bf16 NHWC, optional: the NEXT conv's
//                                                           pre-activation, applied by the producer)
//
// The input x is already activated (BN affine + ReLU (+ style shift, + skip add) of this conv were
// applied by the producer's epilogue), so the kernel is a pure GEMM: M = pixels, N = Cout,
// K = 9 taps x Cin, and both operands go HBM/L2 -> LDS by LDS-DMA (global_load_lds_dwordx4) with no
// VGPR staging and no VALU work on the way in.  The reference reaches these layers through
// cellpose==3.1.1.2's nn.Sequential(BatchNorm2d, ReLU, Conv2d) (apps/model-runner/
// runtime_deployment.py:19).
//
// MI355X design (cdna_hip_programming.md §5, T1, T2; MI355X_MICROARCH.md §LDS):
//  * Tile = BM CONSECUTIVE output pixels in (n, y, x) order x BN output channels, so no pixel of the
//    grid is wasted on a ragged 28x28 / 56x56 image edge (a 2-D 8x32 tile wastes 30 % at 28x28).
//    The tile's input halo is a contiguous range of "padded rows" R = n (H+2) + y + 1 (rows y = -1
//    and y = H of every image are the zero rows), each W+2 pixels wide, so image boundaries inside a
//    tile need no special case: a pixel's 3x3 taps never leave its own image's padded rows.
//  * Waves = WM (pixels) x WN (channels); each wave owns 64 pixels x 64 channels = 2 x 2 tiles of
//    v_mfma_f32_32x32x16_bf16 (64 fp32 accumulators/lane).  Weights are the A operand (rows = Cout),
//    pixels the B operand, so a lane ends with 4 consecutive output channels of one pixel.  The
//    default block is 256 pixels x 64 channels on 4 waves with ~65-75 KB of LDS, so two blocks share
//    a CU and one's barrier wait and epilogue stores overlap the other's MFMAs (one 8-wave block per
//    CU measured no faster than the per-layer kernel: profiles/r04/conv/igemm_v1.jsonl).
//  * K chunk = 16 input channels (one 32x32x16 K-step per tap, 9 per chunk).  Two LDS stage buffers:
//    chunk c+1's DMA is issued right after the barrier that publishes chunk c, and lands under
//    chunk c's 36 MFMAs per wave.  One barrier per chunk.
//  * Halo image: 32 bytes per pixel (two 16-byte channel halves, swapped on every other group of 8
//    pixels, hslot()): every fragment read is conflict-free at every tap shift.  The per-(tap,
//    fragment) LDS addresses are computed once per tile (18 VGPRs).  The DMA writes slots
//    lane-linearly, so the swizzle lives in the per-lane SOURCE address; out-of-image pixels read
//    the zero page (conv zero padding).
//  * Weights are pre-packed on the host in exactly the LDS image order ([tap][co frag][64 lanes x 16
//    bytes]): each lane's A fragment is slot `lane` of a 1 KiB block, a linear, conflict-free read.
//  * XCD-aware block order (T1): the co-blocks of one pixel tile are consecutive logical blocks on
//    one XCD, so the second reads the halo from L2.
#include <cstdlib>

#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int SLOT = 16;  // bytes per LDS slot (one dwordx4 DMA lane); a halo pixel = 2 slots (16 channels)

// Halo slot of channel half h of halo pixel i: two slots per pixel, the halves swapped on every
// other group of 8 pixels.  A B-fragment read (ds_read_b128, 16-lane groups {0-3,12-15,20-27},
// {4-11,16-19,28-31}, ... = 16 pixels at one half) then lands on bank slots
// 2 (i mod 8) + ((i >> 3) & 1) ^ h, a bijection of i mod 16, and the 16 pixels of a group are
// distinct mod 16 for ANY tap shift: conflict-free without the 50 % pad slot of a 48-byte stride.
__device__ __forceinline__ int hslot(int i, int h) { return 2 * i + (h ^ ((i >> 3) & 1)); }

struct IgArgs {
  const bf16_t* x;     // [N, H, W, Cin] activated input
  const bf16_t* w;     // packed [Cout/BN][Cin/16][9][BN/32][64][8]
  const float* bias;   // [Cout] or null
  const bf16_t* res;   // [N, H, W, Cout] or null
  bf16_t* out;         // [N, H, W, Cout] or null
  bf16_t* aout;        // [N, H, W, Cout] or null
  const float* as;     // [Cout] scale of the activated copy (null = 1)
  const float* at;     // [Cout] (at_ns = 0) or [N, at_ns] shift (null = 0)
  const bf16_t* zero;  // zero page (>= 2 * Cin + 64 bytes)
  int at_ns, arelu, post_relu;
  int N, H, W, Cin, Cout, NP, HW;
  int nchunk, tiles, cob;
  int hbytes;  // halo bytes per stage buffer (multiple of 1 KiB)
};

template <int WM, int WN, int HIMAX>
struct IgCfg {
  static constexpr int NW = WM * WN, NT = NW * 64;
  static constexpr int BM = 64 * WM, BN = 64 * WN;
  static constexpr int NCF = BN / 32;            // 32-channel output fragments per block
  static constexpr int WBLK = 9 * NCF;           // 1 KiB weight blocks per stage
  static constexpr int WBYTES = WBLK * 1024;
  static constexpr int WPW = (WBLK + NW - 1) / NW;  // weight DMAs per wave per stage
};

// s_waitcnt immediate waiting for vmcnt <= n only (gfx9 encoding)
constexpr int vm_imm(int n) { return (n & 0xf) | (0x7 << 4) | (0xf << 8) | ((n >> 4) << 14); }

// vmcnt <= n for a wave-uniform runtime n (the immediate field needs a constant: one case each)
__device__ __forceinline__ void wait_vm_dyn(int n) {
  switch (n) {
#define BE_VM_CASE(k) \
  case k: __builtin_amdgcn_s_waitcnt(vm_imm(k)); break;
    BE_VM_CASE(1) BE_VM_CASE(2) BE_VM_CASE(3) BE_VM_CASE(4) BE_VM_CASE(5) BE_VM_CASE(6) BE_VM_CASE(7)
    BE_VM_CASE(8) BE_VM_CASE(9) BE_VM_CASE(10) BE_VM_CASE(11) BE_VM_CASE(12) BE_VM_CASE(13) BE_VM_CASE(14)
    BE_VM_CASE(15) BE_VM_CASE(16)
#undef BE_VM_CASE
    default: __builtin_amdgcn_s_waitcnt(vm_imm(0)); break;
  }
}

template <int WM, int WN, int HIMAX, int NSTAGE>
__global__ __launch_bounds__(WM * WN * 64, 2) void conv3_igemm_kernel(IgArgs a) {
  using C = IgCfg<WM, WN, HIMAX>;
  static_assert(NSTAGE == 2 || NSTAGE == 3, "two or three stage buffers");
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform: scalar branches
  const int wm = wave / WN, wn = wave % WN;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = lid / a.cob, cb = lid % a.cob;
  const int m0 = tile * C::BM;
  const int m1 = min(m0 + C::BM, a.NP) - 1;
  const int W2 = a.W + 2, H2 = a.H + 2;
  // padded-row range of the tile's halo
  const int n0 = m0 / a.HW, y0 = (m0 - n0 * a.HW) / a.W;
  const int n1 = m1 / a.HW, y1 = (m1 - n1 * a.HW) / a.W;
  const int Rlo = n0 * H2 + y0;          // = R(n0, y0) - 1
  const int Rhi = n1 * H2 + y1 + 2;      // = R(n1, y1) + 1
  const int npix = (Rhi - Rlo + 1) * W2;
  const int nhi = (2 * npix + 63) / 64;  // halo DMAs per stage (<= HIMAX * NW, host-checked)
  const int bufb = C::WBYTES + a.hbytes;

  // ---- per-lane DMA sources for this tile (chunk 0; chunk c adds 16 channels per step)
  const bf16_t* hsrc[HIMAX];
#pragma unroll
  for (int k = 0; k < HIMAX; ++k) {
    const int i = wave + k * C::NW;
    const int s = i * 64 + lane;
    const int p = s >> 1, q = (s & 1) ^ ((p >> 3) & 1);  // inverse of hslot(): source of DMA slot s
    const bf16_t* src = a.zero;
    if (i < nhi && p < npix) {
      const int r = Rlo + p / W2;
      const int c = p - (p / W2) * W2 - 1;
      const int n = r / H2;
      const int y = r - n * H2 - 1;
      if (n < a.N && y >= 0 && y < a.H && c >= 0 && c < a.W)
        src = a.x + ((long long)(n * a.H + y) * a.W + c) * a.Cin + q * 8;
    }
    hsrc[k] = src;
  }
  const bf16_t* wsrc = a.w + (long long)cb * a.nchunk * C::WBLK * 512 + lane * 8;

  auto stage = [&](int c, unsigned char* buf) {
#pragma unroll
    for (int k = 0; k < C::WPW; ++k) {
      const int i = wave + k * C::NW;
      if (i < C::WBLK)
        __builtin_amdgcn_global_load_lds((const void*)(wsrc + ((long long)c * C::WBLK + i) * 512),
                                         (lds_void*)(buf + i * 1024), 16, 0, 0);
    }
    const int zoff = c * 16;  // the zero page is long enough for every chunk offset
#pragma unroll
    for (int k = 0; k < HIMAX; ++k) {
      const int i = wave + k * C::NW;
      if (i < nhi)
        __builtin_amdgcn_global_load_lds((const void*)(hsrc[k] + zoff), (lds_void*)(buf + C::WBYTES + i * 1024), 16,
                                         0, 0);
    }
  };

  // ---- per-lane B-fragment (pixel) addresses, one per (tap, fragment): halo byte offsets
  int paddr[9][2];
  int pn[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    int m = m0 + wm * 64 + j * 32 + (lane & 31);
    m = m < a.NP ? m : m1;
    const int n = m / a.HW;
    const int rem = m - n * a.HW;
    const int y = rem / a.W, x = rem - (rem / a.W) * a.W;
    const int hidx = (n * H2 + y + 1 - Rlo) * W2 + x + 1;
    pn[j] = n;
#pragma unroll
    for (int t = 0; t < 9; ++t) paddr[t][j] = hslot(hidx + (t / 3 - 1) * W2 + (t % 3 - 1), lane >> 5) * SLOT;
  }

  f32x16 acc[2][2];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[f][j][r] = 0.f;

  const int wfrag0 = wn * 2;
  // this wave's DMAs per stage (wave-uniform, the same for every chunk of the tile)
  int nw_loads = 0;
#pragma unroll
  for (int k = 0; k < C::WPW; ++k) nw_loads += (wave + k * C::NW < C::WBLK);
#pragma unroll
  for (int k = 0; k < HIMAX; ++k) nw_loads += (wave + k * C::NW < nhi);
  stage(0, smem);
  if (NSTAGE == 3 && a.nchunk > 1) stage(1, smem + bufb);
  for (int c = 0; c < a.nchunk; ++c) {
    int cur_buf;
    if constexpr (NSTAGE == 2) {
      __syncthreads();  // vmcnt(0): chunk c landed (every wave); WAR: chunk c-1's buffer is free
      if (c + 1 < a.nchunk) stage(c + 1, smem + ((c + 1) & 1) * bufb);
      cur_buf = c & 1;
    } else {
      // three buffers, chunk c+1's DMA stays in flight across the barrier: wait until at most this
      // wave's per-stage DMA count is outstanding (a counted wait; the count is wave-uniform)
      if (c + 1 < a.nchunk) wait_vm_dyn(nw_loads);
      else __builtin_amdgcn_s_waitcnt(vm_imm(0));
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();  // chunk c is in LDS for every wave; chunk c-1's buffer is free
      __builtin_amdgcn_sched_barrier(0);
      if (c + 2 < a.nchunk) stage(c + 2, smem + ((c + 2) % 3) * bufb);
      cur_buf = c % 3;
    }
    const unsigned char* wb = smem + cur_buf * bufb;
    const unsigned char* hb = wb + C::WBYTES;
    bf16x8 wf[2][2], pf[2][2];
    auto ld = [&](int t, bf16x8 (&wfr)[2], bf16x8 (&pfr)[2]) {
#pragma unroll
      for (int f = 0; f < 2; ++f)
        wfr[f] = *reinterpret_cast<const bf16x8*>(wb + (t * C::NCF + wfrag0 + f) * 1024 + lane * SLOT);
#pragma unroll
      for (int j = 0; j < 2; ++j) pfr[j] = *reinterpret_cast<const bf16x8*>(hb + paddr[t][j]);
    };
    ld(0, wf[0], pf[0]);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int cur = t & 1;
      if (t + 1 < 9) ld(t + 1, wf[cur ^ 1], pf[cur ^ 1]);
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[f][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[cur][f], pf[cur][j], acc[f][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // ---- epilogue: lane = pixel (lane & 31), registers = channels (r&3) + 8 (r>>2) + 4 (lane>>5)
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int cbase = cb * C::BN + wn * 64 + f * 32 + 4 * (lane >> 5);
    float4 bv[4], sv[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      bv[g] = a.bias ? *reinterpret_cast<const float4*>(a.bias + cbase + 8 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
      sv[g] = a.as ? *reinterpret_cast<const float4*>(a.as + cbase + 8 * g) : make_float4(1.f, 1.f, 1.f, 1.f);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int m = m0 + wm * 64 + j * 32 + (lane & 31);
      if (m >= a.NP) continue;
      const long long po = (long long)m * a.Cout;
      u32x2 rv[4];
#pragma unroll
      for (int g = 0; g < 4; ++g)
        rv[g] = a.res ? *reinterpret_cast<const u32x2*>(a.res + po + cbase + 8 * g) : (u32x2){0u, 0u};
      float4 tv[4];
#pragma unroll
      for (int g = 0; g < 4; ++g)
        tv[g] = a.at ? *reinterpret_cast<const float4*>(a.at + (long long)pn[j] * a.at_ns + cbase + 8 * g)
                     : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float v0 = acc[f][j][4 * g + 0] + bv[g].x + lo_bf(rv[g][0]);
        float v1 = acc[f][j][4 * g + 1] + bv[g].y + hi_bf(rv[g][0]);
        float v2 = acc[f][j][4 * g + 2] + bv[g].z + lo_bf(rv[g][1]);
        float v3 = acc[f][j][4 * g + 3] + bv[g].w + hi_bf(rv[g][1]);
        u32x2 st;
        st[0] = pack2bf(v0, v1);
        st[1] = pack2bf(v2, v3);
        if (a.post_relu) {
          st[0] = relu_bf16x2(st[0]);
          st[1] = relu_bf16x2(st[1]);
        }
        if (a.out) *reinterpret_cast<u32x2*>(a.out + po + cbase + 8 * g) = st;
        if (a.aout) {
          // the consumer's pre-activation acts on the bf16-rounded tensor, as if it had re-read `out`
          float q0 = fmaf(lo_bf(st[0]), sv[g].x, tv[g].x), q1 = fmaf(hi_bf(st[0]), sv[g].y, tv[g].y);
          float q2 = fmaf(lo_bf(st[1]), sv[g].z, tv[g].z), q3 = fmaf(hi_bf(st[1]), sv[g].w, tv[g].w);
          u32x2 at;
          at[0] = pack2bf(q0, q1);
          at[1] = pack2bf(q2, q3);
          if (a.arelu) {
            at[0] = relu_bf16x2(at[0]);
            at[1] = relu_bf16x2(at[1]);
          }
          *reinterpret_cast<u32x2*>(a.aout + po + cbase + 8 * g) = at;
        }
      }
    }
  }
}

template <int WM, int WN, int NSTAGE>
int launch_ig(IgArgs a, hipStream_t s) {
  constexpr int HIMAX = WM * WN == 4 ? 8 : 6;
  using C = IgCfg<WM, WN, HIMAX>;
  if (a.Cout % C::BN) return -20;
  a.cob = a.Cout / C::BN;
  a.tiles = (a.NP + C::BM - 1) / C::BM;
  // worst-case padded rows of BM consecutive pixels: output rows + 2 halo rows + 2 per image crossed
  const int rows_out = (C::BM - 1) / a.W + 2;
  const int cross = (C::BM - 1) / a.HW + 1;
  int rows = rows_out + 2 * cross + 2;
  const int rmax = a.N * (a.H + 2);
  if (rows > rmax) rows = rmax;
  const int npix = rows * (a.W + 2);
  const int nhi = (2 * npix + 63) / 64;
  if (nhi > HIMAX * C::NW) return -21;
  a.hbytes = nhi * 1024;
  const size_t lds = NSTAGE * (size_t)(C::WBYTES + a.hbytes);
  if (lds > 160 * 1024) return -22;
  const long long nblk = (long long)a.tiles * a.cob;
  if (nblk >= (1LL << 31)) return -23;
  static bool attr_set[BE_MAX_DEV] = {};
  if (!attr_set[be_cur_dev()]) {
    (void)hipFuncSetAttribute((const void*)conv3_igemm_kernel<WM, WN, HIMAX, NSTAGE>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set[be_cur_dev()] = true;
  }
  hipLaunchKernelGGL((conv3_igemm_kernel<WM, WN, HIMAX, NSTAGE>), dim3((unsigned)nblk), dim3(C::NT), lds, s, a);
  return BE_CHECK_LAUNCH();
}

static const bf16_t* zero_page() { return be_zero_page(0, 1 << 20); }

}  // namespace

extern "C" {

static int ig_geometry(int bn, int* BM, int* NW, int* HIMAX) {
  // bn 64: 256 pixels x 64 channels, 4 waves (two workgroups per CU when the halo fits: one's
  // barrier / epilogue overlaps the other's MFMAs); bn 128: 256 x 128, 8 waves; bn 65: 512 x 64,
  // 8 waves (A/B configurations)
  if (bn == 64) { *BM = 256; *NW = 4; *HIMAX = 8; return 64; }
  if (bn == 128) { *BM = 256; *NW = 8; *HIMAX = 6; return 128; }
  if (bn == 65) { *BM = 512; *NW = 8; *HIMAX = 6; return 64; }
  return 0;
}

// LDS bytes a launch would use (0 = shape not supported by this kernel): lets the host pick a path.
// bn + 1000: the three-stage variant.
int be_conv3_igemm_lds(int N, int H, int W, int Cout, int bn) {
  const int nst = bn >= 1000 ? 3 : 2;
  bn %= 1000;
  int BM, NW, HIMAX;
  const int bnc = ig_geometry(bn, &BM, &NW, &HIMAX);
  if (!bnc || Cout % bnc) return 0;
  const int HW = H * W;
  int rows = (BM - 1) / W + 2 + 2 * ((BM - 1) / HW + 1) + 2;
  if (rows > N * (H + 2)) rows = N * (H + 2);
  const int nhi = (2 * rows * (W + 2) + 63) / 64;
  if (nhi > HIMAX * NW) return 0;
  const long long lds = (long long)nst * (9 * (bnc / 32) * 1024 + nhi * 1024);
  return lds > 160 * 1024 ? 0 : (int)lds;
}

// Packed weight layout: [Cout/bn][Cin/16][9][bn/32][2][32][8] bf16 (see ops/conv_igemm.py).
int be_conv3_igemm(const void* x, const void* w, const float* bias, const void* res, void* out, void* aout,
                   const float* as, const float* at, int at_ns, int arelu, int post_relu, int N, int H, int W, int Cin,
                   int Cout, int bn, hipStream_t stream) {
  if (Cin % 16 || Cout % 64 || (long long)N * H * W >= (1LL << 31)) return -10;
  if ((long long)N * H * W * (Cin > Cout ? Cin : Cout) * 2 >= (1LL << 40)) return -11;
  if (2 * Cin + 64 > (1 << 20)) return -12;
  IgArgs a;
  a.x = (const bf16_t*)x; a.w = (const bf16_t*)w; a.bias = bias; a.res = (const bf16_t*)res;
  a.out = (bf16_t*)out; a.aout = (bf16_t*)aout; a.as = as; a.at = at; a.at_ns = at_ns; a.arelu = arelu;
  a.post_relu = post_relu;
  a.zero = zero_page();
  if (!a.zero) return -13;
  a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.HW = H * W; a.NP = N * H * W;
  a.nchunk = Cin / 16;
  switch (bn) {  // bn + 1000: three stage buffers (DMA two chunks ahead, counted waits)
    case 128: return launch_ig<4, 2, 2>(a, stream);
    case 64: return launch_ig<4, 1, 2>(a, stream);
    case 65: return launch_ig<8, 1, 2>(a, stream);
    case 1128: return launch_ig<4, 2, 3>(a, stream);
    case 1065: return launch_ig<8, 1, 3>(a, stream);
  }
  return -14;
}

}  // extern "C"

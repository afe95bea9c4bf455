// EM instance separation on the GPU (reference
// apps/fibsem-mito-analysis/analysis_deployment.py:160-176): marker-controlled watershed on -EDT in
// 2-D and 3-D, and the 3-D exact Euclidean distance transform it floods.
//
// Watershed as a parallel fixpoint.  skimage's watershed is a priority flood: pixels leave a heap
// in order of (elevation, insertion age) and take the label of the neighbour that inserted them.
// Its GPU form here follows the flood's own recursion: every mask voxel q takes its label from the
// neighbour p with the smallest key, key = (c = flooding level at which the voxel leaves the heap,
// h = breadth-first steps inside that level's plateau -- the heap's FIFO age --, label), and
//     key(q) = ( max(elev(q), c_p),  elev(q) > c_p ? 0 : h_p + 1,  label_p ).
// (c, h) strictly increase from p to q, so the labels follow a DAG and the fixpoint is unique: any
// update order reaches it.  Workgroups stage a 16x16(xTZ) tile + 1-voxel halo of packed 64-bit
// keys in LDS, relax Gauss-Seidel style until the tile is stable, write back, and the host
// repeats launches until no tile changed.  A key packs ordered-float(c):32 | h:12 | label:20 into
// one word, so a relaxation never pairs one label's cost with another label (no torn updates).
// Tie-breaking inside equal (c, h) can differ from the heap's insertion order, so boundary voxels
// between basins may differ from the CPU priority flood (csrc/runtime/watershed.cpp) -- the GPU
// test bounds that fraction.
//
// EDT 3-D: separable passes -- a 1-D scan along z (squared distance to the nearest background voxel
// in the column), then d(q) = min_p (q - p)^2 + f(p) along y and along x, sqrt at the end.  The two
// min passes run one thread per VOXEL with a search that stops once r^2 >= the best value so far
// (every farther candidate is at least r^2): EM foreground is thin, so the window is a few voxels,
// and neighbouring threads read neighbouring addresses.  The old thread-per-LINE lower envelope of
// parabolas (Felzenszwalb-Huttenlocher, its stack in global memory) took 0.33 s per 256 x 2048^2
// slab.  A voxel whose search passes EDT_RCAP flags its line, and the envelope kernel then redoes
// exactly the flagged lines (thick objects, columns with no background).  Squared distances are
// integers below 2^24, exact in fp32, so both paths give the exact transform.
#include <cstdlib>

#include "common.h"

namespace {

constexpr int WS_TX = 16, WS_TY = 16;
constexpr unsigned long long WS_NONE = ~0ull;
constexpr int WS_LABEL_BITS = 20;
constexpr unsigned WS_LABEL_MASK = (1u << WS_LABEL_BITS) - 1u;
constexpr unsigned WS_HOP_MAX = 4095u;

__device__ __forceinline__ unsigned ordered(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ unsigned long long pack_key(unsigned c, unsigned h, unsigned lab) {
  return ((unsigned long long)c << 32) | ((unsigned long long)(h < WS_HOP_MAX ? h : WS_HOP_MAX) << WS_LABEL_BITS) |
         (unsigned long long)lab;
}

// key[p]: WS_NONE = unreached.  fixed[p] = marker voxel (keeps its initial key).  Each block owns a
// TZ x 16 x 16 tile; LDS holds tile + halo of keys, elevations and mask/fixed flags.
template <int TZ>
__global__ __launch_bounds__(WS_TX* WS_TY* TZ) void ws_relax_kernel(const float* __restrict__ elev,
                                                                      const unsigned char* __restrict__ flags,
                                                                      unsigned long long* __restrict__ key, int D, int H,
                                                                      int W, int tiles_x, int tiles_y, int max_local,
                                                                      int* __restrict__ changed,
                                                                      const unsigned char* __restrict__ dirty_in,
                                                                      unsigned char* __restrict__ dirty_out) {
  constexpr int HX = WS_TX + 2, HY = WS_TY + 2, HZ = TZ == 1 ? 1 : TZ + 2;
  constexpr int NH = HX * HY * HZ;
  constexpr int NT = WS_TX * WS_TY * TZ;
  __shared__ unsigned long long k_s[NH];
  __shared__ unsigned e_s[NH];
  __shared__ unsigned char f_s[NH];  // bit0 = in mask, bit1 = fixed (marker)
  __shared__ int any_s;
  const int tid = threadIdx.x;
  const int bx = blockIdx.x % tiles_x, by = blockIdx.x / tiles_x;
  const int bz = blockIdx.y;
  // active-tile sweeps: a tile is relaxed only if it or a face neighbour changed in the previous
  // sweep (dirty_in), so after the first sweeps only the flood front is touched
  const long long tile = (long long)bz * tiles_x * tiles_y + blockIdx.x;
  if (dirty_in && !dirty_in[tile]) return;  // workgroup-uniform
  const int x0 = bx * WS_TX - 1, y0 = by * WS_TY - 1, z0 = TZ == 1 ? bz : bz * TZ - 1;
  for (int e = tid; e < NH; e += NT) {
    const int lx = e % HX, ly = (e / HX) % HY, lz = e / (HX * HY);
    const int gx = x0 + lx, gy = y0 + ly, gz = z0 + lz;
    unsigned long long kv = WS_NONE;
    unsigned ev = 0xffffffffu;
    unsigned char fv = 0;
    if (gx >= 0 && gx < W && gy >= 0 && gy < H && gz >= 0 && gz < D) {
      const long long g = ((long long)gz * H + gy) * W + gx;
      kv = key[g];
      ev = ordered(elev[g]);
      fv = flags[g];
    }
    k_s[e] = kv;
    e_s[e] = ev;
    f_s[e] = fv;
  }
  if (tid == 0) any_s = 0;
  __syncthreads();
  const int tx = tid % WS_TX, ty = (tid / WS_TX) % WS_TY, tz = tid / (WS_TX * WS_TY);
  const int c = (tz + (TZ == 1 ? 0 : 1)) * HX * HY + (ty + 1) * HX + (tx + 1);
  const int gx = x0 + 1 + tx, gy = y0 + 1 + ty, gz = TZ == 1 ? z0 : z0 + 1 + tz;
  const bool active = gx < W && gy < H && gz < D && (f_s[c] & 1) && !(f_s[c] & 2);
  const unsigned ep = e_s[c];
  bool mine = false;  // this voxel improved at least once
  for (int it = 0; it < max_local; ++it) {
    bool ch = false;
    if (active) {
      // the flood labels a voxel from the neighbour that leaves the heap first: take the
      // neighbour with the smallest key and derive this voxel's key from it
      unsigned long long bn = WS_NONE;
      const int nb[6] = {c - 1, c + 1, c - HX, c + HX, c - HX * HY, c + HX * HY};
      const int nn = TZ == 1 ? 4 : 6;
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        if (j >= nn) break;
        const unsigned long long kq = k_s[nb[j]];
        if (kq < bn) bn = kq;
      }
      if (bn != WS_NONE) {
        const unsigned cq = (unsigned)(bn >> 32);
        const unsigned hq = (unsigned)((bn >> WS_LABEL_BITS) & WS_HOP_MAX);
        const unsigned lab = (unsigned)(bn & WS_LABEL_MASK);
        const unsigned long long nk = pack_key(ep > cq ? ep : cq, ep > cq ? 0u : hq + 1u, lab);
        if (nk != k_s[c]) {
          k_s[c] = nk;
          ch = true;
          mine = true;
        }
      }
    }
    if (__syncthreads_or(ch) == 0) break;
  }
  if (mine) {
    key[((long long)gz * H + gy) * W + gx] = k_s[c];
    any_s = 1;
  }
  __syncthreads();
  if (tid == 0 && any_s) {
    atomicOr(changed, 1);
    if (dirty_out) {
      const int tz_n = TZ == 1 ? D : (D + TZ - 1) / TZ;
      const long long txy = (long long)tiles_x * tiles_y;
      dirty_out[tile] = 1;
      if (bx > 0) dirty_out[tile - 1] = 1;
      if (bx + 1 < tiles_x) dirty_out[tile + 1] = 1;
      if (by > 0) dirty_out[tile - tiles_x] = 1;
      if (by + 1 < tiles_y) dirty_out[tile + tiles_x] = 1;
      if (TZ > 1 && bz > 0) dirty_out[tile - txy] = 1;
      if (TZ > 1 && bz + 1 < tz_n) dirty_out[tile + txy] = 1;
    }
  }
}

// Wide-tile variant: TZ x 32 x 32 voxels per 1024-thread block, TZ / (1024 / (32 * 32)) = TZ voxels
// per thread (one (y, x) column of the tile, z inner).  The flood crosses at most one tile boundary per
// sweep, so on the EM lines (one basin front spanning the 2048^2 plane) the sweep count is set by
// W / 16 = 128 tiles of the 16 x 16 kernel; 32 x 32 tiles halve it.  The thread's z voxels are relaxed
// in order within an iteration (their updates are visible to the next z at once).
template <int TZ>
__global__ __launch_bounds__(1024) void ws_relax_wide_kernel(const float* __restrict__ elev,
                                                             const unsigned char* __restrict__ flags,
                                                             unsigned long long* __restrict__ key, int D, int H,
                                                             int W, int tiles_x, int tiles_y, int max_local,
                                                             int* __restrict__ changed,
                                                             const unsigned char* __restrict__ dirty_in,
                                                             unsigned char* __restrict__ dirty_out) {
  constexpr int TX = 32, TY = 32;
  constexpr int HX = TX + 2, HY = TY + 2, HZ = TZ == 1 ? 1 : TZ + 2;
  constexpr int NH = HX * HY * HZ;
  constexpr int NT = 1024;
  __shared__ unsigned long long k_s[NH];
  __shared__ unsigned e_s[NH];
  __shared__ unsigned char f_s[NH];
  __shared__ int any_s;
  const int tid = threadIdx.x;
  const int bx = blockIdx.x % tiles_x, by = blockIdx.x / tiles_x;
  const int bz = blockIdx.y;
  const long long tile = (long long)bz * tiles_x * tiles_y + blockIdx.x;
  if (dirty_in && !dirty_in[tile]) return;  // workgroup-uniform
  const int x0 = bx * TX - 1, y0 = by * TY - 1, z0 = TZ == 1 ? bz : bz * TZ - 1;
  for (int e = tid; e < NH; e += NT) {
    const int lx = e % HX, ly = (e / HX) % HY, lz = e / (HX * HY);
    const int gx = x0 + lx, gy = y0 + ly, gz = z0 + lz;
    unsigned long long kv = WS_NONE;
    unsigned ev = 0xffffffffu;
    unsigned char fv = 0;
    if (gx >= 0 && gx < W && gy >= 0 && gy < H && gz >= 0 && gz < D) {
      const long long g = ((long long)gz * H + gy) * W + gx;
      kv = key[g];
      ev = ordered(elev[g]);
      fv = flags[g];
    }
    k_s[e] = kv;
    e_s[e] = ev;
    f_s[e] = fv;
  }
  if (tid == 0) any_s = 0;
  __syncthreads();
  const int tx = tid % TX, ty = tid / TX;
  const int gx = x0 + 1 + tx, gy = y0 + 1 + ty;
  const int c0 = (TZ == 1 ? 0 : 1) * HX * HY + (ty + 1) * HX + (tx + 1);
  bool act[TZ];
  unsigned ep[TZ];
#pragma unroll
  for (int z = 0; z < TZ; ++z) {
    const int c = c0 + z * HX * HY;
    const int gz = TZ == 1 ? z0 : z0 + 1 + z;
    act[z] = gx < W && gy < H && gz < D && (f_s[c] & 1) && !(f_s[c] & 2);
    ep[z] = e_s[c];
  }
  unsigned mine = 0;  // bit z: voxel z improved at least once
  for (int it = 0; it < max_local; ++it) {
    bool ch = false;
#pragma unroll
    for (int z = 0; z < TZ; ++z) {
      if (!act[z]) continue;
      const int c = c0 + z * HX * HY;
      auto mn = [](unsigned long long a, unsigned long long b) { return a < b ? a : b; };
      unsigned long long bn = mn(k_s[c - 1], k_s[c + 1]);
      bn = mn(bn, mn(k_s[c - HX], k_s[c + HX]));
      if (TZ > 1) bn = mn(bn, mn(k_s[c - HX * HY], k_s[c + HX * HY]));
      if (bn != WS_NONE) {
        const unsigned cq = (unsigned)(bn >> 32);
        const unsigned hq = (unsigned)((bn >> WS_LABEL_BITS) & WS_HOP_MAX);
        const unsigned lab = (unsigned)(bn & WS_LABEL_MASK);
        const unsigned long long nk = pack_key(ep[z] > cq ? ep[z] : cq, ep[z] > cq ? 0u : hq + 1u, lab);
        if (nk != k_s[c]) {
          k_s[c] = nk;
          ch = true;
          mine |= 1u << z;
        }
      }
    }
    if (__syncthreads_or(ch) == 0) break;
  }
  if (mine) {
#pragma unroll
    for (int z = 0; z < TZ; ++z)
      if (mine & (1u << z)) {
        const int gz = TZ == 1 ? z0 : z0 + 1 + z;
        key[((long long)gz * H + gy) * W + gx] = k_s[c0 + z * HX * HY];
      }
    any_s = 1;
  }
  __syncthreads();
  if (tid == 0 && any_s) {
    atomicOr(changed, 1);
    if (dirty_out) {
      const int tz_n = TZ == 1 ? D : (D + TZ - 1) / TZ;
      const long long txy = (long long)tiles_x * tiles_y;
      dirty_out[tile] = 1;
      if (bx > 0) dirty_out[tile - 1] = 1;
      if (bx + 1 < tiles_x) dirty_out[tile + 1] = 1;
      if (by > 0) dirty_out[tile - tiles_x] = 1;
      if (by + 1 < tiles_y) dirty_out[tile + tiles_x] = 1;
      if (TZ > 1 && bz > 0) dirty_out[tile - txy] = 1;
      if (TZ > 1 && bz + 1 < tz_n) dirty_out[tile + txy] = 1;
    }
  }
}

// Tile width of the relaxation sweeps: 32 (ws_relax_wide_kernel) or 16 (the 16 x 16 (x 4) kernel).
// Wide tiles halve the sweeps when few basins span the volume (3-D EM line: 136 -> 72 sweeps, 0.27 ->
// 0.20 s) but cost more per active tile when many small basins keep the front sparse (2-D EM line,
// ~10^4 basins: 0.27 -> 0.35 s), so the host picks per call from the marker density
// (be_ws_set_tile); BE_WS_TILE=16 / 32 pins it.
static int g_ws_tile = 0;
static int ws_tile() {
  static int env = [] {
    const char* e = getenv("BE_WS_TILE");
    return e ? (atoi(e) == 16 ? 16 : 32) : 0;
  }();
  if (env) return env;
  return g_ws_tile == 16 ? 16 : 32;
}

__global__ void ws_init_kernel(const float* __restrict__ elev, const int* __restrict__ markers,
                               const unsigned char* __restrict__ mask, long long n, unsigned long long* __restrict__ key,
                               unsigned char* __restrict__ flags) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int m = markers[i];
  const bool in = mask == nullptr || mask[i];
  unsigned char f = in ? 1 : 0;
  unsigned long long k = WS_NONE;
  if (in && m > 0) {
    f |= 2;
    k = pack_key(ordered(elev[i]), 0u, (unsigned)m);
  }
  key[i] = k;
  flags[i] = f;
}

__global__ void ws_labels_kernel(const unsigned long long* __restrict__ key, const unsigned char* __restrict__ flags,
                                 long long n, int* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned long long k = key[i];
  out[i] = ((flags[i] & 1) && k != WS_NONE) ? (int)(k & WS_LABEL_MASK) : 0;
}

// ---------------------------------------------------------------- 3-D EDT
// z scan: f[z, y, x] = (distance along z to the nearest background voxel)^2, or INF
__global__ void edt3_z(const unsigned char* __restrict__ fg, float* __restrict__ f, int D, int H, int W) {
  const long long col = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long HW = (long long)H * W;
  if (col >= HW) return;
  int last = -1;
  for (int z = 0; z < D; ++z) {
    if (!fg[z * HW + col]) last = z;
    f[z * HW + col] = last < 0 ? -1.f : (float)(z - last);
  }
  last = -1;
  for (int z = D - 1; z >= 0; --z) {
    if (!fg[z * HW + col]) last = z;
    float d = f[z * HW + col];
    if (last >= 0 && (d < 0.f || (float)(last - z) < d)) d = (float)(last - z);
    f[z * HW + col] = d < 0.f ? 3.0e38f : d * d;
  }
}

constexpr int EDT_RCAP = 64;

// bounded search along one axis (stride st, length L); line id of voxel i = (i / lo_div) * lo_mul +
// i % lo_mod (the edt3_axis line order); only[line] = 1 when a voxel of it passed EDT_RCAP
__global__ __launch_bounds__(256) void edt3_bf(const float* __restrict__ fin, float* __restrict__ fout, long long n, int L,
                                               long long st, long long lo_div, long long lo_mul, long long lo_mod,
                                               int take_sqrt, unsigned char* __restrict__ only) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int q = (int)((i / st) % L);
  float best = fin[i];
  const int rmax = max(q, L - 1 - q);
  int r = 1;
  for (; r <= rmax && r <= EDT_RCAP; ++r) {
    const float r2 = (float)(r * r);
    if (r2 >= best) break;
    if (q - r >= 0) best = fminf(best, r2 + fin[i - r * st]);
    if (q + r < L) best = fminf(best, r2 + fin[i + r * st]);
  }
  if (r > EDT_RCAP && r <= rmax && (float)(r * r) < best) only[(i / lo_div) * lo_mul + i % lo_mod] = 1;
  fout[i] = (!take_sqrt || best >= 3.0e38f) ? best : (float)sqrt((double)best);
}

// lower envelope of parabolas along one axis: lines of length L, element stride `st`, line bases
// from (line / inner) * outer_st + (line % inner) * inner_st.  f == 3e38 marks "no site".
// only (optional): skip the lines whose flag is 0.  The per-line stacks (parabola sites v, boundaries
// z) are interleaved across lines -- entry k of line l at k * nlines + l -- so the threads of a wave,
// which hold neighbouring lines at similar stack depths, touch neighbouring addresses (a line-major
// stack put every thread's entry on its own cache line).
__global__ void edt3_axis(const float* __restrict__ fin, float* __restrict__ fout, int* __restrict__ vbuf,
                          double* __restrict__ zbuf, long long nlines, int L, long long st, long long inner,
                          long long inner_st, long long outer_st, int take_sqrt,
                          const unsigned char* __restrict__ only = nullptr) {
  const long long line = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (line >= nlines) return;
  if (only && !only[line]) return;
  const long long base = (line / inner) * outer_st + (line % inner) * inner_st;
  int* v = vbuf + line;     // v[k * nlines]
  double* z = zbuf + line;  // z[k * nlines], k <= L
  const long long S = nlines;
  int k = -1;
  for (int q = 0; q < L; ++q) {
    const float fq = fin[base + q * st];
    if (fq >= 3.0e38f) continue;
    if (k < 0) {
      k = 0; v[0] = q; z[0] = -1e300; z[S] = 1e300;
      continue;
    }
    double s;
    for (;;) {
      const int p = v[k * S];
      const double fp = fin[base + p * st];
      s = ((double)fq + (double)q * q - (fp + (double)p * p)) / (2.0 * (q - p));
      if (s <= z[k * S] && k > 0) { --k; continue; }
      break;
    }
    ++k; v[k * S] = q; z[k * S] = s; z[(k + 1) * S] = 1e300;
  }
  if (k < 0) {
    for (int q = 0; q < L; ++q) fout[base + q * st] = 3.0e38f;
    return;
  }
  int j = 0;
  for (int q = 0; q < L; ++q) {
    while (z[(j + 1) * S] < (double)q) ++j;
    const int vj = v[j * S];
    const double d = (double)(q - vj);
    const double r = d * d + (double)fin[base + vj * st];
    fout[base + q * st] = take_sqrt ? (float)sqrt(r) : (float)r;
  }
}

// ---------------------------------------------------------------- component size filter
// Sizes of CCL components (root = a voxel index, -1 = background).  A workgroup takes CS_CHUNK
// consecutive voxels (coalesced: thread t reads voxel i * 256 + t of the chunk) and counts them in
// an LDS hash map (root -> count, open addressing); a wave whose 64 voxels share one root (the
// inside of a component) inserts them as one entry.  Each root of the chunk then costs ONE global
// atomic.  Per-voxel global atomics serialised on large components (5 s per 128 x 2048^2), and so
// did per-thread run-length atomics over uncoalesced 256-voxel runs (0.50 s per 256 x 2048^2, s39,
// against 0.25 s for the torch.unique sort).  A chunk with more distinct roots than the map holds
// sends the overflow straight to global atomics.
constexpr int CS_CHUNK = 256 * 64;
constexpr int CS_HASH = 2048;

__device__ __forceinline__ void cs_insert(int* keys, int* vals, int r, int c, int* __restrict__ counts) {
  unsigned h = ((unsigned)r * 2654435761u) & (CS_HASH - 1);
  for (int probe = 0; probe < 32; ++probe) {
    const int old = atomicCAS(keys + h, -1, r);
    if (old == -1 || old == r) {
      atomicAdd(vals + h, c);
      return;
    }
    h = (h + 1) & (CS_HASH - 1);
  }
  atomicAdd(counts + r, c);  // crowded map: global
}

__global__ __launch_bounds__(256) void comp_count_kernel(const int* __restrict__ roots, long long n, int* __restrict__ counts,
                                                         int bg) {
  __shared__ int keys[CS_HASH], vals[CS_HASH];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < CS_HASH; i += 256) { keys[i] = -1; vals[i] = 0; }
  __syncthreads();
  const long long base = (long long)blockIdx.x * CS_CHUNK;
  for (int it = 0; it < CS_CHUNK / 256; ++it) {
    const long long i = base + (long long)it * 256 + tid;
    int r = i < n ? roots[i] : -1;
    if (r == bg) r = -1;
    const int r0 = __shfl(r, 0, 64);
    if (__all(r == r0)) {
      if (lane == 0 && r0 >= 0) cs_insert(keys, vals, r0, 64, counts);
    } else if (r >= 0) {
      cs_insert(keys, vals, r, 1, counts);
    }
  }
  __syncthreads();
  for (int i = tid; i < CS_HASH; i += 256)
    if (keys[i] >= 0) atomicAdd(counts + keys[i], vals[i]);
}

__global__ __launch_bounds__(256) void comp_keep_kernel(const int* __restrict__ roots, long long n,
                                                        const int* __restrict__ counts, int min_size,
                                                        unsigned char* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int r = roots[i];
  out[i] = (r >= 0 && counts[r] >= min_size) ? 1 : 0;
}

}  // namespace

extern "C" {

// out[i] = 1 where voxel i's component (roots: CCL root voxel index, -1 background, all < n) has
// >= min_size voxels.  counts: n ints of scratch.
int be_component_keep(const int* roots, long long n, int* counts, int min_size, unsigned char* out, hipStream_t s) {
  if (n == 0) return 0;
  (void)hipMemsetAsync(counts, 0, (size_t)n * sizeof(int), s);
  const long long nchunk = (n + CS_CHUNK - 1) / CS_CHUNK;
  hipLaunchKernelGGL(comp_count_kernel, dim3((unsigned)nchunk), dim3(256), 0, s, roots, n, counts, -1);
  hipLaunchKernelGGL(comp_keep_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, roots, n, counts, min_size, out);
  return BE_CHECK_LAUNCH();
}


// counts[l] = voxels with label l for l in [1, nbins) (labels: int32 in [0, nbins), 0 = background,
// counts[0] = 0), with the LDS-hash chunk counter above.  Replaces torch.bincount on the sharded EM
// path, which died with SIGFPE on a 256 x 2048^2 slab of the 3-D line (profiles/r06/rehearsal/).
int be_em_label_counts(const int* labels, long long n, int* counts, int nbins, hipStream_t s) {
  if (nbins <= 0) return -10;
  (void)hipMemsetAsync(counts, 0, (size_t)nbins * sizeof(int), s);
  if (n == 0) return 0;
  const long long nchunk = (n + CS_CHUNK - 1) / CS_CHUNK;
  if (nchunk >= (1LL << 31)) return -11;
  hipLaunchKernelGGL(comp_count_kernel, dim3((unsigned)nchunk), dim3(256), 0, s, labels, n, counts, 0);
  return BE_CHECK_LAUNCH();
}

// Marker watershed on elev (e.g. -EDT) restricted to mask (uint8, optional), markers int32 (>0),
// D = 1 for 2-D.  key: [n] uint64 scratch, flags: [n] uint8 scratch, changed: 1 int (device).
// One call = one relaxation sweep over all tiles; returns 0 and the caller loops while *changed.
int be_ws_init(const float* elev, const int* markers, const unsigned char* mask, long long n, unsigned long long* key,
               unsigned char* flags, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(ws_init_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, elev, markers, mask, n, key, flags);
  return BE_CHECK_LAUNCH();
}

int be_ws_relax(const float* elev, const unsigned char* flags, unsigned long long* key, int D, int H, int W, int max_local,
                int* changed, hipStream_t s) {
  if (ws_tile() == 32) {
    const int tiles_x = (W + 31) / 32, tiles_y = (H + 31) / 32;
    if (D == 1)
      hipLaunchKernelGGL(ws_relax_wide_kernel<1>, dim3(tiles_x * tiles_y, 1), dim3(1024), 0, s, elev, flags, key, D, H, W,
                         tiles_x, tiles_y, max_local, changed, nullptr, nullptr);
    else
      hipLaunchKernelGGL(ws_relax_wide_kernel<4>, dim3(tiles_x * tiles_y, (D + 3) / 4), dim3(1024), 0, s, elev, flags, key,
                         D, H, W, tiles_x, tiles_y, max_local, changed, nullptr, nullptr);
    return BE_CHECK_LAUNCH();
  }
  const int tiles_x = (W + WS_TX - 1) / WS_TX, tiles_y = (H + WS_TY - 1) / WS_TY;
  if (D == 1) {
    hipLaunchKernelGGL(ws_relax_kernel<1>, dim3(tiles_x * tiles_y, 1), dim3(WS_TX * WS_TY), 0, s, elev, flags, key, D, H, W,
                       tiles_x, tiles_y, max_local, changed, nullptr, nullptr);
  } else {
    constexpr int TZ = 4;
    hipLaunchKernelGGL(ws_relax_kernel<TZ>, dim3(tiles_x * tiles_y, (D + TZ - 1) / TZ), dim3(WS_TX * WS_TY * TZ), 0, s,
                       elev, flags, key, D, H, W, tiles_x, tiles_y, max_local, changed, nullptr, nullptr);
  }
  return BE_CHECK_LAUNCH();
}

// Number of relaxation tiles (the size of the dirty-tile arrays of be_ws_relax_active).
long long be_ws_tiles(int D, int H, int W) {
  const int t = ws_tile() == 32 ? 32 : WS_TX;
  const long long txy = (long long)((W + t - 1) / t) * ((H + t - 1) / t);
  return D == 1 ? txy : txy * ((D + 3) / 4);
}

// One sweep over the tiles flagged in dirty_in (all ones for the first sweep); the tiles that
// changed and their face neighbours are flagged in dirty_out, which this call zeroes first.
int be_ws_relax_active(const float* elev, const unsigned char* flags, unsigned long long* key, int D, int H, int W,
                       int max_local, int* changed, const unsigned char* dirty_in, unsigned char* dirty_out, hipStream_t s) {
  (void)hipMemsetAsync(dirty_out, 0, (size_t)be_ws_tiles(D, H, W), s);
  if (ws_tile() == 32) {
    const int tiles_x = (W + 31) / 32, tiles_y = (H + 31) / 32;
    if (D == 1)
      hipLaunchKernelGGL(ws_relax_wide_kernel<1>, dim3(tiles_x * tiles_y, 1), dim3(1024), 0, s, elev, flags, key, D, H, W,
                         tiles_x, tiles_y, max_local, changed, dirty_in, dirty_out);
    else
      hipLaunchKernelGGL(ws_relax_wide_kernel<4>, dim3(tiles_x * tiles_y, (D + 3) / 4), dim3(1024), 0, s, elev, flags, key,
                         D, H, W, tiles_x, tiles_y, max_local, changed, dirty_in, dirty_out);
    return BE_CHECK_LAUNCH();
  }
  const int tiles_x = (W + WS_TX - 1) / WS_TX, tiles_y = (H + WS_TY - 1) / WS_TY;
  if (D == 1) {
    hipLaunchKernelGGL(ws_relax_kernel<1>, dim3(tiles_x * tiles_y, 1), dim3(WS_TX * WS_TY), 0, s, elev, flags, key, D, H, W,
                       tiles_x, tiles_y, max_local, changed, dirty_in, dirty_out);
  } else {
    constexpr int TZ = 4;
    hipLaunchKernelGGL(ws_relax_kernel<TZ>, dim3(tiles_x * tiles_y, (D + TZ - 1) / TZ), dim3(WS_TX * WS_TY * TZ), 0, s,
                       elev, flags, key, D, H, W, tiles_x, tiles_y, max_local, changed, dirty_in, dirty_out);
  }
  return BE_CHECK_LAUNCH();
}

int be_ws_labels(const unsigned long long* key, const unsigned char* flags, long long n, int* out, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(ws_labels_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, key, flags, n, out);
  return BE_CHECK_LAUNCH();
}

int be_ws_max_label() { return (int)WS_LABEL_MASK; }

// 16 or 32: the tile width of the following be_ws_tiles / be_ws_relax* calls (unless BE_WS_TILE is set)
int be_ws_set_tile(int t) {
  g_ws_tile = t == 16 ? 16 : 32;
  return 0;
}

// 3-D EDT of fg [D, H, W] uint8 -> dist fp32.  tmp: [D*H*W] fp32; v: [D*H*W + D*max(H, W)] int
// scratch (the tail holds the per-line fallback flags); z: [D*H*W + D*max(H, W)] double scratch
// (L + 1 per line; both only touched on fallback lines).
int be_edt3d(const unsigned char* fg, float* dist, float* tmp, int* v, double* z, int D, int H, int W, hipStream_t s) {
  const long long HW = (long long)H * W, n = (long long)D * HW;
  if (n == 0) return 0;
  unsigned char* only = reinterpret_cast<unsigned char*>(v + n);
  const unsigned nb = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(edt3_z, dim3((unsigned)((HW + 255) / 256)), dim3(256), 0, s, fg, dist, D, H, W);
  // along y: lines = D*W, line (zz, x) base = zz*HW + x, stride W; voxel i -> line (i / HW) * W + i % W
  long long nl = (long long)D * W;
  (void)hipMemsetAsync(only, 0, nl, s);
  hipLaunchKernelGGL(edt3_bf, dim3(nb), dim3(256), 0, s, dist, tmp, n, H, (long long)W, HW, (long long)W, (long long)W, 0, only);
  hipLaunchKernelGGL(edt3_axis, dim3((unsigned)((nl + 255) / 256)), dim3(256), 0, s, dist, tmp, v, z, nl, H, (long long)W,
                     (long long)W, 1LL, HW, 0, only);
  // along x: lines = D*H, line (zz, y) base = (zz*H + y)*W, stride 1; voxel i -> line i / W
  nl = (long long)D * H;
  (void)hipMemsetAsync(only, 0, nl, s);
  hipLaunchKernelGGL(edt3_bf, dim3(nb), dim3(256), 0, s, tmp, dist, n, W, 1LL, (long long)W, 1LL, 1LL, 1, only);
  hipLaunchKernelGGL(edt3_axis, dim3((unsigned)((nl + 255) / 256)), dim3(256), 0, s, tmp, dist, v, z, nl, W, 1LL, nl,
                     (long long)W, 0LL, 1, only);
  return BE_CHECK_LAUNCH();
}

}  // extern "C"

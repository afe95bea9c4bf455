// Per-mask Cellpose post-processing: bounding boxes, heat-diffusion flows (masks_to_flows),
// flow-error QC and hole filling.  SURVEY.md §2.5 K5 (flow QC, flow_threshold at
// apps/cellpose-finetuning/main.py:5005-5012), K6 (fill holes / min_size), K10 (label -> flow
// training targets, invoked at main.py:1370-1387).  Oracle: bioengine_worker_amd/cellpose/reference.py.
//
// MI355X mapping: one workgroup per mask.  The mask's bounding box (+1 ring) is staged in LDS
// (membership bytes + two fp64 heat buffers), the whole Jacobi diffusion runs on-chip with one
// barrier per sweep, and only log(1 + T) of the mask pixels goes back to HBM.  Masks whose box
// exceeds the LDS budget are tiled across many workgroups with time-blocked sweeps and a grid
// barrier per block of iterations (diffuse_tiled_kernel).  Centres are exact medians from
// row/column histograms in LDS, ties broken in raster order with a 64-bit atomicMin key.
#include <cstdlib>

#include "common.h"

namespace {

constexpr int MT = 256;
constexpr int kDiffuseVariant = 0;

// Run-length scans: one thread walks RL consecutive pixels of one row and issues its atomics once
// per run of equal labels instead of once per pixel (labels come in long horizontal runs, so this
// is ~RL x fewer atomics on the same few hundred counters).
constexpr int RL = 16;

// bbox[b, lab] = (ymin, ymax, xmin, xmax); init (INT_MAX, -1, INT_MAX, -1) by the caller.
__global__ __launch_bounds__(256) void bbox_kernel(const int* __restrict__ M, int B, int H, int W, int nlab,
                                                   int* __restrict__ bbox) {
  const int segs = (W + RL - 1) / RL;
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long long)B * H * segs) return;
  const int seg = (int)(gid % segs);
  const long long row = gid / segs;  // b * H + y
  const int b = (int)(row / H), y = (int)(row % H);
  const int* Mr = M + row * W;
  const int x0 = seg * RL, x1 = min(x0 + RL, W);
  int cur = 0, xs = x0;
  auto flush = [&](int lab, int a, int e) {
    if (lab <= 0) return;
    int* bb = bbox + ((size_t)b * nlab + lab) * 4;
    atomicMin(bb + 0, y);
    atomicMax(bb + 1, y);
    atomicMin(bb + 2, a);
    atomicMax(bb + 3, e);
  };
  for (int x = x0; x < x1; ++x) {
    const int lab = Mr[x];
    if (lab != cur) {
      flush(cur, xs, x - 1);
      cur = lab;
      xs = x;
    }
  }
  flush(cur, xs, x1 - 1);
}

struct MaskJob {
  int b, lab, y0, x0, ly, lx;  // box origin (inclusive) and extent
  long long scratch;           // float offset into the global scratch arena (big masks), else -1
};

// Heat diffusion of one mask; writes L = log(1 + T) for its pixels into Lout [B, H, W].
// The heat field spans hundreds of orders of magnitude far from the centre of large masks (T decays
// like exp(-d^2/t)); cellpose runs it in float64 for that reason and so do we (gfx950 runs fp64 VALU
// at full vector rate, and this kernel is latency/LDS bound anyway).
constexpr int FG_RUN = 4;  // pixels per thread in flow_grad_kernel

// Largest mask the one-workgroup sparse sweep takes from global scratch: 1024 threads x SP_K (4).
constexpr int SPARSE_BIG_PX = 4096;

template <bool USE_LDS, int MT = 256, int DV = 8>
__global__ __launch_bounds__(MT) void diffuse_kernel(const int* __restrict__ M, const MaskJob* __restrict__ jobs, int H,
                                                     int W, const int* __restrict__ niter_img, double* __restrict__ scratch,
                                                     double* __restrict__ Lout, int* __restrict__ centers_out,
                                                     int variant = 0) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const MaskJob J = jobs[blockIdx.x];
  const int RY = J.ly + 2, RX = J.lx + 2, R = RY * RX;
  double* T0;
  double* T1;
  int* hy;
  int* hx;
  unsigned char* inm;
  if (USE_LDS) {
    T0 = reinterpret_cast<double*>(smem);
    T1 = T0 + R;
    hy = reinterpret_cast<int*>(T1 + R);
    hx = hy + RY;
    inm = reinterpret_cast<unsigned char*>(hx + RX);
  } else {
    T0 = scratch + J.scratch;
    T1 = T0 + R;
    hy = reinterpret_cast<int*>(T1 + R);
    hx = hy + RY;
    inm = reinterpret_cast<unsigned char*>(hx + RX);
  }
  __shared__ unsigned long long best;
  __shared__ int total;
  const int tid = threadIdx.x;
  const int* Mb = M + (size_t)J.b * H * W;
  for (int e = tid; e < R; e += MT) { T0[e] = 0.0; T1[e] = 0.0; }
  for (int e = tid; e < RY; e += MT) hy[e] = 0;
  for (int e = tid; e < RX; e += MT) hx[e] = 0;
  if (tid == 0) { best = ~0ull; total = 0; }
  __syncthreads();
  int cnt = 0;
  for (int e = tid; e < R; e += MT) {
    const int ry = e / RX, rx = e % RX;
    const int y = J.y0 + ry - 1, x = J.x0 + rx - 1;
    unsigned char m = 0;
    if (ry >= 1 && ry <= J.ly && rx >= 1 && rx <= J.lx) m = (Mb[y * W + x] == J.lab);
    inm[e] = m;
    if (m) { atomicAdd(&hy[ry], 1); atomicAdd(&hx[rx], 1); ++cnt; }
  }
  atomicAdd(&total, cnt);
  __syncthreads();
  // exact medians (numpy semantics: mean of the two middle values for even counts)
  __shared__ float med[2];
  if (tid < 2) {
    const int* h = tid == 0 ? hy : hx;
    const int L = tid == 0 ? RY : RX;
    const int n = total;
    const int k1 = (n - 1) / 2, k2 = n / 2;
    int acc = 0, v1 = -1, v2 = -1;
    for (int i = 0; i < L; ++i) {
      const int c = h[i];
      if (v1 < 0 && acc + c > k1) v1 = i;
      if (v2 < 0 && acc + c > k2) { v2 = i; break; }
      acc += c;
    }
    med[tid] = 0.5f * (float)(v1 + v2);
  }
  __syncthreads();
  for (int e = tid; e < R; e += MT) {
    if (!inm[e]) continue;
    const float dy = (float)(e / RX) - med[0], dx = (float)(e % RX) - med[1];
    const float d = dx * dx + dy * dy;
    const unsigned long long key = ((unsigned long long)__float_as_uint(d) << 32) | (unsigned)e;
    atomicMin(&best, key);
  }
  __syncthreads();
  const int ce = (int)(best & 0xffffffffu);
  if (centers_out) {  // big masks: the tiled multi-workgroup diffusion below runs the iterations
    if (tid == 0) centers_out[blockIdx.x] = ce;
    return;
  }
  const int niter = niter_img[J.b];
  // Column-segment register blocking: a work item is DV consecutive rows of one column; the three
  // horizontal 3-sums it needs per row are formed once and slid down the segment, so a cell costs
  // ~3 reads instead of 9.  Non-mask cells hold 0 in both buffers, so neighbour reads need no mask.
  const int nseg = (RY - 2 + DV - 1) / DV;
  const int nitems = (RX - 2) * nseg;
  double* cur = T0;
  double* nxt = T1;
  // Sparse sweep (the default whenever it fits): candidate masks are thin and irregular (flow-QC
  // census of the headline batch: 212 masks per image filling 14 % of their boxes), so sweeping
  // the whole box wastes most of the LDS traffic.  Each thread instead owns up to SP_K of the
  // mask's own pixels, balanced by rank (pixel r -> thread r % MT), kept in registers for all
  // iterations; a pixel update reads its 3x3 neighbourhood (non-mask cells hold 0 in both
  // buffers).  The centre source is folded into the reads of that one cell (cur[ce] + 1.0, the
  // value variant 0 stores before its sweep) and every sum is formed in variant 0's order, so the
  // result is bit-identical to the dense sweep with one barrier per iteration instead of two.
  constexpr int SP_K = 4;
  const bool sparse = variant == 0 && total <= SP_K * MT && total * 5 < R * 3;
  if (sparse) {
    const int cy = ce / RX, cx = ce % RX;
    // rank the mask pixels: per-thread counts over contiguous cell ranges, wave + block scans
    const int seg = (R + MT - 1) / MT;
    const int e0 = tid * seg, e1 = min(R, e0 + seg);
    int c = 0;
    for (int e = e0; e < e1; ++e) c += inm[e];
    int incl = c;
    const int lane = tid & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    __shared__ int wsum[MT / 64];
    if (lane == 63) wsum[tid >> 6] = incl;
    __syncthreads();
    int rank = incl - c;
    for (int w = 0; w < (tid >> 6); ++w) rank += wsum[w];
    int* list = reinterpret_cast<int*>(T1);  // 8R bytes >= 4 * total: free until the sweep starts
    for (int e = e0; e < e1; ++e)
      if (inm[e]) list[rank++] = e;
    __syncthreads();
    int own[SP_K];  // empty slots point at the centre (interior, so its 3x3 reads stay in the box)
    int nown = 0;
#pragma unroll
    for (int j = 0; j < SP_K; ++j) {
      const int r = tid + j * MT;
      own[j] = r < total ? list[r] : ce;
      nown += r < total;
    }
    __syncthreads();
    for (int e = tid; e < R; e += MT) T1[e] = 0.0;
    __syncthreads();
    for (int it = 0; it < niter; ++it) {
      // every slot's reads are issued unconditionally (one batch of independent ds_reads instead
      // of a branch per slot); only the stores are predicated
#pragma unroll
      for (int j = 0; j < SP_K; ++j) {
        {
          const int e = own[j];
          const double* cp = cur + e;
          const int dy = cy - e / RX + 1, dx = cx - e % RX + 1;
          const int pos = (dy >= 0 && dy <= 2 && dx >= 0 && dx <= 2) ? dy * 3 + dx : -1;
          double v[3][3];  // (+ 0.0 is exact for the non-negative heat values)
#pragma unroll
          for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int q = 0; q < 3; ++q) v[r][q] = cp[(r - 1) * RX + (q - 1)] + (r * 3 + q == pos ? 1.0 : 0.0);
          const double hp = v[0][0] + v[0][1] + v[0][2];
          const double hc = v[1][0] + v[1][1] + v[1][2];
          const double hn = v[2][0] + v[2][1] + v[2][2];
          if (j < nown) nxt[e] = (hp + hc + hn) * (1.0 / 9.0);
        }
      }
      __syncthreads();
      double* t = cur; cur = nxt; nxt = t;
    }
  }
  if (USE_LDS && variant == 2) {
    // One barrier per sweep: the centre source is folded into the sweep (T' = A (T + e_c) adds 1
    // to the 9-sums of the centre's 3x3 neighbourhood) instead of a separate write + barrier, and
    // a work item loads all DV+2 row sums of its segment at once (independent ds_reads in flight
    // instead of a DV-deep dependent chain).  Rows past the box clamp to its last (all-zero) ring
    // row, so every read stays inside T.
    const int cy = ce / RX, cx = ce % RX;
    for (int it = 0; it < niter; ++it) {
      for (int w = tid; w < nitems; w += MT) {
        const int x = 1 + w % (RX - 2);
        const int y0 = 1 + (w / (RX - 2)) * DV;
        const int nrow = RY - 1 - y0;  // >= 1 rows of this segment lie inside the box
        const double* c = cur + (y0 - 1) * RX + x;
        double h[DV + 2];
#pragma unroll
        for (int r = 0; r < DV + 2; ++r) {
          const double* cr = c + min(r, nrow + 1) * RX;
          h[r] = cr[-1] + cr[0] + cr[1];
        }
        const bool nearx = x - cx <= 1 && cx - x <= 1;
#pragma unroll
        for (int r = 0; r < DV; ++r) {
          if (r < nrow) {
            const int y = y0 + r;
            const int e = y * RX + x;
            double sum = h[r] + h[r + 1] + h[r + 2];
            if (nearx && y - cy <= 1 && cy - y <= 1) sum += 1.0;
            nxt[e] = inm[e] ? sum * (1.0 / 9.0) : 0.0;
          }
        }
      }
      __syncthreads();
      double* t = cur; cur = nxt; nxt = t;
    }
  }
  if (USE_LDS && variant == 1) {  // sliding-window sweep with the centre source folded in: one barrier
    const int cy = ce / RX, cx = ce % RX;
    for (int it = 0; it < niter; ++it) {
      for (int w = tid; w < nitems; w += MT) {
        const int x = 1 + w % (RX - 2);
        const int y0 = 1 + (w / (RX - 2)) * DV;
        const int y1 = min(y0 + DV, RY - 1);
        const bool nearx = x - cx <= 1 && cx - x <= 1;
        const double* c = cur + (y0 - 1) * RX + x;
        double hp = c[-1] + c[0] + c[1];
        c += RX;
        double hc = c[-1] + c[0] + c[1];
        for (int y = y0; y < y1; ++y) {
          c += RX;
          const double hn = c[-1] + c[0] + c[1];
          const int e = y * RX + x;
          double sum = hp + hc + hn;
          if (nearx && y - cy <= 1 && cy - y <= 1) sum += 1.0;
          nxt[e] = inm[e] ? sum * (1.0 / 9.0) : 0.0;
          hp = hc;
          hc = hn;
        }
      }
      __syncthreads();
      double* t = cur; cur = nxt; nxt = t;
    }
  }
  const bool dense0 = !sparse && (!USE_LDS || variant == 0 || variant == 3);  // 3 = variant 0 forced dense
  for (int it = 0; dense0 && it < niter; ++it) {
    if (tid == 0) cur[ce] += 1.0;
    __syncthreads();
    for (int w = tid; w < nitems; w += MT) {
      const int x = 1 + w % (RX - 2);
      const int y0 = 1 + (w / (RX - 2)) * DV;
      const int y1 = min(y0 + DV, RY - 1);
      const double* c = cur + (y0 - 1) * RX + x;
      double hp = c[-1] + c[0] + c[1];
      c += RX;
      double hc = c[-1] + c[0] + c[1];
      for (int y = y0; y < y1; ++y) {
        c += RX;
        const double hn = c[-1] + c[0] + c[1];
        const int e = y * RX + x;
        nxt[e] = inm[e] ? (hp + hc + hn) * (1.0 / 9.0) : 0.0;
        hp = hc;
        hc = hn;
      }
    }
    __syncthreads();
    double* t = cur; cur = nxt; nxt = t;
  }
  double* Lb = Lout + (size_t)J.b * H * W;
  for (int e = tid; e < R; e += MT) {
    if (!inm[e]) continue;
    const int y = J.y0 + e / RX - 1, x = J.x0 + e % RX - 1;
    Lb[y * W + x] = log1p(cur[e]);
  }
}

// ---------------------------------------------------------------------------------------------
// Masks too large for one workgroup's LDS: the Jacobi sweep of every big mask is split into
// DT_CORE x DT_CORE tiles, and the iterations are blocked in time — a workgroup stages its tile
// plus a DT_K-pixel halo in LDS, runs DT_K iterations on-chip (the valid region shrinks one pixel
// per step, so the core stays exact), and writes the core back.  Rounds are separated by a grid
// barrier (agent-scope release/acquire counter, bounded spin), so one cooperative launch runs all
// niter iterations of all big masks across the whole chip instead of one CU per mask.
#ifndef CP_DT_K
#define CP_DT_K 16
#endif
constexpr int DT_K = CP_DT_K;
constexpr int DT_CORE = 64 - 2 * DT_K;
constexpr int DT_RG = DT_CORE + 2 * DT_K;  // 64
constexpr int DT_LDS = 2 * DT_RG * DT_RG * 8 + DT_RG * DT_RG;
// threads per tile workgroup: the sweep is one column segment of DT_RG^2 / DT_MT rows per thread,
// so 1024 threads make a step ~4x shorter than 256 did (the big masks' tiled sweep is the critical
// path of flow QC on a few dozen CUs; the other CUs are busy with the LDS buckets meanwhile).
#ifndef CP_DT_MT
#define CP_DT_MT 1024
#endif
constexpr int DT_MT = CP_DT_MT;

__device__ __forceinline__ bool grid_barrier(unsigned* bar, unsigned target, unsigned* timeout_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ int ok;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    int good = 1;
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 24) || __hip_atomic_load(timeout_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        __hip_atomic_store(timeout_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        good = 0;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ok = good;
  }
  __syncthreads();
  return ok != 0;
}

// tiles: int4 {job, ry0, rx0, 0} (core origin in the job's padded box coordinates).
// bar[0] = arrival counter, bar[1] = timeout flag (both zeroed by the launcher).
__global__ __launch_bounds__(DT_MT) void diffuse_tiled_kernel(const int* __restrict__ M, const MaskJob* __restrict__ jobs,
                                                           int njobs, const int4* __restrict__ tiles, int ntiles, int H,
                                                           int W, const int* __restrict__ niter_img,
                                                           const int* __restrict__ centers, double* scratch,
                                                           double* __restrict__ Lout, unsigned* bar) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* A = reinterpret_cast<double*>(smem);
  double* Bf = A + DT_RG * DT_RG;
  unsigned char* mk = reinterpret_cast<unsigned char*>(Bf + DT_RG * DT_RG);
  const int tid = threadIdx.x;
  int maxn = 0;
  for (int j = 0; j < njobs; ++j) maxn = max(maxn, niter_img[jobs[j].b]);
  const int rounds = (maxn + DT_K - 1) / DT_K;
  for (int r = 0; r < rounds; ++r) {
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
      const int4 td = tiles[t];
      const MaskJob J = jobs[td.x];
      const int niter = niter_img[J.b];
      const int r0 = r * DT_K;
      if (r0 >= niter) continue;
      const int steps = min(DT_K, niter - r0);
      const bool last = r0 + steps == niter;
      const int RY = J.ly + 2, RX = J.lx + 2, R = RY * RX;
      double* cur = scratch + J.scratch + ((r & 1) ? R : 0);
      double* nxt = scratch + J.scratch + ((r & 1) ? 0 : R);
      const int oy = td.y - DT_K, ox = td.z - DT_K;  // region origin in box coordinates
      const int* Mb = M + (size_t)J.b * H * W;
      for (int e = tid; e < DT_RG * DT_RG; e += DT_MT) {
        const int ry = oy + e / DT_RG, rx = ox + e % DT_RG;
        unsigned char m = 0;
        double v = 0.0;
        if (ry >= 1 && ry <= J.ly && rx >= 1 && rx <= J.lx &&
            Mb[(J.y0 + ry - 1) * W + (J.x0 + rx - 1)] == J.lab) {
          m = 1;
          v = r == 0 ? 0.0 : cur[ry * RX + rx];
        }
        mk[e] = m;
        A[e] = v;
        Bf[e] = v;
      }
      const int ce = centers[td.x];
      const int cy = ce / RX - oy, cx = ce % RX - ox;
      const int cl = (cy >= 0 && cy < DT_RG && cx >= 0 && cx < DT_RG) ? cy * DT_RG + cx : -1;
      __syncthreads();
      double* a = A;
      double* b = Bf;
      // thread = one column x, rows [r0, r0 + 16): the whole region is swept every step (cells
      // outside the shrinking valid window turn to garbage that never reaches the core).
      const int x = tid & (DT_RG - 1);
      const int sr0 = (tid / DT_RG) * (DT_RG * DT_RG / DT_MT);
      const bool xl = x > 0, xr = x < DT_RG - 1;
      // centre source folded into the sweep (see diffuse_kernel): one barrier per step, and all
      // row sums of a thread's column segment are loaded before any is used
      constexpr int SEG = DT_RG * DT_RG / DT_MT;
      const bool nearx = x - cx <= 1 && cx - x <= 1;
      (void)cl;
      for (int s = 0; s < steps; ++s) {
        auto hsum = [&](int r) -> double {
          if (r < 0 || r >= DT_RG) return 0.0;
          const double* c = a + r * DT_RG + x;
          return (xl ? c[-1] : 0.0) + c[0] + (xr ? c[1] : 0.0);
        };
        double h[SEG + 2];
#pragma unroll
        for (int i = 0; i < SEG + 2; ++i) h[i] = hsum(sr0 - 1 + i);
#pragma unroll
        for (int i = 0; i < SEG; ++i) {
          const int y = sr0 + i;
          const int q = y * DT_RG + x;
          double sum = h[i] + h[i + 1] + h[i + 2];
          if (nearx && y - cy <= 1 && cy - y <= 1) sum += 1.0;
          b[q] = mk[q] ? sum * (1.0 / 9.0) : 0.0;
        }
        __syncthreads();
        double* tmp = a; a = b; b = tmp;
      }
      double* Lb = Lout + (size_t)J.b * H * W;
      for (int e = tid; e < DT_CORE * DT_CORE; e += DT_MT) {
        const int ly_ = DT_K + e / DT_CORE, lx_ = DT_K + e % DT_CORE;
        const int ry = oy + ly_, rx = ox + lx_;
        if (ry >= RY || rx >= RX) continue;
        const int q = ly_ * DT_RG + lx_;
        if (last) {
          if (mk[q]) Lb[(J.y0 + ry - 1) * W + (J.x0 + rx - 1)] = log1p(a[q]);
        } else {
          nxt[ry * RX + rx] = mk[q] ? a[q] : 0.0;
        }
      }
      __syncthreads();  // LDS reuse by the next tile of this round
    }
    if (r + 1 < rounds && !grid_barrier(bar, (unsigned)(r + 1) * gridDim.x, bar + 1)) return;
  }
}

// mu = normalised central-difference gradient of L inside masks; per-mask squared error vs dP/5.
// dp: optional [B, 2(or 3), H, W] network output (channel stride H*W, image stride dp_bstride).
__global__ __launch_bounds__(256) void flow_grad_kernel(const int* __restrict__ M, const double* __restrict__ L, int B, int H,
                                                        int W, float* __restrict__ mu, const float* __restrict__ dp,
                                                        long long dp_bstride, float* __restrict__ err, int nlab) {
  // FG_RUN consecutive pixels of one row per thread: the squared flow errors of a run of equal
  // labels are summed in registers and flushed with one atomic (was one atomic per mask pixel)
  const int WG = (W + FG_RUN - 1) / FG_RUN;
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int HW = H * W;
  if (gid >= (long long)B * H * WG) return;
  const int b = (int)(gid / ((long long)H * WG));
  const int rem = (int)(gid % ((long long)H * WG));
  const int y = rem / WG, x0 = (rem % WG) * FG_RUN;
  const double* Lb = L + (size_t)b * HW;
  const float* db = dp ? dp + (size_t)b * dp_bstride : nullptr;
  int run_lab = 0;
  float run = 0.f;
#pragma unroll
  for (int k = 0; k < FG_RUN; ++k) {
    const int x = x0 + k;
    if (x >= W) break;
    const int p = y * W + x;
    const int lab = M[(size_t)b * HW + p];
    float gy = 0.f, gx = 0.f;
    if (lab > 0) {
      const double up = y > 0 ? Lb[p - W] : 0.0, dn = y < H - 1 ? Lb[p + W] : 0.0;
      const double lf = x > 0 ? Lb[p - 1] : 0.0, rt = x < W - 1 ? Lb[p + 1] : 0.0;
      const double dgy = dn - up, dgx = rt - lf;
      const double nrm = sqrt(dgy * dgy + dgx * dgx) + 1e-60;
      gy = (float)(dgy / nrm);
      gx = (float)(dgx / nrm);
      if (db && err) {
        const float ey = gy - db[p] * 0.2f, ex = gx - db[HW + p] * 0.2f;
        if (lab != run_lab) {
          if (run_lab > 0) atomicAdd(err + (size_t)b * nlab + run_lab, run);
          run_lab = lab;
          run = 0.f;
        }
        run += ey * ey + ex * ex;
      }
    }
    if (mu) {
      mu[(size_t)b * 2 * HW + p] = gy;
      mu[(size_t)b * 2 * HW + HW + p] = gx;
    }
  }
  if (run_lab > 0) atomicAdd(err + (size_t)b * nlab + run_lab, run);
}

// Hole filling: background of the box (+1 ring) that is 4-connected to the ring is "outside";
// everything else in the box is the filled mask.  Writes lut[lab] into out (atomicMax for claimed
// hole pixels, plain for own pixels).  Masks with lut[lab] == 0 are skipped by the caller.
template <bool USE_LDS>
__global__ __launch_bounds__(MT) void fill_holes_kernel(const int* __restrict__ M, const MaskJob* __restrict__ jobs, int H,
                                                        int W, const int* __restrict__ lut, int nlab,
                                                        unsigned char* __restrict__ scratch, int* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const MaskJob J = jobs[blockIdx.x];
  const int RY = J.ly + 2, RX = J.lx + 2, R = RY * RX;
  unsigned char* st = USE_LDS ? smem : scratch + J.scratch;  // 0 = inside/undecided, 1 = mask, 2 = outside
  __shared__ int changed;
  const int tid = threadIdx.x;
  const int* Mb = M + (size_t)J.b * H * W;
  for (int e = tid; e < R; e += MT) {
    const int ry = e / RX, rx = e % RX;
    unsigned char v;
    if (ry == 0 || ry == RY - 1 || rx == 0 || rx == RX - 1) {
      v = 2;
    } else {
      v = (Mb[(J.y0 + ry - 1) * W + (J.x0 + rx - 1)] == J.lab) ? 1 : 0;
    }
    st[e] = v;
  }
  if (tid == 0) changed = 0;
  __syncthreads();
  for (;;) {
    int ch = 0;
    for (int e = tid; e < R; e += MT) {
      if (st[e] != 0) continue;
      const int ry = e / RX, rx = e % RX;
      if ((ry > 0 && st[e - RX] == 2) || (ry < RY - 1 && st[e + RX] == 2) || (rx > 0 && st[e - 1] == 2) ||
          (rx < RX - 1 && st[e + 1] == 2)) {
        st[e] = 2;
        ch = 1;
      }
    }
    if (ch) changed = 1;
    __syncthreads();
    const int c = changed;
    __syncthreads();  // everyone has read the flag before it is reset
    if (!c) break;
    if (tid == 0) changed = 0;
    __syncthreads();
  }
  const int newlab = lut[(size_t)J.b * nlab + J.lab];
  int* ob = out + (size_t)J.b * H * W;
  for (int e = tid; e < R; e += MT) {
    const unsigned char v = st[e];
    if (v == 2) continue;
    const int ry = e / RX, rx = e % RX;
    const int idx = (J.y0 + ry - 1) * W + (J.x0 + rx - 1);
    if (v == 1) {
      atomicMax(ob + idx, newlab);
    } else if (Mb[idx] == 0) {
      atomicMax(ob + idx, newlab);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Compact heat diffusion on one persistent work queue (flow QC and training targets, every mask
// of <= DQ_BCAP pixels).  The box-shaped kernels above keep the mask's whole bounding box in LDS,
// and the masks of the headline batch fill 14 % of their boxes (tools/mask_census.py), so most of
// their LDS and threads hold zeros; they also ran as six launches per batch on three streams, each
// with its own tail.  Here a mask is its pixel list only: raster-ordered ranks, heat values
// indexed by rank (+ one zero slot that stands for every non-mask neighbour), and per pixel the
// byte offsets of its 3x3 neighbours, found once by binary search over the sorted list and then
// kept in registers for all iterations.  Masks of <= 256 pixels are one WAVE's job (no barrier at
// all: the wave's LDS accesses are ordered), larger ones a workgroup's; each wave / workgroup
// pulls its next job from a global counter, so the chip stays full until the queue drains.
// Sums are formed in the sparse sweep's order (rows of 3, then the 3 row sums) and the centre
// source is stored as T + 1 at the centre (the dense sweep's cur[ce] += 1), the unshifted value
// kept in the owner's register: results are bit-identical to diffuse_kernel.
// DQ_T = 512 (default): 49 KiB per workgroup, workgroup jobs up to 2,048 pixels.  256 (A/B build)
// fits beside a pair-kernel workgroup on a CU but caps workgroup jobs at 1,024 pixels, and the
// masks above that went back to the box kernels: masks_to_flows 1.82 vs 0.96 ms, headline 1,902 /
// 1,951 vs 2,001 / 2,017 img/s (profiles/r05/masks/s29).
#ifndef DQ_T_BUILD
#define DQ_T_BUILD 512
#endif
constexpr int DQ_T = DQ_T_BUILD, DQ_K = 4;
#ifndef DQ_DPP
// 1: horizontal neighbours by DPP from the adjacent lanes (3 LDS reads per pixel instead of 9).
// Measured slower (s32: masks_to_flows 1.12 vs 0.97 ms, batch-1 2.03 vs 1.82 ms): the sweep is
// bound by its dependent latency, not LDS bandwidth, and the DPP moves + the divergent run-edge
// reads lengthen the chain.  Kept as an A/B build.
#define DQ_DPP 0
#endif
constexpr int DQ_WCAP = 64 * DQ_K, DQ_WHX = 256;   // wave jobs: pixels, box width + 2
constexpr int DQ_BCAP = DQ_T * DQ_K, DQ_BHX = 1024;  // workgroup jobs
template <int CAP, int HX>
struct DQL {
  static constexpr int T_B = 2 * (CAP + 1) * 8;  // two heat buffers, slot CAP = the zero slot
  static constexpr int BYTES = T_B + CAP * 4 + HX * 4 + 64;
};
using DQW = DQL<DQ_WCAP, DQ_WHX>;
using DQB = DQL<DQ_BCAP, DQ_BHX>;
constexpr int DQ_NWV = DQ_T / 64;  // waves (wave-job slots) per workgroup
constexpr int DQ_LDS = DQ_NWV * DQW::BYTES > DQB::BYTES ? DQ_NWV * DQW::BYTES : DQB::BYTES;
static_assert((DQ_T == 256 || DQ_T == 512) && DQW::BYTES % 16 == 0 && DQ_LDS <= 64 * 1024, "diffuse queue LDS layout");

// lane l <- lane l - 1 (prev) / l + 1 (next) of a double, across the whole wave (DPP wave_shr /
// wave_shl: VALU, no LDS traffic); the end lanes get 0
__device__ __forceinline__ double dq_from_prev(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x138, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x138, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double dq_from_next(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x130, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x130, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// smallest bin i with sum(h[0..i]) > k (one wave)
__device__ __forceinline__ int dq_kth(const int* h, int n, int k, int lane) {
  int acc = 0;
  for (int b0 = 0; b0 < n; b0 += 64) {
    int inc = b0 + lane < n ? h[b0 + lane] : 0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(inc, o, 64);
      if (lane >= o) inc += u;
    }
    const unsigned long long bal = __ballot(acc + inc > k);
    if (bal) return b0 + __ffsll((unsigned long long)bal) - 1;
    acc += __shfl(inc, 63, 64);
  }
  return n - 1;
}

template <int NTH, int CAP, int HX>
__device__ __forceinline__ void dq_job(const MaskJob& J, const int* __restrict__ M, int H, int W,
                                       const int* __restrict__ niter_img, double* __restrict__ Lout, unsigned char* lds,
                                       int t) {
  constexpr int K = CAP / NTH;
  double* T0 = reinterpret_cast<double*>(lds);
  double* T1 = T0 + CAP + 1;
  int* list = reinterpret_cast<int*>(T1 + CAP + 1);
  int* hx = list + CAP;
  unsigned long long* best = reinterpret_cast<unsigned long long*>(hx + HX);
  float* med = reinterpret_cast<float*>(best + 1);
  int* wc = reinterpret_cast<int*>(med + 2);  // NTH / 64 wave counts (workgroup jobs)
  auto sync = [&]() {
    if constexpr (NTH == 64) {  // one wave: its LDS accesses complete in order; compiler ordering only
      asm volatile("" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    } else {
      __syncthreads();
    }
  };
  const int lane = t & 63;
  const int RX = J.lx + 2;
  const int ncell = J.ly * J.lx;
  const int* Mb = M + (size_t)J.b * H * W;
  for (int i = t; i < RX; i += NTH) hx[i] = 0;
  if (t == 0) *best = ~0ull;
  sync();
  // the mask's pixels in raster order (ranks = ballot prefix counts), x histogram for the median
  int P = 0;
  for (int c0 = 0; c0 < ncell; c0 += NTH) {
    const int c = c0 + t;
    int cy = 0, cx = 0;
    bool m = false;
    if (c < ncell) {
      cy = c / J.lx;
      cx = c - cy * J.lx;
      m = Mb[(size_t)(J.y0 + cy) * W + J.x0 + cx] == J.lab;
    }
    const unsigned long long bal = __ballot(m);
    int rank = __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
    int tot = __popcll(bal);
    if constexpr (NTH > 64) {
      if (lane == 0) wc[t >> 6] = tot;
      sync();
      int pre = 0;
      tot = 0;
#pragma unroll
      for (int w = 0; w < NTH / 64; ++w) {
        const int x = wc[w];
        pre += w < (t >> 6) ? x : 0;
        tot += x;
      }
      rank += pre;
    }
    if (m && P + rank < CAP) {
      list[P + rank] = (cy + 1) * RX + cx + 1;
      atomicAdd(&hx[cx + 1], 1);
    }
    P += tot;
    if constexpr (NTH > 64) sync();  // wc is rewritten by the next chunk
  }
  P = min(P, CAP);  // (the planner sized the job from the exact pixel count)
  sync();
  if (P == 0) return;
  // exact medians in padded-box coordinates (numpy: mean of the two middle values); the list is
  // raster-ordered, so its ry are sorted
  if (t < 64) {
    const int k1 = (P - 1) / 2, k2 = P / 2;
    const int y1 = list[k1] / RX, y2 = list[k2] / RX;
    const int x1 = dq_kth(hx, RX, k1, lane), x2 = dq_kth(hx, RX, k2, lane);
    if (lane == 0) {
      med[0] = 0.5f * (float)(y1 + y2);
      med[1] = 0.5f * (float)(x1 + x2);
    }
  }
  sync();
  int myr[K], off[K][9];
  bool own[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const int r = t + j * NTH;
    own[j] = r < P;
    myr[j] = own[j] ? r : CAP;
    if (own[j]) {
      const int e = list[r];
      const float dy = (float)(e / RX) - med[0], dx = (float)(e % RX) - med[1];
      const float d = dx * dx + dy * dy;  // exact: half-integer coordinates
      atomicMin(best, ((unsigned long long)__float_as_uint(d) << 32) | (unsigned)r);  // ties: raster order
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        if (k == 4) { off[j][k] = r * 8; continue; }
        const int e2 = e + (k / 3 - 1) * RX + (k % 3 - 1);
        int lo = 0, hi = P;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (list[mid] < e2) lo = mid + 1;
          else hi = mid;
        }
        off[j][k] = (lo < P && list[lo] == e2 ? lo : CAP) * 8;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 9; ++k) off[j][k] = CAP * 8;
    }
  }
  for (int i = t; i < P; i += NTH) { T0[i] = 0.0; T1[i] = 0.0; }
  if (t == 0) { T0[CAP] = 0.0; T1[CAP] = 0.0; }
  sync();
  const int cidx = (int)(*best & 0xffffffffu);
  if (t == 0) T0[cidx] = 1.0;  // S = T + e_c: the centre source of the first sweep
  sync();
  // DQ_DPP builds: horizontal neighbours from the adjacent lanes: ranks are raster-ordered and lane l - 1 of the
  // same slot holds rank r - 1, so when the left pixel is rank r - 1 the left column (up-left,
  // left, down-left) is exactly lane l - 1's own column, which it reads anyway; likewise on the
  // right.  A sweep then reads 3 values per pixel from LDS (its column) and takes the other 6 by
  // DPP, reading them itself only where a row run starts or ends (or at the wave's end lanes).
  // The 9 values and the order they are summed in are unchanged.
  bool lok[K], rok[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    lok[j] = own[j] && lane > 0 && off[j][3] == (myr[j] - 1) * 8;
    rok[j] = own[j] && lane < 63 && off[j][5] == (myr[j] + 1) * 8;
  }
  const int niter = niter_img[J.b];
  const int nsl = (P + NTH - 1) / NTH;  // slots in use (uniform)
  double* cur = T0;
  double* nxt = T1;
  double tc = 0.0;  // the centre's own (unshifted) value, in its owner's register
  for (int it = 0; it < niter; ++it) {
    const unsigned char* cb = reinterpret_cast<const unsigned char*>(cur);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (j < nsl) {
        double v[9];
        v[1] = *reinterpret_cast<const double*>(cb + off[j][1]);
        v[4] = *reinterpret_cast<const double*>(cb + off[j][4]);
        v[7] = *reinterpret_cast<const double*>(cb + off[j][7]);
        const double l1 = dq_from_prev(v[1]), l4 = dq_from_prev(v[4]), l7 = dq_from_prev(v[7]);
        const double r1 = dq_from_next(v[1]), r4 = dq_from_next(v[4]), r7 = dq_from_next(v[7]);
        if (DQ_DPP && lok[j]) {
          v[0] = l1; v[3] = l4; v[6] = l7;
        } else {
          v[0] = *reinterpret_cast<const double*>(cb + off[j][0]);
          v[3] = *reinterpret_cast<const double*>(cb + off[j][3]);
          v[6] = *reinterpret_cast<const double*>(cb + off[j][6]);
        }
        if (DQ_DPP && rok[j]) {
          v[2] = r1; v[5] = r4; v[8] = r7;
        } else {
          v[2] = *reinterpret_cast<const double*>(cb + off[j][2]);
          v[5] = *reinterpret_cast<const double*>(cb + off[j][5]);
          v[8] = *reinterpret_cast<const double*>(cb + off[j][8]);
        }
        const double hp = v[0] + v[1] + v[2];
        const double hc = v[3] + v[4] + v[5];
        const double hn = v[6] + v[7] + v[8];
        const double tn = (hp + hc + hn) * (1.0 / 9.0);
        const bool isc = myr[j] == cidx;
        if (isc) tc = tn;
        if (own[j]) nxt[myr[j]] = isc ? tn + 1.0 : tn;
      }
    }
    sync();
    double* tt = cur; cur = nxt; nxt = tt;
  }
  double* Lb = Lout + (size_t)J.b * H * W;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    if (!own[j]) continue;
    const int e = list[myr[j]];
    const int ry = e / RX, rx = e - ry * RX;
    const double val = myr[j] == cidx ? tc : cur[myr[j]];
    Lb[(size_t)(J.y0 + ry - 1) * W + (J.x0 + rx - 1)] = log1p(val);
  }
  sync();  // the LDS slot is reused by the next job
}

// q[0] / q[1]: workgroup / wave job cursors (zeroed by the launcher).  Workgroup jobs first (all
// waves), then every wave drains the wave-job queue on its own; every wave exits once both cursors
// pass their counts.
__global__ __launch_bounds__(DQ_T) void diffuse_q_kernel(const int* __restrict__ M, const MaskJob* __restrict__ wjobs,
                                                         int nw, const MaskJob* __restrict__ bjobs, int nb, int H, int W,
                                                         const int* __restrict__ niter_img, double* __restrict__ Lout,
                                                         unsigned* __restrict__ q) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int sj;
  const int t = threadIdx.x;
  for (;;) {
    if (t == 0) sj = (int)atomicAdd(q, 1u);
    __syncthreads();
    const int j = sj;
    __syncthreads();
    if (j >= nb) break;
    const MaskJob J = bjobs[j];
    dq_job<DQ_T, DQ_BCAP, DQ_BHX>(J, M, H, W, niter_img, Lout, smem, t);
  }
  const int lane = t & 63;
  unsigned char* slot = smem + (t >> 6) * DQW::BYTES;
  for (;;) {
    int j = 0;
    if (lane == 0) j = (int)atomicAdd(q + 1, 1u);
    j = __builtin_amdgcn_readfirstlane(__shfl(j, 0, 64));
    if (j >= nw) break;
    const MaskJob J = wjobs[j];
    dq_job<64, DQ_WCAP, DQ_WHX>(J, M, H, W, niter_img, Lout, slot, lane);
  }
}

// Hole filling of a mask whose box (+1 ring) fits NS * 64 rows x NWD * 64 columns: one WAVE, no
// LDS, no barriers.  Box row r lives in lane r % 64, slot r / 64, as NWD 64-bit words (bit x of the
// row = column x); "outside" grows from the ring through the cells that are not this label: within
// a row by carry propagation (adding the seed bits to the row's free bits clears every free run
// upward of a seed, carrying across words; the bit-reversed sum does the same downward), across
// rows through the neighbour lanes, until no lane changes.  Same 4-connectivity and writes as
// fill_holes_kernel (which keeps the larger boxes).  <1, 1>: boxes <= 64 x 64 (nearly all masks);
// <4, 2>: <= 256 rows x 128 columns (the long tail the one-workgroup LDS kernel spent 0.44 ms on).
template <int NS, int NWD>
__global__ __launch_bounds__(256) void fill_holes_bits_kernel(const int* __restrict__ M, const MaskJob* __restrict__ jobs,
                                                              int njobs, int H, int W, const int* __restrict__ lut, int nlab,
                                                              int* __restrict__ out) {
  using u64 = unsigned long long;
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= njobs) return;  // wave-uniform
  const MaskJob J = jobs[j];
  const int RY = J.ly + 2, RX = J.lx + 2;
  const int* Mb = M + (size_t)J.b * H * W;
  u64 full[NWD];
#pragma unroll
  for (int w = 0; w < NWD; ++w) {
    const int nbits = min(max(RX - 64 * w, 0), 64);
    full[w] = nbits >= 64 ? ~0ull : ((1ull << nbits) - 1ull);
  }
  u64 mrow[NS][NWD];
#pragma unroll
  for (int k = 0; k < NS; ++k)
#pragma unroll
    for (int w = 0; w < NWD; ++w) mrow[k][w] = 0ull;
  // rows in batches of 8: the 8 x NWD loads of a batch are in flight together (a tall box loaded
  // row by row waited for each load before the next)
  for (int r0 = 1; r0 <= J.ly; r0 += 8) {
    bool mv[8][NWD];
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int w = 0; w < NWD; ++w) {
        const int r = r0 + q, col = 64 * w + lane;
        mv[q][w] = r <= J.ly && col >= 1 && col <= J.lx && Mb[(size_t)(J.y0 + r - 1) * W + J.x0 + col - 1] == J.lab;
      }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int r = r0 + q;
#pragma unroll
      for (int w = 0; w < NWD; ++w) {
        const u64 bal = __ballot(mv[q][w]);
#pragma unroll
        for (int k = 0; k < NS; ++k)
          if (k == (r >> 6) && lane == (r & 63)) mrow[k][w] = bal;
      }
    }
  }
  u64 fr[NS][NWD], o[NS][NWD];
  const int wl = (RX - 1) >> 6;  // word of the last column
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    const int row = 64 * k + lane;
    const bool rowin = row < RY;
    const bool ringrow = row == 0 || row == RY - 1;
#pragma unroll
    for (int w = 0; w < NWD; ++w) {
      fr[k][w] = rowin ? (~mrow[k][w] & full[w]) : 0ull;
      u64 ring = ringrow ? full[w] : 0ull;
      if (w == 0) ring |= 1ull;
      if (w == wl) ring |= 1ull << ((RX - 1) & 63);
      o[k][w] = ring & fr[k][w];
    }
  }
  for (;;) {
    u64 h[NS][NWD];
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      u64 up[NWD], dn[NWD], rf[NWD], ro[NWD];
      unsigned long long carry = 0ull;
#pragma unroll
      for (int w = 0; w < NWD; ++w) {  // multi-word add fr + o
        const u64 t = fr[k][w] + o[k][w];
        const u64 sum = t + carry;
        carry = (t < fr[k][w]) || (sum < t) ? 1ull : 0ull;
        up[w] = fr[k][w] & ~sum;
      }
#pragma unroll
      for (int w = 0; w < NWD; ++w) {  // bit reversal of the whole row (word order swapped)
        rf[w] = __builtin_bitreverse64(fr[k][NWD - 1 - w]);
        ro[w] = __builtin_bitreverse64(o[k][NWD - 1 - w]);
      }
      carry = 0ull;
#pragma unroll
      for (int w = 0; w < NWD; ++w) {
        const u64 t = rf[w] + ro[w];
        const u64 sum = t + carry;
        carry = (t < rf[w]) || (sum < t) ? 1ull : 0ull;
        dn[NWD - 1 - w] = __builtin_bitreverse64(rf[w] & ~sum);
      }
#pragma unroll
      for (int w = 0; w < NWD; ++w) h[k][w] = o[k][w] | up[w] | dn[w];
    }
    bool ch = false;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
#pragma unroll
      for (int w = 0; w < NWD; ++w) {
        u64 above = __shfl_up(h[k][w], 1, 64), below = __shfl_down(h[k][w], 1, 64);
        if (k > 0) {
          const u64 prev = __shfl(h[k > 0 ? k - 1 : 0][w], 63, 64);
          if (lane == 0) above = prev;
        }
        if (k + 1 < NS) {
          const u64 next = __shfl(h[k + 1 < NS ? k + 1 : k][w], 0, 64);
          if (lane == 63) below = next;
        }
        const u64 n = h[k][w] | ((above | below) & fr[k][w]);
        ch |= n != o[k][w];
        o[k][w] = n;
      }
    }
    if (!__any(ch)) break;
  }
  const int newlab = lut[(size_t)J.b * nlab + J.lab];
  int* ob = out + (size_t)J.b * H * W;
  for (int r = 1; r <= J.ly; ++r) {
#pragma unroll
    for (int w = 0; w < NWD; ++w) {
      u64 iv = 0ull, mv = 0ull;
#pragma unroll
      for (int k = 0; k < NS; ++k)
        if (k == (r >> 6)) { iv = ~o[k][w] & full[w]; mv = mrow[k][w]; }
      const u64 in_r = __shfl(iv, r & 63, 64), m_r = __shfl(mv, r & 63, 64);
      const int col = 64 * w + lane;
      if (col >= 1 && col <= J.lx && ((in_r >> lane) & 1ull)) {
        const size_t idx = (size_t)(J.y0 + r - 1) * W + J.x0 + col - 1;
        if (((m_r >> lane) & 1ull) || Mb[idx] == 0) atomicMax(ob + idx, newlab);
      }
    }
  }
}

// LDS variant with a block size matched to the masks (the launcher buckets small masks by their
// LDS need, so a 20x20 mask no longer reserves the 48 KiB of the largest one).  dv = rows per work
// item of the sliding-window sweep: 4 gives each mask twice the lanes and half the serial LDS
// chain per iteration of 8 (the sweep is latency-bound: SQ_WAIT_ANY 45-67 % of wave cycles).
template <int T, int DV>
static void launch_diffuse_nt(const int* M, const void* jobs, int njobs, int H, int W, const int* niter_img, double* Lout,
                              int lds_bytes, int variant, hipStream_t s) {
  if (lds_bytes > 64 * 1024) {  // > 64 KiB of dynamic LDS (up to the 160 KiB of a CU) needs the opt-in
    static int attr[BE_MAX_DEV] = {};
    if (attr[be_cur_dev()] < lds_bytes) {
      const hipError_t ae = hipFuncSetAttribute(reinterpret_cast<const void*>(diffuse_kernel<true, T, DV>),
                                                hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
      if (ae != hipSuccess) fprintf(stderr, "be_cp_diffuse_nt: hipFuncSetAttribute(%d): %s\n", lds_bytes, hipGetErrorString(ae));
      attr[be_cur_dev()] = lds_bytes;
    }
  }
  hipLaunchKernelGGL((diffuse_kernel<true, T, DV>), dim3(njobs), dim3(T), lds_bytes, s, M, (const MaskJob*)jobs, H, W,
                     niter_img, nullptr, Lout, nullptr, variant);
}

}  // namespace

extern "C" {

int be_cp_bbox(const int* M, int B, int H, int W, int nlab, int* bbox, hipStream_t s) {
  const long long n = (long long)B * H * ((W + RL - 1) / RL);
  hipLaunchKernelGGL(bbox_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, M, B, H, W, nlab, bbox);
  return BE_CHECK_LAUNCH();
}

// jobs: device array of MaskJob (7 x int64-aligned fields: see struct); lds_bytes > 0 => LDS variant.
int be_cp_diffuse(const int* M, const void* jobs, int njobs, int H, int W, const int* niter_img, double* scratch,
                  double* Lout, int lds_bytes, hipStream_t s) {
  if (njobs == 0) return 0;
  if (lds_bytes > 0)
    hipLaunchKernelGGL((diffuse_kernel<true>), dim3(njobs), dim3(MT), lds_bytes, s, M, (const MaskJob*)jobs, H, W, niter_img,
                       scratch, Lout, nullptr);
  else
    hipLaunchKernelGGL((diffuse_kernel<false>), dim3(njobs), dim3(MT), 0, s, M, (const MaskJob*)jobs, H, W, niter_img, scratch,
                       Lout, nullptr);
  return BE_CHECK_LAUNCH();
}

// Big masks the sparse sweep can take (plan bucket ncap): one 1024-thread workgroup per mask, heat
// field in global scratch (L2-resident: a box of R cells holds 16 R bytes), SP_K pixels per thread.
int be_cp_diffuse_sparse_big(const int* M, const void* jobs, int njobs, int H, int W, const int* niter_img,
                             double* scratch, double* Lout, hipStream_t s) {
  if (njobs == 0) return 0;
  hipLaunchKernelGGL((diffuse_kernel<false, 1024, 4>), dim3(njobs), dim3(1024), 0, s, M, (const MaskJob*)jobs, H, W,
                     niter_img, scratch, Lout, nullptr, 0);
  return BE_CHECK_LAUNCH();
}

int be_cp_diffuse_nt(const int* M, const void* jobs, int njobs, int H, int W, const int* niter_img, double* Lout,
                     int lds_bytes, int threads, int dv, hipStream_t s) {
  if (njobs == 0) return 0;
  if (lds_bytes <= 0) return -1;
  // sweep variant (A/B switch, read per call): 0 = sparse pixel-list sweep where it fits (see
  // diffuse_kernel), else source write + 2 barriers per iteration; 1 = source folded into the
  // sliding-window sweep, 2 = folded + all row loads issued together; 3 = variant 0 always dense
  const char* ev = getenv("BE_DIFFUSE_VARIANT");
  const int variant = ev ? atoi(ev) : kDiffuseVariant;
#define BE_DNT(T, D)                                                                                   \
  if (threads == T && dv == D) {                                                                     \
    launch_diffuse_nt<T, D>(M, jobs, njobs, H, W, niter_img, Lout, lds_bytes, variant, s);           \
  } else
  BE_DNT(64, 8) BE_DNT(128, 8) BE_DNT(256, 8) BE_DNT(512, 8) BE_DNT(1024, 8)
  BE_DNT(64, 4) BE_DNT(128, 4) BE_DNT(256, 4) BE_DNT(512, 4) BE_DNT(1024, 4)
  BE_DNT(64, 2) BE_DNT(128, 2) BE_DNT(256, 2) BE_DNT(512, 2) BE_DNT(1024, 2)
  return -2;
#undef BE_DNT
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    fprintf(stderr, "be_cp_diffuse_nt(njobs=%d, lds=%d, threads=%d, dv=%d): %s\n", njobs, lds_bytes, threads, dv,
            hipGetErrorString(e));
  return (int)e;
}

// Compact work-queue diffusion (see diffuse_q_kernel): wjobs = masks of <= 256 pixels with box
// width + 2 <= 256, bjobs = <= 2048 pixels, box width + 2 <= 1024 (plan kind 2 buckets 0 / 1);
// q: >= 8 bytes of device memory (the two job cursors).
int be_cp_diffuse_q(const int* M, const void* wjobs, int nw, const void* bjobs, int nb, int H, int W, const int* niter_img,
                    double* Lout, unsigned* q, hipStream_t s) {
  if (nw + nb == 0) return 0;
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu <= 0) ncu = 256;
  }
  const int want = max(nb, (nw + DQ_NWV - 1) / DQ_NWV);
  const int grid = max(1, min(want, (DQ_T == 256 ? 6 : 3) * ncu));  // LDS: 25 / 49 KiB per workgroup
  (void)hipMemsetAsync(q, 0, 8, s);
  hipLaunchKernelGGL(diffuse_q_kernel, dim3(grid), dim3(DQ_T), DQ_LDS, s, M, (const MaskJob*)wjobs, nw,
                     (const MaskJob*)bjobs, nb, H, W, niter_img, Lout, q);
  return BE_CHECK_LAUNCH();
}

int be_cp_diffuse_q_caps(int* out4) {
  out4[0] = DQ_WCAP;
  out4[1] = DQ_WHX;
  out4[2] = DQ_BCAP;
  out4[3] = DQ_BHX;
  return 0;
}

int be_cp_diffuse_tile_params(int* out3) {
  out3[0] = DT_CORE;
  out3[1] = DT_K;
  out3[2] = DT_LDS;
  return 0;
}

// Big masks, multi-workgroup: centres (one block per mask), then one cooperative launch for all
// iterations.  tiles: int4 per tile (see diffuse_tiled_kernel); ws: >= 16 bytes of device memory
// (barrier counter + timeout flag); centers: njobs ints.  Returns 1 if the barrier timed out.
// stages: bit 0 = the per-mask centre kernel, bit 1 = the cooperative tiled sweep (the caller can
// start other streams' work between the two, once the short centre kernel is queued).
int be_cp_diffuse_tiled(const int* M, const void* jobs, int njobs, const void* tiles, int ntiles, int H, int W,
                        const int* niter_img, double* scratch, double* Lout, int* centers, unsigned* ws, int stages,
                        hipStream_t s) {
  if (njobs == 0 || ntiles == 0) return 0;
  if (stages & 1) {
    hipLaunchKernelGGL((diffuse_kernel<false>), dim3(njobs), dim3(MT), 0, s, M, (const MaskJob*)jobs, H, W, niter_img,
                       scratch, Lout, centers);
    if (BE_CHECK_LAUNCH()) return -1;
  }
  if (!(stages & 2)) return 0;
  static int max_grid = 0;
  if (max_grid == 0) {
    int dev = 0, ncu = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(diffuse_tiled_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                        DT_LDS);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(diffuse_tiled_kernel), DT_MT,
                                                 DT_LDS);
    max_grid = max(1, ncu * max(1, per_cu));
  }
  const int grid = min(ntiles, max_grid);
  (void)hipMemsetAsync(ws, 0, 16, s);
  const MaskJob* jp = (const MaskJob*)jobs;
  const int4* tp = (const int4*)tiles;
  void* args[] = {(void*)&M, (void*)&jp, (void*)&njobs, (void*)&tp, (void*)&ntiles, (void*)&H, (void*)&W,
                  (void*)&niter_img, (void*)&centers, (void*)&scratch, (void*)&Lout, (void*)&ws};
  hipError_t e = hipLaunchCooperativeKernel(reinterpret_cast<const void*>(diffuse_tiled_kernel), dim3(grid), dim3(DT_MT),
                                            args, DT_LDS, s);
  if (e != hipSuccess) {
    fprintf(stderr, "be_cp_diffuse_tiled: cooperative launch failed: %s\n", hipGetErrorString(e));
    return -2;
  }
  return 0;
}

int be_cp_flow_grad(const int* M, const double* L, int B, int H, int W, float* mu, const float* dp, long long dp_bstride,
                    float* err, int nlab, hipStream_t s) {
  const long long n = (long long)B * H * ((W + FG_RUN - 1) / FG_RUN);
  hipLaunchKernelGGL(flow_grad_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, M, L, B, H, W, mu, dp, dp_bstride,
                     err, nlab);
  return BE_CHECK_LAUNCH();
}

int be_cp_fill_holes(const int* M, const void* jobs, int njobs, int H, int W, const int* lut, int nlab, void* scratch,
                     int* out, int lds_bytes, hipStream_t s) {
  if (njobs == 0) return 0;
  if (lds_bytes > 0)
    hipLaunchKernelGGL((fill_holes_kernel<true>), dim3(njobs), dim3(MT), lds_bytes, s, M, (const MaskJob*)jobs, H, W, lut, nlab,
                       (unsigned char*)scratch, out);
  else
    hipLaunchKernelGGL((fill_holes_kernel<false>), dim3(njobs), dim3(MT), 0, s, M, (const MaskJob*)jobs, H, W, lut, nlab,
                       (unsigned char*)scratch, out);
  return BE_CHECK_LAUNCH();
}

// One-wave hole filling (plan kind 3): big = 0: boxes (+ ring) <= 64 x 64 (bucket 0), big = 1:
// <= 256 rows x 128 columns (bucket 1).  4 waves per workgroup.
int be_cp_fill_holes_wave(const int* M, const void* jobs, int njobs, int H, int W, const int* lut, int nlab, int* out,
                          int big, hipStream_t s) {
  if (njobs == 0) return 0;
  const dim3 g((unsigned)((njobs + 3) / 4));
  if (big)
    hipLaunchKernelGGL((fill_holes_bits_kernel<4, 2>), g, dim3(256), 0, s, M, (const MaskJob*)jobs, njobs, H, W, lut, nlab, out);
  else
    hipLaunchKernelGGL((fill_holes_bits_kernel<1, 1>), g, dim3(256), 0, s, M, (const MaskJob*)jobs, njobs, H, W, lut, nlab, out);
  return BE_CHECK_LAUNCH();
}

int be_cp_mask_job_bytes() { return (int)sizeof(MaskJob); }

// Job planning for the per-mask kernels in one launch (replaces ~80 small torch ops and their host
// gaps): every (image, label) with a box and (optional) valid[] flag computes its LDS need,
// picks the first bucket with caps[k] >= need (k = ncap: too big for LDS -> scratch offset from
// an atomic cursor), and appends its MaskJob to jobs[k][slot].  kind 0 = diffusion (need =
// 16R + 4(RY+RX) + R + 16 bytes, scratch = the fp64 slab of _diffuse_scratch_doubles), kind 1 =
// hole filling (need = R bytes, scratch = R bytes).  niter_img[b] (kind 0) = 2 * max over the
// image's masks of (ly + lx + 4), cellpose's per-image iteration count.
// counts: [ncap + 1] (+1 with cnts) int32 zeroed; scratch_total: int64 zeroed; niter_img: [B] int32 zeroed.
int be_cp_plan_masks(const int* bbox, const unsigned char* valid, const int* cnts, int B, int nlab, int kind,
                     const int* caps, int ncap, long long* jobs, int* counts, long long* scratch_total, int* niter_img,
                     hipStream_t s);
}  // extern "C"

namespace {
struct Caps8 {
  int v[8];
};

__global__ __launch_bounds__(256) void plan_masks_kernel(const int* __restrict__ bbox, const unsigned char* __restrict__ valid,
                                                         const int* __restrict__ cnts,
                                                         int B, int nlab, int kind, Caps8 caps, int ncap,
                                                         MaskJob* __restrict__ jobs, int* __restrict__ counts,
                                                         unsigned long long* __restrict__ scratch_total,
                                                         int* __restrict__ niter_img) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long n = (long long)B * nlab;
  if (i >= n) return;
  const int b = (int)(i / nlab), lab = (int)(i % nlab);
  const int* bb = bbox + i * 4;
  const int y0 = bb[0], y1 = bb[1], x0 = bb[2], x1 = bb[3];
  if (lab == 0 || y1 < 0) return;
  const int ly = y1 - y0 + 1, lx = x1 - x0 + 1;
  // kind 2 = kind 0 with the compact work-queue buckets in front: 0 = wave jobs, 1 = workgroup
  // jobs (diffuse_q_kernel), 2.. = kind 0's buckets for the masks those cannot take
  // kind 3 = kind 1 with the one-wave hole-filling buckets in front: 0 = box + ring <= 64 x 64,
  // 1 = <= 256 rows x 128 columns
  const int q2 = kind == 2 ? 2 : (kind == 3 ? 2 : 0);
  if (kind == 2) kind = 0;
  if (kind == 3) {
    kind = 1;
    const int kw = (ly + 2 <= 64 && lx + 2 <= 64) ? 0 : ((ly + 2 <= 256 && lx + 2 <= 128) ? 1 : -1);
    if (!(valid && !valid[i]) && kw >= 0) {
      const int slot = atomicAdd(counts + kw, 1);
      MaskJob J;
      J.b = b; J.lab = lab; J.y0 = y0; J.x0 = x0; J.ly = ly; J.lx = lx; J.scratch = -1;
      jobs[(size_t)kw * n + slot] = J;
      return;
    }
  }
  if (kind == 0) atomicMax(niter_img + b, 2 * (ly + lx + 2));  // 2 * ((y1-y0)+(x1-x0)+4)
  if (valid && !valid[i]) return;
  const long long RY = ly + 2, RX = lx + 2, R = RY * RX;
  const long long need = kind == 0 ? 16 * R + 4 * (RY + RX) + R + 16 : R;
  int k = 0;
  if (q2 && cnts) {
    const long long c = cnts[i];
    int kq = -1;
    if (c <= DQ_WCAP && RX <= DQ_WHX) kq = 0;
    else if (c <= DQ_BCAP && RX <= DQ_BHX) kq = 1;
    if (kq >= 0) {
      const int slot = atomicAdd(counts + kq, 1);
      MaskJob J;
      J.b = b; J.lab = lab; J.y0 = y0; J.x0 = x0; J.ly = ly; J.lx = lx; J.scratch = -1;
      jobs[(size_t)kq * n + slot] = J;
      return;
    }
  }
  while (k < ncap && need > caps.v[k]) ++k;
  // kind 0 with pixel counts: a too-big-for-LDS mask that the sparse sweep can take (box fill
  // < 60 %, <= SPARSE_BIG_PX pixels) goes to bucket ncap (one workgroup, heat field in global
  // scratch), the rest to bucket ncap + 1 (the tiled multi-workgroup kernel)
  if (k == ncap && kind == 0 && cnts) {
    const long long c = cnts[i];
    if (!(c * 5 < R * 3 && c <= SPARSE_BIG_PX)) k = ncap + 1;
  }
  long long scr = -1;
  if (k >= ncap) {
    const long long sz = kind == 0 ? 2 * R + (RY + RX + 1) / 2 + (R + 7) / 8 + 2 : R;
    scr = (long long)atomicAdd(scratch_total, (unsigned long long)sz);
  }
  k += q2;
  const int slot = atomicAdd(counts + k, 1);
  MaskJob J;
  J.b = b;
  J.lab = lab;
  J.y0 = y0;
  J.x0 = x0;
  J.ly = ly;
  J.lx = lx;
  J.scratch = scr;
  jobs[(size_t)k * n + slot] = J;
}
}  // namespace

extern "C" {
// cnts (optional, kind 0): per-label pixel counts [B, nlab]; with it the jobs form ncap + 2 buckets
// (LDS caps..., big-sparse, tiled) instead of ncap + 1.
int be_cp_plan_masks(const int* bbox, const unsigned char* valid, const int* cnts, int B, int nlab, int kind,
                     const int* caps, int ncap, long long* jobs, int* counts, long long* scratch_total, int* niter_img,
                     hipStream_t s) {
  if (ncap < 0 || ncap > 8) return -1;
  Caps8 c{};
  for (int k = 0; k < ncap; ++k) c.v[k] = caps[k];  // host array
  const long long n = (long long)B * nlab;
  if (n == 0) return 0;
  hipLaunchKernelGGL(plan_masks_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, bbox, valid, cnts, B, nlab, kind, c,
                     ncap, reinterpret_cast<MaskJob*>(jobs), counts, reinterpret_cast<unsigned long long*>(scratch_total),
                     niter_img);
  return BE_CHECK_LAUNCH();
}

}  // extern "C"

// Pixel count per label (label 0 skipped, so background never contends on one counter).
namespace {
// Run-length form: RL consecutive pixels per thread (segments never straddle images), one atomic
// per run of equal labels.
__global__ __launch_bounds__(256) void label_counts_kernel(const int* __restrict__ M, long long n, int HW, int nlab,
                                                           int* __restrict__ counts) {
  const int segs = (HW + RL - 1) / RL;
  const long long nseg = (n / HW) * segs;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x; g < nseg; g += stride) {
    const long long b = g / segs;
    const int p0 = (int)(g % segs) * RL, p1 = min(p0 + RL, HW);
    const int* Mb = M + b * HW;
    int* cb = counts + (size_t)b * nlab;
    int cur = 0, run = 0;
    for (int p = p0; p < p1; ++p) {
      const int lab = Mb[p];
      if (lab != cur) {
        if (cur > 0) atomicAdd(cb + cur, run);
        cur = lab;
        run = 0;
      }
      ++run;
    }
    if (cur > 0) atomicAdd(cb + cur, run);
  }
}
}  // namespace

extern "C" int be_label_counts(const int* M, int B, int HW, int nlab, int* counts, hipStream_t s) {
  const long long n = (long long)B * HW;
  const long long nseg = (long long)B * ((HW + RL - 1) / RL);
  int blocks = (int)((nseg + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(label_counts_kernel, dim3(blocks), dim3(256), 0, s, M, n, HW, nlab, counts);
  return BE_CHECK_LAUNCH();
}

// Host-side (CPU, C++) parts of the EM mitochondria post-processing that are inherently serial
// (reference apps/fibsem-mito-analysis/analysis_deployment.py:160-176):
//
//  * be_rt_watershed — marker-controlled priority-flood watershed with skimage.segmentation.watershed
//    semantics for compactness 0: markers seed a min-heap ordered by (image value, insertion age);
//    a popped pixel labels its unlabeled in-mask neighbours (4- / 6-connectivity, or 8 / 26) at push
//    time.  2-D and 3-D.
//  * be_rt_ensure_spacing — skimage ensure_spacing for peak_local_max: points are visited in the
//    given (priority) order; each kept point rejects later points closer than `spacing` in the
//    Chebyshev norm.  A uniform grid with cell = spacing makes it O(N).
//
// The GPU produces the distance transform, the peak candidates and every other dense stage; these
// two serial passes run here on host threads of the worker.
#include <cstdint>
#include <cstring>
#include <queue>
#include <unordered_map>
#include <vector>

namespace {

struct Elem {
  float value;
  uint64_t age;
  int64_t index;
};

struct Cmp {
  bool operator()(const Elem& a, const Elem& b) const {
    if (a.value != b.value) return a.value > b.value;  // min-heap on value
    return a.age > b.age;                              // then FIFO
  }
};

}  // namespace

extern "C" {

// image f32 [D, H, W]; markers int32 (0 = unlabeled); mask uint8 (nullptr = all); out int32
int be_rt_watershed(const float* image, const int* markers, const unsigned char* mask, int D, int H, int W, int conn,
                    int* out) {
  const int64_t HW = (int64_t)H * W, N = HW * D;
  std::vector<int64_t> offs;
  std::vector<int> dz, dy, dx;
  for (int z = -1; z <= 1; ++z)
    for (int y = -1; y <= 1; ++y)
      for (int x = -1; x <= 1; ++x) {
        if (!z && !y && !x) continue;
        if (D == 1 && z) continue;
        const int manh = (z != 0) + (y != 0) + (x != 0);
        if (conn == 1 && manh > 1) continue;  // face neighbours only
        dz.push_back(z); dy.push_back(y); dx.push_back(x);
      }
  std::priority_queue<Elem, std::vector<Elem>, Cmp> hp;
  for (int64_t i = 0; i < N; ++i) {
    const bool in = !mask || mask[i];
    out[i] = in ? markers[i] : 0;
    if (in && markers[i] > 0) hp.push(Elem{image[i], 0, i});
  }
  uint64_t age = 1;
  while (!hp.empty()) {
    const Elem e = hp.top();
    hp.pop();
    const int z = (int)(e.index / HW), y = (int)((e.index / W) % H), x = (int)(e.index % W);
    const int lab = out[e.index];
    for (size_t k = 0; k < dz.size(); ++k) {
      const int zz = z + dz[k], yy = y + dy[k], xx = x + dx[k];
      if (zz < 0 || zz >= D || yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
      const int64_t j = ((int64_t)zz * H + yy) * W + xx;
      if ((mask && !mask[j]) || out[j]) continue;
      out[j] = lab;
      hp.push(Elem{image[j], age++, j});
    }
  }
  return 0;
}

// coords int32 [N, ndim] in priority order; keep uint8 [N] (1 = kept)
int be_rt_ensure_spacing(const int* coords, int N, int ndim, int spacing, unsigned char* keep) {
  if (spacing <= 0) {
    std::memset(keep, 1, N);
    return 0;
  }
  auto key = [&](const int* c) {
    int64_t k = 0;
    for (int d = 0; d < ndim; ++d) k = k * 1000003 + (int64_t)(c[d] / spacing + 1);
    return k;
  };
  std::unordered_map<int64_t, std::vector<int>> grid;
  grid.reserve(N * 2 + 1);
  for (int i = 0; i < N; ++i) grid[key(coords + (int64_t)i * ndim)].push_back(i);
  std::vector<unsigned char> rejected(N, 0);
  std::vector<int> cell(ndim);
  for (int i = 0; i < N; ++i) {
    keep[i] = 0;
    if (rejected[i]) continue;
    keep[i] = 1;
    const int* ci = coords + (int64_t)i * ndim;
    // visit the 3^ndim neighbouring cells
    int total = 1;
    for (int d = 0; d < ndim; ++d) total *= 3;
    for (int t = 0; t < total; ++t) {
      int tt = t;
      int64_t k = 0;
      for (int d = 0; d < ndim; ++d) {
        const int off = tt % 3 - 1;
        tt /= 3;
        cell[d] = ci[d] / spacing + 1 + off;
      }
      for (int d = 0; d < ndim; ++d) k = k * 1000003 + cell[d];
      auto it = grid.find(k);
      if (it == grid.end()) continue;
      for (int j : it->second) {
        if (j == i || rejected[j] || (j < i && keep[j])) continue;
        int cheb = 0;
        const int* cj = coords + (int64_t)j * ndim;
        for (int d = 0; d < ndim; ++d) {
          const int a = ci[d] - cj[d];
          cheb = a < 0 ? (-a > cheb ? -a : cheb) : (a > cheb ? a : cheb);
        }
        if (cheb < spacing) rejected[j] = 1;
      }
    }
  }
  return 0;
}

}  // extern "C"

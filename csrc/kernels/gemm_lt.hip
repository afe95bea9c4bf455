// Library GEMMs of the ViT training / embedding paths on hipBLASLt, driven directly (not through
// torch.mm) so that
//   * the elementwise work around a GEMM runs in its epilogue: bias, GELU with the pre-activation
//     stored as an aux output (MLP lin1 forward), GELU-backward from that aux plus the bias gradient
//     (lin2 dgrad -> d(lin1 pre-activation) and d(lin1 bias) in one pass) -- the separate GELU
//     forward / backward passes over the [tokens, 4*dim] activation disappear;
//   * fp32 outputs (weight gradients straight into the flat fp32 gradient buffer) and beta = 1
//     accumulation are plain options;
//   * every distinct (shape, layout, epilogue) is autotuned once: up to 32 heuristic candidates are
//     timed on the real operands (outputs redirected to scratch) and the fastest is cached.  A GEMM
//     first seen inside a HIP-graph capture uses the heuristic's first choice (nothing may be timed
//     or allocated while capturing); the training engine runs eager warm-up steps before it captures.
//
// Row-major interface: D[M, N] = alpha * op(X)[M, K] . op(Y)[K, N] (+ beta * D), with
//   tx = 0: X stored [M, K]; tx = 1: X stored [K, M] (used transposed)
//   ty = 0: Y stored [K, N]; ty = 1: Y stored [N, K] (nn.Linear weight layout)
// mapped onto hipBLASLt's column-major D^T = op(Y)^T op(X)^T, so per-output-feature vectors (bias,
// bias gradient) run along D's column-major rows.
#include "common.h"

#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <cmath>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

namespace {

enum Epi { EPI_NONE = 0, EPI_BIAS = 1, EPI_GELU_AUX_BIAS = 2, EPI_DGELU_BGRAD = 3, EPI_GELU_BIAS = 4, EPI_BGRAD = 5,
           EPI_DGELU = 6 };

struct Key {
  int dev, M, N, K, tx, ty, dt_out, epi, accum, bias_fp32;
  bool operator<(const Key& o) const {
    return std::tie(dev, M, N, K, tx, ty, dt_out, epi, accum, bias_fp32) <
           std::tie(o.dev, o.M, o.N, o.K, o.tx, o.ty, o.dt_out, o.epi, o.accum, o.bias_fp32);
  }
};

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, ld = nullptr;
  hipblasLtMatmulAlgo_t algo;
  size_t ws = 0;
  bool tuned = false;
  float best_us = 0.f;
  int candidates = 0;
  int rejected = 0;  // candidates whose output disagreed with the reference candidate
};

std::mutex g_mu;
std::map<int, hipblasLtHandle_t> g_handles;
std::map<Key, Plan> g_plans;
int g_tune = -1;  // BE_LT_TUNE: 1 time the candidates (default), 0 heuristic first choice
int g_force = -1;  // be_lt_force: use heuristic candidate #i for plans built from now on (validation)

hipblasLtHandle_t handle_for(int dev) {
  auto it = g_handles.find(dev);
  if (it != g_handles.end()) return it->second;
  hipblasLtHandle_t h = nullptr;
  if (hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) return nullptr;
  g_handles[dev] = h;
  return h;
}

hipblasLtEpilogue_t lt_epi(int e) {
  switch (e) {
    case EPI_BIAS: return HIPBLASLT_EPILOGUE_BIAS;
    case EPI_GELU_AUX_BIAS: return HIPBLASLT_EPILOGUE_GELU_AUX_BIAS;
    case EPI_DGELU_BGRAD: return HIPBLASLT_EPILOGUE_DGELU_BGRAD;
    case EPI_GELU_BIAS: return HIPBLASLT_EPILOGUE_GELU_BIAS;
    case EPI_BGRAD: return HIPBLASLT_EPILOGUE_BGRADB;
    case EPI_DGELU: return HIPBLASLT_EPILOGUE_DGELU;
    default: return HIPBLASLT_EPILOGUE_DEFAULT;
  }
}

// per-call pointer attributes of the descriptor
hipblasStatus_t set_ptrs(const Plan& p, int epi, const void* bias, void* aux, void* bgrad, long long ldaux) {
  hipblasStatus_t st = HIPBLAS_STATUS_SUCCESS;
  if (epi == EPI_BIAS || epi == EPI_GELU_AUX_BIAS || epi == EPI_GELU_BIAS)
    st = hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias));
  if (st == HIPBLAS_STATUS_SUCCESS && (epi == EPI_DGELU_BGRAD || epi == EPI_BGRAD))
    st = hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bgrad, sizeof(bgrad));
  if (st == HIPBLAS_STATUS_SUCCESS && (epi == EPI_GELU_AUX_BIAS || epi == EPI_DGELU_BGRAD || epi == EPI_DGELU)) {
    st = hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux, sizeof(aux));
    if (st == HIPBLAS_STATUS_SUCCESS)
      st = hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ldaux, sizeof(ldaux));
  }
  return st;
}

int build_plan(Plan& p, const Key& k) {
  const hipDataType bt = HIP_R_16BF;
  const hipDataType dt = k.dt_out ? HIP_R_32F : HIP_R_16BF;
  if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return -10;
  // column-major problem: m = N, n = M; A := Y side, B := X side
  hipblasOperation_t opA = k.ty ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  hipblasOperation_t opB = k.tx ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opA, sizeof(opA));
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opB, sizeof(opB));
  hipblasLtEpilogue_t e = lt_epi(k.epi);
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e));
  // flags (bias_fp32 argument): bit 0 bias / bias-gradient vector in fp32, bit 1 leave the aux
  // type at its default (D's type), bit 2 leave the bias type at its default
  if (k.epi != EPI_NONE && k.epi != EPI_DGELU && !(k.bias_fp32 & 4)) {
    const int32_t bdt = (k.bias_fp32 & 1) ? HIP_R_32F : HIP_R_16BF;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bdt, sizeof(bdt));
  }
  if ((k.epi == EPI_GELU_AUX_BIAS || k.epi == EPI_DGELU_BGRAD || k.epi == EPI_DGELU) && !(k.bias_fp32 & 2)) {
    const int32_t adt = HIP_R_16BF;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &adt, sizeof(adt));
  }
  const uint64_t m = k.N, n = k.M, kk = k.K;
  if (k.ty) hipblasLtMatrixLayoutCreate(&p.la, bt, kk, m, kk);
  else hipblasLtMatrixLayoutCreate(&p.la, bt, m, kk, m);
  if (k.tx) hipblasLtMatrixLayoutCreate(&p.lb, bt, n, kk, n);
  else hipblasLtMatrixLayoutCreate(&p.lb, bt, kk, n, kk);
  hipblasLtMatrixLayoutCreate(&p.ld, dt, m, n, m);
  return 0;
}

long long out_bytes(const Key& k) { return (long long)k.M * k.N * (k.dt_out ? 4 : 2); }

// acc[0] += sum (a - b)^2, acc[1] += sum b^2 over n elements (bf16 or fp32): candidate validation
__global__ __launch_bounds__(256) void lt_sqdiff_kernel(const void* a, const void* b, long long n, int fp32,
                                                        float* acc) {
  float d2 = 0.f, r2 = 0.f;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float x = fp32 ? ((const float*)a)[i] : bf2f(((const uint16_t*)a)[i]);
    const float y = fp32 ? ((const float*)b)[i] : bf2f(((const uint16_t*)b)[i]);
    d2 += (x - y) * (x - y);
    r2 += y * y;
  }
  for (int o = 32; o > 0; o >>= 1) {
    d2 += __shfl_xor(d2, o, 64);
    r2 += __shfl_xor(r2, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(acc, d2);
    atomicAdd(acc + 1, r2);
  }
}

// relative L2 distance of a candidate's output from the reference candidate's (synchronises)
float rel_l2(const void* a, const void* b, long long n, int fp32, float* acc_dev, hipStream_t s) {
  hipMemsetAsync(acc_dev, 0, 2 * sizeof(float), s);
  const int grid = (int)std::min<long long>(1024, (n + 255) / 256);
  hipLaunchKernelGGL(lt_sqdiff_kernel, dim3(grid), dim3(256), 0, s, a, b, n, fp32, acc_dev);
  float h[2] = {0.f, 0.f};
  hipMemcpyAsync(h, acc_dev, sizeof(h), hipMemcpyDeviceToHost, s);
  hipStreamSynchronize(s);
  return h[1] > 0.f ? sqrtf(h[0] / h[1]) : (h[0] > 0.f ? 1.f : 0.f);
}

}  // namespace

extern "C" {

// D[M,N] (bf16 or fp32 when dt_out = 1) = alpha op(X) op(Y) + beta D, epilogue per `epi`:
//   1 bias[N] (bf16, or fp32 with bias_fp32)   2 gelu(. + bias) with aux[M,N] = pre-activation (bf16)
//   3 D = dgelu(aux) * (op(X) op(Y)), bgrad[N] = column sums of D (fp32 with bias_fp32)
//   4 gelu(. + bias)                           5 bgrad[N] = column sums of op(X) (X's rows summed)
// ws: device workspace of ws_bytes.  Returns 0, or a negative code / hipBLASLt status.
int be_lt_gemm(const void* X, const void* Y, void* D, const void* bias, void* aux, void* bgrad, void* ws,
               long long ws_bytes, int M, int N, int K, int tx, int ty, int dt_out, int epi, int bias_fp32,
               float alpha, float beta, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  int dev = 0;
  hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_tune < 0) {
    const char* e = getenv("BE_LT_TUNE");
    g_tune = (e && e[0] == '0') ? 0 : 1;
  }
  hipblasLtHandle_t h = handle_for(dev);
  if (!h) return -11;
  const Key key{dev, M, N, K, tx, ty, dt_out, epi, beta != 0.f ? 1 : 0, bias_fp32};
  Plan& p = g_plans[key];
  if (!p.desc) {
    int rc = build_plan(p, key);
    if (rc) return rc;
  }
  const long long ldaux = N;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  hipStreamIsCapturing(stream, &cap);
  const bool capturing = cap != hipStreamCaptureStatusNone;
  if (!p.tuned) {
    hipblasLtMatmulPreference_t pref;
    hipblasLtMatmulPreferenceCreate(&pref);
    uint64_t wsb = (uint64_t)ws_bytes;
    hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb));
    hipblasLtMatmulHeuristicResult_t res[32];
    int nres = 0;
    // heuristics need the epilogue pointers set (validity checks read the descriptor)
    set_ptrs(p, epi, bias, aux, bgrad, ldaux);
    hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, p.desc, p.la, p.lb, p.ld, p.ld, pref,
                                                         (g_tune && !capturing) ? 32 : 1, res, &nres);
    hipblasLtMatmulPreferenceDestroy(pref);
    if (st != HIPBLAS_STATUS_SUCCESS || nres == 0) return -12;
    int best = 0;
    p.candidates = nres;
    if (g_tune && !capturing && nres > 1) {
      // Time each candidate with the outputs redirected to scratch (inputs are only read).  Every
      // candidate is first checked against the heuristic's first choice: some epilogue kernels of
      // this hipBLASLt build return wrong results (tools/lt_validate.py found DGELU_BGRAD
      // candidates with a wrong output or a wrong bias gradient), and they can be the fastest.
      void *d2 = nullptr, *dref = nullptr, *aux2 = nullptr, *bg2 = nullptr, *bgref = nullptr;
      float* acc = nullptr;
      const bool aux_out = epi == EPI_GELU_AUX_BIAS;
      const bool has_bg = epi == EPI_DGELU_BGRAD || epi == EPI_BGRAD;
      const long long ob = out_bytes(key);
      bool ok = hipMalloc(&d2, ob) == hipSuccess && hipMalloc(&dref, ob) == hipSuccess &&
                hipMalloc(&acc, 2 * sizeof(float)) == hipSuccess;
      if (ok && aux_out) ok = hipMalloc(&aux2, (long long)M * N * 2) == hipSuccess;
      if (ok && has_bg) ok = hipMalloc(&bg2, (long long)N * 4) == hipSuccess && hipMalloc(&bgref, (long long)N * 4) == hipSuccess;
      auto release = [&]() {
        hipStreamSynchronize(stream);
        for (void* q : {d2, dref, aux2, bg2, bgref, (void*)acc})
          if (q) hipFree(q);
      };
      if (!ok) { release(); return -13; }
      const int bg_fp32 = key.bias_fp32 & 1;
      auto run = [&](int i, void* d, void* bg) {
        hipMemsetAsync(d, 0, ob, stream);
        set_ptrs(p, epi, bias, aux_out ? aux2 : aux, bg, ldaux);
        return hipblasLtMatmul(h, p.desc, &alpha, Y, p.la, X, p.lb, &beta, d, p.ld, d, p.ld, &res[i].algo, ws,
                               (size_t)ws_bytes, stream) == HIPBLAS_STATUS_SUCCESS;
      };
      int ref = -1;
      for (int i = 0; i < nres && ref < 0; ++i)
        if (res[i].state == HIPBLAS_STATUS_SUCCESS && res[i].workspaceSize <= (size_t)ws_bytes && run(i, dref, bgref))
          ref = i;
      if (ref < 0) { release(); return -14; }
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      float best_t = 1e30f;
      p.rejected = 0;
      for (int i = ref; i < nres; ++i) {
        if (res[i].state != HIPBLAS_STATUS_SUCCESS || res[i].workspaceSize > (size_t)ws_bytes) continue;
        if (!run(i, d2, bg2)) continue;
        if (i != ref) {
          float e = rel_l2(d2, dref, (long long)M * N, key.dt_out, acc, stream);
          if (has_bg) e = std::max(e, rel_l2(bg2, bgref, N, bg_fp32, acc, stream));
          if (!(e < 2e-2f)) { ++p.rejected; continue; }
        }
        hipEventRecord(e0, stream);
        constexpr int REPS = 5;
        for (int r = 0; r < REPS; ++r)
          hipblasLtMatmul(h, p.desc, &alpha, Y, p.la, X, p.lb, &beta, d2, p.ld, d2, p.ld, &res[i].algo, ws,
                          (size_t)ws_bytes, stream);
        hipEventRecord(e1, stream);
        hipEventSynchronize(e1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best_t) { best_t = ms; best = i; }
      }
      hipEventDestroy(e0);
      hipEventDestroy(e1);
      release();
      if (best_t >= 1e30f) return -14;
      p.best_us = best_t * 1e3f / 5;
    }
    if (g_force >= 0) best = g_force < nres ? g_force : nres - 1;
    p.algo = res[best].algo;
    p.ws = res[best].workspaceSize;
    p.tuned = g_tune == 0 || !capturing || nres == 1;  // a capture-time pick is re-tuned later
  }
  hipblasStatus_t st = set_ptrs(p, epi, bias, aux, bgrad, ldaux);
  if (st != HIPBLAS_STATUS_SUCCESS) return -(1000 + (int)st);
  st = hipblasLtMatmul(h, p.desc, &alpha, Y, p.la, X, p.lb, &beta, D, p.ld, D, p.ld, &p.algo, ws, (size_t)ws_bytes,
                       stream);
  return st == HIPBLAS_STATUS_SUCCESS ? 0 : -(2000 + (int)st);
}

// Drop every cached plan (the next call of each shape re-runs the heuristic / tuning) and force
// heuristic candidate `force` for the plans built next (-1: tuned choice).  Returns the plans dropped.
int be_lt_reset(int force) {
  std::lock_guard<std::mutex> lk(g_mu);
  int n = (int)g_plans.size();
  for (auto& kv : g_plans) {
    Plan& p = kv.second;
    if (p.la) hipblasLtMatrixLayoutDestroy(p.la);
    if (p.lb) hipblasLtMatrixLayoutDestroy(p.lb);
    if (p.ld) hipblasLtMatrixLayoutDestroy(p.ld);
    if (p.desc) hipblasLtMatmulDescDestroy(p.desc);
  }
  g_plans.clear();
  g_force = force;
  return n;
}

// Tuning table for reports: writes up to `cap` rows of {M, N, K, tx, ty, dt_out, epi, accum,
// candidates * 1000 + rejected, best_us * 1000} as long longs; returns the number of plans.
int be_lt_plans(long long* out, int cap) {
  std::lock_guard<std::mutex> lk(g_mu);
  int i = 0;
  for (auto& kv : g_plans) {
    if (i < cap) {
      const Key& k = kv.first;
      long long* r = out + 10 * i;
      r[0] = k.M; r[1] = k.N; r[2] = k.K; r[3] = k.tx; r[4] = k.ty; r[5] = k.dt_out; r[6] = k.epi; r[7] = k.accum;
      r[8] = kv.second.candidates * 1000 + kv.second.rejected; r[9] = (long long)(kv.second.best_us * 1000.f);
    }
    ++i;
  }
  return i;
}

}  // extern "C"

// hipBLASLt GEMMs with the trunk's fused epilogue: the 1x1 convolutions of the
// frozen ResNet bottlenecks (reference: the torchvision trunk of
// lib/model.py:37-44, frozen BN folded into the conv bias) as
//
//   Y[m][co] = act( sum_ci X[m][ci] W[co][ci] + bias[co] + R[m][co] )
//
// X [M, Cin], W [Cout, Cin], R / Y [M, Cout], all row-major bf16 (NHWC
// activations: M = N*H*W), bias fp32.  In hipBLASLt's column-major terms this
// is D (Cout x M, ld Cout) = W^T(op T) * X(op N) + beta C, epilogue BIAS or
// RELU_BIAS (bias per D row = per output channel, applied with beta*C before the
// ReLU) -- the residual add, bias and ReLU in one pass over Y instead of a GEMM
// followed by an elementwise kernel that re-reads and re-writes it.
//
// Algorithm choice: hipBLASLt's heuristic returns up to NALGO candidates; with
// `tune` (the trunk's eager warm-up, never inside a HIP graph capture) every
// candidate is timed on the caller's stream and the fastest is kept for the
// shape, else the heuristic's first.  One workspace per device.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <tuple>
#include <vector>

namespace {

constexpr int NALGO = 16;
constexpr size_t WS_BYTES = 64ull << 20;

struct LtDev {
  hipblasLtHandle_t h = nullptr;
  void* ws = nullptr;
};

struct LtPlan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr;
  std::vector<hipblasLtMatmulHeuristicResult_t> algos;
  int chosen = 0;
  bool tuned = false;
};

using Key = std::tuple<int, int, int, int, int, int, int, int>;   // dev, m, n, k, relu, has_c, f16, has_bias

std::map<int, LtDev>& devs() {
  static std::map<int, LtDev> d;
  return d;
}
std::map<Key, LtPlan>& plans() {
  static std::map<Key, LtPlan> p;
  return p;
}

int dev_state(LtDev*& out) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -10;
  LtDev& d = devs()[dev];
  if (!d.h) {
    if (hipblasLtCreate(&d.h) != HIPBLAS_STATUS_SUCCESS) return -11;
    if (hipMalloc(&d.ws, WS_BYTES) != hipSuccess) return -12;
  }
  out = &d;
  return dev;
}

#define LT_OK(x) do { if ((x) != HIPBLAS_STATUS_SUCCESS) return -20; } while (0)

int make_plan(LtDev& d, LtPlan& p, int cout, int m, int cin, int relu, int has_c, int f16, int has_bias) {
  const hipDataType dt = f16 ? HIP_R_16F : HIP_R_16BF;
  LT_OK(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const int32_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  LT_OK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  LT_OK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  const uint32_t epi = has_bias ? (relu ? HIPBLASLT_EPILOGUE_RELU_BIAS : HIPBLASLT_EPILOGUE_BIAS)
                                : (relu ? HIPBLASLT_EPILOGUE_RELU : HIPBLASLT_EPILOGUE_DEFAULT);
  LT_OK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
  if (has_bias) {
    const int32_t bt = HIP_R_32F;
    LT_OK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  }
  // A = W stored [Cout][Cin] row-major = (Cin x Cout) col-major, op T; B = X (Cin x M), op N
  LT_OK(hipblasLtMatrixLayoutCreate(&p.a, dt, cin, cout, cin));
  LT_OK(hipblasLtMatrixLayoutCreate(&p.b, dt, cin, m, cin));
  LT_OK(hipblasLtMatrixLayoutCreate(&p.c, dt, cout, m, cout));
  hipblasLtMatmulPreference_t pref;
  LT_OK(hipblasLtMatmulPreferenceCreate(&pref));
  const uint64_t wsb = WS_BYTES;
  LT_OK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
  p.algos.resize(NALGO);
  int got = 0;
  const hipblasStatus_t st =
      hipblasLtMatmulAlgoGetHeuristic(d.h, p.desc, p.a, p.b, p.c, p.c, pref, NALGO, p.algos.data(), &got);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (st != HIPBLAS_STATUS_SUCCESS || got <= 0) return -21;
  p.algos.resize(got);
  (void)has_c;
  return 0;
}

int run(LtDev& d, LtPlan& p, int i, const void* W, const void* X, const void* R, void* Y, const float* bias,
        hipStream_t st) {
  const float alpha = 1.f, beta = R ? 1.f : 0.f;
  if (bias && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)) !=
                  HIPBLAS_STATUS_SUCCESS)
    return -22;
  const hipblasStatus_t s = hipblasLtMatmul(d.h, p.desc, &alpha, W, p.a, X, p.b, &beta, R ? R : Y, p.c, Y, p.c,
                                            &p.algos[i].algo, d.ws, WS_BYTES, st);
  return s == HIPBLAS_STATUS_SUCCESS ? 0 : -23;
}

}  // namespace

// Y = act(X W^T + bias + R); returns 0, or a negative code.  tune != 0: time
// every heuristic candidate once for this shape (not while the stream is
// being captured) and keep the fastest.
extern "C" int ncnet_gemm_lt(const void* X, const void* W, const float* bias, const void* R, void* Y, int m, int cin,
                             int cout, int relu, int f16, int tune, hipStream_t st) {
  LtDev* d = nullptr;
  const int dev = dev_state(d);
  if (dev < 0) return dev;
  const Key key{dev, m, cout, cin, relu, R != nullptr, f16, bias != nullptr};
  auto it = plans().find(key);
  if (it == plans().end()) {
    LtPlan p;
    const int rc = make_plan(*d, p, cout, m, cin, relu, R != nullptr, f16, bias != nullptr);
    if (rc) return rc;
    it = plans().emplace(key, std::move(p)).first;
  }
  LtPlan& p = it->second;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) return -24;
  if (tune && !p.tuned && cs == hipStreamCaptureStatusNone && p.algos.size() > 1) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f;
    int besti = 0;
    for (int i = 0; i < (int)p.algos.size(); ++i) {
      if (run(*d, p, i, W, X, R, Y, bias, st)) continue;   // warm (and skip a candidate that fails)
      hipEventRecord(e0, st);
      for (int r = 0; r < 3; ++r) run(*d, p, i, W, X, R, Y, bias, st);
      hipEventRecord(e1, st);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) { best = ms; besti = i; }
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    p.chosen = besti;
    p.tuned = true;
  }
  return run(*d, p, p.chosen, W, X, R, Y, bias, st);
}

// Vendor GEMM (hipBLASLt) reference of the GEMM microbenchmarks (tools/g8bench, g9bench, kbench):
// the library ran these shapes on hipBLASLt until round 4; since round 5 they run on gemm9.hip.
//
// Measured on MI355X (tools/torch_gemm_probe.py vs tools/kbench): the in-tree kernels win the
// LayerNorm-folded, multi-source, implicit-3x3 and narrow high-M shapes (levels 1-2), hipBLASLt
// wins the MFMA-heavier low-M projections (latent level, K >= 512) and the L3 residual
// projections (project_out 130560x256x640: 85 vs 117 us). Only plain GEMMs go here:
//   D[M][N] = X[M][K] . W[N][K]^T (+ bias[N]) (+ C[M][N]), bf16 storage, fp32 accumulation,
// pixel-major activations = column-major [K][M] for hipBLASLt, so D^T = W . X^T with op(A) = T.
// One hipBLASLt handle, one 64 MiB workspace and a descriptor/algorithm cache per TurtleHandle;
// every call is ordered on the caller's stream.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdint>
#include <map>
#include <tuple>

#include "blas_ref.h"

namespace turtle {

struct BlasPlan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr, d = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  bool ok = false;
};

struct BlasCtx {
  hipblasLtHandle_t h = nullptr;
  void* ws = nullptr;
  size_t ws_bytes = (size_t)64 << 20;
  std::map<std::tuple<int64_t, int, int, int64_t, int64_t, int64_t, int64_t, int, int>, BlasPlan> plans;
};

BlasCtx* blas_create() {
  BlasCtx* c = new BlasCtx;
  if (hipblasLtCreate(&c->h) != HIPBLAS_STATUS_SUCCESS || hipMalloc(&c->ws, c->ws_bytes) != hipSuccess) {
    if (c->h) hipblasLtDestroy(c->h);
    delete c;
    return nullptr;
  }
  return c;
}

void blas_destroy(BlasCtx* c) {
  if (!c) return;
  for (auto& kv : c->plans) {
    BlasPlan& p = kv.second;
    if (p.desc) hipblasLtMatmulDescDestroy(p.desc);
    for (auto l : {p.a, p.b, p.c, p.d})
      if (l) hipblasLtMatrixLayoutDestroy(l);
  }
  if (c->ws) (void)hipFree(c->ws);
  if (c->h) hipblasLtDestroy(c->h);
  delete c;
}

static BlasPlan& plan(BlasCtx* c, int64_t M, int N, int K, int64_t ldx, int64_t ldw, int64_t ldc, int64_t ldd,
                      bool has_c, bool has_bias) {
  auto key = std::make_tuple(M, N, K, ldx, ldw, ldc, ldd, (int)has_c, (int)has_bias);
  auto it = c->plans.find(key);
  if (it != c->plans.end()) return it->second;
  BlasPlan& p = c->plans[key];
  hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return p;
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof ta);
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof tb);
  if (has_bias) {
    hipblasLtEpilogue_t ep = HIPBLASLT_EPILOGUE_BIAS;
    hipDataType bt = HIP_R_32F;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof ep);
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof bt);
  }
  // column-major views: A = W as [K][N] (op T), B = X as [K][M], C/D as [N][M]
  if (hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16BF, K, N, ldw) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16BF, K, M, ldx) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.c, HIP_R_16BF, N, M, has_c ? ldc : ldd) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.d, HIP_R_16BF, N, M, ldd) != HIPBLAS_STATUS_SUCCESS)
    return p;
  hipblasLtMatmulPreference_t pref;
  if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return p;
  uint64_t wsb = c->ws_bytes;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof wsb);
  hipblasLtMatmulHeuristicResult_t res[1];
  int n = 0;
  if (hipblasLtMatmulAlgoGetHeuristic(c->h, p.desc, p.a, p.b, p.c, p.d, pref, 1, res, &n) == HIPBLAS_STATUS_SUCCESS &&
      n > 0 && res[0].workspaceSize <= c->ws_bytes) {
    p.algo = res[0].algo;
    p.ok = true;
  }
  hipblasLtMatmulPreferenceDestroy(pref);
  return p;
}

bool blas_ready(BlasCtx* c, int64_t M, int N, int K, int64_t ldx, int64_t ldw, int64_t ldc, int64_t ldd, bool has_c,
                bool has_bias) {
  return c && plan(c, M, N, K, ldx, ldw, ldc, ldd, has_c, has_bias).ok;
}

bool blas_gemm_bf16(BlasCtx* c, int64_t M, int N, int K, const void* X, int64_t ldx, const void* W, int64_t ldw,
                    const float* bias, const void* C, int64_t ldc, void* D, int64_t ldd, hipStream_t st) {
  if (!c) return false;
  BlasPlan& p = plan(c, M, N, K, ldx, ldw, ldc, ldd, C != nullptr, bias != nullptr);
  if (!p.ok) return false;
  if (bias && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof bias) !=
                  HIPBLAS_STATUS_SUCCESS)
    return false;
  const float alpha = 1.f, beta = C ? 1.f : 0.f;
  return hipblasLtMatmul(c->h, p.desc, &alpha, W, p.a, X, p.b, &beta, C ? C : D, p.c, D, p.d, &p.algo, c->ws,
                         c->ws_bytes, st) == HIPBLAS_STATUS_SUCCESS;
}

// LayerNorm prologue of the vendor path: the in-tree GEMMs fold LayerNorm into their operand
// staging; hipBLASLt cannot, so LN-folded latent projections first write the normalised rows
// xn = (x - mu) * rstd (BiasFree: x * rstd, turtle_t1_arch.py:68-80) in storage precision and run
// D = W' xn + (W b_ln + bias) (W' = W diag(g_ln), packed by pack_gemm). One wave per pixel row,
// fp32 statistics (biased variance, eps 1e-5: turtle_t1_arch.py:83-112).
template <typename T>
__global__ __launch_bounds__(256) void ln_rows_kernel(LnRowsArgs a) {
  constexpr int VEC = Vec<T>::N;
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= a.M) return;
  const T* x = reinterpret_cast<const T*>(a.x) + r * a.ldx + a.offx;
  T* o = reinterpret_cast<T*>(a.out) + r * a.ldo;
  constexpr int MAXV = 4;                               // K <= 64 lanes * VEC * MAXV
  float v[MAXV][VEC];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int k = (j * 64 + lane) * VEC;
    if (k < a.K) {
      Vec<T> q; q.load(x + k);
#pragma unroll
      for (int i = 0; i < VEC; ++i) { v[j][i] = q.v[i]; s += q.v[i]; }
    }
  }
  const float mu = wave_sum(s) / a.K;
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int k = (j * 64 + lane) * VEC;
    if (k < a.K) {
#pragma unroll
      for (int i = 0; i < VEC; ++i) { const float d = v[j][i] - mu; ss += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(ss) / a.K + 1e-5f);
  const float sub = a.centred ? mu : 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int k = (j * 64 + lane) * VEC;
    if (k < a.K) {
      Vec<T> q;
#pragma unroll
      for (int i = 0; i < VEC; ++i) q.v[i] = (v[j][i] - sub) * rstd;
      q.store(o + k);
    }
  }
}

template <typename T>
void launch_ln_rows(const LnRowsArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(ln_rows_kernel<T>, dim3((unsigned)((a.M + 3) / 4)), dim3(256), 0, st, a);
}
template void launch_ln_rows<float>(const LnRowsArgs&, hipStream_t);
template void launch_ln_rows<bf16>(const LnRowsArgs&, hipStream_t);

}  // namespace turtle

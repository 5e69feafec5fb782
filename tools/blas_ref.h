// hipBLASLt reference for the GEMM microbenchmarks (tools/g8bench, g9bench, kbench only; the library
// has no vendor GEMM since round 5): D = X W^T (+ bias) (+ C), bf16, fp32 accumulation; LN rows pass
// that feeds it the normalised operand of a LayerNorm-folded projection.
#pragma once
#include "kernels.h"

namespace turtle {
// hipBLASLt plain-GEMM path (tools/blas_ref.cpp): D = X W^T (+ bias) (+ C), bf16, fp32 accumulation
struct BlasCtx;
BlasCtx* blas_create();
void blas_destroy(BlasCtx* c);
bool blas_ready(BlasCtx* c, int64_t M, int N, int K, int64_t ldx, int64_t ldw, int64_t ldc, int64_t ldd, bool has_c,
                bool has_bias);
bool blas_gemm_bf16(BlasCtx* c, int64_t M, int N, int K, const void* X, int64_t ldx, const void* W, int64_t ldw,
                    const float* bias, const void* C, int64_t ldc, void* D, int64_t ldd, hipStream_t st);

struct LnRowsArgs {                // blas_ref.cpp: out[r] = (x[r] - mu) * rstd (centred) or x[r] * rstd
  const void* x; int64_t ldx; int offx; void* out; int64_t ldo; int64_t M; int K; int centred;
};
template <typename T> void launch_ln_rows(const LnRowsArgs& a, hipStream_t st);   // K <= 64 * VEC * 4

}  // namespace turtle

// Training-path kernels with hand-written backward (include/turtle_train.h), NCHW tensors as the
// torch autograd graph holds them, fp32 or bf16 storage, fp32 arithmetic:
//
//   channel LayerNorm   y = (x - mu) * rstd * w + b  (BiasFree: x * rstd * w), per pixel over C
//                       (turtle_t1_arch.py:67-112); backward gives dx, dw, db
//   depthwise 3x3       y = dw3x3(x) + b, pad 1 (qkv_dwconv / conv2 / dwconv / kv_dwconv);
//                       backward dx (the same stencil with the taps flipped) and dw, db
//   GELU gate           y = gelu(x1) * x2 over the two channel halves (GatedFeedForward 176)
//
// Weight gradients are per-channel reductions over all pixels: each block reduces its pixels in
// registers / LDS and adds one fp32 partial per channel (and tap) with a device atomic; the
// caller zeroes the gradient buffers first (torch.zeros).
#include "common.h"
#include "../../include/turtle_train.h"

namespace turtle {

template <typename T> TURTLE_DEV float ldf(const T* p, int64_t i) { return to_f(p[i]); }
template <typename T> TURTLE_DEV void stf(T* p, int64_t i, float v) { p[i] = from_f<T>(v); }

TURTLE_DEV float gelu_exact(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
TURTLE_DEV float gelu_exact_grad(float x) {   // d/dx x * Phi(x) = Phi(x) + x * phi(x)
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// ---------------------------------------------------------------------------------------------
// channel LayerNorm: one thread per pixel, channel loop strided by HW (coalesced across threads)
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ b, T* __restrict__ y,
                                                     float* __restrict__ mu, float* __restrict__ rstd,
                                                     int64_t N, int C, int64_t HW, int biasfree) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= N * HW) return;
  const int64_t n = i / HW, p = i - n * HW;
  const T* xp = x + n * C * HW + p;
  const float sh = ldf(xp, 0);
  float s = 0.f, q = 0.f;
  for (int c = 0; c < C; ++c) {
    const float d = ldf(xp, (int64_t)c * HW) - sh;
    s += d;
    q = fmaf(d, d, q);
  }
  const float md = s / C, m = sh + md;
  const float r = rsqrtf(fmaxf(q / C - md * md, 0.f) + 1e-5f);
  mu[i] = m;
  rstd[i] = r;
  T* yp = y + n * C * HW + p;
  for (int c = 0; c < C; ++c) {
    const float v = ldf(xp, (int64_t)c * HW);
    stf(yp, (int64_t)c * HW, biasfree ? v * r * w[c] : fmaf((v - m) * r, w[c], b[c]));
  }
}

// backward: per pixel, g = w * dy;
//   WithBias: xh = (x - mu) r,  dx = r (g - mean(g) - xh mean(g xh))
//   BiasFree: y = w x r (r of the centred variance), dx = r g - (x - mu) r^3 mean(g x)
// dw[c] = sum_p dy xhat_c (xhat = (x - mu) r, BiasFree: x r), db[c] = sum_p dy: block partials in
// LDS, one atomic per channel per block
template <typename T>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ mu, const float* __restrict__ rstd,
                                                     const T* __restrict__ dy, T* __restrict__ dx,
                                                     float* __restrict__ dw, float* __restrict__ db,
                                                     int64_t N, int C, int64_t HW, int biasfree) {
  extern __shared__ float sred[];                  // [2][C] block partials of dw, db
  for (int c = threadIdx.x; c < 2 * C; c += 256) sred[c] = 0.f;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool live = i < N * HW;
  const int64_t ii = live ? i : 0;
  const int64_t n = ii / HW, p = ii - n * HW;
  const T* xp = x + n * C * HW + p;
  const T* gp = dy + n * C * HW + p;
  const float m = mu[ii], r = rstd[ii];
  float sg = 0.f, sgx = 0.f;
  for (int c = 0; c < C; ++c) {
    const float g = w[c] * ldf(gp, (int64_t)c * HW);
    const float v = ldf(xp, (int64_t)c * HW);
    sg += g;
    sgx = fmaf(g, biasfree ? v : (v - m) * r, sgx);
  }
  const float mg = sg / C, mgx = sgx / C;
  T* dp = dx + n * C * HW + p;
  const int lane = threadIdx.x & 63;
  for (int c = 0; c < C; ++c) {
    const float gy = ldf(gp, (int64_t)c * HW);
    const float v = ldf(xp, (int64_t)c * HW);
    const float g = w[c] * gy;
    float d;
    if (biasfree) d = r * g - (v - m) * r * r * r * mgx;
    else d = r * (g - mg - (v - m) * r * mgx);
    if (live) stf(dp, (int64_t)c * HW, d);
    // channel partials: wave sums, then one LDS atomic per wave
    float pw = live ? gy * (biasfree ? v * r : (v - m) * r) : 0.f;
    float pb = live ? gy : 0.f;
    pw = wave_sum(pw);
    pb = wave_sum(pb);
    if (lane == 0) {
      atomicAdd(&sred[c], pw);
      atomicAdd(&sred[C + c], pb);
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    atomicAdd(&dw[c], sred[c]);
    if (db) atomicAdd(&db[c], sred[C + c]);
  }
}

// ---------------------------------------------------------------------------------------------
// depthwise 3x3, pad 1: one block per (image, channel) row band; 256 threads = 256 pixels of a
// 16 x 16 output tile, haloed 18 x 18 input tile in LDS
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void dw_fwd_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ b, T* __restrict__ y, int C, int H, int W,
                                                     int flip) {
  __shared__ float tile[18][19];
  const int tx_n = (W + 15) / 16;
  const int tile_id = blockIdx.x, plane = blockIdx.y;   // plane = n * C + c
  const int c = plane % C;
  const int ty0 = (tile_id / tx_n) * 16, tx0 = (tile_id % tx_n) * 16;
  const T* xp = x + (int64_t)plane * H * W;
  for (int e = threadIdx.x; e < 18 * 18; e += 256) {
    const int r = e / 18, q = e - r * 18;
    const int yy = ty0 - 1 + r, xx = tx0 - 1 + q;
    tile[r][q] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? ldf(xp, (int64_t)yy * W + xx) : 0.f;
  }
  __syncthreads();
  const int oy = threadIdx.x >> 4, ox = threadIdx.x & 15;
  const int yy = ty0 + oy, xx = tx0 + ox;
  if (yy >= H || xx >= W) return;
  float acc = b ? b[c] : 0.f;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const float wt = w[c * 9 + (flip ? 8 - t : t)];
    acc = fmaf(wt, tile[oy + t / 3][ox + t % 3], acc);
  }
  stf(y + (int64_t)plane * H * W, (int64_t)yy * W + xx, acc);
}

// dw[c][t] = sum_{n,p} dy[n,c,p] x[n,c,p + off(t)], db[c] = sum dy: tile as in the forward, each
// thread 10 partial sums, block reduction, 10 atomics per block
template <typename T>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                       float* __restrict__ dw, float* __restrict__ db, int C, int H, int W) {
  __shared__ float tile[18][19];
  __shared__ float red[4][10];
  const int tx_n = (W + 15) / 16;
  const int tile_id = blockIdx.x, plane = blockIdx.y;
  const int c = plane % C;
  const int ty0 = (tile_id / tx_n) * 16, tx0 = (tile_id % tx_n) * 16;
  const T* xp = x + (int64_t)plane * H * W;
  for (int e = threadIdx.x; e < 18 * 18; e += 256) {
    const int r = e / 18, q = e - r * 18;
    const int yy = ty0 - 1 + r, xx = tx0 - 1 + q;
    tile[r][q] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? ldf(xp, (int64_t)yy * W + xx) : 0.f;
  }
  __syncthreads();
  const int oy = threadIdx.x >> 4, ox = threadIdx.x & 15;
  const int yy = ty0 + oy, xx = tx0 + ox;
  const bool ok = yy < H && xx < W;
  const float g = ok ? ldf(dy + (int64_t)plane * H * W, (int64_t)(ok ? yy : 0) * W + (ok ? xx : 0)) : 0.f;
  float part[10];
#pragma unroll
  for (int t = 0; t < 9; ++t) part[t] = wave_sum(g * tile[oy + t / 3][ox + t % 3]);
  part[9] = wave_sum(g);
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int t = 0; t < 10; ++t) red[wid][t] = part[t];
  __syncthreads();
  if (threadIdx.x < 10) {
    const float s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    if (threadIdx.x < 9) atomicAdd(&dw[c * 9 + threadIdx.x], s);
    else if (db) atomicAdd(&db[c], s);
  }
}

// ---------------------------------------------------------------------------------------------
// GELU gate: x [N][2h][HW] -> y [N][h][HW] = gelu(x1) * x2 (exact erf GELU, F.gelu's default)
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void gate_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t N, int h, int64_t HW) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t tot = N * h * HW;
  if (i >= tot) return;
  const int64_t n = i / (h * HW), r = i - n * h * HW;
  const T* xb = x + n * 2 * h * HW;
  stf(y, i, gelu_exact(ldf(xb, r)) * ldf(xb, (int64_t)h * HW + r));
}
template <typename T>
__global__ __launch_bounds__(256) void gate_bwd_kernel(const T* __restrict__ x, const T* __restrict__ dy, T* __restrict__ dx,
                                                       int64_t N, int h, int64_t HW) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t tot = N * h * HW;
  if (i >= tot) return;
  const int64_t n = i / (h * HW), r = i - n * h * HW;
  const T* xb = x + n * 2 * h * HW;
  T* db = dx + n * 2 * h * HW;
  const float a = ldf(xb, r), bb = ldf(xb, (int64_t)h * HW + r), g = ldf(dy, i);
  stf(db, r, g * bb * gelu_exact_grad(a));
  stf(db, (int64_t)h * HW + r, g * gelu_exact(a));
}

// ---------------------------------------------------------------------------------------------
template <typename T>
void ln_fwd(const void* x, const float* w, const float* b, void* y, float* mu, float* rstd, int64_t N, int C, int64_t HW,
            int biasfree, hipStream_t st) {
  const int64_t P = N * HW;
  hipLaunchKernelGGL(ln_fwd_kernel<T>, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, st, (const T*)x, w, b, (T*)y, mu, rstd,
                     N, C, HW, biasfree);
}
template <typename T>
void ln_bwd(const void* x, const float* w, const float* mu, const float* rstd, const void* dy, void* dx, float* dw, float* db,
            int64_t N, int C, int64_t HW, int biasfree, hipStream_t st) {
  const int64_t P = N * HW;
  hipLaunchKernelGGL(ln_bwd_kernel<T>, dim3((unsigned)((P + 255) / 256)), dim3(256), 2 * C * sizeof(float), st, (const T*)x, w,
                     mu, rstd, (const T*)dy, (T*)dx, dw, db, N, C, HW, biasfree);
}
template <typename T>
void dw_fwd(const void* x, const float* w, const float* b, void* y, int64_t N, int C, int H, int W, int flip, hipStream_t st) {
  const int tiles = ((H + 15) / 16) * ((W + 15) / 16);
  hipLaunchKernelGGL(dw_fwd_kernel<T>, dim3(tiles, (unsigned)(N * C)), dim3(256), 0, st, (const T*)x, w, b, (T*)y, C, H, W, flip);
}
template <typename T>
void dw_wgrad(const void* x, const void* dy, float* dw, float* db, int64_t N, int C, int H, int W, hipStream_t st) {
  const int tiles = ((H + 15) / 16) * ((W + 15) / 16);
  hipLaunchKernelGGL(dw_wgrad_kernel<T>, dim3(tiles, (unsigned)(N * C)), dim3(256), 0, st, (const T*)x, (const T*)dy, dw, db, C, H, W);
}
template <typename T>
void gate_fwd(const void* x, void* y, int64_t N, int h, int64_t HW, hipStream_t st) {
  const int64_t tot = N * h * HW;
  hipLaunchKernelGGL(gate_fwd_kernel<T>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, (const T*)x, (T*)y, N, h, HW);
}
template <typename T>
void gate_bwd(const void* x, const void* dy, void* dx, int64_t N, int h, int64_t HW, hipStream_t st) {
  const int64_t tot = N * h * HW;
  hipLaunchKernelGGL(gate_bwd_kernel<T>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, (const T*)x, (const T*)dy, (T*)dx,
                     N, h, HW);
}

}  // namespace turtle

// ---------------------------------------------------------------------------------------------
// C ABI (include/turtle_train.h): dtype 0 = fp32, 1 = bf16 activations; returns 0 or a HIP error
// ---------------------------------------------------------------------------------------------
using namespace turtle;
#define TT_DISPATCH(dt, fn, ...)                                   \
  do {                                                             \
    if ((dt) == 1) fn<bf16>(__VA_ARGS__); else fn<float>(__VA_ARGS__); \
    return (int)hipGetLastError();                                 \
  } while (0)

extern "C" {

int turtle_train_ln_fwd(const void* x, const float* w, const float* b, void* y, float* mu, float* rstd, int64_t N, int C,
                        int64_t HW, int biasfree, int dtype, void* stream) {
  if (!x || !w || !y || !mu || !rstd || N <= 0 || C <= 0 || HW <= 0 || (!biasfree && !b)) return -1;
  TT_DISPATCH(dtype, ln_fwd, x, w, b, y, mu, rstd, N, C, HW, biasfree, (hipStream_t)stream);
}

int turtle_train_ln_bwd(const void* x, const float* w, const float* mu, const float* rstd, const void* dy, void* dx,
                        float* dw, float* db, int64_t N, int C, int64_t HW, int biasfree, int dtype, void* stream) {
  if (!x || !w || !mu || !rstd || !dy || !dx || !dw || N <= 0 || C <= 0 || HW <= 0) return -1;
  TT_DISPATCH(dtype, ln_bwd, x, w, mu, rstd, dy, dx, dw, biasfree ? nullptr : db, N, C, HW, biasfree, (hipStream_t)stream);
}

int turtle_train_dw3x3_fwd(const void* x, const float* w, const float* b, void* y, int64_t N, int C, int H, int W, int flip,
                           int dtype, void* stream) {
  if (!x || !w || !y || N <= 0 || C <= 0 || H <= 0 || W <= 0 || N * C > 65535) return -1;
  TT_DISPATCH(dtype, dw_fwd, x, w, b, y, N, C, H, W, flip, (hipStream_t)stream);
}

int turtle_train_dw3x3_wgrad(const void* x, const void* dy, float* dw, float* db, int64_t N, int C, int H, int W, int dtype,
                             void* stream) {
  if (!x || !dy || !dw || N <= 0 || C <= 0 || H <= 0 || W <= 0 || N * C > 65535) return -1;
  TT_DISPATCH(dtype, dw_wgrad, x, dy, dw, db, N, C, H, W, (hipStream_t)stream);
}

int turtle_train_gate_fwd(const void* x, void* y, int64_t N, int h, int64_t HW, int dtype, void* stream) {
  if (!x || !y || N <= 0 || h <= 0 || HW <= 0) return -1;
  TT_DISPATCH(dtype, gate_fwd, x, y, N, h, HW, (hipStream_t)stream);
}

int turtle_train_gate_bwd(const void* x, const void* dy, void* dx, int64_t N, int h, int64_t HW, int dtype, void* stream) {
  if (!x || !dy || !dx || N <= 0 || h <= 0 || HW <= 0) return -1;
  TT_DISPATCH(dtype, gate_bwd, x, dy, dx, N, h, HW, (hipStream_t)stream);
}

}  // extern "C"

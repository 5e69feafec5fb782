// t0 StateAlignBlock (basicsr/models/archs/turtle_arch.py:459-533) on CDNA4.
//
// The t0 network's aligner computes an attention and then discards it (`out = v`, 521-523), so
// its live data path is: k = normalize(dilated(dw(qk(x + pos))[k half])) for the cache, and
// out = project_out(v) of every cached + current frame. The pointwise/depthwise parts run on the
// shared fused / GEMM / depthwise kernels; this file holds the three pieces specific to t0:
//   * t0_pe:    the 2-D sinusoidal encoding (positionalencoding2d, turtle_arch.py:412-439),
//               generated on the device per level shape, pixel-major [H*W][C];
//   * t0_knorm: adds dw(W_k pe) (the encoding's contribution, linear through the 1x1 and the
//               zero-padded 3x3, pre-transformed into the dilated token layout) to the cached k
//               tokens and L2-normalises each token over its ws*ws*C features (F.normalize);
//   * t0_untok: inverse dilated regroup 'b t 1 (h w) (p1 p2 d) -> (b t) d (p1 h) (p2 w)' of the
//               v tokens of every frame into pixel-major frames for the project_out/kv GEMM.
// All three are HBM-bound streaming kernels (16-byte vector accesses, fp32 arithmetic).
#include "kernels.h"

namespace turtle {

template <typename T>
__global__ __launch_bounds__(256) void t0_pe_kernel(T0PeArgs a) {
  const int half = a.C / 2;
  // torch: div = exp(arange(0, half, 2) * -(log(10000) / half)) in fp32
  const float sc = (float)(-(9.210340371976184 / (double)half));   // log(10000) = 9.2103...
  const int64_t total = (int64_t)a.H * a.W * a.C;
  T* out = reinterpret_cast<T*>(a.out);
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int ch = (int)(e % a.C);
    const int64_t p = e / a.C;
    const int y = (int)(p / a.W), x = (int)(p % a.W);
    const int cc = ch < half ? ch : ch - half;
    const float div = expf((float)(cc & ~1) * sc);
    const float arg = (float)(ch < half ? x : y) * div;
    out[e] = from_f<T>((cc & 1) ? cosf(arg) : sinf(arg));
  }
}

template <typename T>
__global__ __launch_bounds__(256) void t0_knorm_kernel(T0KnormArgs a) {
  constexpr int VEC = Vec<T>::N;
  __shared__ float ss[4];
  const int b = blockIdx.x / a.N, n = blockIdx.x % a.N, tid = threadIdx.x;
  T* k = reinterpret_cast<T*>(a.k) + b * a.k_bstride + (int64_t)n * a.D;
  const T* kp = reinterpret_cast<const T*>(a.kpos) + (int64_t)n * a.D;
  float s = 0.f;
  for (int f = tid * VEC; f < a.D; f += 256 * VEC) {
    Vec<T> u, v;
    u.load(k + f); v.load(kp + f);
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      const float z = to_f(from_f<T>(u.v[i] + v.v[i]));   // k as stored (bf16 pipeline: rounded)
      s += z * z;
    }
  }
  s = wave_sum(s);
  if ((tid & 63) == 0) ss[tid >> 6] = s;
  __syncthreads();
  const float inv = 1.f / fmaxf(sqrtf(ss[0] + ss[1] + ss[2] + ss[3]), 1e-12f);
  for (int f = tid * VEC; f < a.D; f += 256 * VEC) {
    Vec<T> u, v;
    u.load(k + f); v.load(kp + f);
#pragma unroll
    for (int i = 0; i < VEC; ++i) u.v[i] = to_f(from_f<T>(u.v[i] + v.v[i])) * inv;
    u.store(k + f);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void t0_untok_kernel(T0UntokArgs a) {
  constexpr int VEC = Vec<T>::N;
  const int cv = a.C / VEC;
  const int hh = a.H / a.ws, ww = a.W / a.ws;
  const int64_t D = (int64_t)a.ws * a.ws * a.C;
  const int64_t per_img = (int64_t)a.H * a.W * cv;
  const int64_t total = per_img * a.B * a.T;
  T* out = reinterpret_cast<T*>(a.out);
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t img = e / per_img, r = e % per_img;
    const int b = (int)(img / a.T), t = (int)(img % a.T);
    const int c0 = (int)(r % cv) * VEC;
    const int64_t p = r / cv;
    const int y = (int)(p / a.W), x = (int)(p % a.W);
    const int p1 = y / hh, i = y - p1 * hh, p2 = x / ww, j = x - p2 * ww;
    const T* src = reinterpret_cast<const T*>(a.v[t]) + b * a.v_bstride[t] + ((int64_t)i * ww + j) * D +
                   (int64_t)(p1 * a.ws + p2) * a.C + c0;
    Vec<T> v;
    v.load(src);
    v.store(out + (img * a.H * a.W + p) * a.C + c0);
  }
}

static unsigned grid_for(int64_t n) {
  const int64_t g = (n + 255) / 256;
  return (unsigned)(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

template <typename T>
void launch_t0_pe(const T0PeArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(t0_pe_kernel<T>, dim3(grid_for((int64_t)a.H * a.W * a.C)), dim3(256), 0, st, a);
}

template <typename T>
void launch_t0_knorm(const T0KnormArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(t0_knorm_kernel<T>, dim3((unsigned)(a.B * a.N)), dim3(256), 0, st, a);
}

template <typename T>
void launch_t0_untok(const T0UntokArgs& a, hipStream_t st) {
  const int64_t n = (int64_t)a.B * a.T * a.H * a.W * (a.C / Vec<T>::N);
  hipLaunchKernelGGL(t0_untok_kernel<T>, dim3(grid_for(n)), dim3(256), 0, st, a);
}

#define INST(T)                                                        \
  template void launch_t0_pe<T>(const T0PeArgs&, hipStream_t);        \
  template void launch_t0_knorm<T>(const T0KnormArgs&, hipStream_t);  \
  template void launch_t0_untok<T>(const T0UntokArgs&, hipStream_t);
INST(float)
INST(bf16)

}  // namespace turtle

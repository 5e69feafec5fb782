// Training-path kernels with hand-written backward (include/turtle_train.h). The training graph
// (turtlevsr_amd/train.py) holds its activations channels-last (NHWC: a pixel's channels
// contiguous, the inference path's layout), so every kernel here reads and writes pixel rows with a
// row stride `ld` (elements) and fp32 / bf16 / fp16 storage, fp32 arithmetic:
//
//   channel LayerNorm   y = (x - mu) rstd w + b (BiasFree: x rstd w) per pixel over C
//                       (turtle_t1_arch.py:67-112); backward dx, dw, db
//   depthwise 3x3       y = dw3x3(x) + b, pad 1 (qkv_dwconv / conv2 / dwconv / kv_dwconv); dgrad =
//                       the same stencil with the taps rotated 180 degrees; wgrad dw, db
//   GELU gate           y = gelu(x1) x2 over the two channel halves (GatedFeedForward 176)
//   column sums         db[n] = sum_p dy[p][n] (1x1 conv bias gradients)
//   reduction GEMM      C[img][n][k] = sum_p A[p][n] B[p][k] over the pixels of each image (or of
//                       all images): 1x1 conv weight gradients (dW = dY^T X), the channel
//                       attention Gram (q^T k over HW) and its backward. bf16 on the matrix cores:
//                       pixel-major tiles staged in LDS, both operands read with the gfx950
//                       transposing LDS read (ds_read_b64_tr_b16) so the contraction runs over
//                       pixels; fp32 partials per pixel split, reduced by a second pass in a fixed
//                       order (deterministic)
//   forward / data GEMM Y[p][n] = sum_k X[p][k] W[n][k] (+ b): the inference GEMM family
//                       (gemm*.hip), per-image weight sets optional (attention W_eff)
//
// Per-channel weight gradients (LN, depthwise, bias) reduce each block's pixels in registers /
// LDS and add one fp32 partial per channel per block with a device atomic into buffers the caller
// zeroed.
#include "common.h"
#include "kernels.h"

#include <type_traits>
#include "../../include/turtle_train.h"

#include <algorithm>
#include <map>
#include <mutex>
#include <vector>

namespace turtle {

__device__ __attribute__((aligned(64))) uint4 g_zero_tw[2];   // zero line for branch-free operand loads

TURTLE_DEV float gelu_exact(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
TURTLE_DEV float gelu_exact_grad(float x) {   // d/dx x Phi(x) = Phi(x) + x phi(x)
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// 8 consecutive elements <-> fp32 (16 B for 2-byte types, 32 B for fp32)
template <typename T> TURTLE_DEV void ld8f(const T* p, float (&v)[8]);
template <> TURTLE_DEV void ld8f<float>(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
template <> TURTLE_DEV void ld8f<bf16>(const bf16* p, float (&v)[8]) {
  const uint4 q = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) { v[2 * i] = __uint_as_float(w[i] << 16); v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u); }
}
template <> TURTLE_DEV void ld8f<f16>(const f16* p, float (&v)[8]) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  const h8 q = *reinterpret_cast<const h8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (float)q[i];
}
template <typename T> TURTLE_DEV void st8f(T* p, const float (&v)[8]) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    typedef T t8 __attribute__((ext_vector_type(8)));
    t8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (T)v[i];
    *reinterpret_cast<t8*>(p) = o;
  }
}

// tools/train_kbench.py ablations (TURTLE_TRAIN_ABL, read once; 0 in the product path):
// bit 0 - skip the end-of-block global atomics of the reduction kernels (ln_bwd, colsum, dw_wgrad)
static int train_abl() {
  static const int v = [] { const char* e = getenv("TURTLE_TRAIN_ABL"); return e ? atoi(e) : 0; }();
  return v;
}
// launch-size sweeps of tools/train_kbench.py (TURTLE_TRAIN_TUNE="ln_blocks,cs_blocks,dwg_blocks,kt_max_px", read once;
// 0 or absent = the built-in choice)
static int train_tune(int i) {
  static const std::vector<int> v = [] {
    std::vector<int> r(4, 0);
    if (const char* e = getenv("TURTLE_TRAIN_TUNE")) sscanf(e, "%d,%d,%d,%d", &r[0], &r[1], &r[2], &r[3]);
    return r;
  }();
  return v[i];
}

template <typename T>
struct Raw8 {                                   // 8 consecutive elements, raw
  uint4 q[sizeof(T) / 2];
  TURTLE_DEV void load(const void* p) {
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 2); ++i) q[i] = reinterpret_cast<const uint4*>(p)[i];
  }
  TURTLE_DEV void unpack(float (&v)[8]) const { ld8f(reinterpret_cast<const T*>(q), v); }
};

// lanes per pixel for a C-channel row: a power of two covering C / 8 chunks (<= 64)
static int ln_group(int C) {
  int g = 1;
  while (g < C / 8 && g < 64) g <<= 1;
  return g;
}
// sum over aligned groups of G lanes, every lane of a group gets the same value: DPP within a row
// (quad swaps, half-row / row mirrors: VALU ops, no LDS round trip), ds_bpermute across rows
template <int CTRL>
TURTLE_DEV float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}
template <int G>
TURTLE_DEV float group_sum(float v) {
  if constexpr (G >= 2) v += dpp_f<0xB1>(v);       // quad_perm [1, 0, 3, 2]
  if constexpr (G >= 4) v += dpp_f<0x4E>(v);       // quad_perm [2, 3, 0, 1]
  if constexpr (G >= 8) v += dpp_f<0x141>(v);      // row_half_mirror: quad q <-> the other quad of the 8
  if constexpr (G >= 16) v += dpp_f<0x140>(v);     // row_mirror: 8-lane half <-> the other half of the row
  if constexpr (G >= 32) v += __shfl_xor(v, 16, 64);
  if constexpr (G >= 64) v += __shfl_xor(v, 32, 64);
  return v;
}

// ---------------------------------------------------------------------------------------------
// channel LayerNorm, NHWC: G lanes per pixel, each lane NCH chunks of 8 channels
// ---------------------------------------------------------------------------------------------
template <typename T, typename TY, int G, int NCH, int U, bool BF>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x, int64_t ldx, const float* __restrict__ w,
                                                     const float* __restrict__ b, TY* __restrict__ y, int64_t ldy,
                                                     float* __restrict__ mu, float* __restrict__ rstd, int64_t P, int C) {
  // U pixels per lane group, strided by the grid's pixel slots (a wave's 64 / G pixels stay adjacent).
  // Every load is unconditional (clamped row / channel, out-of-range values zeroed by a select after
  // the unpack) and issued before the first use: a load inside a per-lane branch makes hipcc wait for
  // it right there, and a load between two stores waits for the stores (vmcnt counts both)
  const int64_t nslots = (int64_t)gridDim.x * (256 / G);
  const int64_t slot = (int64_t)blockIdx.x * (256 / G) + threadIdx.x / G;
  const int l = threadIdx.x % G;
  const float invC = 1.f / C;
  float wv[NCH][8], bv[NCH][8];
  Raw8<T> raw[U][NCH];
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = min(8 * (l + G * j), C - 8);
    ld8f(w + c, wv[j]);
    ld8f(BF ? w + c : b + c, bv[j]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t p = slot + u * nslots;
      raw[u][j].load(x + (p < P ? p : 0) * ldx + c);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t p = slot + u * nslots;
    const bool live = p < P;
    float v[NCH][8];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const bool cin = 8 * (l + G * j) < C;
      raw[u][j].unpack(v[j]);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[j][e] = cin ? v[j][e] : 0.f;
        s += v[j][e];
      }
    }
    const float m = group_sum<G>(s) * invC;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const bool cin = 8 * (l + G * j) < C;
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = cin ? v[j][e] - m : 0.f; q = fmaf(d, d, q); }
    }
    const float r = rsqrtf(group_sum<G>(q) * invC + 1e-5f);
    if (live && l == 0) { mu[p] = m; rstd[p] = r; }
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int c = 8 * (l + G * j);
      if (!live || c >= C) continue;
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = BF ? v[j][e] * r * wv[j][e] : fmaf((v[j][e] - m) * r, wv[j][e], bv[j][e]);
      st8f(y + p * ldy + c, o);
    }
  }
}

// backward: g = w dy;  WithBias: xh = (x - mu) r, dx = r (g - mean(g) - xh mean(g xh));
// BiasFree (y = w x r, r of the centred variance): dx = r g - (x - mu) r^3 mean(g x).
// dw[c] = sum_p dy xhat (BiasFree xhat = x r), db[c] = sum_p dy: per-lane accumulators over the
// block's pixels -> LDS -> one atomic per channel per block. dres (or NULL): the residual use's
// gradient, added into dx.
template <typename T, typename TY, int G, int NCH, int U, bool BF>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const T* __restrict__ x, int64_t ldx, const float* __restrict__ w,
                                                     const float* __restrict__ mu, const float* __restrict__ rstd,
                                                     const TY* __restrict__ dy, int64_t lddy, T* __restrict__ dx, int64_t lddx,
                                                     const T* __restrict__ dres, int64_t lddres,
                                                     float* __restrict__ dw, float* __restrict__ db, int64_t P, int C,
                                                     int ppb, int noatom) {
  extern __shared__ float sred[];                  // [2][C]
  for (int c = threadIdx.x; c < 2 * C; c += 256) sred[c] = 0.f;
  __syncthreads();
  const int l = threadIdx.x % G, slot = threadIdx.x / G, nslot = 256 / G;
  const float invC = 1.f / C;
  float wv[NCH][8], aw[NCH][8], ab[NCH][8];
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = 8 * (l + G * j);
    ld8f(w + min(c, C - 8), wv[j]);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      wv[j][e] = c < C ? wv[j][e] : 0.f;           // lanes past C: gamma 0 -> no contribution
      aw[j][e] = ab[j][e] = 0.f;
    }
  }
  const int64_t p0 = (int64_t)blockIdx.x * ppb;
  const int64_t p1 = min(P, p0 + ppb);
  // U pixels per lane group per trip (block pixel slots, then U of those strides): every row load of
  // the trip is unconditional (clamped) and in flight before the first reduction
  for (int64_t pb = p0; pb < p1; pb += nslot * U) {     // uniform trip count across the block
    Raw8<T> rx[U][NCH], rr[U][NCH];
    Raw8<TY> rg[U][NCH];
    float m[U], r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t p = pb + slot + u * nslot;
      const int64_t pp = p < p1 ? p : p0;
      m[u] = mu[pp];
      r[u] = rstd[pp];
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        const int c = min(8 * (l + G * j), C - 8);
        rx[u][j].load(x + pp * ldx + c);
        rg[u][j].load(dy + pp * lddy + c);
      }
    }
    if (dres) {                                    // uniform: the residual gradient rows
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t p = pb + slot + u * nslot;
        const int64_t pp = p < p1 ? p : p0;
#pragma unroll
        for (int j = 0; j < NCH; ++j) rr[u][j].load(dres + pp * lddres + min(8 * (l + G * j), C - 8));
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t p = pb + slot + u * nslot;
      const bool live = p < p1;
      const float mm = m[u], rs = r[u];
      float xv[NCH][8], gy[NCH][8];
      float sg = 0.f, sgx = 0.f;
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        rx[u][j].unpack(xv[j]);
        rg[u][j].unpack(gy[j]);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float g = wv[j][e] * gy[j][e];
          sg += g;
          sgx = fmaf(g, BF ? xv[j][e] : (xv[j][e] - mm) * rs, sgx);
        }
      }
      const float mg = group_sum<G>(sg) * invC, mgx = group_sum<G>(sgx) * invC;
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        const int c = 8 * (l + G * j);
        float o[8], res[8];
        if (dres) rr[u][j].unpack(res);
        else {
#pragma unroll
          for (int e = 0; e < 8; ++e) res[e] = 0.f;
        }
        const bool ok = live && c < C;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float g = wv[j][e] * gy[j][e];
          const float xe = xv[j][e];
          o[e] = res[e] + (BF ? rs * g - (xe - mm) * rs * rs * rs * mgx : rs * (g - mg - (xe - mm) * rs * mgx));
          aw[j][e] = fmaf(ok ? gy[j][e] : 0.f, BF ? xe * rs : (xe - mm) * rs, aw[j][e]);
          ab[j][e] += ok ? gy[j][e] : 0.f;
        }
        if (ok) st8f(dx + p * lddx + c, o);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = 8 * (l + G * j);
    if (c >= C) continue;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      atomicAdd(&sred[c + e], aw[j][e]);
      atomicAdd(&sred[C + c + e], ab[j][e]);
    }
  }
  __syncthreads();
  if (noatom) return;
  for (int c = threadIdx.x; c < C; c += 256) {
    atomicAdd(&dw[c], sred[c]);
    if (db) atomicAdd(&db[c], sred[C + c]);
  }
}

// ---------------------------------------------------------------------------------------------
// depthwise 3x3, pad 1, NHWC: one thread per (pixel, 8-channel chunk); w9 tap-major [9][C] fp32
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void dw_fwd_kernel(const T* __restrict__ x, int64_t ldx, const float* __restrict__ w9,
                                                     const float* __restrict__ b, T* __restrict__ y, int64_t ldy, int64_t N,
                                                     int C, int H, int W, int flip) {
  const int nch = C / 8;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t tot = N * H * W * nch;
  if (gid >= tot) return;
  const int ch = (int)(gid % nch);
  const int64_t pix = gid / nch;
  const int xx = (int)(pix % W);
  const int64_t t = pix / W;
  const int yy = (int)(t % H);
  const int64_t n = t / H;
  const int c = 8 * ch;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = b ? b[c + e] : 0.f;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int sy = yy + tap / 3 - 1, sx = xx + tap % 3 - 1;
    if (sy < 0 || sy >= H || sx < 0 || sx >= W) continue;
    float v[8];
    ld8f(x + ((n * H + sy) * W + sx) * ldx + c, v);
    const float* wt = w9 + (flip ? 8 - tap : tap) * C + c;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = fmaf(wt[e], v[e], acc[e]);
  }
  st8f(y + pix * ldy + c, acc);
}

// dw9[t][c] = sum dy[n,y,x,c] x[n, y + dy_t, x + dx_t, c], db[c] = sum dy: a block takes a slice
// of CPB 8-channel chunks (blockIdx.y) and a contiguous pixel range (blockIdx.x); thread = (chunk,
// pixel lane), 80 accumulators, LDS block reduction, one atomic per (tap, channel) per block
constexpr int DWG_CPB = 32;
template <typename T>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(const T* __restrict__ x, int64_t ldx, const T* __restrict__ dy,
                                                       int64_t lddy, float* __restrict__ dw9, float* __restrict__ db,
                                                       int64_t N, int C, int H, int W, int64_t ppb) {
  __shared__ float sred[10 * DWG_CPB * 8];
  for (int i = threadIdx.x; i < 10 * DWG_CPB * 8; i += 256) sred[i] = 0.f;
  __syncthreads();
  const int nch = min(C / 8 - (int)blockIdx.y * DWG_CPB, DWG_CPB);   // chunks in this slice
  const int lanes = 256 / nch;                     // pixel lanes per block
  const int ch = threadIdx.x % nch, pl = threadIdx.x / nch;
  const int c = 8 * ((int)blockIdx.y * DWG_CPB + ch), cl = 8 * ch;   // global / slice channel
  float a[10][8];
#pragma unroll
  for (int t = 0; t < 10; ++t)
#pragma unroll
    for (int e = 0; e < 8; ++e) a[t][e] = 0.f;
  const int64_t P = N * H * W;
  const int64_t p0 = (int64_t)blockIdx.x * ppb, p1 = min(P, p0 + ppb);
  if (pl < lanes) {
    for (int64_t pix = p0 + pl; pix < p1; pix += lanes) {
      const int xx = (int)(pix % W);
      const int64_t t = pix / W;
      const int yy = (int)(t % H);
      const int64_t n = t / H;
      float g[8];
      ld8f(dy + pix * lddy + c, g);
#pragma unroll
      for (int e = 0; e < 8; ++e) a[9][e] += g[e];
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int sy = yy + tap / 3 - 1, sx = xx + tap % 3 - 1;
        if (sy < 0 || sy >= H || sx < 0 || sx >= W) continue;
        float v[8];
        ld8f(x + ((n * H + sy) * W + sx) * ldx + c, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) a[tap][e] = fmaf(g[e], v[e], a[tap][e]);
      }
    }
#pragma unroll
    for (int t = 0; t < 10; ++t)
#pragma unroll
      for (int e = 0; e < 8; ++e) atomicAdd(&sred[(t * DWG_CPB * 8) + cl + e], a[t][e]);
  }
  __syncthreads();
  const int c0 = (int)blockIdx.y * DWG_CPB * 8, ncl = nch * 8;
  for (int i = threadIdx.x; i < 10 * ncl; i += 256) {
    const int t = i / ncl, j = i - t * ncl;
    if (t < 9) atomicAdd(&dw9[t * C + c0 + j], sred[t * DWG_CPB * 8 + j]);
    else if (db) atomicAdd(&db[c0 + j], sred[9 * DWG_CPB * 8 + j]);
  }
}

// Row-sweeping depthwise weight gradient (the forward's dw_rows geometry, spatial.hip): a block
// owns a (32-column strip) x (64 channels) x (band of RB rows) box of one image, thread =
// (column, 8-channel vector); walking down the band it keeps the 3 x 3 x-neighbourhood of its
// column as a rolling window of three rows (raw, one new row loaded ahead of the math) and
// accumulates dw9[t] += dy * x[p + off_t], db += dy. Column sums by cross-lane shuffles, the 4
// waves meet in LDS, one global atomic per (tap, channel) per block.
constexpr int TW_SX = 32, TW_CV = 8;
template <typename T>
__global__ __launch_bounds__(256) void dw_wgrad_rows_kernel(const T* __restrict__ x, int64_t ldx, const T* __restrict__ dy,
                                                            int64_t lddy, float* __restrict__ dw9, float* __restrict__ db,
                                                            int C, int H, int W, int RB, int nstrip, int nchunk, int nband,
                                                            int noatom) {
  __shared__ float sred[10][TW_CV * 8];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < 10 * TW_CV * 8; i += 256) (&sred[0][0])[i] = 0.f;
  int t = blockIdx.x;
  const int band = t % nband;
  t /= nband;
  const int strip = t % nstrip;
  t /= nstrip;
  const int chunk = t % nchunk;
  const int64_t img = t / nchunk;
  const int cvl = tid % TW_CV, xs = tid / TW_CV;
  const int CV = C / 8;
  const int xcol = strip * TW_SX + xs, cv = chunk * TW_CV + cvl;
  const bool live = xcol < W && cv < CV;
  const int xc = min(xcol, W - 1), c0 = min(cv, CV - 1) * 8;
  const int y0 = band * RB, y1 = min(H, y0 + RB);
  const T* xin = x + img * H * W * ldx + c0;
  const T* gin = dy + img * H * W * lddy + c0;
  const bool okl = xc > 0, okr = xc + 1 < W;
  auto load_row = [&](int y, Raw8<T> (&r)[3]) {
    const bool oky = y >= 0 && y < H;
    const T* p = xin + ((int64_t)(oky ? y : 0) * W + xc) * ldx;
    r[0].load(oky && okl ? reinterpret_cast<const void*>(p - ldx) : g_zero_tw);
    r[1].load(oky ? reinterpret_cast<const void*>(p) : g_zero_tw);
    r[2].load(oky && okr ? reinterpret_cast<const void*>(p + ldx) : g_zero_tw);
  };
  float a[10][8];
#pragma unroll
  for (int k = 0; k < 10; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) a[k][e] = 0.f;
  // dy row y + 1 and x row y + 2 are loaded while row y is consumed; every load unconditional (rows
  // past the band / image read the zero line): a conditional load makes hipcc wait for it in place
  auto dy_row = [&](int y) {
    return live && y < y1 ? reinterpret_cast<const void*>(gin + ((int64_t)y * W + xc) * lddy) : g_zero_tw;
  };
  Raw8<T> w0[3], w1[3], w2[3], nx[3], gr, gn;
  load_row(y0 - 1, w0);
  load_row(y0, w1);
  load_row(y0 + 1, w2);
  gr.load(dy_row(y0));
  for (int y = y0; y < y1; ++y) {
    load_row(y + 2, nx);
    gn.load(dy_row(y + 1));
    float g[8];
    gr.unpack(g);
#pragma unroll
    for (int e = 0; e < 8; ++e) a[9][e] += g[e];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const Raw8<T>& q = tap < 3 ? w0[tap] : tap < 6 ? w1[tap - 3] : w2[tap - 6];
      float v[8];
      q.unpack(v);
#pragma unroll
      for (int e = 0; e < 8; ++e) a[tap][e] = fmaf(g[e], v[e], a[tap][e]);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) { w0[k] = w1[k]; w1[k] = w2[k]; w2[k] = nx[k]; }
    gr = gn;
  }
  // sum over the 8 columns of a wave (lane bits 3..5), then over the 4 waves in LDS
#pragma unroll
  for (int k = 0; k < 10; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = a[k][e];
      v += __shfl_xor(v, 8, 64);
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      a[k][e] = v;
    }
  __syncthreads();
  if (lane < TW_CV) {
#pragma unroll
    for (int k = 0; k < 10; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) atomicAdd(&sred[k][lane * 8 + e], a[k][e]);
  }
  __syncthreads();
  if (noatom) return;
  for (int i = tid; i < 10 * TW_CV * 8; i += 256) {
    const int k = i / (TW_CV * 8), j = i - k * TW_CV * 8, c = chunk * TW_CV * 8 + j;
    if (c >= C) continue;
    if (k < 9) atomicAdd(&dw9[k * C + c], sred[k][j]);
    else if (db) atomicAdd(&db[c], sred[9][j]);
  }
}

// ---------------------------------------------------------------------------------------------
// GELU gate, NHWC: x [P][ldx] (x1 = channels [0, h), x2 = [h, 2h)) -> y [P][ldy] (h channels)
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void gate_fwd_kernel(const T* __restrict__ x, int64_t ldx, T* __restrict__ y, int64_t ldy,
                                                       int64_t P, int h) {
  const int nch = h / 8;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= P * nch) return;
  const int64_t p = gid / nch;
  const int c = 8 * (int)(gid % nch);
  float a[8], b[8], o[8];
  ld8f(x + p * ldx + c, a);
  ld8f(x + p * ldx + h + c, b);
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = gelu_exact(a[e]) * b[e];
  st8f(y + p * ldy + c, o);
}
template <typename T>
__global__ __launch_bounds__(256) void gate_bwd_kernel(const T* __restrict__ x, int64_t ldx, const T* __restrict__ dy, int64_t lddy,
                                                       T* __restrict__ dx, int64_t lddx, int64_t P, int h) {
  const int nch = h / 8;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= P * nch) return;
  const int64_t p = gid / nch;
  const int c = 8 * (int)(gid % nch);
  float a[8], b[8], g[8], o1[8], o2[8];
  ld8f(x + p * ldx + c, a);
  ld8f(x + p * ldx + h + c, b);
  ld8f(dy + p * lddy + c, g);
#pragma unroll
  for (int e = 0; e < 8; ++e) { o1[e] = g[e] * b[e] * gelu_exact_grad(a[e]); o2[e] = g[e] * gelu_exact(a[e]); }
  st8f(dx + p * lddx + c, o1);
  st8f(dx + p * lddx + h + c, o2);
}

// plain GELU (exact erf form; FeedForward 181-210 after conv4, ReducedAttn 704-742 after conv2):
// y = gelu(x); backward dx = dy gelu'(x)
template <typename T>
__global__ __launch_bounds__(256) void gelu_fwd_kernel(const T* __restrict__ x, int64_t ldx, T* __restrict__ y, int64_t ldy,
                                                       int64_t P, int C) {
  const int nch = C / 8;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= P * nch) return;
  const int64_t p = gid / nch;
  const int c = 8 * (int)(gid % nch);
  float a[8], o[8];
  ld8f(x + p * ldx + c, a);
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = gelu_exact(a[e]);
  st8f(y + p * ldy + c, o);
}
template <typename T>
__global__ __launch_bounds__(256) void gelu_bwd_kernel(const T* __restrict__ x, int64_t ldx, const T* __restrict__ dy, int64_t lddy,
                                                       T* __restrict__ dx, int64_t lddx, int64_t P, int C) {
  const int nch = C / 8;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= P * nch) return;
  const int64_t p = gid / nch;
  const int c = 8 * (int)(gid % nch);
  float a[8], g[8], o[8];
  ld8f(x + p * ldx + c, a);
  ld8f(dy + p * lddy + c, g);
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = g[e] * gelu_exact_grad(a[e]);
  st8f(dx + p * lddx + c, o);
}

// ---------------------------------------------------------------------------------------------
// SAB window convolution (k2_dwconv / q2_dwconv, turtle_t1_arch.py:306-308, 560-571):
// nn.Conv2d(C, C, ws, stride=ws, padding=1, groups=C) on NHWC rows. Token (i, j) of the th x tw
// output grid covers input rows i ws - 1 .. i ws + ws - 2 and columns j ws - 1 .. (zero padding
// outside; the last input rows / columns past the grid are not read). Weights transposed on the
// host to wt [ws*ws][C] fp32 (tap-major: 8 channels of a tap are one 32-byte read).
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void win_fwd_kernel(const T* __restrict__ x, int64_t ldx, const float* __restrict__ wt,
                                                      const float* __restrict__ b, T* __restrict__ y, int64_t ldy, int64_t N,
                                                      int C, int H, int W, int ws, int th, int tw) {
  const int nch = C / 8;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= N * th * tw * nch) return;
  const int c = 8 * (int)(gid % nch);
  const int64_t t = gid / nch;                     // token row of y: (img, i, j)
  const int j = (int)(t % tw), i = (int)((t / tw) % th);
  const int64_t img = t / ((int64_t)tw * th);
  float acc[8];
  if (b) {
    const float4 b0 = *reinterpret_cast<const float4*>(b + c), b1 = *reinterpret_cast<const float4*>(b + c + 4);
    acc[0] = b0.x; acc[1] = b0.y; acc[2] = b0.z; acc[3] = b0.w; acc[4] = b1.x; acc[5] = b1.y; acc[6] = b1.z; acc[7] = b1.w;
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  }
  const int y0 = i * ws - 1, x0 = j * ws - 1;
  for (int u = 0; u < ws; ++u) {
    const int yy = y0 + u;
    if (yy < 0 || yy >= H) continue;
    const T* row = x + ((img * H + yy) * W) * ldx + c;
    for (int v = 0; v < ws; ++v) {
      const int xx = x0 + v;
      if (xx < 0 || xx >= W) continue;
      float a[8];
      ld8f(row + (int64_t)xx * ldx, a);
      const float* wp = wt + (int64_t)(u * ws + v) * C + c;
      const float4 w0 = *reinterpret_cast<const float4*>(wp), w1 = *reinterpret_cast<const float4*>(wp + 4);
      const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = fmaf(a[e], wv[e], acc[e]);
    }
  }
  st8f(y + t * ldy + c, acc);
}
// input gradient: every input pixel feeds exactly one token (or none): dx = dy[token] wt[tap]
template <typename T>
__global__ __launch_bounds__(256) void win_dgrad_kernel(const T* __restrict__ dy, int64_t lddy, const float* __restrict__ wt,
                                                        T* __restrict__ dx, int64_t lddx, int64_t N, int C, int H, int W, int ws,
                                                        int th, int tw) {
  const int nch = C / 8;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= N * H * W * nch) return;
  const int c = 8 * (int)(gid % nch);
  const int64_t p = gid / nch;
  const int xx = (int)(p % W), yy = (int)((p / W) % H);
  const int64_t img = p / ((int64_t)W * H);
  const int i = (yy + 1) / ws, u = (yy + 1) - i * ws, j = (xx + 1) / ws, v = (xx + 1) - j * ws;
  float o[8];
  if (i < th && j < tw) {
    float g[8];
    ld8f(dy + ((img * th + i) * tw + j) * lddy + c, g);
    const float* wp = wt + (int64_t)(u * ws + v) * C + c;
    const float4 w0 = *reinterpret_cast<const float4*>(wp), w1 = *reinterpret_cast<const float4*>(wp + 4);
    const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = g[e] * wv[e];
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.f;
  }
  st8f(dx + p * lddx + c, o);
}
// weight gradient dwt[tap][c] += sum over (img, token) of dy[token][c] x[pixel(token, tap)][c]: block
// = (tap, 64-channel chunk, token split); thread = (token lane 0..31, channel vector 0..7); token-lane
// partials reduced by shuffles inside a wave and through LDS across the 4 waves, one fp32 atomic
// add per (tap, channel) and block into the caller-zeroed dwt
template <typename T>
__global__ __launch_bounds__(256) void win_wgrad_kernel(const T* __restrict__ x, int64_t ldx, const T* __restrict__ dy,
                                                        int64_t lddy, float* __restrict__ dwt, int64_t N, int C, int H, int W,
                                                        int ws, int th, int tw, int64_t tpb) {
  __shared__ float red[4][64];
  const int tap = blockIdx.x, u = tap / ws, v = tap - u * ws;
  const int cv = threadIdx.x & 7, tl = threadIdx.x >> 3;         // channel vector, token lane (0..31)
  const int c = blockIdx.y * 64 + cv * 8;
  const int64_t ntok = N * th * tw;
  const int64_t t0 = (int64_t)blockIdx.z * tpb, t1 = min(ntok, t0 + tpb);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    for (int64_t t = t0 + tl; t < t1; t += 32) {
      const int j = (int)(t % tw), i = (int)((t / tw) % th);
      const int64_t img = t / ((int64_t)tw * th);
      const int yy = i * ws - 1 + u, xx = j * ws - 1 + v;
      if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
      float a[8], g[8];
      ld8f(x + ((img * H + yy) * W + xx) * ldx + c, a);
      ld8f(dy + t * lddy + c, g);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = fmaf(a[e], g[e], acc[e]);
    }
  }
  // token lanes tl and tl ^ 1, ^ 2, ^ 4 share a wave (lane = 8 tl + cv): xor 8, 16, 32
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    acc[e] += __shfl_xor(acc[e], 8, 64);
    acc[e] += __shfl_xor(acc[e], 16, 64);
    acc[e] += __shfl_xor(acc[e], 32, 64);
  }
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane < 8)
#pragma unroll
    for (int e = 0; e < 8; ++e) red[wv][lane * 8 + e] = acc[e];
  __syncthreads();
  if (threadIdx.x < 64) {
    const int cc = blockIdx.y * 64 + threadIdx.x;
    const float s = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
    if (cc < C) atomicAdd(dwt + (int64_t)tap * C + cc, s);
  }
}

// Per-image column L2 normalisation over the pixels (F.normalize(x, dim=-1) of a [b, heads, ch, HW]
// view, turtle_t1_arch.py:236-237 / 649-651, on NHWC rows): y[p][c] = x[p][c] s[img(p)][c] with
// s = 1 / max(|x_col|, 1e-12); backward dx = (dy - y d) s with d[img][c] = sum_p dy y (0 where the clamp
// was active, whose norm gets no gradient)
template <typename T>
__global__ __launch_bounds__(256) void colscale_kernel(const T* __restrict__ x, int64_t ldx, const float* __restrict__ s,
                                                       T* __restrict__ y, int64_t ldy, int64_t P, int C, int64_t img_px) {
  const int nch = C / 8;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= P * nch) return;
  const int64_t p = gid / nch;
  const int c = 8 * (int)(gid % nch);
  const float* sp = s + (p / img_px) * C + c;
  float v[8];
  ld8f(x + p * ldx + c, v);
  const float4 s0 = *reinterpret_cast<const float4*>(sp), s1 = *reinterpret_cast<const float4*>(sp + 4);
  const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] *= sv[e];
  st8f(y + p * ldy + c, v);
}
template <typename T>
__global__ __launch_bounds__(256) void l2n_bwd_kernel(const T* __restrict__ dy, int64_t lddy, const T* __restrict__ y, int64_t ldy,
                                                      const float* __restrict__ d, const float* __restrict__ s, T* __restrict__ dx,
                                                      int64_t lddx, int64_t P, int C, int64_t img_px) {
  const int nch = C / 8;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= P * nch) return;
  const int64_t p = gid / nch;
  const int c = 8 * (int)(gid % nch);
  const int64_t o = (p / img_px) * C + c;
  float g[8], v[8];
  ld8f(dy + p * lddy + c, g);
  ld8f(y + p * ldy + c, v);
  const float4 d0 = *reinterpret_cast<const float4*>(d + o), d1 = *reinterpret_cast<const float4*>(d + o + 4);
  const float4 s0 = *reinterpret_cast<const float4*>(s + o), s1 = *reinterpret_cast<const float4*>(s + o + 4);
  const float dv[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
  const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
  for (int e = 0; e < 8; ++e) g[e] = (g[e] - v[e] * dv[e]) * sv[e];
  st8f(dx + p * lddx + c, g);
}

// ---------------------------------------------------------------------------------------------
// StateAlignBlock score -> attention row (turtle_t1_arch.py:394-416 top-5, 448-464 L1 ball,
// 115-132 clipped_softmax, as used in 585-599): per row i of s [R][n] (n keys, rows ordered (b, t,
// i)), m_j = [j in top-5 of the row] + [|dy| + |dx| <= radius on the th x tw token grid] (0 / 1 / 2,
// the reference's s * (top + ball)), se = s m, entries with se == 0 masked, a = softmax over the rest,
// renormalised. One wave per row, NV keys per lane (j = lane + 64 q). Writes a (output dtype) and
// a fp32 + m (uint8) for the backward ds_j = m_j a_j (da_j - sum_k da_k a_k) (the clipped softmax's
// renormalisation and masks differentiated: train_ops._SabSoftmax).
// ---------------------------------------------------------------------------------------------
TURTLE_DEV float wave_max_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
TURTLE_DEV float wave_sum_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <int NV, typename TO>
__global__ __launch_bounds__(256) void sab_softmax_fwd_kernel(const float* __restrict__ s, int64_t R, int n, int tw, int radius,
                                                              TO* __restrict__ a_out, float* __restrict__ a_save,
                                                              uint8_t* __restrict__ m_save) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;                              // wave-uniform
  const int i = (int)(r % n), qy = i / tw, qx = i - (i / tw) * tw;
  const float* sr = s + r * n;
  float v[NV];
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    const int j = lane + 64 * q;
    v[q] = j < n ? sr[j] : -INFINITY;
  }
  // top-5: five wave-wide arg-max rounds (largest value, lowest index on ties), the winner excluded
  unsigned sel = 0;
  for (int kk = 0; kk < 5 && kk < n; ++kk) {
    float best = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int j = lane + 64 * q;
      if (j < n && !((sel >> q) & 1u) && (v[q] > best || (v[q] == best && j < bi) || bi == 0x7fffffff)) { best = v[q]; bi = j; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
    }
    if (bi != 0x7fffffff && (bi & 63) == lane) sel |= 1u << (bi >> 6);
  }
  float se[NV], mk[NV];
  float mx = -INFINITY;
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    const int j = lane + 64 * q;
    const int ky = j / tw, kx = j - (j / tw) * tw;
    const int dd = abs(ky - qy) + abs(kx - qx);
    mk[q] = j < n ? (float)((sel >> q) & 1u) + (dd <= radius ? 1.f : 0.f) : 0.f;
    se[q] = j < n ? v[q] * mk[q] : 0.f;
    if (se[q] != 0.f) mx = fmaxf(mx, se[q]);
  }
  mx = wave_max_f(mx);
  float e[NV], sum = 0.f;
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    e[q] = se[q] != 0.f ? __expf(se[q] - mx) : 0.f;
    sum += e[q];
  }
  sum = wave_sum_f(sum);
  float ps = 0.f;
#pragma unroll
  for (int q = 0; q < NV; ++q) { e[q] = e[q] / sum; ps += e[q]; }
  ps = wave_sum_f(ps);
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    const int j = lane + 64 * q;
    if (j >= n) continue;
    const float a = e[q] / ps;
    a_out[r * n + j] = (TO)a;
    a_save[r * n + j] = a;
    m_save[r * n + j] = (uint8_t)(se[q] != 0.f ? mk[q] : 0.f);
  }
}
template <int NV, typename TG>
__global__ __launch_bounds__(256) void sab_softmax_bwd_kernel(const TG* __restrict__ da, const float* __restrict__ a_save,
                                                              const uint8_t* __restrict__ m_save, int64_t R, int n,
                                                              float* __restrict__ ds) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  float g[NV], a[NV], dot = 0.f;
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    const int j = lane + 64 * q;
    g[q] = j < n ? (float)da[r * n + j] : 0.f;
    a[q] = j < n ? a_save[r * n + j] : 0.f;
    dot = fmaf(g[q], a[q], dot);
  }
  dot = wave_sum_f(dot);
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    const int j = lane + 64 * q;
    if (j < n) ds[r * n + j] = (float)m_save[r * n + j] * a[q] * (g[q] - dot);
  }
}

// column sums db[n] = sum_p dy[p][n] (8 channels per thread, pixel lanes, LDS reduction, atomics);
// MODE 1: sums of squares; MODE 2: column dot products sum_p dy[p][n] dy2[p][n]
template <typename T, int MODE, int NT = 256>
__global__ __launch_bounds__(NT) void colsum_kernel(const T* __restrict__ dy, int64_t ld, float* __restrict__ db, int64_t P,
                                                    int N, int64_t ppb, const T* __restrict__ dy2, int64_t ld2, int noatom) {
  extern __shared__ float sred[];
  dy += (int64_t)blockIdx.y * P * ld;              // image blockIdx.y of P pixels (one image: y = 0)
  if (MODE == 2) dy2 += (int64_t)blockIdx.y * P * ld2;
  db += (int64_t)blockIdx.y * N;
  for (int i = threadIdx.x; i < N; i += NT) sred[i] = 0.f;
  __syncthreads();
  const int nch = N / 8, lanes = NT / nch;
  const int ch = min((int)threadIdx.x % nch, nch - 1), pl = threadIdx.x / nch;
  const bool lane_live = pl < lanes;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int64_t p0 = (int64_t)blockIdx.x * ppb, p1 = min(P, p0 + ppb);
  // 4 pixel rows per trip, all loads unconditional (clamped rows, zeroed by a select after the unpack)
  // and issued before the first add
  for (int64_t pq = p0 + min(pl, lanes - 1); pq < p1; pq += 4 * lanes) {
    Raw8<T> r1[4], r2[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t p = pq + u * lanes;
      const int64_t pp = p < p1 ? p : p0;
      r1[u].load(dy + pp * ld + 8 * ch);
      if constexpr (MODE == 2) r2[u].load(dy2 + pp * ld2 + 8 * ch);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool live = lane_live && pq + u * lanes < p1;
      float v[8], v2[8];
      r1[u].unpack(v);
      if constexpr (MODE == 2) r2[u].unpack(v2);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float t = MODE == 2 ? v[e] * v2[e] : MODE == 1 ? v[e] * v[e] : v[e];
        a[e] += live ? t : 0.f;
      }
    }
  }
  if (lane_live)
#pragma unroll
    for (int e = 0; e < 8; ++e) atomicAdd(&sred[8 * ch + e], a[e]);
  __syncthreads();
  if (noatom) return;
  for (int i = threadIdx.x; i < N; i += NT) atomicAdd(&db[i], sred[i]);
}


// The per-image weight of the normalised channel-attention Gram backward (train_ops._NormGram):
// Wd[b] = [[diag(aq[b]), D[b]], [D[b]^T, diag(ak[b])]] with D block-diagonal per head
// (D[b][h] = dL/dG of head h), written densely in the GEMM dtype in one pass (zeros included):
// dqk = qk Wd^T is then one per-image GEMM over the [q | k] rows.
template <typename T>
__global__ __launch_bounds__(256) void gram_wd_kernel(const float* __restrict__ D, const float* __restrict__ aq,
                                                      const float* __restrict__ ak, T* __restrict__ wd, int c, int heads,
                                                      int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int c2 = 2 * c, ch = c / heads;
  const int64_t per = (int64_t)c2 * c2;
  const int b = (int)(i / per);
  const int r = (int)((i % per) / c2), col = (int)(i % c2);
  const bool rq = r < c, cq = col < c;
  const int rr = rq ? r : r - c, cc = cq ? col : col - c;
  float v = 0.f;
  if (r == col) {
    v = rq ? aq[(int64_t)b * c + rr] : ak[(int64_t)b * c + rr];
  } else if (rq != cq && rr / ch == cc / ch) {
    const int h = rr / ch;
    const float* Dh = D + ((int64_t)b * heads + h) * ch * ch;
    v = rq ? Dh[(rr % ch) * ch + cc % ch] : Dh[(cc % ch) * ch + rr % ch];
  }
  wd[i] = T(v);
}

// ---------------------------------------------------------------------------------------------
// reduction GEMM  C[img][n][k] = sum_{p in img} A[p][n] B[p][k]
//   bf16: block = 64 (n) x 64 (k) output tile, 4 waves of 32 x 32 (2 x 2 MFMA 16x16x32 tiles);
//   per stage 64 pixels of A (64 n) and B (64 k) staged in LDS (rows of 128 B + 32 B pad), both
//   read with ds_read_b64_tr_b16. A lane group g (16 lanes) of the transposed read h covers the
//   pixel rows 4 g + 16 h + q (q = 0..3): the 8 rows a 32-lane half reads are consecutive, which
//   with the 160-B row pitch (40 dwords) puts them on 8 distinct 8-bank sets (conflict-free); the
//   same pixel order is used for A and B, so the contraction is exact. Two LDS stages: the next
//   stage's global loads (unconditional, clamped addresses, masked rows) are in flight during this
//   stage's MFMAs. Pixel splits write fp32 partials [split][img][N][K]; rgemm_reduce sums them in
//   split order.
//   fp32 (parity builds): the same tiling on the VALU.
// ---------------------------------------------------------------------------------------------
constexpr int RG_BN = 64, RG_BK = 64, RG_BP = 64, RG_PITCH = 160;

TURTLE_DEV uint2 ds_read_tr16(const char* lds_ptr) {
  uint2 r;
  const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)lds_ptr;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}

// Output tile TN x TK per block (64 or 128 each; 128 x 128 on the wide weights, where the 64 x 64 tile
// left the matrix cores at ~200 TF/s: 4x fewer transposed LDS reads per MFMA), four waves of
// (TN / 2) x (TK / 2), RG_BP pixel rows per stage.
// shW > 0 (3x3 convolution weight gradient, img_px = 0): blockIdx.y = tap t of a 3x3 stencil
// (dy, dx) = (t / 3 - 1, t % 3 - 1), B's pixel p read at (y + dy, x + dx) of its shH x shW image (zero
// outside): part[split][t] = sum_p A[p] B[p + shift(t)]^T
template <int TN, int TK>
__global__ __launch_bounds__(256) void rgemm_bf16_kernel(const bf16* __restrict__ A, int64_t lda, const bf16* __restrict__ B,
                                                         int64_t ldb, float* __restrict__ part, int64_t img_px, int nimg_out,
                                                         int N, int K, int64_t P, int64_t ppb, int shH = 0, int shW = 0) {
  typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
  // row pitches: 32 B past the row (40 / 72 dwords): the 8 consecutive rows a 32-lane half of a
  // transposed read covers land on 8 distinct 8-bank sets
  constexpr int PA = 2 * TN + 32, PB = 2 * TK + 32;
  constexpr int CA = TN / 32, CB = TK / 32;        // 16-B chunks per staging thread (4 threads per pixel row)
  constexpr int FI = TN / 32, FJ = TK / 32;        // 16 x 16 fragments per wave along N / K
  // two stage buffers: the global loads of stage s + 1 are in flight (in registers) while the
  // MFMAs of stage s read the other buffer; one barrier per stage
  __shared__ __attribute__((aligned(16))) char sA[2][RG_BP * PA];
  __shared__ __attribute__((aligned(16))) char sB[2][RG_BP * PB];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ntn = (N + TN - 1) / TN, ntk = (K + TK - 1) / TK;
  const int tile = blockIdx.x % (ntn * ntk);
  const int n0 = (tile / ntk) * TN, k0 = (tile % ntk) * TK;
  const int split = blockIdx.x / (ntn * ntk);
  const int img = blockIdx.y;
  const int64_t pbase = img_px > 0 ? (int64_t)img * img_px : 0;
  const int64_t plen = img_px > 0 ? img_px : P;
  const int64_t p0 = (int64_t)split * ppb, p1 = min(plen, p0 + ppb);
  const int wn = wid >> 1, wk = wid & 1;
  const int sdy = img / 3 - 1, sdx = img % 3 - 1;   // (tap mode only)
  f32x4 acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // staging: thread -> pixel row tid >> 2, 16-B chunks CA (tid & 3) .. + CA - 1 of A (CB of B).
  // Loads are unconditional: a column chunk past N / K is clamped to the last one (it only feeds
  // output rows / columns that are not stored), a pixel row past the split's end is clamped to its
  // last row and zeroed by a mask when it is written to LDS (both operands: no inf * 0).
  const int srow = tid >> 2, sca = CA * (tid & 3), scb = CB * (tid & 3);
  const bf16* pa[CA];
  const bf16* pb_[CB];
#pragma unroll
  for (int u = 0; u < CA; ++u) pa[u] = A + pbase * lda + min(n0 + 8 * (sca + u), N - 8);
#pragma unroll
  for (int u = 0; u < CB; ++u) pb_[u] = B + pbase * ldb + min(k0 + 8 * (scb + u), K - 8);
  uint4 ra[CA], rb[CB];
  uint32_t live_mask = 0, b_mask = 0;
  auto gload = [&](int64_t pbk) {
    const int64_t p = pbk + srow;
    live_mask = p < p1 ? 0xffffffffu : 0u;
    const int64_t pc = p < p1 ? p : p1 - 1;
    int64_t pcb = pc;
    b_mask = live_mask;
    if (shW > 0) {                                 // (uniform branch)
      const int64_t xq = pc % shW, yq = (pc / shW) % shH;
      const bool ok = yq + sdy >= 0 && yq + sdy < shH && xq + sdx >= 0 && xq + sdx < shW;
      pcb = ok ? pc + (int64_t)sdy * shW + sdx : pc;
      b_mask = ok ? live_mask : 0u;
    }
#pragma unroll
    for (int u = 0; u < CA; ++u) ra[u] = *reinterpret_cast<const uint4*>(pa[u] + pc * lda);
#pragma unroll
    for (int u = 0; u < CB; ++u) rb[u] = *reinterpret_cast<const uint4*>(pb_[u] + pcb * ldb);
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int u = 0; u < CA; ++u) {
      const uint4 va = make_uint4(ra[u].x & live_mask, ra[u].y & live_mask, ra[u].z & live_mask, ra[u].w & live_mask);
      *reinterpret_cast<uint4*>(sA[buf] + srow * PA + 16 * (sca + u)) = va;
    }
#pragma unroll
    for (int u = 0; u < CB; ++u) {
      const uint4 vb = make_uint4(rb[u].x & b_mask, rb[u].y & b_mask, rb[u].z & b_mask, rb[u].w & b_mask);
      *reinterpret_cast<uint4*>(sB[buf] + srow * PB + 16 * (scb + u)) = vb;
    }
  };
  // transposed reads: lane group g = lane >> 4, row q = (lane >> 2) & 3, column quad pq = lane & 3
  const int g = lane >> 4, q = (lane >> 2) & 3, pq = lane & 3;
  if (p0 < p1) {
    gload(p0);
    lstore(0);
  }
  __syncthreads();
  int buf = 0;
  for (int64_t pbk = p0; pbk < p1; pbk += RG_BP) {
    const bool more = pbk + RG_BP < p1;           // block-uniform
    if (more) gload(pbk + RG_BP);
    const char* cA = sA[buf];
    const char* cB = sB[buf];
#pragma unroll
    for (int ks = 0; ks < RG_BP / 32; ++ks) {      // 32 pixels per MFMA K step
      uint2 ra0[FI], ra1[FI], rb0[FJ], rb1[FJ];
      const int r0 = 32 * ks + 4 * g + q;
#pragma unroll
      for (int t = 0; t < FI; ++t) {
        const int cn = (TN / 2) * wn + 16 * t + 4 * pq;
        ra0[t] = ds_read_tr16(cA + r0 * PA + 2 * cn);
        ra1[t] = ds_read_tr16(cA + (r0 + 16) * PA + 2 * cn);
      }
#pragma unroll
      for (int t = 0; t < FJ; ++t) {
        const int ck = (TK / 2) * wk + 16 * t + 4 * pq;
        rb0[t] = ds_read_tr16(cB + r0 * PB + 2 * ck);
        rb1[t] = ds_read_tr16(cB + (r0 + 16) * PB + 2 * ck);
      }
      // the compiler does not see the asm reads as LDS loads: the wait is an ordered volatile asm and
      // every read result passes through an (ordered) empty asm after it before an MFMA may use it
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int t = 0; t < FI; ++t) asm volatile("" : "+v"(ra0[t]), "+v"(ra1[t]));
#pragma unroll
      for (int t = 0; t < FJ; ++t) asm volatile("" : "+v"(rb0[t]), "+v"(rb1[t]));
      bf16x8v af[FI], bfr[FJ];
#pragma unroll
      for (int t = 0; t < FI; ++t) af[t] = __builtin_bit_cast(bf16x8v, make_uint4(ra0[t].x, ra0[t].y, ra1[t].x, ra1[t].y));
#pragma unroll
      for (int t = 0; t < FJ; ++t) bfr[t] = __builtin_bit_cast(bf16x8v, make_uint4(rb0[t].x, rb0[t].y, rb1[t].x, rb1[t].y));
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) lstore(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // lane holds C[n0 + (TN / 2) wn + 16 i + 4 g + e][k0 + (TK / 2) wk + 16 j + (lane & 15)]
  float* out = part + ((int64_t)split * nimg_out + img) * N * K;
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = n0 + (TN / 2) * wn + 16 * i + 4 * g + e, k = k0 + (TK / 2) * wk + 16 * j + (lane & 15);
        if (n < N && k < K) out[(int64_t)n * K + k] = acc[i][j][e];
      }
}

__global__ __launch_bounds__(256) void rgemm_f32_kernel(const float* __restrict__ A, int64_t lda, const float* __restrict__ B,
                                                        int64_t ldb, float* __restrict__ part, int64_t img_px, int nimg_out,
                                                        int N, int K, int64_t P, int64_t ppb, int shH = 0, int shW = 0) {
  __shared__ float sA[32][65], sB[32][65];
  const int tid = threadIdx.x;
  const int ntn = (N + 63) / 64, ntk = (K + 63) / 64;
  const int tile = blockIdx.x % (ntn * ntk);
  const int n0 = (tile / ntk) * 64, k0 = (tile % ntk) * 64;
  const int split = blockIdx.x / (ntn * ntk);
  const int img = blockIdx.y;
  const int64_t pbase = img_px > 0 ? (int64_t)img * img_px : 0;
  const int64_t plen = img_px > 0 ? img_px : P;
  const int64_t p0 = (int64_t)split * ppb, p1 = min(plen, p0 + ppb);
  const int tn = tid >> 4, tk = tid & 15;          // 4 x 4 outputs per thread
  const int sdy = img / 3 - 1, sdx = img % 3 - 1;   // (tap mode: shW > 0, see rgemm_bf16_kernel)
  float acc[4][4] = {};
  for (int64_t pb = p0; pb < p1; pb += 32) {
    for (int i = tid; i < 32 * 64; i += 256) {
      const int r = i / 64, cc = i % 64;
      const int64_t p = pb + r;
      int64_t pbq = pbase + p;
      bool bok = true;
      if (shW > 0) {
        const int64_t xq = p % shW, yq = (p / shW) % shH;
        bok = yq + sdy >= 0 && yq + sdy < shH && xq + sdx >= 0 && xq + sdx < shW;
        pbq = p + (int64_t)sdy * shW + sdx;
      }
      sA[r][cc] = (p < p1 && n0 + cc < N) ? A[(pbase + p) * lda + n0 + cc] : 0.f;
      sB[r][cc] = (p < p1 && bok && k0 + cc < K) ? B[pbq * ldb + k0 + cc] : 0.f;
    }
    __syncthreads();
    for (int r = 0; r < 32; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(sA[r][4 * tn + i], sB[r][4 * tk + j], acc[i][j]);
    __syncthreads();
  }
  float* out = part + ((int64_t)split * nimg_out + img) * N * K;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + 4 * tn + i, k = k0 + 4 * tk + j;
      if (n < N && k < K) out[(int64_t)n * K + k] = acc[i][j];
    }
}

// Sum of the split partials: c[i] (+)= sum_k part[k][i]. Block = EL consecutive entries x (256 / EL)
// split groups; each lane keeps 8 loads in flight and the group sums meet in LDS in a fixed order
// (deterministic). Few entries with many splits (small weights over many pixels: n = 4096,
// nsplit = 1024) take EL = 16, i.e. 16 groups, so a thread walks nsplit / 16 partials instead of
// all of them.
template <int EL>
__global__ __launch_bounds__(256) void rgemm_reduce_kernel(const float* __restrict__ part, float* __restrict__ c, int64_t n,
                                                           int nsplit, int accumulate) {
  constexpr int G = 256 / EL;
  __shared__ float ps[G][EL];
  const int lane = threadIdx.x % EL, g = threadIdx.x / EL;
  const int64_t i = (int64_t)blockIdx.x * EL + lane;
  const float* p = part + (i < n ? i : n - 1);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int k = g;
  for (; k + 7 * G < nsplit; k += 8 * G) {
#pragma unroll
    for (int u = 0; u < 8; ++u) s[u] += p[(int64_t)(k + u * G) * n];
  }
  for (; k < nsplit; k += G) s[0] += p[(int64_t)k * n];
  ps[g][lane] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  if (g == 0 && i < n) {
    float t = accumulate ? c[i] : 0.f;
#pragma unroll
    for (int q = 0; q < G; ++q) t += ps[q][lane];
    c[i] = t;
  }
}

// ---------------------------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------------------------
template <typename T, typename TY = T>
int ln_fwd(const void* x, int64_t ldx, const float* w, const float* b, void* y, int64_t ldy, float* mu, float* rstd, int64_t P,
           int C, int biasfree, hipStream_t st) {
  const int G = ln_group(C), nch = (C / 8 + G - 1) / G;
  // U = 4 / NCH pixels per lane group (4 row loads in flight per lane)
#define LNF(GG, NN)                                                                                                  \
  if (G == GG && nch <= NN) {                                                                                        \
    constexpr int U = NN >= 4 ? 1 : 4 / NN;                                                                          \
    const int64_t blocks = std::max<int64_t>(1, (P * G + 256 * U - 1) / (256 * U));                                  \
    if (biasfree)                                                                                                    \
      hipLaunchKernelGGL((ln_fwd_kernel<T, TY, GG, NN, U, true>), dim3((unsigned)blocks), dim3(256), 0, st, (const T*)x, \
                         ldx, w, b, (TY*)y, ldy, mu, rstd, P, C);                                                     \
    else                                                                                                             \
      hipLaunchKernelGGL((ln_fwd_kernel<T, TY, GG, NN, U, false>), dim3((unsigned)blocks), dim3(256), 0, st, (const T*)x, \
                         ldx, w, b, (TY*)y, ldy, mu, rstd, P, C);                                                     \
    return 0;                                                                                                        \
  }
  LNF(1, 1) LNF(2, 1) LNF(4, 1) LNF(8, 1) LNF(16, 1) LNF(32, 1) LNF(64, 1) LNF(64, 2) LNF(64, 4)
#undef LNF
  return -1;
}
template <typename T, typename TY = T>
int ln_bwd(const void* x, int64_t ldx, const float* w, const float* mu, const float* rstd, const void* dy, int64_t lddy, void* dx,
           int64_t lddx, const void* dres, int64_t lddres, float* dw, float* db, int64_t P, int C, int biasfree, hipStream_t st) {
  const int G = ln_group(C), nch = (C / 8 + G - 1) / G;
  // ~256 blocks whatever P is (a fixed 256 pixels per block left a 32 x 32 x 8 latent map on 32
  // blocks; 512 - 1024 blocks measured slower: more end-of-block atomics, tools/train_kbench.py);
  // pixels per block a multiple of the block's pixel slots x U
  const int64_t nslot = 256 / G;
#define LNB(GG, NN)                                                                                                       \
  if (G == GG && nch <= NN) {                                                                                             \
    constexpr int U = NN >= 4 ? 1 : 4 / NN;                                                                               \
    const int64_t nbt = train_tune(0) > 0 ? train_tune(0) : 256;                                                           \
    int64_t ppb = std::max<int64_t>(nslot * U, (P + nbt - 1) / nbt);                                                      \
    ppb = (ppb + nslot * U - 1) / (nslot * U) * (nslot * U);                                                              \
    const int64_t blocks = (P + ppb - 1) / ppb;                                                                           \
    if (biasfree)                                                                                                         \
      hipLaunchKernelGGL((ln_bwd_kernel<T, TY, GG, NN, U, true>), dim3((unsigned)blocks), dim3(256), 2 * C * sizeof(float), st, \
                         (const T*)x, ldx, w, mu, rstd, (const TY*)dy, lddy, (T*)dx, lddx, (const T*)dres, lddres, dw, db, P, C, \
                         (int)ppb, train_abl() & 1);                                                                     \
    else                                                                                                                  \
      hipLaunchKernelGGL((ln_bwd_kernel<T, TY, GG, NN, U, false>), dim3((unsigned)blocks), dim3(256), 2 * C * sizeof(float), st, \
                         (const T*)x, ldx, w, mu, rstd, (const TY*)dy, lddy, (T*)dx, lddx, (const T*)dres, lddres, dw, db, P, C, \
                         (int)ppb, train_abl() & 1);                                                                     \
    return 0;                                                                                                             \
  }
  LNB(1, 1) LNB(2, 1) LNB(4, 1) LNB(8, 1) LNB(16, 1) LNB(32, 1) LNB(64, 1) LNB(64, 2) LNB(64, 4)
#undef LNB
  return -1;
}
template <typename T>
int dw_fwd(const void* x, int64_t ldx, const float* w9, const float* b, void* y, int64_t ldy, int64_t N, int C, int H, int W,
           int flip, hipStream_t st) {
  if constexpr (!std::is_same<T, f16>::value) {
    if (!flip && N <= INT32_MAX) {
      // the inference path's row-sweeping kernel (spatial.hip: each input byte leaves HBM about
      // once, rolling 3-row register window) instead of the per-pixel 9-load gather
      DwArgs a{};
      a.in = x; a.ldi = ldx; a.offi = 0; a.out = y; a.ldo = ldy; a.offo = 0; a.w = w9; a.bias = b;
      a.nimg = (int)N; a.H = H; a.W = W; a.C = C; a.mode = DW_PLAIN; a.tok_ws = 0; a.rows = 1;
      launch_dw<T>(a, st);
      return 0;
    }
  }
  const int64_t tot = N * H * W * (C / 8);
  hipLaunchKernelGGL(dw_fwd_kernel<T>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, (const T*)x, ldx, w9, b, (T*)y,
                     ldy, N, C, H, W, flip);
  return 0;
}
template <typename T>
int dw_wgrad(const void* x, int64_t ldx, const void* dy, int64_t lddy, float* dw9, float* db, int64_t N, int C, int H, int W,
             hipStream_t st) {
  if (N <= INT32_MAX) {
    const int nstrip = (W + TW_SX - 1) / TW_SX, nchunk = (C / 8 + TW_CV - 1) / TW_CV;
    int RB = 32;
    auto nblk = [&](int rb) { return N * nchunk * nstrip * ((H + rb - 1) / rb); };
    // ~512 blocks: longer row bands amortise the block's column / tap reduction (2048 blocks of 8-row
    // bands: 80 us at level 1 against 42 us, tools/train_kbench.py)
    const int64_t target = train_tune(2) > 0 ? train_tune(2) : 512;
    while (RB > 4 && nblk(RB) < target) RB /= 2;
    const int nband = (H + RB - 1) / RB;
    hipLaunchKernelGGL(dw_wgrad_rows_kernel<T>, dim3((unsigned)nblk(RB)), dim3(256), 0, st, (const T*)x, ldx, (const T*)dy, lddy,
                       dw9, db, C, H, W, RB, nstrip, nchunk, nband, train_abl() & 1);
    return 0;
  }
  const int64_t P = N * H * W;
  const int nsl = (C / 8 + DWG_CPB - 1) / DWG_CPB;
  const int64_t blocks = std::min<int64_t>(std::max<int64_t>(1, 1024 / nsl), std::max<int64_t>(1, P / 64));
  const int64_t ppb = (P + blocks - 1) / blocks;
  hipLaunchKernelGGL(dw_wgrad_kernel<T>, dim3((unsigned)blocks, (unsigned)nsl), dim3(256), 0, st, (const T*)x, ldx,
                     (const T*)dy, lddy, dw9, db, N, C, H, W, ppb);
  return 0;
}
template <typename T>
int gate_fwd(const void* x, int64_t ldx, void* y, int64_t ldy, int64_t P, int h, hipStream_t st) {
  const int64_t tot = P * (h / 8);
  hipLaunchKernelGGL(gate_fwd_kernel<T>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, (const T*)x, ldx, (T*)y, ldy, P, h);
  return 0;
}
template <typename T>
int gate_bwd(const void* x, int64_t ldx, const void* dy, int64_t lddy, void* dx, int64_t lddx, int64_t P, int h, hipStream_t st) {
  const int64_t tot = P * (h / 8);
  hipLaunchKernelGGL(gate_bwd_kernel<T>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, (const T*)x, ldx, (const T*)dy,
                     lddy, (T*)dx, lddx, P, h);
  return 0;
}
template <typename T>
int gelu_fwd(const void* x, int64_t ldx, void* y, int64_t ldy, int64_t P, int C, hipStream_t st) {
  const int64_t tot = P * (C / 8);
  hipLaunchKernelGGL(gelu_fwd_kernel<T>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, (const T*)x, ldx, (T*)y, ldy, P, C);
  return 0;
}
template <typename T>
int gelu_bwd(const void* x, int64_t ldx, const void* dy, int64_t lddy, void* dx, int64_t lddx, int64_t P, int C, hipStream_t st) {
  const int64_t tot = P * (C / 8);
  hipLaunchKernelGGL(gelu_bwd_kernel<T>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, (const T*)x, ldx, (const T*)dy,
                     lddy, (T*)dx, lddx, P, C);
  return 0;
}
template <typename T>
int win_fwd(const void* x, int64_t ldx, const float* wt, const float* b, void* y, int64_t ldy, int64_t N, int C, int H, int W,
            int ws, int th, int tw, hipStream_t st) {
  const int64_t tot = N * th * tw * (C / 8);
  hipLaunchKernelGGL(win_fwd_kernel<T>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, (const T*)x, ldx, wt, b, (T*)y, ldy,
                     N, C, H, W, ws, th, tw);
  return 0;
}
template <typename T>
int win_dgrad(const void* dy, int64_t lddy, const float* wt, void* dx, int64_t lddx, int64_t N, int C, int H, int W, int ws, int th,
              int tw, hipStream_t st) {
  const int64_t tot = N * H * W * (C / 8);
  hipLaunchKernelGGL(win_dgrad_kernel<T>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, (const T*)dy, lddy, wt, (T*)dx,
                     lddx, N, C, H, W, ws, th, tw);
  return 0;
}
template <typename T>
int win_wgrad(const void* x, int64_t ldx, const void* dy, int64_t lddy, float* dwt, int64_t N, int C, int H, int W, int ws, int th,
              int tw, hipStream_t st) {
  const int64_t ntok = N * th * tw;
  const int nchunk = (C + 63) / 64;
  // token splits: ~2048 blocks in all, each split at least 64 tokens
  int64_t nsplit = std::max<int64_t>(1, std::min<int64_t>((2048 + ws * ws * nchunk - 1) / (ws * ws * nchunk), ntok / 64));
  nsplit = std::min<int64_t>(nsplit, 65535);
  const int64_t tpb = (ntok + nsplit - 1) / nsplit;
  nsplit = (ntok + tpb - 1) / tpb;
  hipLaunchKernelGGL(win_wgrad_kernel<T>, dim3((unsigned)(ws * ws), (unsigned)nchunk, (unsigned)nsplit), dim3(256), 0, st,
                     (const T*)x, ldx, (const T*)dy, lddy, dwt, N, C, H, W, ws, th, tw, tpb);
  return 0;
}
template <typename T>
int colsum(const void* dy, int64_t ld, float* db, int64_t P, int N, hipStream_t st) {
  // 1024-thread blocks, at most 256 of them: the end-of-block global atomics (N per block) cost more
  // than the column reads once there are ~1000 blocks (L1: 38 vs 21 us without them)
  const int cap = train_tune(1) > 0 ? train_tune(1) : 256;
  const int64_t blocks = std::min<int64_t>(cap, std::max<int64_t>(1, P * (N / 8) / 4096));   // >= 4 rows per thread
  const int64_t ppb = (P + blocks - 1) / blocks;
  hipLaunchKernelGGL((colsum_kernel<T, 0, 1024>), dim3((unsigned)blocks), dim3(1024), N * sizeof(float), st, (const T*)dy, ld, db, P,
                     N, ppb, nullptr, 0, train_abl() & 1);
  return 0;
}
// per-image column sums of squares: out[img][n] += sum over the image's img_px pixels of x^2
template <typename T>
int colsumsq(const void* x, int64_t ld, float* out, int64_t P, int N, int64_t img_px, hipStream_t st) {
  const int64_t nimg = P / img_px;
  const int64_t blocks = std::min<int64_t>(std::max<int64_t>(1, 512 / nimg), std::max<int64_t>(1, img_px / 256));
  const int64_t ppb = (img_px + blocks - 1) / blocks;
  hipLaunchKernelGGL((colsum_kernel<T, 1>), dim3((unsigned)blocks, (unsigned)nimg), dim3(256), N * sizeof(float), st, (const T*)x, ld,
                     out, img_px, N, ppb, nullptr, 0, 0);
  return 0;
}

// per-image column dot products out[img][n] += sum over the image's pixels of a[p][n] b[p][n]
template <typename T>
int coldot(const void* a, int64_t lda, const void* b, int64_t ldb, float* out, int64_t P, int N, int64_t img_px, hipStream_t st) {
  const int64_t nimg = P / img_px;
  const int64_t blocks = std::min<int64_t>(std::max<int64_t>(1, 512 / nimg), std::max<int64_t>(1, img_px / 256));
  const int64_t ppb = (img_px + blocks - 1) / blocks;
  hipLaunchKernelGGL((colsum_kernel<T, 2>), dim3((unsigned)blocks, (unsigned)nimg), dim3(256), N * sizeof(float), st, (const T*)a, lda,
                     out, img_px, N, ppb, (const T*)b, ldb, 0);
  return 0;
}
template <typename T>
int colscale(const void* x, int64_t ldx, const float* s, void* y, int64_t ldy, int64_t P, int C, int64_t img_px, hipStream_t st) {
  const int64_t tot = P * (C / 8);
  hipLaunchKernelGGL(colscale_kernel<T>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, (const T*)x, ldx, s, (T*)y, ldy, P, C,
                     img_px);
  return 0;
}
template <typename T>
int l2n_bwd(const void* dy, int64_t lddy, const void* y, int64_t ldy, const float* d, const float* s, void* dx, int64_t lddx, int64_t P,
            int C, int64_t img_px, hipStream_t st) {
  const int64_t tot = P * (C / 8);
  hipLaunchKernelGGL(l2n_bwd_kernel<T>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, (const T*)dy, lddy, (const T*)y, ldy, d,
                     s, (T*)dx, lddx, P, C, img_px);
  return 0;
}
template <typename TO>
int sab_softmax_fwd(const float* s, int64_t R, int n, int tw, int radius, void* a, float* a_save, uint8_t* m_save, hipStream_t st) {
  const dim3 grid((unsigned)((R + 3) / 4));
#define SSF(NVV) hipLaunchKernelGGL((sab_softmax_fwd_kernel<NVV, TO>), grid, dim3(256), 0, st, s, R, n, tw, radius, (TO*)a, a_save, m_save)
  if (n <= 64) SSF(1);
  else if (n <= 128) SSF(2);
  else if (n <= 256) SSF(4);
  else if (n <= 512) SSF(8);
  else if (n <= 1024) SSF(16);
  else return -1;
#undef SSF
  return 0;
}
template <typename TG>
int sab_softmax_bwd(const void* da, const float* a_save, const uint8_t* m_save, int64_t R, int n, float* ds, hipStream_t st) {
  const dim3 grid((unsigned)((R + 3) / 4));
#define SSB(NVV) hipLaunchKernelGGL((sab_softmax_bwd_kernel<NVV, TG>), grid, dim3(256), 0, st, (const TG*)da, a_save, m_save, R, n, ds)
  if (n <= 64) SSB(1);
  else if (n <= 128) SSB(2);
  else if (n <= 256) SSB(4);
  else if (n <= 512) SSB(8);
  else if (n <= 1024) SSB(16);
  else return -1;
#undef SSB
  return 0;
}
// per-image Gram-backward weights (gram_wd_kernel)
template <typename T>
int gram_wd(const float* D, const float* aq, const float* ak, void* wd, int64_t B, int c, int heads, hipStream_t st) {
  const int64_t total = B * 4 * (int64_t)c * c;
  hipLaunchKernelGGL(gram_wd_kernel<T>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, D, aq, ak, (T*)wd, c, heads, total);
  return 0;
}

// device constants of the GEMM family (zero / one vectors for branch-free operands), per device
static const float* train_consts(int which) {
  static std::mutex mu;
  static std::map<int, float*> mem;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  auto it = mem.find(dev);
  if (it == mem.end()) {
    float* p = nullptr;
    // zeros then ones, TURTLE_CONST_VEC each (the GEMMs read them at every output channel: a shorter
    // ones vector gave wrong outputs past channel 8192)
    if (hipMalloc(&p, 2 * (size_t)TURTLE_CONST_VEC * sizeof(float)) != hipSuccess) return nullptr;
    std::vector<float> h(2 * (size_t)TURTLE_CONST_VEC, 0.f);
    for (int i = TURTLE_CONST_VEC; i < 2 * TURTLE_CONST_VEC; ++i) h[i] = 1.f;
    if (hipMemcpy(p, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    it = mem.emplace(dev, p).first;
  }
  return which ? it->second + TURTLE_CONST_VEC : it->second;
}

// the bf16 reduction GEMM's output tile: 128 along N (K) when N (K) is a multiple of 128 or >= 256 (little
// padding), else 64; fp32 runs 64 x 64
static int rgemm_tn(int N, int dtype) { return dtype == 1 && (N % 128 == 0 || N >= 256) ? 128 : 64; }
static int64_t rgemm_splits(int64_t P, int N, int K, int64_t img_px, int ntap = 1, int dtype = 0) {
  const int64_t plen = img_px > 0 ? img_px : P;
  const int64_t nimg = (img_px > 0 ? P / img_px : 1) * ntap;
  const int tn = rgemm_tn(N, dtype), tk = rgemm_tn(K, dtype);
  const int64_t tiles = ((N + tn - 1) / tn) * ((K + tk - 1) / tk) * nimg;
  // ~1024 blocks (64-wide tiles), ~512 of the 128 x 128 tile (74 KB of LDS: 2 per
  // CU) - every split adds N K fp32 partials written here and read back by rgemm_reduce
  const int64_t target = (tn == 128 && tk == 128) ? 512 : 1024;
  return std::max<int64_t>(1, std::min<int64_t>((target + tiles - 1) / tiles, (plen + 511) / 512));
}
template <typename... Args>
static void launch_rgemm_bf16(int tn, int tk, dim3 grid, hipStream_t st, Args... args) {
  if (tn == 128 && tk == 128) hipLaunchKernelGGL((rgemm_bf16_kernel<128, 128>), grid, dim3(256), 0, st, args...);
  else if (tn == 128) hipLaunchKernelGGL((rgemm_bf16_kernel<128, 64>), grid, dim3(256), 0, st, args...);
  else if (tk == 128) hipLaunchKernelGGL((rgemm_bf16_kernel<64, 128>), grid, dim3(256), 0, st, args...);
  else hipLaunchKernelGGL((rgemm_bf16_kernel<64, 64>), grid, dim3(256), 0, st, args...);
}

}  // namespace turtle

// ---------------------------------------------------------------------------------------------
// C ABI (include/turtle_train.h): dtype 0 = fp32, 1 = bf16, 2 = fp16 activations; returns 0, a
// negative argument error or a positive hipError_t
// ---------------------------------------------------------------------------------------------
using namespace turtle;
#define TT_DISPATCH(dt, fn, ...)                                   \
  do {                                                             \
    int rc_;                                                       \
    if ((dt) == 1) rc_ = fn<bf16>(__VA_ARGS__);                    \
    else if ((dt) == 2) rc_ = fn<f16>(__VA_ARGS__);                \
    else if ((dt) == 0) rc_ = fn<float>(__VA_ARGS__);              \
    else return -1;                                                \
    if (rc_) return rc_;                                           \
    return (int)hipGetLastError();                                 \
  } while (0)

static bool rows_ok(const void* p, int64_t ld, int dtype) {
  const int es = dtype == 0 ? 4 : 2;
  return p && ld > 0 && (reinterpret_cast<uintptr_t>(p) % 16) == 0 && (ld * es) % 16 == 0;
}

extern "C" {

int turtle_train_ln_fwd(const void* x, int64_t ldx, const float* w, const float* b, void* y, int64_t ldy, float* mu, float* rstd,
                        int64_t P, int C, int biasfree, int dtype, void* stream) {
  // dtype: x's type in bits 0-3; bits 4-7 = 1 + y's type when it differs (fp32 residual stream in,
  // autocast bf16 / fp16 out: the cast folded into the LayerNorm)
  const int xdt = dtype & 15, ydt = (dtype >> 4) ? (dtype >> 4) - 1 : xdt;
  if (!rows_ok(x, ldx, xdt) || !rows_ok(y, ldy, ydt) || !w || !mu || !rstd || P <= 0 || C <= 0 || C % 8 || C > 2048 ||
      ldx < C || ldy < C || (!biasfree && !b))
    return -1;
  if (xdt != ydt) {
    int rc;
    if (xdt == 0 && ydt == 1) rc = ln_fwd<float, bf16>(x, ldx, w, b, y, ldy, mu, rstd, P, C, biasfree, (hipStream_t)stream);
    else if (xdt == 0 && ydt == 2) rc = ln_fwd<float, f16>(x, ldx, w, b, y, ldy, mu, rstd, P, C, biasfree, (hipStream_t)stream);
    else return -1;
    return rc ? rc : (int)hipGetLastError();
  }
  TT_DISPATCH(xdt, ln_fwd, x, ldx, w, b, y, ldy, mu, rstd, P, C, biasfree, (hipStream_t)stream);
}

int turtle_train_ln_bwd(const void* x, int64_t ldx, const float* w, const float* mu, const float* rstd, const void* dy,
                        int64_t lddy, void* dx, int64_t lddx, const void* dres, int64_t lddres, float* dw, float* db, int64_t P,
                        int C, int biasfree, int dtype, void* stream) {
  // dtype as turtle_train_ln_fwd: x, dx and dres in x's type, dy in y's type
  const int xdt = dtype & 15, ydt = (dtype >> 4) ? (dtype >> 4) - 1 : xdt;
  if (!rows_ok(x, ldx, xdt) || !rows_ok(dy, lddy, ydt) || !rows_ok(dx, lddx, xdt) || (dres && !rows_ok(dres, lddres, xdt)) ||
      !w || !mu || !rstd || !dw || P <= 0 || C <= 0 || C % 8 || C > 2048)
    return -1;
  float* dbb = biasfree ? nullptr : db;
  if (xdt != ydt) {
    int rc;
    if (xdt == 0 && ydt == 1)
      rc = ln_bwd<float, bf16>(x, ldx, w, mu, rstd, dy, lddy, dx, lddx, dres, lddres, dw, dbb, P, C, biasfree, (hipStream_t)stream);
    else if (xdt == 0 && ydt == 2)
      rc = ln_bwd<float, f16>(x, ldx, w, mu, rstd, dy, lddy, dx, lddx, dres, lddres, dw, dbb, P, C, biasfree, (hipStream_t)stream);
    else return -1;
    return rc ? rc : (int)hipGetLastError();
  }
  TT_DISPATCH(xdt, ln_bwd, x, ldx, w, mu, rstd, dy, lddy, dx, lddx, dres, lddres, dw, dbb, P, C, biasfree, (hipStream_t)stream);
}

int turtle_train_dw3x3_fwd(const void* x, int64_t ldx, const float* w9, const float* b, void* y, int64_t ldy, int64_t N, int C,
                           int H, int W, int flip, int dtype, void* stream) {
  if (!rows_ok(x, ldx, dtype) || !rows_ok(y, ldy, dtype) || !w9 || N <= 0 || C <= 0 || C % 8 || H <= 0 || W <= 0)
    return -1;
  TT_DISPATCH(dtype, dw_fwd, x, ldx, w9, b, y, ldy, N, C, H, W, flip, (hipStream_t)stream);
}

int turtle_train_dw3x3_wgrad(const void* x, int64_t ldx, const void* dy, int64_t lddy, float* dw9, float* db, int64_t N, int C,
                             int H, int W, int dtype, void* stream) {
  if (!rows_ok(x, ldx, dtype) || !rows_ok(dy, lddy, dtype) || !dw9 || N <= 0 || C <= 0 || C % 8 || H <= 0 || W <= 0)
    return -1;
  TT_DISPATCH(dtype, dw_wgrad, x, ldx, dy, lddy, dw9, db, N, C, H, W, (hipStream_t)stream);
}

int turtle_train_gate_fwd(const void* x, int64_t ldx, void* y, int64_t ldy, int64_t P, int h, int dtype, void* stream) {
  if (!rows_ok(x, ldx, dtype) || !rows_ok(y, ldy, dtype) || P <= 0 || h <= 0 || h % 8) return -1;
  TT_DISPATCH(dtype, gate_fwd, x, ldx, y, ldy, P, h, (hipStream_t)stream);
}

int turtle_train_gate_bwd(const void* x, int64_t ldx, const void* dy, int64_t lddy, void* dx, int64_t lddx, int64_t P, int h,
                          int dtype, void* stream) {
  if (!rows_ok(x, ldx, dtype) || !rows_ok(dy, lddy, dtype) || !rows_ok(dx, lddx, dtype) || P <= 0 || h <= 0 || h % 8) return -1;
  TT_DISPATCH(dtype, gate_bwd, x, ldx, dy, lddy, dx, lddx, P, h, (hipStream_t)stream);
}

int turtle_train_gelu_fwd(const void* x, int64_t ldx, void* y, int64_t ldy, int64_t P, int C, int dtype, void* stream) {
  if (!rows_ok(x, ldx, dtype) || !rows_ok(y, ldy, dtype) || P <= 0 || C <= 0 || C % 8 || ldx < C || ldy < C) return -1;
  TT_DISPATCH(dtype, gelu_fwd, x, ldx, y, ldy, P, C, (hipStream_t)stream);
}

int turtle_train_gelu_bwd(const void* x, int64_t ldx, const void* dy, int64_t lddy, void* dx, int64_t lddx, int64_t P, int C,
                          int dtype, void* stream) {
  if (!rows_ok(x, ldx, dtype) || !rows_ok(dy, lddy, dtype) || !rows_ok(dx, lddx, dtype) || P <= 0 || C <= 0 || C % 8) return -1;
  TT_DISPATCH(dtype, gelu_bwd, x, ldx, dy, lddy, dx, lddx, P, C, (hipStream_t)stream);
}

static bool win_ok(int64_t N, int C, int H, int W, int ws, int th, int tw) {
  return N > 0 && C > 0 && C % 8 == 0 && H > 0 && W > 0 && ws > 0 && ws <= 64 && th > 0 && tw > 0 &&
         th == (H + 2 - ws) / ws + 1 && tw == (W + 2 - ws) / ws + 1 && H + 2 >= ws && W + 2 >= ws;
}

int turtle_train_window_fwd(const void* x, int64_t ldx, const float* wt, const float* b, void* y, int64_t ldy, int64_t N, int C,
                            int H, int W, int ws, int th, int tw, int dtype, void* stream) {
  if (!rows_ok(x, ldx, dtype) || !rows_ok(y, ldy, dtype) || !wt || !win_ok(N, C, H, W, ws, th, tw)) return -1;
  TT_DISPATCH(dtype, win_fwd, x, ldx, wt, b, y, ldy, N, C, H, W, ws, th, tw, (hipStream_t)stream);
}

int turtle_train_window_dgrad(const void* dy, int64_t lddy, const float* wt, void* dx, int64_t lddx, int64_t N, int C, int H, int W,
                              int ws, int th, int tw, int dtype, void* stream) {
  if (!rows_ok(dy, lddy, dtype) || !rows_ok(dx, lddx, dtype) || !wt || !win_ok(N, C, H, W, ws, th, tw)) return -1;
  TT_DISPATCH(dtype, win_dgrad, dy, lddy, wt, dx, lddx, N, C, H, W, ws, th, tw, (hipStream_t)stream);
}

int turtle_train_window_wgrad(const void* x, int64_t ldx, const void* dy, int64_t lddy, float* dwt, int64_t N, int C, int H, int W,
                              int ws, int th, int tw, int dtype, void* stream) {
  if (!rows_ok(x, ldx, dtype) || !rows_ok(dy, lddy, dtype) || !dwt || !win_ok(N, C, H, W, ws, th, tw)) return -1;
  TT_DISPATCH(dtype, win_wgrad, x, ldx, dy, lddy, dwt, N, C, H, W, ws, th, tw, (hipStream_t)stream);
}

int turtle_train_colsum(const void* dy, int64_t ld, float* db, int64_t P, int N, int dtype, void* stream) {
  if (!rows_ok(dy, ld, dtype) || !db || P <= 0 || N <= 0 || N % 8 || N > 2048) return -1;
  TT_DISPATCH(dtype, colsum, dy, ld, db, P, N, (hipStream_t)stream);
}

int turtle_train_colsumsq(const void* x, int64_t ld, float* out, int64_t P, int N, int64_t img_px, int dtype, void* stream) {
  if (!rows_ok(x, ld, dtype) || !out || P <= 0 || N <= 0 || N % 8 || N > 2048 || img_px <= 0 || P % img_px || P / img_px > 65535)
    return -1;
  TT_DISPATCH(dtype, colsumsq, x, ld, out, P, N, img_px, (hipStream_t)stream);
}

int turtle_train_coldot(const void* a, int64_t lda, const void* b, int64_t ldb, float* out, int64_t P, int N, int64_t img_px,
                        int dtype, void* stream) {
  if (!rows_ok(a, lda, dtype) || !rows_ok(b, ldb, dtype) || !out || P <= 0 || N <= 0 || N % 8 || N > 2048 || img_px <= 0 ||
      P % img_px || P / img_px > 65535)
    return -1;
  TT_DISPATCH(dtype, coldot, a, lda, b, ldb, out, P, N, img_px, (hipStream_t)stream);
}

int turtle_train_colscale(const void* x, int64_t ldx, const float* s, void* y, int64_t ldy, int64_t P, int C, int64_t img_px,
                          int dtype, void* stream) {
  if (!rows_ok(x, ldx, dtype) || !rows_ok(y, ldy, dtype) || !s || P <= 0 || C <= 0 || C % 8 || img_px <= 0 || P % img_px)
    return -1;
  TT_DISPATCH(dtype, colscale, x, ldx, s, y, ldy, P, C, img_px, (hipStream_t)stream);
}

int turtle_train_l2n_bwd(const void* dy, int64_t lddy, const void* y, int64_t ldy, const float* d, const float* s, void* dx,
                         int64_t lddx, int64_t P, int C, int64_t img_px, int dtype, void* stream) {
  if (!rows_ok(dy, lddy, dtype) || !rows_ok(y, ldy, dtype) || !rows_ok(dx, lddx, dtype) || !d || !s || P <= 0 || C <= 0 || C % 8 ||
      img_px <= 0 || P % img_px)
    return -1;
  TT_DISPATCH(dtype, l2n_bwd, dy, lddy, y, ldy, d, s, dx, lddx, P, C, img_px, (hipStream_t)stream);
}

int turtle_train_sab_softmax_fwd(const float* s, int64_t R, int n, int tw, int radius, void* a, float* a_save, void* m_save,
                                 int dtype, void* stream) {
  if (!s || !a || !a_save || !m_save || R <= 0 || n <= 0 || n > 1024 || tw <= 0 || n % tw || radius < 0) return -1;
  TT_DISPATCH(dtype, sab_softmax_fwd, s, R, n, tw, radius, a, a_save, (uint8_t*)m_save, (hipStream_t)stream);
}

int turtle_train_sab_softmax_bwd(const void* da, const float* a_save, const void* m_save, int64_t R, int n, float* ds, int dtype,
                                 void* stream) {
  if (!da || !a_save || !m_save || !ds || R <= 0 || n <= 0 || n > 1024) return -1;
  TT_DISPATCH(dtype, sab_softmax_bwd, da, a_save, (const uint8_t*)m_save, R, n, ds, (hipStream_t)stream);
}

int turtle_train_gram_wd(const float* D, const float* aq, const float* ak, void* wd, int64_t B, int c, int heads, int dtype,
                         void* stream) {
  if (!D || !aq || !ak || !wd || B <= 0 || c <= 0 || heads <= 0 || c % heads || B * 4 * (int64_t)c * c > ((int64_t)1 << 40))
    return -1;
  TT_DISPATCH(dtype, gram_wd, D, aq, ak, wd, B, c, heads, (hipStream_t)stream);
}

int turtle_train_gemm(const void* x, int64_t ldx, const void* w, int64_t wstride, int64_t img_px, const float* bias,
                      const void* res, int64_t ldr, void* y, int64_t ldy, int64_t P, int K, int N, int dtype, void* stream) {
  if (dtype != 0 && dtype != 1) return -1;
  if (res && (!rows_ok(res, ldr, dtype) || ldr < N)) return -1;
  if (!rows_ok(x, ldx, dtype) || !rows_ok(y, ldy, dtype) || !w || P <= 0 || K <= 0 || N <= 0 || K % 8 || N % 8 || ldx < K ||
      ldy < N || (wstride && (img_px <= 0 || P % img_px)) || (img_px > 0 && img_px >= ((int64_t)1 << 31)) || N > TURTLE_CONST_VEC ||
      K > TURTLE_CONST_VEC)
    return -1;
  GemmArgs g{};
  g.a.n = 1; g.a.Ktot = K;
  g.a.s[0] = SrcDesc{x, ldx, 0, K, 1, 0};
  g.M = P; g.N = N;
  g.HW = (int)(img_px > 0 ? img_px : std::min<int64_t>(P, (int64_t)1 << 30)); g.Wimg = g.HW;
  g.w = w; g.ldw = K; g.wstride = wstride; g.wdiv = 1;
  g.bias = bias; g.out = y; g.ldo = ldy; g.offo = 0; g.store_mode = STORE_NHWC;
  g.res = res; g.ldr = ldr; g.offr = 0;
  g.zeros = train_consts(0); g.ones = train_consts(1);
  if (!g.zeros) return (int)hipErrorOutOfMemory;
  g.allow_panel = g.allow_lds = g.allow_pn = g.allow_ar = g.allow_kt = 1;
  if (train_tune(3) > 0) g.kt_max_px = train_tune(3);   // tools/train_kbench.py routing sweep
  try {
    if (dtype == 1) launch_gemm<bf16>(g, (hipStream_t)stream);
    else launch_gemm<float>(g, (hipStream_t)stream);
  } catch (...) {
    return -1;
  }
  return (int)hipGetLastError();
}

/* dense 3x3 convolution, stride 1, padding 1 (Down / Upsample body[0], turtle_t1_arch.py:136-154):
 * y[p][n] = sum_{tap, ci} x[p + off(tap)][ci] w[n][tap][ci] (+ bias[n]) on the inference implicit-GEMM
 * family (GemmArgs.conv3: no im2col); the input gradient is the same call on dy with the rotated,
 * transposed weights */
int turtle_train_conv3x3(const void* x, int64_t ldx, const void* w, const float* bias, void* y, int64_t ldy, int64_t B, int H,
                         int W, int Cin, int N, int dtype, void* stream) {
  if (dtype != 0 && dtype != 1) return -1;
  const int64_t P = B * H * W;
  if (!rows_ok(x, ldx, dtype) || !rows_ok(y, ldy, dtype) || !w || B <= 0 || H <= 0 || W <= 0 || Cin <= 0 || N <= 0 ||
      Cin % 8 || N % 8 || ldx < Cin || ldy < N || (int64_t)H * W >= ((int64_t)1 << 31) || N > TURTLE_CONST_VEC ||
      9 * Cin > TURTLE_CONST_VEC)
    return -1;
  GemmArgs g{};
  g.a.n = 1; g.a.Ktot = 9 * Cin;
  g.a.s[0] = SrcDesc{x, ldx, 0, 9 * Cin, 1, 0};
  g.M = P; g.N = N; g.HW = H * W; g.Wimg = W;
  g.conv3 = 1; g.cin = Cin;
  g.w = w; g.ldw = 9 * Cin; g.wdiv = 1;
  g.bias = bias; g.out = y; g.ldo = ldy; g.offo = 0; g.store_mode = STORE_NHWC;
  g.zeros = train_consts(0); g.ones = train_consts(1);
  if (!g.zeros) return (int)hipErrorOutOfMemory;
  g.allow_panel = g.allow_lds = g.allow_pn = g.allow_ar = g.allow_kt = 1;
  try {
    if (dtype == 1) launch_gemm<bf16>(g, (hipStream_t)stream);
    else launch_gemm<float>(g, (hipStream_t)stream);
  } catch (...) {
    return -1;
  }
  return (int)hipGetLastError();
}

size_t turtle_train_conv3x3_wgrad_workspace(int64_t P, int N, int Cin) {
  return (size_t)rgemm_splits(P, N, Cin, 0, 9) * 9 * N * Cin * sizeof(float);
}

/* its weight gradient dw[tap][n][ci] = sum_p dy[p][n] x[p + off(tap)][ci] (fp32 [9][N][Cin]): the reduction
 * GEMM with its B operand read at the tap's shifted pixel (zero outside the image), one block row per
 * tap; deterministic */
int turtle_train_conv3x3_wgrad(const void* dy, int64_t lddy, const void* x, int64_t ldx, float* dw, int64_t B, int H, int W, int N,
                               int Cin, int dtype, void* ws, size_t ws_bytes, void* stream) {
  if (dtype != 0 && dtype != 1) return -1;
  const int64_t P = B * H * W;
  if (!rows_ok(dy, lddy, dtype) || !rows_ok(x, ldx, dtype) || !dw || B <= 0 || H <= 0 || W <= 0 || N <= 0 || Cin <= 0 || N % 8 ||
      Cin % 8 || lddy < N || ldx < Cin)
    return -1;
  int64_t nsplit = rgemm_splits(P, N, Cin, 0, 9);
  if (!ws || ws_bytes < (size_t)nsplit * 9 * N * Cin * sizeof(float)) return -1;
  int64_t ppb = (P + nsplit - 1) / nsplit;
  ppb = (ppb + RG_BP - 1) / RG_BP * RG_BP;
  nsplit = (P + ppb - 1) / ppb;
  hipStream_t st = (hipStream_t)stream;
  float* part = reinterpret_cast<float*>(ws);
  if (dtype == 1) {
    const dim3 grid((unsigned)(((N + RG_BN - 1) / RG_BN) * ((Cin + RG_BK - 1) / RG_BK) * nsplit), 9u);
    hipLaunchKernelGGL((rgemm_bf16_kernel<64, 64>), grid, dim3(256), 0, st, (const bf16*)dy, lddy, (const bf16*)x, ldx, part,
                       (int64_t)0, 9, N, Cin, P, ppb, H, W);
  } else {
    const dim3 grid((unsigned)(((N + 63) / 64) * ((Cin + 63) / 64) * nsplit), 9u);
    hipLaunchKernelGGL(rgemm_f32_kernel, grid, dim3(256), 0, st, (const float*)dy, lddy, (const float*)x, ldx, part, (int64_t)0, 9,
                       N, Cin, P, ppb, H, W);
  }
  const int64_t n = 9 * (int64_t)N * Cin;
  if ((n + 63) / 64 >= 512)
    hipLaunchKernelGGL(rgemm_reduce_kernel<64>, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, st, part, dw, n, (int)nsplit, 0);
  else
    hipLaunchKernelGGL(rgemm_reduce_kernel<16>, dim3((unsigned)((n + 15) / 16)), dim3(256), 0, st, part, dw, n, (int)nsplit, 0);
  return (int)hipGetLastError();
}

size_t turtle_train_rgemm_workspace(int64_t P, int N, int K, int64_t img_px) {
  // sized for the larger of the two dtype plans (the bf16 plan splits less for its wider tiles)
  const int64_t nimg = img_px > 0 ? P / img_px : 1;
  const int64_t ns = std::max(rgemm_splits(P, N, K, img_px, 1, 0), rgemm_splits(P, N, K, img_px, 1, 1));
  return (size_t)ns * nimg * N * K * sizeof(float);
}

int turtle_train_rgemm(const void* a, int64_t lda, const void* b, int64_t ldb, float* c, int64_t P, int N, int K, int64_t img_px,
                       int accumulate, int dtype, void* ws, size_t ws_bytes, void* stream) {
  if (dtype != 0 && dtype != 1) return -1;
  if (!rows_ok(a, lda, dtype) || !rows_ok(b, ldb, dtype) || !c || P <= 0 || N <= 0 || K <= 0 || N % 8 || K % 8 || lda < N ||
      ldb < K || (img_px > 0 && P % img_px))
    return -1;
  const int64_t plen = img_px > 0 ? img_px : P;
  const int64_t nimg = img_px > 0 ? P / img_px : 1;
  int64_t nsplit = rgemm_splits(P, N, K, img_px, 1, dtype);
  if (!ws || ws_bytes < (size_t)nsplit * nimg * N * K * sizeof(float) || nimg > 65535) return -1;
  int64_t ppb = (plen + nsplit - 1) / nsplit;
  ppb = (ppb + RG_BP - 1) / RG_BP * RG_BP;
  nsplit = (plen + ppb - 1) / ppb;
  const int tn = rgemm_tn(N, dtype), tk = rgemm_tn(K, dtype);
  const dim3 grid((unsigned)(((N + tn - 1) / tn) * ((K + tk - 1) / tk) * nsplit), (unsigned)nimg);
  hipStream_t st = (hipStream_t)stream;
  float* part = reinterpret_cast<float*>(ws);
  if (dtype == 1)
    launch_rgemm_bf16(tn, tk, grid, st, (const bf16*)a, lda, (const bf16*)b, ldb, part, img_px, (int)nimg, N, K, P, ppb, 0, 0);
  else
    hipLaunchKernelGGL(rgemm_f32_kernel, grid, dim3(256), 0, st, (const float*)a, lda, (const float*)b, ldb, part, img_px,
                       (int)nimg, N, K, P, ppb);
  const int64_t n = nimg * N * K;
  if ((n + 63) / 64 >= 512)
    hipLaunchKernelGGL(rgemm_reduce_kernel<64>, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, st, part, c, n, (int)nsplit, accumulate);
  else
    hipLaunchKernelGGL(rgemm_reduce_kernel<16>, dim3((unsigned)((n + 15) / 16)), dim3(256), 0, st, part, c, n, (int)nsplit, accumulate);
  return (int)hipGetLastError();
}

}  // extern "C"

// Channel ("transposed") attention for ChannelAttention / FrameHistoryRouter / the FHR inside the
// Causal History Model (turtle_t1_arch.py:218-286, 612-662, 666-702), restructured for HBM:
//
//   1. gram:      split over pixels, per (batch, head): G = q^T [k_seg0 | k_seg1 | ...] and the
//                 per-channel sums of squares (for F.normalize over HW), fp32 MFMA 16x16x4.
//   2. finalize:  reduce the pixel splits, logits = G / (|q_i| |k_j|) * temperature, row softmax
//                 (over all cached + current key rows of the head), 1/|k_cur| for the FHR cache.
//   3. weff:      fold attention into the projection: W_eff = project_out . blockdiag(A_h), so
//                 project_out(A v) becomes ONE pointwise GEMM over the K-concatenated value
//                 sources (current v, cached v rows, CHM history frames) with the residual add
//                 in its epilogue (gemm.hip). No attention output map is ever written.
#include "common.h"
#include "kernels.h"

namespace turtle {

constexpr int GP = 32;           // pixels per Gram staging tile
constexpr int GMAXT = 24;        // max 16x16 accumulator tiles per wave (ch=64, 6 segments)

template <typename T>
__global__ __launch_bounds__(256) void gram_kernel(GramArgs a) {
  extern __shared__ __attribute__((aligned(16))) float gsm[];
  const int ch = a.ch, ncol = a.nseg * ch;
  float* sq = gsm;                 // [GP][ch]
  float* sk = gsm + GP * ch;       // [GP][ncol]
  const int bh = blockIdx.x / a.nchunk, chunk = blockIdx.x % a.nchunk;
  const int b = bh / a.heads, h = bh % a.heads;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int p_beg = chunk * a.chunk, p_end = min(a.HW, p_beg + a.chunk);
  const int ti_n = ch / 16, tj_n = ncol / 16, TT = ti_n * tj_n;
  constexpr int VEC = Vec<T>::N;
  const int qv = ch / VEC, kvn = ncol / VEC;

  f32x4 acc[GMAXT];
#pragma unroll
  for (int t = 0; t < GMAXT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float nq = 0.f, nk0 = 0.f, nk1 = 0.f;   // column sums of squares (threads own columns)

  for (int p0 = p_beg; p0 < p_end; p0 += GP) {
    // stage q and the key segments of GP pixels as fp32
    for (int v = tid; v < GP * (qv + kvn); v += 256) {
      const int pr = v / (qv + kvn), cvi = v % (qv + kvn);
      const int p = p0 + pr;
      Vec<T> x; x.zero();
      float* dst;
      if (cvi < qv) {
        if (p < p_end)
          x.load(reinterpret_cast<const T*>(a.q) + ((int64_t)b * a.HW + p) * a.ldq + a.qoff + h * ch + cvi * VEC);
        dst = sq + pr * ch + cvi * VEC;
      } else {
        const int kc = (cvi - qv) * VEC, s = kc / ch, j = kc % ch;
        const GramSeg& g = a.seg[s];
        if (p < p_end)
          x.load(reinterpret_cast<const T*>(g.base) +
                 (((int64_t)b * g.img_mul + g.img_add) * a.HW + p) * g.ld + g.off + (int64_t)h * g.hstride + j);
        dst = sk + pr * ncol + kc;
      }
#pragma unroll
      for (int i = 0; i < VEC; ++i) dst[i] = x.v[i];
    }
    __syncthreads();
    // column sums of squares
    if (tid < ch + ncol) {
      for (int pr = 0; pr < GP; ++pr) {
        float x = tid < ch ? sq[pr * ch + tid] : sk[pr * ncol + tid - ch];
        nq += x * x;
      }
    }
    if (tid + 256 < ch + ncol) {
      for (int pr = 0; pr < GP; ++pr) {
        float x = sk[pr * ncol + tid + 256 - ch];
        nk0 += x * x;
      }
    }
    // MFMA: D[i][j] += sum_kk q[kk][i] k[kk][j]; lane supplies A[i=l&15][kk=l>>4], B[kk][j=l&15]
#pragma unroll
    for (int kk = 0; kk < GP; kk += 4) {
      const int pr = kk + (lane >> 4);
#pragma unroll
      for (int t = 0; t < GMAXT; ++t) {
        const int tile = wid + 4 * t;
        if (tile < TT) {
          const int it = tile / tj_n, jt = tile % tj_n;
          const float av = sq[pr * ch + it * 16 + (lane & 15)];
          const float bv = sk[pr * ncol + jt * 16 + (lane & 15)];
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[t], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  (void)nk1;
  const int stride = ch * ncol + ch + ncol;
  float* out = a.part + ((int64_t)bh * a.nchunk + chunk) * stride;
#pragma unroll
  for (int t = 0; t < GMAXT; ++t) {
    const int tile = wid + 4 * t;
    if (tile < TT) {
      const int it = tile / tj_n, jt = tile % tj_n;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out[(it * 16 + (lane >> 4) * 4 + r) * ncol + jt * 16 + (lane & 15)] = acc[t][r];
    }
  }
  if (tid < ch + ncol) out[ch * ncol + tid] = nq;          // [nq (ch) | nk (ncol)]
  if (tid + 256 < ch + ncol) out[ch * ncol + tid + 256] = nk0;
}

template <typename T>
void launch_gram(const GramArgs& a, hipStream_t st) {
  const int ncol = a.nseg * a.ch;
  const size_t lds = (size_t)GP * (a.ch + ncol) * sizeof(float);
  hipLaunchKernelGGL(gram_kernel<T>, dim3((unsigned)(a.B * a.heads * a.nchunk)), dim3(256), lds, st, a);
}

// reduce the pixel splits: red[bh][e] = sum_c part[bh][c][e]
__global__ __launch_bounds__(256) void gram_reduce_kernel(const float* part, float* red, int nchunk, int stride, int nbh) {
  const int64_t total = (int64_t)nbh * stride;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    const int64_t bh = idx / stride, e = idx % stride;
    const float* p = part + bh * nchunk * stride + e;
    float s = 0.f;
    for (int c = 0; c < nchunk; ++c) s += p[(int64_t)c * stride];
    red[idx] = s;
  }
}

// one block per (b, h): logits, softmax over all key columns, 1/|k_cur|
__global__ __launch_bounds__(256) void attn_softmax_kernel(AttnFinArgs a) {
  const int ch = a.ch, ncol = a.nseg * ch, stride = ch * ncol + ch + ncol;
  const int bh = blockIdx.x, b = bh / a.heads, h = bh % a.heads;
  const float* G = a.red + (int64_t)bh * stride;
  const float* nq = G + ch * ncol;
  const float* nk = nq + ch;
  __shared__ float kinv_s[512];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int j = tid; j < ncol; j += 256) {
    const int s = j / ch;
    kinv_s[j] = ((a.norm_mask >> s) & 1) ? 1.f / fmaxf(sqrtf(nk[j]), 1e-12f) : 1.f;
  }
  __syncthreads();
  const float tau = a.tau[h];
  float* A = a.attn + (int64_t)bh * ch * ncol;
  for (int i = wid; i < ch; i += 4) {
    const float qi = tau / fmaxf(sqrtf(nq[i]), 1e-12f);
    float mx = -INFINITY;
    for (int j = lane; j < ncol; j += 64) mx = fmaxf(mx, G[i * ncol + j] * qi * kinv_s[j]);
    mx = wave_max(mx);
    float sum = 0.f;
    for (int j = lane; j < ncol; j += 64) {
      const float e = expf(G[i * ncol + j] * qi * kinv_s[j] - mx);
      A[i * ncol + j] = e;
      sum += e;
    }
    sum = wave_sum(sum);
    const float inv = 1.f / sum;
    for (int j = lane; j < ncol; j += 64) A[i * ncol + j] *= inv;
  }
  if (a.kinv && a.cur_seg >= 0)
    for (int j = tid; j < ch; j += 256) a.kinv[(int64_t)b * a.heads * ch + h * ch + j] = kinv_s[a.cur_seg * ch + j];
}

void launch_attn_finalize(const AttnFinArgs& a, hipStream_t st) {
  const int ncol = a.nseg * a.ch, stride = a.ch * ncol + a.ch + ncol, nbh = a.B * a.heads;
  int64_t blocks = ((int64_t)nbh * stride + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(gram_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a.part, a.red, a.nchunk, stride, nbh);
  hipLaunchKernelGGL(attn_softmax_kernel, dim3((unsigned)nbh), dim3(256), 0, st, a);
}

// W_eff[b][o][seg_col[s] + h*seg_hstride[s] + j] = sum_i Wp[o][h*ch + i] * A[b,h][i][s*ch + j]
template <typename T>
__global__ __launch_bounds__(256) void weff_kernel(WeffArgs a) {
  const int ch = a.ch, ncol = a.nseg * ch;
  const int64_t total = (int64_t)a.B * a.C * a.heads * ncol;
  T* W = reinterpret_cast<T*>(a.weff);
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    const int col = (int)(idx % ncol);
    int64_t t = idx / ncol;
    const int h = (int)(t % a.heads); t /= a.heads;
    const int o = (int)(t % a.C);
    const int b = (int)(t / a.C);
    const int s = col / ch, j = col % ch;
    const float* wp = a.wp + (int64_t)o * a.C + h * ch;
    const float* A = a.attn + ((int64_t)(b * a.heads + h) * ch) * ncol + col;
    float acc = 0.f;
    for (int i = 0; i < ch; ++i) acc = fmaf(wp[i], A[(int64_t)i * ncol], acc);
    W[((int64_t)b * a.C + o) * a.Keff + a.seg_col[s] + (int64_t)h * a.seg_hstride[s] + j] = from_f<T>(acc);
  }
}

template <typename T>
void launch_weff(const WeffArgs& a, hipStream_t st) {
  const int64_t total = (int64_t)a.B * a.C * a.heads * a.nseg * a.ch;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(weff_kernel<T>, dim3((unsigned)blocks), dim3(256), 0, st, a);
}

template void launch_gram<float>(const GramArgs&, hipStream_t);
template void launch_gram<bf16>(const GramArgs&, hipStream_t);
template void launch_weff<float>(const WeffArgs&, hipStream_t);
template void launch_weff<bf16>(const WeffArgs&, hipStream_t);

}  // namespace turtle

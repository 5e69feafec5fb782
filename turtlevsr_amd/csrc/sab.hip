// State-Align Block cross-frame attention (turtle_t1_arch.py:548-610 live forward, with
// zero_out_non_top_k 394-416, create_local_attention_mask 448-464, clipped_softmax 115-132).
//
// The reference materialises S = q k^T * tau as a dense [B,T,1,N,N] tensor, a top-5 mask, an
// N x N L1-ball mask built on the CPU, and a dense A.v. Only the entries in (top-5 U ball) survive
// the clipped softmax (<= 5 + 41 per row), so here:
//
//   sab_score: streams key tiles through LDS, MFMA score tiles (fp32 accumulate), keeps a
//              per-query running top-5 in registers -> [B,T,N,5] values + indices. The N x N
//              score matrix never reaches HBM.
//   sab_av:    per (b, t, query): re-scores the analytic ball (|di|+|dj| <= 4 on the token grid),
//              merges with the top-5 (an entry in both counts twice: logit 2*s), drops exact-zero
//              logits, softmaxes (per frame, never joint over T) and gathers the <= 46 dilated
//              value tokens straight into the pixel-major aligned frame (inverse dilated regroup,
//              602-604, fused).
// Tie-break of equal scores: lower key index first.
#include "common.h"
#include "kernels.h"
#include "mma.h"

namespace turtle {

constexpr int SAB_K = 5;

struct Top5 {
  float v[SAB_K];
  int i[SAB_K];
  TURTLE_DEV void init() {
#pragma unroll
    for (int k = 0; k < SAB_K; ++k) { v[k] = -INFINITY; i[k] = 0x7fffffff; }
  }
  TURTLE_DEV static bool better(float a, int ia, float b, int ib) { return a > b || (a == b && ia < ib); }
  TURTLE_DEV void insert(float x, int ix) {
    if (!better(x, ix, v[SAB_K - 1], i[SAB_K - 1])) return;
    v[SAB_K - 1] = x; i[SAB_K - 1] = ix;
#pragma unroll
    for (int k = SAB_K - 1; k > 0; --k) {
      if (better(v[k], i[k], v[k - 1], i[k - 1])) {
        float tv = v[k]; v[k] = v[k - 1]; v[k - 1] = tv;
        int ti = i[k]; i[k] = i[k - 1]; i[k - 1] = ti;
      }
    }
  }
};

// block: 64 queries (16 per wave) x all keys of one (b, t); key tiles of 64 through LDS
template <typename T>
__global__ __launch_bounds__(256) void sab_score_kernel(SabScoreArgs a) {
  using M = Mma<T>;
  constexpr int BK = M::BK, VEC = M::VEC, KV = BK / VEC;
  __shared__ __attribute__((aligned(16))) char smem[2 * 64 * ROWB];
  __shared__ float mv[64][4][SAB_K];
  __shared__ int mi[64][4][SAB_K];
  char* sQ = smem;
  char* sK = smem + 64 * ROWB;
  const int nqt = (a.N + 63) / 64;
  const int qt = blockIdx.x % nqt;
  const int bt = blockIdx.x / nqt;
  const int b = bt / a.T, t = bt % a.T;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const T* q = reinterpret_cast<const T*>(a.q) + (int64_t)b * a.q_bstride;
  const T* k = reinterpret_cast<const T*>(a.k[t]) + (int64_t)b * a.k_bstride[t];
  const float tau = *a.tau;
  const int kv = tid % KV;
  Top5 top; top.init();
  for (int m0 = 0; m0 < a.N; m0 += 64) {
    f32x4 acc[4][4];
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int d0 = 0; d0 < a.d; d0 += BK) {
#pragma unroll
      for (int rr = 0; rr < 64 * KV / 256; ++rr) {
        const int r = tid / KV + rr * (256 / KV);
        const int dd = d0 + kv * VEC;
        Vec<T> xq, xk; xq.zero(); xk.zero();
        const int n = qt * 64 + r, m = m0 + r;
        if (dd < a.d) {
          if (n < a.N) xq.load(q + (int64_t)n * a.d + dd);
          if (m < a.N) xk.load(k + (int64_t)m * a.d + dd);
        }
        xq.store(reinterpret_cast<T*>(sQ + r * ROWB) + kv * VEC);
        xk.store(reinterpret_cast<T*>(sK + r * ROWB) + kv * VEC);
      }
      __syncthreads();
#pragma unroll
      for (int ks = 0; ks < BK / M::KSUB; ++ks) mma_step<T>(sK, sQ, lane, ks, acc, 1, 4, 0, wid * 16);
      __syncthreads();
    }
    // lane: query wid*16 + (lane&15); keys m0 + tn*16 + (lane>>4)*4 + r
#pragma unroll
    for (int tn = 0; tn < 4; ++tn)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + tn * 16 + (lane >> 4) * 4 + r;
        if (m < a.N) top.insert(acc[0][tn][r] * tau, m);
      }
  }
  const int ql = wid * 16 + (lane & 15);
#pragma unroll
  for (int x = 0; x < SAB_K; ++x) { mv[ql][lane >> 4][x] = top.v[x]; mi[ql][lane >> 4][x] = top.i[x]; }
  __syncthreads();
  if (tid < 64) {
    const int n = qt * 64 + tid;
    Top5 m; m.init();
    for (int g = 0; g < 4; ++g)
      for (int x = 0; x < SAB_K; ++x) m.insert(mv[tid][g][x], mi[tid][g][x]);
    if (n < a.N) {
      const int64_t o = ((int64_t)bt * a.N + n) * SAB_K;
      for (int x = 0; x < SAB_K; ++x) { a.topv[o + x] = m.v[x]; a.topi[o + x] = m.i[x]; }
    }
  }
}

template <typename T>
void launch_sab_score(const SabScoreArgs& a, hipStream_t st) {
  const int nqt = (a.N + 63) / 64;
  hipLaunchKernelGGL(sab_score_kernel<T>, dim3((unsigned)(a.B * a.T * nqt)), dim3(256), 0, st, a);
}

// ------------------------------------------------------------------------------------------
// block per (b, t, query n): candidates, clipped softmax, sparse gather of dilated v tokens
// ------------------------------------------------------------------------------------------
constexpr int BALL = 41;         // |di| + |dj| <= 4
constexpr int MAXC = BALL + SAB_K;

template <typename T>
__global__ __launch_bounds__(256) void sab_av_kernel(SabAvArgs a) {
  constexpr int VEC = Vec<T>::N;
  __shared__ int cm[MAXC];       // key index or -1
  __shared__ float cl[MAXC];     // logit
  __shared__ int cmul[MAXC];
  __shared__ float cw[MAXC];     // softmax weight
  const int n = blockIdx.x % a.N;
  const int bt = blockIdx.x / a.N;
  const int b = bt / a.T, t = bt % a.T;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ti = n / a.tw, tj = n % a.tw;
  const int64_t o5 = ((int64_t)bt * a.N + n) * SAB_K;
  const float tau = *a.tau;
  const T* q = reinterpret_cast<const T*>(a.q) + (int64_t)b * a.q_bstride + (int64_t)n * a.d;
  const T* k = reinterpret_cast<const T*>(a.k[t]) + (int64_t)b * a.k_bstride[t];
  const T* v = reinterpret_cast<const T*>(a.v[t]) + (int64_t)b * a.v_bstride[t];

  if (tid < MAXC) {
    int m = -1, mul = 0;
    float s = 0.f;
    if (tid < BALL) {
      // enumerate the L1 ball: rows di = -4..4 hold 2*(4-|di|)+1 entries
      int c = tid, di = -4;
      while (c >= 2 * (4 - abs(di)) + 1) { c -= 2 * (4 - abs(di)) + 1; ++di; }
      const int dj = c - (4 - abs(di));
      const int ii = ti + di, jj = tj + dj;
      if (ii >= 0 && ii < a.th && jj >= 0 && jj < a.tw) {
        m = ii * a.tw + jj; mul = 1;
        for (int x = 0; x < SAB_K; ++x)
          if (a.topi[o5 + x] == m) { mul = 2; s = a.topv[o5 + x]; }
      }
    } else {
      const int x = tid - BALL;
      const int mm = a.topi[o5 + x];
      const int mi = mm / a.tw, mj = mm % a.tw;
      if (abs(mi - ti) + abs(mj - tj) > 4) { m = mm; mul = 1; s = a.topv[o5 + x]; }
    }
    cm[tid] = m; cmul[tid] = mul; cl[tid] = s;
  }
  __syncthreads();
  // score the ball-only candidates: one wave per candidate
  for (int c = wid; c < BALL; c += 4) {
    if (cm[c] < 0 || cmul[c] == 2) continue;
    const T* kr = k + (int64_t)cm[c] * a.d;
    float s = 0.f;
    for (int e = lane; e < a.d; e += 64) s = fmaf(to_f(q[e]), to_f(kr[e]), s);
    s = wave_sum(s);
    if (lane == 0) cl[c] = s * tau;
  }
  __syncthreads();
  if (tid < 64) {
    // clipped softmax over candidates whose logit s*mult is not exactly zero
    float l = -INFINITY;
    bool ok = false;
    if (tid < MAXC && cm[tid] >= 0) {
      l = cl[tid] * (float)cmul[tid];
      ok = l != 0.f;
      if (!ok) l = -INFINITY;
    }
    const float mx = wave_max(l);
    const float e = ok ? expf(l - mx) : 0.f;
    const float sum = wave_sum(e);
    if (tid < MAXC) cw[tid] = e / sum;
  }
  __syncthreads();
  // gather: out[(p1*ws+p2)*C + c] of token n -> pixel (p1*th + ti, p2*tw + tj)
  const int D = a.ws * a.ws * a.C;
  const int Hl = a.th * a.ws, Wl = a.tw * a.ws;
  T* out = reinterpret_cast<T*>(a.out) + (int64_t)bt * Hl * Wl * a.C;
  for (int e0 = tid * VEC; e0 < D; e0 += 256 * VEC) {
    float acc[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[i] = 0.f;
    for (int c = 0; c < MAXC; ++c) {
      const float w = cw[c];
      if (w == 0.f) continue;
      Vec<T> x; x.load(v + (int64_t)cm[c] * D + e0);
#pragma unroll
      for (int i = 0; i < VEC; ++i) acc[i] = fmaf(w, x.v[i], acc[i]);
    }
    const int sub = e0 / a.C, c0 = e0 % a.C;
    const int p1 = sub / a.ws, p2 = sub % a.ws;
    const int y = p1 * a.th + ti, x = p2 * a.tw + tj;
    Vec<T> o;
#pragma unroll
    for (int i = 0; i < VEC; ++i) o.v[i] = acc[i];
    o.store(out + ((int64_t)y * Wl + x) * a.C + c0);
  }
}

template <typename T>
void launch_sab_av(const SabAvArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(sab_av_kernel<T>, dim3((unsigned)(a.B * a.T * a.N)), dim3(256), 0, st, a);
}

template void launch_sab_score<float>(const SabScoreArgs&, hipStream_t);
template void launch_sab_score<bf16>(const SabScoreArgs&, hipStream_t);
template void launch_sab_av<float>(const SabAvArgs&, hipStream_t);
template void launch_sab_av<bf16>(const SabAvArgs&, hipStream_t);

}  // namespace turtle

// State-Align Block cross-frame attention (turtle_t1_arch.py:548-610 live forward, with
// zero_out_non_top_k 394-416, create_local_attention_mask 448-464, clipped_softmax 115-132).
//
// The reference materialises S = q k^T * tau as a dense [B,T,1,N,N] tensor, a top-5 mask, an
// N x N L1-ball mask built on the CPU, and a dense A.v. Only the entries in (top-5 U ball) survive
// the clipped softmax (<= 5 + 41 per row), so here three kernels:
//
//   sab_score:  MFMA score tiles (keys in a double-buffered LDS ring, the block's 64 queries as
//               register fragments), per-query running top-5 in registers, and the scores of the
//               41 L1-ball keys recorded as they stream past. The key range is split over
//               `nsplit` blocks (partial top-5 lists) so the grid fills the chip. The N x N score
//               matrix never reaches HBM.
//   sab_prep:   per (b, t, query): merge the partial top-5 lists, candidates = ball U top-5 (an
//               entry in both counts twice: logit 2*s), drop exact-zero logits, softmax (per
//               frame, never joint over T), compact the surviving (key, weight) pairs.
//   sab_gather: out = sum_c w_c v[key_c], one wave per (D chunk, b, t, query) with the D chunk
//               the slowest grid index: consecutive waves walk the queries of one chunk, so the
//               9-token-row window of value rows they share stays in L2 and the random top-5
//               rows of the chunk (N x 1 KB) stay in the Infinity Cache. Writes the inverse
//               dilated regroup (602-604) straight into the pixel-major aligned frame.
// Tie-break of equal scores: lower key index first.
#include "common.h"
#include "kernels.h"
#include "mma.h"

namespace turtle {

constexpr int SAB_K = 5;
constexpr int BALL = 41;         // |di| + |dj| <= 4

__device__ __attribute__((aligned(64))) uint4 g_zero_sab[4];

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

// ball slot of offset (di, dj), |di| + |dj| <= 4: rows di = -4..4 hold 1,3,5,7,9,7,5,3,1 entries
TURTLE_DEV int ball_slot(int di, int dj) {
  const int a = di < 0 ? -di : di;
  const int start = di <= 0 ? (4 + di) * (4 + di) : 41 - (5 - di) * (5 - di);   // rows before di
  return start + dj + (4 - a);
}
TURTLE_DEV void ball_offset(int slot, int& di, int& dj) {
  int c = slot;
  di = -4;
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    const int len = 2 * (4 - (di < 0 ? -di : di)) + 1;
    if (c >= len) { c -= len; ++di; }
  }
  dj = c - (4 - (di < 0 ? -di : di));
}

// exact m / tw for 0 <= m < 2^24 (float reciprocal + one correction each way)
TURTLE_DEV int div_tw(int m, int tw, float inv) {
  int r = (int)((float)m * inv);
  r += (r + 1) * tw <= m;
  r -= r * tw > m;
  return r;
}

// ------------------------------------------------------------------------------------------
// scores + top-5 + ball scores. Block = 64 queries (16 per wave) x one key range; key tiles of KT
// rows are staged in a 2-slot LDS ring (register staging, one barrier per tile)
// ------------------------------------------------------------------------------------------
template <typename T, int KT, int QK>
__global__ __launch_bounds__(256) void sab_score_kernel(SabScoreArgs a) {
  using FR = typename Frag<T>::type;
  constexpr int KF = Frag<T>::K, VEC = Vec<T>::N, ES = sizeof(T), MT = KT / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ROW = a.d * ES + 16;
  char* sK0 = smem;
  char* sK1 = smem + KT * ROW;
  float* mv = reinterpret_cast<float*>(smem + 2 * KT * ROW);   // [64][4][5]
  int* mi = reinterpret_cast<int*>(mv + 64 * 4 * SAB_K);

  const int nqt = (a.N + 63) / 64;
  int bid = blockIdx.x;
  const int ks = bid % a.nsplit;
  bid /= a.nsplit;
  const int qt = bid % nqt, bt = bid / nqt;
  const int b = bt / a.T, t = bt % a.T;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const T* q = reinterpret_cast<const T*>(a.q) + (int64_t)b * a.q_bstride;
  // frame t's key base: static-index select scan (no dynamic kernel-argument indexing)
  const T* k = reinterpret_cast<const T*>(a.k[0]);
  int64_t kbs = a.k_bstride[0];
#pragma unroll
  for (int j = 1; j < TURTLE_MAX_T; ++j)
    if (t == j) { k = reinterpret_cast<const T*>(a.k[j]); kbs = a.k_bstride[j]; }
  k += (int64_t)b * kbs;
  const float tau = *a.tau;
  const int d = a.d, nk = d / KF, N = a.N;

  // this lane's query (B operand rows) and its fragments for every K step
  const int nq = qt * 64 + wid * 16 + (lane & 15);
  const bool qok = nq < N;
  FR qf[QK];
  {
    const T* qr = q + (int64_t)min(nq, N - 1) * d;
#pragma unroll
    for (int kk = 0; kk < QK; ++kk) {
      if constexpr (sizeof(T) == 2) {
        const int e = min(kk * KF + (lane >> 4) * 8, d - 8);
        qf[kk] = __builtin_bit_cast(bf16x8, ld16(qr + e));
      } else {
        qf[kk] = ld4f(qr + min(kk * KF + (lane >> 4), d - 1));
      }
    }
  }
  // key tiles of this split
  const int ntile = (N + KT - 1) / KT;
  const int tb = ks * ntile / a.nsplit, te = (ks + 1) * ntile / a.nsplit;
  const int cv = d / VEC;                      // vectors per key row
  constexpr int NVMAX = KT * (QK * KF / VEC) / 256;
  const int nv = KT * cv / 256;                // staged vectors per thread (<= NVMAX)
  uint4 stg[NVMAX];
  auto load_tile = [&](int it) {
#pragma unroll
    for (int i = 0; i < NVMAX; ++i) {
      if (i < nv) {
        const int v = tid + 256 * i, r = v / cv, e = (v - r * cv) * VEC;
        const int m = min(it * KT + r, N - 1);
        stg[i] = ld16(k + (int64_t)m * d + e);
      }
    }
  };
  auto store_tile = [&](char* dst) {
#pragma unroll
    for (int i = 0; i < NVMAX; ++i) {
      if (i < nv) {
        const int v = tid + 256 * i, r = v / cv, e = (v - r * cv) * VEC;
        *reinterpret_cast<uint4*>(dst + r * ROW + e * ES) = stg[i];
      }
    }
  };

  // ball band of this block's queries (token rows), scalar
  const float inv_tw = 1.f / (float)a.tw;
  const int qrow_lo = (qt * 64) / a.tw, qrow_hi = min(qt * 64 + 63, N - 1) / a.tw;
  const int nrow = div_tw(min(nq, N - 1), a.tw, inv_tw), ncol = min(nq, N - 1) - nrow * a.tw;
  float* ballq = a.ballv + ((int64_t)bt * N + min(nq, N - 1)) * BALL;

  Top5 top; top.init();
  if (tb < te) {
    load_tile(tb);
    store_tile(sK0);
    if (tb + 1 < te) load_tile(tb + 1);
  }
  __syncthreads();
  for (int it = tb; it < te; ++it) {
    const char* sK = ((it - tb) & 1) ? sK1 : sK0;
    f32x4 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < QK; ++kk) {
      if (kk < nk) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[mt] = mfma(frag_at<T>(sK + mt * 16 * ROW, ROW, kk * KF, lane), qf[kk], acc[mt]);
      }
    }
    // next tile into the other slot (its last readers passed the previous barrier), then refill
    if (it + 1 < te) store_tile(((it - tb) & 1) ? sK0 : sK1);
    if (it + 2 < te) load_tile(it + 2);
    // lane: query nq; keys it*KT + mt*16 + 4(l>>4) + r
    const int m0 = it * KT;
    const int krow_lo = m0 / a.tw, krow_hi = min(m0 + KT - 1, N - 1) / a.tw;
    const bool band = krow_hi >= qrow_lo - 4 && krow_lo <= qrow_hi + 4;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + mt * 16 + (lane >> 4) * 4 + r;
        const float s = acc[mt][r] * tau;
        if (m < N) top.insert(s, m);
        if (band && qok && m < N) {
          const int mrow = div_tw(m, a.tw, inv_tw), mcol = m - mrow * a.tw;
          const int di = mrow - nrow, dj = mcol - ncol;
          if ((di < 0 ? -di : di) + (dj < 0 ? -dj : dj) <= 4) ballq[ball_slot(di, dj)] = s;
        }
      }
    __syncthreads();
  }
  // merge the 4 lane groups' lists of each query
  const int ql = wid * 16 + (lane & 15);
#pragma unroll
  for (int x = 0; x < SAB_K; ++x) { mv[(ql * 4 + (lane >> 4)) * SAB_K + x] = top.v[x]; mi[(ql * 4 + (lane >> 4)) * SAB_K + x] = top.i[x]; }
  __syncthreads();
  if (tid < 64) {
    const int n = qt * 64 + tid;
    Top5 m; m.init();
    for (int g = 0; g < 4; ++g)
      for (int x = 0; x < SAB_K; ++x) m.insert(mv[(tid * 4 + g) * SAB_K + x], mi[(tid * 4 + g) * SAB_K + x]);
    if (n < N) {
      const int64_t o = (((int64_t)bt * a.nsplit + ks) * N + n) * SAB_K;
      for (int x = 0; x < SAB_K; ++x) { a.topv[o + x] = m.v[x]; a.topi[o + x] = m.i[x]; }
    }
  }
}

int sab_score_nsplit(int B, int T, int N) {
  const int blocks = B * T * ((N + 63) / 64);
  int ns = (1024 + blocks - 1) / blocks;           // ~4 blocks per CU
  const int ntile = (N + 63) / 64;
  return std::max(1, std::min(ns, std::min(8, ntile)));
}

template <typename T, int KT, int QK>
static void launch_score_cfg(const SabScoreArgs& a, hipStream_t st) {
  const size_t lds = 2 * (size_t)KT * (a.d * sizeof(T) + 16) + 64 * 4 * SAB_K * 8;
  const int nqt = (a.N + 63) / 64;
  static bool attr = false;                        // > 64 KB of dynamic LDS must be opted into
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&sab_score_kernel<T, KT, QK>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((sab_score_kernel<T, KT, QK>), dim3((unsigned)(a.B * a.T * nqt * a.nsplit)), dim3(256), lds, st, a);
}

template <typename T>
void launch_sab_score(const SabScoreArgs& a, hipStream_t st) {
  // d = 2c in {128, 256, 512} for the GoPro widths; K tiles of 64 keys (32 at d = 512: LDS ring)
  constexpr int KF = Frag<T>::K;
  if (a.d <= 128) launch_score_cfg<T, 64, 128 / KF>(a, st);
  else if (a.d <= 256) launch_score_cfg<T, 64, 256 / KF>(a, st);
  else launch_score_cfg<T, 32, 512 / KF>(a, st);
}

// ------------------------------------------------------------------------------------------
// candidates + clipped softmax, one wave per (bt, query)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sab_prep_kernel(SabPrepArgs a) {
  __shared__ float sv[4][64];
  __shared__ int si[4][64];
  __shared__ float t5v[4][SAB_K];
  __shared__ int t5i[4][SAB_K];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t qi = (int64_t)blockIdx.x * 4 + w;           // (bt, n)
  if (qi >= (int64_t)a.BT * a.N) return;
  const int bt = (int)(qi / a.N), n = (int)(qi - (int64_t)bt * a.N);
  // 1) merge the nsplit partial top-5 lists: rank of each entry among all of them
  const int ne = a.nsplit * SAB_K;
  float v = -INFINITY;
  int ix = 0x7fffffff;
  if (lane < ne) {
    const int ks = lane / SAB_K, x = lane - ks * SAB_K;
    const int64_t o = (((int64_t)bt * a.nsplit + ks) * a.N + n) * SAB_K + x;
    v = a.topv[o];
    ix = a.topi[o];
  }
  sv[w][lane] = v;
  si[w][lane] = ix;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  int rank = 0;
  for (int j = 0; j < ne; ++j) rank += Top5::better(sv[w][j], si[w][j], v, ix);
  if (lane < ne && rank < SAB_K) { t5v[w][rank] = v; t5i[w][rank] = ix; }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  // 2) candidates: lanes 0..40 the ball, 41..45 the top-5 keys outside it
  const int ti = n / a.tw, tj = n - ti * a.tw;
  int m = -1, mul = 0;
  float s = 0.f;
  if (lane < BALL) {
    int di, dj;
    ball_offset(lane, di, dj);
    const int ii = ti + di, jj = tj + dj;
    if (ii >= 0 && ii < a.th && jj >= 0 && jj < a.tw) {
      m = ii * a.tw + jj; mul = 1;
      s = a.ballv[((int64_t)bt * a.N + n) * BALL + lane];
#pragma unroll
      for (int x = 0; x < SAB_K; ++x)
        if (t5i[w][x] == m) { mul = 2; s = t5v[w][x]; }
    }
  } else if (lane < BALL + SAB_K) {
    const int x = lane - BALL;
    const int mm = t5i[w][x];
    const int mr = mm / a.tw, mc = mm - mr * a.tw;
    if (abs(mr - ti) + abs(mc - tj) > 4) { m = mm; mul = 1; s = t5v[w][x]; }
  }
  // 3) clipped softmax over the candidates whose logit s*mult is not exactly zero
  float l = -INFINITY;
  const bool ok = m >= 0 && s * (float)mul != 0.f;
  if (ok) l = s * (float)mul;
  const float mx = wave_max(l);
  const float e = ok ? expf(l - mx) : 0.f;
  const float sum = wave_sum(e);
  const float wgt = e / sum;
  // 4) compact (key, weight) of the survivors; pad the slot list with (n, 0)
  const uint64_t bal = __ballot(ok);
  const int slot = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
  const int cnt = __popcll(bal);
  const int64_t o = qi * SAB_MAXC;
  if (ok) { a.ci[o + slot] = m; a.cw[o + slot] = wgt; }
  if (lane >= cnt && lane < SAB_MAXC) { a.ci[o + lane] = n; a.cw[o + lane] = 0.f; }
  if (lane == 0) a.cnt[qi] = cnt;
}

void launch_sab_prep(const SabPrepArgs& a, hipStream_t st) {
  const int64_t waves = (int64_t)a.BT * a.N;
  hipLaunchKernelGGL(sab_prep_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, a);
}

// ------------------------------------------------------------------------------------------
// sparse A.v gather: one wave per (D chunk of 64*VEC, bt, query); chunk slowest
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void sab_gather_kernel(SabGatherArgs a) {
  constexpr int VEC = Vec<T>::N, CH = 64 * VEC;
  const int D = a.ws * a.ws * a.C;
  const int64_t BTN = (int64_t)a.B * a.T * a.N;
  int lin = blockIdx.x;
  {
    const int nblk = gridDim.x, q = nblk / 8, r = nblk % 8, x = lin % 8, y = lin / 8;
    lin = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;
  }
  const int lane = threadIdx.x & 63;
  const int64_t wv = (int64_t)lin * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int chunk = (int)(wv / BTN);
  if (chunk * CH >= D) return;
  const int64_t qi = wv - (int64_t)chunk * BTN;       // bt * N + n
  const int bt = (int)(qi / a.N), n = (int)(qi - (int64_t)bt * a.N);
  const int t = bt % a.T, b = bt / a.T;
  const T* v = reinterpret_cast<const T*>(a.v[0]);
  int64_t vbs = a.v_bstride[0];
#pragma unroll
  for (int j = 1; j < TURTLE_MAX_T; ++j)
    if (t == j) { v = reinterpret_cast<const T*>(a.v[j]); vbs = a.v_bstride[j]; }
  v += (int64_t)b * vbs;
  const int e_l = chunk * CH + lane * VEC;
  const bool lok = e_l < D;                        // D need not be a multiple of the chunk
  const int e0 = lok ? e_l : 0;
  const int cnt = a.cnt[qi];
  const int* ci = a.ci + qi * SAB_MAXC;
  const float* cw = a.cw + qi * SAB_MAXC;
  float acc[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) acc[i] = 0.f;
  for (int c0 = 0; c0 < cnt; c0 += 8) {
    uint4 x[8];
    float w[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {               // slots past cnt are (n, 0) padding
      w[u] = cw[c0 + u];
      x[u] = ld16(v + (int64_t)ci[c0 + u] * D + e0);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      Vec<T> xv;
      xv.from_raw(x[u]);
#pragma unroll
      for (int i = 0; i < VEC; ++i) acc[i] = fmaf(w[u], xv.v[i], acc[i]);
    }
  }
  // token n, sub-position (p1, p2) of channel block e0 -> pixel (p1*th + ti, p2*tw + tj)
  const int ti = n / a.tw, tj = n - ti * a.tw;
  const int sub = e0 / a.C, c0 = e0 - sub * a.C;
  const int p1 = sub / a.ws, p2 = sub - p1 * a.ws;
  const int Hl = a.th * a.ws, Wl = a.tw * a.ws;
  T* out = reinterpret_cast<T*>(a.out) + (int64_t)bt * Hl * Wl * a.C;
  Vec<T> o;
#pragma unroll
  for (int i = 0; i < VEC; ++i) o.v[i] = acc[i];
  if (lok) o.store(out + ((int64_t)(p1 * a.th + ti) * Wl + p2 * a.tw + tj) * a.C + c0);
}

template <typename T>
void launch_sab_gather(const SabGatherArgs& a, hipStream_t st) {
  constexpr int CH = 64 * Vec<T>::N;
  const int D = a.ws * a.ws * a.C;
  const int64_t waves = (int64_t)((D + CH - 1) / CH) * a.B * a.T * a.N;
  hipLaunchKernelGGL(sab_gather_kernel<T>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, a);
}

template void launch_sab_score<float>(const SabScoreArgs&, hipStream_t);
template void launch_sab_score<bf16>(const SabScoreArgs&, hipStream_t);
template void launch_sab_gather<float>(const SabGatherArgs&, hipStream_t);
template void launch_sab_gather<bf16>(const SabGatherArgs&, hipStream_t);

}  // namespace turtle

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
  // branch-free insert (no-op unless x beats the 5th entry): one compare per slot and a shift
  TURTLE_DEV void insert_nb(float x, int ix) {
    bool c[SAB_K];
#pragma unroll
    for (int k = 0; k < SAB_K; ++k) c[k] = better(x, ix, v[k], i[k]);
#pragma unroll
    for (int k = SAB_K - 1; k >= 1; --k) {
      v[k] = c[k - 1] ? v[k - 1] : (c[k] ? x : v[k]);
      i[k] = c[k - 1] ? i[k - 1] : (c[k] ? ix : i[k]);
    }
    v[0] = c[0] ? x : v[0];
    i[0] = c[0] ? ix : i[0];
  }
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

// v[j] for a per-lane j < NS by a select tree on the bits of j. The selects are v_cndmask from
// inline asm on a lane mask: written as C selects, hipcc turns the tree into a stack copy of v plus
// an indexed scratch load.
TURTLE_DEV float sel_lanes(uint64_t m, float f, float t) {   // lane bit set: t, else f
  float r;
  asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
  return r;
}
template <int NS>
TURTLE_DEV float pick(const float (&v)[NS], int j) {
  static_assert(NS == 8 || NS == 16, "pick width");
  float h8[8], h4[4], h2[2];
  int b = 0;
  if constexpr (NS == 16) {
    const uint64_t m = __builtin_amdgcn_ballot_w64(j & 1);
#pragma unroll
    for (int k = 0; k < 8; ++k) h8[k] = sel_lanes(m, v[2 * k], v[2 * k + 1]);
    b = 1;
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) h8[k] = v[k];
  }
  const uint64_t m1 = __builtin_amdgcn_ballot_w64((j >> b) & 1);
#pragma unroll
  for (int k = 0; k < 4; ++k) h4[k] = sel_lanes(m1, h8[2 * k], h8[2 * k + 1]);
  const uint64_t m2 = __builtin_amdgcn_ballot_w64((j >> (b + 1)) & 1);
#pragma unroll
  for (int k = 0; k < 2; ++k) h2[k] = sel_lanes(m2, h4[2 * k], h4[2 * k + 1]);
  const uint64_t m3 = __builtin_amdgcn_ballot_w64((j >> (b + 2)) & 1);
  return sel_lanes(m3, h2[0], h2[1]);
}

// exact m / tw for 0 <= m < 2^24 (float reciprocal + one correction each way)
TURTLE_DEV int div_tw(int m, int tw, float inv) {
  int r = (int)((float)m * inv);
  r += (r + 1) * tw <= m;
  r -= r * tw > m;
  return r;
}

// ------------------------------------------------------------------------------------------
// scores + top-5 + ball scores. Block = QG x 64 queries (QG groups of 16 per wave) x one key range;
// key tiles of KT rows are staged in a 2-slot LDS ring (register staging, one barrier per tile).
// QG = 2 would let every staged key fragment feed two query groups (half the L2 -> LDS key traffic).
// ------------------------------------------------------------------------------------------
// NWQ waves per block (4 or 8): with 8, one staged key tile feeds 128 queries instead of 64, which
// halves the key stream from L2 / the Infinity Cache (the key set of a 1080p frame, 8 MB at d = 512,
// does not fit one XCD's L2)
template <typename T, int KT, int QK, int QG, int NWQ = 4>
__global__ __launch_bounds__(NWQ * 64) void sab_score_kernel(SabScoreArgs a) {
  using FR = typename Frag<T>::type;
  constexpr int NT = NWQ * 64;
  constexpr int KF = Frag<T>::K, VEC = Vec<T>::N, ES = sizeof(T), MT = KT / 16, QB = 16 * NWQ * QG;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ROW = a.d * ES + 16;
  char* sK0 = smem;
  char* sK1 = smem + KT * ROW;
  float* mv = reinterpret_cast<float*>(smem + 2 * KT * ROW);   // [QB][4][5]
  int* mi = reinterpret_cast<int*>(mv + QB * 4 * SAB_K);

  const int nqt = (a.N + QB - 1) / QB;
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
  const float inv_tw = 1.f / (float)a.tw;

  // this lane's queries (B operand rows, one per group) and their fragments for every K step
  FR qf[QG][QK];
  int nqc[QG], nrow[QG], ncol[QG];
  bool qok[QG];
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    const int nq = qt * QB + (wid * QG + g) * 16 + (lane & 15);
    qok[g] = nq < N;
    nqc[g] = min(nq, N - 1);
    nrow[g] = div_tw(nqc[g], a.tw, inv_tw);
    ncol[g] = nqc[g] - nrow[g] * a.tw;
    const T* qr = q + (int64_t)nqc[g] * d;
#pragma unroll
    for (int kk = 0; kk < QK; ++kk) {
      if constexpr (sizeof(T) == 2) {
        const int e = min(kk * KF + (lane >> 4) * 8, d - 8);
        qf[g][kk] = __builtin_bit_cast(bf16x8, ld16(qr + e));
      } else {
        qf[g][kk] = ld4f(qr + min(kk * KF + (lane >> 4), d - 1));
      }
    }
  }
  // key tiles of this split
  const int ntile = (N + KT - 1) / KT;
  const int tb = ks * ntile / a.nsplit, te = (ks + 1) * ntile / a.nsplit;
  const int cv = d / VEC;                      // vectors per key row
  constexpr int NVMAX = KT * (QK * KF / VEC) / NT;
  const int nv = KT * cv / NT;                 // staged vectors per thread (<= NVMAX)
  uint4 stg[NVMAX];
  auto load_tile = [&](int it) {
#pragma unroll
    for (int i = 0; i < NVMAX; ++i) {
      if (i < nv) {
        const int v = tid + NT * i, r = v / cv, e = (v - r * cv) * VEC;
        const int m = min(it * KT + r, N - 1);
        stg[i] = ld16(k + (int64_t)m * d + e);
      }
    }
  };
  auto store_tile = [&](char* dst) {
#pragma unroll
    for (int i = 0; i < NVMAX; ++i) {
      if (i < nv) {
        const int v = tid + NT * i, r = v / cv, e = (v - r * cv) * VEC;
        *reinterpret_cast<uint4*>(dst + r * ROW + e * ES) = stg[i];
      }
    }
  };

  // ball band of this block's queries (token rows), scalar
  const int qrow_lo = (qt * QB) / a.tw, qrow_hi = min(qt * QB + QB - 1, N - 1) / a.tw;

  Top5 top[QG];
#pragma unroll
  for (int g = 0; g < QG; ++g) top[g].init();
  if (tb < te) {
    load_tile(tb);
    store_tile(sK0);
    if (tb + 1 < te) load_tile(tb + 1);
  }
  __syncthreads();
  for (int it = tb; it < te; ++it) {
    const char* sK = ((it - tb) & 1) ? sK1 : sK0;
    f32x4 acc[QG][MT];
#pragma unroll
    for (int g = 0; g < QG; ++g)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[g][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < QK; ++kk) {
      if (kk < nk && !(a.dbg & 4)) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const FR kf = frag_at<T>(sK + mt * 16 * ROW, ROW, kk * KF, lane);
#pragma unroll
          for (int g = 0; g < QG; ++g) acc[g][mt] = mfma(kf, qf[g][kk], acc[g][mt]);
        }
      }
    }
    // next tile into the other slot (its last readers passed the previous barrier), then refill
    if (it + 1 < te) store_tile(((it - tb) & 1) ? sK0 : sK1);
    if (it + 2 < te) load_tile(it + 2);
    // lane: query of group g; keys it*KT + mt*16 + 4(l>>4) + r
    const int m0 = it * KT;
    const int krow_lo = m0 / a.tw, krow_hi = min(m0 + KT - 1, N - 1) / a.tw;
    const bool band = krow_hi >= qrow_lo - 4 && krow_lo <= qrow_hi + 4 && !(a.dbg & 2);
#pragma unroll
    for (int g = 0; g < QG; ++g) {
      // top-5: a cheap filter over the whole tile, then the candidates popped one per iteration
      // (the wave iterates max-popcount times: a few once the lists have warmed up). The 4 lanes
      // of a query (l, l^16, l^32, l^48) keep lists over disjoint key subsets; the query's final
      // 5th score is >= each list's 5th, so the largest of the four filters all of them. The
      // filter (>=) is a superset of the exact test with the index tie-break.
      float thr = top[g].v[SAB_K - 1];
      thr = fmaxf(thr, __shfl_xor(thr, 16, 64));
      thr = fmaxf(thr, __shfl_xor(thr, 32, 64));
      unsigned cand = 0;
      float sv[MT * 4];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + mt * 16 + (lane >> 4) * 4 + r;
          sv[mt * 4 + r] = acc[g][mt][r] * tau;
          cand |= (sv[mt * 4 + r] >= thr && m < N) ? 1u << (mt * 4 + r) : 0u;
        }
      if (a.dbg & 1) cand = 0;
      while (cand) {
        const int j = __builtin_ctz(cand);
        cand &= cand - 1;
        top[g].insert_nb(pick<MT * 4>(sv, j), m0 + (j >> 2) * 16 + (lane >> 4) * 4 + (j & 3));
      }
      if (band && qok[g]) {
        float* ballq = a.ballv + ((int64_t)bt * N + nqc[g]) * BALL;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = m0 + mt * 16 + (lane >> 4) * 4 + r;
            if (m < N) {
              const int mrow = div_tw(m, a.tw, inv_tw), mcol = m - mrow * a.tw;
              const int di = mrow - nrow[g], dj = mcol - ncol[g];
              if ((di < 0 ? -di : di) + (dj < 0 ? -dj : dj) <= 4) ballq[ball_slot(di, dj)] = sv[mt * 4 + r];
            }
          }
      }
    }
    __syncthreads();
  }
  // merge the 4 lane groups' lists of each query
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    const int ql = (wid * QG + g) * 16 + (lane & 15);
#pragma unroll
    for (int x = 0; x < SAB_K; ++x) {
      mv[(ql * 4 + (lane >> 4)) * SAB_K + x] = top[g].v[x];
      mi[(ql * 4 + (lane >> 4)) * SAB_K + x] = top[g].i[x];
    }
  }
  __syncthreads();
  if (tid < QB) {
    const int n = qt * QB + tid;
    Top5 m; m.init();
    for (int g = 0; g < 4; ++g)
      for (int x = 0; x < SAB_K; ++x) m.insert(mv[(tid * 4 + g) * SAB_K + x], mi[(tid * 4 + g) * SAB_K + x]);
    if (n < N) {
      const int64_t o = (((int64_t)bt * a.nsplit + ks) * N + n) * SAB_K;
      for (int x = 0; x < SAB_K; ++x) { a.topv[o + x] = m.v[x]; a.topi[o + x] = m.i[x]; }
    }
  }
}

// QG = 2 measured slower on MI355X (tools/sabbench: the second group's registers cost a wave per
// SIMD and the halved grid needs more key splits, i.e. more top-5 warm-ups); kept for tuning.
static int sab_qg(int) { return 1; }

int sab_score_nsplit(int B, int T, int N, int d, int waves) {
  // as many key splits as keep the whole grid resident in one round: each split restarts the
  // top-5 warm-up, a second round of blocks costs more than the split saves (tools/sabbench:
  // d = 128 / T = 3 / N = 8160 best at 2 splits = 768 blocks = 3 per CU, d >= 256 at 1)
  const int nw = waves == 8 ? 8 : 4;
  const int qb = 16 * nw * sab_qg(d);
  const int blocks = B * T * ((N + qb - 1) / qb);
  const int cap = 256 * (d <= 128 ? 3 : 2) * 4 / nw;   // resident score blocks on MI355X (LDS / VGPRs)
  const int ntile = (N + 63) / 64;
  return std::max(1, std::min(cap / std::max(1, blocks), std::min(8, ntile)));
}

template <typename T, int KT, int QK, int QG, int NWQ = 4>
static void launch_score_cfg(const SabScoreArgs& a, hipStream_t st) {
  constexpr int QB = 16 * NWQ * QG;
  const size_t lds = 2 * (size_t)KT * (a.d * sizeof(T) + 16) + QB * 4 * SAB_K * 8;
  const int nqt = (a.N + QB - 1) / QB;
  static bool attr = false;                        // > 64 KB of dynamic LDS must be opted into
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&sab_score_kernel<T, KT, QK, QG, NWQ>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((sab_score_kernel<T, KT, QK, QG, NWQ>), dim3((unsigned)(a.B * a.T * nqt * a.nsplit)), dim3(NWQ * 64), lds, st, a);
}

template <typename T>
void launch_sab_score(const SabScoreArgs& a, hipStream_t st) {
  // d = 2c in {128, 256, 512} for the GoPro widths; K tiles of 64 keys (32 at d = 512: LDS ring)
  constexpr int KF = Frag<T>::K;
  if (a.waves == 8) {
    if (a.d <= 128) launch_score_cfg<T, 64, 128 / KF, 1, 8>(a, st);
    else if (a.d <= 256) launch_score_cfg<T, 64, 256 / KF, 1, 8>(a, st);
    else launch_score_cfg<T, 32, 512 / KF, 1, 8>(a, st);
    return;
  }
  if (a.d <= 128) launch_score_cfg<T, 64, 128 / KF, 1>(a, st);
  else if (a.d <= 256) launch_score_cfg<T, 64, 256 / KF, 1>(a, st);
  else launch_score_cfg<T, 32, 512 / KF, 1>(a, st);
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
  // slots no entry ranks into (non-finite scores tie) stay "no key", never stale LDS
  if (lane < SAB_K) { t5v[w][lane] = -INFINITY; t5i[w][lane] = -1; }
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
    // only real keys reach the gather (a NaN frame must give NaN output, not an out-of-range read)
    if (mm >= 0 && mm < a.N && abs(mr - ti) + abs(mc - tj) > 4) { m = mm; mul = 1; s = t5v[w][x]; }
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
  // dense ball weights (0 = excluded / outside the grid) for the matrix-core A.v (in place of the
  // ball scores this lane read above)
  if (lane < BALL) a.ballw[((int64_t)bt * a.N + n) * BALL + lane] = ok ? wgt : 0.f;
  if (lane >= cnt && lane < SAB_MAXC) { a.ci[o + lane] = n; a.cw[o + lane] = 0.f; }
  const int nball = __popcll(bal & ((1ull << BALL) - 1));     // ball candidates come first
  if (lane == 0) a.cnt[qi] = cnt | (nball << 16);
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
  const int cnt = a.cnt[qi] & 0xffff;
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

// ------------------------------------------------------------------------------------------
// sparse A.v on the matrix cores. The 41 L1-ball keys of the 8 x 8 query tokens of a tile all lie
// in the 16 x 16 token square around it, so the ball part of A.v for the tile is a dense product
//   O[64 q][e] = W'[64 q][256 square keys] . V[256 keys][e]          (41 non-zeros per W' row)
// (bf16 MFMA 16x16x32, fp32 accumulation). W' is built once per block from the dense ball
// weights sab_prep leaves in `ballw` and kept in registers as MFMA A fragments; the block then
// walks its range of 64-element chunks of D: V chunk [256][64] staged in LDS (register double
// buffer, padded rows, transposed ds_read_b64_tr_b16 B fragments), MFMA, then the <= 5 top-k
// keys outside the ball are added per query from L2 and the result is written with the inverse
// dilated regroup (turtle_t1_arch.py:602-604) into the pixel-major aligned frame.
// ------------------------------------------------------------------------------------------
constexpr int SM_T = 8, SM_S = 16;                 // query tile / key square side (tokens)
constexpr int SM_E = 64;                           // D elements per chunk
constexpr int SM_RV = SM_E * 2 + 16;               // staged V row bytes (padded)
constexpr int SM_RO = SM_E + 4;                    // output staging row (floats)
// DB: V chunk double-buffered in LDS and the tail rows prefetched one chunk ahead (1 block per CU,
// one wave per SIMD); !DB: one V buffer (the register staging is the second stage), tail rows
// fetched at the top of their own chunk, <= 256 registers: two blocks per CU
template <bool DB> constexpr int sm_lds() { return (DB ? 2 : 1) * 256 * SM_RV + 64 * SM_RO * 4 + 64 * SAB_K * 8; }

// PF (with !DB): the tail rows of chunk c + 1 are fetched at the top of chunk c into a second
// register set, so their L2 latency overlaps a whole chunk at two blocks per CU. Measured slower
// than fetching them at the top of their own chunk (level 1 757 vs 724 us at 1080p); sab_db = 2.
template <bool DB, bool PF>
__global__ __launch_bounds__(256, DB ? 1 : 2) void sab_av_mfma_kernel(SabGatherArgs a, int nsplit) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  char* sV = sm;                                   // [1 or 2][256][SM_RV]
  float* sO = reinterpret_cast<float*>(sm + (DB ? 2 : 1) * 256 * SM_RV);   // [64][SM_RO]
  int* sTi = reinterpret_cast<int*>(sO + 64 * SM_RO);           // [64][5] tail keys
  float* sTw = reinterpret_cast<float*>(sTi + 64 * SAB_K);      // [64][5] tail weights
  const int D = a.ws * a.ws * a.C, nch = D / SM_E;
  const int tty = (a.th + SM_T - 1) / SM_T, ttx = (a.tw + SM_T - 1) / SM_T;
  int lin = blockIdx.x;
  {
    const int nblk = gridDim.x, q = nblk / 8, r = nblk % 8, x = lin % 8, y = lin / 8;
    lin = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;
  }
  const int split = lin % nsplit;
  int rest = lin / nsplit;
  const int tile = rest % (tty * ttx);
  const int bt = rest / (tty * ttx);
  const int ch_beg = split * nch / nsplit, ch_end = (split + 1) * nch / nsplit;
  const int ti0 = (tile / ttx) * SM_T, tj0 = (tile % ttx) * SM_T;
  const int t = bt % a.T, b = bt / a.T;
  const bf16* v = reinterpret_cast<const bf16*>(a.v[0]);
  int64_t vbs = a.v_bstride[0];
#pragma unroll
  for (int j = 1; j < TURTLE_MAX_T; ++j)
    if (t == j) { v = reinterpret_cast<const bf16*>(a.v[j]); vbs = a.v_bstride[j]; }
  v += (int64_t)b * vbs;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

  // ---- tail lists (top-k keys outside the ball), 64 queries x <= 5 ----
  for (int e = tid; e < 64 * SAB_K; e += 256) {
    const int ql = e / SAB_K, x = e - ql * SAB_K;
    const int ti = ti0 + ql / SM_T, tj = tj0 + ql % SM_T;
    int m = 0;
    float w = 0.f;
    if (ti < a.th && tj < a.tw) {
      const int64_t qi = (int64_t)bt * a.N + ti * a.tw + tj;
      const int cc = a.cnt[qi], cnt = cc & 0xffff, nb = cc >> 16;
      if (nb + x < cnt) { m = a.ci[qi * SAB_MAXC + nb + x]; w = a.cw[qi * SAB_MAXC + nb + x]; }
    }
    sTi[e] = m;
    sTw[e] = w;
  }

  // dense ball weights of the 64 queries -> LDS (in the output staging area, free until the loop)
  float* sB = sO;
  for (int e = tid; e < 64 * BALL; e += 256) {
    const int ql = e / BALL, s = e - ql * BALL;
    const int ti = ti0 + ql / SM_T, tj = tj0 + ql % SM_T;
    sB[e] = (ti < a.th && tj < a.tw) ? a.ballw[((int64_t)bt * a.N + ti * a.tw + tj) * BALL + s] : 0.f;
  }
  __syncthreads();
  // ---- W' A fragments in registers: wave wid owns q-tile qt = wid (16 queries) for all 64
  // elements of a chunk; K-step ks = qt + s (32 square keys: query rows 2 qt, 2 qt + 1 reach
  // key-square rows 2 qt .. 2 qt + 9 only, the other 3 steps are all zero and skipped) - 20
  // registers per wave instead of 4 tiles x 8 steps ----
  // lane: query row qt*16 + (l & 15), keys 32 ks + 8 (l >> 4) + j
  bf16x8 wf[5];
  {
    const int ql_lo = lane & 15, kg = lane >> 4;
    {
      const int qt = wid;
      const int ql = qt * 16 + ql_lo;
      const int qy = ql / SM_T, qx = ql % SM_T;                 // query offset in the tile
      const float* bw = sB + ql * BALL;
#pragma unroll
      for (int s = 0; s < 5; ++s) {
        const int ks = qt + s;
        bf16x8 f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = ks * 32 + kg * 8 + j;                   // square key: row k / 16, col k % 16
          const int di = k / SM_S - 4 - qy, dj = k % SM_S - 4 - qx;
          const int ad = (di < 0 ? -di : di) + (dj < 0 ? -dj : dj);
          float w = 0.f;
          if (ad <= 4) w = bw[ball_slot(di, dj)];
          f[j] = (bf16)w;
        }
        wf[s] = f;
      }
    }
  }

  // ---- V chunk staging: 256 rows x 64 elements, 8 x 16 B per thread ----
  uint4 stg[8];
  auto load_v = [&](int chn) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int pc = tid + 256 * i, r = pc >> 3, k = pc & 7;
      const int ki = ti0 - 4 + r / SM_S, kj = tj0 - 4 + r % SM_S;
      const bool ok = ki >= 0 && ki < a.th && kj >= 0 && kj < a.tw;
      stg[i] = ld16(ok ? reinterpret_cast<const void*>(v + (int64_t)(ki * a.tw + kj) * D + chn * SM_E + k * 8) : g_zero_sab);
    }
  };
  auto store_v = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int pc = tid + 256 * i, r = pc >> 3, k = pc & 7;
      *reinterpret_cast<uint4*>(sV + (buf * 256 + r) * SM_RV + k * 16) = stg[i];
    }
  };
  const int Hl = a.th * a.ws, Wl = a.tw * a.ws;
  bf16* out = reinterpret_cast<bf16*>(a.out) + (int64_t)bt * Hl * Wl * a.C;
  const int g16 = lane >> 4, li = lane & 15, qq = li >> 2, pp = li & 3;
  typedef short v4s __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) v4s lds_v4s;
  typedef short v8s __attribute__((ext_vector_type(8)));

  __syncthreads();                                 // sB reads done before sO is reused
  // tail rows of this thread's query / element group, fetched one chunk ahead (their L2 latency
  // was the critical path of a chunk)
  const int tq = tid >> 2, teg = (tid & 3) * 16;
  uint4 tcur[2 * SAB_K], tnext[(DB || PF) ? 2 * SAB_K : 1];
  auto load_tail = [&](int chn, uint4 (&r)[2 * SAB_K]) {
#pragma unroll
    for (int x = 0; x < SAB_K; ++x) {
      const bf16* src = v + (int64_t)sTi[tq * SAB_K + x] * D + chn * SM_E + teg;
      r[2 * x] = ld16(src);
      r[2 * x + 1] = ld16(src + 8);
    }
  };
  if (ch_beg < ch_end) {
    load_v(ch_beg);
    if constexpr (DB || PF) load_tail(ch_beg, tcur);
    store_v(0);
  }
  __syncthreads();
  for (int chn = ch_beg; chn < ch_end; ++chn) {
    const int buf = DB ? (chn - ch_beg) & 1 : 0;
    if constexpr (!DB && !PF) load_tail(chn, tcur);   // lands during this chunk's MFMAs
    if (chn + 1 < ch_end) {
      load_v(chn + 1);
      if constexpr (DB || PF) load_tail(chn + 1, tnext);
    }
    // MFMA: wave w owns queries w*16 .. +15 (q-tile w), all 64 elements of the chunk (4 groups of 16)
    f32x4 acc[4];
#pragma unroll
    for (int eg = 0; eg < 4; ++eg) acc[eg] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* vb = sV + buf * 256 * SM_RV;
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      const int ks = wid + s;
#pragma unroll
      for (int eg = 0; eg < 4; ++eg) {
        const char* va = vb + (ks * 32 + 8 * g16 + qq) * SM_RV + (eg * 16 + 4 * pp) * 2;
        const v4s b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)va);
        const v4s b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(va + 4 * SM_RV));
        const bf16x8 bfr = __builtin_bit_cast(bf16x8, (v8s)__builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7));
        acc[eg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[s], bfr, acc[eg], 0, 0, 0);
      }
    }
    // C: column (l & 15) = element eg*16 + (l & 15), rows 4 (l >> 4) + i = query wid*16 + ..
#pragma unroll
    for (int eg = 0; eg < 4; ++eg)
#pragma unroll
      for (int i = 0; i < 4; ++i) sO[(wid * 16 + g16 * 4 + i) * SM_RO + eg * 16 + li] = acc[eg][i];
    __syncthreads();                               // (!DB: every wave's V reads of this chunk are done)
    if constexpr (!DB) {
      if (chn + 1 < ch_end) store_v(0);
    }
    // tail + store: thread = (query tid / 4, 16 elements (tid % 4) * 16)
    {
      const int ql = tq, eg = teg;
      const int ti = ti0 + ql / SM_T, tj = tj0 + ql % SM_T;
      float o[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) o[e] = sO[ql * SM_RO + eg + e];
      const int e0 = chn * SM_E + eg;
#pragma unroll
      for (int x = 0; x < SAB_K; ++x) {
        const float w = sTw[ql * SAB_K + x];
        Vec<bf16> v0, v1;
        v0.from_raw(tcur[2 * x]);
        v1.from_raw(tcur[2 * x + 1]);
#pragma unroll
        for (int e = 0; e < 8; ++e) { o[e] = fmaf(w, v0.v[e], o[e]); o[8 + e] = fmaf(w, v1.v[e], o[8 + e]); }
      }
      if (ti < a.th && tj < a.tw) {
        const int sub = e0 / a.C, c0 = e0 - sub * a.C;
        const int p1 = sub / a.ws, p2 = sub - p1 * a.ws;
        bf16* dst = out + ((int64_t)(p1 * a.th + ti) * Wl + p2 * a.tw + tj) * a.C + c0;
        Vec<bf16> s0, s1;
#pragma unroll
        for (int e = 0; e < 8; ++e) { s0.v[e] = o[e]; s1.v[e] = o[8 + e]; }
        s0.store(dst);
        s1.store(dst + 8);
      }
    }
    if constexpr (DB) {
      if (chn + 1 < ch_end) {
        store_v(buf ^ 1);
#pragma unroll
        for (int x = 0; x < 2 * SAB_K; ++x) tcur[x] = tnext[x];
      }
    } else if constexpr (PF) {
      if (chn + 1 < ch_end) {
#pragma unroll
        for (int x = 0; x < 2 * SAB_K; ++x) tcur[x] = tnext[x];
      }
    }
    __syncthreads();
  }
}

bool sab_av_mfma_ok(const SabGatherArgs& a) {
  const int D = a.ws * a.ws * a.C;
  return a.ballw != nullptr && D % SM_E == 0 && a.C % 16 == 0;
}

void launch_sab_av_mfma(const SabGatherArgs& a, hipStream_t st) {
  const int D = a.ws * a.ws * a.C, nch = D / SM_E;
  const int tiles = ((a.th + SM_T - 1) / SM_T) * ((a.tw + SM_T - 1) / SM_T) * a.B * a.T;
  // split each tile's chunk range so the grid reaches ~4 blocks per CU
  const int nsplit = std::max(1, std::min(nch, (1024 + tiles - 1) / tiles));
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&sab_av_mfma_kernel<true, false>), hipFuncAttributeMaxDynamicSharedMemorySize, sm_lds<true>());
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&sab_av_mfma_kernel<false, false>), hipFuncAttributeMaxDynamicSharedMemorySize, sm_lds<false>());
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&sab_av_mfma_kernel<false, true>), hipFuncAttributeMaxDynamicSharedMemorySize, sm_lds<false>());
    attr = true;
  }
  const dim3 grid((unsigned)(tiles * nsplit));
  constexpr int l1 = sm_lds<true>(), l2 = sm_lds<false>();
  if (a.db == 1) hipLaunchKernelGGL((sab_av_mfma_kernel<true, false>), grid, dim3(256), l1, st, a, nsplit);
  else if (a.db == 2) hipLaunchKernelGGL((sab_av_mfma_kernel<false, true>), grid, dim3(256), l2, st, a, nsplit);
  else hipLaunchKernelGGL((sab_av_mfma_kernel<false, false>), grid, dim3(256), l2, st, a, nsplit);
}

template void launch_sab_score<float>(const SabScoreArgs&, hipStream_t);
template void launch_sab_score<bf16>(const SabScoreArgs&, hipStream_t);
template void launch_sab_gather<float>(const SabGatherArgs&, hipStream_t);
template void launch_sab_gather<bf16>(const SabGatherArgs&, hipStream_t);

}  // namespace turtle

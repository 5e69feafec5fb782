// Pointwise / implicit-3x3 convolution as an MFMA GEMM on pixel-major feature maps.
//
//   out[m][n] = epilogue( sum_k A[m][k] * W[n][k] )        m = pixel, n = output channel
//
// A is the K-concatenation of up to TURTLE_MAX_SRC pixel-major sources (skip concats, cached
// history frames, the multi-frame K of the Frame History Router), or the 9 shifted taps of a dense
// 3x3 convolution (Downsample / Upsample, turtle_t1_arch.py:136-154) - no im2col buffer.
// LayerNorm (turtle_t1_arch.py:83-99) costs no extra pass: its affine is folded into W at pack
// time and the per-pixel statistics are accumulated from the A tiles already staged in LDS, so
//   v = rstd_m * (acc - mu_m * s[n]) + t[n]      (s = rowsum(W*g), t = W.b)
// Epilogue: + bias, GELU, * per-channel scale (ReducedAttn beta / FeedForward gamma), + residual,
// store remap (plain, PixelShuffle(2), PixelUnshuffle(2)).
//
// Most Turtle GEMMs are HBM-bound (K = 64..640 against N = 64..2560 at 0.1-2 M pixels), so the
// kernel is organised for bytes, not FLOPs:
//   * grid: output-channel tiles vary fastest and the block id is remapped so that the tiles of
//     one pixel panel run on the same XCD - the A panel is fetched from HBM once and re-read
//     from that XCD's L2;
//   * single LDS buffer + register prefetch of the next K tile (2 barriers per K step) keeps LDS
//     at (BM+BN)*144 B so 3-4 blocks share a CU;
//   * the accumulator tile is staged through LDS and written (and the residual read) as whole
//     16-byte row chunks.
// MFMA 16x16x32 bf16 (16x16x4 f32 in parity mode); i = output channel (A operand = W rows),
// j = pixel (B operand = X rows): both operands are k-contiguous 16-byte LDS reads.
#include "common.h"
#include "kernels.h"
#include "mma.h"

namespace turtle {

// Out-of-range operand lanes load from this zero line instead of being masked after the load,
// so no instruction consumes a load result before the tile is written to LDS and all loads of
// a K step stay in flight together (guide §5, trap (c)).
__device__ __attribute__((aligned(64))) uint4 g_zero_line[4];

template <typename T, int BM, int BN>
struct GemmSmem {
  static constexpr int PIPE = (BM + BN) * ROWB;
  static constexpr int OROW = BN * (int)sizeof(T) + 16;       // staged output row bytes
  static constexpr int OUT = BM * OROW;
  static constexpr int BYTES = (PIPE > OUT ? PIPE : OUT) + 2 * BM * 4 + 4 * BN * 4;
};

template <typename T, int BM, int BN>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs g) {
  using M = Mma<T>;
  using S = GemmSmem<T, BM, BN>;
  constexpr int BK = M::BK, VEC = M::VEC, KV = BK / VEC;        // vectors per tile row
  constexpr int TM = BM / 32, TN = BN / 32;                      // 16x16 tiles per wave
  constexpr int XV = BM * KV / 256, WV = BN * KV / 256;          // vectors per thread
  __shared__ __attribute__((aligned(16))) char smem[S::BYTES];
  char* sX = smem;
  char* sW = smem + BM * ROWB;
  float* s_mu = reinterpret_cast<float*>(smem + (S::BYTES - 2 * BM * 4 - 4 * BN * 4));
  float* s_rs = s_mu + BM;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  // ---- block -> (pixel tile, channel tile); XCD-aware bijective remap of the linear id ----
  const int ntn = (g.N + BN - 1) / BN;
  const int nblk = gridDim.x;
  int lin = blockIdx.x;
  {
    const int q = nblk / 8, r = nblk % 8, x = lin % 8, y = lin / 8;
    lin = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;   // blocks of one XCD: contiguous ids
  }
  const int nt = lin % ntn;
  const int mt = lin / ntn;
  int64_t m0, mlim;
  if (g.wstride) {    // per-image weights (W_eff): a block never spans two images
    const int tpi = (g.HW + BM - 1) / BM;
    const int64_t im = mt / tpi;
    m0 = im * g.HW + (int64_t)(mt % tpi) * BM;
    mlim = min(g.M, (im + 1) * (int64_t)g.HW);
  } else {
    m0 = (int64_t)mt * BM;
    mlim = g.M;
  }
  const int n0 = nt * BN;
  const int K = g.a.Ktot;
  const int nk = (K + BK - 1) / BK;
  const int img0 = (int)(m0 / g.HW);
  const T* Wp = reinterpret_cast<const T*>(g.w) + (g.wstride ? (int64_t)(img0 / g.wdiv) * g.wstride : 0);

  // ---- per-channel epilogue vectors staged once in LDS (no per-element global loads) ----
  float* e_s = s_mu + 2 * BM;                       // [BN] each: ln_s, ln_t, bias, scale
  float* e_t = e_s + BN;
  float* e_b = e_t + BN;
  float* e_c = e_b + BN;
  if (tid < BN) {
    // unconditional loads (absent vectors read the constant zero / one lines)
    const int n = min(n0 + tid, g.N - 1);
    const float vs = (g.ln_s ? g.ln_s : g.zeros)[n], vt = (g.ln_t ? g.ln_t : g.zeros)[n];
    const float vb = (g.bias ? g.bias : g.zeros)[n], vc = (g.scale ? g.scale : g.ones)[n];
    e_s[tid] = vs; e_t[tid] = vt; e_b[tid] = vb; e_c[tid] = vc;
  }

  // ---- per-thread load geometry: rows are fixed over K, so resolve pixel coordinates once ----
  const int kv = tid % KV;
  int r_img[XV], r_p[XV], r_y[XV], r_x[XV];
  bool r_ok[XV];
#pragma unroll
  for (int i = 0; i < XV; ++i) {
    const int r = tid / KV + i * (256 / KV);
    const int64_t m = m0 + r;
    r_ok[i] = m < mlim;
    const int mm = r_ok[i] ? (int)m : (int)m0;
    r_img[i] = mm / g.HW;
    r_p[i] = mm - r_img[i] * g.HW;
    r_y[i] = g.conv3 ? r_p[i] / g.Wimg : 0;
    r_x[i] = g.conv3 ? r_p[i] - r_y[i] * g.Wimg : 0;
  }
  const int Himg = g.conv3 ? g.HW / g.Wimg : 0;
  uint4 xr[XV], wr[WV];

  auto load_tile = [&](int kt) {
    const int k = kt * BK + kv * VEC;
    const bool kin = k < K;
    // source of this k: static-index scan over the (uniform, SGPR-resident) descriptors with
    // per-lane selects - no dynamic indexing of the kernel-argument block
    const T* base = reinterpret_cast<const T*>(g.a.s[0].base);
    int64_t sld = g.a.s[0].ld;
    int soff = g.a.s[0].off, smul = g.a.s[0].img_mul, sadd = g.a.s[0].img_add, kb = 0;
    if (!g.conv3) {
      int kbj = g.a.s[0].K;
#pragma unroll
      for (int j = 1; j < TURTLE_MAX_SRC; ++j) {
        if (j < g.a.n) {
          const bool hit = k >= kbj;
          base = hit ? reinterpret_cast<const T*>(g.a.s[j].base) : base;
          sld = hit ? g.a.s[j].ld : sld;
          soff = hit ? g.a.s[j].off : soff;
          smul = hit ? g.a.s[j].img_mul : smul;
          sadd = hit ? g.a.s[j].img_add : sadd;
          kb = hit ? kbj : kb;
          kbj += g.a.s[j].K;
        }
      }
    }
    // branch-free addressing (one basic block, so the loads issue back to back): a plain source
    // is the conv3 formula with dy = dx = 0 and no border test
    const int tap = g.conv3 ? k / g.cin : 4;
    const int ci = g.conv3 ? k - (tap * g.cin) : k - kb;
    const int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
#pragma unroll
    for (int i = 0; i < XV; ++i) {
      const int y = r_y[i] + dy, x = r_x[i] + dx;
      const bool inb = !g.conv3 || (y >= 0 && y < Himg && x >= 0 && x < g.Wimg);
      const bool ok = kin && r_ok[i] && inb;
      const int64_t off = ((int64_t)(r_img[i] * smul + sadd) * g.HW + r_p[i] + dy * g.Wimg + dx) * sld + soff + ci;
      xr[i] = ld16(ok ? reinterpret_cast<const void*>(base + off) : g_zero_line);
    }
#pragma unroll
    for (int i = 0; i < WV; ++i) {
      const int n = n0 + tid / KV + i * (256 / KV);
      const bool ok = kin && n < g.N;
      wr[i] = ld16(ok ? reinterpret_cast<const void*>(Wp + (int64_t)n * g.ldw + k) : g_zero_line);
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < XV; ++i) {
      const int r = tid / KV + i * (256 / KV);
      *reinterpret_cast<uint4*>(sX + r * ROWB + kv * 16) = xr[i];
    }
#pragma unroll
    for (int i = 0; i < WV; ++i) {
      const int r = tid / KV + i * (256 / KV);
      *reinterpret_cast<uint4*>(sW + r * ROWB + kv * 16) = wr[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // LN statistics: 2 threads per pixel row, shifted sums over the staged A tiles
  const int lr = tid >> 1, lh = tid & 1;
  float ls = 0.f, lq = 0.f, lsh = 0.f;

  load_tile(0);
  for (int kt = 0; kt < nk; ++kt) {
    store_tile();
    __syncthreads();
    if (kt + 1 < nk) load_tile(kt + 1);            // in flight during the MFMAs below
    if (g.ln && lr < BM) {
      const T* row = reinterpret_cast<const T*>(sX + lr * ROWB);
      if (kt == 0) lsh = to_f(row[0]);
      const int kend = min(BK, K - kt * BK);
      for (int c = lh * VEC; c < kend; c += 2 * VEC) {
        Vec<T> v; v.load(row + c);
#pragma unroll
        for (int i = 0; i < VEC; ++i) { const float d = v.v[i] - lsh; ls += d; lq = fmaf(d, d, lq); }
      }
    }
#pragma unroll
    for (int ks = 0; ks < BK / M::KSUB; ++ks)
      mma_step<T>(sW, sX, lane, ks, acc, TM, TN, wn * (BN / 2), wm * (BM / 2));
    __syncthreads();
  }
  if (g.ln) {
    ls += __shfl_xor(ls, 1, 64);
    lq += __shfl_xor(lq, 1, 64);
    if (lh == 0 && lr < BM) {
      const float md = ls / K;
      s_mu[lr] = lsh + md;
      s_rs[lr] = rsqrtf(fmaxf(lq / K - md * md, 0.f) + 1e-5f);
    }
    __syncthreads();
  }

  // ---- epilogue phase 1: per-element math in registers, stage the tile in LDS as T ----
  const int q = lane >> 4, c16 = lane & 15;
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int r = wm * (BM / 2) + tm * 16 + c16;
    const float mu = g.ln ? s_mu[r] : 0.f, rs = g.ln ? s_rs[r] : 1.f;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int cl = wn * (BN / 2) + tn * 16 + q * 4;
      const float4 es = *reinterpret_cast<const float4*>(e_s + cl), et = *reinterpret_cast<const float4*>(e_t + cl);
      const float4 eb = *reinterpret_cast<const float4*>(e_b + cl), ec = *reinterpret_cast<const float4*>(e_c + cl);
      const float fs[4] = {es.x, es.y, es.z, es.w}, ft[4] = {et.x, et.y, et.z, et.w};
      const float fb[4] = {eb.x, eb.y, eb.z, eb.w}, fc[4] = {ec.x, ec.y, ec.z, ec.w};
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = acc[tm][tn][e];
        if (g.ln) x = rs * (x - mu * fs[e]) + ft[e];
        x += fb[e];
        if (g.gelu) x = gelu_t<T>(x);
        v[e] = x * fc[e];
      }
      if constexpr (sizeof(T) == 4) {
        *reinterpret_cast<float4*>(smem + r * S::OROW + cl * 4) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        *reinterpret_cast<bf16x4*>(smem + r * S::OROW + cl * 2) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      }
    }
  }
  __syncthreads();

  // ---- epilogue phase 2: 16-byte row chunks, residual add, store remap ----
  // every chunk's loads (staged tile + residual) are issued before any store, unconditionally
  constexpr int CV = BN / VEC;                    // chunks per row
  constexpr int NCH = BM * CV / 256;              // chunks per thread
  T* o = reinterpret_cast<T*>(g.out);
  const T* res = reinterpret_cast<const T*>(g.res);
  Vec<T> v[NCH];
  bool okc[NCH];
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int idx = tid + j * 256, r = idx / CV, cc = idx % CV;
    const int64_t m = m0 + r;
    const int nb = n0 + cc * VEC;
    okc[j] = m < mlim && nb < g.N;
    v[j].load(reinterpret_cast<const T*>(smem + r * S::OROW) + cc * VEC);
    if (res) {
      const bool full = okc[j] && nb + VEC <= g.N;
      Vec<T> rv; rv.load_pred(res + (full ? m * g.ldr + g.offr + nb : 0), full);
#pragma unroll
      for (int e = 0; e < VEC; ++e) v[j].v[e] += rv.v[e];
      if (okc[j] && !full) {
#pragma unroll
        for (int e = 0; e < VEC; ++e)
          if (nb + e < g.N) v[j].v[e] += to_f(res[m * g.ldr + g.offr + nb + e]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    if (!okc[j]) continue;
    const int idx = tid + j * 256, r = idx / CV, cc = idx % CV;
    const int64_t m = m0 + r;
    const int nb = n0 + cc * VEC;
    const bool full = nb + VEC <= g.N;
    int64_t dst;
    if (g.store_mode == STORE_NHWC) {
      dst = m * g.ldo + g.offo + nb;
    } else {
      const int mi = (int)m, img = mi / g.HW, p = mi - img * g.HW;
      const int Wi = g.Wimg, Hi = g.HW / Wi;
      const int y = p / Wi, x = p - y * Wi;
      if (g.store_mode == STORE_UNSHUFFLE) {
        const int64_t dp = ((int64_t)img * (Hi / 2) + y / 2) * (Wi / 2) + x / 2;
        const int sub = (y & 1) * 2 + (x & 1);
#pragma unroll
        for (int e = 0; e < VEC; ++e)
          if (nb + e < g.N) o[dp * g.ldo + g.offo + (nb + e) * 4 + sub] = from_f<T>(v[j].v[e]);
        continue;
      }
      // PixelShuffle: weights were permuted so output channel n' = s*Cq + c (a chunk stays in
      // one sub-pixel s)
      const int Cq = g.N / 4, sp = nb / Cq, cn = nb - sp * Cq;
      dst = (((int64_t)img * 2 * Hi + 2 * y + (sp >> 1)) * (2 * Wi) + 2 * x + (sp & 1)) * g.ldo + g.offo + cn;
    }
    if (full) {
      v[j].store(o + dst);
    } else {
#pragma unroll
      for (int e = 0; e < VEC; ++e)
        if (nb + e < g.N) o[dst + e] = from_f<T>(v[j].v[e]);
    }
  }
}

// ------------------------------------------------------------------------------------------
// Panel GEMM (bf16, plain pixel-major store, K <= 512): the block's BM x K pixel panel is loaded
// into LDS once (all loads in flight together, LayerNorm statistics taken from it), then the
// block sweeps its range of 128-channel output tiles with no further barrier: each wave owns 32
// channels, reads its W fragments straight from L2 into registers (refilled for the next tile
// right after their last use, so the fetch hides behind a whole tile of MFMAs), and its epilogue
// vectors / residual are fetched at tile start and consumed at tile end. The output tile goes
// out as 8-byte stores (4 channels per lane, 32 contiguous bytes per pixel per wave).
// Against the K-loop kernel above this trades per-K-step barriers and exposed load latency for
// one load phase per block; X is read from HBM exactly once per split.
// ------------------------------------------------------------------------------------------
__device__ __attribute__((aligned(64))) float g_one_line[16] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f,
                                                                1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
constexpr int PANEL_BN = 128;

template <int BM, int KS>
__global__ __launch_bounds__(256, 2) void gemm_panel_kernel(GemmArgs g, int nsplit) {
  constexpr int KP = KS * 32;                    // padded K (elements)
  constexpr int XROWB = KP * 2 + 16;             // LDS row bytes (16 B pad: conflict-free fragments)
  constexpr int KV = KP / 8;                     // 16-byte vectors per row
  constexpr int NV = BM * KV / 256;              // panel vectors per thread
  constexpr int MT = BM / 16, TN = 2;
  constexpr int TPR = 256 / BM;                  // threads per row for the LN statistics
  static_assert(BM * KV % 256 == 0, "panel tiling");
  __shared__ __attribute__((aligned(16))) char smem[BM * XROWB + 2 * BM * 4];
  char* sX = smem;
  float* s_mu = reinterpret_cast<float*>(smem + BM * XROWB);
  float* s_rs = s_mu + BM;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

  int lin = blockIdx.x;
  {
    const int nblk = gridDim.x, q = nblk / 8, r = nblk % 8, x = lin % 8, y = lin / 8;
    lin = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;
  }
  const int split = lin % nsplit, panel = lin / nsplit;
  int64_t m0, mlim;
  if (g.wstride) {
    const int tpi = (g.HW + BM - 1) / BM;
    const int64_t im = panel / tpi;
    m0 = im * g.HW + (int64_t)(panel % tpi) * BM;
    mlim = min(g.M, (im + 1) * (int64_t)g.HW);
  } else {
    m0 = (int64_t)panel * BM;
    mlim = g.M;
  }
  const int K = g.a.Ktot;
  const int ntiles = (g.N + PANEL_BN - 1) / PANEL_BN;
  const int nt_beg = split * ntiles / nsplit, nt_end = (split + 1) * ntiles / nsplit;
  const bf16* Wp = reinterpret_cast<const bf16*>(g.w) + (g.wstride ? (int64_t)((int)(m0 / g.HW) / g.wdiv) * g.wstride : 0);

  // ---- X panel -> LDS (source select scan per vector, zero line for padding / missing rows) ----
  {
    uint4 xv[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = tid + 256 * i, r = v / KV, k = (v - r * KV) * 8;
      const int64_t m = m0 + r;
      const bool ok = m < mlim && k < K;
      const int mm = ok ? (int)m : (int)m0;
      const int img = mm / g.HW, p = mm - img * g.HW;
      const bf16* base = reinterpret_cast<const bf16*>(g.a.s[0].base);
      int64_t sld = g.a.s[0].ld;
      int soff = g.a.s[0].off, smul = g.a.s[0].img_mul, sadd = g.a.s[0].img_add, kb = 0, kbj = g.a.s[0].K;
#pragma unroll
      for (int j = 1; j < TURTLE_MAX_SRC; ++j) {
        if (j < g.a.n) {
          const bool hit = k >= kbj;
          base = hit ? reinterpret_cast<const bf16*>(g.a.s[j].base) : base;
          sld = hit ? g.a.s[j].ld : sld;
          soff = hit ? g.a.s[j].off : soff;
          smul = hit ? g.a.s[j].img_mul : smul;
          sadd = hit ? g.a.s[j].img_add : sadd;
          kb = hit ? kbj : kb;
          kbj += g.a.s[j].K;
        }
      }
      const int64_t off = ((int64_t)(img * smul + sadd) * g.HW + p) * sld + soff + (k - kb);
      xv[i] = ld16(ok ? reinterpret_cast<const void*>(base + off) : g_zero_line);
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = tid + 256 * i, r = v / KV, kv = v - r * KV;
      *reinterpret_cast<uint4*>(sX + r * XROWB + kv * 16) = xv[i];
    }
  }

  // ---- this wave's W fragments / epilogue vectors / residual for output tile nt ----
  // Every load below is unconditional from a uniform base with a clamped 32-bit offset: rows past
  // the panel and channels past N read valid memory that is never stored, K padding meets zeros
  // in the X panel, and absent vectors / residual point at the constant zero / one lines.
  const float* ps = g.ln_s ? g.ln_s : g.zeros;
  const float* pt = g.ln_t ? g.ln_t : g.zeros;
  const float* pb = g.bias ? g.bias : g.zeros;
  const float* pc = g.scale ? g.scale : g.ones;
  const bf16* pr = g.res ? reinterpret_cast<const bf16*>(g.res) : reinterpret_cast<const bf16*>(g.zeros);
  const int ldr = g.res ? (int)g.ldr : 0, offr = g.res ? g.offr : 0;
  const int mlast = (int)(mlim - m0) - 1;               // last valid row of the panel
  bf16x8 wf[TN][KS];
  auto load_w = [&](int nt, int ks) {
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int n = min(nt * PANEL_BN + wid * 32 + tn * 16 + (lane & 15), g.N - 1);
      const int k = min(ks * 32 + (lane >> 4) * 8, K - 8);
      wf[tn][ks] = *reinterpret_cast<const bf16x8*>(Wp + n * (int)g.ldw + k);
    }
  };
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4 vs[TN], vt[TN], vb[TN], vc[TN];
  uint2 rv[MT][TN];                                     // residual, 4 bf16 per lane
  const bf16* prow = pr + (int64_t)m0 * ldr + offr;     // residual rows of this panel
  auto load_epi = [&](int nt) {
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int n = min(nt * PANEL_BN + wid * 32 + tn * 16 + (lane >> 4) * 4, g.N - 4);
      vs[tn] = *reinterpret_cast<const f4*>(ps + n);
      vt[tn] = *reinterpret_cast<const f4*>(pt + n);
      vb[tn] = *reinterpret_cast<const f4*>(pb + n);
      vc[tn] = *reinterpret_cast<const f4*>(pc + n);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int r = min(mt * 16 + (lane & 15), mlast);
        rv[mt][tn] = *reinterpret_cast<const uint2*>(prow + r * ldr + n);
      }
    }
  };
  if (nt_beg < nt_end) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) load_w(nt_beg, ks);
    load_epi(nt_beg);
  }
  __syncthreads();

  // ---- LayerNorm statistics of the panel rows (shifted sums, TPR threads per row) ----
  if (g.ln) {
    const int lr = tid / TPR, lh = tid % TPR;
    const bf16* row = reinterpret_cast<const bf16*>(sX + lr * XROWB);
    const float sh = to_f(row[0]);
    float ls = 0.f, lq = 0.f;
    for (int k = lh * 8; k < K; k += TPR * 8) {
      Vec<bf16> v; v.load(row + k);
#pragma unroll
      for (int i = 0; i < 8; ++i) { const float d = v.v[i] - sh; ls += d; lq = fmaf(d, d, lq); }
    }
#pragma unroll
    for (int o = 1; o < TPR; o <<= 1) { ls += __shfl_xor(ls, o, 64); lq += __shfl_xor(lq, o, 64); }
    if (lh == 0) {
      const float md = ls / K;
      s_mu[lr] = sh + md;
      s_rs[lr] = rsqrtf(fmaxf(lq / K - md * md, 0.f) + 1e-5f);
    }
    __syncthreads();
  }

  bf16* orow = reinterpret_cast<bf16*>(g.out) + (int64_t)m0 * g.ldo + g.offo;
  const int ldo = (int)g.ldo;
  for (int nt = nt_beg; nt < nt_end; ++nt) {
    const bool more = nt + 1 < nt_end;
    const int nw = nt * PANEL_BN + wid * 32;          // wave's first channel (wave-uniform)
    f32x4 acc[MT][TN];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) acc[mt][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (nw < g.N) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if (ks * 32 < K) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            const bf16x8 xf = *reinterpret_cast<const bf16x8*>(sX + (mt * 16 + (lane & 15)) * XROWB + ks * 64 + (lane >> 4) * 16);
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) acc[mt][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[tn][ks], xf, acc[mt][tn], 0, 0, 0);
          }
        }
        if (more) load_w(nt + 1, ks);                  // refill behind this K step's MFMAs
      }
    } else if (more) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) load_w(nt + 1, ks);
    }
    // epilogue of tile nt (vectors / residual fetched a whole tile ago; refetched after it)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      int r = mt * 16 + (lane & 15);
      asm volatile("" : "+v"(r));   // per-tile reload of the row statistics (not hoisted: VGPRs)
      const float mu = g.ln ? s_mu[r] : 0.f, rs = g.ln ? s_rs[r] : 1.f;
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int n = nw + tn * 16 + (lane >> 4) * 4;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = acc[mt][tn][e];
          if (g.ln) x = rs * (x - mu * vs[tn][e]) + vt[tn][e];
          x += vb[tn][e];
          if (g.gelu) x = gelu_bf16(x);
          const uint32_t rw = e < 2 ? rv[mt][tn].x : rv[mt][tn].y;
          v[e] = x * vc[tn][e] + __uint_as_float((e & 1) ? (rw & 0xffff0000u) : (rw << 16));
        }
        if (r <= mlast && n < g.N) {
          typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
          *reinterpret_cast<bf16x4*>(orow + r * ldo + n) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
        }
      }
    }
    if (more) load_epi(nt + 1);
  }
}

template <int BM, int KS>
static void launch_panel(const GemmArgs& g, hipStream_t st) {
  const int64_t np = g.wstride ? (g.M / g.HW) * ((g.HW + BM - 1) / BM) : (g.M + BM - 1) / BM;
  const int ntiles = (g.N + PANEL_BN - 1) / PANEL_BN;
  // split the channel tiles so the grid reaches ~4 blocks per CU
  int nsplit = (int)std::min<int64_t>(ntiles, std::max<int64_t>(1, (1024 + np - 1) / np));
  hipLaunchKernelGGL((gemm_panel_kernel<BM, KS>), dim3((unsigned)(np * nsplit)), dim3(256), 0, st, g, nsplit);
}

// the panel kernel applies to bf16 plain stores with K <= 512 (one LDS panel)
static bool panel_ok(const GemmArgs& g) {
  if (g.a.cb_px) return false;                   // channel-blocked operand: 2-D tiled kernel only
  // 32-bit in-panel offsets: rows x leading dimension must stay below 2^31 elements
  const int64_t big = (int64_t)1 << 30;
  return g.allow_panel && !g.conv3 && g.store_mode == STORE_NHWC && g.N % 16 == 0 && g.a.Ktot % 8 == 0 && g.a.Ktot >= 8 &&
         g.a.Ktot <= 512 && g.ldw % 8 == 0 && (g.res == nullptr || (g.ldr % 4 == 0 && g.offr % 4 == 0)) &&
         g.ldo % 4 == 0 && g.offo % 4 == 0 && (int64_t)g.N * g.ldw < big && 128 * g.ldo < big && 128 * g.ldr < big &&
         g.zeros && g.ones && g.N <= 8192;
}
static void launch_panel_any(const GemmArgs& g, hipStream_t st) {
  const int K = g.a.Ktot;
  if (K <= 64) launch_panel<128, 2>(g, st);
  else if (K <= 128) launch_panel<128, 4>(g, st);
  else if (K <= 192) launch_panel<128, 6>(g, st);
  else if (K <= 256) launch_panel<128, 8>(g, st);
  else if (K <= 384) launch_panel<64, 12>(g, st);
  else launch_panel<64, 16>(g, st);
}

template <typename T, int BM, int BN>
static void launch_cfg(const GemmArgs& g, hipStream_t st) {
  const int64_t mt = g.wstride ? (g.M / g.HW) * ((g.HW + BM - 1) / BM) : (g.M + BM - 1) / BM;
  const int64_t nblk = mt * ((g.N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_kernel<T, BM, BN>), dim3((unsigned)nblk), dim3(256), 0, st, g);
}

template <typename T>
void launch_gemm(const GemmArgs& g, hipStream_t st) {
  if (g.store_mode == STORE_CB16) {                // produced only for the pn / g8 kernels (turtle.cpp)
    if constexpr (sizeof(T) == 2)
      if (gemm8_ok(g)) { launch_gemm8(g, st); return; }
    if (sizeof(T) != 2 || !gemm_pn_ok(g)) kernel_arg_error("channel-blocked GEMM store needs the bf16 pn or g8 kernel");
    launch_gemm_pn(g, st);
    return;
  }
  if (g.a.cb_px) {                                 // channel-blocked operand (tilepd.hip): 2-D tiled kernel only
    if (sizeof(T) != 2 || !gemm_kt_ok(g)) kernel_arg_error("channel-blocked GEMM operand needs the bf16 2-D tiled kernel");
    launch_gemm_kt(g, st);
    return;
  }
  if constexpr (sizeof(T) == 2) {
    if (gemm8_ok(g)) { launch_gemm8(g, st); return; }   // allow_g8: the caller's per-shape choice (turtle.cpp)
    // measured per shape class (tools/kbench, MI355X): the 2-D tiled kernel for the resampling 3x3
    // convolutions and K >= 640 (incl. the five-source W_eff GEMM), the A-resident kernel for the
    // K = 256 residual projections, else the persistent panel kernel
    // small frames (fewer than 32768 pixels: < 256 pn panels, i.e. a partly idle chip) also go to
    // the 2-D tiled kernel, whose channel tiles multiply the grid
    const int K = g.a.Ktot;
    if (((g.conv3 && g.N >= 256) || (!g.conv3 && K >= 640) || (!g.ln && K == 512 && g.N >= 512) || g.M < (g.kt_max_px ? g.kt_max_px : 32768)) &&
        gemm_kt_ok(g)) {
      launch_gemm_kt(g, st);
      return;
    }
    if (K == 256 && g.res && gemm_ar_ok(g)) { launch_gemm_ar(g, st); return; }
    if (gemm_pn_ok(g)) { launch_gemm_pn(g, st); return; }
    if (gemm_lds_ok(g)) { launch_gemm_lds(g, st); return; }
    if (panel_ok(g)) { launch_panel_any(g, st); return; }
  }
  if constexpr (sizeof(T) == 4)
    if (gemm_f32_preferred(g)) { launch_gemm_f32(g, st); return; }
  // BN = 128 when it tiles N exactly (or N is large), else 64 (N = 64, 192, 320, tiny widths)
  const bool wide = g.N >= 128 && (g.N % 128 == 0 || g.N > 1024);
  if (wide) launch_cfg<T, 128, 128>(g, st);
  else launch_cfg<T, 128, 64>(g, st);
}

template void launch_gemm<float>(const GemmArgs&, hipStream_t);
template void launch_gemm<bf16>(const GemmArgs&, hipStream_t);

}  // namespace turtle

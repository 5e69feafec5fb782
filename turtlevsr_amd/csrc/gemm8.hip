// bf16 projection GEMM, 256 x 256 x 64 tiles, four-phase staggered LDS-DMA schedule ("g8" kernel):
// the large plain / LayerNorm-folded 1x1 projections (latent level, and wherever it measures faster
// than the resident-panel kernels).
//
//   out[m][n] = epilogue( sum_k A[m][k] * W[n][k] )        m = pixel, n = output channel
//
// Contract: GemmArgs with K-concatenated sources (img_mul 1 / img_add 0, every source but the last
// a multiple of 64 wide), optional LayerNorm folded into the epilogue (statistics accumulated from
// the A fragments while they are in registers), bias / GELU / scale / residual, NHWC or
// channel-blocked (STORE_CB16, the GatedFFN hidden map for dwgemm.hip) store, per-image weight sets
// (W_eff).
//
// Structure (MI355X, one 512-thread block per CU, 128 KB of LDS):
//   * 8 waves as 2 (pixel halves of 128) x 4 (channel quarters of 64); a wave's 128 x 64 output is
//     four quadrants of 64 px x 32 ch, one quadrant (16 MFMA 16x16x32, K = 64) per PHASE, four
//     phases per K tile:  P1 reads X-a + W-a, P2 W-b, P3 X-b, P4 nothing (W-a kept in registers);
//   * the K tile lives in LDS as four 16 KB UNITS in the order they are first read: X-a (pixel rows
//     0-63 of each half), W-a (channels 0-31 of each quarter), W-b, X-b; two buffers (even / odd
//     K tiles). Every phase issues ONE unit (two global_load_lds per thread), four phases ahead:
//         P1: W-b(t+1)   P2: X-b(t+1)   P3: X-a(t+2)   P4: W-a(t+2)
//     and before it waits vmcnt(6), which retires the unit issued four phases earlier - the one
//     the NEXT phase reads (RAW: wait one phase before the read). Each unit is overwritten >= 2
//     phases after its last read (WAR across the stagger below); past the last K tile the issue
//     reads a zero line, so the count never changes;
//   * the two wave groups (pixel halves) run one barrier apart (T3+T4 of the HIP guide): while one
//     group issues its fragment reads and DMA the other runs its 16 MFMAs, so each SIMD (one wave
//     of each group) alternates between them;
//   * LDS rows are 128 B (64 k), chunk c of row r stored at c ^ ((r >> 1) & 7): conflict-free
//     ds_read_b128 for 16 consecutive rows on gfx950's lane groups; the swizzle is applied on the
//     DMA's per-lane source address (the LDS side of global_load_lds is lane-linear);
//   * weight rows are placed in LDS in pn's permuted order (MFMA row 4g+e of sub-tile s <- channel
//     8g+4s+e of a 32-channel group) by choosing each DMA lane's source row, so a lane's
//     accumulators hold 8 CONSECUTIVE channels of one pixel: 16-byte residual loads and stores.
#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace turtle {

__device__ __attribute__((aligned(64))) uint4 g_zero_g8[4];

namespace {

constexpr int G8_UNIT = 16384, G8_BUF = 4 * G8_UNIT;
constexpr int G8_BYTES = 2 * G8_BUF + 2 * 256 * 4;     // two buffers + LN statistics
enum { U_XA = 0, U_WA = 1, U_WB = 2, U_XB = 3 };

// 64 lanes x 16 B -> LDS at M0 (M0 is compiler-reserved: restored). Inline asm so hipcc does not
// treat it as a pending LDS write and drain the ring (vmcnt(0)) before every ds_read.
TURTLE_DEV void g8_dma16(const void* g, uint32_t lds_wave_base) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(lds_wave_base) : "memory");
}
template <int N>
TURTLE_DEV void g8_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}
// MFMA row -> channel within a wave's 64-channel quarter (two 32-channel groups of two sub-tiles)
TURTLE_DEV int g8_perm(int r) { return 32 * (r >> 5) + 8 * ((r >> 2) & 3) + 4 * ((r >> 4) & 1) + (r & 3); }

}  // namespace

// DBG (tools/g8bench ablation builds only, 0 in the library): 1 no MFMA, 2 no LDS-DMA, 4 no fragment
// reads, 8 no barriers in the K loop, 16 no epilogue stores
template <bool LN, int DBG = 0>
__global__ __launch_bounds__(512, 1) void gemm8_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_mu = reinterpret_cast<float*>(smem + 2 * G8_BUF);
  float* s_rs = s_mu + 256;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int fr = lane & 15, fq = lane >> 4;

  // ---- tile: the channel tiles of one pixel panel are consecutive ids on one XCD ----
  const int ntn = (g.N + 255) / 256;
  int lin = blockIdx.x;
  {
    const int nblk = gridDim.x, q = nblk / 8, r = nblk % 8, x = lin % 8, y = lin / 8;
    lin = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;
  }
  const int nt = lin % ntn, mt = lin / ntn;
  int64_t m0, mlim;
  if (g.wstride) {
    const int tpi = (g.HW + 255) / 256;
    const int64_t im = mt / tpi;
    m0 = im * g.HW + (int64_t)(mt % tpi) * 256;
    mlim = min(g.M, (im + 1) * (int64_t)g.HW);
  } else {
    m0 = (int64_t)mt * 256;
    mlim = g.M;
  }
  const int n0 = nt * 256;
  const int K = g.a.Ktot, nk = (K + 63) / 64;
  const bf16* Wp = reinterpret_cast<const bf16*>(g.w) + (g.wstride ? (int64_t)(m0 / g.HW / g.wdiv) * g.wstride : 0);

  // ---- DMA geometry: instruction i (0, 1) of wave w fills unit rows (8 i + w) 8 + lane / 8, 16-byte
  // position lane % 8, which holds source chunk kc / 8 = (lane % 8) ^ swz(row) ----
  const int kc = (((lane & 7) ^ (((wid & 1) << 2) | (lane >> 4))) & 7) * 8;
  int xm[4];                        // pixel rows: X-a i0, i1, X-b i0, i1 (clamped into the tile's valid range)
  int wrow[4];                      // weight rows: W-a i0, i1, W-b i0, i1
  int xyp[4];                       // implicit 3x3: (y << 16) | x of those pixels in their image
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int io = (i * 8 + wid) * 8 + (lane >> 3);
    const int pr = (io >> 6) * 128 + (io & 63);
    const int64_t ma = m0 + pr, mb = m0 + pr + 64;
    xm[i] = (int)(ma < mlim ? ma : m0);
    xm[2 + i] = (int)(mb < mlim ? mb : m0);
    if (g.conv3) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int mm = xm[2 * h + i], p = mm % g.HW, y = p / g.Wimg;
        xyp[2 * h + i] = (y << 16) | (p - y * g.Wimg);
      }
    } else {
      xyp[i] = xyp[2 + i] = 0;
    }
    const int wa = n0 + (io >> 5) * 64 + g8_perm(io & 31), wb = n0 + (io >> 5) * 64 + g8_perm(32 + (io & 31));
    wrow[i] = min(wa, g.N - 1);
    wrow[2 + i] = min(wb, g.N - 1);
  }
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  // unit u of K tile t (zero line past the last tile / beyond K)
  auto issue = [&](int t, int u) __attribute__((always_inline)) {
    const int k0 = t * 64;
    const uint32_t dst = lds_base + (t & 1) * G8_BUF + u * G8_UNIT + wid * 1024;
    const bool live = t < nk && k0 + kc < K;
    if (u == U_XA || u == U_XB) {
      // the K tile's source (K tiles never straddle two sources)
      const bf16* base = reinterpret_cast<const bf16*>(g.a.s[0].base);
      int64_t sld = g.a.s[0].ld;
      int soff = g.a.s[0].off, kb = 0, kbj = g.a.s[0].K;
#pragma unroll
      for (int j = 1; j < TURTLE_MAX_SRC; ++j) {
        const bool hit = j < g.a.n && k0 >= kbj;
        base = hit ? reinterpret_cast<const bf16*>(g.a.s[j].base) : base;
        sld = hit ? g.a.s[j].ld : sld;
        soff = hit ? g.a.s[j].off : soff;
        kb = hit ? kbj : kb;
        kbj += j < g.a.n ? g.a.s[j].K : 0;
      }
      const int o = u == U_XA ? 0 : 2;
      if (g.conv3) {                              // tap-major K: tap = k0 / cin, its 64 channels
        const int tap = k0 / g.cin, dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
        const bf16* b2 = base + g.a.s[0].off + (k0 - tap * g.cin) + kc;
        const int Himg = g.HW / g.Wimg;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int y = (xyp[o + i] >> 16) + dy, x = (xyp[o + i] & 0xffff) + dx;
          const bool ok = live && y >= 0 && y < Himg && x >= 0 && x < g.Wimg;
          uint64_t pa = reinterpret_cast<uint64_t>(b2 + (int64_t)(xm[o + i] + dy * g.Wimg + dx) * sld);
          asm volatile("" : "+v"(pa));
          if constexpr (!(DBG & 2)) g8_dma16(ok ? reinterpret_cast<const void*>(pa) : reinterpret_cast<const void*>(g_zero_g8), dst + i * 8192);
        }
      } else {
        const bf16* b2 = base + soff + (k0 - kb) + kc;
#pragma unroll
        for (int i = 0; i < 2; ++i)
          if constexpr (!(DBG & 2)) g8_dma16(live ? reinterpret_cast<const void*>(b2 + (int64_t)xm[o + i] * sld) : reinterpret_cast<const void*>(g_zero_g8),
                   dst + i * 8192);
      }
    } else {
      const int o = u == U_WA ? 0 : 2;
#pragma unroll
      for (int i = 0; i < 2; ++i)
        if constexpr (!(DBG & 2)) g8_dma16(live ? reinterpret_cast<const void*>(Wp + (int64_t)wrow[o + i] * g.ldw + k0 + kc) : reinterpret_cast<const void*>(g_zero_g8),
                 dst + i * 8192);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment reads: 16 consecutive unit rows from `row0`, K step ks; swizzle depends on fr only
  const int sw = (fr >> 1) & 7;
  const int loff0 = fr * 128 + ((fq ^ sw) << 4), loff1 = fr * 128 + (((fq ^ sw) ^ 4) << 4);
  bf16x8 zfrag;                                   // DBG & 4: a loop-invariant stand-in fragment
#pragma unroll
  for (int e = 0; e < 8; ++e) zfrag[e] = (bf16)(float)(lane + e);
  auto frag = [&](const char* unit, int row0, int ks) __attribute__((always_inline)) {
    if constexpr ((DBG & 4) != 0) return zfrag;
    return *reinterpret_cast<const bf16x8*>(unit + row0 * 128 + (ks ? loff1 : loff0));
  };

  // LN statistics: wave wn sums pixel tiles 2 (wn & 1) + {0, 1} of X-a (wn < 2) or X-b (wn >= 2)
  float lsum[2] = {0.f, 0.f}, lsq[2] = {0.f, 0.f};
  auto stats2 = [&](const bf16x8 (&xa)[2], const bf16x8 (&xb)[2]) __attribute__((always_inline)) {
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    const bf16x2 one2 = __builtin_bit_cast(bf16x2, 0x3F803F80u);
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        // (uint4 members: element access on a bit-cast u32x4 vector here made hipcc read the first
        // dword four times)
        const uint4 q = __builtin_bit_cast(uint4, tt ? xb[ks] : xa[ks]);
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bf16x2 v2 = __builtin_bit_cast(bf16x2, w[e]);
          lsum[tt] = __builtin_amdgcn_fdot2_f32_bf16(v2, one2, lsum[tt], false);
          lsq[tt] = __builtin_amdgcn_fdot2_f32_bf16(v2, v2, lsq[tt], false);
        }
      }
  };
  // (wave-uniform branch on wn & 1: no per-register selects)
  auto stats = [&](const bf16x8 (&xf)[4][2]) __attribute__((always_inline)) {
    if (wn & 1) stats2(xf[2], xf[3]);
    else stats2(xf[0], xf[1]);
  };

  // ---- prologue: X-a, W-a, W-b, X-b of tile 0, X-a, W-a of tile 1; the first two have landed ----
  issue(0, U_XA); issue(0, U_WA); issue(0, U_WB); issue(0, U_XB); issue(1, U_XA); issue(1, U_WA);
  g8_vm<8>();
  __builtin_amdgcn_s_barrier();
  if (wm == 1) __builtin_amdgcn_s_barrier();      // stagger: group 1 runs one barrier behind

#define G8_MFMA_BEGIN                                   \
  __builtin_amdgcn_sched_barrier(0);                    \
  if constexpr (!(DBG & 8)) __builtin_amdgcn_s_barrier(); \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");    \
  __builtin_amdgcn_sched_barrier(0);                    \
  __builtin_amdgcn_s_setprio(1);
#define G8_MFMA_END                                     \
  __builtin_amdgcn_s_setprio(0);                        \
  __builtin_amdgcn_sched_barrier(0);                    \
  if constexpr (!(DBG & 8)) __builtin_amdgcn_s_barrier(); \
  asm volatile("" ::: "memory");                        \
  __builtin_amdgcn_sched_barrier(0);

  bf16x8 xf[4][2], wa[2][2], wb[2][2];
  for (int t = 0; t < nk; ++t) {
    const char* ub = smem + (t & 1) * G8_BUF;
    // P1: X-a, W-a -> pixel tiles 0-3 x channel tiles 0-1
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) xf[i][ks] = frag(ub + U_XA * G8_UNIT, wm * 64 + 16 * i, ks);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) wa[j][ks] = frag(ub + U_WA * G8_UNIT, wn * 32 + 16 * j, ks);
    g8_vm<6>();
    issue(t + 1, U_WB);
    G8_MFMA_BEGIN
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) if constexpr (!(DBG & 1)) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[j][ks], xf[i][ks], acc[i][j], 0, 0, 0);
    if (LN && !(DBG & 64) && wn < 2) stats(xf);
    G8_MFMA_END
    // P2: W-b -> pixel tiles 0-3 x channel tiles 2-3
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) wb[j][ks] = frag(ub + U_WB * G8_UNIT, wn * 32 + 16 * j, ks);
    g8_vm<6>();
    issue(t + 1, U_XB);
    G8_MFMA_BEGIN
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) if constexpr (!(DBG & 1)) acc[i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[j][ks], xf[i][ks], acc[i][2 + j], 0, 0, 0);
    G8_MFMA_END
    // P3: X-b -> pixel tiles 4-7 x channel tiles 2-3
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) xf[i][ks] = frag(ub + U_XB * G8_UNIT, wm * 64 + 16 * i, ks);
    g8_vm<6>();
    issue(t + 2, U_XA);
    G8_MFMA_BEGIN
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) if constexpr (!(DBG & 1)) acc[4 + i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[j][ks], xf[i][ks], acc[4 + i][2 + j], 0, 0, 0);
    if (LN && !(DBG & 64) && wn >= 2) stats(xf);
    G8_MFMA_END
    // P4: (no reads) -> pixel tiles 4-7 x channel tiles 0-1
    g8_vm<6>();
    issue(t + 2, U_WA);
    G8_MFMA_BEGIN
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) if constexpr (!(DBG & 1)) acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[j][ks], xf[i][ks], acc[4 + i][j], 0, 0, 0);
    G8_MFMA_END
  }
#undef G8_MFMA_BEGIN
#undef G8_MFMA_END
  if (wm == 0) __builtin_amdgcn_s_barrier();      // re-align the groups
  g8_vm<0>();                                     // zero-line DMA of the tiles past the end

  if (LN) {
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      lsum[tt] += __shfl_xor(lsum[tt], 16, 64); lsum[tt] += __shfl_xor(lsum[tt], 32, 64);
      lsq[tt] += __shfl_xor(lsq[tt], 16, 64); lsq[tt] += __shfl_xor(lsq[tt], 32, 64);
      if (fq == 0) {
        const int r = wm * 128 + (wn >= 2 ? 64 : 0) + 16 * (2 * (wn & 1) + tt) + fr;
        const float mu = lsum[tt] / K;
        s_mu[r] = mu;
        s_rs[r] = rsqrtf(fmaxf(lsq[tt] / K - mu * mu, 0.f) + 1e-5f);
      }
    }
    __syncthreads();
  }

  if constexpr ((DBG & 32) != 0) {                 // no epilogue: one sink store keeps the MFMAs alive
    float sum = 0.f;
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) sum += acc[a][b][0];
    if (sum == 1.2345f) reinterpret_cast<float*>(g.out)[tid] = sum;
    return;
  }
  // ---- epilogue: lane holds channels c .. c+7 (c = n0 + 64 wn + 32 jj + 8 fq) of pixel row
  // m0 + 128 wm + 16 i + fr ----
  bf16* o = reinterpret_cast<bf16*>(g.out);
  const bf16* res = reinterpret_cast<const bf16*>(g.res);
  const float* vs = g.ln_s ? g.ln_s : g.zeros;
  const float* vt = g.ln_t ? g.ln_t : g.zeros;
  const float* vb = g.bias ? g.bias : g.zeros;
  const float* vc = g.scale ? g.scale : g.ones;
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int c = n0 + wn * 64 + 32 * jj + 8 * fq;
    if (c >= g.N) continue;                       // N % 8 == 0: a group of 8 is all in or all out
    float fs[8], ft[8], fb[8], fc[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(vs + c + 4 * h), b = *reinterpret_cast<const f32x4*>(vt + c + 4 * h);
      const f32x4 d = *reinterpret_cast<const f32x4*>(vb + c + 4 * h), e = *reinterpret_cast<const f32x4*>(vc + c + 4 * h);
#pragma unroll
      for (int i = 0; i < 4; ++i) { fs[4 * h + i] = a[i]; ft[4 * h + i] = b[i]; fb[4 * h + i] = d[i]; fc[4 * h + i] = e[i]; }
    }
    uint4 rv[8];
    if (res) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int64_t m = m0 + wm * 128 + 16 * i + fr;
        rv[i] = ld16(res + (m < mlim ? m : m0) * g.ldr + g.offr + c);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = wm * 128 + 16 * i + fr;
      const int64_t m = m0 + r;
      if (m >= mlim) continue;
      const float mu = LN ? s_mu[r] : 0.f, rs = LN ? s_rs[r] : 1.f;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float x = acc[i][2 * jj + (e >> 2)][e & 3];
        if (LN) x = rs * (x - mu * fs[e]) + ft[e];
        x += fb[e];
        if (g.gelu) x = gelu_bf16(x);
        v[e] = x * fc[e];
      }
      if (res) {
        const uint32_t rw[4] = {rv[i].x, rv[i].y, rv[i].z, rv[i].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[2 * e] += __uint_as_float(rw[e] << 16);
          v[2 * e + 1] += __uint_as_float(rw[e] & 0xffff0000u);
        }
      }
      bf16x8 ov;
#pragma unroll
      for (int e = 0; e < 8; ++e) ov[e] = (bf16)v[e];
      // NHWC, channel-blocked (STORE_CB16: channel k of pixel m at ((k / 16) cb_px + m) 16 + k % 16),
      // or PixelShuffle / PixelUnshuffle (the 3x3 resampling convolutions, as gemm5.hip)
      int64_t dst;
      if (g.store_mode == STORE_NHWC) {
        dst = m * g.ldo + g.offo + c;
      } else if (g.store_mode == STORE_CB16) {
        dst = (((int64_t)(c >> 4) * g.cb_px + m) << 4) + (c & 15);
      } else {
        const int mi = (int)m, img = mi / g.HW, p = mi - img * g.HW;
        const int Wi = g.Wimg, Hi = g.HW / Wi;
        const int y = p / Wi, x = p - y * Wi;
        if (g.store_mode == STORE_UNSHUFFLE) {
          const int64_t dp = ((int64_t)img * (Hi / 2) + y / 2) * (Wi / 2) + x / 2;
          const int sub = (y & 1) * 2 + (x & 1);
#pragma unroll
          for (int e = 0; e < 8; ++e) o[dp * g.ldo + g.offo + (c + e) * 4 + sub] = ov[e];
          continue;
        }
        const int Cq = g.N / 4, sp = c / Cq, cn = c - sp * Cq;
        dst = (((int64_t)img * 2 * Hi + 2 * y + (sp >> 1)) * (2 * Wi) + 2 * x + (sp & 1)) * g.ldo + g.offo + cn;
      }
      if constexpr (!(DBG & 16)) *reinterpret_cast<bf16x8*>(o + dst) = ov;
    }
  }
}

// ---- persistent form ("g8p"): one block per CU walks tiles lin, lin + G, .. as ONE stream of K
// tiles (step s = tile-local index x nk + t), so the four-phase schedule never drains: the units of
// the next tile's first two K tiles are in flight during the current tile's last phases and its
// epilogue. Per tile, the epilogue's per-channel vectors (LN s / t, bias, scale; 4 x 1 KB) go to an
// LDS slot by LDS-DMA at phase 1 of the previous tile's last K tile (every wave issues one: waves w
// and w + 4 copy the same vector), so the epilogue issues no global loads but the residual's. The
// LN statistics are written to LDS at the tile's last K tile (phase 1 / 3) and read in its
// epilogue after the phase-4 barrier (each group reads only its own pixel half). Needs nk >= 2
// (a slot / statistics row is rewritten one K tile after its last read at the earliest).
constexpr int G8P_VEC = 2 * G8_BUF + 2 * 256 * 4;        // 2 slots x [4 vectors][256] fp32
constexpr int G8P_BYTES = G8P_VEC + 2 * 4 * 256 * 4;

template <bool LN, bool RES>
__global__ __launch_bounds__(512, 1) void gemm8p_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_mu = reinterpret_cast<float*>(smem + 2 * G8_BUF);
  float* s_rs = s_mu + 256;
  const float* s_vec = reinterpret_cast<const float*>(smem + G8P_VEC);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int fr = lane & 15, fq = lane >> 4;

  const int ntn = (g.N + 255) / 256;
  const int tpi = g.wstride ? (g.HW + 255) / 256 : 0;
  const int ntm = g.wstride ? (int)(g.M / g.HW) * tpi : (int)((g.M + 255) / 256);
  const int ntiles = ntm * ntn;
  const int G = gridDim.x;
  int lin = blockIdx.x;
  {
    const int q = G / 8, r = G % 8, x = lin % 8, y = lin / 8;
    lin = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;
  }
  const int K = g.a.Ktot, nk = (K + 63) / 64;
  const int ntl = (ntiles - lin + G - 1) / G;      // tiles of this block (G <= ntiles)
  const int nsteps = ntl * nk;
  // tile-local index -> geometry (wave-uniform; computed once per tile, the divisions are not cheap)
  struct Geo { int64_t m0, mlim; int n0; int64_t woff; };
  auto geo = [&](int tl) __attribute__((always_inline)) {
    Geo r;
    const int tile = lin + min(tl, ntl - 1) * G;
    const int nt = tile % ntn, mt = tile / ntn;
    if (g.wstride) {
      const int im = mt / tpi;
      r.m0 = (int64_t)im * g.HW + (int64_t)(mt - im * tpi) * 256;
      r.mlim = min(g.M, (int64_t)(im + 1) * g.HW);
      r.woff = (int64_t)(im / g.wdiv) * g.wstride;
    } else {
      r.m0 = (int64_t)mt * 256;
      r.mlim = g.M;
      r.woff = 0;
    }
    r.n0 = nt * 256;
    return r;
  };

  // DMA geometry (as gemm8_kernel): unit row of instruction i, source chunk, W channel offsets
  const int kc = (((lane & 7) ^ (((wid & 1) << 2) | (lane >> 4))) & 7) * 8;
  // unit row of DMA instruction i: (8 i + wid) 8 + lane / 8 (recomputed per issue: registers)
  auto unit_row = [&](int i) __attribute__((always_inline)) { return (i * 8 + wid) * 8 + (lane >> 3); };
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const bf16* W0 = reinterpret_cast<const bf16*>(g.w);

  // unit u of step (tl, t) of tile geometry q; zero line past the block's last step / beyond K
  auto issue = [&](int tl, int t, const Geo& q, int u) __attribute__((always_inline)) {
    const int k0 = t * 64;
    const uint32_t dst = lds_base + ((tl * nk + t) & 1) * G8_BUF + u * G8_UNIT + wid * 1024;
    const bool live = tl < ntl && k0 + kc < K;
    const int64_t m0 = q.m0, mlim = q.mlim;
    const int n0 = q.n0;
    if (u == U_XA || u == U_XB) {
      const bf16* base = reinterpret_cast<const bf16*>(g.a.s[0].base);
      int64_t sld = g.a.s[0].ld;
      int soff = g.a.s[0].off, kb = 0, kbj = g.a.s[0].K;
#pragma unroll
      for (int j = 1; j < TURTLE_MAX_SRC; ++j) {
        const bool hit = j < g.a.n && k0 >= kbj;
        base = hit ? reinterpret_cast<const bf16*>(g.a.s[j].base) : base;
        sld = hit ? g.a.s[j].ld : sld;
        soff = hit ? g.a.s[j].off : soff;
        kb = hit ? kbj : kb;
        kbj += j < g.a.n ? g.a.s[j].K : 0;
      }
      const bf16* b2 = base + soff + (k0 - kb) + kc;
      const int xo = u == U_XA ? 0 : 64;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int io = unit_row(i);
        const int64_t m = m0 + (io >> 6) * 128 + (io & 63) + xo;
        const int64_t mc = m < mlim ? m : m0;
        uint64_t pa = reinterpret_cast<uint64_t>(b2 + mc * sld);
        asm volatile("" : "+v"(pa));               // computed for every lane, then selected (no branch)
        g8_dma16(live ? reinterpret_cast<const void*>(pa) : reinterpret_cast<const void*>(g_zero_g8), dst + i * 8192);
      }
    } else {
      const bf16* Wp = W0 + q.woff;
      const int wo = u == U_WA ? 0 : 32;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int io = unit_row(i);
        const int n = n0 + (io >> 5) * 64 + g8_perm(wo + (io & 31));
        uint64_t pa = reinterpret_cast<uint64_t>(Wp + (int64_t)min(n, g.N - 1) * g.ldw + k0 + kc);
        asm volatile("" : "+v"(pa));
        g8_dma16(live ? reinterpret_cast<const void*>(pa) : reinterpret_cast<const void*>(g_zero_g8), dst + i * 8192);
      }
    }
  };
  // per-channel vectors of tile tl -> slot tl & 1: wave w copies vector w & 3 (LN s, LN t, bias,
  // scale; absent ones from the zero / one lines), lane l channels n0 + 4 l .. (clamped into N)
  auto issue_vec = [&](int tl, const Geo& q) __attribute__((always_inline)) {
    const int n0 = q.n0;
    const int v = wid & 3;
    const float* src = v == 0 ? g.ln_s : v == 1 ? g.ln_t : v == 2 ? g.bias : g.scale;
    const float* dflt = v == 3 ? g.ones : g.zeros;
    const float* p = src ? src + min(n0 + 4 * lane, g.N - 4) : dflt + 4 * lane;
    g8_dma16(p, lds_base + G8P_VEC + (tl & 1) * 4096 + v * 1024);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int sw = (fr >> 1) & 7;
  const int loff0 = fr * 128 + ((fq ^ sw) << 4), loff1 = fr * 128 + (((fq ^ sw) ^ 4) << 4);
  auto frag = [&](const char* unit, int row0, int ks) __attribute__((always_inline)) {
    return *reinterpret_cast<const bf16x8*>(unit + row0 * 128 + (ks ? loff1 : loff0));
  };

  float lsum[2] = {0.f, 0.f}, lsq[2] = {0.f, 0.f};
  auto stats2 = [&](const bf16x8 (&xa)[2], const bf16x8 (&xb)[2]) __attribute__((always_inline)) {
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    const bf16x2 one2 = __builtin_bit_cast(bf16x2, 0x3F803F80u);
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        // (uint4 members: element access on a bit-cast u32x4 vector here made hipcc read the first
        // dword four times)
        const uint4 q = __builtin_bit_cast(uint4, tt ? xb[ks] : xa[ks]);
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bf16x2 v2 = __builtin_bit_cast(bf16x2, w[e]);
          lsum[tt] = __builtin_amdgcn_fdot2_f32_bf16(v2, one2, lsum[tt], false);
          lsq[tt] = __builtin_amdgcn_fdot2_f32_bf16(v2, v2, lsq[tt], false);
        }
      }
  };
  auto stats = [&](const bf16x8 (&xf)[4][2]) __attribute__((always_inline)) {
    if (wn & 1) stats2(xf[2], xf[3]);
    else stats2(xf[0], xf[1]);
  };
  // the tile's statistics of this wave's two pixel tiles -> LDS (last K tile), sums reset
  auto stats_out = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      float a = lsum[tt], q = lsq[tt];
      a += __shfl_xor(a, 16, 64); a += __shfl_xor(a, 32, 64);
      q += __shfl_xor(q, 16, 64); q += __shfl_xor(q, 32, 64);
      if (fq == 0) {
        int fro = fr;                              // opaque: keeps hipcc from hoisting (and spilling)
        asm volatile("" : "+v"(fro));              // the LDS addresses out of the tile loop
        const int r = wm * 128 + (wn >= 2 ? 64 : 0) + 16 * (2 * (wn & 1) + tt) + fro;
        const float mu = a / K;
        s_mu[r] = mu;
        s_rs[r] = rsqrtf(fmaxf(q / K - mu * mu, 0.f) + 1e-5f);
      }
      lsum[tt] = 0.f; lsq[tt] = 0.f;
    }
  };

  // ---- epilogue of tile tl (registers + LDS only, but the residual) ----
  auto epilogue = [&](int tl, const Geo& q) __attribute__((always_inline)) {
    const int64_t m0 = q.m0, mlim = q.mlim;
    const int n0 = q.n0;
    int fro = fr, fqo = fq;                        // opaque lane indices (see stats_out)
    asm volatile("" : "+v"(fro), "+v"(fqo));
    const float* sv = s_vec + (tl & 1) * 1024;
    bf16* o = reinterpret_cast<bf16*>(g.out);
    const bf16* res = reinterpret_cast<const bf16*>(g.res);
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int cl = wn * 64 + 32 * jj + 8 * fqo, c = n0 + cl;
      if (c >= g.N) continue;
      float fs[8], ft[8], fb[8], fc[8];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(sv + cl + 4 * h);
        const f32x4 b = *reinterpret_cast<const f32x4*>(sv + 256 + cl + 4 * h);
        const f32x4 d = *reinterpret_cast<const f32x4*>(sv + 512 + cl + 4 * h);
        const f32x4 e = *reinterpret_cast<const f32x4*>(sv + 768 + cl + 4 * h);
#pragma unroll
        for (int i = 0; i < 4; ++i) { fs[4 * h + i] = a[i]; ft[4 * h + i] = b[i]; fb[4 * h + i] = d[i]; fc[4 * h + i] = e[i]; }
      }
      uint4 rv[8];
      if (RES) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int64_t m = m0 + wm * 128 + 16 * i + fro;
          rv[i] = ld16(res + (m < mlim ? m : m0) * g.ldr + g.offr + c);
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = wm * 128 + 16 * i + fro;
        const int64_t m = m0 + r;
        if (m >= mlim) continue;
        const float mu = LN ? s_mu[r] : 0.f, rs = LN ? s_rs[r] : 1.f;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float x = acc[i][2 * jj + (e >> 2)][e & 3];
          if (LN) x = rs * (x - mu * fs[e]) + ft[e];
          x += fb[e];
          if (g.gelu) x = gelu_bf16(x);
          v[e] = x * fc[e];
        }
        if (RES) {
          const uint32_t rw[4] = {rv[i].x, rv[i].y, rv[i].z, rv[i].w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[2 * e] += __uint_as_float(rw[e] << 16);
            v[2 * e + 1] += __uint_as_float(rw[e] & 0xffff0000u);
          }
        }
        bf16x8 ov;
#pragma unroll
        for (int e = 0; e < 8; ++e) ov[e] = (bf16)v[e];
        const int64_t dst = g.store_mode == STORE_CB16 ? ((((int64_t)(c >> 4) * g.cb_px + m) << 4) + (c & 15)) : m * g.ldo + g.offo + c;
        *reinterpret_cast<bf16x8*>(o + dst) = ov;
      }
    }
  };

  // ---- prologue: the first tile's vectors, then X-a, W-a, W-b, X-b of step 0, X-a, W-a of step 1 ----
  // (steps 0 and 1 belong to tile 0: nk >= 2)
  Geo q0 = geo(0);
  issue_vec(0, q0);
  issue(0, 0, q0, U_XA); issue(0, 0, q0, U_WA); issue(0, 0, q0, U_WB); issue(0, 0, q0, U_XB); issue(0, 1, q0, U_XA); issue(0, 1, q0, U_WA);
  g8_vm<8>();
  __builtin_amdgcn_s_barrier();
  if (wm == 1) __builtin_amdgcn_s_barrier();

#define G8_MFMA_BEGIN                                   \
  __builtin_amdgcn_sched_barrier(0);                    \
  __builtin_amdgcn_s_barrier();                         \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");    \
  __builtin_amdgcn_sched_barrier(0);                    \
  __builtin_amdgcn_s_setprio(1);
#define G8_MFMA_END                                     \
  __builtin_amdgcn_s_setprio(0);                        \
  __builtin_amdgcn_sched_barrier(0);                    \
  __builtin_amdgcn_s_barrier();                         \
  asm volatile("" ::: "memory");                        \
  __builtin_amdgcn_sched_barrier(0);

  // (tl, t) of steps s, s + 1, s + 2
  int tl0 = 0, t0 = 0, tl1 = nk > 1 ? 0 : 1, t1 = nk > 1 ? 1 : 0;
  int tl2 = t1 + 1 < nk ? tl1 : tl1 + 1, t2 = t1 + 1 < nk ? t1 + 1 : 0;
  Geo q1 = tl1 == 0 ? q0 : geo(tl1), q2 = tl2 == tl1 ? q1 : geo(tl2);
  bf16x8 xf[4][2], wa[2][2], wb[2][2];
  for (int s = 0; s < nsteps; ++s) {
    const char* ub = smem + (s & 1) * G8_BUF;
    const bool last = t0 == nk - 1;                // the tile's last K tile
    const bool vnext = t1 == 0;                    // step s + 1 starts a tile: its vectors go out at P1
    // P1: X-a, W-a -> pixel tiles 0-3 x channel tiles 0-1
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) xf[i][ks] = frag(ub + U_XA * G8_UNIT, wm * 64 + 16 * i, ks);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) wa[j][ks] = frag(ub + U_WA * G8_UNIT, wn * 32 + 16 * j, ks);
    g8_vm<6>();
    if (vnext) issue_vec(tl1, q1);
    issue(tl1, t1, q1, U_WB);
    G8_MFMA_BEGIN
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[j][ks], xf[i][ks], acc[i][j], 0, 0, 0);
    if (LN && wn < 2) {
      stats(xf);
      if (last) stats_out();
    }
    G8_MFMA_END
    // P2: W-b -> pixel tiles 0-3 x channel tiles 2-3 (one more DMA outstanding after a vector issue)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) wb[j][ks] = frag(ub + U_WB * G8_UNIT, wn * 32 + 16 * j, ks);
    if (vnext) g8_vm<7>(); else g8_vm<6>();
    issue(tl1, t1, q1, U_XB);
    G8_MFMA_BEGIN
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) acc[i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[j][ks], xf[i][ks], acc[i][2 + j], 0, 0, 0);
    G8_MFMA_END
    // P3: X-b -> pixel tiles 4-7 x channel tiles 2-3
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) xf[i][ks] = frag(ub + U_XB * G8_UNIT, wm * 64 + 16 * i, ks);
    if (vnext) g8_vm<7>(); else g8_vm<6>();
    issue(tl2, t2, q2, U_XA);
    G8_MFMA_BEGIN
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) acc[4 + i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[j][ks], xf[i][ks], acc[4 + i][2 + j], 0, 0, 0);
    if (LN && wn >= 2) {
      stats(xf);
      if (last) stats_out();
    }
    G8_MFMA_END
    // P4: (no reads) -> pixel tiles 4-7 x channel tiles 0-1
    if (vnext) g8_vm<7>(); else g8_vm<6>();
    issue(tl2, t2, q2, U_WA);
    G8_MFMA_BEGIN
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[j][ks], xf[i][ks], acc[4 + i][j], 0, 0, 0);
    G8_MFMA_END
    if (last) {
      epilogue(tl0, q0);
#pragma unroll
      for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    tl0 = tl1; t0 = t1; tl1 = tl2; t1 = t2;
    q0 = q1; q1 = q2;
    if (++t2 == nk) { t2 = 0; ++tl2; q2 = geo(tl2); }
  }
#undef G8_MFMA_BEGIN
#undef G8_MFMA_END
  if (wm == 0) __builtin_amdgcn_s_barrier();
  g8_vm<0>();
}

// Eligible: bf16 NHWC store, 16-byte aligned rows, N % 8 == 0, sources with img_mul 1 / img_add 0
// and every source but the last a multiple of 64 wide (a K tile never straddles two)
bool gemm8_ok(const GemmArgs& g) {
  if (g.store_mode == STORE_CB16 && (g.cb_px < g.M || g.N % 16 || g.wstride)) return false;
  if (g.store_mode == STORE_SHUFFLE && ((g.N / 4) % 8 || g.N % 4)) return false;
  if (g.conv3)                                    // implicit 3x3: one source, whole 64-channel K tiles per tap
    return g.allow_g8 && g.a.n == 1 && g.cin % 64 == 0 && g.a.Ktot == 9 * g.cin && !g.ln && !g.wstride && g.N % 8 == 0 &&
           g.ldo % 8 == 0 && g.offo % 8 == 0 && g.ldw % 8 == 0 && g.a.s[0].ld % 8 == 0 && g.a.s[0].off % 8 == 0 &&
           g.a.s[0].img_mul == 1 && g.a.s[0].img_add == 0 && reinterpret_cast<uintptr_t>(g.a.s[0].base) % 16 == 0 &&
           reinterpret_cast<uintptr_t>(g.out) % 16 == 0 && reinterpret_cast<uintptr_t>(g.w) % 16 == 0 &&
           (!g.res || (g.ldr % 8 == 0 && g.offr % 8 == 0 && reinterpret_cast<uintptr_t>(g.res) % 16 == 0)) &&
           g.Wimg > 0 && g.HW % g.Wimg == 0 && g.M % g.HW == 0 && g.HW / g.Wimg < 65536;
  if (!g.allow_g8 || (g.store_mode != STORE_NHWC && g.store_mode != STORE_CB16) || g.conv3 || g.a.cb_px || g.N % 8 || g.ldo % 8 || g.offo % 8 ||
      g.ldw % 8 || g.a.Ktot % 8 || g.a.n < 1)
    return false;
  if (g.ln && g.a.n != 1) return false;
  if (g.res && (g.ldr % 8 || g.offr % 8 || reinterpret_cast<uintptr_t>(g.res) % 16)) return false;
  if (reinterpret_cast<uintptr_t>(g.out) % 16 || reinterpret_cast<uintptr_t>(g.w) % 16) return false;
  if (g.wstride && (g.HW <= 0 || g.M % g.HW || g.wstride % 8)) return false;
  if (g.M > INT32_MAX) return false;
  for (int j = 0; j < g.a.n; ++j) {
    const SrcDesc& s = g.a.s[j];
    if (s.img_mul != 1 || s.img_add != 0 || s.K % 8 || s.ld % 8 || s.off % 8 || reinterpret_cast<uintptr_t>(s.base) % 16) return false;
    if (j + 1 < g.a.n && s.K % 64) return false;
  }
  return true;
}

// g.allow_g8 == 2: the persistent form (nk >= 2), one block per CU (or per tile when fewer)
void launch_gemm8(const GemmArgs& g, hipStream_t st) {
  const int64_t mt = g.wstride ? (g.M / g.HW) * ((g.HW + 255) / 256) : (g.M + 255) / 256;
  const int64_t nblk = mt * ((g.N + 255) / 256);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm8_kernel<false>), hipFuncAttributeMaxDynamicSharedMemorySize, G8_BYTES);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm8_kernel<true>), hipFuncAttributeMaxDynamicSharedMemorySize, G8_BYTES);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm8p_kernel<false, false>), hipFuncAttributeMaxDynamicSharedMemorySize, G8P_BYTES);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm8p_kernel<true, false>), hipFuncAttributeMaxDynamicSharedMemorySize, G8P_BYTES);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm8p_kernel<false, true>), hipFuncAttributeMaxDynamicSharedMemorySize, G8P_BYTES);
    attr_set = true;
  }
  if (g.allow_g8 == 2 && g.a.Ktot > 64 && !(g.ln && g.res) && !g.conv3 && (g.store_mode == STORE_NHWC || g.store_mode == STORE_CB16)) {
    const int64_t grid = std::min<int64_t>(nblk, 256);
    const dim3 gd((unsigned)grid);
    if (g.ln) hipLaunchKernelGGL((gemm8p_kernel<true, false>), gd, dim3(512), G8P_BYTES, st, g);
    else if (g.res) hipLaunchKernelGGL((gemm8p_kernel<false, true>), gd, dim3(512), G8P_BYTES, st, g);
    else hipLaunchKernelGGL((gemm8p_kernel<false, false>), gd, dim3(512), G8P_BYTES, st, g);
    return;
  }
  if (g.ln) hipLaunchKernelGGL((gemm8_kernel<true>), dim3((unsigned)nblk), dim3(512), G8_BYTES, st, g);
  else hipLaunchKernelGGL((gemm8_kernel<false>), dim3((unsigned)nblk), dim3(512), G8_BYTES, st, g);
}

#ifdef TURTLE_G8_ABLATIONS
// tools/g8bench ablation launcher (non-persistent kernel, one instantiation per DBG value)
template <int DBG>
static void g8_launch_dbg(const GemmArgs& g, hipStream_t st) {
  const int64_t mt = (g.M + 255) / 256, nblk = mt * ((g.N + 255) / 256);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm8_kernel<false, DBG>), hipFuncAttributeMaxDynamicSharedMemorySize, G8_BYTES);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm8_kernel<true, DBG>), hipFuncAttributeMaxDynamicSharedMemorySize, G8_BYTES);
  if (g.ln) hipLaunchKernelGGL((gemm8_kernel<true, DBG>), dim3((unsigned)nblk), dim3(512), G8_BYTES, st, g);
  else hipLaunchKernelGGL((gemm8_kernel<false, DBG>), dim3((unsigned)nblk), dim3(512), G8_BYTES, st, g);
}
void launch_gemm8_dbg(const GemmArgs& g, int dbg, hipStream_t st) {
  switch (dbg) {
    case 1: g8_launch_dbg<1>(g, st); break;
    case 2: g8_launch_dbg<2>(g, st); break;
    case 4: g8_launch_dbg<4>(g, st); break;
    case 8: g8_launch_dbg<8>(g, st); break;
    case 16: g8_launch_dbg<16>(g, st); break;
    case 5: g8_launch_dbg<5>(g, st); break;
    case 6: g8_launch_dbg<6>(g, st); break;
    case 14: g8_launch_dbg<14>(g, st); break;
    case 7: g8_launch_dbg<7>(g, st); break;
    case 15: g8_launch_dbg<15>(g, st); break;
    case 22: g8_launch_dbg<22>(g, st); break;
    case 32: g8_launch_dbg<32>(g, st); break;
    case 34: g8_launch_dbg<34>(g, st); break;
    case 38: g8_launch_dbg<38>(g, st); break;
    case 46: g8_launch_dbg<46>(g, st); break;
    case 39: g8_launch_dbg<39>(g, st); break;
    case 47: g8_launch_dbg<47>(g, st); break;
    case 64: g8_launch_dbg<64>(g, st); break;
    case 96: g8_launch_dbg<96>(g, st); break;
    case 33: g8_launch_dbg<33>(g, st); break;
    default: g8_launch_dbg<0>(g, st);
  }
}
#endif

}  // namespace turtle

// bf16 GEMM, 2-D tiled, deep LDS-DMA ring ("kt" kernel): the projections whose weights are too
// large to stream per pixel panel (pn / ar kernels) and the implicit-3x3 resampling convolutions.
//
//   out[m][n] = epilogue( sum_k A[m][k] * W[n][k] )        m = pixel, n = output channel
//
// Same contract as gemm_lds_kernel (gemm2.hip): K-concatenated multi-source A, implicit 3x3 taps,
// LayerNorm folded into the epilogue with statistics from the staged A tiles, bias / GELU / scale /
// residual, NHWC / PixelShuffle / PixelUnshuffle stores, per-image weight sets (W_eff).
//
// Structure (MI355X):
//   * BM x BN output tile per block of WM x WN waves; BK = 32, so one K tile is one MFMA K step and
//     a STAGES-deep ring of tiles fits in LDS (4 x 32 KB at 256 x 256): three tiles stay in flight
//     behind the one being consumed, ~48 KB of pixel rows per CU, enough to cover HBM latency with
//     one block per CU. One barrier per K tile (the ring slot refilled at tile kt was consumed at
//     kt - 1, before that barrier);
//   * both operands go HBM/L2 -> LDS by global_load_lds (64 lanes x 16 B per instruction), rows of
//     64 B, chunk c of row r stored at position c ^ h(r), h(r) = (r >> 2) & 2: conflict-free
//     ds_read_b128 on gfx950's lane groups for the pixel fragments (natural rows) and for the
//     weight fragments (permuted rows below) - checked exhaustively on the host;
//   * weight rows are read in pn's permuted order (MFMA row 4g+e of sub-tile s <- channel 8g+4s+e of
//     a 32-channel group), so a lane's accumulators hold 8 CONSECUTIVE channels of one pixel and the
//     epilogue is register-direct: one 16-byte residual load and one 16-byte store per lane, pixel
//     row and 32 channels, no LDS staging;
//   * a K tile never straddles two sources or two 3x3 taps (source widths / cin multiples of 32):
//     its source resolves on the scalar unit once per tile.
#include "common.h"
#include "kernels.h"

namespace turtle {

__device__ __attribute__((aligned(64))) uint4 g_zero_kt[4];

// LDS-DMA from inline asm: hipcc treats a builtin global_load_lds as a pending LDS write and puts
// vmcnt(0) in front of the next ds_read, which would drain the whole ring every K tile. The ring's
// waits are counted by hand (kt_wait_vm before each tile's barrier).
TURTLE_DEV void kt_dma16(const void* g, uint32_t lds_wave_base) {   // 64 lanes x 16 B -> LDS at M0
  unsigned keep;                                                   // M0 is compiler-reserved: restore it
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(lds_wave_base) : "memory");
}
template <int N>
TURTLE_DEV void kt_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}
TURTLE_DEV int kt_h(int r) { return (r >> 2) & 2; }

template <int BM, int BN, int WM, int WN>
struct KT {
  static constexpr int NW = WM * WN, NT = NW * 64;
  static constexpr int PM = BM / WM, PN = BN / WN;       // wave tile
  static constexpr int TM = PM / 16, TN = PN / 16, NG = TN / 2;
  static constexpr int STAGES = 4;
  static constexpr int A_BYTES = BM * 64, W_BYTES = BN * 64, STAGE = A_BYTES + W_BYTES;
  static constexpr int AI = BM * 4 / NT, WI = BN * 4 / NT, NL = AI + WI;   // DMA instructions per thread per stage
  static constexpr int TPR = NT / BM;                    // LN statistics: threads per pixel row
  static constexpr int BYTES = STAGES * STAGE + 2 * BM * 4;
  static_assert(BM * 4 % NT == 0 && BN * 4 % NT == 0 && TN % 2 == 0 && TM >= 1 && (TPR == 1 || TPR == 2 || TPR == 4), "kt geometry");
};

template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(WM * WN * 64, (WM * WN <= 4) ? 2 : 1) void gemm_kt_kernel(GemmArgs g) {
  using S = KT<BM, BN, WM, WN>;
  constexpr int TM = S::TM, TN = S::TN, NG = S::NG, AI = S::AI, WI = S::WI, NL = S::NL, NW = S::NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_mu = reinterpret_cast<float*>(smem + S::STAGES * S::STAGE);
  float* s_rs = s_mu + BM;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int fr = lane & 15, fq = lane >> 4;

  // ---- tile: output-channel tiles of one pixel panel are consecutive ids on one XCD ----
  const int ntn = (g.N + BN - 1) / BN;
  int lin = blockIdx.x;
  {
    const int nblk = gridDim.x, q = nblk / 8, r = nblk % 8, x = lin % 8, y = lin / 8;
    lin = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;
  }
  const int nt = lin % ntn, mt = lin / ntn;
  int64_t m0, mlim;
  if (g.wstride) {
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
  const int nk = (K + 31) / 32;
  const int img0 = (int)(m0 / g.HW);
  const bf16* Wp = reinterpret_cast<const bf16*>(g.w) + (g.wstride ? (int64_t)(img0 / g.wdiv) * g.wstride : 0);

  // ---- DMA geometry: instruction i of wave w fills LDS chunks (i * NW + w) * 64 + lane of the A
  // (i < AI) or W part; chunk q -> row q / 4, position q % 4, holding k-chunk (q % 4) ^ h(row) ----
  int a_img[AI], a_p[AI], a_y[AI], a_x[AI], a_cc[AI];
  bool a_ok[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int q = (i * NW + wid) * 64 + lane, r = q >> 2;
    a_cc[i] = ((q & 3) ^ kt_h(r)) * 8;
    const int64_t m = m0 + r;
    a_ok[i] = m < mlim;
    const int mm = a_ok[i] ? (int)m : (int)m0;
    a_img[i] = mm / g.HW;
    a_p[i] = mm - a_img[i] * g.HW;
    a_y[i] = g.conv3 ? a_p[i] / g.Wimg : 0;
    a_x[i] = g.conv3 ? a_p[i] - a_y[i] * g.Wimg : 0;
  }
  const bf16* w_src[WI];
  bool w_ok[WI];
  int w_cc[WI];
#pragma unroll
  for (int i = 0; i < WI; ++i) {
    const int q = (i * NW + wid) * 64 + lane, r = q >> 2;
    w_cc[i] = ((q & 3) ^ kt_h(r)) * 8;
    w_ok[i] = n0 + r < g.N;
    w_src[i] = Wp + (int64_t)min(n0 + r, g.N - 1) * g.ldw + w_cc[i];
  }
  const int Himg = g.conv3 ? g.HW / g.Wimg : 0;

  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  auto issue = [&](int kt, int stage) {
    const uint32_t sA = lds_base + stage * S::STAGE;
    const uint32_t sW = sA + S::A_BYTES;
    const int k0 = kt * 32;
    const bf16* base = reinterpret_cast<const bf16*>(g.a.s[0].base);
    int64_t sld = g.a.s[0].ld;
    int soff = g.a.s[0].off, smul = g.a.s[0].img_mul, sadd = g.a.s[0].img_add, kb = 0;
    int dy = 0, dx = 0;
    if (g.conv3) {
      const int tap = k0 / g.cin;
      soff += k0 - tap * g.cin;
      dy = tap / 3 - 1; dx = tap - (tap / 3) * 3 - 1;
    } else {
      int kbj = g.a.s[0].K;
#pragma unroll
      for (int j = 1; j < TURTLE_MAX_SRC; ++j) {
        const bool hit = j < g.a.n && k0 >= kbj;
        base = hit ? reinterpret_cast<const bf16*>(g.a.s[j].base) : base;
        sld = hit ? g.a.s[j].ld : sld;
        soff = hit ? g.a.s[j].off : soff;
        smul = hit ? g.a.s[j].img_mul : smul;
        sadd = hit ? g.a.s[j].img_add : sadd;
        kb = hit ? kbj : kb;
        kbj += j < g.a.n ? g.a.s[j].K : 0;
      }
      soff += k0 - kb;
    }
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int y = a_y[i] + dy, x = a_x[i] + dx;
      const bool inb = !g.conv3 || (y >= 0 && y < Himg && x >= 0 && x < g.Wimg);
      const bool ok = a_ok[i] && inb && k0 + a_cc[i] < K;
      const int pix = (a_img[i] * smul + sadd) * g.HW + a_p[i] + dy * g.Wimg + dx;
      // channel-blocked source: channel k of pixel p at ((k / 16) cb_px + p) 16 + k % 16
      const bf16* src = g.a.cb_px ? base + ((((int64_t)((k0 + a_cc[i]) >> 4) * g.a.cb_px + pix) << 4) + ((k0 + a_cc[i]) & 15))
                                  : base + (int64_t)pix * sld + soff + a_cc[i];
      kt_dma16(ok ? reinterpret_cast<const void*>(src) : reinterpret_cast<const void*>(g_zero_kt), sA + (i * NW + wid) * 1024);
    }
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      const bool ok = w_ok[i] && k0 + w_cc[i] < K;
      kt_dma16(ok ? reinterpret_cast<const void*>(w_src[i] + k0) : reinterpret_cast<const void*>(g_zero_kt),
               sW + (i * NW + wid) * 1024);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // LN statistics: TPR threads per pixel row, 4 / TPR chunks each per K tile
  const int lr = tid / S::TPR, lh = tid % S::TPR;
  float ls = 0.f, lq = 0.f;
  // fragment rows: pixel rows (natural) and permuted weight rows of this wave
  const int prow0 = wm * S::PM + fr;
  const int wrow0 = wn * S::PN + 8 * (fr >> 2) + (fr & 3);

#pragma unroll
  for (int s = 0; s < S::STAGES - 1; ++s)
    if (s < nk) issue(s, s);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(nk - 1, kt + S::STAGES - 2) - kt;   // tiles issued after kt
    if (ahead >= 2) kt_wait_vm<2 * NL>();
    else if (ahead == 1) kt_wait_vm<NL>();
    else kt_wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                 // tile kt landed everywhere; tile kt - 1 consumed everywhere
    asm volatile("" ::: "memory");
    if (kt + S::STAGES - 1 < nk) issue(kt + S::STAGES - 1, (kt + S::STAGES - 1) % S::STAGES);
    const char* sA = smem + (kt % S::STAGES) * S::STAGE;
    const char* sW = sA + S::A_BYTES;
    if (g.ln) {
      typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
      const bf16x2 one2 = __builtin_bit_cast(bf16x2, 0x3F803F80u);
      const char* row = sA + lr * 64;
#pragma unroll
      for (int pc = 0; pc < 4 / S::TPR; ++pc) {
        const uint4 x = *reinterpret_cast<const uint4*>(row + (((lh * (4 / S::TPR) + pc) ^ kt_h(lr)) << 4));
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bf16x2 v2 = __builtin_bit_cast(bf16x2, w[e]);
          ls = __builtin_amdgcn_fdot2_f32_bf16(v2, one2, ls, false);
          lq = __builtin_amdgcn_fdot2_f32_bf16(v2, v2, lq, false);
        }
      }
    }
    bf16x8 wf[TN], xf[TM];
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const int r = wrow0 + 32 * (t >> 1) + 4 * (t & 1);
      wf[t] = *reinterpret_cast<const bf16x8*>(sW + r * 64 + ((fq ^ kt_h(r)) << 4));
    }
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      const int r = prow0 + 16 * t;
      xf[t] = *reinterpret_cast<const bf16x8*>(sA + r * 64 + ((fq ^ kt_h(r)) << 4));
    }
    // every fragment read of the tile is in flight before the first MFMA (left to itself the
    // scheduler interleaves read -> wait -> MFMAs per pixel fragment, one LDS round trip each)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[tn], xf[tm], acc[tm][tn], 0, 0, 0);
  }
  if (g.ln) {
#pragma unroll
    for (int o = 1; o < S::TPR; o <<= 1) { ls += __shfl_xor(ls, o, 64); lq += __shfl_xor(lq, o, 64); }
    if (lh == 0) {
      const float mu = ls / K;
      s_mu[lr] = mu;
      s_rs[lr] = rsqrtf(fmaxf(lq / K - mu * mu, 0.f) + 1e-5f);
    }
    __syncthreads();
  }

  // ---- epilogue: lane holds channels c .. c+7 (c = n0 + wn PN + 32 j + 8 fq) of pixel row
  // m0 + wm PM + 16 tm + fr ----
  bf16* o = reinterpret_cast<bf16*>(g.out);
  const bf16* res = reinterpret_cast<const bf16*>(g.res);
  const float* vs = g.ln_s ? g.ln_s : g.zeros;
  const float* vt = g.ln_t ? g.ln_t : g.zeros;
  const float* vb = g.bias ? g.bias : g.zeros;
  const float* vc = g.scale ? g.scale : g.ones;
#pragma unroll
  for (int j = 0; j < NG; ++j) {
    const int c = n0 + wn * S::PN + 32 * j + 8 * fq;
    if (c >= g.N) continue;                       // N % 8 == 0: a group of 8 is all in or all out
    float fs[8], ft[8], fb[8], fc[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(vs + c + 4 * h), b = *reinterpret_cast<const f32x4*>(vt + c + 4 * h);
      const f32x4 d = *reinterpret_cast<const f32x4*>(vb + c + 4 * h), e = *reinterpret_cast<const f32x4*>(vc + c + 4 * h);
#pragma unroll
      for (int i = 0; i < 4; ++i) { fs[4 * h + i] = a[i]; ft[4 * h + i] = b[i]; fb[4 * h + i] = d[i]; fc[4 * h + i] = e[i]; }
    }
    uint4 rv[TM];
    if (res) {
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int64_t m = m0 + wm * S::PM + 16 * tm + fr;
        rv[tm] = ld16(res + (m < mlim ? m : m0) * g.ldr + g.offr + c);
      }
    }
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      const int r = wm * S::PM + 16 * tm + fr;
      const int64_t m = m0 + r;
      if (m >= mlim) continue;
      const float mu = g.ln ? s_mu[r] : 0.f, rs = g.ln ? s_rs[r] : 1.f;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float x = acc[tm][2 * j + (e >> 2)][e & 3];
        if (g.ln) x = rs * (x - mu * fs[e]) + ft[e];
        x += fb[e];
        if (g.gelu) x = gelu_bf16(x);
        v[e] = x * fc[e];
      }
      if (res) {
        const uint32_t rw[4] = {rv[tm].x, rv[tm].y, rv[tm].z, rv[tm].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[2 * e] += __uint_as_float(rw[e] << 16);
          v[2 * e + 1] += __uint_as_float(rw[e] & 0xffff0000u);
        }
      }
      bf16x8 ov;
#pragma unroll
      for (int e = 0; e < 8; ++e) ov[e] = (bf16)v[e];
      int64_t dst;
      if (g.store_mode == STORE_NHWC) {
        dst = m * g.ldo + g.offo + c;
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
      *reinterpret_cast<bf16x8*>(o + dst) = ov;
    }
  }
}

// Eligible: bf16, 16-byte aligned operand rows, N % 8 == 0 (PixelShuffle: N / 4 % 8), K tiles never
// straddle sources / taps (all but the last source K % 32 == 0, conv3 cin % 32 == 0).
bool gemm_kt_ok(const GemmArgs& g) {
  if (!g.allow_kt || g.store_mode == STORE_CB16 || g.N % 8 || g.ldo % 8 || g.offo % 8 || g.ldw % 8) return false;
  if (g.res && (g.ldr % 8 || g.offr % 8)) return false;
  if (g.store_mode == STORE_SHUFFLE && (g.N / 4) % 8) return false;
  if (reinterpret_cast<uintptr_t>(g.out) % 16 || reinterpret_cast<uintptr_t>(g.w) % 16 ||
      (g.res && reinterpret_cast<uintptr_t>(g.res) % 16))
    return false;
  if (g.a.cb_px)                                  // channel-blocked A (tilepd.hip output): one plain source
    return !g.conv3 && g.a.n == 1 && g.a.s[0].off == 0 && g.a.s[0].img_mul == 1 && g.a.s[0].img_add == 0 &&
           g.a.Ktot % 16 == 0 && g.a.cb_px >= g.M && reinterpret_cast<uintptr_t>(g.a.s[0].base) % 16 == 0;
  if (g.conv3) return g.cin % 32 == 0 && g.a.n == 1 && g.a.s[0].ld % 8 == 0 && g.a.s[0].off % 8 == 0;
  for (int j = 0; j < g.a.n; ++j) {
    if (g.a.s[j].K % 8 || g.a.s[j].ld % 8 || g.a.s[j].off % 8 || reinterpret_cast<uintptr_t>(g.a.s[j].base) % 16) return false;
    if (j + 1 < g.a.n && g.a.s[j].K % 32) return false;
  }
  return g.a.Ktot % 8 == 0;
}

template <int BM, int BN, int WM, int WN>
static void launch_kt_cfg(const GemmArgs& g, hipStream_t st) {
  using S = KT<BM, BN, WM, WN>;
  const int64_t mt = g.wstride ? (g.M / g.HW) * ((g.HW + BM - 1) / BM) : (g.M + BM - 1) / BM;
  const int64_t nblk = mt * ((g.N + BN - 1) / BN);
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_kt_kernel<BM, BN, WM, WN>), hipFuncAttributeMaxDynamicSharedMemorySize, S::BYTES);
    attr_set = true;
  }
  hipLaunchKernelGGL((gemm_kt_kernel<BM, BN, WM, WN>), dim3((unsigned)nblk), dim3(S::NT), S::BYTES, st, g);
}

// tile choice (tools/kbench): 256 x 256 with 8 waves where N >= 256 fills the chip, else 128 x 128
// with 4 waves (two blocks per CU); g.dbg & 0x30 forces a configuration for kbench
void launch_gemm_kt(const GemmArgs& g, hipStream_t st) {
  // the largest tile that still gives every CU a block (one round), else 128 x 128
  const int cfg = (g.dbg >> 4) & 3;
  const int64_t t256 = ((g.M + 255) / 256) * ((g.N + 255) / 256), t128x256 = ((g.M + 127) / 128) * ((g.N + 255) / 256);
  const int pick = cfg ? cfg : (g.N >= 256 && t256 >= 256) ? 1 : (g.N >= 256 && t128x256 >= 256) ? 3 : 2;
  if (pick == 1) launch_kt_cfg<256, 256, 2, 4>(g, st);
  else if (pick == 3) launch_kt_cfg<128, 256, 2, 4>(g, st);
  else launch_kt_cfg<128, 128, 2, 2>(g, st);
}

}  // namespace turtle

// bf16 1x1-convolution GEMM over resident pixel panels ("pn" kernel): the shape of every
// LayerNorm -> pointwise projection of the Turtle blocks (K = dim <= 512, N = 2..5 x dim).
//
//   out[m][n] = epilogue( sum_k A[m][k] * W[n][k] )        m = pixel, n = output channel
//
// Why a separate kernel: at K <= 512 a 128 x 128 output tile is only 4..8 K steps of MFMAs, so the
// K-loop GEMMs spend most of their issue slots on per-tile fixed costs (operand address setup,
// LayerNorm statistics, a generic epilogue); PMC on gemm_lds for the L3 GFFW projection showed
// ~1800 VALU against 128 MFMA per wave. And these GEMMs write 3..5x more than they read, so the
// store stream has to run while the matrix cores work. Here:
//   * persistent: one 512-thread block per CU walks the pixel panels p = block, block + grid, ...;
//     a BM x K panel goes HBM -> LDS by LDS-DMA (global_load_lds, 16 B per lane) into one of two
//     buffers while the block computes on the other, so panel loads never stall the MFMAs;
//   * XOR-swizzled 16-byte chunks (chunk c of row r at c ^ (r & 15)): conflict-free ds_read_b128
//     B fragments; LayerNorm statistics once per panel (v_dot2 sums), two barriers per panel and
//     none inside the channel-tile sweep;
//   * each wave owns 32 output channels x BM / WM pixels of a tile; W fragments come from L2
//     straight into a register ring D K steps deep that wraps into the next tile / panel;
//   * W rows are read in a permuted order (MFMA row 4g+e of sub-tile t <- channel 8g+4t+e), so a
//     lane's accumulators hold 8 CONSECUTIVE channels of one pixel: the epilogue is 2 FMAs per
//     element (LN folded: rs*acc + (tb - rs*mu*s)) and one 16-byte store per lane and pixel row;
//   * rows past the end of M load (and store) copies of the last row, so every wave issues the
//     same number of stores per tile and the panel-top wait can leave exactly those in flight.
// Eligible: bf16, plain NHWC store, no 3x3, K in {64, 128, 256, 384, 512}, N % 64 == 0 (N % 256
// for the 8-wave-wide tile), 16-byte aligned operand rows. tools/kbench compares it with the
// K-loop (gemm2.hip) and panel (gemm.hip) kernels.
#include "common.h"
#include "kernels.h"

#include <type_traits>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

namespace turtle {

// Stores and the panel LDS-DMA are issued from inline asm, so hipcc's waitcnt bookkeeping sees
// only this kernel's loads. Its own waits treat a mix of pending loads and stores as unordered and
// fall back to vmcnt(0), which would make every channel tile wait for the previous tile's stores;
// with the stores hidden it counts its loads exactly (the hardware retires vmcnt in issue order,
// so a hidden store younger than a waited load only ever makes that wait longer, never short).
// The DMA is waited for by hand (panel-top vmcnt) before the barrier that publishes the panel.
TURTLE_DEV void pn_gstore(void* p, const bf16x8& v) {   // s_nop 1: the >8-byte store reads its data late
  asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" : : "v"(p), "v"(v) : "memory");
}
TURTLE_DEV void pn_dma16(const void* g, uint32_t lds_wave_base) {   // 64 lanes x 16 B -> LDS at M0
  unsigned keep;                                                   // M0 is compiler-reserved: restore it
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(lds_wave_base) : "memory");
}
// s_memtime stamps for tools/kbench (GemmArgs::stamps; null in the product path)
TURTLE_DEV void pn_stamp(unsigned long long* buf, int& si) {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  if (si < 255) {
    asm volatile("global_store_dwordx2 %0, %1, off" : : "v"(buf + si), "v"(t) : "memory");
    ++si;
  }
}

template <int N>
TURTLE_DEV void pn_vmwait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" : : "n"(N) : "memory");
}

template <int N, int I = 0, typename F>
TURTLE_DEV void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}

template <int CPR>
TURTLE_DEV int pn_swz(int r) {           // XOR applied to the 16-byte chunk index of panel row r
  if constexpr (CPR >= 16) return r & 15;
  else return (r >> 1) & 7;              // 128-byte rows: two rows share the 64 banks
}

constexpr int PN_WAVES = 8;

struct PnSrc {                           // A source of one 16-byte K chunk
  const bf16* base;                      // source base + channel offset of the chunk
  int64_t ld;                            // pixel stride (elements)
  int smul, sadd;                        // source image = img * smul + sadd
};

struct PnPanel {                         // geometry of one pixel panel
  int64_t m0, mlim;
  int img0, p0;
  const bf16* w;
};

template <int BM>
TURTLE_DEV PnPanel pn_panel(const GemmArgs& g, int p) {   // 32-bit math: M < 2^31 (gemm_pn_ok)
  PnPanel P;
  const int M = (int)g.M;
  int m0, mlim, img0;
  if (g.wstride) {
    const int tpi = (g.HW + BM - 1) / BM;
    img0 = p / tpi;
    m0 = img0 * g.HW + (p - img0 * tpi) * BM;
    mlim = min(M, (img0 + 1) * g.HW);
  } else {
    m0 = p * BM;
    mlim = M;
    img0 = m0 / g.HW;
  }
  P.m0 = m0;
  P.mlim = mlim;
  P.img0 = img0;
  P.p0 = m0 - img0 * g.HW;
  P.w = reinterpret_cast<const bf16*>(g.w) + (g.wstride ? (int64_t)(img0 / g.wdiv) * g.wstride : 0);
  return P;
}

template <int BM, int KP, int WN, bool RES>
__global__ __launch_bounds__(512, 1) void gemm_pn_kernel(GemmArgs g, int npanel) {
  constexpr int CPR = KP / 8;            // 16-byte chunks per panel row
  constexpr int KS = KP / 32;            // MFMA K steps (K == KP)
  constexpr int WM = PN_WAVES / WN;      // waves along the pixel dimension
  constexpr int MT = BM / WM / 16;       // 16-pixel tiles per wave
  constexpr int NT = 32 * WN;            // output channels per tile
  constexpr int PANEL = BM * KP * 2;
  constexpr int NDMA = PANEL / (PN_WAVES * 1024);   // LDS-DMA instructions per thread per panel
  constexpr int TPR = 64 * PN_WAVES / BM;           // threads per row for the LN statistics
  // W fragments in flight: a ring of D K steps (D divides KS, so it wraps into the next tile)
  constexpr int D = (KS % 8 == 0 && MT < 8) ? 8 : (KS % 4 == 0 ? 4 : 2);
  static_assert(PANEL % (PN_WAVES * 1024) == 0 && MT >= 1 && CPR % 8 == 0 && (CPR < 16 || CPR % 16 == 0),
                "panel geometry");
  // dynamic LDS: [panel buffer 0][panel buffer 1][source table CPR][ln_t + bias N][scale N]
  extern __shared__ __attribute__((aligned(16))) char smem[];
  PnSrc* s_src = reinterpret_cast<PnSrc*>(smem + 2 * PANEL);
  float* e_tb = reinterpret_cast<float*>(s_src + CPR);
  float* e_c = e_tb + g.N;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wid % WN, wm = wid / WN;
  const int fr = lane & 15, fq = lane >> 4;
  const int G = gridDim.x;
  const int ntiles = g.N / NT;
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  // ---- panel p -> LDS buffer `buf`: chunk q = row q / CPR, LDS position q % CPR, holding k-chunk
  // (q % CPR) ^ swz(row); rows past the end of M repeat the last row ----
  auto issue_panel = [&](int p, int buf) {
    const PnPanel P = pn_panel<BM>(g, p);
    const int rmax = (int)(P.mlim - P.m0) - 1;
#pragma unroll
    for (int i = 0; i < NDMA; ++i) {
      const int q = (i * PN_WAVES + wid) * 64 + lane, r = min(q / CPR, rmax), pc = q % CPR;
      const PnSrc e = s_src[pc ^ pn_swz<CPR>(q / CPR)];
      int pp = P.p0 + r, img = P.img0;
      if (pp >= g.HW) { pp -= g.HW; ++img; }
      const int64_t off = ((int64_t)(img * e.smul + e.sadd) * g.HW + pp) * e.ld;
      pn_dma16(e.base + off, lds_base + buf * PANEL + (i * PN_WAVES + wid) * 1024);
    }
  };

  // source of each 16-byte K chunk (one scan per block; multi-source A = concatenated inputs)
  if (tid < CPR) {
    const int k = tid * 8;
    int j = 0, kb = 0;
    while (j + 1 < g.a.n && k >= kb + g.a.s[j].K) kb += g.a.s[j++].K;
    const SrcDesc& sd = g.a.s[j];
    s_src[tid] = PnSrc{reinterpret_cast<const bf16*>(sd.base) + sd.off + (k - kb), sd.ld, sd.img_mul, sd.img_add};
  }
  // per-channel epilogue vectors (LayerNorm itself is applied to the panel in LDS)
  for (int n = tid; n < g.N; n += 64 * PN_WAVES) {
    e_tb[n] = (g.ln_t ? g.ln_t[n] : 0.f) + (g.bias ? g.bias[n] : 0.f);
    if (g.scale) e_c[n] = g.scale[n];
  }
  __syncthreads();

  // ---- W fragments of (tile nt of weights wp, K step KSTEP) into ring slot `slot` ----
  bf16x8 wb[D][2];
  auto wrow = [&](const bf16* wp, int nt, int tn) {   // lane's W row for sub-tile tn of tile nt
    return wp + (int64_t)(nt * NT + wn * 32 + (fr >> 2) * 8 + tn * 4 + (fr & 3)) * g.ldw + fq * 8;
  };
  auto load_w = [&](auto kstep, const bf16* r0, const bf16* r1, int slot) {
    constexpr int KSTEP = decltype(kstep)::value;
    wb[slot][0] = *reinterpret_cast<const bf16x8*>(r0 + KSTEP * 32);
    wb[slot][1] = *reinterpret_cast<const bf16x8*>(r1 + KSTEP * 32);
  };

  // waves 4..7 (the later-dispatched half, paired with 0..3 on the same SIMDs) win VALU / MFMA
  // issue arbitration: their epilogues do not queue behind their partners' MFMA phases
  if (wid >= PN_WAVES / 2) __builtin_amdgcn_s_setprio(1);

  int p = blockIdx.x;
  issue_panel(p, 0);
  {
    const PnPanel P = pn_panel<BM>(g, p);
    const bf16 *r0 = wrow(P.w, 0, 0), *r1 = wrow(P.w, 0, 1);
    static_for<D>([&](auto j) { load_w(j, r0, r1, decltype(j)::value); });
  }
  pn_vmwait<0>();

  const bf16* pr = reinterpret_cast<const bf16*>(g.res);   // non-null iff RES

  unsigned long long* sbuf = g.stamps && lane == 0 && blockIdx.x < 2 ? g.stamps + (blockIdx.x * PN_WAVES + wid) * 256 : nullptr;
  int si = 0;
#define PN_STAMP() do { if (sbuf) pn_stamp(sbuf, si); } while (0)
  for (int it = 0; p < npanel; ++it, p += G) {
    const int buf = it & 1;
    const int pnext = p + G;
    // panel p landed: its DMA is older than the last tile's 2 KS ring loads and MT stores; and
    // every wave is through panel p - G, whose buffer the next panel's DMA now overwrites
    PN_STAMP();
    if (it > 0) pn_vmwait<2 * KS + MT>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const bool hasdma = pnext < npanel;
    if (hasdma) issue_panel(pnext, buf ^ 1);
    PN_STAMP();
    const PnPanel P = pn_panel<BM>(g, p);
    const bf16* wnext = pnext < npanel ? pn_panel<BM>(g, pnext).w : P.w;
    const char* pan = smem + buf * PANEL;

    // ---- LayerNorm of the panel rows, in place: TPR threads per row take its statistics from
    // their CH chunks (chunk order rotated per row to spread banks) and rewrite them as
    // (x - mu) * rstd in bf16, so the tile epilogue is only acc + (W.b + bias) ----
    if (g.ln) {
      typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
      const bf16x2 one2 = __builtin_bit_cast(bf16x2, 0x3F803F80u);
      constexpr int CH = CPR / TPR;
      const int lr = tid / TPR, lh = tid % TPR;
      char* row = smem + buf * PANEL + lr * (KP * 2);
      uint4 xs[CH];
      float ls = 0.f, lq = 0.f;
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        xs[j] = *reinterpret_cast<const uint4*>(row + (lh * CH + ((j + lr * TPR + lh) % CH)) * 16);
        const uint32_t w[4] = {xs[j].x, xs[j].y, xs[j].z, xs[j].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bf16x2 v2 = __builtin_bit_cast(bf16x2, w[e]);
          ls = __builtin_amdgcn_fdot2_f32_bf16(v2, one2, ls, false);
          lq = __builtin_amdgcn_fdot2_f32_bf16(v2, v2, lq, false);
        }
      }
#pragma unroll
      for (int o = 1; o < TPR; o <<= 1) { ls += __shfl_xor(ls, o, 64); lq += __shfl_xor(lq, o, 64); }
      // BiasFree LayerNorm (packed with ln_s = null): x * rstd, uncentred (turtle_t1_arch.py:68-80)
      const float mu = ls / KP, rs = rsqrtf(fmaxf(lq / KP - mu * mu, 0.f) + 1e-5f), nm = g.ln_s ? -mu * rs : 0.f;
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const uint32_t w[4] = {xs[j].x, xs[j].y, xs[j].z, xs[j].w};
        uint32_t o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float a = fmaf(__uint_as_float(w[e] << 16), rs, nm), b = fmaf(__uint_as_float(w[e] & 0xffff0000u), rs, nm);
          typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
          o[e] = __builtin_bit_cast(uint32_t, bf2{(bf16)a, (bf16)b});
        }
        *reinterpret_cast<uint4*>(row + (lh * CH + ((j + lr * TPR + lh) % CH)) * 16) = uint4{o[0], o[1], o[2], o[3]};
      }
      __syncthreads();
    }
    const int mlast = (int)(P.mlim - P.m0) - 1;
    const bf16* prb = RES ? pr + P.m0 * g.ldr + g.offr : nullptr;     // panel row 0 of the residual
    bf16* pob = reinterpret_cast<bf16*>(g.out) + P.m0 * g.ldo + g.offo;

    PN_STAMP();
    for (int nt = 0; nt < ntiles; ++nt) {
      const bool last = nt + 1 == ntiles;
      const bool more = !last || pnext < npanel;
      const bf16* wn_p = last ? wnext : P.w;           // weights of the next tile
      const int nn = last ? 0 : nt + 1;
      const int cb = nt * NT + wn * 32 + fq * 8;       // lane's 8 consecutive channels
      const bf16 *wr0 = wrow(P.w, nt, 0), *wr1 = wrow(P.w, nt, 1);                 // this tile's rows
      const bf16 *wx0 = more ? wrow(wn_p, nn, 0) : wr0, *wx1 = more ? wrow(wn_p, nn, 1) : wr1;   // next
      // residual of this tile, in flight across the MFMAs
      u32x4 rv[RES ? MT : 1];
      if constexpr (RES) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)   // 32-bit in-panel offsets
          rv[mt] = *reinterpret_cast<const u32x4*>(prb + (min(wm * (BM / WM) + mt * 16 + fr, mlast) * (int)g.ldr + cb));
      }
      f32x4 acc[MT][2];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt][0] = acc[mt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      // B fragments one K step ahead in a single buffer: xf[mt] for step ks + 1 is read right after
      // the two MFMAs of step ks that consume it; a scheduling fence per step keeps the compiler
      // from hoisting the whole tile's LDS reads (register pressure)
      bf16x8 xf[MT];
      auto read_x = [&](int ks, int mt) {
        const int r = wm * (BM / WM) + mt * 16 + fr;
        const int c = (ks * 4 + fq) ^ pn_swz<CPR>(r);
        xf[mt] = *reinterpret_cast<const bf16x8*>(pan + r * (KP * 2) + c * 16);
      };
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) read_x(0, mt);
      static_for<KS>([&](auto ksc) {
        constexpr int ks = decltype(ksc)::value;
        constexpr int slot = ks % D;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          acc[mt][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[slot][0], xf[mt], acc[mt][0], 0, 0, 0);
          acc[mt][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[slot][1], xf[mt], acc[mt][1], 0, 0, 0);
          if constexpr (ks + 1 < KS) { if (!(g.dbg & 4)) read_x(ks + 1, mt); }
        }
        // refill the slot behind this step's MFMAs: step ks + D of this tile, or of the next one
        // (always 2 loads per step, so the panel-top count holds; the last tile of the last
        // panel reloads its own rows)
        if (!(g.dbg & 2)) {
          if constexpr (ks + D < KS) load_w(std::integral_constant<int, ks + D>{}, wr0, wr1, slot);
          else load_w(std::integral_constant<int, ks + D - KS>{}, wx0, wx1, slot);
        }
        __builtin_amdgcn_sched_barrier(0);
      });
      PN_STAMP();
      // ---- epilogue: lane holds channels cb .. cb+7 of pixel row (mt*16 + fr) ----
      const f32x4 vt0 = *reinterpret_cast<const f32x4*>(e_tb + cb), vt1 = *reinterpret_cast<const f32x4*>(e_tb + cb + 4);
      const float tb[8] = {vt0[0], vt0[1], vt0[2], vt0[3], vt1[0], vt1[1], vt1[2], vt1[3]};
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float a = acc[mt][e >> 2][e & 3];
          v[e] = a + tb[e];
        }
        if (g.gelu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = gelu_bf16(v[e]);
        }
        if (g.scale) {
          const f32x4 vc0 = *reinterpret_cast<const f32x4*>(e_c + cb), vc1 = *reinterpret_cast<const f32x4*>(e_c + cb + 4);
          const float fc[8] = {vc0[0], vc0[1], vc0[2], vc0[3], vc1[0], vc1[1], vc1[2], vc1[3]};
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= fc[e];
        }
        if constexpr (RES) {
          const uint32_t rw[4] = {rv[mt][0], rv[mt][1], rv[mt][2], rv[mt][3]};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[2 * e] += __uint_as_float(rw[e] << 16);
            v[2 * e + 1] += __uint_as_float(rw[e] & 0xffff0000u);
          }
        }
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (bf16)v[e];
        // rows past the panel end hold copies of its last row: same value, same address
        const int prow = min(wm * (BM / WM) + mt * 16 + fr, mlast);
        if (g.store_mode == STORE_CB16) {   // channel-blocked: 16-channel block cb >> 4, 32-byte pixel rows
          if (!(g.dbg & 1)) pn_gstore(reinterpret_cast<bf16*>(g.out) + (((int64_t)(cb >> 4) * g.cb_px + P.m0 + prow) << 4) + (cb & 15), o);
        } else if (!(g.dbg & 1)) {
          pn_gstore(pob + (prow * (int)g.ldo + cb), o);
        }
      }
      PN_STAMP();
    }
  }
#undef PN_STAMP
  pn_vmwait<0>();
}

static size_t pn_lds_bytes(int bm, int kp, int N, bool scale) {
  return (size_t)2 * bm * kp * 2 + (size_t)(kp / 8) * sizeof(PnSrc) + (size_t)N * 4 * (scale ? 2 : 1);
}

// waves along N: 8 (one 256-channel tile row of waves, MT = BM / 16) unless the residual tile
// would not fit the registers next to 8 accumulator tiles
static int pn_wn(int N, bool res) { return (N % 256 == 0 && !res) ? 8 : (N % 128 == 0 ? 4 : 2); }

bool gemm_pn_ok(const GemmArgs& g) {
  if (g.a.cb_px) return false;                   // channel-blocked operand: 2-D tiled kernel only
  if (!g.allow_pn || g.conv3) return false;
  if (g.store_mode == STORE_CB16) {
    if (g.res || g.offo || g.N % 16 || g.cb_px != g.M || g.scale) return false;
  } else if (g.store_mode != STORE_NHWC) {
    return false;
  }
  const int K = g.a.Ktot;
  if (K != 64 && K != 128 && K != 256 && K != 384 && K != 512) return false;
  if (g.N % 64 || g.N > 8192 || g.ldw % 8 || g.ldo % 8 || g.offo % 8) return false;
  const int bm = K <= 256 ? 128 : 64;
  if (bm * g.ldo >= ((int64_t)1 << 31)) return false;                   // 32-bit in-panel offsets
  if (g.res && (g.ldr % 8 || g.offr % 8 || bm * g.ldr >= ((int64_t)1 << 31))) return false;
  if (pn_lds_bytes(bm, K, g.N, g.scale != nullptr) > 160 * 1024) return false;
  if (g.HW < bm) return false;                      // a panel spans at most two images
  if (g.M >= ((int64_t)1 << 31) - 1024) return false;
  // the BM / WM pixel rows of a wave must be a multiple of 16 (MT >= 1)
  if (bm / (PN_WAVES / pn_wn(g.N, g.res != nullptr)) < 16) return false;
  int kb = 0;
  for (int j = 0; j < g.a.n; ++j) {
    const SrcDesc& s = g.a.s[j];
    if (s.K % 8 || s.ld % 8 || s.off % 8 || reinterpret_cast<uintptr_t>(s.base) % 16) return false;
    kb += s.K;
  }
  return kb == K && reinterpret_cast<uintptr_t>(g.out) % 16 == 0 && reinterpret_cast<uintptr_t>(g.w) % 16 == 0 &&
         (!g.res || reinterpret_cast<uintptr_t>(g.res) % 16 == 0);
}

template <int BM, int KP, int WN>
static void launch_pn(const GemmArgs& g, hipStream_t st) {
  const int64_t np = g.wstride ? (g.M / g.HW) * ((g.HW + BM - 1) / BM) : (g.M + BM - 1) / BM;
  static const int ncu = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n;
  }();
  const int grid = (int)std::min<int64_t>(np, ncu);   // one block per CU (2 panel buffers of LDS)
  const size_t lds = pn_lds_bytes(BM, KP, g.N, g.scale != nullptr);
  auto kern = g.res ? gemm_pn_kernel<BM, KP, WN, true> : gemm_pn_kernel<BM, KP, WN, false>;
  static bool attr_set = false;        // per instantiation: allow the full 160 KB of LDS
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_pn_kernel<BM, KP, WN, true>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_pn_kernel<BM, KP, WN, false>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * PN_WAVES), lds, st, g, (int)np);
}

template <int BM, int KP>
static void launch_pn_wn(const GemmArgs& g, hipStream_t st) {
  const int wn = pn_wn(g.N, g.res != nullptr);
  if constexpr (BM / (PN_WAVES / 8) >= 16) { if (wn == 8) { launch_pn<BM, KP, 8>(g, st); return; } }
  if constexpr (BM / (PN_WAVES / 4) >= 16) { if (wn == 4) { launch_pn<BM, KP, 4>(g, st); return; } }
  if constexpr (BM / (PN_WAVES / 2) >= 16) { if (wn == 2) { launch_pn<BM, KP, 2>(g, st); return; } }
}

void launch_gemm_pn(const GemmArgs& g, hipStream_t st) {
  switch (g.a.Ktot) {
    case 64: launch_pn_wn<128, 64>(g, st); break;
    case 128: launch_pn_wn<128, 128>(g, st); break;
    case 256: launch_pn_wn<128, 256>(g, st); break;
    case 384: launch_pn_wn<64, 384>(g, st); break;
    default: launch_pn_wn<64, 512>(g, st); break;
  }
}


// ============================================================================================
// "ar" kernel: A-resident, one panel per block (not persistent). For the projections where the
// persistent pn kernel cannot amortise its start-up or does not fit two panels: the latent level
// (M = 32640 pixels: two panels per CU in all) and K = 640 / 1280 (L3 GFFW project_out, latent
// project_out, the CHM / FHR five-source W_eff GEMM). Measured against hipBLASLt in tools/kbench.
//   * a 256-thread block owns a BM-pixel panel; the whole BM x K panel goes HBM -> LDS by LDS-DMA
//     in one burst (<= 80 KB, XOR-swizzled chunks as in pn), so two blocks share a CU and one
//     block's MFMA sweep overlaps the other's panel load;
//   * the block then sweeps all N output channels in passes of 4 x CPW: each wave owns CPW
//     channels x all BM pixels, W fragments stream from L2 through a register ring D K-steps deep
//     that wraps into the next pass; the pass's residual and epilogue vectors are in flight across
//     its K loop;
//   * same permuted W rows as pn (lane = 8 consecutive channels of one pixel): epilogue
//     acc + (W.b_ln + bias) (+ residual), one 16-byte store per lane, pixel row and 32 channels;
//   * LayerNorm (single source): statistics and normalisation of the panel rows in LDS, as pn.
// Eligible: bf16, NHWC store, no 3x3 / GELU / scale, K in {256, 512, 640, 1280}, N % (4 CPW) == 0.
// ============================================================================================
template <int BM, int KP, int NTW, bool RES>
__global__ __launch_bounds__(256, 2) void gemm_ar_kernel(GemmArgs g) {
  constexpr int CPR = KP / 8, KS = KP / 32, MT = BM / 16, CPW = NTW * 16, CPP = 4 * CPW, NG = NTW / 2;
  constexpr int PANEL = BM * KP * 2, NDMA = PANEL / 4096, TPR = 256 / BM;
  constexpr int D = 4;
  static_assert(PANEL % 4096 == 0 && KS % D == 0 && NTW % 2 == 0 && MT >= 1 && (CPR < 16 || CPR % 16 == 0) &&
                    CPR % TPR == 0, "ar geometry");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const PnPanel P = pn_panel<BM>(g, blockIdx.x);
  const int rmax = (int)(P.mlim - P.m0) - 1;

  // ---- the panel: LDS chunk q = row q / CPR, position q % CPR, holding k-chunk pos ^ swz(row);
  // rows past the end of M repeat the last row. Source of a chunk by a select scan (<= 5 sources).
#pragma unroll
  for (int i = 0; i < NDMA; ++i) {
    const int q = (i * 4 + wid) * 64 + lane, lr = q / CPR, r = min(lr, rmax);
    const int k = ((q % CPR) ^ pn_swz<CPR>(lr)) * 8;
    const bf16* base = reinterpret_cast<const bf16*>(g.a.s[0].base) + g.a.s[0].off;
    int64_t ld = g.a.s[0].ld;
    int smul = g.a.s[0].img_mul, sadd = g.a.s[0].img_add, kb = 0, kbj = g.a.s[0].K;
#pragma unroll
    for (int s = 1; s < TURTLE_MAX_SRC; ++s) {
      const bool hit = s < g.a.n && k >= kbj;
      base = hit ? reinterpret_cast<const bf16*>(g.a.s[s].base) + g.a.s[s].off : base;
      ld = hit ? g.a.s[s].ld : ld;
      smul = hit ? g.a.s[s].img_mul : smul;
      sadd = hit ? g.a.s[s].img_add : sadd;
      kb = hit ? kbj : kb;
      kbj += s < g.a.n ? g.a.s[s].K : 0;
    }
    int pp = P.p0 + r, img = P.img0;
    if (pp >= g.HW) { pp -= g.HW; ++img; }
    pn_dma16(base + ((int64_t)(img * smul + sadd) * g.HW + pp) * ld + (k - kb), lds_base + (i * 4 + wid) * 1024);
  }
  pn_vmwait<0>();
  __syncthreads();

  if (g.ln) {   // LayerNorm of the panel rows in place (TPR threads per row), as pn
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    const bf16x2 one2 = __builtin_bit_cast(bf16x2, 0x3F803F80u);
    constexpr int CH = CPR / TPR;
    const int lr = tid / TPR, lh = tid % TPR;
    char* row = smem + lr * (KP * 2);
    uint4 xs[CH];
    float ls = 0.f, lq = 0.f;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      xs[j] = *reinterpret_cast<const uint4*>(row + (lh * CH + ((j + lr * TPR + lh) % CH)) * 16);
      const uint32_t w[4] = {xs[j].x, xs[j].y, xs[j].z, xs[j].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bf16x2 v2 = __builtin_bit_cast(bf16x2, w[e]);
        ls = __builtin_amdgcn_fdot2_f32_bf16(v2, one2, ls, false);
        lq = __builtin_amdgcn_fdot2_f32_bf16(v2, v2, lq, false);
      }
    }
#pragma unroll
    for (int o = 1; o < TPR; o <<= 1) { ls += __shfl_xor(ls, o, 64); lq += __shfl_xor(lq, o, 64); }
    const float mu = ls / KP, rs = rsqrtf(fmaxf(lq / KP - mu * mu, 0.f) + 1e-5f), nm = g.ln_s ? -mu * rs : 0.f;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const uint32_t w[4] = {xs[j].x, xs[j].y, xs[j].z, xs[j].w};
      uint32_t o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float a = fmaf(__uint_as_float(w[e] << 16), rs, nm), b = fmaf(__uint_as_float(w[e] & 0xffff0000u), rs, nm);
        typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
        o[e] = __builtin_bit_cast(uint32_t, bf2{(bf16)a, (bf16)b});
      }
      *reinterpret_cast<uint4*>(row + (lh * CH + ((j + lr * TPR + lh) % CH)) * 16) = uint4{o[0], o[1], o[2], o[3]};
    }
    __syncthreads();
  }

  // lane's W row of n-tile t: channel pass * CPP + wid * CPW + 32 (t / 2) + 8 (fr / 4) + 4 (t % 2) + fr % 4
  const int64_t ldw = g.ldw;
  const bf16* wl = P.w + (int64_t)(wid * CPW + (fr >> 2) * 8 + (fr & 3)) * ldw + fq * 8;
  bf16x8 wb[D][NTW];
  auto load_w = [&](const bf16* wp, int kstep, int slot) {
#pragma unroll
    for (int t = 0; t < NTW; ++t)
      wb[slot][t] = *reinterpret_cast<const bf16x8*>(wp + (int64_t)((t >> 1) * 32 + (t & 1) * 4) * ldw + kstep * 32);
  };
  const int npass = g.N / CPP;
#pragma unroll
  for (int j = 0; j < D; ++j) load_w(wl, j, j);
  const bf16* prb = RES ? reinterpret_cast<const bf16*>(g.res) + P.m0 * g.ldr + g.offr : nullptr;
  bf16* pob = reinterpret_cast<bf16*>(g.out) + P.m0 * g.ldo + g.offo;
  const float* vt = g.ln_t ? g.ln_t : g.zeros;
  const float* vb = g.bias ? g.bias : g.zeros;

  for (int pass = 0; pass < npass; ++pass) {
    const bf16* wcur = wl + (int64_t)pass * CPP * ldw;
    const bf16* wnx = pass + 1 < npass ? wcur + (int64_t)CPP * ldw : wcur;
    const int cb = pass * CPP + wid * CPW + fq * 8;   // + 32 j: the lane's 8 consecutive channels of group j
    u32x4 rv[RES ? MT : 1][NG];
    if constexpr (RES) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int j = 0; j < NG; ++j)
          rv[mt][j] = *reinterpret_cast<const u32x4*>(prb + (min(mt * 16 + fr, rmax) * (int)g.ldr + cb + 32 * j));
    }
    f32x4 tb[NG][2];
#pragma unroll
    for (int j = 0; j < NG; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(vt + cb + 32 * j + 4 * h);
        const f32x4 b = *reinterpret_cast<const f32x4*>(vb + cb + 32 * j + 4 * h);
        tb[j][h] = a + b;
      }
    f32x4 acc[MT][NTW];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int t = 0; t < NTW; ++t) acc[mt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 xf[MT];
    auto read_x = [&](int ks, int mt) {
      const int r = mt * 16 + fr;
      const int c = (ks * 4 + fq) ^ pn_swz<CPR>(r);
      xf[mt] = *reinterpret_cast<const bf16x8*>(smem + r * (KP * 2) + c * 16);
    };
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) read_x(0, mt);
    static_for<KS>([&](auto ksc) {
      constexpr int ks = decltype(ksc)::value;
      constexpr int slot = ks % D;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
        for (int t = 0; t < NTW; ++t) acc[mt][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[slot][t], xf[mt], acc[mt][t], 0, 0, 0);
        if constexpr (ks + 1 < KS) read_x(ks + 1, mt);
      }
      if constexpr (ks + D < KS) load_w(wcur, ks + D, slot);
      else load_w(wnx, ks + D - KS, slot);
      __builtin_amdgcn_sched_barrier(0);
    });
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int j = 0; j < NG; ++j) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = acc[mt][2 * j + (e >> 2)][e & 3] + tb[j][e >> 2][e & 3];
        if constexpr (RES) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[2 * e] += __uint_as_float(rv[mt][j][e] << 16);
            v[2 * e + 1] += __uint_as_float(rv[mt][j][e] & 0xffff0000u);
          }
        }
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (bf16)v[e];
        pn_gstore(pob + (min(mt * 16 + fr, rmax) * (int)g.ldo + cb + 32 * j), o);
      }
  }
  pn_vmwait<0>();
}

struct ArCfg { int bm, ntw; };
static ArCfg ar_cfg(int K) {
  switch (K) {
    case 256: return {128, 2};
    case 512: return {64, 4};
    case 640: return {64, 4};
    case 1280: return {32, 4};
    default: return {0, 0};
  }
}

bool gemm_ar_ok(const GemmArgs& g) {
  if (g.a.cb_px) return false;                   // channel-blocked operand: 2-D tiled kernel only
  if (!g.allow_ar || g.conv3 || g.store_mode != STORE_NHWC || g.gelu || g.scale) return false;
  const ArCfg c = ar_cfg(g.a.Ktot);
  if (!c.bm || g.N % (64 * c.ntw) || g.N > 8192) return false;
  if (g.ldw % 8 || g.ldo % 8 || g.offo % 8) return false;
  if (c.bm * g.ldo >= ((int64_t)1 << 31) || g.M >= ((int64_t)1 << 31) - 1024) return false;
  if (g.res && (g.ldr % 8 || g.offr % 8 || c.bm * g.ldr >= ((int64_t)1 << 31))) return false;
  if (g.HW < c.bm) return false;                    // a panel spans at most two images
  if (g.ln && g.a.n != 1) return false;
  int kb = 0;
  for (int j = 0; j < g.a.n; ++j) {
    const SrcDesc& s = g.a.s[j];
    if (s.K % 8 || s.ld % 8 || s.off % 8 || reinterpret_cast<uintptr_t>(s.base) % 16) return false;
    kb += s.K;
  }
  return kb == g.a.Ktot && reinterpret_cast<uintptr_t>(g.out) % 16 == 0 && reinterpret_cast<uintptr_t>(g.w) % 16 == 0 &&
         (!g.res || reinterpret_cast<uintptr_t>(g.res) % 16 == 0);
}

template <int BM, int KP, int NTW>
static void launch_ar(const GemmArgs& g, hipStream_t st) {
  const int64_t np = g.wstride ? (g.M / g.HW) * ((g.HW + BM - 1) / BM) : (g.M + BM - 1) / BM;
  constexpr size_t lds = (size_t)BM * KP * 2;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_ar_kernel<BM, KP, NTW, true>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_ar_kernel<BM, KP, NTW, false>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  auto kern = g.res ? gemm_ar_kernel<BM, KP, NTW, true> : gemm_ar_kernel<BM, KP, NTW, false>;
  hipLaunchKernelGGL(kern, dim3((unsigned)np), dim3(256), lds, st, g);
}

void launch_gemm_ar(const GemmArgs& g, hipStream_t st) {
  switch (g.a.Ktot) {
    case 256: launch_ar<128, 256, 2>(g, st); break;
    case 512: launch_ar<64, 512, 4>(g, st); break;
    case 640: launch_ar<64, 640, 4>(g, st); break;
    default: launch_ar<32, 1280, 4>(g, st); break;
  }
}

}  // namespace turtle

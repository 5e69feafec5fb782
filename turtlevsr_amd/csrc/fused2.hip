// Row-walk block fusion of "[LN ->] pointwise -> depthwise 3x3 -> [act -> pointwise (+ residual)]"
// for bf16, input widths C in {32, 64, 96, 128} (levels 1-2 of Turtle, ~80 % of the pixels):
//
//   F_GATE   GatedFeedForward  LN -> project_in (c->2h) -> dwconv -> gelu(x1)*x2 -> project_out + x
//            (turtle_t1_arch.py:159-178, 804-811)
//   F_GELU   ReducedAttn       LN -> conv1 (+b) -> conv2 dw (+b) -> gelu -> conv3 (+b) * beta + x
//            (turtle_t1_arch.py:704-742)
//   F_DWONLY [LN ->] pointwise -> dw 3x3, stored (qkv / SAB qk,v / CHM kv inputs, 555-557, 649, 674-684)
//
// Geometry. A block owns an output tile of 14 columns x R rows. Its haloed input (16 columns x R+2
// rows) sits in LDS raw (bf16). GEMM1 runs one image ROW of 16 haloed pixels at a time as the
// MFMA B operand, so a 16x16 accumulator holds, per lane, 4 consecutive hidden channels of ONE pixel
// (pixel = lane & 15, channels 4 (lane >> 4) ..): the x-neighbours of the depthwise stencil are the
// neighbouring lanes of the same 16-lane DPP row (row_shr:1 / row_shl:1), the y-neighbours are the
// previous / next rows the wave has just produced (a 3-row register window). The depthwise conv
// therefore never touches LDS; lanes 0 and 15 are the x-halo and produce no output.
//
// Work split. The hidden channels are cut into 16-channel "units" dealt round-robin to the NW waves;
// a wave walks its unit down all R+2 rows (GEMM1 row -> LN epilogue -> window -> depthwise row).
// The gate runs the x1 unit first (gelu(x1) parked in the G tile), then the x2 unit (G *= x2).
// GEMM2 (G [pixels][hidden] from LDS as the B operand, W2 fragments from L2) runs once per pass of
// UP units, each wave owning (output tile, row) pairs; its residual is the raw input tile in LDS.
//
// LayerNorm is folded algebraically: W1' = W1 diag(g) (packed), s = rowsum(W1'), t = W1 b_ln, and
// per pixel  LN-GEMM1 = rs * (W1' x) - rs * mu * s + t  (BiasFree: rs * (W1' x) + 0, s = 0).
//
// Per output pixel HBM traffic: C in (+ 2/R, 2/14 halo re-reads from L2) + C (or N1) out; the hidden
// tensor never leaves the CU.
#include "common.h"
#include "kernels.h"
#include "mma.h"

#include <type_traits>

namespace turtle {

#ifndef F2_WALK_UNROLL
#define F2_WALK_UNROLL 0   // 1: the walk's 3-row trips fully unrolled (A/B builds of tools/f2bench)
#endif

constexpr int F2_TX = 14;   // output columns per tile (16 haloed lanes)

template <int N, int I = 0, typename F>
TURTLE_DEV void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}

__device__ __attribute__((aligned(64))) uint4 g_zero_f2[8];

// d += w * src[lane -/+ 1] inside each 16-lane DPP row: one VOP2 with a DPP source (hipcc does not
// fold a separate v_mov_dpp into the FMA). Lanes whose neighbour is outside the row (0 / 15, the
// x-halo lanes) are left unchanged. The source must not be written by the immediately preceding
// VALU instruction (DPP read hazard): the walk pins each new row with an empty asm well before
// its first DPP read.
TURTLE_DEV void fmac_shr1(float& d, float src, float w) {   // src from x - 1
  asm volatile("v_fmac_f32_dpp %0, %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(src), "v"(w));
}
TURTLE_DEV void fmac_shl1(float& d, float src, float w) {   // src from x + 1
  asm volatile("v_fmac_f32_dpp %0, %1, %2 row_shl:1 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(src), "v"(w));
}

TURTLE_DEV f32x4 ld_f4(const float* p) {
  const uint4 q = ld16(p);
  return f32x4{__uint_as_float(q.x), __uint_as_float(q.y), __uint_as_float(q.z), __uint_as_float(q.w)};
}

template <int CM, int R, int HPM, int N1M>
struct F2L {
  // row pads: conflict-free ds_read_b128 fragment reads on gfx950's lane grouping for X (+32 B),
  // 2-way reads / writes for G (+16 B), checked against the MI355X LDS bank rules
  static constexpr int XP = CM * 2 + 32;                 // LDS bytes per haloed pixel
  static constexpr int NXP = (R + 2) * 16;               // haloed pixels
  static constexpr int GP = HPM * 2 + 16;                // LDS bytes per G pixel row
  static constexpr int OFF_ST = NXP * XP;                // (mu, rs) per haloed pixel
  static constexpr int OFF_TAP = OFF_ST + NXP * 8;       // depthwise taps, bf16 pairs [5][N1]
  static constexpr int OFF_VEC = OFF_TAP + 5 * N1M * 4;  // s, t + b1, dw bias: [3][N1] fp32
  static constexpr int OFF_G = OFF_VEC + 3 * N1M * 4;
  static constexpr int BYTES = OFF_G + (HPM ? R * 16 * GP : 0);
};

// MODE, input width CM (= GEMM2 width), tile rows R (multiple of 3), waves NW, hidden channels per
// pass HPM (0: dw-only), max GEMM1 width N1M, minimum waves per SIMD WPE (register budget)
// TPB tiles per block (TPB > 1: a block walks a run of consecutive tiles; the next tile's haloed
// input is fetched into registers while the current one computes, and the per-channel tables are
// loaded once per block instead of once per tile)
// TG: per-channel tables (taps, LN / bias vectors) read from global memory (L2) at the start of each
// walk instead of staged in LDS: 32 * N1M fewer LDS bytes per block, i.e. more blocks per CU
// ABL: per-phase ablations (tools/f2bench built with TURTLE_F2_ABLATIONS; 0 in the library): 1 no GELU,
// 2 no depthwise (the centre row only), 4 no GEMM2 MFMAs, 8 no LayerNorm prologue, 16 no output
// stores, 32 no GEMM1 (MFMAs and their LDS reads)
// PF (TPB > 1): the next tile's input fetched into registers during this tile's walks (true), or at
// the start of each tile (false: no registers live across the walks, the occupancy of TPB = 1)
template <int MODE, int CM, int R, int NW, int HPM, int N1M, int WPE, int TPB = 1, bool TG = false, int ABL = 0, bool PF = true>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(WPE))) void fused2_kernel(FusedArgs a) {
  using L = F2L<CM, R, HPM, TG ? 0 : N1M>;
  constexpr int KS = CM / 32;                       // GEMM1 K steps
  static_assert((R + 4) * 16 * L::XP <= L::BYTES, "the walk's last trip reads two rows past the X tile");
  constexpr int NT = NW * 64;
  __shared__ __attribute__((aligned(16))) char smem[L::BYTES];
  char* sX = smem;
  float2* sSt = reinterpret_cast<float2*>(smem + L::OFF_ST);
  uint32_t* sTap = reinterpret_cast<uint32_t*>(smem + L::OFF_TAP);
  float* sVec = reinterpret_cast<float*>(smem + L::OFF_VEC);
  char* sG = smem + L::OFF_G;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int px = lane & 15, grp = lane >> 4;
  const int N1 = a.N1;

  // ---- tiles (XCD-aware: consecutive tiles on one XCD share halo rows in its L2) ----
  const int tx_n = (a.W + F2_TX - 1) / F2_TX, ty_n = (a.H + R - 1) / R;
  const int ntiles = a.nimg * tx_n * ty_n;
  int lin = blockIdx.x;
  {
    const int nblk = gridDim.x, q = nblk / 8, r = nblk % 8, x = lin % 8, y = lin / 8;
    lin = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;
  }
  const int t_begin = lin * TPB, t_end = min(ntiles, t_begin + TPB);
  const bf16* W1 = reinterpret_cast<const bf16*>(a.w1);
  const float* zf = reinterpret_cast<const float*>(g_zero_f2);

  // ---- per-channel tables (taps, LN / bias vectors) -> LDS, once per block ----
  if constexpr (!TG) {
    // taps: bf16 pairs [5][N1] (lo = tap 2i, hi = tap 2i + 1), straight copy
    const uint32_t* tg = a.dww2;
    for (int e = tid * 4; e < 5 * N1; e += NT * 4)
      *reinterpret_cast<uint4*>(sTap + e) = ld16(tg + e);
    for (int c = tid; c < N1; c += NT) {
      const float sv = a.ln && a.ln_s ? a.ln_s[c] : 0.f;
      const float tv = (a.ln && a.ln_t ? a.ln_t[c] : 0.f) + (a.b1 ? a.b1[c] : 0.f);
      const float dv = a.dwb ? a.dwb[c] : 0.f;
      sVec[c] = sv; sVec[N1M + c] = tv; sVec[2 * N1M + c] = dv;
    }
  }
  // ---- raw haloed input tile: registers (vx) -> LDS; the LDS slot of a chunk depends on tid only ----
  constexpr int CV = CM / 8;                         // 16-byte chunks per pixel
  constexpr int NV = (L::NXP * CV + NT - 1) / NT;
  uint4 vx[NV];
  auto fetch_x = [&](int tile) {
    const bf16* X = reinterpret_cast<const bf16*>(a.x);
    const int timg = tile / (tx_n * ty_n), trem = tile - timg * tx_n * ty_n;
    const int ty0 = (trem / tx_n) * R, tx0 = (trem % tx_n) * F2_TX;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = tid + NT * i;
      const int p = e / CV, k = (e - p * CV) * 8;
      const int hr = p >> 4, hp = p & 15;
      const int y = ty0 - 1 + hr, x = tx0 - 1 + hp;
      const bool ok = p < L::NXP && y >= 0 && y < a.H && x >= 0 && x < a.W;
      const int64_t off = (((int64_t)timg * a.H + (ok ? y : 0)) * a.W + (ok ? x : 0)) * a.ldx + a.offx + k;
      vx[i] = ld16(ok ? reinterpret_cast<const void*>(X + off) : g_zero_f2);
    }
  };
  if (PF && t_begin < t_end) fetch_x(t_begin);
  for (int tile = t_begin; tile < t_end; ++tile) {
  const int img = tile / (tx_n * ty_n);
  const int trem = tile - img * tx_n * ty_n;
  const int y0 = (trem / tx_n) * R, x0 = (trem % tx_n) * F2_TX;
  if constexpr (!PF) fetch_x(tile);
  if (tile > t_begin) __syncthreads();               // every wave is done with the previous tile's LDS
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int e = tid + NT * i, p = e / CV, k = (e - p * CV) * 8;
    if (p < L::NXP) *reinterpret_cast<uint4*>(sX + p * L::XP + k * 2) = vx[i];
  }
  if (PF && tile + 1 < t_end) fetch_x(tile + 1);     // in flight during this tile's walks
  __syncthreads();
  // ---- LayerNorm of every haloed pixel in place (2 threads per pixel, shifted sums): the tile
  // becomes (x - mu) rs (BiasFree: x rs, uncentred), rounded to bf16 once - the resident-panel
  // GEMM does the same - so GEMM1's epilogue is only + (W1 b_ln + b1), carried in as the MFMA's
  // initial accumulator. The residual of GEMM2 is re-read from HBM/L2 (the raw tile is gone). ----
  if (a.ln && !(ABL & 8)) {                       // uniform: the shuffles run in whole waves
    for (int e = tid; e < 2 * L::NXP; e += NT) {
      const int p = e >> 1, h = e & 1;
      bf16* row = reinterpret_cast<bf16*>(sX + p * L::XP);
      const float sh = (float)row[0];
      constexpr int NC = CM / 16;                  // 16-byte chunks of this thread: h, h + 2, ..
      uint4 raw[NC];
      float ls = 0.f, lq = 0.f;
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        raw[j] = *reinterpret_cast<const uint4*>(row + h * 8 + 16 * j);
        Vec<bf16> v; v.from_raw(raw[j]);
#pragma unroll
        for (int i = 0; i < 8; ++i) { const float d = v.v[i] - sh; ls += d; lq = fmaf(d, d, lq); }
      }
      ls += __shfl_xor(ls, 1, 64);
      lq += __shfl_xor(lq, 1, 64);
      const float md = ls / CM;
      const float rs = rsqrtf(fmaxf(lq / CM - md * md, 0.f) + 1e-5f);
      const float c0 = a.ln_s ? -(sh + md) * rs : 0.f;
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        Vec<bf16> v; v.from_raw(raw[j]);
        uint32_t o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const f32x2 r = __builtin_elementwise_fma(f32x2{v.v[2 * i], v.v[2 * i + 1]}, f32x2{rs, rs}, f32x2{c0, c0});
          o[i] = (uint32_t)__builtin_bit_cast(unsigned short, (bf16)r.x) | ((uint32_t)__builtin_bit_cast(unsigned short, (bf16)r.y) << 16);
        }
        *reinterpret_cast<uint4*>(row + h * 8 + 16 * j) = make_uint4(o[0], o[1], o[2], o[3]);
      }
    }
  }
  __syncthreads();

  const int xg = x0 - 1 + px;
  const float colok = (xg >= 0 && xg < a.W) ? 1.f : 0.f;
  const char* xbase = sX + px * L::XP + grp * 16;

  // W1 fragments of the 16-row tile starting at r0 (global, L2-resident)
  auto load_w1 = [&](bf16x8 (&wf)[KS], int r0) {
#pragma unroll
    for (int k = 0; k < KS; ++k) wf[k] = __builtin_bit_cast(bf16x8, ld16(W1 + (int64_t)(r0 + px) * CM + k * 32 + grp * 8));
  };

  // Walk one 16-channel GEMM1 tile (W1 rows r0 .. r0+15, fragments wf) down the tile: GEMM1 row ->
  // LN / bias -> window -> depthwise row `emit(orow, d)` (d = the lane's 4 channels r0 + 4 grp ..).
  auto walk = [&](int r0, const bf16x8 (&wf)[KS], auto&& emit) {
    const int ch = r0 + grp * 4;
    f32x4 s4, tb, db;
    uint4 tp[5];
    if constexpr (TG) {                            // unconditional loads (zero line for absent vectors)
      s4 = ld_f4(a.ln && a.ln_s ? a.ln_s + ch : zf);
      tb = ld_f4(a.ln && a.ln_t ? a.ln_t + ch : zf) + ld_f4(a.b1 ? a.b1 + ch : zf);
      db = ld_f4(a.dwb ? a.dwb + ch : zf);
#pragma unroll
      for (int i = 0; i < 5; ++i) tp[i] = ld16(a.dww2 + i * N1 + ch);
    } else {
      s4 = *reinterpret_cast<const f32x4*>(sVec + ch);
      tb = *reinterpret_cast<const f32x4*>(sVec + N1M + ch);
      db = *reinterpret_cast<const f32x4*>(sVec + 2 * N1M + ch);
#pragma unroll
      for (int i = 0; i < 5; ++i) tp[i] = *reinterpret_cast<const uint4*>(sTap + i * N1 + ch);
    }
    f32x4 wt[9];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const uint4 p = tp[i];
      const uint32_t u[4] = {p.x, p.y, p.z, p.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        wt[2 * i][q] = __uint_as_float(u[q] << 16);
        if (2 * i + 1 < 9) wt[2 * i + 1][q] = __uint_as_float(u[q] & 0xffff0000u);
      }
    }
    auto load_x = [&](bf16x8 (&xf)[KS], int hr) {
#pragma unroll
      for (int k = 0; k < KS; ++k) xf[k] = *reinterpret_cast<const bf16x8*>(xbase + hr * 16 * L::XP + k * 64);
    };
    // GEMM1 of one haloed row from the bias (0 in the columns outside the image: the depthwise
    // zero-pads, and the normalised tile is 0 there)
    const f32x4 tbm = tb * colok;
    (void)s4;
    auto gemm1 = [&](const bf16x8 (&xf)[KS]) {
      f32x4 acc = tbm;
      if constexpr (!(ABL & 32)) {
#pragma unroll
        for (int k = 0; k < KS; ++k) acc = mfma(wf[k], xf[k], acc);
      }
      return acc;
    };
    // rows outside the image are 0 (depthwise zero padding): one packed multiply by a wave-uniform
    // 0 / 1 (the statistics of the pre-normalised tile are already applied)
    auto epi = [&](const f32x4& acc, int hr, float2, f32x4& w) {
      const int yg = y0 - 1 + hr;
      const float m = (yg >= 0 && yg < a.H) ? 1.f : 0.f;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x2 r = f32x2{m, m} * f32x2{acc[2 * h], acc[2 * h + 1]};
        w[2 * h] = r.x; w[2 * h + 1] = r.y;
      }
      // pin the row here in the asm order: its first DPP read (as row y+1 of the next depthwise
      // row) comes >= 24 VALU instructions later (the DPP read-after-VALU-write hazard needs 2)
#pragma unroll
      for (int q = 0; q < 4; ++q) asm volatile("" : "+v"(w[q]));
    };
    // Software pipeline per haloed row hr: MFMAs of row hr+1 (fragments read one row earlier),
    // LDS reads of row hr+2 and of row hr+1's statistics, then the VALU work of row hr
    // (epilogue + depthwise row hr-2): no LDS or MFMA latency sits in front of its consumer.
    // Register window: row hr in slot hr % 3, static inside 3-row trips after a 2-row prologue.
    f32x4 wc[3];
    bf16x8 xf[KS];
    load_x(xf, 0);
    float2 st_c = float2{0.f, 1.f};
    f32x4 acc_c = gemm1(xf);
    load_x(xf, 1);
    float2 st_n = float2{0.f, 1.f};
    f32x4 acc_n = gemm1(xf);
    load_x(xf, 2);
    epi(acc_c, 0, st_c, wc[0]);
    acc_c = acc_n; st_c = st_n;
    acc_n = gemm1(xf);
    st_n = float2{0.f, 1.f};
    load_x(xf, 3);
    epi(acc_c, 1, st_c, wc[1]);
    acc_c = acc_n; st_c = st_n;
    // 3-row trips. The last trip's GEMM1 of row R + 2 and its reads of rows R + 2, R + 3 (past the
    // X tile, inside the block's LDS tables) are computed and dropped: no branches in the body
#if F2_WALK_UNROLL
#pragma unroll
#else
#pragma nounroll
#endif
    for (int hb = 2; hb < R + 2; hb += 3) {
      static_for<3>([&](auto J) {
        constexpr int j = decltype(J)::value;
        constexpr int s2 = (2 + j) % 3, s0 = (s2 + 1) % 3, s1 = (s2 + 2) % 3;   // rows y+1, y-1, y
        const int hr = hb + j;
        acc_n = gemm1(xf);                             // row hr+1
        st_n = float2{0.f, 1.f};
        load_x(xf, hr + 2);
        epi(acc_c, hr, st_c, wc[s2]);
        acc_c = acc_n; st_c = st_n;
        float d[4];
        // tap-major, channel-minor: 4 independent accumulation chains in flight; the first row's
        // centre tap starts the chains from the bias (no copies of it)
        auto row = [&](const f32x4& w, int t0) {
          if (t0 != 0) {
#pragma unroll
            for (int q = 0; q < 4; ++q) fmac_shr1(d[q], w[q], wt[t0][q]);
          }
#pragma unroll
          for (int h = 0; h < 2; ++h) {   // centre tap: packed pairs
            const f32x2 r = __builtin_elementwise_fma(f32x2{wt[t0 + 1][2 * h], wt[t0 + 1][2 * h + 1]}, f32x2{w[2 * h], w[2 * h + 1]},
                                                      t0 == 0 ? f32x2{db[2 * h], db[2 * h + 1]} : f32x2{d[2 * h], d[2 * h + 1]});
            d[2 * h] = r.x; d[2 * h + 1] = r.y;
          }
          if (t0 == 0) {
#pragma unroll
            for (int q = 0; q < 4; ++q) fmac_shr1(d[q], w[q], wt[t0][q]);
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) fmac_shl1(d[q], w[q], wt[t0 + 2][q]);
        };
        if constexpr (!(ABL & 2)) {
          row(wc[s0], 0);
          row(wc[s1], 3);
          row(wc[s2], 6);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) d[q] = wc[s1][q];
        }
        emit(hr - 2, f32x4{d[0], d[1], d[2], d[3]});
      });
    }
  };

  const bool out_lane = px >= 1 && px <= F2_TX && xg < a.W;
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

  if constexpr (MODE == F_DWONLY) {
    const int nunit = N1 / 16;
    bf16x8 wa[KS], wb[KS];
    if (wid < nunit) load_w1(wa, wid * 16);
    for (int u = wid; u < nunit; u += 2 * NW) {
      // two units per trip with ping-pong W1 fragments: the next unit's loads fly during this walk
      auto unit = [&](int uu, const bf16x8 (&wf)[KS]) {
        const int chb = uu * 16;
        const int di = (a.ndst > 1 && chb >= a.dst[0].cend) ? ((a.ndst > 2 && chb >= a.dst[1].cend) ? 2 : 1) : 0;
        const FusedDst D = di == 0 ? a.dst[0] : (di == 1 ? a.dst[1] : a.dst[2]);
        const int cl = chb - D.cbeg + grp * 4;
        bf16* dp = reinterpret_cast<bf16*>(D.p);
        int64_t colpart, rowstep;
        int hh = 1, ws = 0;
        if (D.tok_ws > 0) {
          ws = D.tok_ws; hh = a.H / ws;
          const int ww = a.W / ws, p2 = xg / ww, jj = xg - p2 * ww;
          colpart = (int64_t)jj * ((int64_t)ws * ws * D.ccount) + (int64_t)p2 * D.ccount + cl;
          rowstep = (int64_t)ww * ws * ws * D.ccount;
        } else {
          colpart = (int64_t)xg * D.ld + D.off + cl;
          rowstep = (int64_t)a.W * D.ld;
        }
        walk(chb, wf, [&](int orow, const f32x4& d) {
          const int y = y0 + orow;
          if (!out_lane || y >= a.H) return;
          int64_t off;
          if (ws > 0) {
            const int p1 = y / hh, i = y - p1 * hh;
            off = img * D.tok_stride + i * rowstep + (int64_t)p1 * ws * D.ccount + colpart;
          } else {
            off = ((int64_t)img * a.H + y) * rowstep + colpart;
          }
          if (!(ABL & 16) || d[0] == 1.2345f) *reinterpret_cast<bf16x4*>(dp + off) = bf16x4{(bf16)d[0], (bf16)d[1], (bf16)d[2], (bf16)d[3]};
        });
      };
      if (u + NW < nunit) load_w1(wb, (u + NW) * 16);
      unit(u, wa);
      if (u + NW < nunit) {
        if (u + 2 * NW < nunit) load_w1(wa, (u + 2 * NW) * 16);
        unit(u + NW, wb);
      }
    }
  } else {
    // ---- passes of `up` units: phase A (units -> G tile), then GEMM2 into per-wave accumulators;
    // wave w owns output tiles w, w + NW, .. for every row (W2 fragments prefetched per pass) ----
    constexpr int NOT = (CM / 16 + NW - 1) / NW;     // output tiles per wave
    constexpr int KP = HPM / 32;                     // GEMM2 K steps per pass
    const int hid = a.hidden, nunit = hid / 16, up = a.up;
    const int n2t = a.N2 / 16;
    const bf16* W2 = reinterpret_cast<const bf16*>(a.w2);
    f32x4 acc2[NOT][R];
#pragma unroll
    for (int o = 0; o < NOT; ++o)
#pragma unroll
      for (int r = 0; r < R; ++r) acc2[o][r] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the walks of this wave, in order: (GEMM1 tile row r0, unit u, x1 / x2 / plain)
    constexpr int WPU = MODE == F_GATE ? 2 : 1;      // walks per unit
    auto walk_r0 = [&](int u, int h) { return MODE == F_GATE && h == 1 ? hid + u * 16 : u * 16; };
    bf16x8 wa[KS], wb[KS];
    if (wid < nunit) load_w1(wa, walk_r0(wid, 0));
    for (int u0 = 0; u0 < nunit; u0 += up) {
      const int u1 = min(nunit, u0 + up);
      bf16x8 w2f[NOT][KP];
#pragma unroll
      for (int o = 0; o < NOT; ++o)
#pragma unroll
        for (int k = 0; k < KP; ++k) {
          const int ot = wid + NW * o;
          const bool ok = ot < n2t && u0 * 16 + k * 32 < u1 * 16;
          w2f[o][k] = __builtin_bit_cast(bf16x8, ld16(ok ? reinterpret_cast<const void*>(W2 + (int64_t)(ot * 16 + px) * hid + u0 * 16 + k * 32 + grp * 8)
                                                        : reinterpret_cast<const void*>(g_zero_f2)));
        }
      if (u0 > 0) __syncthreads();                   // the previous pass's GEMM2 has read sG
      for (int u = u0 + wid; u < u1; u += NW) {
        char* gcol = sG + ((u - u0) * 16 + grp * 4) * 2;
        // next walk of this wave: (u, 1) for the gate, else the first walk of its next unit
        static_for<WPU>([&](auto H) {
          constexpr int h = decltype(H)::value;
          const bool cur_a = h == 0;
          int nu = u, nh = h + 1;
          if (nh == WPU) { nu = u + NW; nh = 0; }
          if (nu < nunit) { if (cur_a) load_w1(wb, walk_r0(nu, nh)); else load_w1(wa, walk_r0(nu, nh)); }
          auto emit_x1 = [&](int orow, const f32x4& d) {         // x1 / plain: park gelu(d)
            bf16x4 g;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const f32x2 r = (ABL & 1) ? f32x2{d[2 * h], d[2 * h + 1]} : gelu_bf16_2(f32x2{d[2 * h], d[2 * h + 1]});
              g[2 * h] = (bf16)r.x; g[2 * h + 1] = (bf16)r.y;
            }
            *reinterpret_cast<bf16x4*>(gcol + (orow * 16 + px) * L::GP) = g;
          };
          auto emit_x2 = [&](int orow, const f32x4& d) {         // x2: G = gelu(x1) * x2
            bf16x4* p = reinterpret_cast<bf16x4*>(gcol + (orow * 16 + px) * L::GP);
            const bf16x4 g1 = *p;
            bf16x4 g;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const f32x2 r = f32x2{(float)g1[2 * h], (float)g1[2 * h + 1]} * f32x2{d[2 * h], d[2 * h + 1]};
              g[2 * h] = (bf16)r.x; g[2 * h + 1] = (bf16)r.y;
            }
            *p = g;
          };
          if constexpr (h == 0) walk(walk_r0(u, 0), wa, emit_x1);
          else walk(walk_r0(u, 1), wb, emit_x2);
          if constexpr (WPU == 1) {                  // plain: the next unit's fragments are in wb
#pragma unroll
            for (int k = 0; k < KS; ++k) wa[k] = wb[k];
          }
        });
      }
      __syncthreads();
      // GEMM2 over this pass's hidden channels [u0*16, u1*16)
      const int kst = (u1 - u0) / 2;                 // 32-deep K steps (units come in pairs)
#pragma unroll
      for (int o = 0; o < NOT; ++o) {
        if (wid + NW * o >= n2t) continue;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const char* grow = sG + (r * 16 + px) * L::GP + grp * 16;
#pragma unroll
          for (int k = 0; k < KP; ++k)
            if (k < kst && !(ABL & 4)) acc2[o][r] = mfma(w2f[o][k], *reinterpret_cast<const bf16x8*>(grow + k * 64), acc2[o][r]);
        }
      }
    }
    // ---- epilogue: (acc + b2) * scale2 + x (re-read from L2), 4 consecutive channels per lane ----
    bf16* out = reinterpret_cast<bf16*>(a.out);
#pragma unroll
    for (int o = 0; o < NOT; ++o) {
      const int ot = wid + NW * o;
      if (ot >= n2t) continue;
      const int ch = ot * 16 + grp * 4;
      const f32x4 b = ld_f4(a.b2 ? a.b2 + ch : zf);
      const f32x4 sc = a.scale2 ? ld_f4(a.scale2 + ch) : f32x4{1.f, 1.f, 1.f, 1.f};
      const bf16* xres = reinterpret_cast<const bf16*>(a.x);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int y = y0 + r;
        // residual = the block input (res == x, ldx == C: fused2_ok), clamped address off-image
        const bool rin = out_lane && y < a.H;
        const bf16x4 xr = *reinterpret_cast<const bf16x4*>(
            xres + (rin ? (((int64_t)img * a.H + y) * a.W + xg) * a.ldx + ch : (int64_t)0));
        bf16x4 ov;
#pragma unroll
        for (int q = 0; q < 4; ++q) ov[q] = (bf16)fmaf(acc2[o][r][q] + b[q], sc[q], (float)xr[q]);
        if (out_lane && y < a.H && (!(ABL & 16) || (float)ov[0] == 1.2345f))
          *reinterpret_cast<bf16x4*>(out + (((int64_t)img * a.H + y) * a.W + xg) * a.ldo + a.offo + ch) = ov;
      }
    }
  }
  }   // tile loop
}

// (MODE, C) -> (tile rows, waves, hidden per pass); units per pass chosen so every wave of a pass
// gets the same number of units
template <int MODE, int CM, int R, int NW, int HPM, int WPE, int TPB = 1, bool TG = false, int ABL = 0, bool PF = true>
static void f2_launch(const FusedArgs& a0, hipStream_t st) {
  FusedArgs a = a0;
  a.up = HPM / 16;
  // widest GEMM1 the per-channel tables hold: 2 int(2.5 C) (gate), 2C (ReducedAttn), 6C (CHM
  // [qk | v | qkv])
  constexpr int N1M = MODE == F_GATE ? 5 * CM : (MODE == F_GELU ? 2 * CM : 6 * CM);
  const int64_t tiles = (int64_t)a.nimg * ((a.H + R - 1) / R) * ((a.W + F2_TX - 1) / F2_TX);
  const int64_t blocks = (tiles + TPB - 1) / TPB;
  hipLaunchKernelGGL((fused2_kernel<MODE, CM, R, NW, HPM, N1M, WPE, TPB, TG, ABL, PF>), dim3((unsigned)blocks), dim3(NW * 64), 0, st, a);
}

bool fused2_ok(const FusedArgs& a) {
  if ((a.C != 64 && a.C != 128) || a.N1 % 16 || !a.dww2) return false;
  const int n1max = a.mode == F_GATE ? 5 * a.C : (a.mode == F_GELU ? 2 * a.C : 6 * a.C);
  if (a.N1 > n1max) return false;
  if (a.mode == F_DWONLY) return a.ndst >= 1;
  if (a.N2 % 16 || a.N2 > 128 || a.N2 != a.C) return false;
  if (a.res != a.x || a.ldx != a.C || a.offx != 0) return false;   // residual = the block input
  if (a.mode == F_GATE) return a.hidden % 32 == 0 && a.N1 == 2 * a.hidden;
  return a.hidden % 32 == 0 && a.N1 == a.hidden;
}

// Configurations: tile rows R (a multiple of 3: window slots), hidden channels per pass HPM,
// minimum waves per SIMD WPE. `a.dbg` (tools/f2bench only; 0 in the product path) selects an
// alternative configuration for the same shape.
#ifdef TURTLE_F2_ABLATIONS
// the default configuration of each shape family with ablation bits `abl` (a.dbg >> 8)
template <int ABL>
static void f2_abl(const FusedArgs& a, hipStream_t st) {
  if (a.mode == F_DWONLY) {
    if (a.C == 64) f2_launch<F_DWONLY, 64, 12, 4, 0, 4, 1, false, ABL>(a, st);
    else f2_launch<F_DWONLY, 128, 9, 4, 0, 4, 1, false, ABL>(a, st);
  } else if (a.mode == F_GATE) {
    if (a.C == 64) f2_launch<F_GATE, 64, 6, 4, 64, 3, 1, false, ABL>(a, st);
    else f2_launch<F_GATE, 128, 6, 4, 64, 2, 1, false, ABL>(a, st);
  } else {
    if (a.C == 64) f2_launch<F_GELU, 64, 6, 4, 128, 3, 1, false, ABL>(a, st);
    else f2_launch<F_GELU, 128, 9, 4, 64, 2, 1, false, ABL>(a, st);
  }
}
#endif

// the default configuration of each shape family walking TPB consecutive tiles per block, each
// tile's input fetched at its start (variants 10 / 11 of tools/f2bench)
template <int TPB>
static void f2_runs(const FusedArgs& a, hipStream_t st) {
  if (a.mode == F_DWONLY) {
    if (a.C == 64) f2_launch<F_DWONLY, 64, 12, 4, 0, 4, TPB, false, 0, false>(a, st);
    else f2_launch<F_DWONLY, 128, 9, 4, 0, 4, TPB, false, 0, false>(a, st);
  } else if (a.mode == F_GATE) {
    if (a.C == 64) f2_launch<F_GATE, 64, 6, 4, 64, 3, TPB, false, 0, false>(a, st);
    else f2_launch<F_GATE, 128, 6, 4, 64, 2, TPB, false, 0, false>(a, st);
  } else {
    if (a.C == 64) f2_launch<F_GELU, 64, 6, 4, 128, 3, TPB, false, 0, false>(a, st);
    else f2_launch<F_GELU, 128, 9, 4, 64, 2, TPB, false, 0, false>(a, st);
  }
}

void launch_fused2(const FusedArgs& a, hipStream_t st) {
  // defaults (v = 0) are the fastest measured per shape family on MI355X (tools/f2bench, 1080p);
  // v = 1..5 are the alternatives of the last sweep (profiles/r02h_f2bench_sweep.log)
  const int v = a.dbg & 255;
  if (v == 10) { f2_runs<2>(a, st); return; }
  if (v == 11) { f2_runs<4>(a, st); return; }
#ifdef TURTLE_F2_ABLATIONS
  switch (a.dbg >> 8) {
    case 0: break;
    case 1: f2_abl<1>(a, st); return;
    case 2: f2_abl<2>(a, st); return;
    case 4: f2_abl<4>(a, st); return;
    case 8: f2_abl<8>(a, st); return;
    case 16: f2_abl<16>(a, st); return;
    case 32: f2_abl<32>(a, st); return;
    case 3: f2_abl<3>(a, st); return;
    case 7: f2_abl<7>(a, st); return;
    case 39: f2_abl<39>(a, st); return;
    case 63: f2_abl<63>(a, st); return;
    default: return;
  }
#endif
  if (a.mode == F_DWONLY) {
    if (a.C == 64) {
      switch (v) {
        case 1: f2_launch<F_DWONLY, 64, 15, 4, 0, 4>(a, st); break;
        case 2: f2_launch<F_DWONLY, 64, 9, 4, 0, 4>(a, st); break;
        case 3: f2_launch<F_DWONLY, 64, 18, 4, 0, 4>(a, st); break;
        case 4: f2_launch<F_DWONLY, 64, 21, 4, 0, 3>(a, st); break;
        case 5: f2_launch<F_DWONLY, 64, 15, 4, 0, 4, 2>(a, st); break;
        default:
          // N1 <= 192 (qkv / the CHM kv over its aligned frames): taller tiles, 3 waves per SIMD (L1 kv x3
          // 905 -> 831 us, qkv unchanged: profiles/r05r_f2bench_sweep.log); wider maps keep R = 12
          if (a.N1 <= 192) f2_launch<F_DWONLY, 64, 21, 4, 0, 3>(a, st);
          else f2_launch<F_DWONLY, 64, 12, 4, 0, 4>(a, st);
      }
    } else {
      switch (v) {
        case 1: f2_launch<F_DWONLY, 128, 6, 4, 0, 4>(a, st); break;
        case 2: f2_launch<F_DWONLY, 128, 12, 4, 0, 3>(a, st); break;
        case 3: f2_launch<F_DWONLY, 128, 6, 4, 0, 3>(a, st); break;
        case 4: f2_launch<F_DWONLY, 128, 15, 4, 0, 2>(a, st); break;
        case 5: f2_launch<F_DWONLY, 128, 9, 4, 0, 3>(a, st); break;
        default: f2_launch<F_DWONLY, 128, 9, 4, 0, 4>(a, st);
      }
    }
  } else if (a.mode == F_GATE) {
    if (a.C == 64) {
      switch (v) {
        case 1: f2_launch<F_GATE, 64, 9, 4, 64, 3>(a, st); break;
        case 2: f2_launch<F_GATE, 64, 12, 4, 64, 2>(a, st); break;
        case 3: f2_launch<F_GATE, 64, 9, 4, 64, 3, 4>(a, st); break;   // 4 tiles per block, next tile prefetched
        case 6: f2_launch<F_GATE, 64, 6, 4, 64, 3, 1, true>(a, st); break;   // tables from L2 (spills: 924 us)
        case 7: f2_launch<F_GATE, 64, 6, 5, 160, 2>(a, st); break;   // 5 waves, one pass (10 units: 2 per wave)
        case 8: f2_launch<F_GATE, 64, 6, 5, 160, 3>(a, st); break;
        case 4: f2_launch<F_GATE, 64, 6, 4, 64, 4>(a, st); break;
        case 5: f2_launch<F_GATE, 64, 3, 4, 64, 4>(a, st); break;
        default: f2_launch<F_GATE, 64, 6, 4, 64, 3>(a, st);           // 46 KB: 3 blocks per CU
      }
    } else {
      switch (v) {
        case 1: f2_launch<F_GATE, 128, 3, 4, 64, 3>(a, st); break;
        case 2: f2_launch<F_GATE, 128, 3, 4, 128, 2>(a, st); break;
        case 3: f2_launch<F_GATE, 128, 6, 4, 64, 3>(a, st); break;
        case 4: f2_launch<F_GATE, 128, 9, 4, 64, 2>(a, st); break;
        case 5: f2_launch<F_GATE, 128, 3, 4, 64, 2>(a, st); break;
        default: f2_launch<F_GATE, 128, 6, 4, 64, 2>(a, st);
      }
    }
  } else {
    if (a.C == 64) {
      switch (v) {
        case 1: f2_launch<F_GELU, 64, 9, 4, 64, 3>(a, st); break;
        case 2: f2_launch<F_GELU, 64, 6, 4, 64, 3>(a, st); break;
        case 3: f2_launch<F_GELU, 64, 6, 4, 64, 4>(a, st); break;
        case 4: f2_launch<F_GELU, 64, 9, 4, 128, 2>(a, st); break;
        case 5: f2_launch<F_GELU, 64, 3, 4, 64, 4>(a, st); break;
        default: f2_launch<F_GELU, 64, 6, 4, 128, 3>(a, st);
      }
    } else {
      switch (v) {
        case 1: f2_launch<F_GELU, 128, 3, 4, 64, 3>(a, st); break;
        case 2: f2_launch<F_GELU, 128, 3, 4, 128, 2>(a, st); break;
        case 3: f2_launch<F_GELU, 128, 6, 4, 64, 3>(a, st); break;
        case 4: f2_launch<F_GELU, 128, 6, 4, 64, 2>(a, st); break;
        case 5: f2_launch<F_GELU, 128, 3, 4, 64, 4>(a, st); break;
        default: f2_launch<F_GELU, 128, 9, 4, 64, 2>(a, st);
      }
    }
  }
}

}  // namespace turtle

// Tile-resident pointwise -> depthwise 3x3 (-> gate) at input width 256 ("tilepd" kernel): the
// first half of a level-3 GatedFeedForward and the qkv -> qkv_dwconv of a level-3 channel
// attention, without their hidden maps ever reaching HBM:
//
//   GATE  G[p][c] = gelu(dw(H)[p][c]) * dw(H)[p][hid + c]       (turtle_t1_arch.py:171-176)
//   DW    Q[p][c] = dw(H)[p][c]                                 (qkv_dwconv, 684-686)
//   H     = LN(x) W1^T + b1      (LayerNorm folded: W1' = W1 diag(g), epilogue t = W1 b_ln + b1)
//
// dw = depthwise 3x3 (+ bias), zero padding of H at the image border. The GatedFeedForward's
// project_out (and the attention's W_eff) then run as a GEMM over G (Q). Against a projection GEMM
// writing the 2h-channel hidden map + a depthwise pass reading it back, this removes the hidden
// map's HBM round trip (level 3 at 1080p: 334 MB written and read per GatedFeedForward).
//
// Structure (MI355X, bf16 operands, fp32 accumulation), one 512-thread block per CU:
//   * tile = RH - 2 output rows x 14 output columns; the haloed RH x 16 input tile sits in LDS for
//     the whole block, LayerNorm-normalised in place (bf16), next to the bf16 tap table and the
//     epilogue vectors of every hidden channel;
//   * a wave owns "passes" of two 16-row GEMM1 tiles (GATE: the x1 unit and its x2 partner; DW: two
//     consecutive units) over ALL RH haloed rows: per K step of 32 the RH pixel fragments are read
//     once from LDS and feed 2 MFMAs each (16x16x32: lane = pixel x, 4 consecutive hidden channels),
//     the W1 fragments stream from L2 into registers;
//   * the depthwise then runs in registers: x-neighbours are the neighbouring lanes of the 16-lane
//     DPP row (one shifted copy per input row and direction, shared by its 3 output rows), the
//     y-neighbours are the other rows the lane already holds; lanes 0 and 15 are the x-halo. The
//     gate / GELU are packed f32 pairs; each lane stores 4 channels (8 bytes) per output pixel.
#include "common.h"
#include "kernels.h"

#include <type_traits>

namespace turtle {

__device__ __attribute__((aligned(64))) uint4 g_zero_tp[8];

constexpr int TP_TX = 14, TP_NT = 512, TP_NW = 8;

template <int CM, int RH, int N1M>
struct TPL {
  static constexpr int XP = CM * 2 + 32;                  // LDS bytes per haloed pixel (+32: conflict-free b128)
  static constexpr int NXP = RH * 16;                     // haloed pixels
  static constexpr int OFF_TAP = NXP * XP;                // bf16 taps [9][N1M]
  static constexpr int OFF_TB = OFF_TAP + 9 * N1M * 2;    // fp32 [N1M]: W1 b_ln + b1
  static constexpr int OFF_DB = OFF_TB + N1M * 4;         // fp32 [N1M]: depthwise bias
  static constexpr int BYTES = OFF_DB + N1M * 4;
  static_assert(BYTES <= 160 * 1024, "tilepd LDS budget");
};

// the 4 channels of the lane's x - 1 (shr) / x + 1 (shl) neighbour in its 16-lane DPP row; lanes
// without one (0 / 15: the x-halo lanes, whose outputs are never stored) read 0. Components are
// named one by one: hipcc (ROCm 7.2) folds a `for (q) r[q] = mov_dpp(v[q])` loop into ONE mov_dpp of
// v[0] broadcast to all four lanes of the vector
TURTLE_DEV float tp_dpp_shr(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x111, 0xf, 0xf, true));
}
TURTLE_DEV float tp_dpp_shl(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x101, 0xf, 0xf, true));
}
TURTLE_DEV f32x4 tp_shr1(const f32x4& v) { return f32x4{tp_dpp_shr(v.x), tp_dpp_shr(v.y), tp_dpp_shr(v.z), tp_dpp_shr(v.w)}; }
TURTLE_DEV f32x4 tp_shl1(const f32x4& v) { return f32x4{tp_dpp_shl(v.x), tp_dpp_shl(v.y), tp_dpp_shl(v.z), tp_dpp_shl(v.w)}; }
TURTLE_DEV f32x4 tp_fma(const f32x4& a, const f32x4& b, const f32x4& c) { return __builtin_elementwise_fma(a, b, c); }

template <int MODE, int CM, int RH, int N1M, int DBG>
__global__ __launch_bounds__(TP_NT, 1) void tilepd_kernel(TilePdArgs a) {
  using L = TPL<CM, RH, N1M>;
  constexpr int KS = CM / 32;                               // GEMM1 K steps
  constexpr int R = RH - 2;                                 // output rows per tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sX = smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int px = lane & 15, grp = lane >> 4;
  const int N1 = a.N1;

  // ---- tile (row-major over the image; consecutive tiles on one XCD share their halo rows) ----
  const int tx_n = (a.W + TP_TX - 1) / TP_TX, ty_n = (a.H + R - 1) / R;
  int lin = blockIdx.x;
  {
    const int nblk = gridDim.x, q = nblk / 8, r = nblk % 8, xx = lin % 8, yy = lin / 8;
    lin = (xx < r ? xx * (q + 1) : r * (q + 1) + (xx - r) * q) + yy;
  }
  const int img = lin / (tx_n * ty_n), trem = lin - img * tx_n * ty_n;
  const int y0 = (trem / tx_n) * R, x0 = (trem % tx_n) * TP_TX;

  // ---- per-channel tables -> LDS (bf16 taps [9][N1], GEMM1 epilogue and depthwise bias fp32) ----
  {
    const uint32_t* t16 = reinterpret_cast<const uint32_t*>(a.dww16);
    for (int e = tid; e < 9 * N1 / 8; e += TP_NT) {       // 16-byte pieces
      const int t = e / (N1 / 8), c8 = (e - t * (N1 / 8)) * 8;
      *reinterpret_cast<uint4*>(smem + L::OFF_TAP + (t * N1M + c8) * 2) = ld16(t16 + (t * N1 + c8) / 2);
    }
    float* sTb = reinterpret_cast<float*>(smem + L::OFF_TB);
    float* sDb = reinterpret_cast<float*>(smem + L::OFF_DB);
    for (int c = tid; c < N1; c += TP_NT) {
      sTb[c] = a.tb ? a.tb[c] : 0.f;
      sDb[c] = a.dwb ? a.dwb[c] : 0.f;
    }
  }
  // ---- haloed input tile -> registers -> LayerNorm in registers -> LDS (bf16). A pixel's CM / 8
  // 16-byte chunks sit in CM / 8 consecutive lanes: its statistics are a lane reduction (two
  // passes, biased variance, eps 1e-5 inside the sqrt: turtle_t1_arch.py:96-99); pixels outside the
  // image are 0 and stay 0 (the depthwise zero-pads H, whose GEMM1 epilogue is masked below) ----
  {
    constexpr int CV = CM / 8;                              // 16-byte chunks per pixel
    constexpr int PPI = TP_NT / CV;                         // pixels per iteration
    constexpr int NI = (L::NXP + PPI - 1) / PPI;
    static_assert(CV == 32 && L::NXP % PPI == 0, "one pixel per half wave");
    const bf16* X = reinterpret_cast<const bf16*>(a.x);
    const int cc = tid % CV, pq = tid / CV;
    uint4 vx[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int p = i * PPI + pq, hr = p >> 4, hp = p & 15;
      const int y = y0 - 1 + hr, x = x0 - 1 + hp;
      const bool ok = y >= 0 && y < a.H && x >= 0 && x < a.W;
      const int64_t off = (((int64_t)img * a.H + (ok ? y : 0)) * a.W + (ok ? x : 0)) * a.ldx + a.offx + cc * 8;
      vx[i] = ld16(ok ? reinterpret_cast<const void*>(X + off) : g_zero_tp);
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int p = i * PPI + pq;
      uint4 o = vx[i];
      if (a.ln && !(DBG & 8)) {
        Vec<bf16> v; v.from_raw(vx[i]);
        float sm = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) sm += v.v[e];
#pragma unroll
        for (int m = 1; m < CV; m <<= 1) sm += __shfl_xor(sm, m, 64);
        const float mu = sm * (1.f / CM);
        float sq = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) { const float d = v.v[e] - mu; sq = fmaf(d, d, sq); }
#pragma unroll
        for (int m = 1; m < CV; m <<= 1) sq += __shfl_xor(sq, m, 64);
        const float rs = rsqrtf(sq * (1.f / CM) + 1e-5f);
        const float c0 = a.centred ? -mu * rs : 0.f;
        uint32_t w[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const f32x2 r = __builtin_elementwise_fma(f32x2{v.v[2 * e], v.v[2 * e + 1]}, f32x2{rs, rs}, f32x2{c0, c0});
          w[e] = (uint32_t)__builtin_bit_cast(unsigned short, (bf16)r.x) | ((uint32_t)__builtin_bit_cast(unsigned short, (bf16)r.y) << 16);
        }
        o = make_uint4(w[0], w[1], w[2], w[3]);
      }
      *reinterpret_cast<uint4*>(sX + p * L::XP + cc * 16) = o;
    }
  }
  __syncthreads();

  // ---- tile steps: step s = GEMM1 tile (s & 1) of this wave's pass s >> 1; the MFMAs of step s
  // are issued in one basic block with the depthwise (+ gate, stores) of step s - 1, so one wave's
  // matrix work overlaps its own VALU work ----
  const int xg = x0 - 1 + px;
  const float colok = (xg >= 0 && xg < a.W) ? 1.f : 0.f;
  const bool out_col = px >= 1 && px <= TP_TX && xg < a.W;
  const char* xb = sX + px * L::XP + grp * 16;
  const bf16* W1 = reinterpret_cast<const bf16*>(a.w1);
  const int hid = MODE == TP_GATE ? N1 / 2 : N1;
  const int npass = MODE == TP_GATE ? hid / 16 : N1 / 32;
  const int np_w = (npass - wid + TP_NW - 1) / TP_NW;       // passes of this wave: u = wid + 8 j
  if (np_w <= 0) return;
  bf16* out = reinterpret_cast<bf16*>(a.out);
  // first W1 row of GEMM1 tile t of pass u
  auto row0 = [&](int u, int t) __attribute__((always_inline)) { return MODE == TP_GATE ? (t ? hid : 0) + 16 * u : 32 * u + 16 * t; };
  const int64_t rstep = (int64_t)a.W * a.ldo;

  // W1 fragments: a 4-slot ring over the K steps (two L2 loads in flight behind the step in use),
  // continuous across tiles: K step k of a tile sits in slot k % 4 (KS % 4 == 0), so the next tile's
  // first two steps - issued during this tile's last two - land in slots 0 and 1
  static_assert(KS % 4 == 0, "W1 ring slots continue across tiles");
  bf16x8 wf[4];
  auto load_w = [&](int row, int k) __attribute__((always_inline)) {
    wf[k % 4] = __builtin_bit_cast(bf16x8, ld16(W1 + (int64_t)(row + px) * CM + grp * 8 + k * 32));
  };
  // stores: 8 bytes (4 channels) per lane and output row, inline asm so that hipcc's waitcnt
  // bookkeeping sees only the W1 loads and counts them exactly (with stores in view it waits
  // vmcnt(0) for any load; the hardware retires vmcnt in issue order, so a hidden store only ever
  // lengthens a wait). The lane's column pointer is opaque to the optimiser (hoisted row pointers
  // cost spills)
  auto colptr = [&](int c) __attribute__((always_inline)) {
    bf16* p = out + (((int64_t)img * a.H + y0) * a.W + (out_col ? xg : 0)) * a.ldo + a.offo + c;
    asm volatile("" : "+v"(p));
    return p;
  };
  auto store = [&](bf16* colp, int o, const f32x4& r) __attribute__((always_inline)) {
    const uint32_t lo = (uint32_t)__builtin_bit_cast(unsigned short, (bf16)r[0]) | ((uint32_t)__builtin_bit_cast(unsigned short, (bf16)r[1]) << 16);
    const uint32_t hi = (uint32_t)__builtin_bit_cast(unsigned short, (bf16)r[2]) | ((uint32_t)__builtin_bit_cast(unsigned short, (bf16)r[3]) << 16);
    if (out_col && y0 + o - 1 < a.H && !(DBG & 4))
      asm volatile("global_store_dwordx2 %0, %1, off" : : "v"(colp + (o - 1) * rstep), "v"(make_uint2(lo, hi)) : "memory");
  };

  // One tile step, K step by K step: the MFMAs of GEMM1 tile `rowB` (all RH haloed rows, from its
  // epilogue vector - 0 outside the image) next to output row k + 1 of the depthwise of the
  // previous tile `rowA` (computed in place: accA[o - 1] <- dw(H)[o]) and its epilogue `epi`. One
  // scheduling region per K step: one wave's matrix work overlaps its own VALU work with a bounded
  // register window. The last two K steps prefetch the first two of the next tile (`next_row`)
  static_assert(R == KS, "one depthwise output row per GEMM1 K step");
  auto step = [&](auto do_gemm, int rowB, int next_row, f32x4 (&accB)[RH], auto do_dw, int rowA, f32x4 (&accA)[RH],
                  auto&& epi) __attribute__((always_inline)) {
    constexpr bool G = decltype(do_gemm)::value && (DBG & 1) == 0;
    constexpr bool D = decltype(do_dw)::value && (DBG & 2) == 0;
    if constexpr (decltype(do_gemm)::value) {
      const f32x4 tb = *reinterpret_cast<const f32x4*>(smem + L::OFF_TB + (rowB + grp * 4) * 4) * colok;
#pragma unroll
      for (int hr = 0; hr < RH; ++hr) {
        const int yg = y0 - 1 + hr;
        accB[hr] = (yg >= 0 && yg < a.H) ? tb : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    f32x4 w[9], db, lw[3], rw[3], prev;
    if constexpr (D) {
      const int ch = rowA + grp * 4;
#pragma unroll
      for (int i = 0; i < 9; ++i) {
        const uint2 q = *reinterpret_cast<const uint2*>(smem + L::OFF_TAP + (i * N1M + ch) * 2);
        w[i] = f32x4{__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xffff0000u), __uint_as_float(q.y << 16),
                     __uint_as_float(q.y & 0xffff0000u)};
      }
      db = *reinterpret_cast<const f32x4*>(smem + L::OFF_DB + ch * 4);
      lw[0] = tp_shr1(accA[0]); rw[0] = tp_shl1(accA[0]);
      lw[1] = tp_shr1(accA[1]); rw[1] = tp_shl1(accA[1]);
      prev = accA[0];                                       // raw row o - 1 (accA[o-2] is overwritten)
    }
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      if constexpr (decltype(do_gemm)::value) {
        if (k + 2 < KS) load_w(rowB, k + 2);
        else load_w(next_row, k + 2 - KS);
      }
      if constexpr (G) {
#pragma unroll
        for (int hr = 0; hr < RH; ++hr)
          accB[hr] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[k % 4], *reinterpret_cast<const bf16x8*>(xb + hr * 16 * L::XP + k * 64),
                                                           accB[hr], 0, 0, 0);
      }
      if constexpr (D) {
        const int o = k + 1, s0 = (o - 1) % 3, s1 = o % 3, s2 = (o + 1) % 3;
        lw[s2] = tp_shr1(accA[o + 1]); rw[s2] = tp_shl1(accA[o + 1]);
        f32x4 d = tp_fma(w[1], prev, db);
        d = tp_fma(w[0], lw[s0], d);
        d = tp_fma(w[2], rw[s0], d);
        d = tp_fma(w[3], lw[s1], d);
        d = tp_fma(w[4], accA[o], d);
        d = tp_fma(w[5], rw[s1], d);
        d = tp_fma(w[6], lw[s2], d);
        d = tp_fma(w[7], accA[o + 1], d);
        d = tp_fma(w[8], rw[s2], d);
        prev = accA[o];
        accA[o - 1] = d;
        epi(o, d);
      } else if constexpr (decltype(do_dw)::value) {
        epi(k + 1, accA[k + 1]);                            // ablation: no depthwise
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  f32x4 accA[RH], accB[RH];                                   // tile 0 / tile 1 of the current pass
  uint2 g1[R];                                                // GATE: gelu(dw(x1)) of the current pass, bf16
  std::true_type yes;
  std::false_type no;
  int u = wid;
  load_w(row0(u, 0), 0);
  load_w(row0(u, 0), 1);
  step(yes, row0(u, 0), row0(u, 1), accA, no, 0, accB, [](int, const f32x4&) {});
  // pass u: step 2j + 1 = GEMM1 of tile 1 || depthwise (+ GELU) of tile 0; step 2j + 2 = GEMM1 of the
  // next pass's tile 0 (last pass: none) || depthwise (+ gate) of tile 1 and the stores
  for (int j = 0; j < np_w; ++j, u += TP_NW) {
    const bool more = j + 1 < np_w;
    const int un = more ? u + TP_NW : u;                      // last pass: harmless in-range prefetches
    if constexpr (MODE == TP_GATE) {
      step(yes, row0(u, 1), row0(un, 0), accB, yes, row0(u, 0), accA, [&](int o, const f32x4& d) {
        const f32x2 q0 = gelu_bf16_2(f32x2{d[0], d[1]}), q1 = gelu_bf16_2(f32x2{d[2], d[3]});
        g1[o - 1] = make_uint2((uint32_t)__builtin_bit_cast(unsigned short, (bf16)q0.x) | ((uint32_t)__builtin_bit_cast(unsigned short, (bf16)q0.y) << 16),
                               (uint32_t)__builtin_bit_cast(unsigned short, (bf16)q1.x) | ((uint32_t)__builtin_bit_cast(unsigned short, (bf16)q1.y) << 16));
      });
    } else {
      bf16* cp = colptr(row0(u, 0) + grp * 4);
      step(yes, row0(u, 1), row0(un, 0), accB, yes, row0(u, 0), accA, [&](int o, const f32x4& d) { store(cp, o, d); });
    }
    bf16* cp = colptr((MODE == TP_GATE ? 16 * u : row0(u, 1)) + grp * 4);
    auto epi2 = [&](int o, const f32x4& d) __attribute__((always_inline)) {
      if constexpr (MODE == TP_GATE) {
        const uint2 g = g1[o - 1];
        store(cp, o, d * f32x4{__uint_as_float(g.x << 16), __uint_as_float(g.x & 0xffff0000u), __uint_as_float(g.y << 16),
                               __uint_as_float(g.y & 0xffff0000u)});
      } else {
        store(cp, o, d);
      }
    };
    if (more) step(yes, row0(un, 0), row0(un, 1), accA, yes, row0(u, 1), accB, epi2);
    else step(no, 0, 0, accA, yes, row0(u, 1), accB, epi2);
  }
}

constexpr int TP_RH = 10;

bool tilepd_ok(const TilePdArgs& a) {
  if (a.C != 256 || a.N1 <= 0 || a.N1 % 32 || a.N1 > 1536) return false;
  if (a.mode != TP_GATE && a.mode != TP_DW) return false;
  if (a.ldx % 8 || a.offx % 8 || a.ldo % 4 || a.offo % 4 || !a.dww16 || !a.w1 || !a.out || !a.x) return false;
  if (reinterpret_cast<uintptr_t>(a.x) % 16 || reinterpret_cast<uintptr_t>(a.w1) % 16 || reinterpret_cast<uintptr_t>(a.out) % 8 ||
      reinterpret_cast<uintptr_t>(a.dww16) % 16)
    return false;
  return a.H > 0 && a.W > 0 && a.nimg > 0;
}

int64_t tilepd_blocks(const TilePdArgs& a) {
  return (int64_t)a.nimg * ((a.H + TP_RH - 3) / (TP_RH - 2)) * ((a.W + TP_TX - 1) / TP_TX);
}

template <int MODE, int N1M, int DBG>
static void tp_launch(const TilePdArgs& a, hipStream_t st) {
  using L = TPL<256, TP_RH, N1M>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(tilepd_kernel<MODE, 256, TP_RH, N1M, DBG>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, L::BYTES);
    attr = true;
  }
  hipLaunchKernelGGL((tilepd_kernel<MODE, 256, TP_RH, N1M, DBG>), dim3((unsigned)tilepd_blocks(a)), dim3(TP_NT), L::BYTES, st, a);
}

template <int DBG>
static void tp_dispatch(const TilePdArgs& a, hipStream_t st) {
  if (a.mode == TP_GATE) {
    if (a.N1 > 1280) kernel_arg_error("tilepd: GATE width > 1280");
    tp_launch<TP_GATE, 1280, DBG>(a, st);
  } else if (a.N1 <= 768) {
    tp_launch<TP_DW, 768, DBG>(a, st);
  } else {
    tp_launch<TP_DW, 1536, DBG>(a, st);
  }
}

void launch_tilepd(const TilePdArgs& a, hipStream_t st) {
  if (!tilepd_ok(a)) kernel_arg_error("tilepd: arguments outside the kernel's contract");
#ifdef TURTLE_TILEPD_ABLATIONS
  // tools/tpbench only (built with the kernel source): dbg bits 1 no GEMM1, 2 no depthwise / gate,
  // 4 no stores, 8 no LayerNorm
  switch (a.dbg) {
    case 1: tp_dispatch<1>(a, st); return;
    case 2: tp_dispatch<2>(a, st); return;
    case 3: tp_dispatch<3>(a, st); return;
    case 4: tp_dispatch<4>(a, st); return;
    case 6: tp_dispatch<6>(a, st); return;
    case 7: tp_dispatch<7>(a, st); return;
    case 8: tp_dispatch<8>(a, st); return;
    default: break;
  }
#endif
  tp_dispatch<0>(a, st);
}

}  // namespace turtle

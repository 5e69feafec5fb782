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

#include <algorithm>
#include <type_traits>

namespace turtle {

__device__ __attribute__((aligned(64))) uint4 g_zero_tp[8];
// lane-private store targets of lanes without an output (x-halo, rows past the image), so every
// store of the pass loop is issued (exact vmcnt accounting) without all lanes hitting one line
constexpr int TP_SINK_BLOCKS = 256;
__device__ __attribute__((aligned(64))) uint2 g_sink_tp[TP_SINK_BLOCKS * 512];

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

// W1 fragment load and its wait, both inline asm (tilepd_kernel's pass loop counts vmcnt by hand);
// the wait redefines the fragments, so no use can be scheduled before it
TURTLE_DEV void tp_gload(bf16x8& d, const bf16* p) {
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(d) : "v"(p) : "memory");
}
template <int N>
TURTLE_DEV void tp_vmwait(bf16x8& a, bf16x8& b) {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N) : "memory");
}
// the same for the two ring slots that are live across the pass loop's back-edge (and its entry):
// those fragments must have landed before the edge, because the register allocator may copy a
// loop-carried value there - an asm load's destination still in flight would be copied half-written
// (tools/check_asm_vmem.py finds such copies; round 4's sab_avt fault was one)
template <int N>
TURTLE_DEV void tp_vmwait_ring(bf16x8 (&w)[3][2]) {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%4)" : "+v"(w[0][0]), "+v"(w[0][1]), "+v"(w[1][0]), "+v"(w[1][1]) : "n"(N) : "memory");
}

template <int MODE, int CM, int RH, int N1M, int DBG>
__global__ __launch_bounds__(TP_NT, 1) void tilepd_kernel(TilePdArgs a) {
  using L = TPL<CM, RH, N1M>;
  constexpr int KS = CM / 32;                               // GEMM1 K steps
  constexpr int R = RH - 2;                                 // output rows per tile
  constexpr int CV = CM / 8;                                // 16-byte chunks per pixel
  static_assert(KS % 4 == 0, "W1 ring slots continue across passes");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sX = smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int px = lane & 15, grp = lane >> 4;
  const int N1 = a.N1;
  // waves 4..7 (each sharing a SIMD with one of 0..3) win issue arbitration: the two waves of a SIMD
  // drift out of phase, so one's MFMA phase runs beside the other's depthwise (VALU) phase
  if (wid >= TP_NW / 2) __builtin_amdgcn_s_setprio(1);

  // W1 fragments: a 3-deep ring of K steps (see the pass loop); the first pass's first two steps are
  // issued here, so they land during the prologue
  const bf16* W1 = reinterpret_cast<const bf16*>(a.w1);
  const int hid = MODE == TP_GATE ? N1 / 2 : N1;
  const int npass = MODE == TP_GATE ? hid / 16 : N1 / 32;
  auto row0 = [&](int u, int t) __attribute__((always_inline)) { return MODE == TP_GATE ? (t ? hid : 0) + 16 * u : 32 * u + 16 * t; };
  bf16x8 wf[3][2];
  auto load_w = [&](int uu, int k) __attribute__((always_inline)) {
    const int uc = uu < npass ? uu : 0;                     // past the last pass: a harmless in-range reload
#pragma unroll
    for (int t = 0; t < 2; ++t) tp_gload(wf[k % 3][t], W1 + (int64_t)(row0(uc, t) + (lane & 15)) * CM + (lane >> 4) * 8 + k * 32);
  };
  load_w(wid, 0);
  load_w(wid, 1);

  // ---- per-channel tables -> LDS once per block (bf16 taps [9][N1], GEMM1 epilogue and depthwise
  // bias fp32) ----
  {
    const uint32_t* t16 = reinterpret_cast<const uint32_t*>(a.dww16);
    for (int e = tid; e < 9 * N1 / 8; e += TP_NT) {         // 16-byte pieces
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

  // ---- tile (row-major over the image; consecutive tiles on one XCD share their halo rows) ----
  const int tx_n = (a.W + TP_TX - 1) / TP_TX, ty_n = (a.H + R - 1) / R;
  int lin = blockIdx.x;
  {
    const int nblk = gridDim.x, q = nblk / 8, r = nblk % 8, xx = lin % 8, yy = lin / 8;
    lin = (xx < r ? xx * (q + 1) : r * (q + 1) + (xx - r) * q) + yy;
  }
  const int img = lin / (tx_n * ty_n), trem = lin - img * tx_n * ty_n;
  const int y0 = (trem / tx_n) * R, x0 = (trem % tx_n) * TP_TX;

  // ---- haloed input tile -> registers -> LayerNorm in registers -> LDS (bf16). A pixel's 32 16-byte
  // chunks are held by an aligned group of 8 lanes (chunks cc, cc + 8, cc + 16, cc + 24): its
  // statistics are an 8-lane DPP reduction (quad_perm xor 1, xor 2, then row_half_mirror), two passes
  // (biased variance, eps 1e-5 inside the sqrt: turtle_t1_arch.py:96-99); pixels outside the image
  // are 0 and stay 0 (the depthwise zero-pads H, whose GEMM1 epilogue is masked below) ----
  {
    constexpr int LPP = 8, CPL = CV / LPP, PPJ = TP_NT / LPP;   // lanes per pixel, chunks per lane, pixels per round
    constexpr int NJ = (L::NXP + PPJ - 1) / PPJ;
    static_assert(CV % LPP == 0, "chunks per lane");
    const bf16* X = reinterpret_cast<const bf16*>(a.x);
    const int cc = tid % LPP, pq = tid / LPP;
    auto sum8 = [](float v) __attribute__((always_inline)) {
      v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xf, 0xf, false));   // xor 1
      v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xf, 0xf, false));   // xor 2
      v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xf, 0xf, false));  // half mirror
      return v;
    };
    uint4 vx[NJ][CPL];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int p = j * PPJ + pq, hr = p >> 4, hp = p & 15;
      const int y = y0 - 1 + hr, x = x0 - 1 + hp;
      const bool ok = p < L::NXP && y >= 0 && y < a.H && x >= 0 && x < a.W;
      const bf16* src = X + (((int64_t)img * a.H + (ok ? y : 0)) * a.W + (ok ? x : 0)) * a.ldx + a.offx + cc * 8;
#pragma unroll
      for (int q = 0; q < CPL; ++q) vx[j][q] = ld16(ok ? reinterpret_cast<const void*>(src + q * LPP * 8) : g_zero_tp);
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int p = j * PPJ + pq;
      if (a.ln && !(DBG & 8)) {
        float sm = 0.f;
#pragma unroll
        for (int q = 0; q < CPL; ++q) {
          Vec<bf16> vv; vv.from_raw(vx[j][q]);
#pragma unroll
          for (int e = 0; e < 8; ++e) sm += vv.v[e];
        }
        const float mu = sum8(sm) * (1.f / CM);
        float sq = 0.f;
#pragma unroll
        for (int q = 0; q < CPL; ++q) {
          Vec<bf16> vv; vv.from_raw(vx[j][q]);
#pragma unroll
          for (int e = 0; e < 8; ++e) { const float d = vv.v[e] - mu; sq = fmaf(d, d, sq); }
        }
        const float rs = rsqrtf(sum8(sq) * (1.f / CM) + 1e-5f);
        const float c0 = a.centred ? -mu * rs : 0.f;
#pragma unroll
        for (int q = 0; q < CPL; ++q) {
          Vec<bf16> vv; vv.from_raw(vx[j][q]);
          uint32_t w[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const f32x2 r = __builtin_elementwise_fma(f32x2{vv.v[2 * e], vv.v[2 * e + 1]}, f32x2{rs, rs}, f32x2{c0, c0});
            w[e] = (uint32_t)__builtin_bit_cast(unsigned short, (bf16)r.x) | ((uint32_t)__builtin_bit_cast(unsigned short, (bf16)r.y) << 16);
          }
          vx[j][q] = make_uint4(w[0], w[1], w[2], w[3]);
        }
      }
      if (p < L::NXP) {
#pragma unroll
        for (int q = 0; q < CPL; ++q) *reinterpret_cast<uint4*>(sX + p * L::XP + (cc + q * LPP) * 16) = vx[j][q];
      }
    }
  }
  __syncthreads();

  // ---- passes: GEMM1 of two 16-row tiles over all RH haloed rows (each pixel fragment read once
  // from LDS feeds 2 MFMAs), then the depthwise (+ gate) and the stores ----
  const int xg = x0 - 1 + px;
  const float colok = (xg >= 0 && xg < a.W) ? 1.f : 0.f;
  const bool out_col = px >= 1 && px <= TP_TX && xg < a.W;
  const char* xb = sX + px * L::XP + grp * 16;
  bf16* out = reinterpret_cast<bf16*>(a.out);
  const int64_t pix0 = ((int64_t)img * a.H + y0) * a.W + (out_col ? xg : 0);   // output row 1 of this lane

  // W1 fragments: a 3-deep ring of K steps (two L2 loads in flight behind the step in use); the
  // first two steps of a wave's next pass are issued before the current pass's depthwise phase.
  // Every vector-memory op of the pass loop - these loads and the output stores - is inline asm in
  // a fixed program order, and each wait counts exactly the ops issued after the awaited load (the
  // hardware retires vmcnt in issue order). hipcc's own counting sees no stores and would wait for
  // a pass's stores at the next pass's first K step
  // stores per pass (unconditional: sink lanes); none in the no-store ablation, whose waits must
  // not count them (an under-waited load lands in a register hipcc has since reused)
  constexpr int NS = (DBG & 16) ? 0 : (MODE == TP_GATE ? R : 2 * R);
  bf16* sinkp = reinterpret_cast<bf16*>(g_sink_tp) + ((blockIdx.x % TP_SINK_BLOCKS) * TP_NT + tid) * 4;
  float chk = 0.f;                                          // DBG 16 only
  tp_vmwait_ring<0>(wf);                                    // loop entry: landed (see tp_vmwait_ring)
  for (int u = wid; u < npass; u += TP_NW) {
    const bool first = u == wid;
    f32x4 acc[2][RH];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const f32x4 tb = *reinterpret_cast<const f32x4*>(smem + L::OFF_TB + (row0(u, t) + grp * 4) * 4) * colok;
#pragma unroll
      for (int hr = 0; hr < RH; ++hr) {
        const int yg = y0 - 1 + hr;
        acc[t][hr] = (yg >= 0 && yg < a.H) ? tb : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      if (k + 2 < KS) load_w(u, k + 2);
      // W(k) ready: ops issued after it are W(k+1), W(k+2) (2 each) and, at k < 2 after the first
      // pass, the previous pass's NS stores (issued between W(1) and W(2))
      if (k < 2) {
        if (first) tp_vmwait<4>(wf[k % 3][0], wf[k % 3][1]);
        else tp_vmwait<4 + NS>(wf[k % 3][0], wf[k % 3][1]);
      } else if (k + 2 < KS) {
        tp_vmwait<4>(wf[k % 3][0], wf[k % 3][1]);
      } else if (k + 1 < KS) {
        tp_vmwait<2>(wf[k % 3][0], wf[k % 3][1]);
      } else {
        tp_vmwait<0>(wf[k % 3][0], wf[k % 3][1]);
      }
      __builtin_amdgcn_sched_barrier(0);                    // the L2 loads issue here, not next to their MFMAs
      if constexpr ((DBG & 1) == 0) {
        bf16x8 xf[RH];
#pragma unroll
        for (int hr = 0; hr < RH; ++hr) xf[hr] = *reinterpret_cast<const bf16x8*>(xb + hr * 16 * L::XP + k * 64);
        __builtin_amdgcn_sched_barrier(0);                  // every pixel fragment in flight before the MFMAs
#pragma unroll
        for (int hr = 0; hr < RH; ++hr) {
          acc[0][hr] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[k % 3][0], xf[hr], acc[0][hr], 0, 0, 0);
          acc[1][hr] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[k % 3][1], xf[hr], acc[1][hr], 0, 0, 0);
        }
      }
    }
    load_w(u + TP_NW, 0);                                   // next pass: its first K steps fly during the depthwise
    load_w(u + TP_NW, 1);
    __builtin_amdgcn_sched_barrier(0);
    // depthwise of tile t in place: acc[t][o - 1] <- dw(H)[output row o], o = 1 .. R
    auto dw_tile = [&](int t) __attribute__((always_inline)) {
      if constexpr ((DBG & 2) != 0) return;                 // ablation: no depthwise
      const int ch = row0(u, t) + grp * 4;
      f32x4 w[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) {
        const uint2 q = *reinterpret_cast<const uint2*>(smem + L::OFF_TAP + (i * N1M + ch) * 2);
        w[i] = f32x4{__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xffff0000u), __uint_as_float(q.y << 16),
                     __uint_as_float(q.y & 0xffff0000u)};
      }
      const f32x4 db = *reinterpret_cast<const f32x4*>(smem + L::OFF_DB + ch * 4);
      f32x4 lw[3], rw[3];                                   // x-1 / x+1 copies of rows o-1, o, o+1
      lw[0] = tp_shr1(acc[t][0]); rw[0] = tp_shl1(acc[t][0]);
      lw[1] = tp_shr1(acc[t][1]); rw[1] = tp_shl1(acc[t][1]);
      f32x4 prev = acc[t][0];                               // raw row o - 1 (acc[t][o-2] is overwritten)
#pragma unroll
      for (int o = 1; o <= R; ++o) {
        const int s0 = (o - 1) % 3, s1 = o % 3, s2 = (o + 1) % 3;
        lw[s2] = tp_shr1(acc[t][o + 1]); rw[s2] = tp_shl1(acc[t][o + 1]);
        f32x4 d = tp_fma(w[1], prev, db);
        d = tp_fma(w[0], lw[s0], d);
        d = tp_fma(w[2], rw[s0], d);
        d = tp_fma(w[3], lw[s1], d);
        d = tp_fma(w[4], acc[t][o], d);
        d = tp_fma(w[5], rw[s1], d);
        d = tp_fma(w[6], lw[s2], d);
        d = tp_fma(w[7], acc[t][o + 1], d);
        d = tp_fma(w[8], rw[s2], d);
        prev = acc[t][o];
        acc[t][o - 1] = d;
        __builtin_amdgcn_sched_barrier(0);                  // one output row per region: bounded live shifted copies
      }
    };
    // stores: 8 bytes (4 channels) per lane and output row, inline asm so that hipcc's waitcnt
    // bookkeeping sees only the loads and counts them exactly (with stores in view it waits
    // vmcnt(0) for any load; the hardware retires vmcnt in issue order, so a hidden store only ever
    // lengthens a wait). Channel-blocked output (cb_px > 0): 16-channel blocks [C / 16][cb_px][16],
    // one unit's output row is 14 pixels x 32 contiguous bytes. The column pointer is opaque to
    // the optimiser (hoisted row pointers cost spills)
    auto store_rows = [&](int c, int t, bool gate) __attribute__((always_inline)) {
      bf16* colp;
      int64_t rstep;
      if (a.cb_px) {
        colp = out + (((int64_t)(c >> 4) * a.cb_px + pix0) << 4) + (c & 15);
        rstep = (int64_t)a.W * 16;
      } else {
        colp = out + pix0 * a.ldo + a.offo + c;
        rstep = (int64_t)a.W * a.ldo;
      }
      asm volatile("" : "+v"(colp));
#pragma unroll
      for (int o = 1; o <= R; ++o) {
        const f32x4 r = gate ? acc[t][o - 1] * acc[0][o - 1] : acc[t][o - 1];
        const uint32_t lo = (uint32_t)__builtin_bit_cast(unsigned short, (bf16)r[0]) | ((uint32_t)__builtin_bit_cast(unsigned short, (bf16)r[1]) << 16);
        const uint32_t hi = (uint32_t)__builtin_bit_cast(unsigned short, (bf16)r[2]) | ((uint32_t)__builtin_bit_cast(unsigned short, (bf16)r[3]) << 16);
        if constexpr ((DBG & 16) != 0) {
          chk += __uint_as_float(lo) + __uint_as_float(hi);   // ablation: no stores (kept alive)
        } else {
          bf16* dst = out_col && y0 + o - 1 < a.H ? colp + (o - 1) * rstep : sinkp;
          asm volatile("global_store_dwordx2 %0, %1, off" : : "v"(dst), "v"(make_uint2(lo, hi)) : "memory");
        }
      }
    };
    dw_tile(0);
    if constexpr (MODE == TP_GATE) {
      // gelu(dw(x1)) parked as bf16 pairs (as the row-walk kernel parks it in LDS): 2 registers per row
      uint2 g1[R];
#pragma unroll
      for (int o = 0; o < R; ++o) {
        const f32x2 q0 = gelu_bf16_2(f32x2{acc[0][o][0], acc[0][o][1]}), q1 = gelu_bf16_2(f32x2{acc[0][o][2], acc[0][o][3]});
        g1[o] = make_uint2((uint32_t)__builtin_bit_cast(unsigned short, (bf16)q0.x) | ((uint32_t)__builtin_bit_cast(unsigned short, (bf16)q0.y) << 16),
                           (uint32_t)__builtin_bit_cast(unsigned short, (bf16)q1.x) | ((uint32_t)__builtin_bit_cast(unsigned short, (bf16)q1.y) << 16));
        // pinned here: left alone, hipcc sinks the GELUs next to the stores, keeping the fp32
        // depthwise rows of x1 live across the whole x2 depthwise (spills)
        asm volatile("" : "+v"(g1[o].x), "+v"(g1[o].y));
      }
      __builtin_amdgcn_sched_barrier(0);                    // tile 1's tables are read after tile 0 is done
      dw_tile(1);
#pragma unroll
      for (int o = 0; o < R; ++o)
        acc[1][o] *= f32x4{__uint_as_float(g1[o].x << 16), __uint_as_float(g1[o].x & 0xffff0000u), __uint_as_float(g1[o].y << 16),
                           __uint_as_float(g1[o].y & 0xffff0000u)};
      store_rows(16 * u + grp * 4, 1, false);
    } else {
      store_rows(row0(u, 0) + grp * 4, 0, false);
      __builtin_amdgcn_sched_barrier(0);
      dw_tile(1);
      store_rows(row0(u, 1) + grp * 4, 1, false);
    }
    // back-edge: the next pass's first two K steps (issued before the depthwise, NS stores ago)
    // have landed before the loop-carried ring slots can be copied
    tp_vmwait_ring<NS>(wf);
  }
  if constexpr ((DBG & 16) != 0) {
    if (chk == -1.2345f) out[tid] = (bf16)chk;             // never true in practice: keeps the work alive
  }
}

// haloed rows per tile: the GATE kernel fits 12 rows in its 256 registers, the DW kernel 10 (with
// 12 it spills)
constexpr int tp_rh(int mode) { return mode == TP_GATE ? 12 : 10; }

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
  const int R = tp_rh(a.mode) - 2;
  return (int64_t)a.nimg * ((a.H + R - 1) / R) * ((a.W + TP_TX - 1) / TP_TX);
}

template <int MODE, int N1M, int DBG>
static void tp_launch(const TilePdArgs& a, hipStream_t st) {
  constexpr int RH = tp_rh(MODE);
  using L = TPL<256, RH, N1M>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(tilepd_kernel<MODE, 256, RH, N1M, DBG>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, L::BYTES);
    attr = true;
  }
    const int64_t grid = tilepd_blocks(a);
  hipLaunchKernelGGL((tilepd_kernel<MODE, 256, RH, N1M, DBG>), dim3((unsigned)grid), dim3(TP_NT), L::BYTES, st, a);
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
    case 8: tp_dispatch<8>(a, st); return;
    case 16: tp_dispatch<16>(a, st); return;
    case 17: tp_dispatch<17>(a, st); return;
    case 18: tp_dispatch<18>(a, st); return;
    case 19: tp_dispatch<19>(a, st); return;
    case 24: tp_dispatch<24>(a, st); return;
    default: break;
  }
#endif
  tp_dispatch<0>(a, st);
}

}  // namespace turtle

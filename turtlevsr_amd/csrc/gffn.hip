// The whole level-3 GatedFeedForward block in one kernel ("gffn"), hidden map never in HBM:
//
//   out = x + W2 (gelu(dw(H1)) * dw(H2)) + b2,   [H1 ; H2] = W1' LN(x) + tb       (turtle_t1_arch.py:159-178,
//                                                                               the block's x + ffn(norm2(x)))
//
// LN = the block's LayerNorm (turtle_t1_arch.py:83-112; W1' = W1 diag(g), tb = W1 b_ln + b1 folded at pack
// time), dw = depthwise 3x3 with zero padding of H at the image border. Input width C = 256 (level 3),
// 128 or 64 (levels 2 / 1, round 6: instead of the fused2 row walk), hidden width hd = 64 k (GoPro level 3:
// hd = 640, H = 2 hd = 1280 channels; level 2: 320; level 1: 160, run as 192 with zero weights for the
// padding channels - exact: their H, G and W2 columns are 0). At width 64 P3's 64 output channels are
// 4 groups of 16 and each group's 7 pixel tiles are split 4 / 3 over two waves. Against project_in GEMM ->
// depthwise + gate -> project_out GEMM with the hidden map in HBM (1080p level 3: 334 MB written and
// read back per block, 20 blocks per frame) only x is read and the output written.
//
// One 512-thread block per CU owns a 14 x 8 output tile (16 x 10 haloed pixels) and walks the hidden
// channels in chunks of 64 gate pairs (128 of H's channels):
//   prologue  the haloed x tile -> LayerNorm in registers -> LDS as f16 (87 KB, resident for the block)
//   P1        H chunk = W1' X + tb on the matrix cores (v_mfma_f32_16x16x32_f16): wave w owns two
//             16-row units x 5 of the 10 haloed rows; W1' fragments stream from L2 into registers
//             (prefetched one chunk ahead); H -> LDS as f16, rows permuted at pack time so a lane's 4
//             accumulators are (x1 c, x1 c+1, x2 c, x2 c+1) of one gate pair: one 8-byte store
//   P2        depthwise + gate on packed f16 (v_pk_fma_f16; x-neighbours by DPP row shifts inside the
//             16-lane row = one haloed image row, y-neighbours from the rows the lane walked), GELU gate
//             on packed f16 too (tanh form, as every bf16 kernel: common.h), G -> LDS f16 [8 ch-groups][112 px][8]
//   P3        out_acc[256 x 112] += W2[:, chunk] G on the matrix cores: wave w owns output channels
//             32 w .. 32 w + 31 (rows permuted: a lane's 8 accumulators are 8 consecutive channels)
//   epilogue  out = x + acc + b2, 16-byte bf16 stores
// P1 -> P2 -> P3 are separated by block barriers; the accumulators of the output tile live in the
// waves' registers for the whole block (56 per lane).
#include "common.h"
#include "kernels.h"

#include <cstring>
#include <type_traits>
#include <vector>

namespace turtle {

typedef _Float16 f16;
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int GF_TX = 14, GF_TR = 8, GF_RH = GF_TR + 2, GF_NXP = 16 * GF_RH, GF_NGP = GF_TX * GF_TR;
constexpr int GF_NT = 512;
constexpr int GF_MAXNC = 12;                                 // hidden width <= 768 (taps / tb tables in LDS)
// geometry per input width C: X rows, K steps per chunk, output channels per wave
template <int C>
struct GfGeom {
  static constexpr int XP = C * 2 + 32;                      // LDS bytes per haloed pixel of X (+32: conflict-free b128)
  static constexpr int OFF_G = GF_NXP * XP;                  // two G buffers: [8 groups][112 px][8 ch] f16 each
  static constexpr int OFF_SINK = OFF_G + 2 * 8 * GF_NGP * 16;   // P2 store target of the x-halo lanes (no branch per row)
  static constexpr int OFF_TAP = OFF_SINK + 8 * 64 * 4;      // depthwise taps + bias of every chunk, P2 lane order
  static constexpr int OFF_TB = OFF_TAP + GF_MAXNC * 8 * 4 * 80;   // P1 epilogue vectors (W1 b_ln + b1) of every chunk
  static constexpr int LDS = OFF_TB + GF_MAXNC * 128 * 4;
  static constexpr int KS = C / 32;                          // P1 K steps per chunk (32 input channels each)
  static constexpr bool SN = C == 64;                        // P3 at width 64: 4 channel groups x 2 pixel halves of waves
  static constexpr int MW = SN ? 1 : C / 128;                // P3: 16 MW output channels per wave (MW MFMA row tiles)
  static constexpr int CW = SN ? 4 : 8;                      // P3 output-channel groups
  static constexpr int NTW = SN ? 4 : 7;                     // P3 pixel N tiles per wave (7 = 112 px / 16)
  static constexpr int CPL = C / 64;                         // prologue: 16-byte chunks per lane of a pixel's 8 lanes
  static constexpr int RPS = GF_TR / KS;                     // P2 output rows per P1 K step
  static_assert(LDS <= 160 * 1024, "gffn LDS budget");
  static_assert(KS * RPS == GF_TR, "P2 rows per K step");
};
static_assert(GF_NGP == 7 * 16, "P3 N tiles");

__device__ __attribute__((aligned(64))) uint4 g_zero_gf[4];

TURTLE_DEV uint32_t gf_shr(uint32_t v) {   // value of the x - 1 neighbour (0 at x = 0)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x111, 0xf, 0xf, true);
}
TURTLE_DEV uint32_t gf_shl(uint32_t v) {   // value of the x + 1 neighbour (0 at x = 15)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x101, 0xf, 0xf, true);
}
TURTLE_DEV f16x2 h2(uint32_t v) { return __builtin_bit_cast(f16x2, v); }
TURTLE_DEV uint32_t u2(f16x2 v) { return __builtin_bit_cast(uint32_t, v); }
TURTLE_DEV f16x8 as_f16x8(uint4 v) { return __builtin_bit_cast(f16x8, v); }
TURTLE_DEV uint32_t pk_f16(float a, float b) { return u2(__builtin_convertvector(f32x2{a, b}, f16x2)); }

// compile-time loop: f(std::integral_constant<int, I>) for I in [I0, N) - the register arrays indexed by it
// (the W1 ring, the H rows) stay registers (a runtime-int index inside a lambda left them in scratch)
template <int I, int N, typename F>
TURTLE_DEV void gf_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    gf_for<I + 1, N>(f);
  }
}

template <int C, int DBG>
__global__ __launch_bounds__(GF_NT, 1) void gffn_kernel(GffnArgs a) {
  using G = GfGeom<C>;
  constexpr int KS = G::KS, MW = G::MW, XP = G::XP, NTW = G::NTW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sX = smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int xl = lane & 15, g4 = lane >> 4;
  const int nc = a.hd / 64;
  // P3 / epilogue ownership: output-channel group cw, pixel N tiles n0 .. n0 + NTW - 1 (ntl of them live)
  const int cw = G::SN ? (wid & 3) : wid;
  const int n0 = G::SN ? (wid >> 2) * 4 : 0;
  const int ntl = G::SN ? ((wid >> 2) ? 3 : 4) : 7;

  // ---- tile (row-major over the image; consecutive tiles on one XCD share halo rows) ----
  const int tx_n = (a.W + GF_TX - 1) / GF_TX, ty_n = (a.H + GF_TR - 1) / GF_TR;
  int lin = blockIdx.x;
  {
    const int nblk = gridDim.x, q = nblk / 8, r = nblk % 8, xx = lin % 8, yy = lin / 8;
    lin = (xx < r ? xx * (q + 1) : r * (q + 1) + (xx - r) * q) + yy;
  }
  const int img = lin / (tx_n * ty_n), trem = lin - img * tx_n * ty_n;
  const int y0 = (trem / tx_n) * GF_TR, x0 = (trem % tx_n) * GF_TX;

  // ---- weight streams of wave `wid` (hidden unit wid of every chunk: no fragment is loaded twice per
  // block). Issue order per interval (vmcnt retires in order; hipcc counts these plain loads exactly
  // because the loop body is one path): W1 K steps three ahead through a 4-slot ring (the next chunk's
  // first three during the last three steps), then the taps of the next P2 and the tb vector of the next
  // P1, then the W2 fragments of the next P3 ----
  const uint4* W1F = reinterpret_cast<const uint4*>(a.w1f);
  const uint4* W2F = reinterpret_cast<const uint4*>(a.w2f);
  const uint32_t* DWP = a.dwp;                              // (no lambda below refers to `a`: a by-reference capture of the
  const float* TBP = a.tbp;                                 // kernel argument would copy it to scratch)
  uint4 wf[4];                                              // 4 slots: 8 (4) steps per chunk keep the slot of step k = k & 3
  uint4 tq[5];
  uint4 w2[MW][2];
  f32x4 tbv;
  auto ld_w1 = [&](int c, auto K) __attribute__((always_inline)) {
    constexpr int k = decltype(K)::value;
    wf[k & 3] = (DBG & 8) ? make_uint4(lane, k, c, 0) : W1F[((c * 8 + wid) * KS + k) * 64 + lane];
  };
  // taps and tb vectors come from LDS tables filled once per block (prologue)
  auto ld_taps = [&](int c) __attribute__((always_inline)) {
    const uint4* tp = reinterpret_cast<const uint4*>(smem + G::OFF_TAP + (((c * 8 + wid) * 4 + g4) * 20) * 4);
#pragma unroll
    for (int q = 0; q < 5; ++q) tq[q] = tp[q];
  };
  auto ld_tb = [&](int c) __attribute__((always_inline)) {
    tbv = *reinterpret_cast<const f32x4*>(smem + G::OFF_TB + ((c * 8 + wid) * 16 + 4 * g4) * 4);
  };
  auto ld_w2 = [&](int c) __attribute__((always_inline)) {
#pragma unroll
    for (int m = 0; m < MW; ++m)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        w2[m][ks] = (DBG & 8) ? make_uint4(lane, m, ks, c) : W2F[(((c * G::CW + cw) * MW + m) * 2 + ks) * 64 + lane];
  };
  ld_w1(0, std::integral_constant<int, 0>{});
  ld_w1(0, std::integral_constant<int, 1>{});
  if constexpr (KS > 2) ld_w1(0, std::integral_constant<int, 2>{});

  // ---- haloed x tile -> LayerNorm in registers -> LDS (f16). A pixel's C / 8 16-byte chunks are held
  // by an aligned group of 8 lanes (chunks cc, cc + 8, ...); statistics by an 8-lane DPP
  // reduction, two passes (biased variance, eps 1e-5 inside the sqrt: turtle_t1_arch.py:78-80, 96-99);
  // pixels outside the image are 0 and stay 0 (and P1 keeps their H at 0: the depthwise zero padding).
  // The two G buffers start zeroed (P3 of the first loop interval multiplies one of them) ----
  {
    constexpr int LPP = 8, CPL = G::CPL, PPJ = GF_NT / LPP, NJ = (GF_NXP + PPJ - 1) / PPJ;
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
      const bool ok = p < GF_NXP && y >= 0 && y < a.H && x >= 0 && x < a.W;
      const bf16* src = X + (((int64_t)img * a.H + (ok ? y : 0)) * a.W + (ok ? x : 0)) * C + cc * 8;
#pragma unroll
      for (int q = 0; q < CPL; ++q)
        vx[j][q] = (DBG & 16) ? make_uint4(p, q, cc, 0x3f803f80u) : ld16(ok ? reinterpret_cast<const void*>(src + q * LPP * 8) : g_zero_gf);
    }
    for (int e = tid; e < 2 * 8 * GF_NGP; e += GF_NT)
      *reinterpret_cast<uint4*>(smem + G::OFF_G + e * 16) = make_uint4(0u, 0u, 0u, 0u);
    {
      const int ntap = nc * 8 * 4 * 5, ntb = nc * 32;             // 16-byte pieces
      for (int e = tid; e < ntap; e += GF_NT)
        *reinterpret_cast<uint4*>(smem + G::OFF_TAP + e * 16) =
            (DBG & 8) ? make_uint4(0x3c003c00u, e, 0u, 0u) : reinterpret_cast<const uint4*>(DWP)[e];
      for (int e = tid; e < ntb; e += GF_NT)
        *reinterpret_cast<uint4*>(smem + G::OFF_TB + e * 16) = (DBG & 8) ? make_uint4(0u, 0u, 0u, 0u) : reinterpret_cast<const uint4*>(TBP)[e];
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int p = j * PPJ + pq;
      float sm = 0.f;
#pragma unroll
      for (int q = 0; q < CPL; ++q) {
        Vec<bf16> vv; vv.from_raw(vx[j][q]);
#pragma unroll
        for (int e = 0; e < 8; ++e) sm += vv.v[e];
      }
      const float mu = sum8(sm) * (1.f / C);
      float sq = 0.f;
#pragma unroll
      for (int q = 0; q < CPL; ++q) {
        Vec<bf16> vv; vv.from_raw(vx[j][q]);
#pragma unroll
        for (int e = 0; e < 8; ++e) { const float d = vv.v[e] - mu; sq = fmaf(d, d, sq); }
      }
      const float rs = rsqrtf(sum8(sq) * (1.f / C) + 1e-5f);
      const float c0 = a.centred ? -mu * rs : 0.f;
      if (p < GF_NXP) {
#pragma unroll
        for (int q = 0; q < CPL; ++q) {
          Vec<bf16> vv; vv.from_raw(vx[j][q]);
          uint32_t w[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) w[e] = pk_f16(fmaf(vv.v[2 * e], rs, c0), fmaf(vv.v[2 * e + 1], rs, c0));
          *reinterpret_cast<uint4*>(sX + p * XP + (cc + q * LPP) * 16) = make_uint4(w[0], w[1], w[2], w[3]);
        }
      }
    }
  }

  // validity of the lane's P1 pixels (column xl of haloed rows 0 .. 9)
  const int xg = x0 - 1 + xl;
  const bool colok = xg >= 0 && xg < a.W;
  uint32_t rowok = 0;
#pragma unroll
  for (int r = 0; r < GF_RH; ++r) {
    const int yg = y0 - 1 + r;
    rowok |= (colok && yg >= 0 && yg < a.H) ? (1u << r) : 0u;
  }

  f32x4 oacc[MW][NTW];
#pragma unroll
  for (int m = 0; m < MW; ++m)
#pragma unroll
    for (int n = 0; n < NTW; ++n) oacc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  // P1 state: acc[r] = the lane's 4 slots (x1 c, x1 c+1, x2 c, x2 c+1 of gate pair 4 wid + g4) of
  // haloed pixel (r, xl); hv = the previous chunk's H as f16 pairs (P2's input)
  f32x4 acc[GF_RH];
  uint32_t hv[GF_RH][2];
#pragma unroll
  for (int r = 0; r < GF_RH; ++r) hv[r][0] = hv[r][1] = 0u;
  const char* xb = sX + xl * XP + g4 * 16;
  f16x8 xa[5];                                              // P1 fragments of haloed rows 0-4, one K step ahead
  const bool wr = xl >= 1 && xl <= GF_TX;
  char* sink = smem + G::OFF_SINK + tid * 4;

  auto p1_init = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < GF_RH; ++r) acc[r] = ((rowok >> r) & 1u) ? tbv : f32x4{0.f, 0.f, 0.f, 0.f};
  };
  // one K step of P1 (chunk c): 10 pixel-row fragments from LDS, one W1 fragment, 10 MFMAs; the W1
  // stream runs three steps ahead (into the next chunk cn during the last three steps)
  auto p1_step = [&](auto K, int c, int cn) __attribute__((always_inline)) {
    constexpr int k = decltype(K)::value;
    // KS >= 4: three steps ahead through the 4-slot ring (slot = step & 3). KS = 2 (width 64): the next
    // chunk's step k replaces this step's slot after its MFMAs (two steps ahead; 3 would overwrite step
    // k + 1 of this chunk)
    if constexpr (KS >= 4) {
      if constexpr (k + 3 < KS) ld_w1(c, std::integral_constant<int, k + 3>{});
      else ld_w1(cn, std::integral_constant<int, k + 3 - KS>{});
    }
    // rows 0-4 of this step were read at the end of the previous step (their latency behind its P2
    // row); rows 5-9 are read before rows 0-4 multiply, and rows 0-4 of the NEXT step (the next chunk's
    // step 0 after step 7: X does not change) after rows 5-9 multiply
    f16x8 xb5[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) xb5[i] = *reinterpret_cast<const f16x8*>(xb + (5 + i) * 16 * XP + k * 64);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      if constexpr ((DBG & 1) == 0) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(wf[k & 3]), xa[i], acc[i], 0, 0, 0);
      else acc[i][0] += (float)xa[i][0] + (float)as_f16x8(wf[k & 3])[1];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      if constexpr ((DBG & 1) == 0) acc[5 + i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(wf[k & 3]), xb5[i], acc[5 + i], 0, 0, 0);
      else acc[5 + i][0] += (float)xb5[i][0] + (float)as_f16x8(wf[k & 3])[1];
    }
    if constexpr (KS < 4) ld_w1(cn, K);
#pragma unroll
    for (int i = 0; i < 5; ++i) xa[i] = *reinterpret_cast<const f16x8*>(xb + i * 16 * XP + ((k + 1) % KS) * 64);
    __builtin_amdgcn_sched_barrier(0);
  };
  auto p1_finish = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < GF_RH; ++r) {
      hv[r][0] = pk_f16(acc[r][0], acc[r][1]);
      hv[r][1] = pk_f16(acc[r][2], acc[r][3]);
    }
  };
  // one output row o (1 .. 8) of P2 for the chunk whose H is in hv: depthwise on packed f16 (taps of
  // row o - 1 + dy, x-neighbours by DPP), gelu(x1) * x2 in f32, one 4-byte G store (x-halo lanes: sink)
  auto p2_row = [&](auto O, char* gbuf) __attribute__((always_inline)) {
    constexpr int o = decltype(O)::value;
    const uint32_t tw[20] = {tq[0].x, tq[0].y, tq[0].z, tq[0].w, tq[1].x, tq[1].y, tq[1].z, tq[1].w, tq[2].x, tq[2].y,
                             tq[2].z, tq[2].w, tq[3].x, tq[3].y, tq[3].z, tq[3].w, tq[4].x, tq[4].y, tq[4].z, tq[4].w};
    uint32_t gout;
    if constexpr ((DBG & 2) == 0) {
      f16x2 s[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        s[h] = h2(tw[18 + h]);
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
          const uint32_t v = hv[o - 1 + dy][h];
          s[h] = __builtin_elementwise_fma(h2(tw[2 * (3 * dy + 0) + h]), h2(gf_shr(v)), s[h]);
          s[h] = __builtin_elementwise_fma(h2(tw[2 * (3 * dy + 1) + h]), h2(v), s[h]);
          s[h] = __builtin_elementwise_fma(h2(tw[2 * (3 * dy + 2) + h]), h2(gf_shl(v)), s[h]);
        }
      }
      // gelu(x1) * x2 on packed f16, the tanh form of every bf16 kernel (common.h gelu_tanh: x / (1 + 2^u),
      // u = -log2(e) 1.5957691 (x + 0.044715 x^3)); f16 rounding of u / 2^u stays below G's own rounding
      const f16x2 x = s[0];
      const f16x2 u = x * (x * x * f16x2{(f16)-0.10294324f, (f16)-0.10294324f} + f16x2{(f16)-2.3022082f, (f16)-2.3022082f});
      const f16x2 e = __builtin_elementwise_exp2(u) + f16x2{(f16)1.f, (f16)1.f};
      gout = u2(x * (f16x2{(f16)1.f, (f16)1.f} / e) * s[1]);
    } else {
      gout = hv[o][0] ^ hv[o][1] ^ tw[o];
    }
    *reinterpret_cast<uint32_t*>(wr ? gbuf + (wid * GF_NGP + (o - 1) * GF_TX + xl - 1) * 16 + 4 * g4 : sink) = gout;
  };
  // P3: out_acc += W2 fragments (in w2) x G (LDS buffer gbuf)
  auto p3 = [&](const char* gbuf) __attribute__((always_inline)) {
    const char* gb = gbuf + xl * 16;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      f16x8 bfr[NTW];
#pragma unroll
      for (int j = 0; j < NTW; ++j) {                        // (a dead 4th tile of the second wave half re-reads tile 6)
        const int n = min(n0 + j, 6);
        bfr[j] = *reinterpret_cast<const f16x8*>(gb + ((ks * 4 + g4) * GF_NGP + n * 16) * 16);
      }
      if constexpr ((DBG & 4) == 0) {
#pragma unroll
        for (int j = 0; j < NTW; ++j)
#pragma unroll
          for (int m = 0; m < MW; ++m)
            oacc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(w2[m][ks]), bfr[j], oacc[m][j], 0, 0, 0);
      } else {
#pragma unroll
        for (int j = 0; j < NTW; ++j) { oacc[0][j][0] += (float)bfr[j][0]; oacc[MW - 1][j][1] += (float)as_f16x8(w2[MW - 1][ks])[0]; }
      }
    }
  };
  char* const G0 = smem + G::OFF_G;
  char* const G1 = smem + G::OFF_G + 8 * GF_NGP * 16;
  auto gbuf = [&](int c) __attribute__((always_inline)) { return (c & 1) ? G1 : G0; };

  __syncthreads();

  // ---- interval 0: P1(0) ----
#pragma unroll
  for (int i = 0; i < 5; ++i) xa[i] = *reinterpret_cast<const f16x8*>(xb + i * 16 * XP);
  ld_tb(0);
  p1_init();
  gf_for<0, KS>([&](auto K) __attribute__((always_inline)) { p1_step(K, 0, nc > 1 ? 1 : 0); });
  p1_finish();
  ld_taps(0);
  ld_tb(nc > 1 ? 1 : 0);
  ld_w2(0);
  __syncthreads();

  // ---- intervals 1 .. nc - 1: P1(c) with P2(c - 1) interleaved row by row (RPS output rows per K step),
  // then P3(c - 2) (at c = 1 over the zeroed G buffer: adds 0) ----
  for (int c = 1; c < nc; ++c) {
    const int cn = c + 1 < nc ? c + 1 : c;
    char* gw = gbuf(c - 1);
    p1_init();
    gf_for<0, KS>([&](auto K) __attribute__((always_inline)) {
      p1_step(K, c, cn);
      gf_for<0, G::RPS>([&](auto J) __attribute__((always_inline)) {
        p2_row(std::integral_constant<int, decltype(K)::value * G::RPS + decltype(J)::value + 1>{}, gw);
      });
    });
    p1_finish();
    ld_taps(c);
    ld_tb(cn);
    p3(gbuf(c));                                            // G of chunk c - 2 (buffer (c - 2) & 1)
    ld_w2(c - 1);
    __syncthreads();
  }
  // ---- interval nc: P2(nc - 1), P3(nc - 2); interval nc + 1: P3(nc - 1) ----
  gf_for<1, GF_TR + 1>([&](auto O) __attribute__((always_inline)) { p2_row(O, gbuf(nc - 1)); });
  p3(gbuf(nc));
  ld_w2(nc - 1);
  __syncthreads();
  p3(gbuf(nc - 1));

  // ---------------- epilogue: out = x + acc + b2 (4 MW consecutive channels per lane and N tile) ----------------
  {
    constexpr int NCH = 4 * MW;
    const int chb = 16 * MW * cw + NCH * g4;
    f32x4 bb[MW];
#pragma unroll
    for (int m = 0; m < MW; ++m)
      bb[m] = a.b2 ? *reinterpret_cast<const f32x4*>(a.b2 + chb + 4 * m) : f32x4{0.f, 0.f, 0.f, 0.f};
    const bf16* X = reinterpret_cast<const bf16*>(a.x);
    bf16* O = reinterpret_cast<bf16*>(a.out);
    typedef uint32_t rawv __attribute__((ext_vector_type(NCH / 2)));   // the lane's NCH bf16 channels, raw
    rawv rv[NTW];                                           // every residual load in flight before the first store
    int64_t offs[NTW];
    bool st[NTW];
#pragma unroll
    for (int n = 0; n < NTW; ++n) {
      const int gp = min(n0 + n, 6) * 16 + xl, o = gp / GF_TX, xo = gp - o * GF_TX;
      const int y = y0 + o, x = x0 + xo;
      st[n] = n < ntl && y < a.H && x < a.W;
      offs[n] = (((int64_t)img * a.H + (st[n] ? y : 0)) * a.W + (st[n] ? x : 0)) * C + chb;
      rv[n] = *reinterpret_cast<const rawv*>(X + offs[n]);
    }
    typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int n = 0; n < NTW; ++n) {
      rawv ov;
#pragma unroll
      for (int q = 0; q < NCH / 2; ++q) {
        const uint32_t wv = rv[n][q];
        const int m = (2 * q) / 4, e = (2 * q) % 4;
        const f32x2 sum2 = {__uint_as_float(wv << 16) + (oacc[m][n][e] + bb[m][e]),
                            __uint_as_float(wv & 0xffff0000u) + (oacc[m][n][e + 1] + bb[m][e + 1])};
        ov[q] = __builtin_bit_cast(uint32_t, __builtin_convertvector(sum2, bf16x2v));
      }
      if (st[n]) *reinterpret_cast<rawv*>(O + offs[n]) = ov;
    }
  }
}

bool gffn_ok(const GffnArgs& a) {
  if (!a.x || !a.out || !a.w1f || !a.tbp || !a.dwp || !a.w2f || a.x == a.out) return false;
  if ((a.C != 256 && a.C != 128 && a.C != 64) || a.hd <= 0 || a.hd % 64 || a.hd > 64 * GF_MAXNC) return false;
  if (reinterpret_cast<uintptr_t>(a.x) % 16 || reinterpret_cast<uintptr_t>(a.out) % 16 || reinterpret_cast<uintptr_t>(a.w1f) % 16 ||
      reinterpret_cast<uintptr_t>(a.w2f) % 16 || reinterpret_cast<uintptr_t>(a.tbp) % 16 || reinterpret_cast<uintptr_t>(a.dwp) % 16 ||
      (a.b2 && reinterpret_cast<uintptr_t>(a.b2) % 16))
    return false;
  return a.H > 0 && a.W > 0 && a.nimg > 0 && (int64_t)a.nimg * a.H * a.W * a.C < ((int64_t)1 << 40);
}

int64_t gffn_blocks(const GffnArgs& a) {
  return (int64_t)a.nimg * ((a.H + GF_TR - 1) / GF_TR) * ((a.W + GF_TX - 1) / GF_TX);
}

template <int C, int DBG>
static void gf_launch_c(const GffnArgs& a, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gffn_kernel<C, DBG>), hipFuncAttributeMaxDynamicSharedMemorySize,
                              GfGeom<C>::LDS);
    attr = true;
  }
  hipLaunchKernelGGL((gffn_kernel<C, DBG>), dim3((unsigned)gffn_blocks(a)), dim3(GF_NT), GfGeom<C>::LDS, st, a);
}
template <int DBG>
static void gf_launch(const GffnArgs& a, hipStream_t st) {
  if (a.C == 64) gf_launch_c<64, DBG>(a, st);
  else if (a.C == 128) gf_launch_c<128, DBG>(a, st);
  else gf_launch_c<256, DBG>(a, st);
}

void launch_gffn(const GffnArgs& a, hipStream_t st) {
  if (!gffn_ok(a)) kernel_arg_error("gffn: arguments outside the kernel's contract");
#ifdef TURTLE_GFFN_ABLATIONS
  // tools/gfbench only: dbg bits 1 no P1 MFMAs, 2 no depthwise / gate, 4 no P3 MFMAs, 8 no weight stream
  // loads, 16 no prologue loads
  switch (a.dbg) {
    case 1: gf_launch<1>(a, st); return;
    case 2: gf_launch<2>(a, st); return;
    case 4: gf_launch<4>(a, st); return;
    case 5: gf_launch<5>(a, st); return;
    case 7: gf_launch<7>(a, st); return;
    case 8: gf_launch<8>(a, st); return;
    case 15: gf_launch<15>(a, st); return;
    case 16: gf_launch<16>(a, st); return;
    case 31: gf_launch<31>(a, st); return;
    default: break;
  }
#endif
  gf_launch<0>(a, st);
}

// ------------------------------------------------------------------------------------------
// host-side packing (turtle.cpp pack_all, tools/gfbench)
// ------------------------------------------------------------------------------------------
static uint16_t f16_bits(double x) {
  const _Float16 h = (_Float16)(float)x;
  uint16_t u;
  std::memcpy(&u, &h, 2);
  return u;
}

void gffn_pack(int C, int hd, const std::vector<double>& w1, const std::vector<double>& tb, const std::vector<double>& dw9,
               const std::vector<double>& dwb, const std::vector<double>& w2, GffnHost& o) {
  const int nc = hd / 64, H2 = 2 * hd, KS = C / 32, MW = C >= 128 ? C / 128 : 1, CW = C == 64 ? 4 : 8;
  // hidden row of slot s of unit u in chunk c: gate pair p = 4 u + s / 4 (chunk-local), e = s % 4:
  // (x1 2p, x1 2p + 1, x2 2p, x2 2p + 1)
  auto hrow = [&](int c, int u, int s) {
    const int p = 4 * u + s / 4, e = s % 4;
    const int g = 64 * c + 2 * p + (e & 1);
    return (e < 2) ? g : hd + g;
  };
  o.w1f.assign((size_t)H2 * C, 0);
  o.tbp.assign((size_t)H2, 0.f);
  for (int c = 0; c < nc; ++c)
    for (int u = 0; u < 8; ++u) {
      for (int s = 0; s < 16; ++s) o.tbp[(size_t)(c * 8 + u) * 16 + s] = tb.empty() ? 0.f : (float)tb[hrow(c, u, s)];
      for (int k = 0; k < KS; ++k)
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 8; ++j)
            o.w1f[((((size_t)(c * 8 + u) * KS + k) * 64 + l) * 8) + j] = f16_bits(w1[(size_t)hrow(c, u, l & 15) * C + 32 * k + 8 * (l >> 4) + j]);
    }
  // depthwise taps for P2 lane (wave w, group g): channels x1 a, a + 1 and x2 a, a + 1 with a = 64 c + 8 w + 2 g
  o.dwp.assign((size_t)nc * 8 * 4 * 20, 0u);
  for (int c = 0; c < nc; ++c)
    for (int w = 0; w < 8; ++w)
      for (int g = 0; g < 4; ++g) {
        const int ca = 64 * c + 8 * w + 2 * g;
        uint32_t* d = &o.dwp[((size_t)(c * 8 + w) * 4 + g) * 20];
        for (int t = 0; t < 9; ++t) {
          d[2 * t] = f16_bits(dw9[(size_t)t * H2 + ca]) | ((uint32_t)f16_bits(dw9[(size_t)t * H2 + ca + 1]) << 16);
          d[2 * t + 1] = f16_bits(dw9[(size_t)t * H2 + hd + ca]) | ((uint32_t)f16_bits(dw9[(size_t)t * H2 + hd + ca + 1]) << 16);
        }
        auto b = [&](int ch) { return dwb.empty() ? 0.0 : dwb[ch]; };
        d[18] = f16_bits(b(ca)) | ((uint32_t)f16_bits(b(ca + 1)) << 16);
        d[19] = f16_bits(b(hd + ca)) | ((uint32_t)f16_bits(b(hd + ca + 1)) << 16);
      }
  // W2 fragment (c, w, m, ks): row i = l & 15 -> output channel 16 MW w + 4 MW (i >> 2) + 4 m + (i & 3)
  // (a lane's MW x 4 accumulators are 4 MW consecutive channels), k = 64 c + 32 ks + 8 (l >> 4) + j
  o.w2f.assign((size_t)C * hd, 0);
  for (int c = 0; c < nc; ++c)
    for (int w = 0; w < CW; ++w)
      for (int m = 0; m < MW; ++m)
        for (int ks = 0; ks < 2; ++ks)
          for (int l = 0; l < 64; ++l)
            for (int j = 0; j < 8; ++j) {
              const int i = l & 15, oc = 16 * MW * w + 4 * MW * (i >> 2) + 4 * m + (i & 3), k = 64 * c + 32 * ks + 8 * (l >> 4) + j;
              o.w2f[(((((size_t)(c * CW + w) * MW + m) * 2 + ks) * 64 + l) * 8) + j] = f16_bits(w2[(size_t)oc * hd + k]);
            }
}

}  // namespace turtle

// Depthwise-prologue GEMM ("dwg" kernel): the second half of a GatedFeedForward, or the value path
// of a channel attention, at widths >= 256 (level 3, latent), in one launch:
//
//   out[m][n] = res[m][n] + b[n] + sum_k W[n][k] * A[m][k]
//   A[m][k]   = gelu(dw(x1)[m][k]) * dw(x2)[m][k]      (GATE: turtle_t1_arch.py:171-178)
//             = dw(x)[m][k]                           (PLAIN: the v of qkv_dwconv, 684-690, whose
//                                                      W_eff = project_out . blockdiag(attn) follows)
//
// with dw = depthwise 3x3 (+bias, zero padding) over the pixel-major hidden map written by the
// preceding projection. The hidden map of dw outputs (640 / 1280 channels per pixel) never goes to
// HBM: each K step of 16 channels computes its A tile from the raw hidden map staged in LDS.
//
// Structure (MI355X, bf16, fp32 accumulation):
//   * block = 512 threads (8 waves, a 4 x 2 wave grid), output tile = 8 image rows x 32 columns
//     (256 pixels) x 256 output channels; wave tile 64 pixels x 128 channels (MFMA 16x16x32,
//     128 accumulators per lane), one block per CU;
//   * K step s (16 hidden channels): the haloed 10 x 34 pixel input tile of step s + 3 (x1 [, x2]
//     16 channels, the bf16 tap table and the fp32 bias) and the weights of step s + 2 go
//     HBM/L2 -> LDS by LDS-DMA into a 4-slot / 5-slot ring while the waves work; wave w computes
//     the depthwise of output row w on the matrix cores (below) and writes its gated A rows to the
//     3-slot A ring; the GEMM runs on pairs of K steps. One barrier per K step;
//   * weight rows are read in the permuted order of the kt / pn GEMMs (MFMA row 4g+e of sub-tile
//     t <- channel 8g+4t+e of a 32-channel group), so a lane's accumulators hold 8 consecutive
//     output channels of one pixel: register-direct epilogue, 16-byte residual loads and stores;
//   * LDS rows of 64 B, 16-byte chunk c of row r at position c ^ h(r), h(r) = (r >> 2) & 2
//     (conflict-free ds_read_b128 for both operands, gemm5.hip).
#include "common.h"
#include "kernels.h"

namespace turtle {

__device__ __attribute__((aligned(64))) uint4 g_zero_dg[4];

// one LDS-DMA wave instruction: 64 lanes x 16 B -> LDS at M0 (inline asm: see gemm5.hip kt_dma16)
TURTLE_DEV void dg_dma16(const void* g, uint32_t lds_wave_base) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(lds_wave_base) : "memory");
}

constexpr int DG_TH = 8, DG_TW = 32, DG_BM = DG_TH * DG_TW, DG_BN = 256, DG_NT = 512, DG_NW = 8;
constexpr int DG_KC = 16;                                 // hidden channels per K step
constexpr int DG_XR = DG_TH + 2, DG_XP = DG_TW + 2;       // haloed input tile: rows x pixels
constexpr int DG_W_BYTES = DG_BN * DG_KC * 2, DG_A_BYTES = DG_BM * DG_KC * 2;   // 32-B rows
constexpr int DG_XSLOTS = 4, DG_WSLOTS = 5, DG_ASLOTS = 3;
template <int NH> struct DGL {
  static constexpr int PB = NH * DG_KC * 2;               // bytes per staged pixel (x1 [, x2] x 16 channels)
  static constexpr int X_BYTES = DG_XR * DG_XP * PB;
  static constexpr int T_OFF = X_BYTES;                   // taps bf16 [half][9][16], then bias fp32 [half][16]
  static constexpr int B_OFF = T_OFF + NH * 9 * DG_KC * 2;
  static constexpr int T_END = B_OFF + NH * DG_KC * 4;
  static constexpr int NINSTR = (T_END + 1023) / 1024;
  static constexpr int XI = (NINSTR + DG_NW - 1) / DG_NW; // DMA instructions per wave per stage (uniform)
  static constexpr int STAGE = XI * DG_NW * 1024;
  static constexpr int OFF_W = DG_XSLOTS * STAGE, OFF_A = OFF_W + DG_WSLOTS * DG_W_BYTES;
  static constexpr int BYTES = OFF_A + DG_ASLOTS * DG_A_BYTES;
  static constexpr int PER_STEP = XI + 1;                 // + one weight instruction per wave
  static_assert(BYTES <= 160 * 1024, "dwgemm LDS budget");
  static_assert(DG_W_BYTES == DG_NW * 1024, "one weight DMA instruction per wave");
  static_assert(T_OFF % 16 == 0 && B_OFF % 16 == 0, "tap table alignment");
};
// 16-byte position of channel chunk c of staged pixel p. The depthwise MFMA operand reads 16
// consecutive pixels x 2 chunks per lane group (lane = pixel l & 15, chunk (l >> 4) & 1), shifted
// by the tap column; this table (exhaustive search) makes every such ds_read_b128 lane group hit 16
// distinct bank quads for 64-B pixels; 32-B pixels need no swizzle
template <int NH> TURTLE_DEV int dg_xpos(int p, int c) { return NH == 2 ? c ^ (((0xFC30 >> (p & 15)) & 1) << 1) : c; }
// 16-byte half of the 32-byte operand rows (A pixels, W channels): the GEMM's ds_read_b128 lane
// groups {0-3,12-15,20-27}, {4-11,16-19,28-31} read rows (l & 15), halves (l >> 4) & 1 - with the
// half flipped on rows 4-7 and 12-15 they cover 16 distinct bank quads
TURTLE_DEV int dg_h(int r) { return (r >> 2) & 1; }
template <int N>
TURTLE_DEV void dg_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

template <int NH>
__global__ __launch_bounds__(DG_NT, 1) void dwgemm_kernel(DwGemmArgs g) {
  using L = DGL<NH>;
  typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;                   // wave tile: pixels 64 wm.., channels 128 wn..
  const int fr = lane & 15, fq = lane >> 4;

  // ---- tile (row-major over the image, channel tiles of one pixel tile adjacent); consecutive ids
  // on one XCD so vertically neighbouring tiles share their halo rows in its L2 ----
  const int ntn = (g.N + DG_BN - 1) / DG_BN;
  const int ntx = (g.W + DG_TW - 1) / DG_TW, nty = (g.H + DG_TH - 1) / DG_TH;
  int lin = blockIdx.x;
  {
    const int nblk = gridDim.x, q = nblk / 8, r = nblk % 8, x = lin % 8, y = lin / 8;
    lin = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;
  }
  const int nt = lin % ntn;
  int t = lin / ntn;
  const int tx = t % ntx;
  t /= ntx;
  const int ty = t % nty;
  const int img = t / nty;
  const int x0 = tx * DG_TW, y0 = ty * DG_TH, n0 = nt * DG_BN;
  const int K = g.K, nk = K / DG_KC, Cw = NH * K;
  const bf16* Wp = reinterpret_cast<const bf16*>(g.w) + (g.wstride ? (int64_t)(img / g.wdiv) * g.wstride : 0);
  const bf16* in = reinterpret_cast<const bf16*>(g.in) + (int64_t)img * g.H * g.W * g.ldi + g.offi;
  const bf16* t16 = reinterpret_cast<const bf16*>(g.dww16);
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  // ---- stage DMA: instruction j = wid + 8 i, lane -> stage byte 1024 j + 16 lane: the haloed input
  // tile (row, pixel, chunk position), the bf16 tap table and the fp32 bias; per lane an element
  // offset + a source kind (0 input, 1 taps, 2 bias, 3 zero line) ----
  const char* s_ptr[L::XI];                       // source of K step 0 (zero line: increment 0)
  int s_inc[L::XI];                               // bytes per K step
#pragma unroll
  for (int i = 0; i < L::XI; ++i) {
    const int b = ((wid + DG_NW * i) * 64 + lane) * 16;
    const char* ptr = reinterpret_cast<const char*>(g_zero_dg);
    int inc = 0;
    if (b < L::X_BYTES) {
      const int r = b / (DG_XP * L::PB), p = (b % (DG_XP * L::PB)) / L::PB, pos = (b % L::PB) >> 4;
      const int c = dg_xpos<NH>(p, pos);                  // involution: position <-> chunk
      const int yy = y0 - 1 + r, xx = x0 - 1 + p;
      if (yy >= 0 && yy < g.H && xx >= 0 && xx < g.W) {
        if (g.cb_px) {                                    // channel-blocked: x2 blocks follow the K / 16 x1 blocks
          const int64_t pix = ((int64_t)img * g.H + yy) * g.W + xx;
          ptr = reinterpret_cast<const char*>(reinterpret_cast<const bf16*>(g.in) + (((int64_t)(c >> 1) * (K / DG_KC) * g.cb_px + pix) << 4) +
                                              (c & 1) * 8);
          inc = (int)(g.cb_px * DG_KC * 2);
        } else {
          ptr = reinterpret_cast<const char*>(in + (yy * g.W + xx) * (int)g.ldi + (c >> 1) * K + (c & 1) * 8);
          inc = DG_KC * 2;
        }
      }
    } else if (b < L::B_OFF) {
      const int q = (b - L::T_OFF) >> 4, hh = q / 18, tap = (q % 18) >> 1, piece = q & 1;
      ptr = reinterpret_cast<const char*>(t16 + tap * Cw + hh * K + piece * 8);
      inc = DG_KC * 2;
    } else if (b < L::T_END && g.dwb) {
      const int q = (b - L::B_OFF) >> 4, hh = q >> 2, c4 = (q & 3) * 4;
      ptr = reinterpret_cast<const char*>(g.dwb + hh * K + c4);
      inc = DG_KC * 4;
    }
    if (g.dbg & 4) { ptr = reinterpret_cast<const char*>(g_zero_dg); inc = 0; }
    s_ptr[i] = ptr; s_inc[i] = inc;
  }
  // weights: LDS row r holds channel pi(r), so a tile's fragment rows are contiguous and a lane's
  // accumulators come out as 8 consecutive channels (gemm5.hip permutation)
  int w_off;
  {
    const int b = (wid * 64 + lane) * 16, r = b / 32, piece = (b / 16) & 1;
    const int rt = r & 127, tt = rt >> 4, ii = rt & 15;
    const int n = n0 + (r >> 7) * 128 + 32 * (tt >> 1) + 8 * (ii >> 2) + 4 * (tt & 1) + (ii & 3);
    w_off = n < g.N ? n * (int)g.ldw + (piece ^ dg_h(r)) * 8 : -1;
  }
  auto issue_stage = [&](int kt) {              // K step kt -> X slot kt % 4 (zeros past the last step)
    const uint32_t sS = lds_base + (kt % DG_XSLOTS) * L::STAGE;
    const bool live = kt < nk;
#pragma unroll
    for (int i = 0; i < L::XI; ++i)
      dg_dma16(live ? reinterpret_cast<const void*>(s_ptr[i] + kt * s_inc[i]) : reinterpret_cast<const void*>(g_zero_dg),
               sS + (wid + DG_NW * i) * 1024);
  };
  auto issue_w = [&](int kt) {                  // weights of K step kt -> W slot kt % 5
    const uint32_t sW = lds_base + L::OFF_W + ((kt + DG_WSLOTS) % DG_WSLOTS) * DG_W_BYTES;
    dg_dma16(kt >= 0 && kt < nk && w_off >= 0 && !(g.dbg & 8) ? reinterpret_cast<const void*>(Wp + w_off + kt * DG_KC)
                                                              : reinterpret_cast<const void*>(g_zero_dg),
             sW + wid * 1024);
  };

  // ---- depthwise on the matrix cores: wave = output row wid, two groups of 16 pixels. Per half,
  // D[channel i][pixel j] = sum over k = (tap, c') of A[i][k] B[k][j] with A block-diagonal
  // (A[i][(t, c')] = w_t[i] if c' == i): 5 MFMA 16x16x32 steps cover the 9 taps x 16 channels
  // (tap 9 = zero). A: one bf16 of the staged tap table placed in the lane's fragment; B: a 16-byte
  // read of the staged tile shifted by the tap. No unpacking, no VALU FMAs ----
  const int d_i = lane & 15, d_c8 = (lane >> 4) & 1, d_tl = lane >> 5;
  // per-lane, step-invariant LDS offsets inside a stage: B operand of tap pair ks (half 0, pixel
  // group 0; group 1 is +16 pixels, half 1 the chunk pair ^ 2, i.e. byte ^ 32 for 64-B pixels) and
  // the dword of the bf16 tap table holding this lane's diagonal element (tap 9: the zeroed tail)
  int d_boff[5], d_toff[5];
#pragma unroll
  for (int ks = 0; ks < 5; ++ks) {
    const int tap = min(2 * ks + d_tl, 8), ty_ = tap / 3, tx_ = tap - 3 * ty_;
    const int p = d_i + tx_;
    d_boff[ks] = (wid + ty_) * (DG_XP * L::PB) + p * L::PB + (dg_xpos<NH>(p, d_c8) << 4);
    d_toff[ks] = 2 * ks + d_tl < 9 ? L::T_OFF + ((2 * ks + d_tl) * DG_KC + (d_i & ~1)) * 2 : L::T_END;
  }
  // fragment masks: the lane's bf16 slot (dword (i & 7) >> 1, half i & 1) if it is on the diagonal
  uint32_t d_m[4];
  {
    const bool diag = (d_i >> 3) == d_c8;
    const uint32_t hm = (d_i & 1) ? 0xFFFF0000u : 0x0000FFFFu;
#pragma unroll
    for (int k = 0; k < 4; ++k) d_m[k] = diag && ((d_i & 7) >> 1) == k ? hm : 0u;
  }
  auto dw_step = [&](int kt) {
    const char* sX = smem + (kt % DG_XSLOTS) * L::STAGE;
    const float* bb = reinterpret_cast<const float*>(sX + L::B_OFF);
    f32x4 d[2][NH];                               // [pixel group][half]
#pragma unroll
    for (int hh = 0; hh < NH; ++hh) {
      bf16x8v af[5];
#pragma unroll
      for (int ks = 0; ks < 5; ++ks) {
        const uint32_t w32 = *reinterpret_cast<const uint32_t*>(sX + d_toff[ks] + hh * (9 * DG_KC * 2));
        const uint4 q = make_uint4(w32 & d_m[0], w32 & d_m[1], w32 & d_m[2], w32 & d_m[3]);
        af[ks] = __builtin_bit_cast(bf16x8v, q);
      }
      const f32x4 bias = *reinterpret_cast<const f32x4*>(bb + hh * DG_KC + 4 * (lane >> 4));
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        d[cb][hh] = bias;
#pragma unroll
        for (int ks = 0; ks < 5; ++ks) {
          const int off = (hh ? (d_boff[ks] ^ 32) : d_boff[ks]) + cb * 16 * L::PB;
          const bf16x8v b = *reinterpret_cast<const bf16x8v*>(sX + off);
          d[cb][hh] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks], b, d[cb][hh], 0, 0, 0);
        }
      }
    }
    // lane holds channels 4 (lane >> 4) + e of pixel d_i of each group; pixels outside the image
    // see a zero-filled tile: finite values in A rows whose outputs are never stored
    char* sA = smem + L::OFF_A + (kt % DG_ASLOTS) * DG_A_BYTES;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      uint32_t pk[2];
#pragma unroll
      for (int e2 = 0; e2 < 2; ++e2) {
        f32x2 r = f32x2{d[cb][0][2 * e2], d[cb][0][2 * e2 + 1]};
        if constexpr (NH == 2) r = gelu_bf16_2(r) * f32x2{d[cb][1][2 * e2], d[cb][1][2 * e2 + 1]};   // packed pairs
        const float r0 = r.x, r1 = r.y;
        const uint32_t lo = __builtin_bit_cast(unsigned short, (bf16)r0);
        const uint32_t hi = __builtin_bit_cast(unsigned short, (bf16)r1);
        pk[e2] = lo | (hi << 16);
      }
      const int p = wid * DG_TW + 16 * cb + d_i;
      *reinterpret_cast<uint2*>(sA + p * 32 + (((lane >> 4) ^ (2 * dg_h(p))) << 3)) = make_uint2(pk[0], pk[1]);
    }
  };

  f32x4 acc[4][8];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  // GEMM over the K-step pair (k0, k0 + 1) with full-rate 16x16x32 MFMAs: lanes with fq < 2 read
  // step k0's 16 channels, fq >= 2 step k0 + 1's (A and W slots of their own step)
  auto mfma_pair = [&](int k0) {
    const int kk = k0 + (fq >> 1), hsel = fq & 1;
    const char* sA = smem + L::OFF_A + (kk % DG_ASLOTS) * DG_A_BYTES;
    const char* sW = smem + L::OFF_W + (kk % DG_WSLOTS) * DG_W_BYTES;
    bf16x8v xf[4], wf[8];
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      const int r = wm * 64 + 16 * tt + fr;
      xf[tt] = *reinterpret_cast<const bf16x8v*>(sA + r * 32 + ((hsel ^ dg_h(r)) << 4));
    }
#pragma unroll
    for (int tt = 0; tt < 8; ++tt) {
      const int r = wn * 128 + 16 * tt + fr;
      wf[tt] = *reinterpret_cast<const bf16x8v*>(sW + r * 32 + ((hsel ^ dg_h(r)) << 4));
    }
#pragma unroll
    for (int tm = 0; tm < 4; ++tm)
#pragma unroll
      for (int tn = 0; tn < 8; ++tn) acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[tn], xf[tm], acc[tm][tn], 0, 0, 0);
  };

  // ---- pipeline: step s computes the depthwise of K step s and (s even) the GEMM of the pair
  // (s - 2, s - 1). Step t issues the weights of step t + 2 and the input tile of step t + 3; every
  // wave issues the same number of DMA instructions per step (zero-line fills outside [0, nk)), so
  // the counted wait at the top of a step is a constant: 2 steps x PER_STEP ----
  issue_w(-1); issue_stage(0);
  issue_w(0); issue_stage(1);
  issue_w(1); issue_stage(2);
  for (int s = 0; s <= nk; ++s) {
    dg_wait_vm<2 * L::PER_STEP>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                 // X(s), W(s - 2), W(s - 1), A(s - 2), A(s - 1) ready
    asm volatile("" ::: "memory");
    issue_w(s + 2);
    issue_stage(s + 3);
    if (s >= 2 && !(s & 1) && !(g.dbg & 2)) mfma_pair(s - 2);
    if (s < nk && !(g.dbg & 1)) dw_step(s);
  }
  dg_wait_vm<0>();                                // no LDS-DMA may land after the workgroup ends

  // ---- epilogue: lane holds channels c .. c+7 (c = n0 + 128 wn + 32 j + 8 fq) of tile pixel
  // 64 wm + 16 tm + fr ----
  bf16* o = reinterpret_cast<bf16*>(g.out);
  const bf16* res = reinterpret_cast<const bf16*>(g.res);
  const float* vb = g.bias ? g.bias : g.zeros;
  int64_t mrow[4];
  bool mok[4];
#pragma unroll
  for (int tm = 0; tm < 4; ++tm) {
    const int p = wm * 64 + 16 * tm + fr, yy = y0 + p / DG_TW, xx = x0 + p % DG_TW;
    mok[tm] = yy < g.H && xx < g.W;
    mrow[tm] = ((int64_t)img * g.H + min(yy, g.H - 1)) * g.W + min(xx, g.W - 1);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = n0 + wn * 128 + 32 * j + 8 * fq;
    if (c >= g.N) continue;                       // N % 8 == 0
    float fb[8];
    {
      const f32x4 a = *reinterpret_cast<const f32x4*>(vb + c), b = *reinterpret_cast<const f32x4*>(vb + c + 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) { fb[i] = a[i]; fb[4 + i] = b[i]; }
    }
    uint4 rv[4];
    if (res) {
#pragma unroll
      for (int tm = 0; tm < 4; ++tm) rv[tm] = ld16(res + mrow[tm] * g.ldr + g.offr + c);
    }
#pragma unroll
    for (int tm = 0; tm < 4; ++tm) {
      if (!mok[tm]) continue;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = acc[tm][2 * j + (e >> 2)][e & 3] + fb[e];
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
      if (!(g.dbg & 16)) *reinterpret_cast<bf16x8*>(o + mrow[tm] * g.ldo + g.offo + c) = ov;
    }
  }
}

// Eligible: 16-byte aligned rows, K % 32 == 0 (whole K-step pairs), N % 8 == 0
bool dwgemm_ok(const DwGemmArgs& g) {
  if ((int64_t)g.N * g.ldw >= (int64_t)1 << 31) return false;   // 32-bit weight / input offsets
  if (!g.cb_px && (int64_t)g.H * g.W * g.ldi >= (int64_t)1 << 31) return false;
  if (g.cb_px && ((int64_t)(g.K / DG_KC + 3) * g.cb_px * DG_KC * 2 >= (int64_t)1 << 31 || g.cb_px < (int64_t)g.nimg * g.H * g.W))
    return false;                                 // per-step byte increments stay 32-bit
  if (g.K % (2 * DG_KC) || g.N % 8 || g.K <= 0 || g.N <= 0 || g.H <= 0 || g.W <= 0) return false;
  if (g.ldi % 8 || g.offi % 8 || g.ldw % 8 || g.ldo % 8 || g.offo % 8 || g.wstride % 8) return false;
  if (g.res && (g.ldr % 8 || g.offr % 8 || reinterpret_cast<uintptr_t>(g.res) % 16)) return false;
  if (reinterpret_cast<uintptr_t>(g.in) % 16 || reinterpret_cast<uintptr_t>(g.out) % 16 || reinterpret_cast<uintptr_t>(g.w) % 16)
    return false;
  if (reinterpret_cast<uintptr_t>(g.dww16) % 16 || (g.dwb && reinterpret_cast<uintptr_t>(g.dwb) % 16)) return false;
  if (g.bias && reinterpret_cast<uintptr_t>(g.bias) % 16) return false;
  return g.gate == 0 || g.gate == 1;
}

int64_t dwgemm_blocks(const DwGemmArgs& g) {
  return (int64_t)g.nimg * ((g.H + DG_TH - 1) / DG_TH) * ((g.W + DG_TW - 1) / DG_TW) * ((g.N + DG_BN - 1) / DG_BN);
}

void launch_dwgemm(const DwGemmArgs& g, hipStream_t st) {
  const int64_t nblk = dwgemm_blocks(g);
  if (g.gate) {
    static bool attr = false;
    if (!attr) { hipFuncSetAttribute(reinterpret_cast<const void*>(dwgemm_kernel<2>), hipFuncAttributeMaxDynamicSharedMemorySize, DGL<2>::BYTES); attr = true; }
    hipLaunchKernelGGL(dwgemm_kernel<2>, dim3((unsigned)nblk), dim3(DG_NT), DGL<2>::BYTES, st, g);
  } else {
    static bool attr = false;
    if (!attr) { hipFuncSetAttribute(reinterpret_cast<const void*>(dwgemm_kernel<1>), hipFuncAttributeMaxDynamicSharedMemorySize, DGL<1>::BYTES); attr = true; }
    hipLaunchKernelGGL(dwgemm_kernel<1>, dim3((unsigned)nblk), dim3(DG_NT), DGL<1>::BYTES, st, g);
  }
}

}  // namespace turtle

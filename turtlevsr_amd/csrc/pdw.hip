// Pointwise -> depthwise -> gate in one kernel at width 256 ("pdw"), the first half of a level-3
// GatedFeedForward (turtle_t1_arch.py:159-178) without its hidden map ever reaching HBM:
//
//   G[p][j] = gelu(dw(H1)[p][j]) * dw(H2)[p][j],   H = LN(x) W_in^T (2h channels: H1 | H2)
//
// (dw = depthwise 3x3 + bias, zero padding of H at the image border). G (h channels, bf16) is the
// A operand of project_out, which a GEMM applies with the residual (turtle.cpp). Against the
// project_in GEMM + dwgemm pair this removes the 2h-channel hidden map's HBM round trip (at 1080p
// level 3: 334 MB written and read back per block, 20 blocks per frame).
//
// Structure (MI355X, bf16 operands, fp32 accumulation), one 512-thread block per CU:
//   * tile = 8 output rows x 32 columns; the haloed 10 x 34 input tile (340 pixels, 22 MFMA pixel
//     tiles of 16) stays in REGISTERS for the whole kernel as the B fragments of project_in (wave w
//     holds pixel tiles w, w + 8, w + 16: 96 VGPRs), loaded once; its LayerNorm statistics are
//     taken from those registers (two-pass, exact) - the affine is folded into W_in at pack time;
//   * K step s = 16 hidden channels of H1 and the matching 16 of H2 (32 W_in rows, 16 KB): the rows
//     of step s + 1 go L2 -> LDS by LDS-DMA (two slots) while the block works on step s;
//   * iteration s runs project_in of step s (MFMA 16x16x32, W_in fragments from LDS, pixels from
//     registers; LN epilogue, border pixels forced to 0) into hidden buffer s & 1 - and the depthwise
//     + gate of step s - 1 from the other buffer: wave w = output row w, the 3x3 taps x 16 channels
//     as block-diagonal MFMAs (dwgemm.hip), gelu(x1) x2, 8-byte stores of G. One barrier per step;
//     the two halves are independent, so one wave's MFMAs overlap the other phase's VALU work;
//   * the per-channel tables (LN rowsums / offsets, taps, dw bias) of all steps are staged in LDS
//     once, so the loop's only vector-memory traffic is the W_in DMA and the G stores, both inline
//     asm with hand-counted vmcnt waits (hipcc never sees them, so it never drains vmcnt(0)).
#include "common.h"
#include "kernels.h"

#include <type_traits>

namespace turtle {

__device__ __attribute__((aligned(64))) uint4 g_zero_pd[4];

constexpr int PD_TH = 8, PD_TW = 32, PD_NT = 512, PD_NW = 8;
constexpr int PD_XR = PD_TH + 2, PD_XP = PD_TW + 2, PD_HPX = PD_XR * PD_XP;   // 10 x 34 = 340
constexpr int PD_NTILE = (PD_HPX + 15) / 16;                                  // 22
constexpr int PD_C = 256, PD_KC = 16, PD_PB = 64;
constexpr int PD_HID = PD_HPX * PD_PB;          // 21760 B per hidden buffer
constexpr int PD_W1 = 32 * PD_C * 2;            // 16384 B per W_in slot
constexpr int PD_OFF_W1 = 2 * PD_HID;
constexpr int PD_OFF_DUMMY = PD_OFF_W1 + 2 * PD_W1;   // 64 lanes x 8 B: hidden stores of pad pixels
constexpr int PD_OFF_TAB = PD_OFF_DUMMY + 512;        // then: taps bf16 [9][N1], dw bias, W_in b_ln + b_in fp32 [N1]
int pdw_lds_bytes(int N1) { return PD_OFF_TAB + 9 * N1 * 2 + 2 * N1 * 4; }

// chunk position of 16-byte chunk c of haloed column p (dwgemm.hip dg_xpos<2>: conflict-free
// ds_read_b128 of the depthwise B operand)
TURTLE_DEV int pd_xpos(int p, int c) { return c ^ (((0xFC30 >> (p & 15)) & 1) << 1); }

// LDS-DMA of 64 lanes x 16 B at (wave-uniform base) + (32-bit lane byte offset) -> LDS at M0; the
// SGPR base keeps the per-lane address to one VGPR
TURTLE_DEV void pd_dma16(const void* base, uint32_t voff, uint32_t lds_wave_base) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(base), "s"(lds_wave_base) : "memory");
}
template <int N>
TURTLE_DEV void pd_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}
TURTLE_DEV void pd_store8(void* base, uint32_t voff, uint2 v) {
  asm volatile("global_store_dwordx2 %0, %1, %2" : : "v"(voff), "v"(v), "s"(base) : "memory");
}

// SPLIT = 1: a scheduling barrier keeps project_in(s) and the depthwise(s - 1) apart in each
// iteration; 0 lets hipcc interleave them (A/B switch "pdw_split")
template <int SPLIT>
__global__ __launch_bounds__(PD_NT, 1) void pdw_kernel(PdwArgs g) {
  typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int N1 = g.N1, hh2 = N1 / 2, nk = hh2 / PD_KC;

  // ---- tile: row-major over the image, XCD-aware (consecutive ids on one XCD share halo rows) ----
  const int ntx = (g.W + PD_TW - 1) / PD_TW, nty = (g.H + PD_TH - 1) / PD_TH;
  int lin = blockIdx.x;
  {
    const int nblk = gridDim.x, q = nblk / 8, r = nblk % 8, x = lin % 8, y = lin / 8;
    lin = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;
  }
  const int tx = lin % ntx;
  int t = lin / ntx;
  const int ty = t % nty;
  const int img = t / nty;
  const int x0 = tx * PD_TW, y0 = ty * PD_TH;
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const bf16* W1 = reinterpret_cast<const bf16*>(g.w1);

  // ---- W_in DMA of step s into slot s & 1: instruction d = wid + 8 i covers LDS rows 2d, 2d + 1
  // (row r: 0-15 H1 rows, 16-31 H2 rows; 512 B = 32 chunks, chunk j at position j ^ (r & 15)) ----
  uint32_t w_off[2];                             // byte offsets into W_in of step 0
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int d = wid + PD_NW * i, r = 2 * d + (lane >> 5), pos = lane & 31, j = pos ^ (r & 15);
    const int row = (r < 16 ? r : hh2 + r - 16);
    w_off[i] = (uint32_t)(row * PD_C + j * 8) * 2u;
  }
  // steps past the last one re-load step 0 into the slot nobody reads (uniform DMA count per wave)
  auto issue_w = [&](int s) {
    const uint32_t sW = lds_base + PD_OFF_W1 + (s & 1) * PD_W1;
    const uint32_t so = s < nk ? (uint32_t)s * PD_KC * PD_C * 2u : 0u;
#pragma unroll
    for (int i = 0; i < 2; ++i) pd_dma16(g.w1, so + w_off[i], sW + (wid + PD_NW * i) * 1024);
  };

  // ---- per-channel tables of every step -> LDS (plain loads, drained before the loop) ----
  {
    char* tab = smem + PD_OFF_TAB;
    const int tap_bytes = 9 * N1 * 2;
    const uint32_t* tsrc = reinterpret_cast<const uint32_t*>(g.dww16);
    for (int i = tid; i < tap_bytes / 4; i += PD_NT) reinterpret_cast<uint32_t*>(tab)[i] = tsrc[i];
    float* fb = reinterpret_cast<float*>(tab + tap_bytes);
    for (int i = tid; i < N1; i += PD_NT) {
      fb[i] = g.dwb ? g.dwb[i] : 0.f;
      fb[N1 + i] = g.ln_tb ? g.ln_tb[i] : 0.f;
    }
  }
  issue_w(0);

  // ---- the haloed input tile as project_in B fragments: pixel tile t = wid + 8 u, lane pixel
  // q = 16 t + (lane & 15), K chunk kk: channels 32 kk + 8 (lane >> 4) .. + 7 ----
  const int ntw = wid + 16 < PD_NTILE ? 3 : 2;
  bf16x8v xf[3][8];
  bool pin[3];
  const bf16* xin = reinterpret_cast<const bf16*>(g.x);
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int q = 16 * (wid + 8 * u) + (lane & 15);
    const int r = q / PD_XP, cc = q - r * PD_XP, yy = y0 - 1 + r, xx = x0 - 1 + cc;
    const bool ok = u < ntw && q < PD_HPX && yy >= 0 && yy < g.H && xx >= 0 && xx < g.W;
    pin[u] = ok;
    const bf16* src = ok ? xin + (((int64_t)img * g.H + yy) * g.W + xx) * g.ldx + g.offx + 8 * (lane >> 4)
                         : reinterpret_cast<const bf16*>(g_zero_pd);
#pragma unroll
    for (int kk = 0; kk < 8; ++kk)
      xf[u][kk] = __builtin_bit_cast(bf16x8v, ld16(ok ? src + 32 * kk : src));
  }
  // LayerNorm statistics per pixel (biased variance, eps 1e-5 inside the sqrt: turtle_t1_arch.py:
  // 96-99); the 4 lanes l, l ^ 16, l ^ 32, l ^ 48 hold a pixel's 256 channels
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    float s = 0.f;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk)
#pragma unroll
      for (int e = 0; e < 8; ++e) s += (float)xf[u][kk][e];
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    const float mu = s * (1.f / PD_C);
    float v = 0.f;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = (float)xf[u][kk][e] - mu;
        v = fmaf(d, d, v);
      }
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    const float r = rsqrtf(v * (1.f / PD_C) + 1e-5f);
    // the B fragments become the normalised rows (x - mu) rstd (BiasFree: x rstd), rounded to bf16
    // once - the pn GEMM's LDS panel does the same - so the epilogue is acc + (W_in b_ln + b_in)
    const float sc = pin[u] ? (g.ln ? r : 1.f) : 0.f, sh = pin[u] && g.ln && g.ln_s ? mu : 0.f;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk)
#pragma unroll
      for (int e = 0; e < 8; ++e) xf[u][kk][e] = (bf16)(((float)xf[u][kk][e] - sh) * sc);
    // pin the packed fragments: without this hipcc keeps unpacked copies live into the loop (spills)
    asm volatile("" : "+v"(xf[u][0]), "+v"(xf[u][1]), "+v"(xf[u][2]), "+v"(xf[u][3]), "+v"(xf[u][4]), "+v"(xf[u][5]),
                 "+v"(xf[u][6]), "+v"(xf[u][7]));
  }

  // hidden-tile store offsets (pixel q, chunk (lane >> 4) >> 1, half (lane >> 4) & 1); the pad
  // pixels q >= 340 of the last tile write a dummy LDS slot, so the stores need no branch
  int h_off[3];
  float h_mk[3];
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int q = 16 * (wid + 8 * u) + (lane & 15), cc = q % PD_XP;
    h_off[u] = q < PD_HPX ? q * PD_PB + (pd_xpos(cc, (lane >> 4) >> 1) << 4) + ((lane >> 4) & 1) * 8
                          : PD_OFF_DUMMY + 8 * lane;
    h_mk[u] = pin[u] ? 1.f : 0.f;
  }
  const char* tab = smem + PD_OFF_TAB;
  const float* t_b = reinterpret_cast<const float*>(tab + 9 * N1 * 2);
  const float* t_tb = t_b + N1;

  // ---- project_in of step s into hidden buffer s & 1 (NTW pixel tiles in this wave: a template
  // argument, so the MFMA stream has no branches and the next K chunk's W_in fragments are read
  // while the current chunk's MFMAs run) ----
  const int fr = lane & 15, fq = lane >> 4;
  auto proj = [&](auto ntw_c, int s) {
    constexpr int NTW = decltype(ntw_c)::value;
    const char* sW = smem + PD_OFF_W1 + (s & 1) * PD_W1;
    f32x4 acc[2][NTW];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int u = 0; u < NTW; ++u) acc[m][u] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8v a0 = *reinterpret_cast<const bf16x8v*>(sW + fr * 512 + ((fq ^ fr) << 4));
    bf16x8v a1 = *reinterpret_cast<const bf16x8v*>(sW + (16 + fr) * 512 + ((fq ^ fr) << 4));
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      bf16x8v n0 = a0, n1 = a1;
      if (kk + 1 < 8) {
        const int pos = ((4 * (kk + 1) + fq) ^ fr) << 4;
        n0 = *reinterpret_cast<const bf16x8v*>(sW + fr * 512 + pos);
        n1 = *reinterpret_cast<const bf16x8v*>(sW + (16 + fr) * 512 + pos);
      }
#pragma unroll
      for (int u = 0; u < NTW; ++u) {
        acc[0][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, xf[u][kk], acc[0][u], 0, 0, 0);
        acc[1][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, xf[u][kk], acc[1][u], 0, 0, 0);
      }
      a0 = n0; a1 = n1;
    }
    // epilogue: lane holds hidden channels 4 fq + e of pixel 16 t + fr: H = acc + tb (0 outside
    // the image: the depthwise zero-pads H)
    char* hid = smem + (s & 1) * PD_HID;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int ch = (m ? hh2 : 0) + s * PD_KC + 4 * fq;
      const f32x4 tv = *reinterpret_cast<const f32x4*>(t_tb + ch);
#pragma unroll
      for (int u = 0; u < NTW; ++u) {
        const f32x2 v01 = __builtin_elementwise_fma(f32x2{tv[0], tv[1]}, f32x2{h_mk[u], h_mk[u]}, f32x2{acc[m][u][0], acc[m][u][1]});
        const f32x2 v23 = __builtin_elementwise_fma(f32x2{tv[2], tv[3]}, f32x2{h_mk[u], h_mk[u]}, f32x2{acc[m][u][2], acc[m][u][3]});
        const uint32_t lo = (uint32_t)__builtin_bit_cast(unsigned short, (bf16)v01.x) |
                            ((uint32_t)__builtin_bit_cast(unsigned short, (bf16)v01.y) << 16);
        const uint32_t hi = (uint32_t)__builtin_bit_cast(unsigned short, (bf16)v23.x) |
                            ((uint32_t)__builtin_bit_cast(unsigned short, (bf16)v23.y) << 16);
        *reinterpret_cast<uint2*>(hid + (h_off[u] ^ (m ? 32 : 0))) = make_uint2(lo, hi);
      }
    }
  };

  // ---- depthwise + gate of step s from hidden buffer s & 1 (dwgemm.hip dw_step): wave = output
  // row wid, two groups of 16 pixels; per half D[channel i][pixel j] = sum over (tap, c') of
  // A[i][(tap, c')] B[(tap, c')][j], A block-diagonal, 5 MFMA K steps cover 9 taps x 16 channels ----
  const int d_i = lane & 15, d_c8 = (lane >> 4) & 1, d_tl = lane >> 5;
  int d_boff[5], d_tap[5];
  uint32_t d_tv[5];
#pragma unroll
  for (int ks = 0; ks < 5; ++ks) {
    const int tap = min(2 * ks + d_tl, 8), ty_ = tap / 3, tx_ = tap - 3 * ty_;
    const int p = d_i + tx_;
    d_boff[ks] = (wid + ty_) * (PD_XP * PD_PB) + p * PD_PB + (pd_xpos(p, d_c8) << 4);
    d_tap[ks] = min(2 * ks + d_tl, 8);
    d_tv[ks] = 2 * ks + d_tl < 9 ? 0xFFFFFFFFu : 0u;
  }
  uint32_t d_m[4];
  {
    const bool diag = (d_i >> 3) == d_c8;
    const uint32_t hm = (d_i & 1) ? 0xFFFF0000u : 0x0000FFFFu;
#pragma unroll
    for (int k = 0; k < 4; ++k) d_m[k] = diag && ((d_i & 7) >> 1) == k ? hm : 0u;
  }
  // G store byte offsets from g.out: row y0 + wid, columns x0 + 16 cb + d_i; pixels outside the
  // image write the lane's slot of the 512-byte pad after the map (g.pad_off)
  uint32_t g_off[2];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int yy = y0 + wid, xx = x0 + 16 * cb + d_i;
    const bool ok = yy < g.H && xx < g.W;
    g_off[cb] = ok ? (uint32_t)(((((int64_t)img * g.H + yy) * g.W + xx) * g.ldo + g.offo + 4 * (lane >> 4)) * 2)
                   : (uint32_t)(g.pad_off + 8 * lane);
  }
  auto dwgate = [&](int s) {
    const char* hid = smem + (s & 1) * PD_HID;
    f32x4 d[2][2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int cbase = (hh ? hh2 : 0) + s * PD_KC;
      bf16x8v af[5];
#pragma unroll
      for (int ks = 0; ks < 5; ++ks) {
        const uint32_t w32 = *reinterpret_cast<const uint32_t*>(tab + (d_tap[ks] * N1 + cbase + (d_i & ~1)) * 2) & d_tv[ks];
        const uint4 q = make_uint4(w32 & d_m[0], w32 & d_m[1], w32 & d_m[2], w32 & d_m[3]);
        af[ks] = __builtin_bit_cast(bf16x8v, q);
      }
      const f32x4 bias = *reinterpret_cast<const f32x4*>(t_b + cbase + 4 * (lane >> 4));
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        d[cb][hh] = bias;
#pragma unroll
        for (int ks = 0; ks < 5; ++ks) {
          const int off = (hh ? (d_boff[ks] ^ 32) : d_boff[ks]) + cb * 16 * PD_PB;
          const bf16x8v b = *reinterpret_cast<const bf16x8v*>(hid + off);
          d[cb][hh] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks], b, d[cb][hh], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);         // bound the operand prefetch (register pressure)
    }
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      uint32_t pk[2];
#pragma unroll
      for (int e2 = 0; e2 < 2; ++e2) {
        const f32x2 r = gelu_bf16_2(f32x2{d[cb][0][2 * e2], d[cb][0][2 * e2 + 1]}) * f32x2{d[cb][1][2 * e2], d[cb][1][2 * e2 + 1]};
        pk[e2] = (uint32_t)__builtin_bit_cast(unsigned short, (bf16)r.x) | ((uint32_t)__builtin_bit_cast(unsigned short, (bf16)r.y) << 16);
      }
      pd_store8(g.out, g_off[cb] + (g_off[cb] < (uint32_t)g.pad_off ? (uint32_t)s * PD_KC * 2u : 0u), make_uint2(pk[0], pk[1]));
    }
  };

  // ---- pipeline: iteration s: project_in(s) -> buffer s & 1, depthwise + gate (s - 1) from the
  // other; the W_in DMA of step s + 1 is issued after the barrier. Per wave and iteration the vector
  // memory queue gets 2 DMA then 2 stores, so at the top of iteration s, vmcnt(2) means "the W_in of
  // step s has landed" (the 2 younger ops are the previous iteration's stores) ----
  const bool drain = (g.split & 2) != 0;          // debug: drain every vector-memory op at the barrier
  auto sync = [&] {
    if (drain) pd_wait_vm<0>();
    pd_wait_vm<2>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // one body per tile count: inside it, project_in(s) and the depthwise(s - 1) are one basic block,
  // so the scheduler interleaves the MFMAs of one with the LDS / VALU work of the other
  auto run = [&](auto ntw_c) {
    issue_w(1);
    proj(ntw_c, 0);
    pd_store8(g.out, (uint32_t)g.pad_off + 8 * lane, make_uint2(0u, 0u));   // uniform store count per iteration
    pd_store8(g.out, (uint32_t)g.pad_off + 8 * lane, make_uint2(0u, 0u));
    for (int s = 1; s < nk; ++s) {
      sync();
      issue_w(s + 1);
      proj(ntw_c, s);
      if constexpr (SPLIT) __builtin_amdgcn_sched_barrier(0);
      dwgate(s - 1);
    }
    sync();
    issue_w(nk + 1);
    dwgate(nk - 1);
  };
  pd_wait_vm<0>();
  __syncthreads();                               // tables staged, W_in(0) landed
  if (ntw == 3) run(std::integral_constant<int, 3>{});
  else run(std::integral_constant<int, 2>{});
  pd_wait_vm<0>();                               // no LDS-DMA may land after the workgroup ends
}

bool pdw_ok(const PdwArgs& g) {
  // 32-bit byte offsets into W_in and G (the pad of 64 x 8 bytes follows the map)
  if (g.pad_off < (int64_t)g.nimg * g.H * g.W * g.ldo * 2 || g.pad_off + 512 >= ((int64_t)1 << 31) || g.pad_off % 8) return false;
  if (g.C != PD_C || g.N1 <= 0 || g.N1 % (2 * PD_KC) || g.nimg <= 0 || g.H <= 0 || g.W <= 0) return false;
  if (pdw_lds_bytes(g.N1) > 160 * 1024) return false;
  if (g.ldx % 8 || g.offx % 8 || g.ldo % 4 || g.offo % 4) return false;
  if ((int64_t)g.N1 * PD_C >= (int64_t)1 << 31) return false;
  const uintptr_t al = reinterpret_cast<uintptr_t>(g.x) | reinterpret_cast<uintptr_t>(g.w1) | reinterpret_cast<uintptr_t>(g.dww16);
  if (al % 16 || reinterpret_cast<uintptr_t>(g.out) % 8 || !g.dww16 || !g.out || !g.x || !g.w1) return false;
  return true;
}

int64_t pdw_blocks(const PdwArgs& g) {
  return (int64_t)g.nimg * ((g.H + PD_TH - 1) / PD_TH) * ((g.W + PD_TW - 1) / PD_TW);
}

void launch_pdw(const PdwArgs& g, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(pdw_kernel<0>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(pdw_kernel<1>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  if (g.split & 1) hipLaunchKernelGGL(pdw_kernel<1>, dim3((unsigned)pdw_blocks(g)), dim3(PD_NT), pdw_lds_bytes(g.N1), st, g);
  else hipLaunchKernelGGL(pdw_kernel<0>, dim3((unsigned)pdw_blocks(g)), dim3(PD_NT), pdw_lds_bytes(g.N1), st, g);
}

}  // namespace turtle

// bf16 projection GEMM with 256 x 256 output tiles, eight waves at two per SIMD ("g9" kernel):
// each wave owns 128 pixels x 64 channels (32 accumulator tiles of 16 x 16, 128 registers in the
// accumulation file), so the two waves of a SIMD fill each other's memory-issue gaps in the matrix
// pipe, and one barrier covers 64 MFMAs (1,024 matrix-pipe cycles) of every SIMD.
// (A four-wave 128 x 128-per-wave form - hipBLASLt's tiling - needs all 512 registers of the SIMD;
// hipcc's allocation of it spilled and shuffled the accumulators.)
//
//   out[m][n] = epilogue( sum_k A[m][k] * W[n][k] )        m = pixel, n = output channel
//
// Where it is used: the large plain / LayerNorm-folded 1x1 projections that ran on hipBLASLt
// (latent level: LN project_in 512 -> 2560, LN qkv 512 -> 1536, project_out 1280 -> 512, W_eff
// 512 -> 512 per image; level 3: W_eff 256 -> 256 per image) - turtle_t1_arch.py:159-178, 666-702.
//
// Structure (MI355X, one 512-thread block per CU):
//   * K steps of 32. The block stages a step's A (256 pixel rows x 64 B) and W (256 channel rows x
//     64 B) tiles through registers: each thread issues 4 global_load_dwordx4 three steps before the
//     step's MFMAs and writes them to one of two 32 KB LDS slots a step later (ds_write_b128), so
//     the global loads have a step of MFMAs (~1,000 cycles) to land; nothing is asm: hipcc counts
//     every vmcnt / lgkmcnt itself (no hand-counted waits);
//   * per step: one barrier, then the next step's 16 fragments are read from the other slot while
//     the 64 MFMAs of this step run (fragment registers double-buffered);
//   * LDS rows of 64 B (32 k): 16-byte chunk c of row r sits at position c ^ ((r >> 2) & 2), which
//     makes the 16-row fragment reads (ds_read_b128) and the staging writes (ds_write_b128)
//     conflict-free on gfx950's lane groups (exhaustive check over the lane groups of both);
//   * weight rows are placed in pn's permuted order (MFMA row 4g+e of sub-tile s <- channel 8g+4s+e
//     of a 32-channel group), so a lane's accumulators of two sub-tiles are 8 CONSECUTIVE channels of
//     one pixel: 16-byte residual loads and stores;
//   * LayerNorm (turtle_t1_arch.py:83-112) folded into the epilogue: W' = W diag(g), s = rowsum(W'),
//     t = W b, and out = rs (acc - mu s) + t + bias with the per-pixel (mu, rs) of a small statistics
//     pass (ln_stats_kernel below, two-pass variance like the reference) - no normalised copy of the
//     activations (the hipBLASLt path wrote one);
//   * XCD-aware tile order: the channel tiles of one pixel panel run on one XCD (shared A panel in L2).
#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace turtle {

namespace {

constexpr int G9_BK = 32;
#ifndef G9_SCHED
#define G9_SCHED 1              // interleave the step's memory operations with its MFMAs (sched groups)
#endif

// MFMA row -> channel inside a 32-channel group (see header)
TURTLE_DEV int g9_perm(int r) { return (r & ~31) | (8 * ((r >> 2) & 3) + 4 * ((r >> 4) & 1) + (r & 3)); }
// byte offset of 16-byte chunk c of LDS row r (64-byte rows, swizzled)
TURTLE_DEV int g9_off(int r, int c) { return r * 64 + ((c ^ ((r >> 2) & 2)) << 4); }

__device__ __attribute__((aligned(64))) uint4 g_zero_g9[4];

// 64 lanes x 16 B -> LDS at M0 (inline asm: hipcc would treat the builtin as an LDS write it must
// drain before every ds_read); M0 is compiler-reserved, so it is restored
TURTLE_DEV void g9_dma16(const void* gp, uint32_t lds_wave_base) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gp), "s"(lds_wave_base) : "memory");
}
template <int N>
TURTLE_DEV void g9_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

}  // namespace

// DBG (tools/g9bench ablations only; 0 in the library): 1 no MFMA, 2 no global loads in the loop,
// 4 no LDS traffic in the loop, 16 no epilogue stores
// MS: K-concatenated multi-source operand (per-step source selection); single source otherwise
// BN: channels per block tile (256: 8 waves, one block per CU; 128: 4 waves, two blocks per CU, so
// one block's epilogue stores overlap the other's main loop)
// NSL: 0 - K steps staged through registers (global_load + ds_write), two LDS slots; 3 / 4 - staged
// by LDS-DMA (global_load_lds_dwordx4: no VGPR round trip, no ds_write) into a ring of NSL slots,
// NSL - 2 steps in flight, waits counted by hand (the loop issues no other vector-memory operation)
template <bool LN, bool MS, int BN, int NSL = 0, int DBG = 0>
__global__ __launch_bounds__(BN * 2, 2) void gemm9_kernel(GemmArgs g, const float2* __restrict__ stats) {
  constexpr int NT = BN * 2;                        // threads: 2 pixel halves x BN / 64 channel groups of waves
  constexpr int NWV = NT / 64;                      // waves
  constexpr int WOFF = 16384;                       // W tile offset in a slot (A: 256 rows x 64 B)
  constexpr int SLOT = WOFF + BN * 64;
  constexpr int NA = 1024 / NT, NW = BN * 4 / NT;   // staged 16-byte chunks per thread and step
  constexpr int NPW = (16 + BN / 16) / NWV;         // LDS-DMA: 1-KB pieces per wave and step
  constexpr int NSLOT = NSL ? NSL : 2;
  static_assert(NSL == 0 || NSL == 3 || NSL == 4, "ring depth");
  __shared__ __attribute__((aligned(16))) char smem[NSLOT * SLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid & 1, wn = wid >> 1;            // pixel half (128 rows), channel group (64)
  const int fr = lane & 15, fq = lane >> 4;

  // ---- tile: the channel tiles of one pixel panel are consecutive ids on one XCD ----
  const int ntn = (g.N + BN - 1) / BN;
  int lin = blockIdx.x;
  {
    const int nblk = gridDim.x, q = nblk / 8, r = nblk % 8, x = lin % 8, y = lin / 8;
    lin = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;
  }
  const int nt = lin % ntn, mt = lin / ntn;
  int64_t m0, mlim;
  if (g.wstride) {                                  // per-image weight sets: tiles never straddle images
    const int tpi = (g.HW + 255) / 256;
    const int64_t im = mt / tpi;
    m0 = im * g.HW + (int64_t)(mt % tpi) * 256;
    mlim = min(g.M, (im + 1) * (int64_t)g.HW);
  } else {
    m0 = (int64_t)mt * 256;
    mlim = g.M;
  }
  const int n0 = nt * BN;
  const int K = g.a.Ktot, nk = K / G9_BK;
  const bf16* Wp = reinterpret_cast<const bf16*>(g.w) + (g.wstride ? (int64_t)(m0 / g.HW / g.wdiv) * g.wstride : 0);

  // ---- staging geometry: thread loads chunk c = tid & 3 of A rows tid / 4 + (NT / 4) i (i < NA)
  // and W rows tid / 4 + (NT / 4) i (i < NW) ----
  const int sc = tid & 3, sr0 = tid >> 2;
  int64_t xrow[NA];                                 // clamped pixel rows
  const bf16* xp0[NA];                              // single source: row pointers
  int soff[NA];                                     // swizzled LDS offsets
  const bf16* wrow[NW];                             // weight rows (permuted, clamped)
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int r = sr0 + (NT / 4) * i;
    const int64_t m = m0 + r;
    xrow[i] = m < mlim ? m : m0;
    xp0[i] = reinterpret_cast<const bf16*>(g.a.s[0].base) + g.a.s[0].off + sc * 8 + (MS ? 0 : xrow[i] * g.a.s[0].ld);
    soff[i] = g9_off(r, sc);
  }
#pragma unroll
  for (int i = 0; i < NW; ++i) wrow[i] = Wp + (int64_t)min(n0 + g9_perm(sr0 + (NT / 4) * i), g.N - 1) * g.ldw + sc * 8;
  uint4 ga[NA], gw[NW];                             // one staged K step
  auto gload = [&](int t) __attribute__((always_inline)) {
    if constexpr ((DBG & 2) != 0) return;
    const int k0 = t * G9_BK;
    if constexpr (!MS) {
#pragma unroll
      for (int i = 0; i < NA; ++i) ga[i] = ld16(xp0[i] + k0);
    } else {
      // the K step's source (steps never straddle two: every source is a multiple of 32 wide)
      const bf16* base = reinterpret_cast<const bf16*>(g.a.s[0].base);
      int64_t sld = g.a.s[0].ld;
      int soffs = g.a.s[0].off, kb = 0, kbj = g.a.s[0].K;
#pragma unroll
      for (int j = 1; j < TURTLE_MAX_SRC; ++j) {
        const bool hit = j < g.a.n && k0 >= kbj;
        base = hit ? reinterpret_cast<const bf16*>(g.a.s[j].base) : base;
        sld = hit ? g.a.s[j].ld : sld;
        soffs = hit ? g.a.s[j].off : soffs;
        kb = hit ? kbj : kb;
        kbj += j < g.a.n ? g.a.s[j].K : 0;
      }
      const bf16* b2 = base + soffs + (k0 - kb) + sc * 8;
#pragma unroll
      for (int i = 0; i < NA; ++i) ga[i] = ld16(b2 + xrow[i] * sld);
    }
#pragma unroll
    for (int i = 0; i < NW; ++i) gw[i] = ld16(wrow[i] + k0);
  };
  auto swrite = [&](int slot) __attribute__((always_inline)) {
    if constexpr ((DBG & 4) != 0) return;
    char* sb = smem + slot * SLOT;
#pragma unroll
    for (int i = 0; i < NA; ++i) *reinterpret_cast<uint4*>(sb + soff[i]) = ga[i];
#pragma unroll
    for (int i = 0; i < NW; ++i) *reinterpret_cast<uint4*>(sb + WOFF + soff[i]) = gw[i];
  };
  // LDS-DMA geometry: piece q = wid + NWV i of a slot is 1 KB = 16 LDS rows of 64 B (A rows for
  // q < 16, then W rows); lane l fills row 16 q + l / 4, position l % 4, which holds source chunk
  // (l % 4) ^ swz(row) - the swizzle goes on the source address (the LDS side is lane-linear)
  const bf16* dsrc[NPW];                            // step-0 source of each piece (A single source / W)
  int64_t drow[NPW];                                // A pixel row (multi-source A)
  int dck[NPW];                                     // source chunk (elements)
  bool disa[NPW];
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
#pragma unroll
  for (int i = 0; i < NPW; ++i) {
    const int q = wid + NWV * i;
    const int r = 16 * (q < 16 ? q : q - 16) + (lane >> 2);
    const int c = ((lane & 3) ^ ((r >> 2) & 2)) * 8;
    disa[i] = q < 16;
    dck[i] = c;
    if (q < 16) {
      const int64_t m = m0 + r;
      drow[i] = m < mlim ? m : m0;
      dsrc[i] = reinterpret_cast<const bf16*>(g.a.s[0].base) + g.a.s[0].off + c + (MS ? 0 : drow[i] * g.a.s[0].ld);
    } else {
      drow[i] = 0;
      dsrc[i] = Wp + (int64_t)min(n0 + g9_perm(r), g.N - 1) * g.ldw + c;
    }
  }
  // K step t -> slot `slot` (past the last step: the zero line, so every step issues NPW pieces)
  auto dma = [&](int t, int slot) __attribute__((always_inline)) {
    if constexpr ((DBG & 2) != 0) return;
    const int k0 = t * G9_BK;
    const bool live = t < nk;
    const bf16* base = nullptr;
    int64_t sld = 0;
    int kb = 0;
    if constexpr (MS) {
      base = reinterpret_cast<const bf16*>(g.a.s[0].base) + g.a.s[0].off;
      sld = g.a.s[0].ld;
      int kbj = g.a.s[0].K;
#pragma unroll
      for (int j = 1; j < TURTLE_MAX_SRC; ++j) {
        const bool hit = j < g.a.n && k0 >= kbj;
        base = hit ? reinterpret_cast<const bf16*>(g.a.s[j].base) + g.a.s[j].off : base;
        sld = hit ? g.a.s[j].ld : sld;
        kb = hit ? kbj : kb;
        kbj += j < g.a.n ? g.a.s[j].K : 0;
      }
    }
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
      const bf16* src;
      if (MS && disa[i]) src = base + drow[i] * sld + (k0 - kb) + dck[i];
      else src = dsrc[i] + k0;
      uint64_t pa = reinterpret_cast<uint64_t>(src);
      asm volatile("" : "+v"(pa));                   // computed for every lane, then selected (no branch)
      g9_dma16(live ? reinterpret_cast<const void*>(pa) : reinterpret_cast<const void*>(g_zero_g9),
               lds_base + slot * SLOT + (wid + NWV * i) * 1024);
    }
  };

  // fragment reads: rows wm*128 + 16 i + fr of A, wn*64 + 16 j + fr of W; chunk fq
  const int foff = g9_off(fr, fq);                  // (rows of a fragment start at multiples of 16)
  const char* fa_base = smem + (wm * 128) * 64 + foff;
  const char* fw_base = smem + WOFF + (wn * 64) * 64 + foff;
  auto rd = [&](const char* p) __attribute__((always_inline)) {
    if constexpr ((DBG & 4) != 0) {
      bf16x8 z;
#pragma unroll
      for (int e = 0; e < 8; ++e) z[e] = (bf16)(float)(lane + e);
      return z;
    }
    return *reinterpret_cast<const bf16x8*>(p);
  };
  bf16x8 fa[8], fw[2][4];                           // A: one set, refilled row by row; W: two sets

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- pipeline. At step t (W register set b = t & 1):
  //   barrier: slot (t+1)&1 holds step t+1 (written at step t-1), every read of slot t&1 is done
  //   W fragments of step t+1 -> set b^1 (from slot (t+1)&1)
  //   MFMA row i of step t (4 MFMAs on A_i), then A_i <- step t+1's (its last use is behind it)
  //   slot t&1 <- staged step t+2; staged <- global loads of step t+3 (a step of MFMAs to land)
  // K % 64 == 0 (gemm9_ok): nk is even, the loop is unrolled by two and every set index static.
  auto step = [&](int t, auto B, auto WRITE, auto LOAD) __attribute__((always_inline)) {
    constexpr int b = decltype(B)::value;
    const int nslot = ((t + 1) & 1) * SLOT;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) fw[b ^ 1][j] = rd(fw_base + nslot + 16 * j * 64);
    if constexpr (decltype(WRITE)::value) swrite(t & 1);
    if constexpr (decltype(LOAD)::value) gload(t + 3);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr ((DBG & 1) == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[b][j], fa[i], acc[i][j], 0, 0, 0);
      }
      fa[i] = rd(fa_base + nslot + 16 * i * 64);
    }
    // issue order: the memory operations one per MFMA gap - the next W fragments, the LDS writes,
    // the global loads - then the next A fragments each behind the last MFMA of its row
    if constexpr (G9_SCHED && (DBG & 7) == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) { __builtin_amdgcn_sched_group_barrier(0x008, 1, 0); __builtin_amdgcn_sched_group_barrier(0x100, 1, 0); }
      if constexpr (decltype(WRITE)::value) {
#pragma unroll
        for (int k = 0; k < NA + NW; ++k) { __builtin_amdgcn_sched_group_barrier(0x008, 1, 0); __builtin_amdgcn_sched_group_barrier(0x200, 1, 0); }
      }
      if constexpr (decltype(LOAD)::value) {
#pragma unroll
        for (int k = 0; k < NA + NW; ++k) { __builtin_amdgcn_sched_group_barrier(0x008, 1, 0); __builtin_amdgcn_sched_group_barrier(0x020, 1, 0); }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) { __builtin_amdgcn_sched_group_barrier(0x008, 2, 0); __builtin_amdgcn_sched_group_barrier(0x100, 1, 0); }
    }
  };
  // LDS-DMA ring: at step t - wait for own pieces of step t+1 (NSL-3 steps stay in flight),
  // barrier (everyone's step t+1 landed; every read of step t-1's slot retired at step t-1's MFMAs),
  // step t+NSL-1 -> that slot, fragments of step t+1, 64 MFMAs of step t
  auto step_dma = [&](int t, auto B) __attribute__((always_inline)) {
    constexpr int b = decltype(B)::value;
    g9_vm<(NSLOT - 3) * NPW>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    dma(t + NSLOT - 1, (t + NSLOT - 1) % NSLOT);
    const int nslot = ((t + 1) % NSLOT) * SLOT;
#pragma unroll
    for (int j = 0; j < 4; ++j) fw[b ^ 1][j] = rd(fw_base + nslot + 16 * j * 64);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr ((DBG & 1) == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[b][j], fa[i], acc[i][j], 0, 0, 0);
      }
      fa[i] = rd(fa_base + nslot + 16 * i * 64);
    }
    if constexpr (G9_SCHED && (DBG & 7) == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) { __builtin_amdgcn_sched_group_barrier(0x008, 1, 0); __builtin_amdgcn_sched_group_barrier(0x100, 1, 0); }
#pragma unroll
      for (int k = 0; k < 8; ++k) { __builtin_amdgcn_sched_group_barrier(0x008, 3, 0); __builtin_amdgcn_sched_group_barrier(0x100, 1, 0); }
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using T_ = std::true_type;
  using F_ = std::false_type;
  if constexpr (NSL > 0) {
    for (int s0 = 0; s0 < NSLOT - 1; ++s0) dma(s0, s0);
    g9_vm<(NSLOT - 2) * NPW>();                     // step 0 landed
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < 4; ++j) fw[0][j] = rd(fw_base + 16 * j * 64);
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[i] = rd(fa_base + 16 * i * 64);
    for (int t = 0; t < nk; t += 2) {
      step_dma(t, I0{});
      step_dma(t + 1, I1{});
    }
    g9_vm<0>();                                     // the zero-line pieces past the end have landed
  } else {
  // prologue: steps 0, 1 -> slots 0, 1; step 2 staged; fragments of step 0
  gload(0);
  swrite(0);
  gload(1);
  swrite(1);
  gload(2);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) fw[0][j] = rd(fw_base + 16 * j * 64);
#pragma unroll
  for (int i = 0; i < 8; ++i) fa[i] = rd(fa_base + 16 * i * 64);
  int t = 0;
  for (; t + 4 < nk; t += 2) {                      // every step that stages t+2 and loads t+3
    step(t, I0{}, T_{}, T_{});
    step(t + 1, I1{}, T_{}, T_{});
  }
  // last four steps (nk even, >= 4): t = nk-4 stages nk-2 and loads nk-1; nk-3 stages nk-1
  step(t, I0{}, T_{}, T_{});
  step(t + 1, I1{}, T_{}, F_{});
  step(t + 2, I0{}, F_{}, F_{});
  step(t + 3, I1{}, F_{}, F_{});
  }

  // ---- epilogue: lane holds channels c .. c+7 (c = n0 + 64 wn + 32 s + 8 fq) of pixel rows
  // m0 + 128 wm + 16 i + fr (sub-tiles 2s, 2s+1 of the permuted weight rows) ----
  bf16* o = reinterpret_cast<bf16*>(g.out);
  const bf16* res = reinterpret_cast<const bf16*>(g.res);
  const float* vs = g.ln_s ? g.ln_s : g.zeros;
  const float* vt = g.ln_t ? g.ln_t : g.zeros;
  const float* vb = g.bias ? g.bias : g.zeros;
  const float* vc = g.scale ? g.scale : g.ones;
  float mu[8], rs[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int64_t m = m0 + wm * 128 + 16 * i + fr;
    if constexpr (LN) {
      const uint2 q = ld8(stats + (m < mlim ? m : m0));
      mu[i] = __uint_as_float(q.x); rs[i] = __uint_as_float(q.y);
    } else {
      mu[i] = 0.f; rs[i] = 1.f;
    }
  }
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int c = n0 + wn * 64 + 32 * s + 8 * fq;   // (N % 8 == 0)
    if (c >= g.N) continue;                         // N % 8 == 0: a group of 8 is all in or all out
    float fs[8], ft[8], fc[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(vs + c + 4 * h), bb = *reinterpret_cast<const f32x4*>(vt + c + 4 * h);
      const f32x4 d = *reinterpret_cast<const f32x4*>(vb + c + 4 * h), e = *reinterpret_cast<const f32x4*>(vc + c + 4 * h);
#pragma unroll
      for (int q = 0; q < 4; ++q) { fs[4 * h + q] = a[q]; ft[4 * h + q] = bb[q] + d[q]; fc[4 * h + q] = e[q]; }
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
      const int64_t m = m0 + wm * 128 + 16 * i + fr;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float x = acc[i][2 * s + (e >> 2)][e & 3];
        if constexpr (LN) x = rs[i] * (x - mu[i] * fs[e]);
        x += ft[e];
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
      if (m >= mlim) continue;
      const int64_t dst = g.store_mode == STORE_CB16 ? ((((int64_t)(c >> 4) * g.cb_px + m) << 4) + (c & 15)) : m * g.ldo + g.offo + c;
      if constexpr (!(DBG & 16)) *reinterpret_cast<bf16x8*>(o + dst) = ov;
      else if (v[0] == 1.2345f) o[tid] = ov[0];
    }
  }
}

// Per-pixel LayerNorm statistics (mu, 1 / sqrt(var + 1e-5)) of a [M][ld] bf16 map's K channels at
// offset `off` (turtle_t1_arch.py:94-99: biased variance about the mean, two passes in registers):
// 8 lanes per pixel, K / 64 16-byte chunks each, an 8-lane DPP reduction.
template <int K>
__global__ __launch_bounds__(256) void ln_stats_kernel(const bf16* __restrict__ x, int64_t ld, int off, int64_t M, float2* __restrict__ out) {
  constexpr int CPL = K / 64;
  const int tid = threadIdx.x, cc = tid & 7;
  const int64_t p = (int64_t)blockIdx.x * 32 + (tid >> 3);
  const int64_t pc = p < M ? p : M - 1;
  const bf16* src = x + pc * ld + off + cc * 8;
  uint4 v[CPL];
#pragma unroll
  for (int q = 0; q < CPL; ++q) v[q] = ld16(src + q * 64);
  auto sum8 = [](float s) __attribute__((always_inline)) {
    s += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, s), 0xB1, 0xf, 0xf, false));   // xor 1
    s += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, s), 0x4E, 0xf, 0xf, false));   // xor 2
    s += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, s), 0x141, 0xf, 0xf, false));  // half mirror
    return s;
  };
  float sm = 0.f;
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    Vec<bf16> vv; vv.from_raw(v[q]);
#pragma unroll
    for (int e = 0; e < 8; ++e) sm += vv.v[e];
  }
  const float mu = sum8(sm) * (1.f / K);
  float sq = 0.f;
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    Vec<bf16> vv; vv.from_raw(v[q]);
#pragma unroll
    for (int e = 0; e < 8; ++e) { const float d = vv.v[e] - mu; sq = fmaf(d, d, sq); }
  }
  const float rstd = rsqrtf(sum8(sq) * (1.f / K) + 1e-5f);
  if (cc == 0 && p < M) out[p] = float2{mu, rstd};
}

// Eligible: bf16, one LN source or K-concatenated plain sources (each a multiple of 32 wide, img_mul
// 1 / img_add 0), K % 64 == 0 and 128 <= K <= 4096, NHWC or channel-blocked store, N % 8 == 0, 16-byte
// aligned rows, no 3x3 / shuffle stores. LN needs K in {256, 512, 1024} (the statistics kernel).
bool gemm9_ok(const GemmArgs& g) {
  if (!g.allow_g9 || g.conv3 || g.a.cb_px || (g.store_mode != STORE_NHWC && g.store_mode != STORE_CB16)) return false;
  if (g.store_mode == STORE_CB16 && (g.cb_px < g.M || g.N % 16 || g.wstride)) return false;
  const int K = g.a.Ktot;
  if (K % 64 || K < 128 || K > 4096 || g.N % 8 || g.ldo % 8 || g.offo % 8 || g.ldw % 8 || g.a.n < 1) return false;
  if (g.ln && (g.a.n != 1 || (K != 256 && K != 512 && K != 1024))) return false;
  if (g.res && (g.ldr % 8 || g.offr % 8 || reinterpret_cast<uintptr_t>(g.res) % 16)) return false;
  if (reinterpret_cast<uintptr_t>(g.out) % 16 || reinterpret_cast<uintptr_t>(g.w) % 16) return false;
  if (g.wstride && (g.HW <= 0 || g.M % g.HW || g.wstride % 8)) return false;
  if (g.M > INT32_MAX) return false;
  for (int j = 0; j < g.a.n; ++j) {
    const SrcDesc& s = g.a.s[j];
    if (s.img_mul != 1 || s.img_add != 0 || s.K % 32 || s.ld % 8 || s.off % 8 || reinterpret_cast<uintptr_t>(s.base) % 16) return false;
  }
  return true;
}

size_t gemm9_stats_bytes(const GemmArgs& g) { return g.ln ? (size_t)g.M * sizeof(float2) : 0; }

// `stats`: workspace of gemm9_stats_bytes(g) (LN GEMMs), filled here before the GEMM
template <int BN, int NSL>
static void g9_launch(const GemmArgs& g, float2* sp, hipStream_t st) {
  const int64_t mt = g.wstride ? (g.M / g.HW) * ((g.HW + 255) / 256) : (g.M + 255) / 256;
  const dim3 grid((unsigned)(mt * ((g.N + BN - 1) / BN))), blk(2 * BN);
  if (g.ln) hipLaunchKernelGGL((gemm9_kernel<true, false, BN, NSL>), grid, blk, 0, st, g, sp);
  else if (g.a.n > 1) hipLaunchKernelGGL((gemm9_kernel<false, true, BN, NSL>), grid, blk, 0, st, g, sp);
  else hipLaunchKernelGGL((gemm9_kernel<false, false, BN, NSL>), grid, blk, 0, st, g, sp);
}
// g.allow_g9: 1 the measured choice per shape; 2..6 a fixed variant (tools/g9bench):
// 2 BN 256 register-staged, 3 BN 128 register-staged, 4 BN 256 DMA ring 4, 5 BN 128 DMA ring 3,
// 6 BN 256 DMA ring 3
// per-pixel (mu, rstd) of the LN source a.s[0] (K in {256, 512, 1024}) into sp[M]; also the split-K
// GEMM's statistics (gemm_sk.hip)
void launch_ln_stats(const GemmArgs& g, float2* sp, hipStream_t st) {
  const SrcDesc& s = g.a.s[0];
  const bf16* x = reinterpret_cast<const bf16*>(s.base);
  const dim3 gs((unsigned)((g.M + 31) / 32));
  if (g.a.Ktot == 256) hipLaunchKernelGGL((ln_stats_kernel<256>), gs, dim3(256), 0, st, x, s.ld, s.off, g.M, sp);
  else if (g.a.Ktot == 512) hipLaunchKernelGGL((ln_stats_kernel<512>), gs, dim3(256), 0, st, x, s.ld, s.off, g.M, sp);
  else hipLaunchKernelGGL((ln_stats_kernel<1024>), gs, dim3(256), 0, st, x, s.ld, s.off, g.M, sp);
}

void launch_gemm9(const GemmArgs& g, void* stats, hipStream_t st) {
  float2* sp = reinterpret_cast<float2*>(stats);
  if (g.ln) launch_ln_stats(g, sp, st);
  int v = g.allow_g9;
  if (v == 1) {
    // 256 channels on the LDS-DMA ring wherever every CU still gets a tile (the A panel is read
    // half as often; fastest on the latent shapes, tools/g9bench), else - and for the K = 256, N = 256
    // level-3 W_eff (47.8 vs 51.5 us, profiles/r05a_g9bench.log) - 128 register-staged
    const int64_t mt = g.wstride ? (g.M / g.HW) * ((g.HW + 255) / 256) : (g.M + 255) / 256;
    v = g.N % 256 == 0 && mt * (g.N / 256) >= 256 && !(g.a.Ktot <= 256 && g.N <= 256) ? 4 : 3;
  }
  switch (v) {
    case 2: g9_launch<256, 0>(g, sp, st); break;
    case 4: g9_launch<256, 4>(g, sp, st); break;
    case 5: g9_launch<128, 3>(g, sp, st); break;
    case 6: g9_launch<256, 3>(g, sp, st); break;
    default: g9_launch<128, 0>(g, sp, st);
  }
}

#ifdef TURTLE_G9_ABLATIONS
template <int DBG, int BN, int NSL>
static void g9_launch_dbg(const GemmArgs& g, void* stats, hipStream_t st) {
  const dim3 grid((unsigned)(((g.M + 255) / 256) * ((g.N + BN - 1) / BN))), blk(2 * BN);
  float2* sp = reinterpret_cast<float2*>(stats);
  if (g.ln) hipLaunchKernelGGL((gemm9_kernel<true, false, BN, NSL, DBG>), grid, blk, 0, st, g, sp);
  else if (g.a.n > 1) hipLaunchKernelGGL((gemm9_kernel<false, true, BN, NSL, DBG>), grid, blk, 0, st, g, sp);
  else hipLaunchKernelGGL((gemm9_kernel<false, false, BN, NSL, DBG>), grid, blk, 0, st, g, sp);
}
template <int DBG>
static void g9_dbg2(const GemmArgs& g, void* stats, hipStream_t st) {
  switch (g.allow_g9) {
    case 2: g9_launch_dbg<DBG, 256, 0>(g, stats, st); break;
    case 4: g9_launch_dbg<DBG, 256, 4>(g, stats, st); break;
    case 5: g9_launch_dbg<DBG, 128, 3>(g, stats, st); break;
    case 6: g9_launch_dbg<DBG, 256, 3>(g, stats, st); break;
    default: g9_launch_dbg<DBG, 128, 0>(g, stats, st);
  }
}
void launch_gemm9_dbg(const GemmArgs& g, void* stats, int dbg, hipStream_t st) {
  switch (dbg) {
    case 1: g9_dbg2<1>(g, stats, st); break;
    case 2: g9_dbg2<2>(g, stats, st); break;
    case 4: g9_dbg2<4>(g, stats, st); break;
    case 16: g9_dbg2<16>(g, stats, st); break;
    case 22: g9_dbg2<22>(g, stats, st); break;
    default: g9_dbg2<0>(g, stats, st);
  }
}
#endif

}  // namespace turtle

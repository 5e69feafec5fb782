// fp32 GEMM on the matrix cores for the fp32 build (config 3: Davis 540p fp32; the parity runs):
// the arguments, operand addressing and epilogue of gemm_kernel<float> (gemm.hip: K-concatenated
// sources, implicit 3x3, per-image weights, folded LayerNorm, bias / GELU / scale / residual, plain
// / PixelShuffle / PixelUnshuffle stores), re-tiled for v_mfma_f32_16x16x4f32 occupancy:
//
//   * block = 256 threads (2 x 2 waves), tile 128 pixels x BN channels, BK = 16 floats (64-B LDS
//     rows, chunk positions swizzled per row: conflict-free ds_read_b128 fragment reads);
//   * K permuted inside a tile: MFMA step s of lane group q takes k = 4q + s, so one ds_read_b128
//     per fragment row feeds four MFMA steps (the sum over k is the same set);
//   * operands go HBM/L2 -> LDS by LDS-DMA (global_load_lds_dwordx4, no register staging) into a
//     3-stage ring issued two K tiles ahead, one barrier per K tile, counted vmcnt waits: the
//     generic kernel's one-tile register prefetch left the MFMAs waiting on HBM latency (both it and
//     a double-buffered register-prefetch form of this kernel ran at ~82 TF/s on the K = 256 LN
//     projections, profiles/r05u_f32bench.log);
//   * epilogue straight from the accumulators: a lane holds 4 consecutive output channels of one
//     pixel (16-byte residual loads and stores), a row's residual loads issued before its stores.
#include "common.h"
#include "kernels.h"

namespace turtle {

__device__ __attribute__((aligned(64))) uint4 g_zero_f32[4];

constexpr int F32_BM = 128, F32_BK = 16, F32_ROW = F32_BK * 4;   // 64-byte LDS rows

// 16-byte position of chunk c in 64-byte row r: c ^ h((r >> 2) & 3) with h = {0, 2, 3, 1}. The
// fragment read (lane = row fr, chunk fq) is a ds_read_b128, serviced in the lane groups {0-3, 12-15,
// 20-27}, {4-11, 16-19, 28-31} (+ 32): with this h each group's 16 lanes hit 16 distinct 16-byte
// bank slots (4 (r mod 4) + position) - the plain c ^ ((r >> 2) & 3) put two lanes on each slot
TURTLE_DEV int f32_pos(int r, int c) { return c ^ ((0x78 >> (2 * ((r >> 2) & 3))) & 3); }

// one LDS-DMA wave instruction: 64 lanes x 16 B -> LDS at M0 + 16 lane (as dg_dma16, dwgemm.hip)
TURTLE_DEV void f32_dma16(const void* g, uint32_t lds_wave_base) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(lds_wave_base) : "memory");
}
template <int N>
TURTLE_DEV void f32_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

template <int BN, int NS>
struct F32L {
  static constexpr int STAGE = (F32_BM + BN) * F32_ROW;   // pixel rows then weight rows
  static constexpr int NI = (F32_BM + BN) / 64;           // LDS-DMA instructions per wave per stage
  static constexpr int VEC_OFF = NS * STAGE;
  static constexpr int BYTES = VEC_OFF + 2 * F32_BM * 4 + 4 * BN * 4;
  static_assert(BYTES <= 160 * 1024, "gemm_f32 LDS budget");
};

template <int BN, int NS>
__global__ __launch_bounds__(256, NS == 3 ? 3 : 2) void gemm_f32_kernel(GemmArgs g) {
  using L = F32L<BN, NS>;
  constexpr int BM = F32_BM, BK = F32_BK, STAGE = L::STAGE, NI = L::NI;
  constexpr int TM = BM / 32, TN = BN / 32;            // 16x16 tiles per wave (wave tile 64 x BN/2)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_mu = reinterpret_cast<float*>(smem + L::VEC_OFF);
  float* s_rs = s_mu + BM;
  float* e_s = s_rs + BM;                              // [BN] each: ln_s, ln_t, bias, scale
  float* e_t = e_s + BN;
  float* e_b = e_t + BN;
  float* e_c = e_b + BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int fr = lane & 15, fq = lane >> 4;

  // ---- block -> (pixel tile, channel tile): channel tiles fastest, XCD-contiguous ids ----
  const int ntn = (g.N + BN - 1) / BN;
  int lin = blockIdx.x;
  {
    const int nblk = gridDim.x, q = nblk / 8, r = nblk % 8, x = lin % 8, y = lin / 8;
    lin = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;
  }
  const int nt = lin % ntn, mt = lin / ntn;
  int64_t m0, mlim;
  if (g.wstride) {                                     // per-image weights: a block never spans two images
    const int tpi = (g.HW + BM - 1) / BM;
    const int64_t im = mt / tpi;
    m0 = im * g.HW + (int64_t)(mt % tpi) * BM;
    mlim = min(g.M, (im + 1) * (int64_t)g.HW);
  } else {
    m0 = (int64_t)mt * BM;
    mlim = g.M;
  }
  const int n0 = nt * BN;
  const int K = g.a.Ktot, nk = (K + BK - 1) / BK;
  const int img0 = (int)(m0 / g.HW);
  const float* Wp = reinterpret_cast<const float*>(g.w) + (g.wstride ? (int64_t)(img0 / g.wdiv) * g.wstride : 0);

  if (tid < BN) {
    const int n = min(n0 + tid, g.N - 1);
    e_s[tid] = (g.ln_s ? g.ln_s : g.zeros)[n];
    e_t[tid] = (g.ln_t ? g.ln_t : g.zeros)[n];
    e_b[tid] = (g.bias ? g.bias : g.zeros)[n];
    e_c[tid] = (g.scale ? g.scale : g.ones)[n];
  }

  // ---- LDS-DMA geometry: wave w issues instructions j = w + 4 i of a stage; lane l of instruction
  // j fills stage chunk 64 j + l = (row, position): rows < BM are pixel rows, the rest weight rows;
  // the position holds chunk c = position ^ ((row >> 2) & 3) of the row's 16-float K slice ----
  int q_img[NI], q_p[NI], q_y[NI], q_x[NI], q_c[NI];
  bool q_ok[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int idx = (wid + 4 * i) * 64 + lane, row = idx >> 2;
    q_c[i] = f32_pos(row, idx & 3);
    if ((wid + 4 * i) * 16 < BM) {                  // wave-uniform: an instruction covers 16 rows of one kind
      const int64_t m = m0 + row;
      q_ok[i] = m < mlim;
      const int mm = q_ok[i] ? (int)m : (int)m0;
      q_img[i] = mm / g.HW;
      q_p[i] = mm - q_img[i] * g.HW;
      q_y[i] = g.conv3 ? q_p[i] / g.Wimg : 0;
      q_x[i] = g.conv3 ? q_p[i] - q_y[i] * g.Wimg : 0;
    } else {
      const int n = n0 + row - BM;
      q_ok[i] = n < g.N;
      q_img[i] = q_ok[i] ? n : 0;
      q_p[i] = q_y[i] = q_x[i] = 0;
    }
  }
  const int Himg = g.conv3 ? g.HW / g.Wimg : 0;
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  // stage kt -> slot kt % NS; past the last K tile the zero line (every wave issues NI instructions
  // per stage, so the counted wait below is a constant)
  auto issue = [&](int kt) {
    if (g.dbg & 2) return;                          // tools/f32bench ablation: no operand loads (timing only)
    const uint32_t sS = lds_base + (kt % NS) * STAGE;
    const bool live = kt < nk;
    // every source's K (and the conv3 cin) is a multiple of BK (gemm_f32_ok), so the source and the
    // tap of a K tile are uniform: selected from kt0 in scalar registers
    const int kt0 = kt * BK;
    const float* base = reinterpret_cast<const float*>(g.a.s[0].base);
    int64_t sld = g.a.s[0].ld;
    int soff = g.a.s[0].off, smul = g.a.s[0].img_mul, sadd = g.a.s[0].img_add, kb = 0;
    if (!g.conv3) {
      int kbj = g.a.s[0].K;
#pragma unroll
      for (int j = 1; j < TURTLE_MAX_SRC; ++j) {
        if (j < g.a.n) {
          const bool hit = kt0 >= kbj;
          base = hit ? reinterpret_cast<const float*>(g.a.s[j].base) : base;
          sld = hit ? g.a.s[j].ld : sld;
          soff = hit ? g.a.s[j].off : soff;
          smul = hit ? g.a.s[j].img_mul : smul;
          sadd = hit ? g.a.s[j].img_add : sadd;
          kb = hit ? kbj : kb;
          kbj += g.a.s[j].K;
        }
      }
    }
    const int tap = g.conv3 ? kt0 / g.cin : 4;
    const int ci0 = g.conv3 ? kt0 - tap * g.cin : kt0 - kb;
    const int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const void* src;
      if ((wid + 4 * i) * 16 < BM) {
        const int y = q_y[i] + dy, x = q_x[i] + dx;
        const bool inb = !g.conv3 || (y >= 0 && y < Himg && x >= 0 && x < g.Wimg);
        const int64_t off = ((int64_t)(q_img[i] * smul + sadd) * g.HW + q_p[i] + dy * g.Wimg + dx) * sld + soff + ci0 + 4 * q_c[i];
        src = live && q_ok[i] && inb ? reinterpret_cast<const void*>(base + off) : reinterpret_cast<const void*>(g_zero_f32);
      } else {
        src = live && q_ok[i] ? reinterpret_cast<const void*>(Wp + (int64_t)q_img[i] * g.ldw + kt0 + 4 * q_c[i])
                              : reinterpret_cast<const void*>(g_zero_f32);
      }
      f32_dma16(src, sS + (wid + 4 * i) * 1024);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // LayerNorm statistics: 2 threads per pixel row, shifted sums over the staged A tiles (the
  // shift is the row's k = 0 element, as in gemm_kernel)
  const int lr = tid >> 1, lh = tid & 1;
  float ls = 0.f, lq = 0.f, lsh = 0.f;

#pragma unroll
  for (int st = 0; st < NS - 1; ++st) issue(st);
  for (int kt = 0; kt < nk; ++kt) {
    if (!(g.dbg & 2)) f32_wait_vm<(NS - 2) * NI>();  // this wave's part of stage kt has landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                     // every part landed; slot (kt - 1) % NS is free
    asm volatile("" ::: "memory");
    issue(kt + NS - 1);
    const char* sX = smem + (kt % NS) * STAGE;
    const char* sW = sX + BM * F32_ROW;
    if (g.ln) {
      const char* row = sX + lr * F32_ROW;
      if (kt == 0) lsh = *reinterpret_cast<const float*>(row + f32_pos(lr, 0) * 16);
#pragma unroll
      for (int j = 0; j < 2; ++j) {                   // positions 2 lh, 2 lh + 1 (all chunks are in range: K % 16 == 0)
        const float4 v = *reinterpret_cast<const float4*>(row + (2 * lh + j) * 16);
        const float d0 = v.x - lsh, d1 = v.y - lsh, d2 = v.z - lsh, d3 = v.w - lsh;
        ls += (d0 + d1) + (d2 + d3);
        lq = fmaf(d0, d0, lq); lq = fmaf(d1, d1, lq); lq = fmaf(d2, d2, lq); lq = fmaf(d3, d3, lq);
      }
    }
    float4 af[TN], bf[TM];                          // k = 4 fq + s in MFMA step s: one ds_read_b128 per fragment row
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const int r = wn * (BN / 2) + 16 * t + fr;
      af[t] = *reinterpret_cast<const float4*>(sW + r * F32_ROW + f32_pos(r, fq) * 16);
    }
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      const int r = wm * (BM / 2) + 16 * t + fr;
      bf[t] = *reinterpret_cast<const float4*>(sX + r * F32_ROW + f32_pos(r, fq) * 16);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[tn][s], bf[tm][s], acc[tm][tn], 0, 0, 0);
  }
  f32_wait_vm<0>();                                   // no LDS-DMA may land after the workgroup ends
  if (g.ln) {
    ls += __shfl_xor(ls, 1, 64);
    lq += __shfl_xor(lq, 1, 64);
    if (lh == 0) {
      const float md = ls / K;
      s_mu[lr] = lsh + md;
      s_rs[lr] = rsqrtf(fmaxf(lq / K - md * md, 0.f) + 1e-5f);
    }
    __syncthreads();
  }

  // ---- epilogue: lane holds channels n0 + cl .. cl + 3 (cl = wn BN/2 + 16 tn + 4 fq) of pixel
  // m0 + wm 64 + 16 tm + fr ----
  float* o = reinterpret_cast<float*>(g.out);
  const float* res = reinterpret_cast<const float*>(g.res);
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int r = wm * (BM / 2) + 16 * tm + fr;
    const int64_t m = m0 + r;
    if (m >= mlim) continue;
    const float mu = g.ln ? s_mu[r] : 0.f, rs = g.ln ? s_rs[r] : 1.f;
    float4 rv[TN];                                  // this row's residual chunks, loaded before its stores
    if (res) {
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int n = n0 + wn * (BN / 2) + 16 * tn + 4 * fq;
        const bool full = n + 4 <= g.N;
        rv[tn] = *reinterpret_cast<const float4*>(full ? res + m * g.ldr + g.offr + n : g.zeros);
        if (!full && n < g.N) {
          float t4[4] = {0.f, 0.f, 0.f, 0.f};
          for (int e = 0; e < 4 && n + e < g.N; ++e) t4[e] = res[m * g.ldr + g.offr + n + e];
          rv[tn] = make_float4(t4[0], t4[1], t4[2], t4[3]);
        }
      }
    }
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int cl = wn * (BN / 2) + 16 * tn + 4 * fq, n = n0 + cl;
      if (n >= g.N) continue;
      const float4 es = *reinterpret_cast<const float4*>(e_s + cl), et = *reinterpret_cast<const float4*>(e_t + cl);
      const float4 eb = *reinterpret_cast<const float4*>(e_b + cl), ec = *reinterpret_cast<const float4*>(e_c + cl);
      const float fs[4] = {es.x, es.y, es.z, es.w}, ft[4] = {et.x, et.y, et.z, et.w};
      const float fb[4] = {eb.x, eb.y, eb.z, eb.w}, fc[4] = {ec.x, ec.y, ec.z, ec.w};
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = acc[tm][tn][e];
        if (g.ln) x = rs * (x - mu * fs[e]) + ft[e];
        x += fb[e];
        if (g.gelu) x = gelu_erf(x);
        v[e] = x * fc[e];
      }
      if (res) { v[0] += rv[tn].x; v[1] += rv[tn].y; v[2] += rv[tn].z; v[3] += rv[tn].w; }
      const bool full = n + 4 <= g.N;
      int64_t dst;
      if (g.store_mode == STORE_NHWC) {
        dst = m * g.ldo + g.offo + n;
      } else {
        const int mi = (int)m, img = mi / g.HW, p = mi - img * g.HW;
        const int Wi = g.Wimg, Hi = g.HW / Wi, y = p / Wi, x = p - y * Wi;
        if (g.store_mode == STORE_UNSHUFFLE) {
          const int64_t dp = ((int64_t)img * (Hi / 2) + y / 2) * (Wi / 2) + x / 2;
          const int sub = (y & 1) * 2 + (x & 1);
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (n + e < g.N) o[dp * g.ldo + g.offo + (n + e) * 4 + sub] = v[e];
          continue;
        }
        // PixelShuffle: output channel n' = s Cq + c (4 channels stay in one sub-pixel: Cq % 4 == 0)
        const int Cq = g.N / 4, sp = n / Cq, cn = n - sp * Cq;
        dst = (((int64_t)img * 2 * Hi + 2 * y + (sp >> 1)) * (2 * Wi) + 2 * x + (sp & 1)) * g.ldo + g.offo + cn;
      }
      if (full) {
        *reinterpret_cast<float4*>(o + dst) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (n + e < g.N) o[dst + e] = v[e];
      }
    }
  }
}

// Eligible: the fp32 GEMMs gemm_kernel<float> takes, with every source's K (and the conv3 cin) a
// multiple of 16 (K-tile-uniform source selection), offsets and row strides multiples of 4 floats
// and 16-byte aligned bases; not the bf16-only modes
// Where it is the faster fp32 kernel (tools/f32bench on MI355X, profiles/r05y_f32bench.log): the LN
// projections (1.03-1.11x), GELU epilogues (1.18x) and multi-source W_eff GEMMs (1.08x); plain
// residual projections and N <= 64 stay on gemm_kernel<float> (0.89-0.98x here)
bool gemm_f32_preferred(const GemmArgs& g) { return gemm_f32_ok(g) && (g.ln || g.gelu || g.a.n > 1); }

bool gemm_f32_ok(const GemmArgs& g) {
  if (!g.allow_f32 || g.store_mode == STORE_CB16 || g.a.cb_px) return false;
  if (g.M <= 0 || g.N <= 0 || g.a.Ktot <= 0 || g.a.n < 1 || g.a.n > TURTLE_MAX_SRC) return false;
  if (g.N > TURTLE_CONST_VEC) return false;
  if (g.conv3) {
    if (g.cin % F32_BK || g.a.Ktot != 9 * g.cin || g.Wimg <= 0 || g.HW % g.Wimg) return false;
  }
  for (int j = 0; j < g.a.n; ++j) {
    const SrcDesc& s = g.a.s[j];
    if (s.K % F32_BK || s.off % 4 || s.ld % 4 || reinterpret_cast<uintptr_t>(s.base) % 16) return false;
  }
  if (g.ldw % 4 || g.wstride % 4 || reinterpret_cast<uintptr_t>(g.w) % 16) return false;
  if (g.res && (g.ldr % 4 || g.offr % 4 || reinterpret_cast<uintptr_t>(g.res) % 16)) return false;
  if (g.ldo % 4 || g.offo % 4 || reinterpret_cast<uintptr_t>(g.out) % 16) return false;
  if (g.store_mode == STORE_SHUFFLE && (g.N % 16 || g.Wimg <= 0)) return false;
  if (g.store_mode == STORE_UNSHUFFLE && g.Wimg <= 0) return false;
  return true;
}

template <int BN, int NS>
static void launch_f32(const GemmArgs& g, int64_t mt, hipStream_t st) {
  using L = F32L<BN, NS>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_f32_kernel<BN, NS>), hipFuncAttributeMaxDynamicSharedMemorySize, L::BYTES);
    attr = true;
  }
  hipLaunchKernelGGL((gemm_f32_kernel<BN, NS>), dim3((unsigned)(mt * ((g.N + BN - 1) / BN))), dim3(256), L::BYTES, st, g);
}

void launch_gemm_f32(const GemmArgs& g, hipStream_t st) {
  const int64_t mt = g.wstride ? (g.M / g.HW) * ((g.HW + F32_BM - 1) / F32_BM) : (g.M + F32_BM - 1) / F32_BM;
  // 4-stage ring for the 128-wide multi-source GEMMs (tools/f32bench, profiles/r05y_f32bench.log), or
  // on request (tools/f32bench dbg bit 0)
  const bool deep = (g.dbg & 1) || (g.a.n > 1 && g.N <= 128);
  if (g.N >= 128 && (g.N % 128 == 0 || g.N > 1024)) {   // as gemm_kernel: BN 128 when it tiles N (or N is large)
    if (deep) launch_f32<128, 4>(g, mt, st); else launch_f32<128, 3>(g, mt, st);
  } else {
    if (deep) launch_f32<64, 4>(g, mt, st); else launch_f32<64, 3>(g, mt, st);
  }
}

}  // namespace turtle

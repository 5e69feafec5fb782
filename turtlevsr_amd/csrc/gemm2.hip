// bf16 1x1 / implicit-3x3 convolution GEMM, LDS-pipelined (the main GEMM of the bf16 build).
//
//   out[m][n] = epilogue( sum_k A[m][k] * W[n][k] )        m = pixel, n = output channel
//
// Same contract as gemm_kernel (gemm.hip): K-concatenated multi-source A, implicit 3x3 taps,
// LayerNorm folded into W with statistics taken from the staged A tiles, bias / GELU / scale /
// residual epilogue, NHWC / PixelShuffle / PixelUnshuffle stores, per-image weight sets (W_eff).
//
// Structure (MI355X): 128 x BN output tile per 256-thread block, 2 x 2 waves, BK = 64.
//   * both operands go HBM/L2 -> LDS by global_load_lds (16 B per lane, no VGPR staging), two
//     LDS stages: tile k+1 streams in while the MFMAs consume tile k (counted vmcnt + raw
//     s_barrier, so the prefetch stays in flight across the barrier);
//   * an LDS-DMA writes 64 lanes x 16 B contiguously, so rows are 128 B unpadded and the
//     bank spread comes from an XOR swizzle of the 16-byte chunk index, applied on the global
//     source address: LDS chunk p of row r holds k-chunk p ^ ((r >> 1) & 7). The MFMA fragment
//     reads (16 rows x 16 B per lane group) then hit 16 distinct 4-bank slots (conflict-free);
//   * a K tile never straddles two sources or two 3x3 taps (widths / cin multiples of 64), so
//     its source is resolved on the scalar unit once per tile;
//   * two blocks per CU (67 KB LDS each), so one block's epilogue overlaps the other's K loop;
//   * output channel tiles of one pixel panel are consecutive block ids on one XCD: the A panel
//     leaves HBM once and is re-read from that XCD's L2.
#include "common.h"
#include "kernels.h"

namespace turtle {

__device__ __attribute__((aligned(64))) uint4 g_zero_g2[4];

template <int BM, int BN>
struct G2 {
  static constexpr int BK = 64;
  static constexpr int A_BYTES = BM * 128;
  static constexpr int W_BYTES = BN * 128;
  static constexpr int STAGE = A_BYTES + W_BYTES;
  static constexpr int PIPE = 2 * STAGE;
  static constexpr int OROW = BN * 2 + 16;          // staged output row (bf16 + pad)
  static constexpr int OUT = BM * OROW;
  static constexpr int MAIN = PIPE > OUT ? PIPE : OUT;
  static constexpr int BYTES = MAIN + 4 * BN * 4 + 2 * BM * 4;
};

typedef __attribute__((address_space(3))) void lds_void;

TURTLE_DEV void glds16(const void* g, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (lds_void*)lds_wave_base, 16, 0, 0);
}

template <int N>
TURTLE_DEV void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

TURTLE_DEV void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int BM, int BN>
__global__ __launch_bounds__(256, 2) void gemm_lds_kernel(GemmArgs g) {
  using S = G2<BM, BN>;
  constexpr int TM = BM / 32, TN = BN / 32;       // 16x16 tiles per wave (2 x 2 waves)
  constexpr int AI = BM * 8 / 256, WI = BN * 8 / 256;   // LDS-DMA chunks per thread per stage
  constexpr int NL = AI + WI;                     // LDS-DMA instructions per thread per stage
  __shared__ __attribute__((aligned(16))) char smem[S::BYTES];
  float* e_s = reinterpret_cast<float*>(smem + S::MAIN);   // [BN] ln_s, ln_t, bias, scale
  float* e_t = e_s + BN;
  float* e_b = e_t + BN;
  float* e_c = e_b + BN;
  float* s_mu = e_c + BN;                                   // [BM] LN mean, rstd
  float* s_rs = s_mu + BM;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;

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
  const int nk = (K + 63) / 64;
  const int img0 = (int)(m0 / g.HW);
  const bf16* Wp = reinterpret_cast<const bf16*>(g.w) + (g.wstride ? (int64_t)(img0 / g.wdiv) * g.wstride : 0);

  if (tid < BN) {
    const int n = min(n0 + tid, g.N - 1);
    e_s[tid] = (g.ln_s ? g.ln_s : g.zeros)[n];
    e_t[tid] = (g.ln_t ? g.ln_t : g.zeros)[n];
    e_b[tid] = (g.bias ? g.bias : g.zeros)[n];
    e_c[tid] = (g.scale ? g.scale : g.ones)[n];
  }

  // ---- LDS-DMA geometry: instruction i of wave w fills LDS chunks (i*4 + w)*64 + lane ----
  // chunk q -> row q/8, position q%8, k-chunk (q%8) ^ ((row>>1)&7). Per lane the row geometry is
  // resolved once; per K tile the source (or 3x3 tap) is wave-uniform (source widths and cin are
  // multiples of 64), so a tile costs one scalar select scan + one 64-bit mad per DMA.
  int a_img[AI], a_p[AI], a_y[AI], a_x[AI], a_cc[AI];
  bool a_ok[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int q = (i * 4 + wid) * 64 + lane, r = q >> 3;
    a_cc[i] = ((q & 7) ^ ((r >> 1) & 7)) * 8;
    const int64_t m = m0 + r;
    a_ok[i] = m < mlim;
    const int mm = a_ok[i] ? (int)m : (int)m0;
    a_img[i] = mm / g.HW;
    a_p[i] = mm - a_img[i] * g.HW;
    a_y[i] = g.conv3 ? a_p[i] / g.Wimg : 0;
    a_x[i] = g.conv3 ? a_p[i] - a_y[i] * g.Wimg : 0;
  }
  const bf16* w_row[WI];
  int w_cc[WI];
  bool w_ok[WI];
#pragma unroll
  for (int i = 0; i < WI; ++i) {
    const int q = (i * 4 + wid) * 64 + lane, r = q >> 3;
    w_cc[i] = ((q & 7) ^ ((r >> 1) & 7)) * 8;
    w_ok[i] = n0 + r < g.N;
    w_row[i] = Wp + (int64_t)min(n0 + r, g.N - 1) * g.ldw + w_cc[i];
  }
  const int Himg = g.conv3 ? g.HW / g.Wimg : 0;

  auto issue = [&](int kt, int stage) {
    char* sA = smem + stage * S::STAGE;
    char* sW = sA + S::A_BYTES;
    const int k0 = kt * 64;
    // wave-uniform source of this K tile
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
      const bf16* src = base + (int64_t)pix * sld + soff + a_cc[i];
      glds16(ok ? reinterpret_cast<const void*>(src) : reinterpret_cast<const void*>(g_zero_g2), sA + (i * 4 + wid) * 1024);
    }
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      const bool ok = w_ok[i] && k0 + w_cc[i] < K;
      glds16(ok ? reinterpret_cast<const void*>(w_row[i] + k0) : reinterpret_cast<const void*>(g_zero_g2),
             sW + (i * 4 + wid) * 1024);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // LN statistics: 2 threads per row (4 chunks each)
  const int lr = tid >> 1, lh = tid & 1;
  float ls = 0.f, lq = 0.f;

  // fragment addressing: lane row (l & 15), k-chunk (l >> 4) + 4 ks
  const int fr = lane & 15, fq = lane >> 4;

  __syncthreads();                     // epilogue vectors staged; all waves start the pipeline together
  issue(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt & 1;
    if (kt + 1 < nk) {
      issue(kt + 1, st ^ 1);
      wait_vm<NL>();                   // own part of tile kt has landed; tile kt+1 stays in flight
    } else {
      wait_vm<0>();
    }
    lds_barrier();                     // every wave's part of tile kt has landed
    const char* sA = smem + st * S::STAGE;
    const char* sW = sA + S::A_BYTES;
    if (g.ln) {
      // row lr, positions 4 lh .. 4 lh + 3 (any order: only row sums matter); chunks past K are
      // zero-filled. Sums and sums of squares by v_dot2_f32_bf16 (x . 1 and x . x per pair).
      typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
      const bf16x2 one2 = __builtin_bit_cast(bf16x2, 0x3F803F80u);
      const char* row = sA + lr * 128;
      const int sw = (lr >> 1) & 7;
#pragma unroll
      for (int pc = 0; pc < 4; ++pc) {
        const uint4 x = *reinterpret_cast<const uint4*>(row + (((lh * 4 + pc) ^ sw) << 4));   // swizzled: no conflicts
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bf16x2 v2 = __builtin_bit_cast(bf16x2, w[e]);
          ls = __builtin_amdgcn_fdot2_f32_bf16(v2, one2, ls, false);
          lq = __builtin_amdgcn_fdot2_f32_bf16(v2, v2, lq, false);
        }
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 4 + fq;
      bf16x8 af[TN], bfr[TM];
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        const int r = wn * (BN / 2) + t * 16 + fr;
        af[t] = *reinterpret_cast<const bf16x8*>(sW + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        const int r = wm * (BM / 2) + t * 16 + fr;
        bfr[t] = *reinterpret_cast<const bf16x8*>(sA + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[tn], bfr[tm], acc[tm][tn], 0, 0, 0);
    }
    lds_barrier();                     // stage st fully read before it is refilled
  }
  if (g.ln) {
    ls += __shfl_xor(ls, 1, 64);
    lq += __shfl_xor(lq, 1, 64);
    if (lh == 0 && lr < BM) {
      const float mu = ls / K;
      s_mu[lr] = mu;
      s_rs[lr] = rsqrtf(fmaxf(lq / K - mu * mu, 0.f) + 1e-5f);
    }
    __syncthreads();
  }

  // ---- epilogue phase 1: per-element math, tile staged in LDS as bf16 ----
  // C/D of 16x16x32: column (lane & 15) = pixel, rows 4 (lane >> 4) + e = channels
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int r = wm * (BM / 2) + tm * 16 + fr;
    const float mu = g.ln ? s_mu[r] : 0.f, rs = g.ln ? s_rs[r] : 1.f;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int cl = wn * (BN / 2) + tn * 16 + fq * 4;
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
        if (g.gelu) x = gelu_bf16(x);
        v[e] = x * fc[e];
      }
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
      *reinterpret_cast<bf16x4*>(smem + r * S::OROW + cl * 2) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
    }
  }
  __syncthreads();

  // ---- epilogue phase 2: 16-byte row chunks, residual add, store remap ----
  constexpr int CV = BN / 8;
  constexpr int NCH = BM * CV / 256;
  bf16* o = reinterpret_cast<bf16*>(g.out);
  const bf16* res = reinterpret_cast<const bf16*>(g.res);
  Vec<bf16> v[NCH];
  bool okc[NCH];
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int idx = tid + j * 256, r = idx / CV, cc = idx % CV;
    const int64_t m = m0 + r;
    const int nb = n0 + cc * 8;
    okc[j] = m < mlim && nb < g.N;
    v[j].load(reinterpret_cast<const bf16*>(smem + r * S::OROW) + cc * 8);
    if (res) {
      Vec<bf16> rv; rv.load_pred(res + (okc[j] ? m * g.ldr + g.offr + nb : 0), okc[j]);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[j].v[e] += rv.v[e];
    }
  }
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    if (!okc[j]) continue;
    const int idx = tid + j * 256, r = idx / CV, cc = idx % CV;
    const int64_t m = m0 + r;
    const int nb = n0 + cc * 8;
    int64_t dst;
    if (g.store_mode == STORE_NHWC) {
      dst = m * g.ldo + g.offo + nb;
    } else {
      const int mi = (int)m, img = mi / g.HW, p = mi - img * g.HW;
      const int Wi = g.Wimg, Hi = g.HW / Wi;
      const int y = p / Wi, x = p - y * Wi;
      if (g.store_mode == STORE_UNSHUFFLE) {
        const int64_t dp = ((int64_t)img * (Hi / 2) + y / 2) * (Wi / 2) + x / 2;
        const int sub = (y & 1) * 2 + (x & 1);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[dp * g.ldo + g.offo + (nb + e) * 4 + sub] = (bf16)v[j].v[e];
        continue;
      }
      const int Cq = g.N / 4, sp = nb / Cq, cn = nb - sp * Cq;
      dst = (((int64_t)img * 2 * Hi + 2 * y + (sp >> 1)) * (2 * Wi) + 2 * x + (sp & 1)) * g.ldo + g.offo + cn;
    }
    v[j].store(o + dst);
  }
}

// Eligible: bf16, every 16-byte operand chunk inside one source and 16-byte aligned, N % 8 == 0
// (whole 16-byte output chunks; PixelShuffle needs N/4 % 8 == 0), conv3 taps aligned to BK.
bool gemm_lds_ok(const GemmArgs& g) {
  if (g.a.cb_px) return false;                   // channel-blocked operand: 2-D tiled kernel only
  if (!g.allow_lds || g.N % 8 || g.ldo % 8 || g.offo % 8) return false;
  // measured (tools/kbench, MI355X): the panel kernel stays ahead for LayerNorm GEMMs with K <= 256
  // (its single panel load amortises the statistics), this kernel wins everywhere else
  if (g.ln && g.a.Ktot <= 256 && g.allow_panel) return false;
  if (g.res && (g.ldr % 8 || g.offr % 8)) return false;
  if (g.ldw % 8) return false;
  if (g.store_mode == STORE_SHUFFLE && (g.N / 4) % 8) return false;
  if (g.conv3) return g.cin % 64 == 0 && g.a.n == 1 && g.a.s[0].ld % 8 == 0 && g.a.s[0].off % 8 == 0;
  for (int j = 0; j < g.a.n; ++j) {
    if (g.a.s[j].K % 8 || g.a.s[j].ld % 8 || g.a.s[j].off % 8) return false;
    if (j + 1 < g.a.n && g.a.s[j].K % 64) return false;      // K tiles never straddle sources
  }
  return g.a.Ktot % 8 == 0;
}

template <int BM, int BN>
static void launch_lds_cfg(const GemmArgs& g, hipStream_t st) {
  const int64_t mt = g.wstride ? (g.M / g.HW) * ((g.HW + BM - 1) / BM) : (g.M + BM - 1) / BM;
  const int64_t nblk = mt * ((g.N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_lds_kernel<BM, BN>), dim3((unsigned)nblk), dim3(256), 0, st, g);
}

void launch_gemm_lds(const GemmArgs& g, hipStream_t st) {
  if (g.N <= 64) launch_lds_cfg<128, 64>(g, st);
  else launch_lds_cfg<128, 128>(g, st);
}

}  // namespace turtle

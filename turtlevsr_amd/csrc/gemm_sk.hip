// Split-K bf16 GEMM for the small-frame 'wide' projections (<= 4096 pixels: the latent / level-3 LN
// projections, project_out K = 1280 and W_eff of a 256x256 frame). Their 256-row gemm9 / 2-D tiled
// tiles leave most of the 256 CUs idle (M = 1024: 4-32 tiles); hipBLASLt split K there until round 4.
//
//   partial[s][m][n] = sum_{k in chunk s} A[m][k] W[n][k]            gemm_sk_kernel (fp32 workspace)
//   out[m][n] = epi( sum_s partial[s][m][n] )                        gemm_sk_epi_kernel
//
// (with >= 256 tiles of 64 x 64 there is one split and gemm_sk_kernel applies the epilogue itself: a
// small-tile GEMM for the shapes whose 256-row tiles would give a few dozen blocks)
//
// with epi the GEMM family's epilogue (LayerNorm correction rs (acc - mu s[n]) + t[n] from the
// per-pixel statistics of ln_stats_kernel (gemm9.hip), + bias, GELU, * scale, + residual). The splits
// are summed in a fixed order: results are bitwise repeatable (no atomics).
//
// gemm_sk_kernel: 256 threads (2 x 2 waves of 32 x 32), tile 64 pixels x 64 channels, BK = 64 staged
// through LDS (register loads of the next K tile in flight during the MFMAs), MFMA 16x16x32 bf16 with
// i = output channel (W rows) and j = pixel, so a lane's accumulator is 4 consecutive channels of one
// pixel (16-byte partial stores). LDS rows of 128 B + 16 B pad: conflict-free ds_read_b128.
#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace turtle {

__device__ __attribute__((aligned(64))) uint4 g_zero_sk[4];

constexpr int SK_BM = 64, SK_BN = 64, SK_BK = 64, SK_ROWB = SK_BK * 2 + 16;

template <bool FUSED>
__global__ __launch_bounds__(256) void gemm_sk_kernel(GemmArgs g, int kchunk, float* __restrict__ part, const float2* __restrict__ stats) {
  typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
  __shared__ __attribute__((aligned(16))) char smem[(SK_BM + SK_BN) * SK_ROWB];
  char* sX = smem;
  char* sW = smem + SK_BM * SK_ROWB;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1, fr = lane & 15, fq = lane >> 4;
  const int ntn = (g.N + SK_BN - 1) / SK_BN, ntm = (int)((g.M + SK_BM - 1) / SK_BM);
  const int split = blockIdx.x / (ntn * ntm), t = blockIdx.x % (ntn * ntm);
  const int n0 = (t % ntn) * SK_BN;
  const int64_t m0 = (int64_t)(t / ntn) * SK_BM;
  const int k0 = split * kchunk, nkt = kchunk / SK_BK;
  const SrcDesc& s = g.a.s[0];
  const bf16* A = reinterpret_cast<const bf16*>(s.base);
  const bf16* W = reinterpret_cast<const bf16*>(g.w);
  // per thread: 2 A chunks + 2 W chunks of 16 B per K tile (row = tid / 8 + 32 i, chunk = tid % 8)
  const int kc = tid & 7;
  const void* pa[2];
  const void* pw[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (tid >> 3) + 32 * i;
    const int64_t m = m0 + r;
    pa[i] = m < g.M ? reinterpret_cast<const void*>(A + m * s.ld + s.off + k0 + kc * 8) : reinterpret_cast<const void*>(g_zero_sk);
    const int n = n0 + r;
    pw[i] = n < g.N ? reinterpret_cast<const void*>(W + (int64_t)n * g.ldw + k0 + kc * 8) : reinterpret_cast<const void*>(g_zero_sk);
  }
  const bool a_live[2] = {m0 + (tid >> 3) < g.M, m0 + (tid >> 3) + 32 < g.M};
  const bool w_live[2] = {n0 + (tid >> 3) < g.N, n0 + (tid >> 3) + 32 < g.N};
  uint4 ra[2], rw[2];
  auto load = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      ra[i] = ld16(a_live[i] ? reinterpret_cast<const char*>(pa[i]) + kt * SK_BK * 2 : reinterpret_cast<const char*>(g_zero_sk));
      rw[i] = ld16(w_live[i] ? reinterpret_cast<const char*>(pw[i]) + kt * SK_BK * 2 : reinterpret_cast<const char*>(g_zero_sk));
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  load(0);
  for (int kt = 0; kt < nkt; ++kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = (tid >> 3) + 32 * i;
      *reinterpret_cast<uint4*>(sX + r * SK_ROWB + kc * 16) = ra[i];
      *reinterpret_cast<uint4*>(sW + r * SK_ROWB + kc * 16) = rw[i];
    }
    __syncthreads();
    if (kt + 1 < nkt) load(kt + 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8v wf[2], xf[2];
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {
        wf[t2] = *reinterpret_cast<const bf16x8v*>(sW + (wn * 32 + 16 * t2 + fr) * SK_ROWB + ks * 64 + fq * 16);
        xf[t2] = *reinterpret_cast<const bf16x8v*>(sX + (wm * 32 + 16 * t2 + fr) * SK_ROWB + ks * 64 + fq * 16);
      }
#pragma unroll
      for (int tm = 0; tm < 2; ++tm)
#pragma unroll
        for (int tn = 0; tn < 2; ++tn) acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[tn], xf[tm], acc[tm][tn], 0, 0, 0);
    }
    __syncthreads();
  }
  // lane: channels n0 + 32 wn + 16 tn + 4 fq + 0..3 of pixel m0 + 32 wm + 16 tm + fr
#pragma unroll
  for (int tm = 0; tm < 2; ++tm) {
    const int64_t m = m0 + wm * 32 + 16 * tm + fr;
    if (m >= g.M) continue;
    float mu = 0.f, rs = 1.f;
    if (FUSED && g.ln) { const float2 st = stats[m]; mu = st.x; rs = st.y; }
#pragma unroll
    for (int tn = 0; tn < 2; ++tn) {
      const int n = n0 + wn * 32 + 16 * tn + 4 * fq;
      if (n >= g.N) continue;                       // N % 8 == 0: 4 channels all in or all out
      if constexpr (!FUSED) {
        *reinterpret_cast<f32x4*>(part + ((int64_t)split * g.M + m) * g.N + n) = acc[tm][tn];
      } else {                                      // one split: the epilogue here (as gemm_sk_epi_kernel)
        const f32x4 vs = *reinterpret_cast<const f32x4*>((g.ln_s ? g.ln_s : g.zeros) + n);
        const f32x4 vt = *reinterpret_cast<const f32x4*>((g.ln_t ? g.ln_t : g.zeros) + n);
        const f32x4 vb = *reinterpret_cast<const f32x4*>((g.bias ? g.bias : g.zeros) + n);
        const f32x4 vc = *reinterpret_cast<const f32x4*>((g.scale ? g.scale : g.ones) + n);
        float r[4] = {0.f, 0.f, 0.f, 0.f};
        if (g.res) {
          const uint2 q = ld8(reinterpret_cast<const bf16*>(g.res) + m * g.ldr + g.offr + n);
          r[0] = __uint_as_float(q.x << 16); r[1] = __uint_as_float(q.x & 0xffff0000u);
          r[2] = __uint_as_float(q.y << 16); r[3] = __uint_as_float(q.y & 0xffff0000u);
        }
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        bf16x4 ov;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = acc[tm][tn][e];
          if (g.ln) x = rs * (x - mu * vs[e]);
          x += vt[e] + vb[e];
          if (g.gelu) x = gelu_bf16(x);
          ov[e] = (bf16)(x * vc[e] + r[e]);
        }
        *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(g.out) + m * g.ldo + g.offo + n) = ov;
      }
    }
  }
}

// one thread per (pixel, 8 channels): the splits summed in order, then the epilogue
__global__ __launch_bounds__(256) void gemm_sk_epi_kernel(GemmArgs g, int nsplit, const float* __restrict__ part,
                                                          const float2* __restrict__ stats) {
  const int n8 = g.N / 8;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= g.M * n8) return;
  const int64_t m = idx / n8;
  const int c = (int)(idx - m * n8) * 8;
  float v[8];
  {
    const f32x4 a = *reinterpret_cast<const f32x4*>(part + m * g.N + c), b = *reinterpret_cast<const f32x4*>(part + m * g.N + c + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { v[e] = a[e]; v[4 + e] = b[e]; }
  }
  for (int s = 1; s < nsplit; ++s) {
    const float* p = part + ((int64_t)s * g.M + m) * g.N + c;
    const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { v[e] += a[e]; v[4 + e] += b[e]; }
  }
  float mu = 0.f, rs = 1.f;
  if (g.ln) { const float2 st = stats[m]; mu = st.x; rs = st.y; }
  const float* vs = g.ln_s ? g.ln_s : g.zeros;
  const float* vt = g.ln_t ? g.ln_t : g.zeros;
  const float* vb = g.bias ? g.bias : g.zeros;
  const float* vc = g.scale ? g.scale : g.ones;
  float r[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (g.res) {
    Vec<bf16> rv;
    rv.load(reinterpret_cast<const bf16*>(g.res) + m * g.ldr + g.offr + c);
#pragma unroll
    for (int e = 0; e < 8; ++e) r[e] = rv.v[e];
  }
  bf16x8 ov;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float x = v[e];
    if (g.ln) x = rs * (x - mu * vs[c + e]);
    x += vt[c + e] + vb[c + e];
    if (g.gelu) x = gelu_bf16(x);
    ov[e] = (bf16)(x * vc[c + e] + r[e]);
  }
  *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(g.out) + m * g.ldo + g.offo + c) = ov;
}

// K splits: about 4 blocks per CU over the 64 x 64 tiles, each split a multiple of 64 deep (a shape-only
// function: the frame driver reserves the workspace in its sizing pass from it)
int gemm_sk_splits(int64_t M, int N, int K) {
  const int64_t tiles = ((M + SK_BM - 1) / SK_BM) * ((N + SK_BN - 1) / SK_BN);
  if (tiles >= 256) return 1;                      // every CU has a tile: no split, epilogue fused
  int s = (int)std::max<int64_t>(1, (1024 + tiles - 1) / tiles);
  s = std::min(s, K / SK_BK);
  while (s > 1 && (K / SK_BK) % s) --s;           // equal chunks of whole K tiles
  return s;
}

size_t gemm_sk_workspace_bytes(int64_t M, int N, int K) {
  return (size_t)gemm_sk_splits(M, N, K) * (size_t)M * N * 4 + (size_t)M * sizeof(float2);
}

// Eligible: bf16, one plain source (no 3x3, no image remap), one weight set, NHWC store, K % 64 == 0,
// N % 8 == 0, 16-byte aligned rows; LN with K in {256, 512, 1024} (the statistics kernel)
bool gemm_sk_ok(const GemmArgs& g) {
  if (g.conv3 || g.a.cb_px || g.a.n != 1 || g.store_mode != STORE_NHWC) return false;
  const SrcDesc& s = g.a.s[0];
  const int K = g.a.Ktot;
  if (s.img_mul != 1 || s.img_add != 0 || s.K != K || K % SK_BK || K <= 0 || g.N % 8 || g.N <= 0) return false;
  if (g.wstride && g.M > g.HW) return false;       // one weight set (set 0)
  if (g.ln && K != 256 && K != 512 && K != 1024) return false;
  if (s.ld % 8 || s.off % 8 || g.ldw % 8 || g.ldo % 8 || g.offo % 8) return false;
  if (reinterpret_cast<uintptr_t>(s.base) % 16 || reinterpret_cast<uintptr_t>(g.w) % 16 || reinterpret_cast<uintptr_t>(g.out) % 16) return false;
  if (g.res && (g.ldr % 8 || g.offr % 8 || reinterpret_cast<uintptr_t>(g.res) % 16)) return false;
  return g.M <= INT32_MAX;
}

// ws: gemm_sk_workspace_bytes(M, N, K) bytes (partials, then the LN statistics)
void launch_gemm_sk(const GemmArgs& g, void* ws, hipStream_t st) {
  const int K = g.a.Ktot, S = gemm_sk_splits(g.M, g.N, K);
  float* part = reinterpret_cast<float*>(ws);
  float2* stats = reinterpret_cast<float2*>(part + (size_t)S * g.M * g.N);
  if (g.ln) launch_ln_stats(g, stats, st);
  const int64_t tiles = ((g.M + SK_BM - 1) / SK_BM) * ((g.N + SK_BN - 1) / SK_BN);
  if (S == 1) {
    hipLaunchKernelGGL(gemm_sk_kernel<true>, dim3((unsigned)tiles), dim3(256), 0, st, g, K, part, stats);
    return;
  }
  hipLaunchKernelGGL(gemm_sk_kernel<false>, dim3((unsigned)(tiles * S)), dim3(256), 0, st, g, K / S, part, stats);
  const int64_t n = g.M * (g.N / 8);
  hipLaunchKernelGGL(gemm_sk_epi_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, g, S, part, stats);
}

}  // namespace turtle

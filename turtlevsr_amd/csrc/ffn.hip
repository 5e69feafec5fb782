// Fused FeedForward block ("ffn" kernel) at widths 64 / 128 (levels 1 and 2), bf16:
//
//   out = x + gamma * (W2 gelu(W1 LN(x) + b1) + b2)            (turtle_t1_arch.py:181-210, 804-811)
//
// in one pass over the pixels: x is read once, out written once; the hidden map (2c channels) never
// leaves the registers. The unfused path writes and re-reads it (2c channels per pixel each way).
//
// Structure (MI355X, 16x16x32 bf16 MFMA, fp32 accumulation):
//   * a wave owns 32 pixels at a time (two 16-pixel MFMA columns) and walks pixel groups
//     persistently; the block (8 waves) only shares the weights, staged once in LDS in MFMA
//     A-fragment order (pack_ffn_frags in turtle.cpp): each fragment is 1 KB read by
//     ds_read_b128 at lane * 16 - conflict-free, no swizzle;
//   * GEMM1 (hidden = W1' x): A = W1' rows of a 32-channel hidden chunk in a permuted order (MFMA
//     row 4g + e of sub-tile s <- hidden channel 8g + 4s + e), B = x, 16-byte loads of 8
//     consecutive channels of the lane's pixel straight from HBM. The lane's two sub-tile
//     accumulators then hold hidden channels 8g .. 8g + 7 of its pixel - after the LayerNorm
//     correction and GELU they ARE the B fragment of GEMM2's K step over that chunk (no LDS
//     round trip, no shuffle);
//   * LayerNorm folded algebraically: W1' = W1 diag(g_ln), s = rowsum(W1'), t = W1 b_ln + b1, per
//     pixel LN-GEMM1 = rs (W1' x - mu s) + t with (mu, rs) from the x fragments (two cross-lane
//     adds); BiasFree LN: s = 0, t = b1;
//   * GEMM2 output rows permuted the same way, so a lane's accumulators hold 8 consecutive output
//     channels of its pixel: the residual is the x fragment the lane already holds, and the
//     store is one 16-byte vector per lane and 32 channels;
//   * the next group's x fragments are loaded before the current group's MFMAs (register double
//     buffer), so each wave keeps one group of HBM loads in flight behind its compute.
#include "common.h"
#include "kernels.h"

namespace turtle {

template <int C>
struct FFN {
  static constexpr int HID = 2 * C;          // FeedForward expansion 2 (turtle_t1_arch.py:184)
  static constexpr int KS1 = C / 32;         // GEMM1 K steps
  static constexpr int HC = HID / 32;        // hidden chunks = GEMM2 K steps
  static constexpr int T2 = C / 16;          // GEMM2 output sub-tiles
  static constexpr int NJ = C / 32;          // 32-channel output groups
  static constexpr int W1_FR = HC * 2 * KS1, W2_FR = HC * T2;   // 1-KB fragments
  static constexpr int W_BYTES = (W1_FR + W2_FR) * 1024;
  static constexpr int TAB = W_BYTES;                           // s1[HID] t1[HID] b2[C] g2[C] fp32
  static constexpr int BYTES = TAB + (2 * HID + 2 * C) * 4;
  static constexpr int NW = 8, NT = NW * 64;
  static constexpr int BPC = C <= 64 ? 2 : 1;                   // blocks per CU (LDS / registers)
  static_assert(BYTES <= 160 * 1024, "ffn LDS budget");
};

template <int C>
__global__ __launch_bounds__(512, FFN<C>::BPC) void ffn_kernel(FfnArgs a) {
  using F = FFN<C>;
  typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, pl = lane & 15;

  // ---- weights -> LDS (fragment order, linear copy), then the per-channel tables ----
  {
    const uint4* w1 = reinterpret_cast<const uint4*>(a.w1f);
    const uint4* w2 = reinterpret_cast<const uint4*>(a.w2f);
    uint4* d = reinterpret_cast<uint4*>(smem);
    constexpr int N1 = F::W1_FR * 64, N2 = F::W2_FR * 64;
#pragma unroll 4
    for (int i = tid; i < N1; i += F::NT) d[i] = w1[i];
#pragma unroll 4
    for (int i = tid; i < N2; i += F::NT) d[N1 + i] = w2[i];
    float* tab = reinterpret_cast<float*>(smem + F::TAB);
    for (int i = tid; i < F::HID; i += F::NT) {
      tab[i] = a.s1 ? a.s1[i] : 0.f;
      tab[F::HID + i] = a.t1 ? a.t1[i] : 0.f;
    }
    for (int i = tid; i < C; i += F::NT) {
      tab[2 * F::HID + i] = a.b2 ? a.b2[i] : 0.f;
      tab[2 * F::HID + C + i] = a.g2 ? a.g2[i] : 1.f;
    }
  }
  __syncthreads();
  const char* sW1 = smem + lane * 16;
  const char* sW2 = smem + F::W1_FR * 1024 + lane * 16;
  const float* sS = reinterpret_cast<const float*>(smem + F::TAB);
  const float* sT = sS + F::HID;
  const float* sB = sT + F::HID;
  const float* sG = sB + C;

  const bf16* x = reinterpret_cast<const bf16*>(a.x);
  bf16* out = reinterpret_cast<bf16*>(a.out);
  const int64_t M = a.M, ngrp = (M + 31) / 32;
  const int64_t stride = (int64_t)gridDim.x * F::NW;

  uint4 xn[2][F::KS1];
  auto load_x = [&](int64_t grp, uint4 (&r)[2][F::KS1]) {
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int64_t p = min(grp * 32 + 16 * n + pl, M - 1);
#pragma unroll
      for (int ks = 0; ks < F::KS1; ++ks) r[n][ks] = ld16(x + p * C + 32 * ks + 8 * g);
    }
  };
  int64_t grp = (int64_t)blockIdx.x * F::NW + wid;
  if (grp < ngrp) load_x(grp, xn);
  for (; grp < ngrp; grp += stride) {
    uint4 xc[2][F::KS1];
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int ks = 0; ks < F::KS1; ++ks) xc[n][ks] = xn[n][ks];
    if (grp + stride < ngrp) load_x(grp + stride, xn);

    // ---- LayerNorm statistics of the lane's two pixels (C / 4 channels per lane, 4 lanes) ----
    float mu[2], rs[2];
    {
      typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
      const bf16x2 one2 = __builtin_bit_cast(bf16x2, 0x3F803F80u);
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        float s = 0.f, q = 0.f;
#pragma unroll
        for (int ks = 0; ks < F::KS1; ++ks) {
          const uint32_t w[4] = {xc[n][ks].x, xc[n][ks].y, xc[n][ks].z, xc[n][ks].w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const bf16x2 v2 = __builtin_bit_cast(bf16x2, w[e]);
            s = __builtin_amdgcn_fdot2_f32_bf16(v2, one2, s, false);
            q = __builtin_amdgcn_fdot2_f32_bf16(v2, v2, q, false);
          }
        }
        s += __shfl_xor(s, 16, 64); q += __shfl_xor(q, 16, 64);
        s += __shfl_xor(s, 32, 64); q += __shfl_xor(q, 32, 64);
        mu[n] = s * (1.f / C);
        rs[n] = rsqrtf(fmaxf(q * (1.f / C) - mu[n] * mu[n], 0.f) + 1e-5f);
      }
    }

    f32x4 acc2[2][F::T2];
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int t = 0; t < F::T2; ++t) acc2[n][t] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int hc = 0; hc < F::HC; ++hc) {
      // GEMM1 over hidden chunk hc
      f32x4 acc1[2][2];
#pragma unroll
      for (int n = 0; n < 2; ++n) acc1[n][0] = acc1[n][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int ks = 0; ks < F::KS1; ++ks) {
          const bf16x8v wf = *reinterpret_cast<const bf16x8v*>(sW1 + ((hc * 2 + s) * F::KS1 + ks) * 1024);
#pragma unroll
          for (int n = 0; n < 2; ++n)
            acc1[n][s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, __builtin_bit_cast(bf16x8v, xc[n][ks]), acc1[n][s], 0, 0, 0);
        }
      // LayerNorm correction + bias + GELU -> bf16 B fragment (hidden 32 hc + 8 g + 0..7)
      const int h0 = 32 * hc + 8 * g;
      const f32x4 s_lo = *reinterpret_cast<const f32x4*>(sS + h0), s_hi = *reinterpret_cast<const f32x4*>(sS + h0 + 4);
      const f32x4 t_lo = *reinterpret_cast<const f32x4*>(sT + h0), t_hi = *reinterpret_cast<const f32x4*>(sT + h0 + 4);
      bf16x8v hf[2];
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        // packed f32 pairs (v_pk_fma / v_pk_mul): two hidden channels per VALU issue
        const f32x2 nm = f32x2{-mu[n], -mu[n]}, r2 = f32x2{rs[n], rs[n]};
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const f32x4 sv = s ? s_hi : s_lo, tv = s ? t_hi : t_lo;
#pragma unroll
          for (int i = 0; i < 4; i += 2) {
            const f32x2 v = __builtin_elementwise_fma(
                r2, __builtin_elementwise_fma(nm, f32x2{sv[i], sv[i + 1]}, f32x2{acc1[n][s][i], acc1[n][s][i + 1]}),
                f32x2{tv[i], tv[i + 1]});
            const f32x2 gv = gelu_bf16_2(v);
            hf[n][4 * s + i] = (bf16)gv.x;
            hf[n][4 * s + i + 1] = (bf16)gv.y;
          }
        }
      }
      // GEMM2 K step hc
#pragma unroll
      for (int t = 0; t < F::T2; ++t) {
        const bf16x8v wf = *reinterpret_cast<const bf16x8v*>(sW2 + (hc * F::T2 + t) * 1024);
#pragma unroll
        for (int n = 0; n < 2; ++n) acc2[n][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, hf[n], acc2[n][t], 0, 0, 0);
      }
    }

    // ---- epilogue: lane holds output channels 32 j + 8 g + 0..7 of its pixels ----
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int64_t p = grp * 32 + 16 * n + pl;
      const bool ok = p < M;
#pragma unroll
      for (int j = 0; j < F::NJ; ++j) {
        const int c = 32 * j + 8 * g;
        const f32x4 b_lo = *reinterpret_cast<const f32x4*>(sB + c), b_hi = *reinterpret_cast<const f32x4*>(sB + c + 4);
        const f32x4 g_lo = *reinterpret_cast<const f32x4*>(sG + c), g_hi = *reinterpret_cast<const f32x4*>(sG + c + 4);
        const uint32_t rw[4] = {xc[n][j].x, xc[n][j].y, xc[n][j].z, xc[n][j].w};
        bf16x8 ov;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float acc = acc2[n][2 * j + (e >> 2)][e & 3];
          const float bb = e < 4 ? b_lo[e & 3] : b_hi[e & 3];
          const float gg = e < 4 ? g_lo[e & 3] : g_hi[e & 3];
          const float r = (e & 1) ? __uint_as_float(rw[e >> 1] & 0xffff0000u) : __uint_as_float(rw[e >> 1] << 16);
          ov[e] = (bf16)fmaf(acc + bb, gg, r);
        }
        if (ok) *reinterpret_cast<bf16x8*>(out + p * C + c) = ov;
      }
    }
  }
}

bool ffn_ok(const FfnArgs& a) {
  if (a.C != 64 && a.C != 128) return false;
  if (a.M <= 0 || !a.w1f || !a.w2f) return false;
  if (reinterpret_cast<uintptr_t>(a.x) % 16 || reinterpret_cast<uintptr_t>(a.out) % 16) return false;
  if (reinterpret_cast<uintptr_t>(a.w1f) % 16 || reinterpret_cast<uintptr_t>(a.w2f) % 16) return false;
  for (const float* p : {a.s1, a.t1, a.b2, a.g2})
    if (p && reinterpret_cast<uintptr_t>(p) % 16) return false;
  return true;
}

template <int C>
static void launch_ffn_c(const FfnArgs& a, hipStream_t st) {
  using F = FFN<C>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(ffn_kernel<C>), hipFuncAttributeMaxDynamicSharedMemorySize, F::BYTES);
    attr = true;
  }
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ncu = v;
  }
  const int64_t ngrp = (a.M + 31) / 32, waves = (int64_t)ncu * F::BPC * F::NW;
  const int64_t nblk = std::max<int64_t>(1, std::min<int64_t>((ngrp + F::NW - 1) / F::NW, waves / F::NW));
  hipLaunchKernelGGL(ffn_kernel<C>, dim3((unsigned)nblk), dim3(F::NT), F::BYTES, st, a);
}

void launch_ffn(const FfnArgs& a, hipStream_t st) {
  if (a.C == 64) launch_ffn_c<64>(a, st);
  else launch_ffn_c<128>(a, st);
}

}  // namespace turtle

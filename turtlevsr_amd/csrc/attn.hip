// Channel ("transposed") attention for ChannelAttention / FrameHistoryRouter / the FHR inside the
// Causal History Model (turtle_t1_arch.py:218-286, 612-662, 666-702), restructured for HBM:
//
//   1. gram:      split over pixels, per (batch, head): G = q^T [k_seg0 | k_seg1 | ...] and the
//                 per-channel sums of squares (for F.normalize over HW), fp32 MFMA 16x16x4.
//   2. rows:      reduce the pixel-chunk partials (deterministic order), logits =
//                 G / (|q_i| |k_j|) * temperature, row softmax (over all cached + current key
//                 rows of the head), 1/|k_cur| for the FHR cache.
//   3. weff:      fold attention into the projection: W_eff = project_out . blockdiag(A_h), so
//                 project_out(A v) becomes ONE pointwise GEMM over the K-concatenated value
//                 sources (current v, cached v rows, CHM history frames) with the residual add
//                 in its epilogue (gemm.hip). No attention output map is ever written.
#include "common.h"
#include "kernels.h"

namespace turtle {

#ifndef TURTLE_GRAM_TR
#define TURTLE_GRAM_TR 1
#endif
constexpr int GMAXT = 24;        // max 16x16 accumulator tiles per wave (ch=64, 6 segments)

__device__ __attribute__((aligned(64))) uint4 g_zero_gram[4];

// q^T [k_seg0 | k_seg1 | ...] over a pixel chunk, plus per-column sums of squares.
// LDS holds [pixel][channel] tiles exactly as they sit in HBM (16-byte row chunks); the MFMA
// operands need 8 consecutive pixels of one channel per lane, which ds_read_b64_tr_b16 delivers
// (two 4-row transposed reads), so nothing is transposed in registers.
// Staging: thread t owns channel vector cv = t % CVt of pixel rows t / CVt + PS u (PS = 256 / CVt
// rows per pass, up to GNU passes), so its sum of squares is a single VEC accumulator; a step of
// GP pixels keeps ~16-32 KB per block in flight. MT = accumulator tiles per wave (compile time,
// so the accumulators of a 1-segment Gram do not cost the registers of a 6-segment one).
constexpr int GNU = 8;
// byte offset of the norms in the Gram kernel's dynamic LDS: past the [GP] operand rows and past
// the [PS][ch + ncol] fp32 norm partials that reuse them after the pixel loop
__host__ __device__ inline int gram_nrm_off(int GP, int ch, int ncol, int ES, int VEC) {
  const int tiles = GP * ((ch + ncol) * ES + 32);
  const int parts = (256 / ((ch + ncol) / VEC)) * (ch + ncol) * 4;
  return tiles > parts ? tiles : parts;
}
template <typename T, int GP, int MT>
// two blocks per CU (<= 256 VGPRs) wherever that costs no spills: up to 20 accumulator tiles per wave
// at 32-pixel steps (the 5-segment CHM Grams: 1 -> 2 waves per SIMD, L2 311 -> 204 us at 1080p)
__global__ __launch_bounds__(256, (MT <= 8 || (MT <= 16 && GP <= 64) || (MT <= 20 && GP <= 32)) ? 2 : 1) void gram_kernel(GramArgs a) {
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  constexpr int VEC = Vec<T>::N, ES = sizeof(T);
  const int ch = a.ch, ncol = a.nseg * ch;
  const int RQ = ch * ES + 16, RK = ncol * ES + 16;          // LDS row strides (bytes)
  char* sq = gsm;                                            // [GP][RQ]
  char* sk = gsm + GP * RQ;                                  // [GP][RK]
  const int bh = blockIdx.x / a.nchunk, chunk = blockIdx.x % a.nchunk;
  const int b = bh / a.heads, h = bh % a.heads;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int p_beg = chunk * a.chunk, p_end = min(a.HW, p_beg + a.chunk);
  const int tj_n = ncol / 16, TT = (ch / 16) * tj_n;
  const int qv = ch / VEC, CVt = (ch + ncol) / VEC;          // vectors per pixel
  const int PS = 256 / CVt;                                  // pixel rows per pass
  // [ch + ncol] norms after the operand tiles / the norm partials, whichever is larger
  float* nrm = reinterpret_cast<float*>(gsm + gram_nrm_off(GP, ch, ncol, ES, VEC));
  const int cv = tid % CVt, pg = tid / CVt;
  const bool tact = pg < PS;

  for (int i = tid; i < ch + ncol; i += 256) nrm[i] = 0.f;

  const T* src;
  int64_t pst;
  char* lrow;
  int lstride;
  if (cv < qv) {
    src = reinterpret_cast<const T*>(a.q) + (int64_t)b * a.HW * a.ldq + a.qoff + h * ch + cv * VEC;
    pst = a.ldq;
    lrow = sq + cv * VEC * ES;
    lstride = RQ;
  } else {
    const int kc = (cv - qv) * VEC, s = kc / ch, jj = kc - s * ch;
    GramSeg g = a.seg[0];
#pragma unroll
    for (int q = 1; q < TURTLE_MAX_SEG; ++q)
      if (s == q) g = a.seg[q];
    src = reinterpret_cast<const T*>(g.base) + ((int64_t)b * g.img_mul + g.img_add) * a.HW * g.ld + g.off +
          (int64_t)h * g.hstride + jj;
    pst = g.ld;
    lrow = sk + kc * ES;
    lstride = RK;
  }

  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float sqs[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) sqs[e] = 0.f;

  uint4 stg[GNU];
  auto load = [&](int p0) {
#pragma unroll
    for (int u = 0; u < GNU; ++u) {
      const int px = pg + PS * u, p = p0 + px;
      const bool ok = tact && px < GP && p < p_end;
      stg[u] = ld16(ok ? reinterpret_cast<const void*>(src + (int64_t)p * pst) : g_zero_gram);
    }
  };

  load(p_beg);
  for (int p0 = p_beg; p0 < p_end; p0 += GP) {
#pragma unroll
    for (int u = 0; u < GNU; ++u) {
      const int px = pg + PS * u;
      if (!tact || px >= GP) continue;
      *reinterpret_cast<uint4*>(lrow + px * lstride) = stg[u];
      float x[VEC];
      if constexpr (sizeof(T) == 2) {
        const uint32_t w[4] = {stg[u].x, stg[u].y, stg[u].z, stg[u].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) { x[2 * i] = __uint_as_float(w[i] << 16); x[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u); }
      } else {
        x[0] = __uint_as_float(stg[u].x); x[1] = __uint_as_float(stg[u].y);
        x[2] = __uint_as_float(stg[u].z); x[3] = __uint_as_float(stg[u].w);
      }
#pragma unroll
      for (int e = 0; e < VEC; ++e) sqs[e] = fmaf(x[e], x[e], sqs[e]);
    }
    __syncthreads();
    if (p0 + GP < p_end) load(p0 + GP);
    if constexpr (sizeof(T) == 2 && TURTLE_GRAM_TR) {
      // lane l: rows (pixels) 8*(l>>4) + q (+4), columns c0 + 4p; receives column c0 + (l&15)
      const int g16 = lane >> 4, li = lane & 15, qq = li >> 2, pp = li & 3;
      typedef short v4s __attribute__((ext_vector_type(4)));
      typedef __attribute__((address_space(3))) v4s lds_v4s;
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int tile = wid + 4 * t;
        if (tile < TT) {
          const int it = tile / tj_n, jt = tile - it * tj_n;
#pragma unroll
          for (int ss = 0; ss < GP / 32; ++ss) {
            const char* qa = sq + (32 * ss + 8 * g16 + qq) * RQ + (it * 16 + 4 * pp) * 2;
            const char* ka = sk + (32 * ss + 8 * g16 + qq) * RK + (jt * 16 + 4 * pp) * 2;
            const v4s a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)qa);
            const v4s a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(qa + 4 * RQ));
            const v4s b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)ka);
            const v4s b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(ka + 4 * RK));
            typedef short v8s __attribute__((ext_vector_type(8)));
            const bf16x8 af = __builtin_bit_cast(bf16x8, (v8s)__builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7));
            const bf16x8 bfr = __builtin_bit_cast(bf16x8, (v8s)__builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7));
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc[t], 0, 0, 0);
          }
        }
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < GP; kk += 4) {
        const int pr = kk + (lane >> 4);
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          const int tile = wid + 4 * t;
          if (tile < TT) {
            const int it = tile / tj_n, jt = tile - it * tj_n;
            const float av = to_f(*reinterpret_cast<const T*>(sq + pr * RQ + (it * 16 + (lane & 15)) * ES));
            const float bv = to_f(*reinterpret_cast<const T*>(sk + pr * RK + (jt * 16 + (lane & 15)) * ES));
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[t], 0, 0, 0);
          }
        }
      }
    }
    __syncthreads();
  }
  // column sums of squares: PS threads per channel vector, summed in a fixed order (the operand
  // tiles are dead after the loop's last barrier, so their LDS holds the [PS][ch + ncol] partials:
  // PS * (ch + ncol) * 4 <= GP * (RQ + RK) for every GP >= 32). LDS float atomics here made the
  // norms - and through bf16 rounding the whole frame - differ run to run.
  {
    float* part = reinterpret_cast<float*>(gsm);
    const int ncw = ch + ncol;
    if (tact) {
#pragma unroll
      for (int e = 0; e < VEC; ++e) part[pg * ncw + cv * VEC + e] = sqs[e];
    }
    __syncthreads();
    for (int i = tid; i < ncw; i += 256) {
      float s = 0.f;
      for (int r = 0; r < PS; ++r) s += part[r * ncw + i];
      nrm[i] = s;
    }
  }
  __syncthreads();
  const int stride = ch * ncol + ch + ncol;
  float* out = a.part + ((int64_t)bh * a.nchunk + chunk) * stride;
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    const int tile = wid + 4 * t;
    if (tile < TT) {
      const int it = tile / tj_n, jt = tile % tj_n;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out[(it * 16 + (lane >> 4) * 4 + r) * ncol + jt * 16 + (lane & 15)] = acc[t][r];
    }
  }
  for (int i = tid; i < ch + ncol; i += 256) out[ch * ncol + i] = nrm[i];   // [nq (ch) | nk (ncol)]
}

template <typename T, int GP, int MT>
static void launch_gram_cfg(const GramArgs& a, hipStream_t st) {
  const int ncol = a.nseg * a.ch;
  const size_t lds = (size_t)gram_nrm_off(GP, a.ch, ncol, (int)sizeof(T), Vec<T>::N) + (a.ch + ncol) * sizeof(float);
  hipLaunchKernelGGL((gram_kernel<T, GP, MT>), dim3((unsigned)(a.B * a.heads * a.nchunk)), dim3(256), lds, st, a);
}

template <typename T, int GP>
static void launch_gram_gp(const GramArgs& a, hipStream_t st) {
  const int tt = (a.ch / 16) * (a.nseg * a.ch / 16), mt = (tt + 3) / 4;
  if (mt <= 4) launch_gram_cfg<T, GP, 4>(a, st);
  else if (mt <= 8) launch_gram_cfg<T, GP, 8>(a, st);
  else if (mt <= 16) launch_gram_cfg<T, GP, 16>(a, st);
  else if (mt <= 20) launch_gram_cfg<T, GP, 20>(a, st);
  else launch_gram_cfg<T, GP, GMAXT>(a, st);
}

template <typename T>
void launch_gram(const GramArgs& a, hipStream_t st) {
  const int cvt = (a.ch + a.nseg * a.ch) / Vec<T>::N;
  const int ps = 256 / cvt, rows = ps * GNU;                  // pixel rows GNU passes can stage
  if constexpr (sizeof(T) == 2) {
    if (rows >= 128) launch_gram_gp<T, 128>(a, st);
    else if (rows >= 64) launch_gram_gp<T, 64>(a, st);
    else launch_gram_gp<T, 32>(a, st);
  } else {
    launch_gram_gp<T, 16>(a, st);
  }
}

// Reduce the per-chunk Gram partials: red[bh][e] = sum_c part[bh][c][e]. Block = 64 consecutive
// entries x 4 chunk groups; each lane keeps 8 loads in flight, the 4 group sums meet in LDS
// (fixed order: deterministic).
__global__ __launch_bounds__(256) void gram_sum_kernel(const float* part, float* red, int nchunk, int stride) {
  __shared__ float ps[4][64];
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + lane, bh = blockIdx.y;
  const int ec = min(e, stride - 1);
  const float* p = part + (int64_t)bh * nchunk * stride + ec;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int c = grp;
  for (; c + 28 < nchunk; c += 32) {
#pragma unroll
    for (int u = 0; u < 8; ++u) s[u] += p[(int64_t)(c + 4 * u) * stride];
  }
  for (; c < nchunk; c += 4) s[0] += p[(int64_t)c * stride];
  ps[grp][lane] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  if (grp == 0 && e < stride) red[(int64_t)bh * stride + e] = (ps[0][lane] + ps[1][lane]) + (ps[2][lane] + ps[3][lane]);
}

// Row softmax of the channel-attention logits, one wave per (query row i, b*h):
//   A[i][j] = softmax_j( G[i][j] * tau_h / (|q_i| |k_j|) )   over all ncol key columns
// (turtle_t1_arch.py:357-366, 686-692). Row 0 also writes 1/|k_cur| for the FHR cache.
constexpr int AR_KC = 8;             // ncol <= 512 = 8 x 64 lanes
__global__ __launch_bounds__(256) void attn_row_kernel(AttnFinArgs a) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), bh = blockIdx.y, b = bh / a.heads, h = bh % a.heads;
  const int ch = a.ch, ncol = a.nseg * ch, stride = ch * ncol + ch + ncol;
  if (i >= ch) return;
  const float* R = a.red + (int64_t)bh * stride;
  float G[AR_KC], N[AR_KC];
#pragma unroll
  for (int k = 0; k < AR_KC; ++k) {
    const int jc = min(lane + 64 * k, ncol - 1);
    G[k] = R[i * ncol + jc];
    N[k] = R[ch * ncol + ch + jc];
  }
  const float qn = a.tau[h] / fmaxf(sqrtf(R[ch * ncol + i]), 1e-12f);
  float lg[AR_KC], kv[AR_KC];
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < AR_KC; ++k) {
    const int j = lane + 64 * k;
    const int sgm = min(j, ncol - 1) / ch;
    kv[k] = ((a.norm_mask >> sgm) & 1) ? 1.f / fmaxf(sqrtf(N[k]), 1e-12f) : 1.f;
    lg[k] = j < ncol ? G[k] * qn * kv[k] : -INFINITY;
    mx = fmaxf(mx, lg[k]);
  }
  mx = wave_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < AR_KC; ++k) {
    lg[k] = lane + 64 * k < ncol ? expf(lg[k] - mx) : 0.f;
    sum += lg[k];
  }
  const float inv = 1.f / wave_sum(sum);
  float* A = a.attn + ((int64_t)bh * ch + i) * ncol;
#pragma unroll
  for (int k = 0; k < AR_KC; ++k)
    if (lane + 64 * k < ncol) A[lane + 64 * k] = lg[k] * inv;
  if (i == 0 && a.kinv && a.cur_seg >= 0) {
#pragma unroll
    for (int k = 0; k < AR_KC; ++k) {
      const int j = lane + 64 * k;
      if (j >= a.cur_seg * ch && j < (a.cur_seg + 1) * ch)
        a.kinv[(int64_t)b * a.heads * ch + h * ch + (j - a.cur_seg * ch)] = kv[k];
    }
  }
}

int attn_nsplit(int nchunk) { return 1; }

void launch_attn_finalize(const AttnFinArgs& a, hipStream_t st) {
  const int ncol = a.nseg * a.ch, stride = a.ch * ncol + a.ch + ncol, nbh = a.B * a.heads;
  hipLaunchKernelGGL(gram_sum_kernel, dim3((unsigned)((stride + 63) / 64), (unsigned)nbh), dim3(256), 0, st, a.part, a.red,
                     a.nchunk, stride);
  if (!a.sum_only) hipLaunchKernelGGL(attn_row_kernel, dim3((unsigned)((a.ch + 3) / 4), (unsigned)nbh), dim3(256), 0, st, a);
}

// Fold the attention into the projection, one block per (32 output channels, 64 key columns,
// b*h): W_eff[b][o][col(j)] = sum_i Wp[o][h*ch + i] * A[i][j] (A and Wp slabs staged in LDS), so
// project_out(A v) becomes one GEMM over the K-concatenated value sources. The launch is tiny
// (tens of blocks) and latency-bound: every slab load of a thread is issued before the first LDS
// store (16-byte loads from clamped addresses, zeroed after), one HBM / L2 round trip per block.
constexpr int WF_MAXCH = 128;
template <typename T, bool V4>
__global__ __launch_bounds__(256) void attn_weff_kernel(WeffArgs a) {
  __shared__ __attribute__((aligned(16))) float sA[WF_MAXCH][64];
  __shared__ __attribute__((aligned(16))) float sW[WF_MAXCH][32];    // [i][o]
  const int ch = a.ch, ncol = a.nseg * ch;
  const int o0 = blockIdx.x * 32, j0 = blockIdx.y * 64, bh = blockIdx.z;
  const int b = bh / a.heads, h = bh % a.heads;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const float* A = a.attn + (int64_t)bh * ch * ncol;
  if constexpr (V4) {
    // A slab [ch][64]: 16 float4 per row; Wp slab [32][ch]: ch / 4 float4 per output row
    constexpr int NA = WF_MAXCH * 16 / 256, NW = 32 * WF_MAXCH / 4 / 256;
    const int nwr = ch / 4;                                    // float4 per Wp row
    float4 ra[NA], rw[NW];
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      const int e = tid + 256 * k, i = min(e >> 4, ch - 1), c = min(j0 + (e & 15) * 4, ncol - 4);
      ra[k] = *reinterpret_cast<const float4*>(A + (int64_t)i * ncol + c);
    }
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      const int e = tid + 256 * k, oo = e / nwr, i4 = e - oo * nwr;
      const int o = min(o0 + oo, a.C - 1);
      rw[k] = *reinterpret_cast<const float4*>(a.wp + (int64_t)o * a.C + h * ch + min(i4, nwr - 1) * 4);
    }
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      const int e = tid + 256 * k, i = e >> 4, jj = (e & 15) * 4;
      if (i < ch) {
        const bool ok = j0 + jj < ncol;
        *reinterpret_cast<float4*>(&sA[i][jj]) = ok ? ra[k] : float4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      const int e = tid + 256 * k, oo = e / nwr, i4 = e - oo * nwr;
      if (oo < 32) {
        const bool ok = o0 + oo < a.C;
        sW[4 * i4][oo] = ok ? rw[k].x : 0.f;
        sW[4 * i4 + 1][oo] = ok ? rw[k].y : 0.f;
        sW[4 * i4 + 2][oo] = ok ? rw[k].z : 0.f;
        sW[4 * i4 + 3][oo] = ok ? rw[k].w : 0.f;
      }
    }
  } else {
    for (int e = tid; e < ch * 64; e += 256) {
      const int i = e >> 6, jj = e & 63;
      sA[i][jj] = j0 + jj < ncol ? A[i * ncol + j0 + jj] : 0.f;
    }
    for (int e = tid; e < 32 * ch; e += 256) {
      const int oo = e / ch, i = e - oo * ch;
      sW[i][oo] = o0 + oo < a.C ? a.wp[(int64_t)(o0 + oo) * a.C + h * ch + i] : 0.f;
    }
  }
  __syncthreads();
  const int jj = lane, og = wid * 8;
  float acc[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) acc[u] = 0.f;
  for (int i = 0; i < ch; ++i) {
    const float av = sA[i][jj];
    const float4 w0 = *reinterpret_cast<const float4*>(&sW[i][og]);
    const float4 w1 = *reinterpret_cast<const float4*>(&sW[i][og + 4]);
    acc[0] = fmaf(w0.x, av, acc[0]); acc[1] = fmaf(w0.y, av, acc[1]);
    acc[2] = fmaf(w0.z, av, acc[2]); acc[3] = fmaf(w0.w, av, acc[3]);
    acc[4] = fmaf(w1.x, av, acc[4]); acc[5] = fmaf(w1.y, av, acc[5]);
    acc[6] = fmaf(w1.z, av, acc[6]); acc[7] = fmaf(w1.w, av, acc[7]);
  }
  const int col = j0 + jj;
  if (col >= ncol) return;
  const int sg = col / ch, j = col - sg * ch;
  int64_t scol = a.seg_col[0];
  int shs = a.seg_hstride[0];
#pragma unroll
  for (int q = 1; q < TURTLE_MAX_SEG; ++q)
    if (sg == q) { scol = a.seg_col[q]; shs = a.seg_hstride[q]; }
  T* W = reinterpret_cast<T*>(a.weff) + (int64_t)b * a.C * a.Keff + scol + (int64_t)h * shs + j;
#pragma unroll
  for (int u = 0; u < 8; ++u)
    if (o0 + og + u < a.C) W[(int64_t)(o0 + og + u) * a.Keff] = from_f<T>(acc[u]);
}

template <typename T>
void launch_weff(const WeffArgs& a, hipStream_t st) {
  const int ncol = a.nseg * a.ch;
  const dim3 grid((unsigned)((a.C + 31) / 32), (unsigned)((ncol + 63) / 64), (unsigned)(a.B * a.heads));
  // 16-byte slab loads need 4-aligned rows: ch, C (and so ncol) multiples of 4
  if (a.ch % 4 == 0 && a.C % 4 == 0 && a.ch <= WF_MAXCH) hipLaunchKernelGGL((attn_weff_kernel<T, true>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((attn_weff_kernel<T, false>), grid, dim3(256), 0, st, a);
}

// attn_row_kernel folded into the W_eff kernel (one launch fewer per attention site, the attention
// matrix never written): every block stages its head's reduced Gram sums (ch x ncol <= 8192 floats)
// and norms in LDS with all loads in flight at once, recomputes the row softmax over all ncol key
// columns and keeps its own 64 columns; the Wp slab loads are in flight meanwhile. Same per-element
// arithmetic as attn_row_kernel + attn_weff_kernel<T, true>.
constexpr int WFF_MAXG = 8192, WFF_MAXCOL = 128;
template <typename T>
__global__ __launch_bounds__(256) void attn_weff_fin_kernel(WeffArgs a, AttnFinArgs f) {
  __shared__ __attribute__((aligned(16))) float sA[WF_MAXCH][64];
  __shared__ __attribute__((aligned(16))) float sW[WF_MAXCH][32];    // [i][o]
  __shared__ __attribute__((aligned(16))) float sG[WFF_MAXG];        // [i][j] Gram sums
  __shared__ float sN[256];                                          // |q_i|^2, then |k_j|^2
  __shared__ float sX[4 * 256];                                      // sink of the out-of-range slab stores
  const int ch = a.ch, ncol = a.nseg * ch, stride = ch * ncol + ch + ncol;
  const int o0 = blockIdx.x * 32, j0 = blockIdx.y * 64, bh = blockIdx.z;
  const int b = bh / a.heads, h = bh % a.heads;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const float* R = f.red + (int64_t)bh * stride;
  const float tau = f.tau[h];
  // every load of the block first: Wp slab [32][ch], the Gram slab, the norms
  constexpr int NW = 32 * WF_MAXCH / 4 / 256, NG = WFF_MAXG / 4 / 256;
  const int nwr = ch / 4, ng4 = ch * ncol / 4;
  float4 rw[NW], rg[NG];
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const int e = tid + 256 * k, oo = e / nwr, i4 = e - oo * nwr;
    const int o = min(o0 + oo, a.C - 1);
    rw[k] = *reinterpret_cast<const float4*>(a.wp + (int64_t)o * a.C + h * ch + min(i4, nwr - 1) * 4);
  }
#pragma unroll
  for (int k = 0; k < NG; ++k) rg[k] = *reinterpret_cast<const float4*>(R + 4 * min(tid + 256 * k, ng4 - 1));
  const float rn = R[ch * ncol + min(tid, ch + ncol - 1)];
  // unconditional LDS stores (entries past the slab are never read; out-of-range W rows go to the
  // sink): a store under a branch would pull its load down next to it, one L2 round trip each
#pragma unroll
  for (int k = 0; k < NG; ++k) *reinterpret_cast<float4*>(&sG[4 * (tid + 256 * k)]) = rg[k];
  sN[tid] = rn;
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const int e = tid + 256 * k, oo = e / nwr, i4 = e - oo * nwr;
    const bool ok = o0 + oo < a.C;
    float* d0 = oo < 32 ? &sW[4 * i4][oo] : &sX[tid];
    const int st = oo < 32 ? 32 : 256;
    d0[0] = ok ? rw[k].x : 0.f;
    d0[st] = ok ? rw[k].y : 0.f;
    d0[2 * st] = ok ? rw[k].z : 0.f;
    d0[3 * st] = ok ? rw[k].w : 0.f;
  }
  __syncthreads();
  // column scales (the same for every row): 1 / |k_j| for normalised segments
  constexpr int KC = WFF_MAXCOL / 64;
  float kv[KC];
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const int jc = min(lane + 64 * k, ncol - 1), sgm = jc / ch;
    kv[k] = ((f.norm_mask >> sgm) & 1) ? 1.f / fmaxf(sqrtf(sN[ch + jc]), 1e-12f) : 1.f;
  }
  if (blockIdx.x == 0 && f.kinv && f.cur_seg >= 0 && wid == 0) {
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int j = lane + 64 * k;
      if (j >= j0 && j < j0 + 64 && j >= f.cur_seg * ch && j < (f.cur_seg + 1) * ch)
        f.kinv[(int64_t)b * a.heads * ch + h * ch + (j - f.cur_seg * ch)] = kv[k];
    }
  }
  for (int i = wid; i < ch; i += 4) {
    const float qn = tau / fmaxf(sqrtf(sN[i]), 1e-12f);
    float lg[KC];
    float mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int j = lane + 64 * k;
      lg[k] = j < ncol ? sG[i * ncol + min(j, ncol - 1)] * qn * kv[k] : -INFINITY;
      mx = fmaxf(mx, lg[k]);
    }
    mx = wave_max(mx);
    float sum = 0.f, mine = 0.f;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      lg[k] = lane + 64 * k < ncol ? expf(lg[k] - mx) : 0.f;
      sum += lg[k];
      mine = (int)blockIdx.y == k ? lg[k] : mine;
    }
    const float inv = 1.f / wave_sum(sum);
    sA[i][lane] = j0 + lane < ncol ? mine * inv : 0.f;
  }
  __syncthreads();
  const int jj = lane, og = wid * 8;
  float acc[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) acc[u] = 0.f;
  for (int i = 0; i < ch; ++i) {
    const float av = sA[i][jj];
    const float4 w0 = *reinterpret_cast<const float4*>(&sW[i][og]);
    const float4 w1 = *reinterpret_cast<const float4*>(&sW[i][og + 4]);
    acc[0] = fmaf(w0.x, av, acc[0]); acc[1] = fmaf(w0.y, av, acc[1]);
    acc[2] = fmaf(w0.z, av, acc[2]); acc[3] = fmaf(w0.w, av, acc[3]);
    acc[4] = fmaf(w1.x, av, acc[4]); acc[5] = fmaf(w1.y, av, acc[5]);
    acc[6] = fmaf(w1.z, av, acc[6]); acc[7] = fmaf(w1.w, av, acc[7]);
  }
  const int col = j0 + jj;
  if (col >= ncol) return;
  const int sg = col / ch, j = col - sg * ch;
  int64_t scol = a.seg_col[0];
  int shs = a.seg_hstride[0];
#pragma unroll
  for (int q = 1; q < TURTLE_MAX_SEG; ++q)
    if (sg == q) { scol = a.seg_col[q]; shs = a.seg_hstride[q]; }
  T* W = reinterpret_cast<T*>(a.weff) + (int64_t)b * a.C * a.Keff + scol + (int64_t)h * shs + j;
#pragma unroll
  for (int u = 0; u < 8; ++u)
    if (o0 + og + u < a.C) W[(int64_t)(o0 + og + u) * a.Keff] = from_f<T>(acc[u]);
}

bool weff_fin_ok(const WeffArgs& a) {
  const int ncol = a.nseg * a.ch;
  return a.ch % 4 == 0 && a.C % 4 == 0 && a.ch <= WF_MAXCH && ncol <= WFF_MAXCOL && a.ch * ncol <= WFF_MAXG;
}

template <typename T>
void launch_weff_fin(const WeffArgs& a, const AttnFinArgs& f, hipStream_t st) {
  const int ncol = a.nseg * a.ch;
  const dim3 grid((unsigned)((a.C + 31) / 32), (unsigned)((ncol + 63) / 64), (unsigned)(a.B * a.heads));
  hipLaunchKernelGGL((attn_weff_fin_kernel<T>), grid, dim3(256), 0, st, a, f);
}

template void launch_gram<float>(const GramArgs&, hipStream_t);
template void launch_gram<bf16>(const GramArgs&, hipStream_t);
template void launch_weff<float>(const WeffArgs&, hipStream_t);
template void launch_weff<bf16>(const WeffArgs&, hipStream_t);
template void launch_weff_fin<float>(const WeffArgs&, const AttnFinArgs&, hipStream_t);
template void launch_weff_fin<bf16>(const WeffArgs&, const AttnFinArgs&, hipStream_t);

}  // namespace turtle

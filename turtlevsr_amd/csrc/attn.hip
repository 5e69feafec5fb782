// Channel ("transposed") attention for ChannelAttention / FrameHistoryRouter / the FHR inside the
// Causal History Model (turtle_t1_arch.py:218-286, 612-662, 666-702), restructured for HBM:
//
//   1. gram:      split over pixels, per (batch, head): G = q^T [k_seg0 | k_seg1 | ...] and the
//                 per-channel sums of squares (for F.normalize over HW), fp32 MFMA 16x16x4.
//   2. finalize:  reduce the pixel splits, logits = G / (|q_i| |k_j|) * temperature, row softmax
//                 (over all cached + current key rows of the head), 1/|k_cur| for the FHR cache.
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
template <typename T> constexpr int gram_gp() { return sizeof(T) == 2 ? 32 : 16; }  // pixels per step
constexpr int GMAXT = 24;        // max 16x16 accumulator tiles per wave (ch=64, 6 segments)
constexpr int GMAXV = 7;         // max 16-byte staging vectors per thread per step

__device__ __attribute__((aligned(64))) uint4 g_zero_gram[4];

// q^T [k_seg0 | k_seg1 | ...] over a pixel chunk, plus per-column sums of squares.
// LDS holds [pixel][channel] tiles exactly as they sit in HBM (16-byte row chunks); the MFMA
// operands need 8 consecutive pixels of one channel per lane, which ds_read_b64_tr_b16 delivers
// (two 4-row transposed reads), so nothing is transposed in registers.
template <typename T>
__global__ __launch_bounds__(256) void gram_kernel(GramArgs a) {
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  constexpr int VEC = Vec<T>::N, ES = sizeof(T), GP = gram_gp<T>();
  const int ch = a.ch, ncol = a.nseg * ch;
  const int RQ = ch * ES + 16, RK = ncol * ES + 16;          // LDS row strides (bytes)
  char* sq = gsm;                                            // [GP][RQ]
  char* sk = gsm + GP * RQ;                                  // [GP][RK]
  float* nrm = reinterpret_cast<float*>(gsm + GP * (RQ + RK)); // [ch + ncol]
  const int bh = blockIdx.x / a.nchunk, chunk = blockIdx.x % a.nchunk;
  const int b = bh / a.heads, h = bh % a.heads;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int p_beg = chunk * a.chunk, p_end = min(a.HW, p_beg + a.chunk);
  const int tj_n = ncol / 16, TT = (ch / 16) * tj_n;
  const int qv = ch / VEC, CVt = (ch + ncol) / VEC;          // vectors per pixel
  const int NV = GP * CVt;

  for (int i = tid; i < ch + ncol; i += 256) nrm[i] = 0.f;

  // per-thread staging geometry (fixed across steps)
  const T* src[GMAXV];
  int64_t pstride[GMAXV];
  int lds_off[GMAXV], vpx[GMAXV];
#pragma unroll
  for (int j = 0; j < GMAXV; ++j) {
    const int v = tid + 256 * j;
    const int px = v / CVt, cv = v % CVt;
    vpx[j] = v < NV ? px : -1;
    if (cv < qv) {
      src[j] = reinterpret_cast<const T*>(a.q) + (int64_t)b * a.HW * a.ldq + a.qoff + h * ch + cv * VEC;
      pstride[j] = a.ldq;
      lds_off[j] = px * RQ + cv * VEC * ES;
    } else {
      const int kc = (cv - qv) * VEC, s = kc / ch, jj = kc - s * ch;
      const GramSeg& g = a.seg[s < a.nseg ? s : 0];
      src[j] = reinterpret_cast<const T*>(g.base) + ((int64_t)b * g.img_mul + g.img_add) * a.HW * g.ld + g.off +
               (int64_t)h * g.hstride + jj;
      pstride[j] = g.ld;
      lds_off[j] = GP * RQ + px * RK + kc * ES;
    }
  }

  f32x4 acc[GMAXT];
#pragma unroll
  for (int t = 0; t < GMAXT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float sqs[GMAXV][VEC];
#pragma unroll
  for (int j = 0; j < GMAXV; ++j)
#pragma unroll
    for (int e = 0; e < VEC; ++e) sqs[j][e] = 0.f;

  uint4 stg[GMAXV];
  auto load = [&](int p0) {
#pragma unroll
    for (int j = 0; j < GMAXV; ++j) {
      const int p = p0 + vpx[j];
      const bool ok = vpx[j] >= 0 && p < p_end;
      stg[j] = ld16(ok ? reinterpret_cast<const void*>(src[j] + (int64_t)p * pstride[j]) : g_zero_gram);
    }
  };

  load(p_beg);
  for (int p0 = p_beg; p0 < p_end; p0 += GP) {
#pragma unroll
    for (int j = 0; j < GMAXV; ++j) {
      if (vpx[j] < 0) continue;
      *reinterpret_cast<uint4*>(gsm + lds_off[j]) = stg[j];
      float x[VEC];
      if constexpr (sizeof(T) == 2) {
        const uint32_t w[4] = {stg[j].x, stg[j].y, stg[j].z, stg[j].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) { x[2 * i] = __uint_as_float(w[i] << 16); x[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u); }
      } else {
        x[0] = __uint_as_float(stg[j].x); x[1] = __uint_as_float(stg[j].y);
        x[2] = __uint_as_float(stg[j].z); x[3] = __uint_as_float(stg[j].w);
      }
#pragma unroll
      for (int e = 0; e < VEC; ++e) sqs[j][e] = fmaf(x[e], x[e], sqs[j][e]);
    }
    __syncthreads();
    if (p0 + GP < p_end) load(p0 + GP);
    if constexpr (sizeof(T) == 2 && TURTLE_GRAM_TR) {
      // lane l: rows (pixels) 8*(l>>4) + q (+4), columns c0 + 4p; receives column c0 + (l&15)
      const int g16 = lane >> 4, li = lane & 15, qq = li >> 2, pp = li & 3;
      typedef short v4s __attribute__((ext_vector_type(4)));
      typedef __attribute__((address_space(3))) v4s lds_v4s;
#pragma unroll
      for (int t = 0; t < GMAXT; ++t) {
        const int tile = wid + 4 * t;
        if (tile < TT) {
          const int it = tile / tj_n, jt = tile - it * tj_n;
          const char* qa = sq + (8 * g16 + qq) * RQ + (it * 16 + 4 * pp) * 2;
          const char* ka = sk + (8 * g16 + qq) * RK + (jt * 16 + 4 * pp) * 2;
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
    } else {
#pragma unroll
      for (int kk = 0; kk < GP; kk += 4) {
        const int pr = kk + (lane >> 4);
#pragma unroll
        for (int t = 0; t < GMAXT; ++t) {
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
  // column sums of squares: per-thread partials -> LDS atomics
#pragma unroll
  for (int j = 0; j < GMAXV; ++j) {
    if (vpx[j] < 0) continue;
    const int cv = (tid + 256 * j) % CVt;
#pragma unroll
    for (int e = 0; e < VEC; ++e) atomicAdd(&nrm[cv * VEC + e], sqs[j][e]);
  }
  __syncthreads();
  const int stride = ch * ncol + ch + ncol;
  float* out = a.part + ((int64_t)bh * a.nchunk + chunk) * stride;
#pragma unroll
  for (int t = 0; t < GMAXT; ++t) {
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

template <typename T>
void launch_gram(const GramArgs& a, hipStream_t st) {
  const int ncol = a.nseg * a.ch;
  const size_t lds = (size_t)gram_gp<T>() * ((a.ch + ncol) * sizeof(T) + 32) + (a.ch + ncol) * sizeof(float);
  hipLaunchKernelGGL(gram_kernel<T>, dim3((unsigned)(a.B * a.heads * a.nchunk)), dim3(256), lds, st, a);
}

// reduce the pixel splits in two deterministic levels: this kernel sums the chunks of split g
// (c = g, g + S, ...) into red[bh][g][e]; the softmax kernel adds the S partial sums it reads
__global__ __launch_bounds__(256) void gram_reduce_kernel(const float* part, float* red, int nchunk, int stride, int S) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= stride) return;
  const int bh = blockIdx.y, g = blockIdx.z;
  const float* p = part + ((int64_t)bh * nchunk + g) * stride + e;
  const int64_t step = (int64_t)S * stride;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int c = g;
  for (; c + 3 * S < nchunk; c += 4 * S, p += 4 * step) {
    s0 += p[0]; s1 += p[step]; s2 += p[2 * step]; s3 += p[3 * step];
  }
  for (; c < nchunk; c += S, p += step) s0 += p[0];
  red[((int64_t)bh * S + g) * stride + e] = (s0 + s1) + (s2 + s3);
}

// one wave per query row i of (b, h): logits over all key columns (sum of the S partials),
// softmax, and 1/|k_cur| for the FHR cache (turtle_t1_arch.py:357-366, 598-600)
constexpr int SM_MAXC = 512 / 64;
__global__ __launch_bounds__(256) void attn_softmax_kernel(AttnFinArgs a) {
  const int ch = a.ch, ncol = a.nseg * ch, stride = ch * ncol + ch + ncol, S = a.nsplit;
  const int bh = blockIdx.x, b = bh / a.heads, h = bh % a.heads;
  const float* R = a.red + (int64_t)bh * S * stride;
  auto sum_s = [&](int e) {
    float v = 0.f;
    for (int g = 0; g < S; ++g) v += R[(int64_t)g * stride + e];
    return v;
  };
  __shared__ float kinv_s[512];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int j = tid; j < ncol; j += 256) {
    const int s = j / ch;
    kinv_s[j] = ((a.norm_mask >> s) & 1) ? 1.f / fmaxf(sqrtf(sum_s(ch * ncol + ch + j)), 1e-12f) : 1.f;
  }
  __syncthreads();
  if (blockIdx.y == 0 && a.kinv && a.cur_seg >= 0)
    for (int j = tid; j < ch; j += 256) a.kinv[(int64_t)b * a.heads * ch + h * ch + j] = kinv_s[a.cur_seg * ch + j];
  const int i = blockIdx.y * 4 + wid;
  if (i >= ch) return;
  const float qi = a.tau[h] / fmaxf(sqrtf(sum_s(ch * ncol + i)), 1e-12f);
  float lg[SM_MAXC];
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < SM_MAXC; ++k) {
    const int j = lane + 64 * k;
    lg[k] = j < ncol ? sum_s(i * ncol + j) * qi * kinv_s[j] : -INFINITY;
    mx = fmaxf(mx, lg[k]);
  }
  mx = wave_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < SM_MAXC; ++k) {
    lg[k] = lane + 64 * k < ncol ? expf(lg[k] - mx) : 0.f;
    sum += lg[k];
  }
  const float inv = 1.f / wave_sum(sum);
  float* A = a.attn + ((int64_t)bh * ch + i) * ncol;
#pragma unroll
  for (int k = 0; k < SM_MAXC; ++k)
    if (lane + 64 * k < ncol) A[lane + 64 * k] = lg[k] * inv;
}

int attn_nsplit(int nchunk) { return nchunk < 32 ? nchunk : 32; }

void launch_attn_finalize(const AttnFinArgs& a, hipStream_t st) {
  const int ncol = a.nseg * a.ch, stride = a.ch * ncol + a.ch + ncol, nbh = a.B * a.heads;
  hipLaunchKernelGGL(gram_reduce_kernel, dim3((unsigned)((stride + 255) / 256), (unsigned)nbh, (unsigned)a.nsplit),
                     dim3(256), 0, st, a.part, a.red, a.nchunk, stride, a.nsplit);
  hipLaunchKernelGGL(attn_softmax_kernel, dim3((unsigned)nbh, (unsigned)((a.ch + 3) / 4)), dim3(256), 0, st, a);
}

// W_eff[b][o][seg_col[s] + h*seg_hstride[s] + j] = sum_i Wp[o][h*ch + i] * A[b,h][i][s*ch + j]
// block = (4 output channels, b*h); threads stride the key columns, so A rows load coalesced and
// the Wp operands are wave-uniform (scalar loads)
constexpr int WE_OT = 4;
template <typename T>
__global__ __launch_bounds__(256) void weff_kernel(WeffArgs a) {
  const int ch = a.ch, ncol = a.nseg * ch;
  const int o0 = blockIdx.x * WE_OT, bh = blockIdx.y, b = bh / a.heads, h = bh % a.heads;
  T* W = reinterpret_cast<T*>(a.weff);
  const float* A = a.attn + (int64_t)bh * ch * ncol;
  for (int col = threadIdx.x; col < ncol; col += 256) {
    float acc[WE_OT];
#pragma unroll
    for (int t = 0; t < WE_OT; ++t) acc[t] = 0.f;
    for (int i = 0; i < ch; ++i) {
      const float av = A[(int64_t)i * ncol + col];
#pragma unroll
      for (int t = 0; t < WE_OT; ++t)
        if (o0 + t < a.C) acc[t] = fmaf(a.wp[(int64_t)(o0 + t) * a.C + h * ch + i], av, acc[t]);
    }
    const int sg = col / ch, jj = col - sg * ch;
    int64_t scol = a.seg_col[0];
    int shs = a.seg_hstride[0];
#pragma unroll
    for (int q = 1; q < TURTLE_MAX_SEG; ++q)
      if (sg == q) { scol = a.seg_col[q]; shs = a.seg_hstride[q]; }
#pragma unroll
    for (int t = 0; t < WE_OT; ++t)
      if (o0 + t < a.C) W[((int64_t)b * a.C + o0 + t) * a.Keff + scol + (int64_t)h * shs + jj] = from_f<T>(acc[t]);
  }
}

template <typename T>
void launch_weff(const WeffArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(weff_kernel<T>, dim3((unsigned)((a.C + WE_OT - 1) / WE_OT), (unsigned)(a.B * a.heads)), dim3(256), 0, st, a);
}

template void launch_gram<float>(const GramArgs&, hipStream_t);
template void launch_gram<bf16>(const GramArgs&, hipStream_t);
template void launch_weff<float>(const WeffArgs&, hipStream_t);
template void launch_weff<bf16>(const WeffArgs&, hipStream_t);

}  // namespace turtle

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
__global__ __launch_bounds__(256) void gram_kernel(GramArgs a) {
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

// Channel-attention Gram with the q / k depthwise 3x3 in its prologue (level-3 ChannelAttention,
// turtle_t1_arch.py:674-697): G = dw(q)^T dw(k) over HW per (batch, head) and the per-channel
// sums of squares, from the raw qkv map. The depthwise is dw_rows' row walk (spatial.hip): a block
// owns a (32-column strip) x (band of RB rows) box of one (image, head), thread = (column, 8-channel
// vector of q or k): 32 x 16 = 512 threads; walking down the band each thread keeps its column's
// 3 x 3 raw neighbourhood as a rolling window of three rows and loads one row ahead. Every 4 rows
// (128 pixels) the block's dw outputs - rounded to bf16 as the stored map was - sit in an LDS
// operand tile [pixel][q 64 | k 64] and the 8 waves fold them into the 64 x 64 Gram with the
// transposed-read MFMAs of gram_kernel (two LDS tiles: one barrier per 4 rows). Against dw_rows +
// gram_kernel: the 2 x 64-channel dw'd q / k map is neither written nor read back.
constexpr int GD_SX = 32, GD_NV = 16, GD_NT = GD_SX * GD_NV, GD_CH = 64, GD_RQ = GD_CH * 2 + 16;
constexpr int GD_TILE = 4 * GD_SX * GD_RQ;      // one operand ([128 px][64 ch] + pad) of 4 rows
__global__ __launch_bounds__(GD_NT) void gram_dw_kernel(GramDwArgs a) {
  __shared__ __attribute__((aligned(16))) char sop[2][2][GD_TILE];   // [buffer][q | k]
  __shared__ __attribute__((aligned(16))) float sw[9][2 * GD_CH];
  __shared__ __attribute__((aligned(16))) float sb[2 * GD_CH];
  __shared__ float snrm[GD_NT / 64][2 * GD_CH];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nchunk = a.nstrip * a.nband;
  const int bh = blockIdx.x / nchunk, chunk = blockIdx.x % nchunk;
  const int b = bh / a.heads, h = bh % a.heads;
  const int strip = chunk % a.nstrip, band = chunk / a.nstrip;
  const int C = a.Cw / 2;
  // thread -> (column, vector): vec < 8 are q channels h*64 + 8 vec, vec >= 8 the k channels
  const int col = tid / GD_NV, vec = tid % GD_NV, isk = vec >> 3, c8 = (vec & 7) * 8;
  for (int e = tid; e < 9 * 2 * GD_CH; e += GD_NT) {
    const int tap = e / (2 * GD_CH), j = e - tap * 2 * GD_CH, kk = j / GD_CH, i = j - kk * GD_CH;
    sw[tap][j] = a.w[tap * a.Cw + kk * C + h * GD_CH + i];
  }
  for (int j = tid; j < 2 * GD_CH; j += GD_NT) {
    const int kk = j / GD_CH, i = j - kk * GD_CH;
    sb[j] = a.bias ? a.bias[kk * C + h * GD_CH + i] : 0.f;
  }
  const int x = strip * GD_SX + col;
  const bool xin = x < a.W;
  const int xc = min(x, a.W - 1);
  const bool okl = xc > 0, okr = xc + 1 < a.W;
  const int y0 = band * a.RB, y1 = min(a.H, y0 + a.RB);
  const bf16* src = reinterpret_cast<const bf16*>(a.in) + (int64_t)b * a.H * a.W * a.ld + (isk ? a.koff : a.qoff) + h * GD_CH + c8;
  auto load_row = [&](int y, uint4 (&r)[3]) {
    const bool oky = y >= 0 && y < a.H;
    const bf16* p = src + ((int64_t)(oky ? y : 0) * a.W + xc) * a.ld;
    r[0] = ld16(oky && okl ? reinterpret_cast<const void*>(p - a.ld) : g_zero_gram);
    r[1] = ld16(oky ? reinterpret_cast<const void*>(p) : g_zero_gram);
    r[2] = ld16(oky && okr ? reinterpret_cast<const void*>(p + a.ld) : g_zero_gram);
  };
  uint4 w0[3], w1[3], w2[3], nx[3];
  load_row(y0 - 1, w0);
  load_row(y0, w1);
  load_row(y0 + 1, w2);
  // MFMA tiles of this wave: t = wid + 8 u over the 4 x 4 16 x 16 tiles of the 64 x 64 Gram
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  float sq[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) sq[e] = 0.f;
  const int g16 = lane >> 4, li = lane & 15, qq = li >> 2, pp = li & 3;
  typedef short v4s __attribute__((ext_vector_type(4)));
  typedef short v8s __attribute__((ext_vector_type(8)));
  typedef __attribute__((address_space(3))) v4s lds_v4s;
  __syncthreads();                                  // tap / bias tables staged
  const int jw = isk * GD_CH + c8;
  int grp = 0;
  for (int yg = y0; yg < y1; yg += 4, grp ^= 1) {
    char* tq = sop[grp][0];
    char* tk = sop[grp][1];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int y = yg + r;
      const bool live = y < y1 && xin;
      if (y + 1 < y1) load_row(y + 2, nx);
      int jr = jw;
      asm volatile("" : "+v"(jr));                  // taps re-read from LDS per row (registers)
      float acc8[8];
      {
        const float4 b0 = *reinterpret_cast<const float4*>(&sb[jr]), b1 = *reinterpret_cast<const float4*>(&sb[jr + 4]);
        acc8[0] = b0.x; acc8[1] = b0.y; acc8[2] = b0.z; acc8[3] = b0.w; acc8[4] = b1.x; acc8[5] = b1.y; acc8[6] = b1.z; acc8[7] = b1.w;
      }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const uint4 q = tap < 3 ? w0[tap] : tap < 6 ? w1[tap - 3] : w2[tap - 6];
        const uint32_t u[4] = {q.x, q.y, q.z, q.w};
        const float4 t0 = *reinterpret_cast<const float4*>(&sw[tap][jr]), t1 = *reinterpret_cast<const float4*>(&sw[tap][jr + 4]);
        const float wt[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const f32x2 r2 = __builtin_elementwise_fma(f32x2{wt[2 * i], wt[2 * i + 1]},
                                                     f32x2{__uint_as_float(u[i] << 16), __uint_as_float(u[i] & 0xffff0000u)},
                                                     f32x2{acc8[2 * i], acc8[2 * i + 1]});
          acc8[2 * i] = r2.x; acc8[2 * i + 1] = r2.y;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(acc8[i]));
      }
      // bf16 operand (the value the stored map held), 0 for rows / columns outside the box
      uint32_t o[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16 lo = (bf16)(live ? acc8[2 * i] : 0.f), hi = (bf16)(live ? acc8[2 * i + 1] : 0.f);
        o[i] = (uint32_t)__builtin_bit_cast(unsigned short, lo) | ((uint32_t)__builtin_bit_cast(unsigned short, hi) << 16);
        const float fl = __uint_as_float(o[i] << 16), fh = __uint_as_float(o[i] & 0xffff0000u);
        sq[2 * i] = fmaf(fl, fl, sq[2 * i]);
        sq[2 * i + 1] = fmaf(fh, fh, sq[2 * i + 1]);
      }
      *reinterpret_cast<uint4*>((isk ? tk : tq) + (r * GD_SX + col) * GD_RQ + c8 * 2) = make_uint4(o[0], o[1], o[2], o[3]);
#pragma unroll
      for (int k = 0; k < 3; ++k) { w0[k] = w1[k]; w1[k] = w2[k]; w2[k] = nx[k]; }
    }
    __syncthreads();                                // this group's operand tile is complete
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int tile = wid + 8 * u, it = tile >> 2, jt = tile & 3;
#pragma unroll
      for (int ss = 0; ss < 4; ++ss) {
        const char* qa = tq + (32 * ss + 8 * g16 + qq) * GD_RQ + (it * 16 + 4 * pp) * 2;
        const char* ka = tk + (32 * ss + 8 * g16 + qq) * GD_RQ + (jt * 16 + 4 * pp) * 2;
        const v4s a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)qa);
        const v4s a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(qa + 4 * GD_RQ));
        const v4s b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)ka);
        const v4s b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(ka + 4 * GD_RQ));
        const bf16x8 af = __builtin_bit_cast(bf16x8, (v8s)__builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7));
        const bf16x8 bfr = __builtin_bit_cast(bf16x8, (v8s)__builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7));
        acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc[u], 0, 0, 0);
      }
    }
  }
  // per-channel sums of squares: the 4 columns of a wave (lane bits 4, 5), then the 8 waves in
  // a fixed order (deterministic)
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sq[e] += __shfl_xor(sq[e], 16, 64);
    sq[e] += __shfl_xor(sq[e], 32, 64);
  }
  if (lane < GD_NV) {
#pragma unroll
    for (int e = 0; e < 8; ++e) snrm[wid][isk * GD_CH + c8 + e] = sq[e];
  }
  __syncthreads();
  const int stride = GD_CH * GD_CH + 2 * GD_CH;
  float* out = a.part + ((int64_t)bh * nchunk + chunk) * stride;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int tile = wid + 8 * u, it = tile >> 2, jt = tile & 3;
#pragma unroll
    for (int r = 0; r < 4; ++r) out[(it * 16 + (lane >> 4) * 4 + r) * GD_CH + jt * 16 + (lane & 15)] = acc[u][r];
  }
  for (int j = tid; j < 2 * GD_CH; j += GD_NT) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < GD_NT / 64; ++w) s += snrm[w][j];
    out[GD_CH * GD_CH + j] = s;                      // [nq (64) | nk (64)]
  }
}

bool gram_dw_ok(const GramDwArgs& a) {
  if (a.ch != GD_CH || a.Cw != 2 * a.heads * GD_CH || !a.w || !a.in || !a.part) return false;
  if (a.ld % 8 || a.qoff % 8 || a.koff % 8 || (reinterpret_cast<uintptr_t>(a.in) & 15)) return false;
  if (a.RB <= 0 || a.RB % 4 || a.nstrip != (a.W + GD_SX - 1) / GD_SX || a.nband != (a.H + a.RB - 1) / a.RB) return false;
  return (int64_t)a.B * a.heads * a.nstrip * a.nband < ((int64_t)1 << 31);
}

void gram_dw_geometry(GramDwArgs& a) {
  a.nstrip = (a.W + GD_SX - 1) / GD_SX;
  // bands of 32 rows while the grid keeps >= ~2 blocks per CU, else shorter (multiples of 4)
  a.RB = 32;
  while (a.RB > 4 && (int64_t)a.B * a.heads * a.nstrip * ((a.H + a.RB - 1) / a.RB) < 512) a.RB /= 2;
  a.nband = (a.H + a.RB - 1) / a.RB;
}

void launch_gram_dw(const GramDwArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(gram_dw_kernel, dim3((unsigned)((int64_t)a.B * a.heads * a.nstrip * a.nband)), dim3(GD_NT), 0, st, a);
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
  hipLaunchKernelGGL(attn_row_kernel, dim3((unsigned)((a.ch + 3) / 4), (unsigned)nbh), dim3(256), 0, st, a);
}

// Fold the attention into the projection, one block per (32 output channels, 64 key columns,
// b*h): W_eff[b][o][col(j)] = sum_i Wp[o][h*ch + i] * A[i][j] (A and Wp slabs staged in LDS by
// coalesced loads), so project_out(A v) becomes one GEMM over the K-concatenated value sources.
constexpr int WF_MAXCH = 128;
template <typename T>
__global__ __launch_bounds__(256) void attn_weff_kernel(WeffArgs a) {
  __shared__ __attribute__((aligned(16))) float sA[WF_MAXCH][64];
  __shared__ __attribute__((aligned(16))) float sW[WF_MAXCH][32];    // [i][o]
  const int ch = a.ch, ncol = a.nseg * ch;
  const int o0 = blockIdx.x * 32, j0 = blockIdx.y * 64, bh = blockIdx.z;
  const int b = bh / a.heads, h = bh % a.heads;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const float* A = a.attn + (int64_t)bh * ch * ncol;
  for (int e = tid; e < ch * 64; e += 256) {
    const int i = e >> 6, jj = e & 63;
    sA[i][jj] = j0 + jj < ncol ? A[i * ncol + j0 + jj] : 0.f;
  }
  for (int e = tid; e < 32 * ch; e += 256) {
    const int oo = e / ch, i = e - oo * ch;
    sW[i][oo] = o0 + oo < a.C ? a.wp[(int64_t)(o0 + oo) * a.C + h * ch + i] : 0.f;
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
  hipLaunchKernelGGL(attn_weff_kernel<T>, dim3((unsigned)((a.C + 31) / 32), (unsigned)((ncol + 63) / 64), (unsigned)(a.B * a.heads)),
                     dim3(256), 0, st, a);
}

// attn_row + attn_weff in one launch: each W_eff block computes the softmax of every attention
// row over all ncol columns from the reduced Gram (rows are <= 512 wide, ch <= 128) and keeps only
// its 64 columns, staged straight into LDS for the projection fold. Same arithmetic order as
// attn_row_kernel. Saves a launch and the A round trip through HBM per channel-attention block.
template <typename T>
__global__ __launch_bounds__(256) void attn_weff_fused_kernel(AttnFinArgs f, WeffArgs a) {
  __shared__ __attribute__((aligned(16))) float sA[WF_MAXCH][64];
  __shared__ __attribute__((aligned(16))) float sW[WF_MAXCH][32];    // [i][o]
  const int ch = a.ch, ncol = a.nseg * ch, stride = ch * ncol + ch + ncol;
  const int o0 = blockIdx.x * 32, j0 = blockIdx.y * 64, bh = blockIdx.z;
  const int b = bh / a.heads, h = bh % a.heads;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int e = tid; e < 32 * ch; e += 256) {
    const int oo = e / ch, i = e - oo * ch;
    sW[i][oo] = o0 + oo < a.C ? a.wp[(int64_t)(o0 + oo) * a.C + h * ch + i] : 0.f;
  }
  const float* R = f.red + (int64_t)bh * stride;
  // key-column scales kv (1/|k_j| on L2-normalised segments) of this lane's columns
  float kv[AR_KC];
#pragma unroll
  for (int k = 0; k < AR_KC; ++k) {
    const int jc = min(lane + 64 * k, ncol - 1);
    kv[k] = ((f.norm_mask >> (jc / ch)) & 1) ? 1.f / fmaxf(sqrtf(R[ch * ncol + ch + jc]), 1e-12f) : 1.f;
  }
  const int jb = j0 / 64;                       // this block's columns are k = jb of every lane
  const int kc = (ncol + 63) / 64;              // column vectors in use (uniform)
  // 4 rows per wave per pass with all their loads in flight (the row loop is latency-bound)
  constexpr int RG = 4;
  for (int i0 = wid * RG; i0 < ch; i0 += 4 * RG) {
    float lg[RG][AR_KC], qn[RG];
#pragma unroll
    for (int u = 0; u < RG; ++u) {
      const int i = min(i0 + u, ch - 1);
      qn[u] = R[ch * ncol + i];
#pragma unroll
      for (int k = 0; k < AR_KC; ++k)
        lg[u][k] = k < kc ? R[i * ncol + min(lane + 64 * k, ncol - 1)] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < RG; ++u) {
      const float q = f.tau[h] / fmaxf(sqrtf(qn[u]), 1e-12f);
      float mx = -INFINITY;
#pragma unroll
      for (int k = 0; k < AR_KC; ++k) {
        lg[u][k] = lane + 64 * k < ncol ? lg[u][k] * q * kv[k] : -INFINITY;
        mx = fmaxf(mx, lg[u][k]);
      }
      mx = wave_max(mx);
      float sum = 0.f, mine = 0.f;
#pragma unroll
      for (int k = 0; k < AR_KC; ++k) {
        lg[u][k] = lane + 64 * k < ncol ? expf(lg[u][k] - mx) : 0.f;
        sum += lg[u][k];
        mine = k == jb ? lg[u][k] : mine;
      }
      const float inv = 1.f / wave_sum(sum);
      if (i0 + u < ch) sA[i0 + u][lane] = mine * inv;     // 0 past ncol
    }
  }
  if (blockIdx.x == 0 && wid == 0 && f.kinv && f.cur_seg >= 0) {
    float mk = 0.f;
#pragma unroll
    for (int k = 0; k < AR_KC; ++k) mk = k == jb ? kv[k] : mk;
    const int j = j0 + lane;
    if (j >= f.cur_seg * ch && j < (f.cur_seg + 1) * ch) f.kinv[(int64_t)b * a.heads * ch + h * ch + (j - f.cur_seg * ch)] = mk;
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
void launch_attn_weff(const AttnFinArgs& f, const WeffArgs& a, hipStream_t st) {
  const int ncol = f.nseg * f.ch, stride = f.ch * ncol + f.ch + ncol, nbh = f.B * f.heads;
  hipLaunchKernelGGL(gram_sum_kernel, dim3((unsigned)((stride + 63) / 64), (unsigned)nbh), dim3(256), 0, st, f.part, f.red,
                     f.nchunk, stride);
  hipLaunchKernelGGL(attn_weff_fused_kernel<T>, dim3((unsigned)((a.C + 31) / 32), (unsigned)((ncol + 63) / 64), (unsigned)nbh),
                     dim3(256), 0, st, f, a);
}

template void launch_attn_weff<float>(const AttnFinArgs&, const WeffArgs&, hipStream_t);
template void launch_attn_weff<bf16>(const AttnFinArgs&, const WeffArgs&, hipStream_t);
template void launch_gram<float>(const GramArgs&, hipStream_t);
template void launch_gram<bf16>(const GramArgs&, hipStream_t);
template void launch_weff<float>(const WeffArgs&, hipStream_t);
template void launch_weff<bf16>(const WeffArgs&, hipStream_t);

}  // namespace turtle

// Spatial (non-GEMM) kernels on pixel-major maps:
//   * depthwise 3x3 (+bias, +GELU, or the GatedFeedForward gate gelu(x1)*x2) with an optional
//     SAB dilated token-major output layout             turtle_t1_arch.py:159-178, 716-740, 555-574
//   * SAB window conv ws x ws / stride ws / pad 1 on q2/k2 + L2 normalisation over d   559-578
//   * input_projection 3x3 from the caller's NCHW frames (zero pad to 32, or SR 4x bilinear)
//     1063, turtlesuper 976-977
//   * ending 3x3 + bias + current frame, crop, NCHW fp32 output                          1128-1132
//   * latent FrameHistoryRouter cache roll (keep the last Rnew rows of [cached ; current])   272-286
#include "common.h"
#include "kernels.h"

namespace turtle {

// ------------------------------------------------------------------------------------------
// depthwise 3x3: one thread = one pixel x VEC channels
// ------------------------------------------------------------------------------------------
template <typename T>
TURTLE_DEV void unpack16(const uint4& q, float (&v)[Vec<T>::N]);
template <>
TURTLE_DEV void unpack16<bf16>(const uint4& q, float (&v)[8]) {
  const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) { v[2 * i] = __uint_as_float(w[i] << 16); v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u); }
}
template <>
TURTLE_DEV void unpack16<float>(const uint4& q, float (&v)[4]) {
  v[0] = __uint_as_float(q.x); v[1] = __uint_as_float(q.y); v[2] = __uint_as_float(q.z); v[3] = __uint_as_float(q.w);
}

__device__ __attribute__((aligned(64))) uint4 g_zero_dw[4];

// raw channel vector of VW elements for the row-sweep depthwise: 16 bytes (bf16 x 8, fp32 x 4), or
// 8 bytes (bf16 x 4: the gate's two halves in the register footprint of one plain vector)
template <typename T, int VW> struct DwRaw;
template <> struct DwRaw<bf16, 8> {
  typedef uint4 raw;
  static TURTLE_DEV raw load(const void* p) { return ld16(p); }
  static TURTLE_DEV void unpack(const raw& q, float (&v)[8]) { unpack16<bf16>(q, v); }
  static TURTLE_DEV void store(bf16* p, const float (&v)[8]) {
    Vec<bf16> o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o.v[i] = v[i];
    o.store(p);
  }
};
template <> struct DwRaw<bf16, 4> {
  typedef uint2 raw;
  static TURTLE_DEV raw load(const void* p) { return ld8(p); }
  static TURTLE_DEV void unpack(const raw& q, float (&v)[4]) {
    v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
    v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
  }
  static TURTLE_DEV void store(bf16* p, const float (&v)[4]) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    *reinterpret_cast<bf16x4*>(p) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
  }
};
template <> struct DwRaw<float, 4> {
  typedef uint4 raw;
  static TURTLE_DEV raw load(const void* p) { return ld16(p); }
  static TURTLE_DEV void unpack(const raw& q, float (&v)[4]) { unpack16<float>(q, v); }
  static TURTLE_DEV void store(float* p, const float (&v)[4]) { *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]); }
};

// Row-sweeping depthwise 3x3. A block owns a (32-column strip) x (DW_CC channel vectors) x (band of
// RB rows) box of one image; thread = (column, channel vector). Walking down the band, each thread
// keeps the 3x3 neighbourhood of its column as a rolling window of three rows in registers and
// loads only the next row (3 vectors, the two side ones L1 hits of its neighbours' loads), one row
// ahead of the math. Every input byte therefore leaves HBM about once (band halo 2/RB) instead of
// the 3 row re-reads of a per-pixel gather. Tap weights of the block's channels sit in LDS (fp32).
// VW = channels per lane: a 16-byte vector, or 4 for the bf16 gate (x1 and x2 vectors of 8 bytes:
// 71 VGPRs, 7 waves per SIMD instead of 129 / 3; slower, kept for tools/dwbench).
constexpr int DW_CC = 8;                                  // channel vectors per block
constexpr int DW_SX = 256 / DW_CC;                        // columns per block
template <typename T, int MODE, int VW>
__global__ __launch_bounds__(256) void dw_rows_kernel(DwArgs a, int RB, int nstrip, int nchunk, int nband) {
  using RW = DwRaw<T, VW>;
  typedef typename RW::raw raw;
  constexpr int NH = MODE == DW_GATE ? 2 : 1;             // gate: x1 and x2 halves
  constexpr int CW = DW_CC * VW;                          // channels per block
  __shared__ __attribute__((aligned(16))) float sw[NH][9][CW];
  __shared__ __attribute__((aligned(16))) float sbias[NH][CW];
  const int tid = threadIdx.x;
  const int CV = a.C / VW;
  const int Cw = NH * a.C;
  int lin = blockIdx.x;
  {
    const int nblk = gridDim.x, q = nblk / 8, r = nblk % 8, x = lin % 8, y = lin / 8;
    lin = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;   // vertical neighbours share an XCD
  }
  const int band = lin % nband;
  int t = lin / nband;
  const int strip = t % nstrip;
  t /= nstrip;
  const int chunk = t % nchunk;
  const int64_t img = t / nchunk;

  // tap weights of this chunk -> LDS (zero past C)
  for (int e = tid; e < NH * 9 * CW; e += 256) {
    const int hh = e / (9 * CW), r = e - hh * 9 * CW, tap = r / CW, c = r - tap * CW;
    const int cg = chunk * CW + c;
    sw[hh][tap][c] = cg < a.C ? a.w[tap * Cw + hh * a.C + cg] : 0.f;
  }
  // bias in LDS too (read per row: registers are the occupancy limit of the gate variant)
  for (int e = tid; e < NH * CW; e += 256) {
    const int hh = e / CW, c = e - hh * CW, cg = chunk * CW + c;
    sbias[hh][c] = a.bias && cg < a.C ? a.bias[hh * a.C + cg] : 0.f;
  }
  const int cvl = tid % DW_CC, xs = tid / DW_CC;
  const int x = strip * DW_SX + xs, cv = chunk * DW_CC + cvl;
  const bool live = x < a.W && cv < CV;
  const int xc = min(x, a.W - 1), c0 = min(cv, CV - 1) * VW;
  const int y0 = band * RB, y1 = min(a.H, y0 + RB);
  const T* in = reinterpret_cast<const T*>(a.in) + img * a.H * a.W * a.ldi + a.offi + c0;
  const bool okl = xc > 0, okr = xc + 1 < a.W;
  // one row of the window: columns x-1, x, x+1 (zero line outside the image)
  auto load_row = [&](int y, raw (&r)[NH][3]) {
    const bool oky = y >= 0 && y < a.H;
    const T* p = in + ((int64_t)(oky ? y : 0) * a.W + xc) * a.ldi;
#pragma unroll
    for (int hh = 0; hh < NH; ++hh) {
      const T* q = p + hh * a.C;
      r[hh][0] = RW::load(oky && okl ? reinterpret_cast<const void*>(q - a.ldi) : g_zero_dw);
      r[hh][1] = RW::load(oky ? reinterpret_cast<const void*>(q) : g_zero_dw);
      r[hh][2] = RW::load(oky && okr ? reinterpret_cast<const void*>(q + a.ldi) : g_zero_dw);
    }
  };
  raw w0[NH][3], w1[NH][3], w2[NH][3], nx[NH][3];
  load_row(y0 - 1, w0);
  load_row(y0, w1);
  load_row(y0 + 1, w2);
  __syncthreads();
  const int wc = cvl * VW;
  for (int y = y0; y < y1; ++y) {
    if (y + 1 < y1) load_row(y + 2, nx);                  // next row in flight during the math
    // re-read the tap weights from LDS every row (opaque offset): hoisted, they would hold
    // 72-144 VGPRs for the whole sweep
    int wcy = wc;
    asm volatile("" : "+v"(wcy));
    float acc[NH][VW];
#pragma unroll
    for (int hh = 0; hh < NH; ++hh) {
#pragma unroll
      for (int i0 = 0; i0 < VW; i0 += 4) {
        const float4 bb = *reinterpret_cast<const float4*>(&sbias[hh][wcy + i0]);
        acc[hh][i0] = bb.x; acc[hh][i0 + 1] = bb.y; acc[hh][i0 + 2] = bb.z; acc[hh][i0 + 3] = bb.w;
      }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const raw q = tap < 3 ? w0[hh][tap] : tap < 6 ? w1[hh][tap - 3] : w2[hh][tap - 6];
        float v[VW];
        RW::unpack(q, v);
        const float* wt = &sw[hh][tap][wcy];
#pragma unroll
        for (int i0 = 0; i0 < VW; i0 += 4) {   // packed f32 pairs (v_pk_fma_f32)
          const float4 ww = *reinterpret_cast<const float4*>(wt + i0);
          const f32x2 a0 = __builtin_elementwise_fma(f32x2{ww.x, ww.y}, f32x2{v[i0], v[i0 + 1]}, f32x2{acc[hh][i0], acc[hh][i0 + 1]});
          const f32x2 a1 = __builtin_elementwise_fma(f32x2{ww.z, ww.w}, f32x2{v[i0 + 2], v[i0 + 3]}, f32x2{acc[hh][i0 + 2], acc[hh][i0 + 3]});
          acc[hh][i0] = a0.x; acc[hh][i0 + 1] = a0.y; acc[hh][i0 + 2] = a1.x; acc[hh][i0 + 3] = a1.y;
        }
        // one tap's weights / unpacked values live at a time (the scheduler would otherwise
        // hoist all 9 taps' LDS reads and unpacks: 200+ VGPRs, one wave per SIMD)
#pragma unroll
        for (int i = 0; i < VW; ++i) asm volatile("" : "+v"(acc[hh][i]));
      }
    }
    if (live) {
      float o[VW];
      if constexpr (sizeof(T) == 2 && MODE != DW_PLAIN) {   // bf16 GELU / gate as packed pairs
#pragma unroll
        for (int i = 0; i < VW; i += 2) {
          f32x2 r = gelu_bf16_2(f32x2{acc[0][i], acc[0][i + 1]});
          if (MODE == DW_GATE) r = r * f32x2{acc[NH - 1][i], acc[NH - 1][i + 1]};
          o[i] = r.x; o[i + 1] = r.y;
        }
      } else {
#pragma unroll
        for (int i = 0; i < VW; ++i) {
          float r = acc[0][i];
          if (MODE == DW_GELU) r = gelu_t<T>(r);
          else if (MODE == DW_GATE) r = gelu_t<T>(r) * acc[NH - 1][i];
          o[i] = r;
        }
      }
      const int64_t pix = (img * a.H + y) * a.W + x;
      int64_t dst;
      if (a.tok_ws > 0) {
        const int ws = a.tok_ws, h = a.H / ws, w = a.W / ws;
        const int p1 = y / h, i = y - p1 * h, p2 = x / w, j = x - p2 * w;
        dst = img * a.tok_img_stride + ((int64_t)i * w + j) * ((int64_t)ws * ws * a.C) + (int64_t)(p1 * ws + p2) * a.C + c0;
      } else {
        dst = pix * a.ldo + a.offo + c0;
      }
      RW::store(reinterpret_cast<T*>(a.out) + dst, o);
    }
#pragma unroll
    for (int hh = 0; hh < NH; ++hh)
#pragma unroll
      for (int k = 0; k < 3; ++k) { w0[hh][k] = w1[hh][k]; w1[hh][k] = w2[hh][k]; w2[hh][k] = nx[hh][k]; }
  }
}

// one thread = one pixel x VEC channels; the 9 (18 for the gate) neighbour vectors are loaded
// unconditionally (out-of-image taps read a zero line), so all of them are in flight together.
// Block ids are remapped so each XCD sweeps a contiguous band of rows (vertical reuse in its L2).
// Kept as the reference variant behind turtle_set_option("dw_rows", 0).
template <typename T, int MODE>
__global__ __launch_bounds__(256) void dw_kernel(DwArgs a) {
  constexpr int VEC = Vec<T>::N;
  const int CV = a.C / VEC;
  const int64_t total = (int64_t)a.nimg * a.H * a.W * CV;
  const int Cw = MODE == DW_GATE ? 2 * a.C : a.C;
  const T* in = reinterpret_cast<const T*>(a.in);
  int lin = blockIdx.x;
  {
    const int nblk = gridDim.x, q = nblk / 8, r = nblk % 8, x = lin % 8, y = lin / 8;
    lin = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;
  }
  const int64_t idx = (int64_t)lin * 256 + threadIdx.x;
  if (idx >= total) return;
  const int cv = (int)(idx % CV);
  const int64_t pix = idx / CV;
  const int x = (int)(pix % a.W);
  const int64_t t = pix / a.W;
  const int y = (int)(t % a.H);
  const int64_t img = t / a.H;
  const int c0 = cv * VEC;
  uint4 q1[9], q2[9];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
    const bool ok = yy >= 0 && yy < a.H && xx >= 0 && xx < a.W;
    const T* p = in + ((img * a.H + yy) * a.W + xx) * a.ldi + a.offi + c0;
    q1[tap] = ld16(ok ? reinterpret_cast<const void*>(p) : g_zero_dw);
    if constexpr (MODE == DW_GATE) q2[tap] = ld16(ok ? reinterpret_cast<const void*>(p + a.C) : g_zero_dw);
  }
  // bias: unconditional vector loads (a per-element "bias ? load : 0" would serialise them)
  float acc1[VEC], acc2[VEC];
  {
    const float* zb = reinterpret_cast<const float*>(g_zero_dw);
    const float* b1 = a.bias ? a.bias + c0 : zb;
    const float* b2 = (MODE == DW_GATE && a.bias) ? a.bias + a.C + c0 : zb;
#pragma unroll
    for (int i0 = 0; i0 < VEC; i0 += 4) {
      const uint4 u1 = ld16(b1 + i0), u2 = ld16(b2 + i0);
      acc1[i0] = __uint_as_float(u1.x); acc1[i0 + 1] = __uint_as_float(u1.y);
      acc1[i0 + 2] = __uint_as_float(u1.z); acc1[i0 + 3] = __uint_as_float(u1.w);
      acc2[i0] = __uint_as_float(u2.x); acc2[i0 + 1] = __uint_as_float(u2.y);
      acc2[i0 + 2] = __uint_as_float(u2.z); acc2[i0 + 3] = __uint_as_float(u2.w);
    }
  }
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const float* wt = a.w + tap * Cw + c0;
    float v[VEC];
    unpack16<T>(q1[tap], v);
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc1[i] = fmaf(wt[i], v[i], acc1[i]);
    if constexpr (MODE == DW_GATE) {
      unpack16<T>(q2[tap], v);
#pragma unroll
      for (int i = 0; i < VEC; ++i) acc2[i] = fmaf(wt[a.C + i], v[i], acc2[i]);
    }
  }
  Vec<T> o;
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    float r = acc1[i];
    if (MODE == DW_GELU) r = gelu_t<T>(r);
    else if (MODE == DW_GATE) r = gelu_t<T>(r) * acc2[i];
    o.v[i] = r;
  }
  int64_t dst;
  if (a.tok_ws > 0) {
    const int ws = a.tok_ws, h = a.H / ws, w = a.W / ws;
    const int p1 = y / h, i = y - p1 * h, p2 = x / w, j = x - p2 * w;
    dst = img * a.tok_img_stride + ((int64_t)i * w + j) * ((int64_t)ws * ws * a.C) + (int64_t)(p1 * ws + p2) * a.C + c0;
  } else {
    dst = pix * a.ldo + a.offo + c0;
  }
  o.store(reinterpret_cast<T*>(a.out) + dst);
}

template <typename T, int MODE, int VW>
static void launch_dw_rows(const DwArgs& a, hipStream_t st) {
  const int CV = a.C / VW;
  const int nstrip = (a.W + DW_SX - 1) / DW_SX, nchunk = (CV + DW_CC - 1) / DW_CC;
  // band height: tall bands (halo 2/RB) while the grid still has >= ~8 blocks per CU
  int RB = 32;
  auto nblk = [&](int rb) { return (int64_t)a.nimg * nchunk * nstrip * ((a.H + rb - 1) / rb); };
  while (RB > 4 && nblk(RB) < 2048) RB /= 2;
  const int nband = (a.H + RB - 1) / RB;
  hipLaunchKernelGGL((dw_rows_kernel<T, MODE, VW>), dim3((unsigned)nblk(RB)), dim3(256), 0, st, a, RB, nstrip, nchunk, nband);
}

template <typename T>
void launch_dw(const DwArgs& a, hipStream_t st) {
  if (a.rows) {
    constexpr int V = Vec<T>::N;
    // a.rows == 3: the bf16 gate at 4 channels per lane (tools/dwbench; measured slower on MI355X:
    // L3 gate 172 -> 227 us despite 7 instead of 3 waves per SIMD - the 8-byte loads cost more than
    // the occupancy buys)
    if (a.mode == DW_GATE && sizeof(T) == 2 && a.rows == 3 && a.C % 4 == 0) launch_dw_rows<T, DW_GATE, 4>(a, st);
    else if (a.mode == DW_GATE) launch_dw_rows<T, DW_GATE, V>(a, st);
    else if (a.mode == DW_GELU) launch_dw_rows<T, DW_GELU, V>(a, st);
    else launch_dw_rows<T, DW_PLAIN, V>(a, st);
    return;
  }
  const int64_t total = (int64_t)a.nimg * a.H * a.W * (a.C / Vec<T>::N);
  const int64_t blocks = (total + 255) / 256;
  if (a.mode == DW_GATE) hipLaunchKernelGGL((dw_kernel<T, DW_GATE>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  else if (a.mode == DW_GELU) hipLaunchKernelGGL((dw_kernel<T, DW_GELU>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((dw_kernel<T, DW_PLAIN>), dim3((unsigned)blocks), dim3(256), 0, st, a);
}

// ------------------------------------------------------------------------------------------
// SAB window conv + L2 normalisation: one block per token
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void window_kernel(WinArgs a) {
  // thread = (channel vector cv, tap subset `part`); C / VEC <= 256 for every Turtle level
  constexpr int VEC = Vec<T>::N;
  __shared__ float red[256 * VEC];
  __shared__ float ss[4];
  const int th = a.H / a.ws, tw = a.W / a.ws, N = th * tw;
  const int n = blockIdx.x % N;
  const int64_t img = blockIdx.x / N;
  const int ti = n / tw, tj = n % tw;
  const int CV = a.C / VEC, nparts = 256 / CV;
  const int tid = threadIdx.x, cv = tid % CV, part = tid / CV;
  const T* in = reinterpret_cast<const T*>(a.in);
  const int taps = a.ws * a.ws;
  float acc[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) acc[i] = 0.f;
  if (part < nparts) {
    for (int tp = part; tp < taps; tp += nparts) {
      const int dy = tp / a.ws, dx = tp % a.ws;
      const int y = ti * a.ws - 1 + dy, x = tj * a.ws - 1 + dx;   // padding = 1
      if (y < 0 || y >= a.H || x < 0 || x >= a.W) continue;
      Vec<T> v; v.load(in + ((img * a.H + y) * a.W + x) * a.ldi + a.offi + cv * VEC);
      const float* wt = a.w + (int64_t)tp * a.C + cv * VEC;
#pragma unroll
      for (int i = 0; i < VEC; ++i) acc[i] = fmaf(wt[i], v.v[i], acc[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < VEC; ++i) red[tid * VEC + i] = acc[i];
  __syncthreads();
  if (tid < CV) {
    for (int pp = 1; pp < nparts; ++pp)
#pragma unroll
      for (int i = 0; i < VEC; ++i) acc[i] += red[(pp * CV + tid) * VEC + i];
  }
  __syncthreads();
  if (tid < CV) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) red[tid * VEC + i] = acc[i];
  }
  __syncthreads();
  // L2 normalisation over the C = 2c token features (F.normalize, eps 1e-12)
  float s = 0.f;
  for (int c = tid; c < a.C; c += 256) {
    float v = red[c] + (a.bias ? a.bias[c] : 0.f);
    red[c] = v;
    s += v * v;
  }
  s = wave_sum(s);
  if ((tid & 63) == 0) ss[tid >> 6] = s;
  __syncthreads();
  const float tot = ss[0] + ss[1] + ss[2] + ss[3];
  const float inv = 1.f / fmaxf(sqrtf(tot), 1e-12f);
  T* out = reinterpret_cast<T*>(a.out) + img * a.out_img_stride + (int64_t)n * a.C;
  for (int c = tid; c < a.C; c += 256) out[c] = from_f<T>(red[c] * inv);
}

template <typename T>
void launch_window(const WinArgs& a, hipStream_t st) {
  const int N = (a.H / a.ws) * (a.W / a.ws);
  hipLaunchKernelGGL(window_kernel<T>, dim3((unsigned)(a.nimg * N)), dim3(256), 0, st, a);
}

// ------------------------------------------------------------------------------------------
// input_projection: zero-padded (or SR bilinear x4 then padded) frame -> 3x3 conv -> pixel-major
// ------------------------------------------------------------------------------------------
TURTLE_DEV float frame_px(const StemArgs& a, int b, int f, int c, int y, int x) {
  // value of channel c of frame f at padded working coordinate (y, x); 0 outside the image.
  // Branch-free: coordinates are clamped so every load is in bounds and issued unconditionally.
  const float* base = a.inp + (int64_t)b * a.in_bstride + (int64_t)f * a.in_fstride + (int64_t)c * a.Hin * a.Win;
  if (!a.sr) {
    const bool in = y >= 0 && y < a.Hin && x >= 0 && x < a.Win;
    const int yc = min(max(y, 0), a.Hin - 1), xc = min(max(x, 0), a.Win - 1);
    const float v = base[(int64_t)yc * a.Win + xc];
    return in ? v : 0.f;
  }
  // TurtleSuper_t1: nn.Upsample(scale_factor=4, bilinear, align_corners=False), then zero pad
  const bool in = y >= 0 && y < 4 * a.Hin && x >= 0 && x < 4 * a.Win;
  const float sy = fmaxf(0.25f * (y + 0.5f) - 0.5f, 0.f), sx = fmaxf(0.25f * (x + 0.5f) - 0.5f, 0.f);
  const int y0 = min((int)sy, a.Hin - 1), x0 = min((int)sx, a.Win - 1);
  const int y1 = y0 < a.Hin - 1 ? y0 + 1 : y0, x1 = x0 < a.Win - 1 ? x0 + 1 : x0;
  const float ly = sy - y0, lx = sx - x0;
  const float v00 = base[(int64_t)y0 * a.Win + x0], v01 = base[(int64_t)y0 * a.Win + x1];
  const float v10 = base[(int64_t)y1 * a.Win + x0], v11 = base[(int64_t)y1 * a.Win + x1];
  const float v = (1.f - ly) * ((1.f - lx) * v00 + lx * v01) + ly * ((1.f - lx) * v10 + lx * v11);
  return in ? v : 0.f;
}

// 16x16 output pixels per block: the (18x18 x CIN) input patch is staged in LDS once, each thread
// keeps its 9*CIN taps in registers and sweeps the output channels 8 at a time; the weights are
// block-uniform (scalar loads), so the inner loop is pure v_fma with SGPR operands.
constexpr int ST_T = 16;
template <typename T, int CIN>
__global__ __launch_bounds__(256) void stem_kernel(StemArgs a) {
  __shared__ float sIn[CIN][ST_T + 2][ST_T + 2];
  const int tid = threadIdx.x;
  const int tx_n = (a.Wp + ST_T - 1) / ST_T;
  const int x0 = (blockIdx.x % tx_n) * ST_T, y0 = (blockIdx.x / tx_n) * ST_T, b = blockIdx.y;
  for (int v = tid; v < CIN * (ST_T + 2) * (ST_T + 2); v += 256) {
    const int ci = v / ((ST_T + 2) * (ST_T + 2)), r = v % ((ST_T + 2) * (ST_T + 2));
    const int yy = y0 - 1 + r / (ST_T + 2), xx = x0 - 1 + r % (ST_T + 2);
    const int f = a.use_both ? (ci < a.Cimg ? 0 : 1) : 1;
    const int c = a.use_both ? ci % a.Cimg : ci;
    // the conv's own zero padding sits at the padded-frame border
    const bool inpad = yy >= 0 && yy < a.Hp && xx >= 0 && xx < a.Wp;
    const float val = frame_px(a, b, f, c, yy, xx);
    sIn[ci][r / (ST_T + 2)][r % (ST_T + 2)] = inpad ? val : 0.f;
  }
  __syncthreads();
  const int ty = tid / ST_T, tx = tid % ST_T, y = y0 + ty, x = x0 + tx;
  float in[CIN * 9];
#pragma unroll
  for (int ci = 0; ci < CIN; ++ci)
#pragma unroll
    for (int t = 0; t < 9; ++t) in[ci * 9 + t] = sIn[ci][ty + t / 3][tx + t % 3];
  if (y >= a.Hp || x >= a.Wp) return;
  T* o = reinterpret_cast<T*>(a.out) + (((int64_t)b * a.Hp + y) * a.Wp + x) * a.Cout;
  for (int co = 0; co < a.Cout; co += 8) {
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = a.bias ? a.bias[co + i] : 0.f;
#pragma unroll
    for (int k = 0; k < CIN * 9; ++k)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = fmaf(a.w[(co + i) * CIN * 9 + k], in[k], acc[i]);
#pragma unroll
    for (int i0 = 0; i0 < 8; i0 += Vec<T>::N) {
      Vec<T> ov;
#pragma unroll
      for (int i = 0; i < Vec<T>::N; ++i) ov.v[i] = acc[i0 + i];
      ov.store(o + co + i0);
    }
  }
}

template <typename T>
void launch_stem(const StemArgs& a, hipStream_t st) {
  const int cin = a.use_both ? 2 * a.Cimg : a.Cimg;
  const dim3 grid((unsigned)(((a.Wp + ST_T - 1) / ST_T) * ((a.Hp + ST_T - 1) / ST_T)), (unsigned)a.B);
  switch (cin) {
    case 1: hipLaunchKernelGGL((stem_kernel<T, 1>), grid, dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL((stem_kernel<T, 2>), grid, dim3(256), 0, st, a); break;
    case 3: hipLaunchKernelGGL((stem_kernel<T, 3>), grid, dim3(256), 0, st, a); break;
    case 4: hipLaunchKernelGGL((stem_kernel<T, 4>), grid, dim3(256), 0, st, a); break;
    case 6: hipLaunchKernelGGL((stem_kernel<T, 6>), grid, dim3(256), 0, st, a); break;
    case 8: hipLaunchKernelGGL((stem_kernel<T, 8>), grid, dim3(256), 0, st, a); break;
    default: break;   // n_colors is 1..4 (turtle.cpp)
  }
}

// ------------------------------------------------------------------------------------------
// ending: 3x3 Cin->Cimg (+bias) + current padded frame, cropped to the output size
// ------------------------------------------------------------------------------------------
// one thread per output pixel; every tap row is fetched with unconditional 16-byte loads (a zero
// line for taps outside the padded map), the weights are wave-uniform scalar loads
__device__ __attribute__((aligned(64))) uint4 g_zero_end[4];
template <typename T, int CO>
__global__ __launch_bounds__(256) void ending_kernel(EndArgs a) {
  constexpr int VEC = Vec<T>::N;
  const int64_t total = (int64_t)a.B * a.Hout * a.Wout;
  const T* xin = reinterpret_cast<const T*>(a.x);
  StemArgs s{};
  s.inp = a.inp; s.in_bstride = a.in_bstride; s.in_fstride = a.in_fstride;
  s.Cimg = a.Cimg; s.Hin = a.Hin; s.Win = a.Win; s.sr = a.sr;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool live = idx < total;
  const int64_t id = live ? idx : 0;
  const int x = (int)(id % a.Wout);
  const int y = (int)((id / a.Wout) % a.Hout);
  const int b = (int)(id / ((int64_t)a.Wout * a.Hout));
  float acc[CO];
#pragma unroll
  for (int co = 0; co < CO; ++co) acc[co] = a.bias[co];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
    const bool ok = yy >= 0 && yy < a.Hp && xx >= 0 && xx < a.Wp;
    const T* p = xin + (((int64_t)b * a.Hp + (ok ? yy : 0)) * a.Wp + (ok ? xx : 0)) * a.Cin;
    for (int c0 = 0; c0 < a.Cin; c0 += 4 * VEC) {
      uint4 q[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        q[u] = ld16(ok && c0 + u * VEC < a.Cin ? reinterpret_cast<const void*>(p + c0 + u * VEC) : g_zero_end);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        Vec<T> v;
        v.from_raw(q[u]);
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const int c = min(c0 + u * VEC + i, a.Cin - 1);
#pragma unroll
          for (int co = 0; co < CO; ++co) acc[co] = fmaf(a.w[(co * a.Cin + c) * 9 + tap], v.v[i], acc[co]);
        }
      }
    }
  }
  if (!live) return;
#pragma unroll
  for (int co = 0; co < CO; ++co)
    a.out[(((int64_t)b * a.Cimg + co) * a.Hout + y) * a.Wout + x] = acc[co] + frame_px(s, b, 1, co, y, x);
}

template <typename T>
void launch_ending(const EndArgs& a, hipStream_t st) {
  const int64_t total = (int64_t)a.B * a.Hout * a.Wout;
  const unsigned blocks = (unsigned)((total + 255) / 256);
  switch (a.Cimg) {
    case 1: hipLaunchKernelGGL((ending_kernel<T, 1>), dim3(blocks), dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL((ending_kernel<T, 2>), dim3(blocks), dim3(256), 0, st, a); break;
    case 3: hipLaunchKernelGGL((ending_kernel<T, 3>), dim3(blocks), dim3(256), 0, st, a); break;
    case 4: hipLaunchKernelGGL((ending_kernel<T, 4>), dim3(blocks), dim3(256), 0, st, a); break;
    default: break;   // n_colors is 1..4 (turtle.cpp)
  }
}

// ------------------------------------------------------------------------------------------
// latent FHR cache roll: out[b][p][h][r'] = concat(old[b][p][h][0:R], cur*kinv)[R + ch - Rnew + r']
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void fhr_cache_kernel(FhrCacheArgs a) {
  const int64_t total = (int64_t)a.B * a.P * a.heads * a.Rnew;
  const T* old = reinterpret_cast<const T*>(a.old);
  const T* cur = reinterpret_cast<const T*>(a.cur);
  T* out = reinterpret_cast<T*>(a.out);
  const int shift = a.R + a.ch - a.Rnew;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    const int rn = (int)(idx % a.Rnew);
    const int64_t t = idx / a.Rnew;
    const int h = (int)(t % a.heads);
    const int64_t bp = t / a.heads;            // b * P + p
    const int b = (int)(bp / a.P);
    const int r = rn + shift;
    T v;
    if (r < a.R) {
      v = old[(bp * a.heads + h) * a.R + r];
    } else {
      const int j = r - a.R;
      float x = to_f(cur[bp * a.ldc + a.coff + h * a.ch + j]);
      if (a.kinv) x *= a.kinv[(int64_t)b * a.heads * a.ch + h * a.ch + j];
      v = from_f<T>(x);
    }
    out[idx] = v;
  }
}

// same, 16 bytes per thread: with R, Rnew, ch and the shift multiples of the vector width every
// output vector comes whole from the old cache or from the current (rescaled) rows
template <typename T>
__global__ __launch_bounds__(256) void fhr_cache_vec_kernel(FhrCacheArgs a) {
  constexpr int VEC = Vec<T>::N;
  const int nv = a.Rnew / VEC;
  const int64_t total = (int64_t)a.B * a.P * a.heads * nv;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const T* old = reinterpret_cast<const T*>(a.old);
  const T* cur = reinterpret_cast<const T*>(a.cur);
  const int shift = a.R + a.ch - a.Rnew;
  const int rv = (int)(idx % nv);
  const int64_t t = idx / nv;
  const int h = (int)(t % a.heads);
  const int64_t bp = t / a.heads;
  const int r = rv * VEC + shift;
  Vec<T> v;
  if (r < a.R) {
    v.load(old + (bp * a.heads + h) * a.R + r);
  } else {
    const int j = r - a.R, b = (int)(bp / a.P);
    v.load(cur + bp * a.ldc + a.coff + h * a.ch + j);
    if (a.kinv) {
      const float* kv = a.kinv + (int64_t)b * a.heads * a.ch + h * a.ch + j;
#pragma unroll
      for (int i = 0; i < VEC; ++i) v.v[i] *= kv[i];
    }
  }
  v.store(reinterpret_cast<T*>(a.out) + (bp * a.heads + h) * a.Rnew + rv * VEC);
}

template <typename T>
void launch_fhr_cache(const FhrCacheArgs& a, hipStream_t st) {
  constexpr int VEC = Vec<T>::N;
  const int shift = a.R + a.ch - a.Rnew;
  if (a.R % VEC == 0 && a.Rnew % VEC == 0 && a.ch % VEC == 0 && shift % VEC == 0 && a.ldc % VEC == 0 && a.coff % VEC == 0) {
    const int64_t total = (int64_t)a.B * a.P * a.heads * (a.Rnew / VEC);
    hipLaunchKernelGGL(fhr_cache_vec_kernel<T>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, a);
    return;
  }
  const int64_t total = (int64_t)a.B * a.P * a.heads * a.Rnew;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(fhr_cache_kernel<T>, dim3((unsigned)blocks), dim3(256), 0, st, a);
}

__global__ void cast_kernel(const float* src, void* dst, int64_t n, int to_bf16) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    if (to_bf16) reinterpret_cast<bf16*>(dst)[i] = (bf16)src[i];
    else reinterpret_cast<float*>(dst)[i] = src[i];
  }
}
void launch_cast_f32(const float* src, void* dst, int64_t n, int to_bf16, hipStream_t st) {
  int64_t blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(cast_kernel, dim3((unsigned)blocks), dim3(256), 0, st, src, dst, n, to_bf16);
}

// ------------------------------------------------------------------------------------------
// bf16 stem / ending on the matrix cores. One wave = a 16-pixel run of a padded row:
//   ending: C[co][px] = W[co][tap*Cin + c] . X[tap*Cin + c][px]   (K = 9 Cin, co < Cimg padded to 16)
//   stem:   C[co][px] = W[co][ci*9 + tap] . F[ci*9 + tap][px]     (K = 9 Cimg padded to 32, 64 co)
// A = weights as register fragments built once per wave, B = the 16 pixels' operands: for the ending
// 16-byte channel vectors straight from the pixel-major map, for the stem 8 gathered frame samples
// (zero pad / SR bilinear, frame_px) per lane. Per-wave work loops over runs (grid-stride).
// ------------------------------------------------------------------------------------------
template <int CIN>
__global__ __launch_bounds__(256) void ending_mfma_kernel(EndArgs a) {
  constexpr int KS = 9 * CIN / 32;
  const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const int wv = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  bf16x8 wf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    bf16x8 f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = s * 32 + g * 8 + j, tap = k / CIN, c = k - tap * CIN;
      f[j] = (bf16)(li < a.Cimg ? a.w[(li * CIN + c) * 9 + tap] : 0.f);
    }
    wf[s] = f;
  }
  float bias[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) bias[i] = i < a.Cimg ? a.bias[i] : 0.f;
  StemArgs s{};
  s.inp = a.inp; s.in_bstride = a.in_bstride; s.in_fstride = a.in_fstride;
  s.Cimg = a.Cimg; s.Hin = a.Hin; s.Win = a.Win; s.sr = a.sr;
  const bf16* X = reinterpret_cast<const bf16*>(a.x);
  const int tpr = (a.Wp + 15) / 16, nt = a.B * a.Hp * tpr;
  for (int t = wv; t < nt; t += nw) {
    const int tx = t % tpr, row = t / tpr, y = row % a.Hp, b = row / a.Hp;
    const int x = tx * 16 + li;
    uint4 xv[KS];
#pragma unroll
    for (int st = 0; st < KS; ++st) {
      const int k0 = st * 32 + g * 8, tap = k0 / CIN, c = k0 - tap * CIN;
      const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
      const bool ok = yy >= 0 && yy < a.Hp && xx >= 0 && xx < a.Wp;
      xv[st] = ld16(ok ? reinterpret_cast<const void*>(X + (((int64_t)b * a.Hp + yy) * a.Wp + xx) * CIN + c) : g_zero_end);
    }
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int st = 0; st < KS; ++st) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[st], __builtin_bit_cast(bf16x8, xv[st]), acc, 0, 0, 0);
    // C: column li = pixel, rows 4 g + i = output channel (only g == 0 holds co < 4)
    if (g == 0 && y < a.Hout && x < a.Wout) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (i < a.Cimg)
          a.out[(((int64_t)b * a.Cimg + i) * a.Hout + y) * a.Wout + x] = acc[i] + bias[i] + frame_px(s, b, 1, i, y, x);
    }
  }
}

// Tiled form of the same ending: a block owns 4 rows x 64 columns of output, stages the haloed
// (6 x 66 pixels x CIN) input once in LDS with coalesced 16-byte loads (1.5x halo instead of every
// tap's 16-byte vector coming from L2: 9x), and each wave runs its row as 4 runs of 16 pixels with
// the MFMA B operands read from LDS (pixel rows padded to CIN * 2 + 16 bytes: conflict-free
// ds_read_b128 for 16 consecutive pixels).
constexpr int ET_R = 4, ET_C = 64;
template <int CIN>
__global__ __launch_bounds__(256) void ending_tile_kernel(EndArgs a) {
  constexpr int KS = 9 * CIN / 32, PB = CIN * 2 + 16, TW = ET_C + 2, NPX = (ET_R + 2) * TW, CV = CIN / 8;
  __shared__ __attribute__((aligned(16))) char sx[NPX * PB];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4, li = lane & 15;
  const int tpr = (a.Wp + ET_C - 1) / ET_C, tpc = (a.Hp + ET_R - 1) / ET_R;
  const int bx = blockIdx.x % tpr, rest = blockIdx.x / tpr, by = rest % tpc, b = rest / tpc;
  const int x0 = bx * ET_C, y0 = by * ET_R;
  const bf16* X = reinterpret_cast<const bf16*>(a.x);
  // haloed tile -> LDS (zero outside the padded image)
  for (int e = tid; e < NPX * CV; e += 256) {
    const int p = e / CV, k = e - p * CV, r = p / TW, c = p - r * TW;
    const int yy = y0 - 1 + r, xx = x0 - 1 + c;
    const bool ok = yy >= 0 && yy < a.Hp && xx >= 0 && xx < a.Wp;
    const uint4 v = ld16(ok ? reinterpret_cast<const void*>(X + (((int64_t)b * a.Hp + yy) * a.Wp + xx) * CIN + k * 8) : g_zero_end);
    *reinterpret_cast<uint4*>(sx + p * PB + k * 16) = v;
  }
  bf16x8 wf[KS];                                   // pre-packed A fragments: one 16-byte load each
#pragma unroll
  for (int s = 0; s < KS; ++s) wf[s] = __builtin_bit_cast(bf16x8, ld16(reinterpret_cast<const bf16*>(a.wfrag) + (s * 64 + lane) * 8));
  float bias[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) bias[i] = i < a.Cimg ? a.bias[i] : 0.f;
  StemArgs s{};
  s.inp = a.inp; s.in_bstride = a.in_bstride; s.in_fstride = a.in_fstride;
  s.Cimg = a.Cimg; s.Hin = a.Hin; s.Win = a.Win; s.sr = a.sr;
  __syncthreads();
  const int y = y0 + wid;                          // wave = output row
#pragma unroll
  for (int run = 0; run < ET_C / 16; ++run) {
    const int xl = run * 16 + li;                  // output column in the tile
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int st = 0; st < KS; ++st) {
      const int k0 = st * 32 + g * 8, tap = k0 / CIN, c = k0 - tap * CIN;
      const int r = wid + tap / 3, cc = xl + tap % 3;   // haloed tile coordinates of the tap
      const bf16x8 bv = *reinterpret_cast<const bf16x8*>(sx + (r * TW + cc) * PB + c * 2);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[st], bv, acc, 0, 0, 0);
    }
    // rows 4..7 (lanes 16..31) hold the split-bf16 remainder part of the weights (turtle.cpp)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] += __shfl_down(acc[i], 16, 64);
    const int x = x0 + xl;
    if (g == 0 && y < a.Hout && x < a.Wout) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (i < a.Cimg)
          a.out[(((int64_t)b * a.Cimg + i) * a.Hout + y) * a.Wout + x] = acc[i] + bias[i] + frame_px(s, b, 1, i, y, x);
    }
  }
}

// Down1_2 (turtle_t1_arch.py:136-144 at level 1): 3x3 conv CIN -> COUT = CIN / 2 + PixelUnshuffle(2),
// LDS-tiled like the ending: a block owns 4 rows x 64 columns of the conv output, stages the
// haloed 6 x 66 x CIN input once (coalesced 16-byte loads), and each wave runs its row as 4 runs of
// 16 pixels x COUT channels on the matrix cores (A = pre-packed weight fragments in registers, B =
// pixel rows from LDS). The unshuffled output tile (2 rows x 32 pixels x 4 COUT channels) is staged
// in LDS and written as 16-byte rows. Against the implicit-GEMM path (9 L2 re-reads of every input
// vector for a 32-channel output): each input byte leaves L2 about 1.5 times.
constexpr int DT_R = 4, DT_C = 64;
template <int CIN>
__global__ __launch_bounds__(256) void down_tile_kernel(DownTileArgs a) {
  constexpr int COUT = CIN / 2, NCT = COUT / 16, KS = 9 * CIN / 32, PB = CIN * 2 + 16, TW = DT_C + 2, NPX = (DT_R + 2) * TW;
  constexpr int CV = CIN / 8, OC = 4 * COUT;               // output channels after the unshuffle
  __shared__ __attribute__((aligned(16))) char sx[NPX * PB];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4, li = lane & 15;
  const int tpr = (a.W + DT_C - 1) / DT_C, tpc = (a.H + DT_R - 1) / DT_R;
  const int bx = blockIdx.x % tpr, rest = blockIdx.x / tpr, by = rest % tpc, b = rest / tpc;
  const int x0 = bx * DT_C, y0 = by * DT_R;
  const bf16* X = reinterpret_cast<const bf16*>(a.x);
  for (int e = tid; e < NPX * CV; e += 256) {
    const int p = e / CV, k = e - p * CV, r = p / TW, c = p - r * TW;
    const int yy = y0 - 1 + r, xx = x0 - 1 + c;
    const bool ok = yy >= 0 && yy < a.H && xx >= 0 && xx < a.W;
    const uint4 v = ld16(ok ? reinterpret_cast<const void*>(X + (((int64_t)b * a.H + yy) * a.W + xx) * a.ldx + k * 8) : g_zero_end);
    *reinterpret_cast<uint4*>(sx + p * PB + k * 16) = v;
  }
  bf16x8 wf[NCT][KS];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
    for (int st = 0; st < KS; ++st)
      wf[ct][st] = __builtin_bit_cast(bf16x8, ld16(reinterpret_cast<const bf16*>(a.wfrag) + ((ct * KS + st) * 64 + lane) * 8));
  __syncthreads();
  const int y = y0 + wid;
  f32x4 acc[DT_C / 16][NCT];
#pragma unroll
  for (int run = 0; run < DT_C / 16; ++run) {
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) acc[run][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int xl = run * 16 + li;
#pragma unroll
    for (int st = 0; st < KS; ++st) {
      const int k0 = st * 32 + g * 8, tap = k0 / CIN, c = k0 - tap * CIN;
      const bf16x8 bv = *reinterpret_cast<const bf16x8*>(sx + ((wid + tap / 3) * TW + xl + tap % 3) * PB + c * 2);
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) acc[run][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ct][st], bv, acc[run][ct], 0, 0, 0);
    }
  }
  __syncthreads();                                  // the input tile is dead: LDS holds the output tile
  // lane: conv-output channels 16 ct + 4 g + i of pixel (y, x0 + 16 run + li) -> unshuffled pixel
  // ((y - y0) / 2, (xl) / 2), channel (16 ct + 4 g + i) * 4 + (y & 1) * 2 + (xl & 1)
  char* so = sx;                                     // [DT_R / 2][DT_C / 2][OC] bf16
#pragma unroll
  for (int run = 0; run < DT_C / 16; ++run) {
    const int xl = run * 16 + li;
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = 16 * ct + 4 * g + i;
        const int off = ((wid >> 1) * (DT_C / 2) + (xl >> 1)) * OC + co * 4 + (wid & 1) * 2 + (xl & 1);
        reinterpret_cast<bf16*>(so)[off] = (bf16)acc[run][ct][i];
      }
  }
  __syncthreads();
  const int Ho = a.H / 2, Wo = a.W / 2, Y0 = y0 / 2, X0 = x0 / 2;
  bf16* O = reinterpret_cast<bf16*>(a.out);
  constexpr int NV16 = (DT_R / 2) * (DT_C / 2) * OC / 8;
  for (int e = tid; e < NV16; e += 256) {
    const int px = e / (OC / 8), k = e - px * (OC / 8), yr = px / (DT_C / 2), xc = px - yr * (DT_C / 2);
    const int Y = Y0 + yr, Xo = X0 + xc;
    if (Y < Ho && Xo < Wo)
      *reinterpret_cast<uint4*>(O + (((int64_t)b * Ho + Y) * Wo + Xo) * a.ldo + k * 8) = *reinterpret_cast<const uint4*>(so + (px * OC + k * 8) * 2);
  }
}

bool down_tile_ok(const DownTileArgs& a) {
  if (a.Cin != 64 || !a.wfrag || !a.x || !a.out || a.H % 2 || a.W % 2 || a.H < 2 || a.W < 2) return false;
  if (a.ldx % 8 || a.ldo % 8 || a.ldo < 2 * a.Cin) return false;
  return ((reinterpret_cast<uintptr_t>(a.x) | reinterpret_cast<uintptr_t>(a.out) | reinterpret_cast<uintptr_t>(a.wfrag)) & 15) == 0;
}

void launch_down_tile(const DownTileArgs& a, hipStream_t st) {
  const int64_t blocks = (int64_t)a.nimg * ((a.H + DT_R - 1) / DT_R) * ((a.W + DT_C - 1) / DT_C);
  hipLaunchKernelGGL(down_tile_kernel<64>, dim3((unsigned)blocks), dim3(256), 0, st, a);
}

template <int CIN>   // frame channels (Cimg, or 2 Cimg with use_both_input); K = 9 CIN padded to 32 KS
__global__ __launch_bounds__(256) void stem_mfma_kernel(StemArgs a) {
  constexpr int KS = (9 * CIN + 31) / 32;
  __shared__ __attribute__((aligned(16))) char stile[4][16 * 144];    // per wave: 16 px x 64 co bf16
  const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15, wid = threadIdx.x >> 6;
  const int wv = blockIdx.x * 4 + wid, nw = gridDim.x * 4;
  // A fragments: W[co][ci][tap] (fp32 [64][CIN][3][3]), co = 16 ct + li, k = ci*9 + tap
  bf16x8 wf[4][KS];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int st = 0; st < KS; ++st) {
      bf16x8 f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = st * 32 + g * 8 + j, co = ct * 16 + li;
        f[j] = (bf16)(k < 9 * CIN && co < a.Cout ? a.w[co * 9 * CIN + k] : 0.f);
      }
      wf[ct][st] = f;
    }
  const int tpr = (a.Wp + 15) / 16, nt = a.B * a.Hp * tpr;
  char* sw = stile[wid];
  for (int t = wv; t < nt; t += nw) {
    const int tx = t % tpr, row = t / tpr, y = row % a.Hp, b = row / a.Hp;
    const int x = tx * 16 + li;
    bf16x8 xf[KS];
#pragma unroll
    for (int st = 0; st < KS; ++st) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = st * 32 + g * 8 + j;
        const int ci = k / 9, tap = k - ci * 9;
        const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
        const int f = a.use_both ? (ci < a.Cimg ? 0 : 1) : 1, c = a.use_both ? ci % a.Cimg : ci;
        const bool inpad = k < 9 * CIN && yy >= 0 && yy < a.Hp && xx >= 0 && xx < a.Wp;
        const float val = frame_px(a, b, f, min(c, a.Cimg - 1), yy, xx);
        xf[st][j] = (bf16)(inpad ? val : 0.f);
      }
    }
    f32x4 acc[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      acc[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < KS; ++st) acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ct][st], xf[st], acc[ct], 0, 0, 0);
    }
    // C: column li = pixel, rows 4 g + i = channel 16 ct + 4 g + i -> LDS [px][co], then 16-byte rows
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) { const int co = ct * 16 + g * 4 + i; v[i] = acc[ct][i] + (a.bias ? a.bias[co] : 0.f); }
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
      *reinterpret_cast<bf16x4*>(sw + li * 144 + (ct * 16 + g * 4) * 2) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    bf16* o = reinterpret_cast<bf16*>(a.out);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int pc = lane + 64 * h, px = pc >> 3, k = pc & 7;
      const uint4 q = *reinterpret_cast<const uint4*>(sw + px * 144 + k * 16);
      const int xo = tx * 16 + px;
      if (xo < a.Wp) *reinterpret_cast<uint4*>(o + (((int64_t)b * a.Hp + y) * a.Wp + xo) * 64 + k * 8) = q;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

bool stem_end_mfma_ok(int cin_end, int cin_stem, int cout_stem) {
  return cin_end == 64 && cout_stem == 64 && (cin_stem == 3 || cin_stem == 6);
}

bool launch_ending_mfma(const EndArgs& a, hipStream_t st) {
  if (!a.wfrag || a.Cin != 64 || a.Cimg < 1 || a.Cimg > 4) return false;   // fragments packed by turtle.cpp; bias[4]
  const int64_t tiles = (int64_t)a.B * ((a.Hp + ET_R - 1) / ET_R) * ((a.Wp + ET_C - 1) / ET_C);
  hipLaunchKernelGGL(ending_tile_kernel<64>, dim3((unsigned)tiles), dim3(256), 0, st, a);
  return true;
}

void launch_stem_mfma(const StemArgs& a, hipStream_t st) {
  const int cin = a.use_both ? 2 * a.Cimg : a.Cimg;
  if (cin == 3) hipLaunchKernelGGL(stem_mfma_kernel<3>, dim3(2048), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(stem_mfma_kernel<6>, dim3(2048), dim3(256), 0, st, a);
}

#define INST(T)                                                          \
  template void launch_dw<T>(const DwArgs&, hipStream_t);                \
  template void launch_window<T>(const WinArgs&, hipStream_t);           \
  template void launch_stem<T>(const StemArgs&, hipStream_t);            \
  template void launch_ending<T>(const EndArgs&, hipStream_t);           \
  template void launch_fhr_cache<T>(const FhrCacheArgs&, hipStream_t);
INST(float)
INST(bf16)

}  // namespace turtle

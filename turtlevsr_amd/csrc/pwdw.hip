// Pointwise GEMM -> depthwise 3x3 (-> gate) in one kernel, for the wide levels (c >= 256, bf16):
//
//   GATE   GatedFeedForward   LN -> project_in (c -> 2h) -> dwconv -> gelu(x1) * x2     (h out)
//          turtle_t1_arch.py:159-178
//   PLAIN  ChannelAttention   LN -> qkv (c -> 3c) -> qkv_dwconv                         (3c out)
//          turtle_t1_arch.py:666-684
//
// so the 2h- / 3c-wide hidden map never reaches HBM (at 1080p L3 that is 334 MB written and read
// back per GatedFeedForward). Block = an 8 x 32 output-pixel tile x a 128-column GEMM1 slice
// (PLAIN: 128 channels; GATE: 64 x1 + the matching 64 x2 channels), 512 threads:
//   1. GEMM1 over the 10 x 34 haloed pixels (340 rows, 22 MFMA row tiles; 1.33x recompute),
//      K = c in BK = 64 steps: both operands by global_load_lds into two LDS stages (XOR-swizzled
//      128-byte rows as in gemm2.hip), 8 waves = 4 row groups x 2 column halves, 16x16x32 MFMA;
//      LayerNorm statistics from the staged A tiles (affine folded into W1 at pack time);
//   2. epilogue: LN / bias -> bf16 hidden tile [352][128] in LDS (over the dead stages), rows
//      outside the image forced to zero (the depthwise conv zero-pads its input);
//   3. depthwise 3x3 (+bias) per (pixel, 8-channel vector) from LDS, GATE: gelu(x1) * x2, 16-byte
//      coalesced stores (a pixel's channel vectors are consecutive lanes).
// Consecutive block ids are the column slices of one pixel tile, so the haloed input tile is read
// from HBM once and from L2 by the other slices.
#include "common.h"
#include "kernels.h"

namespace turtle {

__device__ __attribute__((aligned(64))) uint4 g_zero_pw[4];

constexpr int PW_TH = 8, PW_TW = 32;                     // output tile
constexpr int PW_HH = PW_TH + 2, PW_HW = PW_TW + 2;      // haloed tile 10 x 34
constexpr int PW_HROWS = PW_HH * PW_HW;                  // 340 haloed pixels
constexpr int PW_MT = 22;                                // 16-row MFMA tiles over 352 rows
constexpr int PW_AROWS = 384;                            // A stage rows (48 uniform DMA per stage)
constexpr int PW_NC = 128;                               // GEMM1 columns per block
constexpr int PW_A_BYTES = PW_AROWS * 128;
constexpr int PW_W_BYTES = PW_NC * 128;
constexpr int PW_STAGE = PW_A_BYTES + PW_W_BYTES;        // 64 KB
constexpr int PW_HROW = PW_NC * 2 + 16;                  // hidden tile row bytes (bf16 + pad)
constexpr int PW_MAIN = 2 * PW_STAGE;                    // 128 KB (hidden tile 94 KB overlays it)
constexpr int PW_EPI = PW_MAIN;                          // ln_t+b1 [128], dw weights [9][128], dw bias [128]
constexpr int PW_STATS = PW_EPI + (PW_NC + 9 * PW_NC + PW_NC + PW_NC) * 4;   // mu, rstd [352]
constexpr int PW_BYTES = PW_STATS + 2 * 352 * 4;
static_assert(352 * PW_HROW <= PW_MAIN, "hidden tile overlays the stages");

typedef __attribute__((address_space(3))) void pw_lds_void;

template <int N>
TURTLE_DEV void pw_wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}
TURTLE_DEV void pw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int GATE>
__global__ __launch_bounds__(512, 2) void pwdw_kernel(PwdwArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* e_b = reinterpret_cast<float*>(smem + PW_EPI);           // ln_t + b1 per column
  float* e_w = e_b + PW_NC;                                      // dw taps [9][128]
  float* e_db = e_w + 9 * PW_NC;                                 // dw bias [128]
  float* e_s = e_db + PW_NC;                                     // ln_s per column
  float* s_mu = reinterpret_cast<float*>(smem + PW_STATS);
  float* s_rs = s_mu + 352;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;                         // 4 row groups x 2 column halves
  const int K = a.C, nk = (K + 63) / 64;
  const int hid = GATE ? a.N1 / 2 : a.N1;                        // output channels
  const int nsl = GATE ? hid / 64 : hid / 128;                   // column slices
  const int tx_n = (a.W + PW_TW - 1) / PW_TW, ty_n = (a.H + PW_TH - 1) / PW_TH;
  int lin = blockIdx.x;
  {
    const int nblk = gridDim.x, q = nblk / 8, r = nblk % 8, x = lin % 8, y = lin / 8;
    lin = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;
  }
  const int sl = lin % nsl;
  int t = lin / nsl;
  const int txi = t % tx_n;
  t /= tx_n;
  const int tyi = t % ty_n;
  const int img = t / ty_n;
  const int ty0 = tyi * PW_TH, tx0 = txi * PW_TW;
  // GEMM1 column n (0..127) of this slice -> W1 / dw row
  auto colrow = [&](int n) -> int {
    if (GATE) return n < 64 ? sl * 64 + n : hid + sl * 64 + (n - 64);
    return sl * 128 + n;
  };

  // ---- per-column vectors -> LDS ----
  if (tid < PW_NC) {
    const int r = colrow(tid);
    e_b[tid] = (a.ln_t ? a.ln_t[r] : 0.f) + (a.b1 ? a.b1[r] : 0.f);
    e_s[tid] = a.ln_s ? a.ln_s[r] : 0.f;
    e_db[tid] = a.dwb ? a.dwb[r] : 0.f;
  }
  for (int e = tid; e < 9 * PW_NC; e += 512) {
    const int tap = e / PW_NC, n = e - tap * PW_NC;
    e_w[e] = a.dww[(int64_t)tap * a.N1 + colrow(n)];
  }

  // ---- LDS-DMA geometry: instruction i of wave w fills chunks (i*8 + w)*64 + lane ----
  constexpr int AI = PW_AROWS * 8 / 512, WI = PW_NC * 8 / 512;   // 6, 2
  const bf16* X = reinterpret_cast<const bf16*>(a.x);
  const bf16* W1 = reinterpret_cast<const bf16*>(a.w1);
  const bf16* a_src[AI];
  int a_cc[AI];
  bool a_ok[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int q = (i * 8 + wid) * 64 + lane, r = q >> 3;
    a_cc[i] = ((q & 7) ^ ((r >> 1) & 7)) * 8;
    const int hy = r / PW_HW, hx = r - hy * PW_HW;
    const int y = ty0 - 1 + hy, x = tx0 - 1 + hx;
    a_ok[i] = r < PW_HROWS && y >= 0 && y < a.H && x >= 0 && x < a.W;
    const int yc = a_ok[i] ? y : 0, xc = a_ok[i] ? x : 0;
    a_src[i] = X + (((int64_t)img * a.H + yc) * a.W + xc) * a.ldx + a.offx + a_cc[i];
  }
  const bf16* w_src[WI];
  int w_cc[WI];
#pragma unroll
  for (int i = 0; i < WI; ++i) {
    const int q = (i * 8 + wid) * 64 + lane, r = q >> 3;
    w_cc[i] = ((q & 7) ^ ((r >> 1) & 7)) * 8;
    w_src[i] = W1 + (int64_t)colrow(r) * K + w_cc[i];
  }
  auto issue = [&](int kt, int stage) {
    char* sA = smem + stage * PW_STAGE;
    char* sW = sA + PW_A_BYTES;
    const int k0 = kt * 64;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const bool ok = a_ok[i] && k0 + a_cc[i] < K;
      __builtin_amdgcn_global_load_lds(ok ? reinterpret_cast<const void*>(a_src[i] + k0) : reinterpret_cast<const void*>(g_zero_pw),
                                       (pw_lds_void*)(sA + (i * 8 + wid) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      const bool ok = k0 + w_cc[i] < K;
      __builtin_amdgcn_global_load_lds(ok ? reinterpret_cast<const void*>(w_src[i] + k0) : reinterpret_cast<const void*>(g_zero_pw),
                                       (pw_lds_void*)(sW + (i * 8 + wid) * 1024), 16, 0, 0);
    }
  };

  // wave tile: row tiles wr*6 .. (< 22), column tiles wc*4 .. +3
  constexpr int RT = 6, CT = 4;
  const int rt0 = wr * RT;
  const int nrt = min(RT, PW_MT - rt0);                          // 6, 6, 6, 4 (wave-uniform)
  f32x4 acc[RT][CT];
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int j = 0; j < CT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  const bf16x2 one2 = __builtin_bit_cast(bf16x2, 0x3F803F80u);
  float ls = 0.f, lq = 0.f;                                      // LN sums of row tid (< 352)

  __syncthreads();
  issue(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt & 1;
    if (kt + 1 < nk) {
      issue(kt + 1, st ^ 1);
      pw_wait_vm<AI + WI>();
    } else {
      pw_wait_vm<0>();
    }
    pw_barrier();
    const char* sA = smem + st * PW_STAGE;
    const char* sW = sA + PW_A_BYTES;
    if (a.ln && tid < 352) {
      // all 8 chunks of row tid, visited in swizzled order so the 16 rows of a lane group hit
      // distinct banks (plain order: 8-way conflicts)
      const char* row = sA + tid * 128;
      const int sw = (tid >> 1) & 7;
#pragma unroll
      for (int p = 0; p < 8; ++p) {
        const uint4 x = *reinterpret_cast<const uint4*>(row + ((p ^ sw) << 4));
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
      bf16x8 wf[CT];
#pragma unroll
      for (int j = 0; j < CT; ++j) {
        const int r = wc * 64 + j * 16 + fr;
        wf[j] = *reinterpret_cast<const bf16x8*>(sW + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < RT; ++i) {
        if (i < nrt) {
          const int r = (rt0 + i) * 16 + fr;
          const bf16x8 xf = *reinterpret_cast<const bf16x8*>(sA + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
#pragma unroll
          for (int j = 0; j < CT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf, acc[i][j], 0, 0, 0);
        }
      }
    }
    pw_barrier();
  }
  if (a.ln && tid < 352) {
    const float mu = ls / K;
    s_mu[tid] = mu;
    s_rs[tid] = rsqrtf(fmaxf(lq / K - mu * mu, 0.f) + 1e-5f);
  }
  __syncthreads();

  // ---- epilogue 1: hidden tile [352][128] bf16 over the dead stages; out-of-image rows = 0 ----
  char* sH = smem;
#pragma unroll
  for (int i = 0; i < RT; ++i) {
    if (i >= nrt) continue;
    const int r = (rt0 + i) * 16 + fr;
    const int hy = r / PW_HW, hx = r - hy * PW_HW;
    const int y = ty0 - 1 + hy, x = tx0 - 1 + hx;
    const float in = (r < PW_HROWS && y >= 0 && y < a.H && x >= 0 && x < a.W) ? 1.f : 0.f;
    const float mu = a.ln ? s_mu[r] : 0.f, rs = a.ln ? s_rs[r] : 1.f;
#pragma unroll
    for (int j = 0; j < CT; ++j) {
      const int cl = wc * 64 + j * 16 + fq * 4;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float xv = acc[i][j][e];
        if (a.ln) xv = rs * (xv - mu * e_s[cl + e]);
        v[e] = (xv + e_b[cl + e]) * in;
      }
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
      *reinterpret_cast<bf16x4*>(sH + r * PW_HROW + cl * 2) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
    }
  }
  __syncthreads();

  // ---- depthwise 3x3 (+ gate): item = (output pixel, 8-channel vector) ----
  constexpr int NV = GATE ? 8 : 16;                              // output vectors per pixel
  constexpr int ITEMS = PW_TH * PW_TW * NV / 512;                // 4 (GATE) / 8 (PLAIN) per thread
  const int cv = tid % NV;
  bf16* out = reinterpret_cast<bf16*>(a.out);
#pragma unroll 1
  for (int it = 0; it < ITEMS; ++it) {
    const int p = tid / NV + it * (512 / NV);                    // output pixel in the tile
    const int oy = p / PW_TW, ox = p - oy * PW_TW;
    const int y = ty0 + oy, x = tx0 + ox;
    float d1[8], d2[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { d1[e] = e_db[cv * 8 + e]; d2[e] = GATE ? e_db[64 + cv * 8 + e] : 0.f; }
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int hr = (oy + tap / 3) * PW_HW + ox + tap % 3;
      const char* hp = sH + hr * PW_HROW;
      Vec<bf16> v1; v1.load(reinterpret_cast<const bf16*>(hp + cv * 16));
      const float* w1 = e_w + tap * PW_NC + cv * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) d1[e] = fmaf(w1[e], v1.v[e], d1[e]);
      if constexpr (GATE) {
        Vec<bf16> v2; v2.load(reinterpret_cast<const bf16*>(hp + 128 + cv * 16));
#pragma unroll
        for (int e = 0; e < 8; ++e) d2[e] = fmaf(w1[64 + e], v2.v[e], d2[e]);
      }
    }
    if (y < a.H && x < a.W) {
      Vec<bf16> o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o.v[e] = GATE ? gelu_bf16(d1[e]) * d2[e] : d1[e];
      const int oc = GATE ? sl * 64 + cv * 8 : sl * 128 + cv * 8;
      o.store(out + (((int64_t)img * a.H + y) * a.W + x) * a.ldo + a.offo + oc);
    }
  }
}

bool pwdw_ok(const PwdwArgs& a) {
  const int hid = a.gate ? a.N1 / 2 : a.N1;
  return a.C % 64 == 0 && a.ldx % 8 == 0 && a.offx % 8 == 0 && a.ldo % 8 == 0 && a.offo % 8 == 0 &&
         (a.gate ? hid % 64 == 0 : hid % 128 == 0) && a.N1 > 0;
}

void launch_pwdw(const PwdwArgs& a, hipStream_t st) {
  const int hid = a.gate ? a.N1 / 2 : a.N1;
  const int nsl = a.gate ? hid / 64 : hid / 128;
  const int64_t blocks = (int64_t)a.nimg * ((a.H + PW_TH - 1) / PW_TH) * ((a.W + PW_TW - 1) / PW_TW) * nsl;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&pwdw_kernel<0>), hipFuncAttributeMaxDynamicSharedMemorySize, PW_BYTES);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&pwdw_kernel<1>), hipFuncAttributeMaxDynamicSharedMemorySize, PW_BYTES);
    attr = true;
  }
  if (a.gate) hipLaunchKernelGGL(pwdw_kernel<1>, dim3((unsigned)blocks), dim3(512), PW_BYTES, st, a);
  else hipLaunchKernelGGL(pwdw_kernel<0>, dim3((unsigned)blocks), dim3(512), PW_BYTES, st, a);
}

}  // namespace turtle

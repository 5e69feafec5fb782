// Check + microbenchmark of the fused project_in -> depthwise -> gate kernel (pdw.hip) on the
// level-3 GatedFeedForward shape (GPU box, no Python).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I turtlevsr_amd/csrc tools/pdbench.cpp -L turtlevsr_amd/lib -lturtle_hip \
//         -Wl,-rpath,$PWD/turtlevsr_amd/lib -o tools/pdbench
//   ./tools/pdbench [reps] [H] [W]
// Compares sampled output pixels with a host reference (LayerNorm two-pass in fp32, the normalised
// row rounded to bf16 as the kernel's operand, project_in in fp64, hidden rounded to bf16, depthwise
// + bias, tanh-form GELU gate) and prints the average launch time of both schedule variants.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kernels.h"

using namespace turtle;

#define CK(x)                                                                                      \
  do {                                                                                             \
    hipError_t e = (x);                                                                            \
    if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); }   \
  } while (0)

static uint16_t f2bf(float f) {
  uint32_t u; memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
static float bf2f(uint16_t b) { uint32_t u = (uint32_t)b << 16; float f; memcpy(&f, &u, 4); return f; }
static float bfr(float f) { return bf2f(f2bf(f)); }
static float frand() { return (float)rand() / (float)RAND_MAX * 2.f - 1.f; }
static float gelu_tanh_h(float x) { return x / (1.f + std::exp2(x * (-0.10294324f * x * x - 2.3022082f))); }

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const int H = argc > 2 ? atoi(argv[2]) : 272, W = argc > 3 ? atoi(argv[3]) : 480;
  const int C = 256, hd = 640, N1 = 2 * hd;
  const int64_t P = (int64_t)H * W;
  srand(7);
  std::vector<uint16_t> x(P * C), w1((size_t)N1 * C), taps(9 * N1);
  std::vector<float> tb(N1), dwb(N1);
  for (auto& v : x) v = f2bf(frand() * 2.f + 0.3f);
  for (auto& v : w1) v = f2bf(frand() * 0.08f);
  for (auto& v : taps) v = f2bf(frand() * 0.3f);
  for (auto& v : tb) v = frand() * 0.2f;
  for (auto& v : dwb) v = frand() * 0.1f;
  void *dx, *dw1, *dt, *dout; float *dtb, *ddb, *ds;
  CK(hipMalloc(&dx, x.size() * 2)); CK(hipMalloc(&dw1, w1.size() * 2)); CK(hipMalloc(&dt, taps.size() * 2));
  CK(hipMalloc(&dtb, N1 * 4)); CK(hipMalloc(&ddb, N1 * 4)); CK(hipMalloc(&ds, N1 * 4));
  CK(hipMalloc(&dout, P * hd * 2 + 512));
  CK(hipMemcpy(dx, x.data(), x.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dw1, w1.data(), w1.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dt, taps.data(), taps.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dtb, tb.data(), N1 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(ddb, dwb.data(), N1 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(ds, tb.data(), N1 * 4, hipMemcpyHostToDevice));   // any non-null rowsum: WithBias path
  PdwArgs a{};
  a.x = dx; a.ldx = C; a.offx = 0; a.C = C; a.nimg = 1; a.H = H; a.W = W;
  a.w1 = dw1; a.N1 = N1; a.ln = 1; a.ln_s = ds; a.ln_tb = dtb; a.dww16 = dt; a.dwb = ddb;
  a.out = dout; a.ldo = hd; a.offo = 0; a.pad_off = P * hd * 2; a.split = 1;
  if (!pdw_ok(a)) { printf("pdw_ok false\n"); return 1; }
  std::vector<uint16_t> out(P * hd);
  for (int split : {1}) {
    a.split = split;
    CK(hipMemset(dout, 0, P * hd * 2));
    launch_pdw(a, 0);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(out.data(), dout, P * hd * 2, hipMemcpyDeviceToHost));
    // host reference at sampled pixels (corners, edges, interior)
    double maxerr = 0, maxref = 0;
    int bad = 0, first_bad_ch = -1, first_bad_px = -1;
    std::vector<float> xn(C);
    auto hidden = [&](int yy, int xx, int ch) -> float {   // bf16-rounded H at (yy, xx), 0 outside
      if (yy < 0 || yy >= H || xx < 0 || xx >= W) return 0.f;
      const uint16_t* xp = &x[((int64_t)yy * W + xx) * C];
      double s = 0; for (int c = 0; c < C; ++c) s += bf2f(xp[c]);
      const float mu = (float)(s / C);
      double v = 0; for (int c = 0; c < C; ++c) { const double d = bf2f(xp[c]) - mu; v += d * d; }
      const float r = 1.f / std::sqrt((float)(v / C) + 1e-5f);
      double acc = 0;
      for (int c = 0; c < C; ++c) acc += (double)bf2f(w1[(size_t)ch * C + c]) * bfr((bf2f(xp[c]) - mu) * r);
      return bfr((float)acc + tb[ch]);
    };
    const int ys[] = {0, 1, 7, 8, H / 2, H - 2, H - 1}, xs[] = {0, 1, 31, 32, 33, W / 2, W - 2, W - 1};
    std::vector<int> chs;
    for (int st = 0; st < hd / 16; ++st) { chs.push_back(16 * st); chs.push_back(16 * st + 7); chs.push_back(16 * st + 15); }
    std::vector<int> bad_ch(hd, 0);
    for (int yy : ys)
      for (int xx : xs)
        for (int j : chs) {
          double d1 = dwb[j], d2 = dwb[hd + j];
          for (int t = 0; t < 9; ++t) {
            const int sy = yy + t / 3 - 1, sx = xx + t % 3 - 1;
            d1 += (double)bf2f(taps[t * N1 + j]) * hidden(sy, sx, j);
            d2 += (double)bf2f(taps[t * N1 + hd + j]) * hidden(sy, sx, hd + j);
          }
          const float ref = gelu_tanh_h((float)d1) * (float)d2;
          const float got = bf2f(out[((int64_t)yy * W + xx) * hd + j]);
          const double err = std::fabs(got - ref);
          maxerr = std::max(maxerr, err);
          maxref = std::max(maxref, (double)std::fabs(ref));
          if (err > 0.02 * std::fabs(ref) + 0.02) {
            if (bad < 8) printf("  split %d mismatch y %d x %d ch %d: got %f ref %f\n", split, yy, xx, j, got, ref);
            if (first_bad_ch < 0) { first_bad_ch = j; first_bad_px = yy * W + xx; }
            ++bad; ++bad_ch[j];
          }
        }
    printf("split %d: max |err| %.5f (max |ref| %.3f), %d bad samples; bad channels:", split, maxerr, maxref, bad);
    for (int j = 0; j < hd; ++j) if (bad_ch[j]) printf(" %d(%d)", j, bad_ch[j]);
    printf("\n");
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    launch_pdw(a, 0);
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch_pdw(a, 0);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms = 0; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("split %d: %.1f us per launch (%dx%d, %lld blocks)\n", split, 1e3 * ms / reps, H, W, (long long)pdw_blocks(a));
  }
  return 0;
}

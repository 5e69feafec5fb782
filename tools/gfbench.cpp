// Check + microbenchmark of the fused level-3 GatedFeedForward kernel (gffn.hip), GPU box, no Python:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DTURTLE_GFFN_ABLATIONS -I turtlevsr_amd/csrc \
//         tools/gfbench.cpp turtlevsr_amd/csrc/gffn.hip -o tools/gfbench
//   ./tools/gfbench [reps] [abl]
// 1. correctness: small ragged shapes (2 images, image borders inside tiles) against a double-precision
//    host evaluation of the block (turtle_t1_arch.py:159-178 after LayerNorm 83-112) on the same bf16
//    input; prints max |err| and RMS(err) / RMS(ffn) (f16 operands: ~1e-3 expected), exits 1 above 1e-2
// 2. timing: the 1080p level-3 shape (272 x 480, hd 640), HIP events, optional ablations
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kernels.h"

using namespace turtle;

#define CK(x)                                                                                         \
  do {                                                                                                \
    hipError_t e = (x);                                                                               \
    if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); }      \
  } while (0)

namespace turtle {
[[noreturn]] void kernel_arg_error(const char* what) { printf("kernel_arg_error: %s\n", what); exit(1); }
}

static uint16_t f2bf(float f) {
  uint32_t u; memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
static float bf2f(uint16_t b) { uint32_t u = (uint32_t)b << 16; float f; memcpy(&f, &u, 4); return f; }
static double frand() { return (double)rand() / (double)RAND_MAX * 2.0 - 1.0; }

struct Model {
  int hd;
  std::vector<double> w1, g, bln, b1, dw9, dwb, w2, b2;
  std::vector<double> w1f, tb;   // folded
  GffnHost hp;
  void *dw1f = nullptr, *dtbp = nullptr, *ddwp = nullptr, *dw2f = nullptr, *db2 = nullptr;
  void init(int hd_) {
    hd = hd_;
    const int C = 256, H2 = 2 * hd;
    w1.resize((size_t)H2 * C); g.resize(C); bln.resize(C); b1.resize(H2); dw9.resize((size_t)9 * H2); dwb.resize(H2);
    w2.resize((size_t)C * hd); b2.resize(C);
    for (auto& v : w1) v = frand() / 16.0;
    for (auto& v : g) v = 1.0 + 0.2 * frand();
    for (auto& v : bln) v = 0.1 * frand();
    for (auto& v : b1) v = 0.1 * frand();
    for (auto& v : dw9) v = frand() / 3.0;
    for (auto& v : dwb) v = 0.1 * frand();
    for (auto& v : w2) v = 8.0 * frand() / std::sqrt((double)hd);
    for (auto& v : b2) v = 0.1 * frand();
    w1f = w1; tb.assign(H2, 0.0);
    for (int n = 0; n < H2; ++n) {
      double t = b1[n];
      for (int k = 0; k < C; ++k) { w1f[(size_t)n * C + k] = w1[(size_t)n * C + k] * g[k]; t += w1[(size_t)n * C + k] * bln[k]; }
      tb[n] = t;
    }
    gffn_pack(256, hd, w1f, tb, dw9, dwb, w2, hp);
    CK(hipMalloc(&dw1f, hp.w1f.size() * 2)); CK(hipMalloc(&dw2f, hp.w2f.size() * 2));
    CK(hipMalloc(&dtbp, hp.tbp.size() * 4)); CK(hipMalloc(&ddwp, hp.dwp.size() * 4)); CK(hipMalloc(&db2, C * 4));
    CK(hipMemcpy(dw1f, hp.w1f.data(), hp.w1f.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw2f, hp.w2f.data(), hp.w2f.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dtbp, hp.tbp.data(), hp.tbp.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(ddwp, hp.dwp.data(), hp.dwp.size() * 4, hipMemcpyHostToDevice));
    std::vector<float> fb(b2.begin(), b2.end());
    CK(hipMemcpy(db2, fb.data(), C * 4, hipMemcpyHostToDevice));
  }
  GffnArgs args(void* x, void* out, int nimg, int H, int W) const {
    GffnArgs a{};
    a.x = x; a.out = out; a.nimg = nimg; a.H = H; a.W = W; a.hd = hd; a.C = 256; a.centred = 1;
    a.w1f = dw1f; a.tbp = (const float*)dtbp; a.dwp = (const uint32_t*)ddwp; a.w2f = dw2f; a.b2 = (const float*)db2;
    return a;
  }
  // reference: x + project_out(gelu(dw(h1)) * dw(h2)) + b2 with h = W1 LN(x) + b1 (exact erf GELU)
  void ref(const std::vector<uint16_t>& x, int nimg, int H, int W, std::vector<double>& out) const {
    const int C = 256, H2 = 2 * hd;
    const size_t P = (size_t)nimg * H * W;
    std::vector<double> h(P * H2), gt(P * hd);
    for (size_t p = 0; p < P; ++p) {
      double mu = 0, var = 0, xn[256];
      for (int k = 0; k < C; ++k) mu += bf2f(x[p * C + k]);
      mu /= C;
      for (int k = 0; k < C; ++k) { const double d = bf2f(x[p * C + k]) - mu; var += d * d; }
      var /= C;
      const double rs = 1.0 / std::sqrt(var + 1e-5);
      for (int k = 0; k < C; ++k) xn[k] = (bf2f(x[p * C + k]) - mu) * rs * g[k] + bln[k];
      for (int n = 0; n < H2; ++n) {
        double s = b1[n];
        const double* wr = &w1[(size_t)n * C];
        for (int k = 0; k < C; ++k) s += wr[k] * xn[k];
        h[p * H2 + n] = s;
      }
    }
    for (int im = 0; im < nimg; ++im)
      for (int y = 0; y < H; ++y)
        for (int xx = 0; xx < W; ++xx) {
          const size_t p = ((size_t)im * H + y) * W + xx;
          for (int cc = 0; cc < hd; ++cc) {
            double d1 = dwb[cc], d2 = dwb[hd + cc];
            for (int ky = 0; ky < 3; ++ky)
              for (int kx = 0; kx < 3; ++kx) {
                const int yy = y + ky - 1, xs = xx + kx - 1;
                if (yy < 0 || yy >= H || xs < 0 || xs >= W) continue;
                const size_t q = ((size_t)im * H + yy) * W + xs;
                d1 += dw9[(size_t)(ky * 3 + kx) * H2 + cc] * h[q * H2 + cc];
                d2 += dw9[(size_t)(ky * 3 + kx) * H2 + hd + cc] * h[q * H2 + hd + cc];
              }
            gt[p * hd + cc] = 0.5 * d1 * (1.0 + std::erf(d1 / std::sqrt(2.0))) * d2;
          }
        }
    out.assign(P * C, 0.0);
    for (size_t p = 0; p < P; ++p)
      for (int o = 0; o < C; ++o) {
        double s = b2[o];
        const double* wr = &w2[(size_t)o * hd];
        for (int k = 0; k < hd; ++k) s += wr[k] * gt[p * hd + k];
        out[p * C + o] = s;   // the FFN part; the residual is added by the caller
      }
  }
};

template <typename F>
static float time_it(F&& f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / reps;
}

static int check(int hd, int nimg, int H, int W) {
  Model m; m.init(hd);
  const int C = 256;
  const size_t P = (size_t)nimg * H * W;
  std::vector<uint16_t> hx(P * C), ho(P * C);
  for (auto& v : hx) v = f2bf((float)(frand() * 0.02 + 0.003));   // small x: the bf16 output rounding stays below the FFN's
  void *dx, *dout;
  CK(hipMalloc(&dx, hx.size() * 2)); CK(hipMalloc(&dout, hx.size() * 2));
  CK(hipMemcpy(dx, hx.data(), hx.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemset(dout, 0xff, hx.size() * 2));
  launch_gffn(m.args(dx, dout, nimg, H, W), 0);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(ho.data(), dout, ho.size() * 2, hipMemcpyDeviceToHost));
  std::vector<double> ref;
  m.ref(hx, nimg, H, W, ref);
  double maxe = 0, se = 0, sr = 0;
  for (size_t i = 0; i < ho.size(); ++i) {
    const double got = bf2f(ho[i]) - bf2f(hx[i]);   // the FFN part as the kernel delivered it (bf16 output)
    const double e = std::fabs(got - ref[i]);
    if (!(e <= maxe)) maxe = e;   // NaN-propagating
    se += e * e; sr += ref[i] * ref[i];
  }
  const double rel = std::sqrt(se / sr);
  printf("check hd=%d nimg=%d %dx%d: max|err| %.3e  rms(err)/rms(ffn) %.3e  rms(ffn) %.3e\n", hd, nimg, H, W, maxe, rel,
         std::sqrt(sr / ho.size()));
  CK(hipFree(dx)); CK(hipFree(dout));
  return (rel < 1e-2 && maxe == maxe) ? 0 : 1;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const bool abl = argc > 2 && !strcmp(argv[2], "abl");
  const bool prof = argc > 2 && !strcmp(argv[2], "prof");   // counter passes: the timed shape only
  int bad = 0;
  if (!prof) {
    bad |= check(128, 2, 19, 33);
    bad |= check(640, 1, 16, 28);
    bad |= check(64, 1, 5, 9);
  }
  if (bad) { printf("CHECK FAILED\n"); return 1; }
  Model m; m.init(640);
  const int H = 272, W = 480, C = 256;
  const size_t P = (size_t)H * W;
  std::vector<uint16_t> hx(P * C);
  for (auto& v : hx) v = f2bf((float)frand());
  void *dx, *dout;
  CK(hipMalloc(&dx, hx.size() * 2)); CK(hipMalloc(&dout, hx.size() * 2));
  CK(hipMemcpy(dx, hx.data(), hx.size() * 2, hipMemcpyHostToDevice));
  GffnArgs a = m.args(dx, dout, 1, H, W);
  const double flops = 2.0 * P * (C * 2.0 * 640 + 640.0 * C) + 18.0 * P * 1280, bytes = 2.0 * P * 2 * C;
  const int dbgs[] = {0, 1, 2, 4, 5, 7, 8, 15, 16, 31};
  for (int d : dbgs) {
    if (d && !abl) break;
    a.dbg = d;
    const float us = time_it([&] { launch_gffn(a, 0); }, reps);
    printf("L3 gffn 272x480 hd=640 dbg=%d  %8.1f us  %7.1f TF/s (algorithmic)  %7.1f GB/s  blocks %lld\n", d, us,
           flops / us * 1e-6, bytes / us * 1e-3, (long long)gffn_blocks(a));
  }
  return 0;
}

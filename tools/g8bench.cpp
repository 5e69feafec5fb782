// Microbenchmark of the 256 x 256 four-phase GEMM (gemm8.hip) against the 2-D tiled kernel (gemm5.hip,
// the parity reference here) and hipBLASLt on the Turtle projection shapes (GPU box, no Python).
//   hipcc -O3 --offload-arch=gfx950 -I turtlevsr_amd/csrc tools/g8bench.cpp tools/blas_ref.cpp -L turtlevsr_amd/lib -lturtle_hip -lhipblaslt \
//         -Wl,-rpath,'$ORIGIN/../turtlevsr_amd/lib' -o tools/g8bench
//   ./g8bench [reps]
// Per shape: max |g8 - kt| over the output, and a race screen - the g8 output of every timed launch
// must equal the first one bit for bit (reps launches, compared after each batch).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kernels.h"
#include "blas_ref.h"

using namespace turtle;

#ifdef TURTLE_G8_ABLATIONS
namespace turtle { void launch_gemm8_dbg(const GemmArgs& g, int dbg, hipStream_t st); }
#endif

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } \
  } while (0)

static uint16_t f2bf(float f) {
  uint32_t u; memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
static float bf2f(uint16_t b) { uint32_t u = (uint32_t)b << 16; float f; memcpy(&f, &u, 4); return f; }

struct Shape { int64_t M; int N, K; int ln, res, gelu; const char* tag; int nsrc = 1, hw = 0, conv3 = 0, Wimg = 1, store = 0; };

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const bool abl = argc > 2 && !strcmp(argv[2], "abl");   // ablation table (built with -DTURTLE_G8_ABLATIONS)
  const Shape shapes[] = {
      {32640, 2560, 512, 1, 0, 0, "latent GFFW project_in"},
      {32640, 1536, 512, 1, 0, 0, "latent qkv"},
      {32640, 512, 1280, 0, 1, 0, "latent project_out"},
      {32640, 512, 512, 0, 1, 0, "latent W_eff"},
      {32640, 512, 2048, 0, 1, 0, "latent 2src K=2048", 2},
      {130560, 1280, 256, 1, 0, 0, "L3 GFFW project_in"},
      {130560, 768, 256, 1, 0, 0, "L3 qkv"},
      {130560, 256, 640, 0, 1, 0, "L3 GFFW project_out"},
      {130560, 256, 256, 0, 1, 0, "L3 W_eff"},
      {130560, 256, 1280, 0, 1, 0, "L3 CHM FHR W_eff 5src", 5},
      {522240, 256, 128, 1, 0, 1, "L2 FFW conv4"},
      {522240, 128, 256, 0, 1, 0, "L2 FFW conv5"},
      {522240, 512, 256, 0, 0, 0, "L2 512 K=256"},
      {2088960, 64, 256, 0, 1, 0, "L1 64 K=256 4src", 4},
      {8160, 512, 512, 0, 1, 0, "small W_eff 8160", 1, 0},
      {2 * 32640, 512, 512, 0, 1, 0, "W_eff per-image x2", 1, 32640},
      {1000, 264, 200, 1, 1, 1, "ragged M N K"},
      {130560, 512, 2304, 0, 0, 0, "L3 up conv3 shuffle", 1, 0, 1, 480, 1},
      {522240, 256, 1152, 0, 0, 0, "L2 down conv3 unshuf", 1, 0, 1, 960, 2},
      {32640, 1024, 4608, 0, 0, 0, "latent up conv3 shuffle", 1, 0, 1, 240, 1},
      {130560, 256, 1152, 0, 1, 0, "L3 conv3 res NHWC", 1, 0, 1, 480, 0},
  };
  size_t maxA = 0, maxW = 0, maxO = 0;
  for (auto& s : shapes) {
    maxA = std::max(maxA, (size_t)s.M * s.K);
    maxW = std::max(maxW, (size_t)s.N * s.K * 2);
    maxO = std::max(maxO, (size_t)s.M * s.N);
  }
  std::vector<uint16_t> h(std::max(maxA, maxO));
  srand(1);
  for (auto& x : h) x = f2bf((rand() / (float)RAND_MAX - 0.5f) * 2.f + 0.3f);
  void *A, *Wt, *R, *Okt, *Og8, *Og8b, *Obl, *XN;
  float *vec, *zeros, *ones;
  CK(hipMalloc(&A, maxA * 2 + 4096));
  CK(hipMalloc(&Wt, maxW * 2));
  CK(hipMalloc(&R, maxO * 2));
  CK(hipMalloc(&Okt, maxO * 2));
  CK(hipMalloc(&Og8, maxO * 2));
  CK(hipMalloc(&Og8b, maxO * 2));
  CK(hipMalloc(&Obl, maxO * 2));
  CK(hipMalloc(&XN, maxA * 2));
  CK(hipMemcpy(A, h.data(), maxA * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(R, h.data(), maxO * 2, hipMemcpyHostToDevice));
  std::vector<uint16_t> hw(maxW);
  for (auto& x : hw) x = f2bf((rand() / (float)RAND_MAX - 0.5f) * 0.1f);
  CK(hipMemcpy(Wt, hw.data(), maxW * 2, hipMemcpyHostToDevice));
  std::vector<float> hv(16384);
  for (auto& x : hv) x = rand() / (float)RAND_MAX - 0.5f;
  CK(hipMalloc(&vec, 16384 * 4));
  CK(hipMemcpy(vec, hv.data(), 16384 * 4, hipMemcpyHostToDevice));
  std::vector<float> z(16384, 0.f), o(16384, 1.f);
  CK(hipMalloc(&zeros, 16384 * 4));
  CK(hipMalloc(&ones, 16384 * 4));
  CK(hipMemcpy(zeros, z.data(), 16384 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(ones, o.data(), 16384 * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  BlasCtx* blas = blas_create();
  std::vector<uint16_t> r1(maxO), r2(maxO);
  int bad = 0;
  printf("%-26s %8s %5s %5s | %8s %7s %6s | %8s %7s %6s | %8s %7s | %8s %7s | %9s %s\n", "shape", "M", "N", "K", "g8 us", "TF/s", "GB/s",
         "g8p us", "TF/s", "GB/s", "kt us", "TF/s", "blas us", "TF/s", "max|d|", "race g8/g8p");
  for (auto& s : shapes) {
    GemmArgs g{};
    g.a.n = s.nsrc; g.a.Ktot = s.K;
    const int kin = s.K / s.nsrc;
    for (int j = 0; j < s.nsrc; ++j) g.a.s[j] = SrcDesc{(char*)A + (size_t)j * 128, kin + 64, 0, kin, 1, 0};
    if (s.nsrc == 1) g.a.s[0].ld = s.K;
    if (s.conv3) g.a.s[0] = SrcDesc{A, s.K / 9, 0, s.K, 1, 0};
    g.conv3 = s.conv3; g.cin = s.K / 9;
    g.M = s.M; g.N = s.N; g.HW = s.hw ? s.hw : (int)s.M; g.Wimg = s.Wimg;
    g.w = Wt; g.ldw = s.K; g.wdiv = 1; g.wstride = s.hw ? (int64_t)s.N * s.K : 0;
    if (s.ln) {
      std::vector<float> rs(s.N, 0.f);
      for (int n = 0; n < s.N; ++n)
        for (int k = 0; k < s.K; ++k) rs[n] += bf2f(hw[(size_t)n * s.K + k]);
      CK(hipMemcpy(vec, rs.data(), s.N * 4, hipMemcpyHostToDevice));
    }
    g.ln = s.ln; g.ln_s = s.ln ? vec : nullptr; g.ln_t = s.ln ? vec + 4096 : nullptr;
    g.bias = vec + 8192; g.scale = nullptr; g.gelu = s.gelu;
    g.res = s.res ? R : nullptr; g.ldr = s.N; g.offr = 0;
    g.ldo = s.store == STORE_UNSHUFFLE ? s.N * 4 : (s.store == STORE_SHUFFLE ? s.N / 4 : s.N); g.offo = 0; g.store_mode = s.store;
    g.zeros = zeros; g.ones = ones;
    const size_t n = (size_t)s.M * s.N;
    double us[4] = {0, 0, 0, 0};
    GemmArgs gk = g; gk.allow_kt = 1; gk.dbg = 0x10; gk.out = Okt;
    GemmArgs g8 = g; g8.allow_g8 = 1; g8.out = Og8;
    if (!gemm8_ok(g8)) { printf("%-26s not eligible\n", s.tag); continue; }
    const bool kt_ok = gemm_kt_ok(gk);
    const bool bl_ok = blas && s.nsrc == 1 && !s.gelu && !s.hw && !s.conv3 &&
                       blas_ready(blas, s.M, s.N, s.K, s.K, s.K, s.res ? s.N : 0, s.N, s.res != 0, true);
    LnRowsArgs la{A, s.K, 0, XN, s.K, s.M, s.K, 1};
    GemmArgs g8p = g8; g8p.allow_g8 = 2; g8p.out = Og8b;
#ifdef TURTLE_G8_ABLATIONS
    if (abl) {                     // 1 no MFMA, 2 no DMA, 4 no fragment reads, 8 no barriers, 16 no stores
      if (s.conv3 || s.hw || s.nsrc > 1 || s.M < 30000) continue;
      printf("%-26s", s.tag);
      for (int dbg : {0, 1, 2, 4, 8, 16, 32, 64, 96, 33, 34, 38, 46, 39, 47, 6, 14, 7}) {
        launch_gemm8_dbg(g8, dbg, 0);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < reps; ++i) launch_gemm8_dbg(g8, dbg, 0);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf(" d%d=%.1f", dbg, ms * 1e3 / reps);
      }
      printf("\n");
      fflush(stdout);
      continue;
    }
#endif
    for (int v = 0; v < 4; ++v) {
      if ((v == 1 && !kt_ok) || (v == 2 && !bl_ok)) continue;
      auto run = [&] {
        if (v == 0) launch_gemm8(g8, 0);
        else if (v == 3) launch_gemm8(g8p, 0);
        else if (v == 1) launch_gemm_kt(gk, 0);
        else {
          if (s.ln) launch_ln_rows<bf16>(la, 0);
          blas_gemm_bf16(blas, s.M, s.N, s.K, s.ln ? XN : A, s.K, Wt, s.K, vec + 8192, s.res ? R : nullptr, s.N, Obl, s.N, 0);
        }
      };
      run();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < reps; ++i) run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      us[v] = ms * 1e3 / reps;
    }
    // race screen: the g8 output of the first launch against fresh launches of g8 and of the
    // persistent g8p (same arithmetic order: bit-identical), 8 rounds each
    CK(hipMemcpy(r1.data(), Og8, n * 2, hipMemcpyDeviceToHost));
    int races = 0, races_p = 0;
    GemmArgs g8b = g8; g8b.out = Og8b;
    for (int it = 0; it < 16; ++it) {
      CK(hipMemset(Og8b, 0xff, n * 2));
      for (int i = 0; i < 2; ++i) launch_gemm8(it & 1 ? g8p : g8b, 0);
      CK(hipMemcpy(r2.data(), Og8b, n * 2, hipMemcpyDeviceToHost));
      if (memcmp(r1.data(), r2.data(), n * 2)) ++(it & 1 ? races_p : races);
    }
    double md = -1;
    if (kt_ok) {
      CK(hipMemcpy(r2.data(), Okt, n * 2, hipMemcpyDeviceToHost));
      md = 0;
      for (size_t i = 0; i < n; ++i) {
        const double d = fabs((double)bf2f(r1[i]) - bf2f(r2[i]));
        md = std::max(md, std::isnan(d) ? 1e30 : d);
      }
    }
    const double fl = 2.0 * s.M * s.N * s.K, by = 2.0 * ((double)s.M * s.K + (double)s.N * s.K + (double)s.M * s.N * (s.res ? 2 : 1));
    printf("%-26s %8lld %5d %5d | %8.1f %7.0f %6.0f | %8.1f %7.0f %6.0f | %8.1f %7.0f | %8.1f %7.0f | %9.4g %d/8 %d/8\n", s.tag, (long long)s.M, s.N,
           s.K, us[0], fl / us[0] / 1e6, by / us[0] / 1e3, us[3], fl / us[3] / 1e6, by / us[3] / 1e3, us[1], us[1] > 0 ? fl / us[1] / 1e6 : 0.0,
           us[2], us[2] > 0 ? fl / us[2] / 1e6 : 0.0, md, races, races_p);
    fflush(stdout);
    if (races || races_p || md > 0.07 || md < 0) ++bad;
  }
  printf("%s\n", bad ? "G8BENCH FAIL" : "G8BENCH OK");
  return bad ? 1 : 0;
}

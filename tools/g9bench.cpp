// Microbenchmark of the 256-pixel-row GEMM (gemm9.hip, BN = 128 and 256 channel tilings) against the 2-D tiled kernel
// (gemm5.hip, the parity reference here) and hipBLASLt on the Turtle projection shapes (GPU box).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DTURTLE_G9_ABLATIONS -I turtlevsr_amd/csrc \
//         tools/g9bench.cpp tools/blas_ref.cpp turtlevsr_amd/csrc/gemm9.hip -L turtlevsr_amd/lib -lturtle_hip -lhipblaslt \
//         -Wl,-rpath,'$ORIGIN/../turtlevsr_amd/lib' -o tools/g9bench
//   ./g9bench [reps] [abl]
// Per shape: max |g9 - kt| (LN shapes: kt on the same folded LN), and a race screen - 8 fresh g9
// launches must equal the first bit for bit. `abl`: the ablation table (DBG bits of gemm9_kernel).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kernels.h"
#include "blas_ref.h"

using namespace turtle;
namespace turtle { void launch_gemm9_dbg(const GemmArgs& g, void* stats, int dbg, hipStream_t st); }

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

struct Shape { int64_t M; int N, K; int ln, res, gelu; const char* tag; int nsrc = 1, hw = 0; };

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const bool abl = argc > 2 && !strcmp(argv[2], "abl");
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
      {2 * 32640, 512, 512, 0, 1, 0, "W_eff per-image x2", 1, 32640},
      {1000, 264, 256, 1, 1, 1, "ragged M N"},
  };
  size_t maxA = 0, maxW = 0, maxO = 0;
  for (auto& s : shapes) {
    maxA = std::max(maxA, (size_t)s.M * s.K + 4096);
    maxW = std::max(maxW, (size_t)s.N * s.K * 2);
    maxO = std::max(maxO, (size_t)s.M * s.N);
  }
  std::vector<uint16_t> h(std::max(maxA, maxO));
  srand(1);
  for (auto& x : h) x = f2bf((rand() / (float)RAND_MAX - 0.5f) * 2.f + 0.3f);
  void *A, *Wt, *R, *Okt, *Og9, *Og9b, *Obl, *XN, *ST;
  float *vec, *zeros, *ones;
  CK(hipMalloc(&A, maxA * 2));
  CK(hipMalloc(&Wt, maxW * 2));
  CK(hipMalloc(&R, maxO * 2));
  CK(hipMalloc(&Okt, maxO * 2));
  CK(hipMalloc(&Og9, maxO * 2));
  CK(hipMalloc(&Og9b, maxO * 2));
  CK(hipMalloc(&Obl, maxO * 2));
  CK(hipMalloc(&XN, maxA * 2));
  CK(hipMalloc(&ST, 3000000 * 8));
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
  if (abl) printf("ablations (us), d<variant><DBG>: DBG 0 full, 1 no MFMA, 2 no global loads, 4 no LDS, 16 no stores, 22\n");
  else
    printf("%-26s %7s %5s %5s | %7s %7s %7s %7s %7s %7s %7s | best g9 | %9s %s\n", "shape (us)", "M", "N", "K", "128r", "256r", "256d4", "128d3",
           "256d3", "kt", "blas", "max|d|", "races");
  for (auto& s : shapes) {
    GemmArgs g{};
    g.a.n = s.nsrc; g.a.Ktot = s.K;
    const int kin = s.K / s.nsrc;
    for (int j = 0; j < s.nsrc; ++j) g.a.s[j] = SrcDesc{(char*)A + (size_t)j * 128, kin + 64, 0, kin, 1, 0};
    if (s.nsrc == 1) g.a.s[0].ld = s.K;
    g.M = s.M; g.N = s.N; g.HW = s.hw ? s.hw : (int)s.M; g.Wimg = 1;
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
    g.ldo = s.N; g.offo = 0; g.store_mode = STORE_NHWC;
    g.zeros = zeros; g.ones = ones;
    const size_t n = (size_t)s.M * s.N;
    GemmArgs gk = g; gk.allow_kt = 1; gk.dbg = 0x10; gk.out = Okt;
    GemmArgs g9 = g; g9.allow_g9 = 3; g9.out = Og9;    // BN = 128
    if (!gemm9_ok(g9)) { printf("%-26s not eligible\n", s.tag); continue; }
    if (abl) {
      if (s.hw || s.M < 30000) continue;
      printf("%-26s", s.tag);
      for (int dbg : {400, 401, 402, 404, 416, 422, 500, 501, 502, 516}) {   // variant * 100 + DBG
        GemmArgs ga = g9; ga.allow_g9 = dbg / 100;
        launch_gemm9_dbg(ga, ST, dbg % 100, 0);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < reps; ++i) launch_gemm9_dbg(ga, ST, dbg % 100, 0);
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
    const bool kt_ok = gemm_kt_ok(gk);
    const bool bl_ok = blas && s.nsrc == 1 && !s.gelu && !s.hw &&
                       blas_ready(blas, s.M, s.N, s.K, s.K, s.K, s.res ? s.N : 0, s.N, s.res != 0, true);
    LnRowsArgs la{A, s.K, 0, XN, s.K, s.M, s.K, 1};
    // variants: g9 allow_g9 = 3 (BN 128 regs), 2 (BN 256 regs), 4 (BN 256 DMA4), 5 (BN 128 DMA3),
    // 6 (BN 256 DMA3); then kt, hipBLASLt. Best of 3 timed batches each.
    const int gv[5] = {3, 2, 4, 5, 6};
    double us[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int v = 0; v < 7; ++v) {
      if ((v == 5 && !kt_ok) || (v == 6 && !bl_ok)) continue;
      GemmArgs gx = g9; if (v < 5) gx.allow_g9 = gv[v];
      auto run = [&] {
        if (v < 5) launch_gemm9(gx, ST, 0);
        else if (v == 5) launch_gemm_kt(gk, 0);
        else {
          if (s.ln) launch_ln_rows<bf16>(la, 0);
          blas_gemm_bf16(blas, s.M, s.N, s.K, s.ln ? XN : A, s.K, Wt, s.K, vec + 8192, s.res ? R : nullptr, s.N, Obl, s.N, 0);
        }
      };
      run();
      CK(hipDeviceSynchronize());
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < reps; ++i) run();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = std::min(best, ms);
      }
      us[v] = best * 1e3 / reps;
    }
    // race / variant screen: every variant's output equals the first launch's bit for bit
    launch_gemm9(g9, ST, 0);
    CK(hipMemcpy(r1.data(), Og9, n * 2, hipMemcpyDeviceToHost));
    int races = 0;
    for (int it = 0; it < 10; ++it) {
      GemmArgs gx = g9; gx.out = Og9b; gx.allow_g9 = gv[it % 5];
      CK(hipMemset(Og9b, 0xff, n * 2));
      launch_gemm9(gx, ST, 0);
      CK(hipMemcpy(r2.data(), Og9b, n * 2, hipMemcpyDeviceToHost));
      if (memcmp(r1.data(), r2.data(), n * 2)) ++races;
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
    const double fl = 2.0 * s.M * s.N * s.K;
    printf("%-26s %7lld %5d %5d |", s.tag, (long long)s.M, s.N, s.K);
    for (int v = 0; v < 7; ++v) printf(" %7.1f", us[v]);
    double bestg = 1e30; for (int v = 0; v < 5; ++v) bestg = std::min(bestg, us[v]);
    printf(" | %6.0f TF/s | %9.4g %d/10\n", fl / bestg / 1e6, md, races);
    fflush(stdout);
    if (races || md > 0.07 || md < 0) ++bad;
  }
  if (!abl) printf("%s\n", bad ? "G9BENCH FAIL" : "G9BENCH OK");
  return bad ? 1 : 0;
}

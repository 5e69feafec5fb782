// fp32 GEMM benchmark (GPU box, no Python): gemm_f32_kernel (gemm_f32.hip) against the
// generic gemm_kernel<float> (gemm.hip) on the GEMM shapes of the 540p fp32 frame (config 3) and
// on ragged / multi-source / per-image / store-remap cases. Prints the average launch time of
// each (HIP events), TF/s, and the max |difference| of the two outputs relative to max |out|.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I turtlevsr_amd/csrc tools/f32bench.cpp \
//     -L turtlevsr_amd/lib -lturtle_hip -Wl,-rpath,'$ORIGIN/../turtlevsr_amd/lib' -o tools/f32bench
//   ./tools/f32bench [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "kernels.h"

using namespace turtle;

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e = (x);                                                                        \
    if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } \
  } while (0)

struct Shape {
  int64_t M; int N, K; int ln, res, gelu; const char* tag;
  int nsrc = 1, conv3 = 0, Wimg = 1, store = 0, nimg = 1, wper = 0, scale = 0;
};

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const Shape shapes[] = {
      {32640, 1280, 256, 1, 0, 0, "L3 GFFW project_in"},
      {32640, 768, 256, 1, 0, 0, "L3 qkv"},
      {8160, 2560, 512, 1, 0, 0, "latent project_in"},
      {32640, 256, 640, 0, 1, 0, "L3 project_out"},
      {130560, 640, 128, 1, 0, 0, "L2 GFFW project_in"},
      {8160, 1536, 512, 1, 0, 0, "latent qkv"},
      {130560, 256, 128, 1, 0, 0, "L2 256 ln"},
      {8160, 512, 1280, 0, 1, 0, "latent project_out"},
      {130560, 128, 256, 0, 1, 0, "L2 128 K=256 res"},
      {522240, 320, 64, 1, 0, 0, "L1 GFFW project_in"},
      {32640, 256, 256, 0, 1, 0, "L3 W_eff"},
      {522240, 128, 64, 1, 0, 0, "L1 128 ln"},
      {522240, 64, 128, 0, 1, 0, "L1 64 res"},
      {130560, 384, 128, 1, 0, 0, "L2 qkv"},
      {130560, 128, 320, 0, 1, 0, "L2 project_out"},
      {130560, 256, 1152, 0, 0, 0, "L2 up conv3 shuffle", 1, 1, 480, STORE_SHUFFLE},
      {32640, 512, 2304, 0, 0, 0, "L3 up conv3 shuffle", 1, 1, 240, STORE_SHUFFLE},
      {522240, 32, 576, 0, 0, 0, "L1 down conv3 unshuf", 1, 1, 960, STORE_UNSHUFFLE},
      {130560, 128, 640, 0, 1, 0, "L2 FHR W_eff 5src", 5},
      {522240, 256, 128, 0, 0, 1, "L1 FFW gelu scale", 1, 0, 1, 0, 1, 0, 1},
      {2 * 16320, 256, 256, 0, 1, 0, "W_eff per-image x2", 1, 0, 1, 0, 2, 1},
      {1000, 36, 48, 1, 1, 1, "ragged M N ln res", 1},
      {999, 200, 96, 0, 1, 0, "ragged 2src", 2},
  };
  size_t maxA = 0, maxW = 0, maxO = 0;
  for (auto& s : shapes) {
    maxA = std::max(maxA, (size_t)s.M * s.K + 1024);
    maxW = std::max(maxW, (size_t)s.N * s.K * 2);
    maxO = std::max(maxO, (size_t)s.M * s.N);
  }
  std::vector<float> h(std::max(maxA, maxO));
  srand(1);
  for (auto& x : h) x = rand() / (float)RAND_MAX - 0.5f;
  float *A, *Wt, *R, *O1, *O2, *O3, *O4, *vec, *zeros, *ones;
  CK(hipMalloc(&A, maxA * 4));
  CK(hipMalloc(&Wt, maxW * 4));
  CK(hipMalloc(&R, maxO * 4));
  CK(hipMalloc(&O1, maxO * 4));
  CK(hipMalloc(&O2, maxO * 4));
  CK(hipMalloc(&O3, maxO * 4));
  CK(hipMalloc(&O4, maxO * 4));
  CK(hipMemcpy(A, h.data(), maxA * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(R, h.data(), maxO * 4, hipMemcpyHostToDevice));
  std::vector<float> hw(maxW);
  for (auto& x : hw) x = (rand() / (float)RAND_MAX - 0.5f) * 0.1f;
  CK(hipMemcpy(Wt, hw.data(), maxW * 4, hipMemcpyHostToDevice));
  std::vector<float> hv(4 * 16384);
  for (auto& x : hv) x = rand() / (float)RAND_MAX - 0.5f;
  CK(hipMalloc(&vec, hv.size() * 4));
  CK(hipMemcpy(vec, hv.data(), hv.size() * 4, hipMemcpyHostToDevice));
  std::vector<float> z(TURTLE_CONST_VEC, 0.f), o(TURTLE_CONST_VEC, 1.f);
  CK(hipMalloc(&zeros, z.size() * 4));
  CK(hipMalloc(&ones, o.size() * 4));
  CK(hipMemcpy(zeros, z.data(), z.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(ones, o.data(), o.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> r1(maxO), r2(maxO);
  printf("%-24s %8s %5s %5s | %9s %7s | %9s %7s | %9s %7s | %9s | %8s | %s\n", "shape", "M", "N", "K", "old us", "TF/s", "f32 us", "TF/s",
         "f32 ns4", "TF/s", "no-load", "speedup", "max|d|/max|out| (ns3, ns4)");
  bool ok_all = true;
  for (auto& s : shapes) {
    GemmArgs g{};
    g.a.n = s.nsrc; g.a.Ktot = s.K;
    const int kin = s.conv3 ? s.K / 9 : s.K / s.nsrc;
    const int64_t HW = s.M / s.nimg;
    for (int j = 0; j < s.nsrc; ++j) g.a.s[j] = SrcDesc{A + (size_t)j * 64, s.conv3 ? kin : s.K, 0, kin, 1, 0};
    g.M = s.M; g.N = s.N; g.HW = (int)HW; g.Wimg = s.Wimg;
    g.conv3 = s.conv3; g.cin = kin; g.store_mode = s.store;
    g.w = Wt; g.ldw = s.K; g.wdiv = 1; g.wstride = s.wper ? (int64_t)s.N * s.K : 0;
    g.ln = s.ln; g.ln_s = s.ln ? vec : nullptr; g.ln_t = s.ln ? vec + 16384 : nullptr;
    g.bias = vec + 2 * 16384; g.scale = s.scale ? vec + 3 * 16384 : nullptr; g.gelu = s.gelu;
    g.res = s.res ? R : nullptr; g.ldr = s.N; g.offr = 0;
    g.ldo = s.store == STORE_UNSHUFFLE ? s.N * 4 : (s.store == STORE_SHUFFLE ? s.N / 4 : s.N); g.offo = 0;
    g.zeros = zeros; g.ones = ones;
    double us[4] = {0, 0, 0, 0};
    bool eligible = true;
    for (int v = 0; v < 4; ++v) {           // 0: gemm_kernel<float>; 1: gemm_f32 3-stage ring; 2: 4-stage ring;
      g.allow_f32 = v > 0;                   // (variants 1-3 launch gemm_f32 directly)
                                             // 3: 3-stage ring without operand loads (timing ablation, output not checked)
      g.dbg = v == 2 ? 1 : (v == 3 ? 2 : 0);
      g.out = v == 0 ? O1 : (v == 1 ? O2 : (v == 2 ? O3 : O4));
      if (v && !gemm_f32_ok(g)) { eligible = false; break; }
      CK(hipMemset(g.out, 0, (size_t)s.M * s.N * 4));
      auto run = [&] { if (v) launch_gemm_f32(g, 0); else launch_gemm<float>(g, 0); };
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
    const double fl = 2.0 * s.M * s.N * s.K;
    if (!eligible) {
      printf("%-24s %8lld %5d %5d | %9.1f %7.1f | not eligible\n", s.tag, (long long)s.M, s.N, s.K, us[0], fl / us[0] / 1e6);
      continue;
    }
    const size_t n = (size_t)s.M * s.N;
    CK(hipMemcpy(r1.data(), O1, n * 4, hipMemcpyDeviceToHost));
    double rel[2];
    bool ok = true;
    for (int v = 0; v < 2; ++v) {
      CK(hipMemcpy(r2.data(), v ? O3 : O2, n * 4, hipMemcpyDeviceToHost));
      double md = 0, mx = 0;
      for (size_t i = 0; i < n; ++i) {
        if (!std::isfinite(r2[i])) ok = false;
        md = std::max(md, (double)fabsf(r1[i] - r2[i]));
        mx = std::max(mx, (double)fabsf(r1[i]));
      }
      rel[v] = md / std::max(mx, 1e-30);
      ok = ok && rel[v] < 1e-5;
    }
    ok_all = ok_all && ok;
    printf("%-24s %8lld %5d %5d | %9.1f %7.1f | %9.1f %7.1f | %9.1f %7.1f | %9.1f | %8.2f | %.3g %.3g%s\n", s.tag, (long long)s.M, s.N, s.K, us[0],
           fl / us[0] / 1e6, us[1], fl / us[1] / 1e6, us[2], fl / us[2] / 1e6, us[3], us[0] / std::min(us[1], us[2]), rel[0], rel[1], ok ? "" : "  MISMATCH");
  }
  printf(ok_all ? "F32BENCH OK\n" : "F32BENCH MISMATCH\n");
  return ok_all ? 0 : 1;
}

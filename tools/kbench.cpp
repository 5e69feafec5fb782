// Kernel microbenchmark for the GEMM variants of libturtle_hip (GPU box, no Python).
//   hipcc -O3 --offload-arch=gfx950 -I turtlevsr_amd/csrc tools/kbench.cpp tools/blas_ref.cpp -L turtlevsr_amd/lib -lturtle_hip -lhipblaslt
//   ./kbench [reps]
// For each Turtle GEMM shape: random bf16 operands, the LDS-pipelined kernel against the panel /
// K-loop kernel (max |diff| over the output), average launch time of each from HIP events.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kernels.h"
#include "blas_ref.h"

using namespace turtle;

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

struct Shape { int64_t M; int N, K; int ln, res, gelu; const char* tag; int nsrc = 1, conv3 = 0, Wimg = 1, store = 0; };

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const int dbg = argc > 2 ? atoi(argv[2]) : 0;     // pn ablation bits: 1 no stores, 2 no W refills, 4 no LDS reads
  const Shape shapes[] = {
      {130560, 1280, 256, 1, 0, 0, "L3 GFFW project_in"},
      {130560, 768, 256, 1, 0, 0, "L3 qkv"},
      {130560, 256, 640, 0, 1, 0, "L3 GFFW project_out"},
      {130560, 256, 256, 0, 1, 0, "L3 W_eff"},
      {130560, 256, 256, 0, 0, 0, "L3 256->256 no res"},
      {32640, 2560, 512, 1, 0, 0, "latent GFFW project_in"},
      {32640, 1536, 512, 1, 0, 0, "latent qkv"},
      {32640, 512, 1280, 0, 1, 0, "latent project_out"},
      {32640, 512, 512, 0, 1, 0, "latent W_eff"},
      {522240, 256, 128, 1, 0, 1, "L2 FFW conv4"},
      {522240, 128, 256, 0, 1, 0, "L2 FFW conv5"},
      {2088960, 128, 64, 1, 0, 1, "L1 FFW conv4"},
      {2088960, 64, 128, 0, 1, 0, "L1 FFW conv5"},
      {130560, 256, 1280, 0, 1, 0, "L3 CHM FHR W_eff 5src", 5},
      {130560, 512, 2304, 0, 0, 0, "L3 up conv3 shuffle", 1, 1, 480, 1},
      {522240, 256, 1152, 0, 0, 0, "L2 down conv3 unshuf", 1, 1, 960, 2},
  };
  size_t maxA = 0, maxW = 0, maxO = 0;
  for (auto& s : shapes) {
    maxA = std::max(maxA, (size_t)s.M * s.K);
    maxW = std::max(maxW, (size_t)s.N * s.K);
    maxO = std::max(maxO, (size_t)s.M * s.N);
  }
  std::vector<uint16_t> h(std::max(maxA, maxO));
  srand(1);
  for (auto& x : h) x = f2bf((rand() / (float)RAND_MAX - 0.5f));
  void *A, *Wt, *R, *O1, *O2, *O3, *O4;
  float *vec, *zeros, *ones;
  CK(hipMalloc(&A, maxA * 2));
  CK(hipMalloc(&Wt, maxW * 2));
  CK(hipMalloc(&R, maxO * 2));
  CK(hipMalloc(&O1, maxO * 2));
  CK(hipMalloc(&O2, maxO * 2));
  CK(hipMalloc(&O3, maxO * 2));
  CK(hipMalloc(&O4, maxO * 2));
  CK(hipMemcpy(A, h.data(), maxA * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(R, h.data(), maxO * 2, hipMemcpyHostToDevice));
  for (size_t i = 0; i < maxW; ++i) h[i] = f2bf((rand() / (float)RAND_MAX - 0.5f) * 0.1f);
  CK(hipMemcpy(Wt, h.data(), maxW * 2, hipMemcpyHostToDevice));
  std::vector<float> hv(16384);
  for (auto& x : hv) x = rand() / (float)RAND_MAX - 0.5f;
  // vec[0..4095] = ln_s: row sums of W (N <= 4096 used with LN), as the model's folded LayerNorm
  std::vector<uint16_t> hw(maxW);
  CK(hipMemcpy(hw.data(), Wt, maxW * 2, hipMemcpyDeviceToHost));
  CK(hipMalloc(&vec, 16384 * 4));
  CK(hipMemcpy(vec, hv.data(), 16384 * 4, hipMemcpyHostToDevice));
  std::vector<float> z(16384, 0.f), o(16384, 1.f);
  CK(hipMalloc(&zeros, 16384 * 4));
  CK(hipMalloc(&ones, 16384 * 4));
  CK(hipMemcpy(zeros, z.data(), 16384 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(ones, o.data(), 16384 * 4, hipMemcpyHostToDevice));
  unsigned long long* stamps = nullptr;
  CK(hipMalloc(&stamps, 2 * 8 * 256 * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<uint16_t> r1(maxO), r2(maxO);
  BlasCtx* blas = blas_create();
  void* XN = nullptr;                 // normalised rows for the hipBLASLt form of an LN GEMM
  CK(hipMalloc(&XN, maxA * 2));
  printf("%-24s %8s %5s %5s | %9s %7s %6s | %9s %7s %6s | %9s %7s %6s | %9s %6s | %9s %6s | %s\n", "shape", "M", "N", "K", "pn us", "TF/s", "GB/s",
         "lds us", "TF/s", "GB/s", "panel us", "TF/s", "GB/s", "ar us", "GB/s", "blas us", "GB/s", "max|d| pn,panel,ar vs lds | kt 256x256 128x256 128x128 us (max|d|)");
  for (auto& s : shapes) {
    GemmArgs g{};
    g.a.n = s.nsrc; g.a.Ktot = s.K;
    const int kin = s.conv3 ? s.K / 9 : s.K / s.nsrc;
    for (int j = 0; j < s.nsrc; ++j) g.a.s[j] = SrcDesc{(char*)A + (size_t)j * 64, s.conv3 ? kin : s.K, 0, kin, 1, 0};
    g.M = s.M; g.N = s.N; g.HW = (int)s.M; g.Wimg = s.Wimg;
    g.conv3 = s.conv3; g.cin = kin; g.store_mode = s.store;
    g.w = Wt; g.ldw = s.K; g.wdiv = 1;
    if (s.ln) {
      std::vector<float> rs(s.N, 0.f);
      for (int n = 0; n < s.N; ++n)
        for (int k = 0; k < s.K; ++k) rs[n] += bf2f(hw[(size_t)n * s.K + k]);
      CK(hipMemcpy(vec, rs.data(), s.N * 4, hipMemcpyHostToDevice));
    }
    g.ln = s.ln; g.ln_s = s.ln ? vec : nullptr; g.ln_t = s.ln ? vec + 4096 : nullptr;
    g.bias = vec + 8192; g.scale = nullptr; g.gelu = s.gelu;
    g.res = s.res ? R : nullptr; g.ldr = s.N; g.offr = 0;
    g.ldo = s.store == STORE_UNSHUFFLE ? s.N * 4 : (s.store == STORE_SHUFFLE ? s.N / 4 : s.N); g.offo = 0;
    g.zeros = zeros; g.ones = ones; g.dbg = dbg;
    double us[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    double md4 = -1, md5[3] = {-1, -1, -1};
    for (int v = 0; v < 8; ++v) {
      g.allow_pn = v == 0;             // variant 0: resident-panel kernel (if eligible); 1: LDS kernel; 2: panel / K-loop
      g.allow_lds = v == 1;            // 3: A-resident kernel (if eligible); 4: hipBLASLt (+ LN rows pass)
      g.allow_panel = v == 2;
      g.allow_ar = v == 3;
      g.allow_kt = v >= 5;             // 5, 6, 7: 2-D tiled kernel at 256 x 256 / 128 x 256 / 128 x 128
      g.dbg = (dbg & 15) | (v == 5 ? 0x10 : v == 6 ? 0x30 : v == 7 ? 0x20 : 0);
      g.out = v == 0 ? O1 : (v == 1 ? O2 : (v == 2 ? O3 : O4));
      if (v == 3 && !gemm_ar_ok(g)) continue;
      if (v >= 5 && !gemm_kt_ok(g)) continue;
      bool blas_ok = false;
      LnRowsArgs la{A, s.K, 0, XN, s.K, s.M, s.K, 1};
      if (v == 4) {
        if (s.nsrc != 1 || s.conv3 || s.gelu || !blas) continue;
        blas_ok = blas_ready(blas, s.M, s.N, s.K, s.K, s.K, s.res ? s.N : 0, s.N, s.res != 0, true);
        if (!blas_ok) continue;
      }
      auto run = [&] {
        if (v < 4) { launch_gemm<bf16>(g, 0); return; }
        if (v >= 5) { launch_gemm_kt(g, 0); return; }
        // LN form: normalised rows, bias = W b_ln + bias (kbench: ln_t + bias vectors as they are)
        if (s.ln) launch_ln_rows<bf16>(la, 0);
        blas_gemm_bf16(blas, s.M, s.N, s.K, s.ln ? XN : A, s.K, Wt, s.K, vec + 8192, s.res ? R : nullptr, s.N, O4, s.N, 0);
      };
      g.stamps = (v == 0 && (dbg & 8) && &s == &shapes[0]) ? stamps : nullptr;
      run();
      CK(hipDeviceSynchronize());
      if (v == 3 || v >= 5) {          // ar / kt output vs the LDS kernel's (O2, variant 1)
        const size_t n = (size_t)s.M * s.N;
        CK(hipMemcpy(r1.data(), O4, n * 2, hipMemcpyDeviceToHost));
        CK(hipMemcpy(r2.data(), O2, n * 2, hipMemcpyDeviceToHost));
        double& md = v == 3 ? md4 : md5[v - 5];
        md = 0;
        for (size_t i = 0; i < n; ++i) md = std::max(md, (double)fabsf(bf2f(r1[i]) - bf2f(r2[i])));
      }
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < reps; ++i) run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      us[v] = ms * 1e3 / reps;
    }
    if ((dbg & 8) && &s == &shapes[0]) {       // s_memtime stamps of block 0, waves 0 and 4 (last launch)
      std::vector<unsigned long long> hs(2 * 8 * 256);
      CK(hipMemcpy(hs.data(), stamps, hs.size() * 8, hipMemcpyDeviceToHost));
      for (int w : {0, 4}) {
        printf("stamps block 0 wave %d (cycles from first):", w);
        const unsigned long long* b = hs.data() + w * 256;
        for (int i = 1; i < 64 && b[i] > b[0] && b[i] - b[0] < (1ull << 32); ++i) printf(" %llu", b[i] - b[i - 1]);
        printf("\n");
      }
      CK(hipMemset(stamps, 0, 2 * 8 * 256 * 8));
    }
    const size_t n = (size_t)s.M * s.N;
    CK(hipMemcpy(r1.data(), O1, n * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r2.data(), O2, n * 2, hipMemcpyDeviceToHost));
    double md = 0, md3 = 0;
    for (size_t i = 0; i < n; ++i) md = std::max(md, (double)fabsf(bf2f(r1[i]) - bf2f(r2[i])));
    CK(hipMemcpy(r1.data(), O3, n * 2, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < n; ++i) md3 = std::max(md3, (double)fabsf(bf2f(r1[i]) - bf2f(r2[i])));
    const double fl = 2.0 * s.M * s.N * s.K, by = 2.0 * ((double)s.M * s.K + (double)s.M * s.N * (s.res ? 2 : 1));
    printf("%-24s %8lld %5d %5d | %9.1f %7.0f %6.0f | %9.1f %7.0f %6.0f | %9.1f %7.0f %6.0f | %9.1f %6.0f | %9.1f %6.0f | %.3g %.3g %.3g | %7.1f %7.1f %7.1f (%.3g %.3g %.3g)%s\n",
           s.tag, (long long)s.M, s.N, s.K, us[0], fl / us[0] / 1e6, by / us[0] / 1e3, us[1], fl / us[1] / 1e6, by / us[1] / 1e3, us[2],
           fl / us[2] / 1e6, by / us[2] / 1e3, us[3], us[3] > 0 ? by / us[3] / 1e3 : 0.0, us[4], us[4] > 0 ? by / us[4] / 1e3 : 0.0,
           md, md3, md4, us[5], us[6], us[7], md5[0], md5[1], md5[2], gemm_pn_ok((g.allow_ar = 0, g.allow_pn = 1, g)) ? "" : "  (pn n/a)");
  }
  return 0;
}

// Microbenchmark of the block-fused pw -> dw -> act -> pw kernel (fused.hip) on the Turtle L1/L2
// shapes, GPU box only:
//   hipcc -O3 --offload-arch=gfx950 -I turtlevsr_amd/csrc tools/fbench.cpp -L turtlevsr_amd/lib -lturtle_hip
//   ./fbench [reps]
// Random bf16 activations / weights; prints the average launch time (HIP events) and the HBM
// bytes / MFMA flops the launch implies, plus a checksum of the output.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kernels.h"

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

struct Shape { int H, W, C, N1, N2, mode; const char* tag; };

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  const int dbg = argc > 2 ? atoi(argv[2]) : 0;   // ablations: 1 no GEMM1 MFMA, 2 no dw, 4 no gelu, 8 no GEMM2 MFMA
  const Shape shapes[] = {
      {1088, 1920, 64, 320, 64, F_GATE, "L1 GFFW (gate)"},
      {1088, 1920, 64, 128, 64, F_GELU, "L1 ReducedAttn (gelu)"},
      {544, 960, 128, 640, 128, F_GATE, "L2 GFFW (gate)"},
      {544, 960, 128, 256, 128, F_GELU, "L2 ReducedAttn (gelu)"},
  };
  const size_t maxX = (size_t)1088 * 1920 * 64;
  std::vector<uint16_t> h(maxX);
  srand(3);
  for (auto& v : h) v = f2bf(rand() / (float)RAND_MAX - 0.5f);
  void *X, *R, *O, *W1, *W2;
  float *vec;
  uint32_t* dww2;
  CK(hipMalloc(&X, maxX * 2));
  CK(hipMalloc(&R, maxX * 2));
  CK(hipMalloc(&O, maxX * 2));
  CK(hipMemcpy(X, h.data(), maxX * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(R, h.data(), maxX * 2, hipMemcpyHostToDevice));
  const size_t maxW = 640 * 128;
  std::vector<uint16_t> hw(maxW);
  for (auto& v : hw) v = f2bf((rand() / (float)RAND_MAX - 0.5f) * 0.1f);
  CK(hipMalloc(&W1, maxW * 2));
  CK(hipMalloc(&W2, maxW * 2));
  CK(hipMemcpy(W1, hw.data(), maxW * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(W2, hw.data(), maxW * 2, hipMemcpyHostToDevice));
  std::vector<float> hv(16384);
  for (auto& v : hv) v = (rand() / (float)RAND_MAX - 0.5f) * 0.2f;
  CK(hipMalloc(&vec, 16384 * 4));
  CK(hipMemcpy(vec, hv.data(), 16384 * 4, hipMemcpyHostToDevice));
  std::vector<uint32_t> h2(5 * 640);
  for (auto& v : h2) v = (uint32_t)f2bf((rand() / (float)RAND_MAX - 0.5f) * 0.3f) | ((uint32_t)f2bf((rand() / (float)RAND_MAX - 0.5f) * 0.3f) << 16);
  CK(hipMalloc(&dww2, 5 * 640 * 4));
  CK(hipMemcpy(dww2, h2.data(), 5 * 640 * 4, hipMemcpyHostToDevice));
  unsigned long long* stamps = nullptr;
  CK(hipMalloc(&stamps, 3 * 4 * 64 * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("%-24s %6s %6s %4s %4s %4s | %9s %7s %7s | %s\n", "shape", "H", "W", "C", "N1", "N2", "us", "GB/s", "TF/s", "checksum");
  for (const Shape& s : shapes) {
    FusedArgs a{};
    a.x = X; a.ldx = s.C; a.offx = 0; a.C = s.C;
    a.nimg = 1; a.H = s.H; a.W = s.W;
    a.w1 = W1; a.N1 = s.N1;
    a.ln = 1; a.ln_s = vec; a.ln_t = vec + 1024; a.b1 = vec + 2048;
    a.dww = vec + 4096; a.dwb = vec + 8192; a.dww2 = dww2;
    a.hidden = s.mode == F_GATE ? s.N1 / 2 : s.N1;
    a.mode = s.mode;
    a.w2 = W2; a.N2 = s.N2; a.b2 = vec + 12288; a.scale2 = vec + 13312;
    a.res = R; a.ldr = s.N2; a.offr = 0;
    a.out = O; a.ldo = s.N2; a.offo = 0;
    a.ndst = 0; a.dbg = dbg; a.stamps = (dbg & 64) ? stamps : nullptr;
    launch_fused<bf16>(a, 0);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) launch_fused<bf16>(a, 0);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    if (dbg & 64) {           // stamps of the last launch: blocks 0, 1, 16000, waves 0-3 (cycles between stamps)
      std::vector<unsigned long long> hs(3 * 4 * 64);
      CK(hipMemcpy(hs.data(), stamps, hs.size() * 8, hipMemcpyDeviceToHost));
      for (int b = 0; b < 3; ++b)
        for (int w = 0; w < 4; w += 3) {
          const unsigned long long* q = hs.data() + (b * 4 + w) * 64;
          printf("  stamps blk %d wave %d:", b, w);
          for (int i = 1; i < 64 && q[i] > q[i - 1] && q[i] - q[0] < (1ull << 32); ++i) printf(" %llu", q[i] - q[i - 1]);
          printf("\n");
        }
      CK(hipMemset(stamps, 0, hs.size() * 8));
    }
    const double px = (double)s.H * s.W;
    const double by = px * 2.0 * (s.C + 2.0 * s.N2);          // x in, residual in, out
    const double fl = px * 2.0 * ((double)s.C * s.N1 + (double)a.hidden * s.N2);
    std::vector<uint16_t> o((size_t)px * s.N2);
    CK(hipMemcpy(o.data(), O, o.size() * 2, hipMemcpyDeviceToHost));
    double cs = 0;
    for (size_t i = 0; i < o.size(); i += 7) cs += bf2f(o[i]);
    printf("%-24s %6d %6d %4d %4d %4d | %9.1f %7.0f %7.0f | %.6g\n", s.tag, s.H, s.W, s.C, s.N1, s.N2, us, by / us / 1e3,
           fl / us / 1e6, cs);
  }
  return 0;
}

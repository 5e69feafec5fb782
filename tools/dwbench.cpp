// Depthwise 3x3 microbenchmark (GPU box, no Python): the launch_dw variants (DwArgs.rows) on the
// Turtle 1080p shapes, bf16. Prints the average launch time (HIP events), the achieved HBM rate on
// the algorithmic bytes (input read once + output written once) and max |diff| vs variant 1.
//   hipcc -O3 --offload-arch=gfx950 -I turtlevsr_amd/csrc tools/dwbench.cpp -L turtlevsr_amd/lib -lturtle_hip -o tools/dwbench
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

struct Shape { int H, W, C, mode; const char* tag; };

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const Shape shapes[] = {
      {272, 480, 640, DW_GATE, "L3 GFFW dw+gate"},
      {272, 480, 768, DW_PLAIN, "L3 qkv dw"},
      {136, 240, 1280, DW_GATE, "L4 GFFW dw+gate"},
      {136, 240, 1536, DW_PLAIN, "L4 qkv dw"},
      {544, 960, 384, DW_PLAIN, "L2 qkv dw"},
  };
  const int variants[] = {1, 3, 0};   // row sweep (default), row sweep with the gate at 4 channels per lane, per-pixel gather
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  srand(1);
  for (const Shape& s : shapes) {
    const int cin = s.mode == DW_GATE ? 2 * s.C : s.C;
    const int64_t px = (int64_t)s.H * s.W;
    std::vector<uint16_t> hx(px * cin);
    for (auto& v : hx) v = f2bf((rand() / (float)RAND_MAX) * 2.f - 1.f);
    std::vector<float> hw(9 * cin), hb(cin);
    for (auto& v : hw) v = (rand() / (float)RAND_MAX - 0.5f) * 0.6f;
    for (auto& v : hb) v = (rand() / (float)RAND_MAX - 0.5f) * 0.2f;
    void *dx, *dy, *dref;
    float *dw, *db;
    CK(hipMalloc(&dx, hx.size() * 2)); CK(hipMalloc(&dy, px * s.C * 2)); CK(hipMalloc(&dref, px * s.C * 2));
    CK(hipMalloc(&dw, hw.size() * 4)); CK(hipMalloc(&db, hb.size() * 4));
    CK(hipMemcpy(dx, hx.data(), hx.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
    DwArgs a{};
    a.in = dx; a.ldi = cin; a.offi = 0; a.ldo = s.C; a.offo = 0; a.w = dw; a.bias = db;
    a.nimg = 1; a.H = s.H; a.W = s.W; a.C = s.C; a.mode = s.mode;
    const double bytes = 2.0 * px * (cin + s.C);
    std::vector<uint16_t> ref(px * s.C), out(px * s.C);
    for (int v : variants) {
      a.rows = v;
      a.out = v == 1 ? dref : dy;
      for (int i = 0; i < 3; ++i) launch_dw<bf16>(a, st);
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < reps; ++i) launch_dw<bf16>(a, st);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / reps;
      float md = 0.f;
      if (v == 1) {
        CK(hipMemcpy(ref.data(), dref, ref.size() * 2, hipMemcpyDeviceToHost));
      } else {
        CK(hipMemcpy(out.data(), dy, out.size() * 2, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < out.size(); ++i) md = fmaxf(md, fabsf(bf2f(out[i]) - bf2f(ref[i])));
      }
      printf("%-18s variant %d: %8.1f us  %7.0f GB/s  maxdiff %.3g\n", s.tag, v, us, bytes / us * 1e-3, md);
      fflush(stdout);
    }
    CK(hipFree(dx)); CK(hipFree(dy)); CK(hipFree(dref)); CK(hipFree(dw)); CK(hipFree(db));
  }
  return 0;
}

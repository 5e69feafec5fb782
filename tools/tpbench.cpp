// Microbenchmark of the tile-resident pointwise -> depthwise (-> gate) kernel (tilepd.hip) on the
// level-3 shapes at 1080p (GPU box, no Python):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I turtlevsr_amd/csrc -I include tools/tpbench.cpp \
//         -L turtlevsr_amd/lib -lturtle_hip -Wl,-rpath,turtlevsr_amd/lib -o tools/tpbench
//   ./tools/tpbench [reps] [only-shape]
// Prints the average launch time (HIP events) of the product kernel and of its ablations (dbg bits:
// 1 no GEMM1, 2 no depthwise / gate, 8 no LayerNorm, 16 no stores - results folded into a checksum).
#include <hip/hip_runtime.h>

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

namespace turtle {
[[noreturn]] void kernel_arg_error(const char* what) { printf("kernel_arg_error: %s\n", what); exit(1); }
}

static uint16_t f2bf(float f) {
  uint32_t u; memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
static float frand() { return (float)rand() / (float)RAND_MAX * 2.f - 1.f; }

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

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const int only = argc > 2 ? atoi(argv[2]) : -1;
  struct S { int H, W, N1, mode; const char* tag; };
  const S shapes[] = {{272, 480, 1280, TP_GATE, "L3 GFFW gate"}, {272, 480, 768, TP_DW, "L3 qkv dw"}};
  for (int si = 0; si < 2; ++si) {
    if (only >= 0 && si != only) continue;
    const S& sh = shapes[si];
    const int C = 256;
    const int64_t P = (int64_t)sh.H * sh.W;
    const int nout = sh.mode == TP_GATE ? sh.N1 / 2 : sh.N1;
    std::vector<uint16_t> hx(P * C), hw((size_t)sh.N1 * C), ht(9 * sh.N1);
    std::vector<float> htb(sh.N1);
    srand(11);
    for (auto& v : hx) v = f2bf(frand());
    for (auto& v : hw) v = f2bf(frand() * 0.06f);
    for (auto& v : ht) v = f2bf(frand() * 0.3f);
    for (auto& v : htb) v = frand() * 0.1f;
    void *dx, *dw, *dt, *dtb, *dout;
    CK(hipMalloc(&dx, hx.size() * 2)); CK(hipMalloc(&dw, hw.size() * 2)); CK(hipMalloc(&dt, ht.size() * 2));
    CK(hipMalloc(&dtb, htb.size() * 4)); CK(hipMalloc(&dout, P * nout * 2));
    CK(hipMemcpy(dx, hx.data(), hx.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw, hw.data(), hw.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dt, ht.data(), ht.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dtb, htb.data(), htb.size() * 4, hipMemcpyHostToDevice));
    TilePdArgs a{};
    a.x = dx; a.ldx = C; a.offx = 0; a.C = C; a.nimg = 1; a.H = sh.H; a.W = sh.W;
    a.w1 = dw; a.N1 = sh.N1; a.ln = 1; a.centred = 1; a.tb = (const float*)dtb; a.dww16 = dt; a.dwb = nullptr;
    a.mode = sh.mode; a.out = dout; a.ldo = nout; a.offo = 0; a.cb_px = sh.mode == TP_GATE ? P : 0;
    const double flops = 2.0 * P * C * sh.N1 + 18.0 * P * sh.N1, bytes = 2.0 * P * (C + nout);
    const int dbgs[] = {0, 1, 2, 8, 3, 16, 17, 18, 19, 24};
    for (int d : dbgs) {
      a.dbg = d;
      const float us = time_it([&] { launch_tilepd(a, 0); }, reps);
      printf("%-14s dbg=%2d  %8.1f us  %7.1f TF/s  %7.1f GB/s  blocks %lld\n", sh.tag, d, us, flops / us * 1e-6,
             bytes / us * 1e-3, (long long)tilepd_blocks(a));
    }
    CK(hipFree(dx)); CK(hipFree(dw)); CK(hipFree(dt)); CK(hipFree(dtb)); CK(hipFree(dout));
  }
  return 0;
}

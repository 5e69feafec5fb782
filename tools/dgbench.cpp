// Microbenchmark of the depthwise-prologue GEMM (dwgemm.hip) against the unfolded dw + GEMM pair,
// on the level-3 / latent GatedFeedForward shapes (GPU box, no Python).
//   hipcc -O3 --offload-arch=gfx950 -I turtlevsr_amd/csrc tools/dgbench.cpp -L turtlevsr_amd/lib -lturtle_hip
//   ./dgbench [reps]
// Prints the average launch time of each (HIP events), the max |diff| between the two outputs, and
// the dwgemm ablations (dbg bits: 1 no depthwise MFMA, 2 no GEMM MFMA, 4 input DMA from the zero
// line, 8 weight DMA from the zero line, 16 no output stores).
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
  const int only = argc > 2 ? atoi(argv[2]) : -1;     // >= 0: that shape only, dwgemm dbg=0 only (PMC passes)
  struct S { int H, W, C, hid; const char* tag; };
  const S shapes[] = {{272, 480, 256, 640, "L3 GFFW"}, {136, 240, 512, 1280, "latent GFFW"}};
  for (int si = 0; si < 2; ++si) {
    if (only >= 0 && si != only) continue;
    const S& sh = shapes[si];
    const int64_t P = (int64_t)sh.H * sh.W;
    const int K = sh.hid, N = sh.C;
    std::vector<uint16_t> hin(P * 2 * K), hw((size_t)N * K), hx(P * N);
    std::vector<float> hdw(9 * 2 * K), hdb(2 * K), hb(N);
    srand(7);
    for (auto& v : hin) v = f2bf(frand());
    for (auto& v : hw) v = f2bf(frand() * 0.05f);
    for (auto& v : hx) v = f2bf(frand());
    for (auto& v : hdw) v = frand() * 0.3f;
    for (auto& v : hdb) v = frand() * 0.1f;
    for (auto& v : hb) v = frand() * 0.1f;
    void *din, *dw2, *dx, *dx2, *dt2; float *ddw, *ddb, *db, *dz;
    CK(hipMalloc(&din, hin.size() * 2)); CK(hipMalloc(&dw2, hw.size() * 2));
    CK(hipMalloc(&dx, hx.size() * 2)); CK(hipMalloc(&dx2, hx.size() * 2)); CK(hipMalloc(&dt2, P * K * 2));
    CK(hipMalloc(&ddw, hdw.size() * 4)); CK(hipMalloc(&ddb, hdb.size() * 4)); CK(hipMalloc(&db, hb.size() * 4));
    float* done;
    CK(hipMalloc(&dz, 65536)); CK(hipMalloc(&done, 65536));
    CK(hipMemset(dz, 0, 65536));
    {
      std::vector<float> ones(16384, 1.f);
      CK(hipMemcpy(done, ones.data(), 65536, hipMemcpyHostToDevice));
    }
    CK(hipMemcpy(din, hin.data(), hin.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw2, hw.data(), hw.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(ddw, hdw.data(), hdw.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(ddb, hdb.data(), hdb.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
    auto reset = [&] {
      CK(hipMemcpy(dx, hx.data(), hx.size() * 2, hipMemcpyHostToDevice));
      CK(hipMemcpy(dx2, hx.data(), hx.size() * 2, hipMemcpyHostToDevice));
    };
    DwGemmArgs a{};
    std::vector<uint16_t> hdw16(hdw.size());
    for (size_t i = 0; i < hdw.size(); ++i) hdw16[i] = f2bf(hdw[i]);
    void* ddw16;
    CK(hipMalloc(&ddw16, hdw16.size() * 2));
    CK(hipMemcpy(ddw16, hdw16.data(), hdw16.size() * 2, hipMemcpyHostToDevice));
    a.in = din; a.ldi = 2 * K; a.offi = 0; a.dww16 = ddw16; a.dwb = ddb; a.gate = 1;
    a.nimg = 1; a.H = sh.H; a.W = sh.W; a.K = K; a.w = dw2; a.ldw = K; a.wstride = 0; a.wdiv = 1; a.N = N;
    a.bias = db; a.res = dx; a.ldr = N; a.out = dx; a.ldo = N; a.zeros = dz;
    if (!dwgemm_ok(a)) { printf("%s: dwgemm not eligible\n", sh.tag); continue; }
    DwArgs d{};
    d.in = din; d.ldi = 2 * K; d.out = dt2; d.ldo = K; d.w = ddw; d.bias = ddb; d.nimg = 1; d.H = sh.H; d.W = sh.W; d.C = K;
    d.mode = DW_GATE; d.rows = 1;
    GemmArgs gm{};
    gm.a.n = 1; gm.a.Ktot = K; gm.a.s[0] = SrcDesc{dt2, K, 0, K, 1, 0};
    gm.M = P; gm.N = N; gm.HW = (int)P; gm.Wimg = sh.W; gm.w = dw2; gm.ldw = K; gm.wdiv = 1; gm.bias = db;
    gm.res = dx2; gm.ldr = N; gm.out = dx2; gm.ldo = N; gm.zeros = dz; gm.ones = done;
    gm.allow_panel = gm.allow_lds = gm.allow_pn = gm.allow_ar = gm.allow_kt = 1;
    // correctness: one launch of each from the same x
    reset();
    launch_dwgemm(a, 0);
    launch_dw<bf16>(d, 0);
    launch_gemm<bf16>(gm, 0);
    CK(hipDeviceSynchronize());
    std::vector<uint16_t> o1(hx.size()), o2(hx.size());
    CK(hipMemcpy(o1.data(), dx, o1.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(o2.data(), dx2, o2.size() * 2, hipMemcpyDeviceToHost));
    double md = 0, mx = 0;
    for (size_t i = 0; i < o1.size(); ++i) {
      md = std::max(md, (double)fabsf(bf2f(o1[i]) - bf2f(o2[i])));
      mx = std::max(mx, (double)fabsf(bf2f(o2[i]) - bf2f(hx[i])));
    }
    const float t_dw = time_it([&] { launch_dw<bf16>(d, 0); }, reps);
    const float t_gm = time_it([&] { launch_gemm<bf16>(gm, 0); }, reps);
    printf("%s: P=%lld K=%d N=%d  max|dwgemm - (dw+gemm)| %.4g (max |update| %.3g)  dw %.1f us + gemm %.1f us = %.1f us\n",
           sh.tag, (long long)P, K, N, md, mx, t_dw, t_gm, t_dw + t_gm);
    // the channel-blocked hidden map of the frame (STORE_CB16: [2K / 16][P][16], x2 blocks after x1's)
    {
      std::vector<uint16_t> hcb(hin.size());
      for (int64_t p = 0; p < P; ++p)
        for (int c = 0; c < 2 * K; ++c) hcb[((size_t)(c / 16) * P + p) * 16 + c % 16] = hin[p * 2 * K + c];
      void* dcb;
      CK(hipMalloc(&dcb, hcb.size() * 2));
      CK(hipMemcpy(dcb, hcb.data(), hcb.size() * 2, hipMemcpyHostToDevice));
      DwGemmArgs c = a;
      c.in = dcb; c.cb_px = P; c.ldi = 0; c.offi = 0;
      {
        reset();
        launch_dwgemm(c, 0);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(o2.data(), dx, o2.size() * 2, hipMemcpyDeviceToHost));
        double mc = 0;
        for (size_t i = 0; i < o1.size(); ++i) mc = std::max(mc, (double)fabsf(bf2f(o1[i]) - bf2f(o2[i])));
        const float t_cb = time_it([&] { launch_dwgemm(c, 0); }, reps);
        const float t_px = time_it([&] { launch_dwgemm(a, 0); }, reps);
        printf("  channel-blocked input %.1f us (max|d| vs pixel-major %.3g), pixel-major %.1f us\n", t_cb, mc, t_px);
      }
      CK(hipFree(dcb));
    }
    const int dbgs[] = {0, 1, 2, 3, 4, 8, 12, 16, 4 | 8 | 16, 1 | 2 | 16, 1 | 2 | 4 | 8 | 16};
    for (int dbg : dbgs) {
      if (only >= 0 && dbg) continue;
      a.dbg = dbg;
      const float t = time_it([&] { launch_dwgemm(a, 0); }, reps);
      printf("  dwgemm dbg=%2d  %8.1f us\n", dbg, t);
    }
    a.dbg = 0;
    CK(hipFree(din)); CK(hipFree(dw2)); CK(hipFree(dx)); CK(hipFree(dx2)); CK(hipFree(dt2));
    CK(hipFree(ddw)); CK(hipFree(ddb)); CK(hipFree(db)); CK(hipFree(dz)); CK(hipFree(done));
  }
  return 0;
}

// SAB score microbenchmark (GPU box, no Python): launch_sab_score on the 1080p token grids, bf16,
// with ablation bits (SabScoreArgs::dbg: 1 no top-5 inserts, 2 no ball scores, 4 no MFMA).
//   hipcc -O3 --offload-arch=gfx950 -I turtlevsr_amd/csrc tools/sabbench.cpp -L turtlevsr_amd/lib -lturtle_hip -o tools/sabbench
#include <hip/hip_runtime.h>

#include <algorithm>
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

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  const int waves = argc > 3 ? atoi(argv[3]) : 4;    // ./sabbench reps nsplit(0: default) waves
  const int th = 68, tw = 120, N = th * tw;
  const int ds[] = {128, 256, 512}, Ts[] = {3, 4, 4};
  const int dbgs[] = {0, 1, 2, 3, 4, 7};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  srand(1);
  for (int c = 0; c < 3; ++c) {
    const int d = ds[c], T = Ts[c];
    std::vector<uint16_t> h((size_t)N * d);
    for (size_t n = 0; n < (size_t)N; ++n) {     // L2-normalised random tokens
      std::vector<float> v(d); float ss = 0;
      for (auto& x : v) { x = rand() / (float)RAND_MAX - 0.5f; ss += x * x; }
      for (int i = 0; i < d; ++i) h[n * d + i] = f2bf(v[i] / sqrtf(ss));
    }
    void* q; std::vector<void*> k(T);
    CK(hipMalloc(&q, h.size() * 2)); CK(hipMemcpy(q, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    for (int t = 0; t < T; ++t) {
      CK(hipMalloc(&k[t], h.size() * 2));
      std::rotate(h.begin(), h.begin() + d * 7, h.end());
      CK(hipMemcpy(k[t], h.data(), h.size() * 2, hipMemcpyHostToDevice));
    }
    float* tau; float one = 8.f;
    CK(hipMalloc(&tau, 4)); CK(hipMemcpy(tau, &one, 4, hipMemcpyHostToDevice));
    SabScoreArgs a{};
    a.q = q; a.q_bstride = 0;
    for (int t = 0; t < T; ++t) { a.k[t] = k[t]; a.k_bstride[t] = 0; }
    a.B = 1; a.T = T; a.N = N; a.d = d; a.th = th; a.tw = tw;
    a.waves = waves;
    a.nsplit = argc > 2 && atoi(argv[2]) > 0 ? atoi(argv[2]) : sab_score_nsplit(1, T, N, d, waves);
    a.tau = tau;
    CK(hipMalloc(&a.topv, (size_t)T * a.nsplit * N * 5 * 4));
    CK(hipMalloc(&a.topi, (size_t)T * a.nsplit * N * 5 * 4));
    CK(hipMalloc(&a.ballv, (size_t)T * N * 41 * 4));
    for (int dbg : dbgs) {
      a.dbg = dbg;
      launch_sab_score<bf16>(a, 0);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < reps; ++i) launch_sab_score<bf16>(a, 0);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      printf("d=%d T=%d N=%d nsplit=%d dbg=%d: %8.1f us\n", d, T, N, a.nsplit, dbg, ms * 1e3 / reps);
      fflush(stdout);
    }
    CK(hipFree(q)); for (auto p : k) CK(hipFree(p));
    CK(hipFree(a.topv)); CK(hipFree(a.topi)); CK(hipFree(a.ballv)); CK(hipFree(tau));
  }
  return 0;
}

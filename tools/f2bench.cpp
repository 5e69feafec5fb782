// Microbenchmark + cross-check of the row-walk fused kernel (fused2.hip) against the tile-fused
// kernel (fused.hip) on the Turtle 1080p launch shapes, GPU box only:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DTURTLE_F2_ABLATIONS -I turtlevsr_amd/csrc tools/f2bench.cpp \
//         turtlevsr_amd/csrc/fused2.hip -L turtlevsr_amd/lib -lturtle_hip -Wl,-rpath,'$ORIGIN/../turtlevsr_amd/lib' \
//         -o tools/f2bench && tools/f2bench [reps] [shape substring] [variants] [abl]
// Same random inputs for every kernel (LayerNorm statistics, biases, scales all live). Reference:
// fused.hip in fp32 (the parity-tested path) on the bf16 values widened to fp32. Prints per kernel
// the average launch time (HIP events) and the relative RMS / max error against that reference.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kernels.h"

using namespace turtle;

#define CK(x)                                                                                    \
  do {                                                                                           \
    hipError_t e = (x);                                                                          \
    if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } \
  } while (0)

static uint16_t f2bf(float f) {
  uint32_t u; memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
static float bf2f(uint16_t b) { uint32_t u = (uint32_t)b << 16; float f; memcpy(&f, &u, 4); return f; }
static float urand() { return rand() / (float)RAND_MAX - 0.5f; }

struct Shape { int H, W, C, N1, N2, mode, nimg; const char* tag; };

template <typename T>
static T* dev_copy(const std::vector<T>& h) {
  T* d; CK(hipMalloc(&d, h.size() * sizeof(T)));
  CK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const char* only = argc > 2 ? argv[2] : nullptr;      // substring of the shape tag
  // fused2 variants: a comma-separated list, or -1 (all, and the tile-fused kernel)
  std::vector<int> vlist;
  if (argc > 3) for (const char* p = argv[3]; *p;) { vlist.push_back(atoi(p)); while (*p && *p != ',') ++p; if (*p) ++p; }
  const int only_v = vlist.empty() ? -1 : vlist[0];
  const bool abl = argc > 4 && !strcmp(argv[4], "abl");   // per-phase ablation table (TURTLE_F2_ABLATIONS build)
  const Shape shapes[] = {
      {1088, 1920, 64, 320, 64, F_GATE, 1, "L1 GFFW gate"},
      {1088, 1920, 64, 128, 64, F_GELU, 1, "L1 ReducedAttn"},
      {544, 960, 128, 640, 128, F_GATE, 1, "L2 GFFW gate"},
      {544, 960, 128, 256, 128, F_GELU, 1, "L2 ReducedAttn"},
      {1088, 1920, 64, 192, 0, F_DWONLY, 1, "L1 qkv dw"},
      {1088, 1920, 64, 384, 0, F_DWONLY, 1, "L1 CHM 6c dw"},
      {1088, 1920, 64, 128, 0, F_DWONLY, 3, "L1 kv dw x3"},
      {544, 960, 128, 384, 0, F_DWONLY, 1, "L2 qkv dw"},
      {544, 960, 128, 768, 0, F_DWONLY, 1, "L2 CHM 6c dw"},
      {544, 960, 128, 256, 0, F_DWONLY, 4, "L2 kv dw x4"},
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  srand(7);
  printf("%-16s %-10s %9s %9s %9s\n", "shape", "kernel", "us", "rel_rms", "max_abs");
  for (const Shape& s : shapes) {
    if (only && !strstr(s.tag, only)) continue;
    const size_t px = (size_t)s.nimg * s.H * s.W;
    const int hid = s.mode == F_GATE ? s.N1 / 2 : s.N1;
    const int Nout = s.mode == F_DWONLY ? s.N1 : s.N2;
    const bool has_ref = true;                            // fused.hip: the fp32 reference
    std::vector<uint16_t> xb(px * s.C);
    std::vector<float> xf(px * s.C);
    for (size_t i = 0; i < xb.size(); ++i) { xb[i] = f2bf(0.3f + 2.f * urand() + 0.5f * urand() * urand()); xf[i] = bf2f(xb[i]); }
    std::vector<uint16_t> w1b((size_t)s.N1 * s.C), w2b((size_t)std::max(s.N2, 1) * hid);
    std::vector<float> w1f(w1b.size()), w2f(w2b.size());
    for (size_t i = 0; i < w1b.size(); ++i) { w1b[i] = f2bf(urand() * 0.25f); w1f[i] = bf2f(w1b[i]); }
    for (size_t i = 0; i < w2b.size(); ++i) { w2b[i] = f2bf(urand() * 0.2f); w2f[i] = bf2f(w2b[i]); }
    std::vector<float> lns(s.N1), lnt(s.N1), b1(s.N1), dwb(s.N1), dww((size_t)9 * s.N1), b2(128), sc2(128);
    for (int n = 0; n < s.N1; ++n) {
      double acc = 0;
      for (int k = 0; k < s.C; ++k) acc += w1f[(size_t)n * s.C + k];
      lns[n] = (float)acc; lnt[n] = urand() * 0.1f; b1[n] = urand() * 0.1f; dwb[n] = urand() * 0.1f;
    }
    for (auto& v : dww) v = urand() * 0.6f;
    for (auto& v : b2) v = urand() * 0.1f;
    for (auto& v : sc2) v = 0.5f + urand();
    std::vector<uint32_t> dww2((size_t)5 * s.N1);
    for (int i = 0; i < 5; ++i)
      for (int c = 0; c < s.N1; ++c) {
        const uint32_t lo = f2bf(dww[(size_t)(2 * i) * s.N1 + c]);
        const uint32_t hi = 2 * i + 1 < 9 ? f2bf(dww[(size_t)(2 * i + 1) * s.N1 + c]) : 0u;
        dww2[(size_t)i * s.N1 + c] = lo | (hi << 16);
      }
    void* Xb = dev_copy(xb); void* Xf = dev_copy(xf);
    void* W1b = dev_copy(w1b); void* W1f = dev_copy(w1f);
    void* W2b = dev_copy(w2b); void* W2f = dev_copy(w2f);
    float* Lns = dev_copy(lns); float* Lnt = dev_copy(lnt); float* B1 = dev_copy(b1); float* Dwb = dev_copy(dwb);
    float* Dww = dev_copy(dww); float* B2 = dev_copy(b2); float* Sc2 = dev_copy(sc2);
    uint32_t* Dww2 = dev_copy(dww2);
    void *Ob, *Of;
    CK(hipMalloc(&Ob, px * Nout * 2));
    CK(hipMalloc(&Of, px * Nout * 4));
    FusedArgs a{};
    a.ldx = s.C; a.offx = 0; a.C = s.C; a.nimg = s.nimg; a.H = s.H; a.W = s.W; a.N1 = s.N1;
    a.ln = s.mode == F_DWONLY && s.nimg > 1 ? 0 : 1;       // the CHM kv projection has no LayerNorm
    a.ln_s = a.ln ? Lns : nullptr; a.ln_t = a.ln ? Lnt : nullptr; a.b1 = B1;
    a.dww = Dww; a.dwb = Dwb; a.dww2 = Dww2; a.hidden = hid; a.mode = s.mode;
    a.N2 = s.N2; a.b2 = s.mode == F_GELU ? B2 : nullptr; a.scale2 = s.mode == F_GELU ? Sc2 : nullptr;
    a.ldr = s.N2; a.offr = 0; a.ldo = s.N2; a.offo = 0;
    auto setup = [&](bool bf) {
      FusedArgs b = a;
      b.x = bf ? Xb : Xf; b.w1 = bf ? W1b : W1f; b.w2 = bf ? W2b : W2f;
      b.res = b.x; b.out = bf ? Ob : Of;
      if (s.mode == F_DWONLY) {
        b.ndst = 1;
        b.dst[0] = FusedDst{b.out, Nout, 0, 0, Nout, Nout, 0, 0};
      }
      return b;
    };
    const FusedArgs af = setup(false), ab = setup(true);
    std::vector<float> ref(px * Nout, 0.f);
    if (has_ref) {
      launch_fused<float>(af, 0);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(ref.data(), Of, ref.size() * 4, hipMemcpyDeviceToHost));
    }
    double rr = 0;
    for (float v : ref) rr += (double)v * v;
    rr = sqrt(rr / ref.size());
    auto run = [&](const char* name, auto&& launch) {
      CK(hipMemset(Ob, 0, px * Nout * 2));
      launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < reps; ++i) launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      std::vector<uint16_t> o(px * Nout);
      CK(hipMemcpy(o.data(), Ob, o.size() * 2, hipMemcpyDeviceToHost));
      double se = 0, mx = 0;
      for (size_t i = 0; i < o.size(); ++i) {
        const double d = bf2f(o[i]) - ref[i];
        se += d * d; mx = std::max(mx, fabs(d));
      }
      printf("%-16s %-10s %9.1f %9.2e %9.2e\n", s.tag, name, ms * 1e3 / reps, sqrt(se / o.size()) / rr, mx);
    };
    if (only_v < 0 && has_ref) run("fused", [&] { launch_fused<bf16>(ab, 0); });
    if (fused2_ok(ab) && abl) {
      // per-phase ablations of the default configuration (fused2.hip ABL bits): 1 no GELU, 2 no
      // depthwise, 4 no GEMM2, 8 no LN, 16 no stores, 32 no GEMM1
      for (int ab_bits : {0, 1, 2, 4, 8, 16, 32, 3, 7, 39, 63}) {
        if (s.mode == F_DWONLY && (ab_bits & 5) && ab_bits != 63) continue;
        FusedArgs c = ab; c.dbg = ab_bits << 8;
        char nm[16]; snprintf(nm, sizeof nm, "abl.%d", ab_bits);
        run(nm, [&] { launch_fused2(c, 0); });
      }
    } else if (fused2_ok(ab)) {
      for (int v = 0; v < 12; ++v) {
        if (only_v >= 0 && std::find(vlist.begin(), vlist.end(), v) == vlist.end()) continue;
        if (v >= 6 && v < 10 && !(ab.mode == F_GATE && ab.C == 64)) continue;
        FusedArgs c = ab; c.dbg = v;
        char nm[16]; snprintf(nm, sizeof nm, "fused2.%d", v);
        run(nm, [&] { launch_fused2(c, 0); });
      }
    } else {
      printf("%-16s fused2 not eligible\n", s.tag);
    }
    for (void* p : {Xb, Xf, W1b, W1f, W2b, W2f, (void*)Lns, (void*)Lnt, (void*)B1, (void*)Dwb, (void*)Dww, (void*)B2,
                    (void*)Sc2, (void*)Dww2, Ob, Of})
      CK(hipFree(p));
  }
  return 0;
}

// Diagnostic: gram_kernel<bf16> vs a CPU reference (build with -DTURTLE_GRAM_TR=0/1).
#include "../turtlevsr_amd/csrc/attn.hip"
#include <cstdio>
#include <cmath>
#include <vector>
using namespace turtle;
int main() {
  const int HW = 1024, ch = 64, heads = 2, C = ch * heads, nseg = 2;
  std::vector<bf16> q(HW * 3 * C);
  for (size_t i = 0; i < q.size(); ++i) q[i] = (bf16)(float)(((i * 2654435761u) >> 8) % 1000 / 500.0 - 1.0);
  bf16* dq; hipMalloc(&dq, q.size() * 2); hipMemcpy(dq, q.data(), q.size() * 2, hipMemcpyHostToDevice);
  const int ncol = nseg * ch, stride = ch * ncol + ch + ncol, nchunk = 4;
  float* dp; hipMalloc(&dp, (size_t)heads * nchunk * stride * 4);
  GramArgs g{};
  g.q = dq; g.ldq = 3 * C; g.qoff = 0; g.nseg = nseg;
  g.seg[0] = GramSeg{dq, 3 * C, C, ch, 1, 0, 1};        // k part
  g.seg[1] = GramSeg{dq, 3 * C, 2 * C, ch, 1, 0, 1};    // v part as a second key segment
  g.B = 1; g.heads = heads; g.ch = ch; g.HW = HW; g.nchunk = nchunk; g.chunk = HW / nchunk; g.part = dp;
  launch_gram<bf16>(g, 0);
  std::vector<float> part((size_t)heads * nchunk * stride);
  hipMemcpy(part.data(), dp, part.size() * 4, hipMemcpyDeviceToHost);
  double maxerr = 0, maxref = 0; int bad = 0;
  for (int h = 0; h < heads; ++h)
    for (int i = 0; i < ch; ++i)
      for (int j = 0; j < ncol; ++j) {
        double ref = 0;
        const int s = j / ch, jj = j % ch;
        for (int p = 0; p < HW; ++p)
          ref += (double)(float)q[p * 3 * C + h * ch + i] * (double)(float)q[p * 3 * C + (s + 1) * C + h * ch + jj];
        double got = 0;
        for (int c = 0; c < nchunk; ++c) got += part[((size_t)h * nchunk + c) * stride + i * ncol + j];
        double e = fabs(got - ref);
        if (e > 1e-2 && bad++ < 10) printf("h%d i%d j%d got %f ref %f\n", h, i, j, got, ref);
        maxerr = fmax(maxerr, e); maxref = fmax(maxref, fabs(ref));
      }
  printf("TR=%d maxerr %g maxref %g bad %d\n", TURTLE_GRAM_TR, maxerr, maxref, bad);
  return 0;
}

// Probe of ds_read_b64_tr_b16 lane semantics (diagnostic, not part of the library).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;
__global__ void k(int* out) {
  __shared__ __attribute__((aligned(16))) short lds[16 * 64];   // [16 rows][64 cols]
  for (int i = threadIdx.x; i < 16 * 64; i += 64) lds[i] = (short)((i / 64) * 100 + (i % 64));
  __syncthreads();
  const int lane = threadIdx.x, g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const short* a = lds + (4 * g + q) * 64 + 4 * p;      // group g: rows 4g..4g+3, cols 0..15
  v4s r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)a);
  for (int e = 0; e < 4; ++e) out[lane * 4 + e] = r[e];
}
int main() {
  int* d; hipMalloc(&d, 64 * 4 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  int h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) { printf("lane %2d:", l); for (int e = 0; e < 4; ++e) printf(" %4d", h[l * 4 + e]); printf("\n"); }
  return 0;
}

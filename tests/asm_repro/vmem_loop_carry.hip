// Minimal reproduction of the round-4 `sab_avt` bring-up fault, kept as the
// positive case of tests/test_asm_vmem_scan.py. NOT part of the library and never run on a GPU.
//
// A two-slot ring of inline-asm loads is rotated in a loop (x0 <- x1, then x1 is reloaded for the
// next iteration). The hand-written wait names only x0, so hipcc copies x1 -> x0 at the top of the
// next iteration while x1's load, issued at the bottom of the previous one, is still in flight: the
// copy reads a half-written register. The loop entry is clean (both loads waited for) and in text
// order the copy comes before the load, so only a scan that follows the loop's back-edge sees it.
#include <hip/hip_runtime.h>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__global__ void vmem_loop_carry_repro(const u32x4* __restrict__ p, u32x4* __restrict__ out, int n) {
  u32x4 x0, x1, acc = {0, 0, 0, 0};
  const u32x4* q = p + threadIdx.x;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(x0) : "v"(q) : "memory");
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(x1) : "v"(q + 64) : "memory");
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(x0), "+v"(x1) : : "memory");   // loop entry: clean
  for (int i = 0; i < n; ++i) {
    asm volatile("s_waitcnt vmcnt(1)" : "+v"(x0) : : "memory");
    acc.x += x0.x; acc.y ^= x0.y; acc.z += x0.z; acc.w ^= x0.w;
    x0 = x1;                                            // rotate the ring: x1 may still be in flight
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(x1) : "v"(q + 64 * (i + 2)) : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(x0), "+v"(x1) : : "memory");
  out[threadIdx.x] = u32x4{acc.x + x0.x, acc.y + x1.y, acc.z, acc.w};
}

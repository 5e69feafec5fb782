// Shared device helpers for the Turtle HIP kernels (gfx950 / CDNA4, wave64).
//
// Storage types: activations and GEMM weights are either float (fp32 parity mode) or __bf16
// (throughput mode); every reduction / accumulation is fp32. Feature maps are pixel-major
// ("NHWC"): [image][y][x][channel], channel contiguous, so a 16-byte vector holds VEC consecutive
// channels of one pixel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#define TURTLE_DEV __device__ __forceinline__

typedef _Float16 f16;          // fp16 activations of the training kernels (the reference's autocast)

TURTLE_DEV float to_f(float x) { return x; }
TURTLE_DEV float to_f(bf16 x) { return (float)x; }
TURTLE_DEV float to_f(f16 x) { return (float)x; }
template <typename T> TURTLE_DEV T from_f(float x);
template <> TURTLE_DEV float from_f<float>(float x) { return x; }
template <> TURTLE_DEV bf16 from_f<bf16>(float x) { return (bf16)x; }
template <> TURTLE_DEV f16 from_f<f16>(float x) { return (f16)x; }

// 16-byte vector of storage elements, unpacked to fp32 registers.
template <typename T> struct Vec;
template <> struct Vec<float> {
  static constexpr int N = 4;
  float v[4];
  TURTLE_DEV void load(const float* p) {
    float4 q = *reinterpret_cast<const float4*>(p);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  }
  TURTLE_DEV void store(float* p) const {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
  TURTLE_DEV void zero() { v[0] = v[1] = v[2] = v[3] = 0.f; }
  TURTLE_DEV void from_raw(uint4 q) {
    v[0] = __uint_as_float(q.x); v[1] = __uint_as_float(q.y); v[2] = __uint_as_float(q.z); v[3] = __uint_as_float(q.w);
  }
  // unconditional load from a valid address, zeroed when !ok (no branch around the load, so the
  // compiler keeps several loads in flight instead of waiting on each: guide §5 trap (c))
  TURTLE_DEV void load_pred(const float* p, bool ok) {
    float4 q = *reinterpret_cast<const float4*>(p);
    v[0] = ok ? q.x : 0.f; v[1] = ok ? q.y : 0.f; v[2] = ok ? q.z : 0.f; v[3] = ok ? q.w : 0.f;
  }
};
template <> struct Vec<bf16> {
  static constexpr int N = 8;
  float v[8];
  TURTLE_DEV void load(const bf16* p) {
    uint4 q = *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  TURTLE_DEV void from_raw(uint4 q) {
    uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  TURTLE_DEV void load_pred(const bf16* p, bool ok) {
    uint4 q = *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {ok ? q.x : 0u, ok ? q.y : 0u, ok ? q.z : 0u, ok ? q.w : 0u};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  TURTLE_DEV void store(bf16* p) const {
    bf16x8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (bf16)v[i];
    *reinterpret_cast<bf16x8*>(p) = o;
  }
  TURTLE_DEV void zero() {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = 0.f;
  }
};

// One unconditional 16-byte global load. The address is made opaque to the optimiser so a
// select between a real and a dummy (zero) address stays a v_cndmask instead of being turned into
// two predicated loads behind branches, each drained with s_waitcnt vmcnt(0).
TURTLE_DEV uint4 ld16(const void* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef __attribute__((address_space(1))) const uint4 gUint4;
  uint64_t a = reinterpret_cast<uint64_t>(p);
  asm volatile("" : "+v"(a));
  return *reinterpret_cast<gUint4*>(a);   // global_load_dwordx4 (not flat)
#else
  return *reinterpret_cast<const uint4*>(p);
#endif
}

// same, 8 bytes
TURTLE_DEV uint2 ld8(const void* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef __attribute__((address_space(1))) const uint2 gUint2;
  uint64_t a = reinterpret_cast<uint64_t>(p);
  asm volatile("" : "+v"(a));
  return *reinterpret_cast<gUint2*>(a);
#else
  return *reinterpret_cast<const uint2*>(p);
#endif
}

// same for one fp32 value
TURTLE_DEV float ld4f(const float* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef __attribute__((address_space(1))) const float gF;
  uint64_t a = reinterpret_cast<uint64_t>(p);
  asm volatile("" : "+v"(a));
  return *reinterpret_cast<gF*>(a);
#else
  return *p;
#endif
}

// Two 8-float scalar loads (s_load_dwordx8 x2) of wave-uniform, read-only data (depthwise weights).
// hipcc will not emit scalar loads through these pointers on its own (the asm in the same loops
// counts as a possible clobber), so they are issued here and retired by sload_wait(): the wait
// redefines the values, so no use can be scheduled before it.
typedef float f32x8 __attribute__((ext_vector_type(8)));
TURTLE_DEV void sload2x8(const float* p0, const float* p1, f32x8& o0, f32x8& o1) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_load_dwordx8 %0, %2, 0x0\n\ts_load_dwordx8 %1, %3, 0x0" : "=&s"(o0), "=&s"(o1) : "s"(p0), "s"(p1));
#else
  for (int i = 0; i < 8; ++i) { o0[i] = p0[i]; o1[i] = p1[i]; }
#endif
}
TURTLE_DEV void sload_wait(f32x8& o0, f32x8& o1) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(o0), "+s"(o1));
#endif
}

// GELU with erf from Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7): two transcendentals
// (v_rcp, v_exp) and a 5-term Horner polynomial, against ~25 instructions for erff
TURTLE_DEV float erf_fast(float x) {
  const float a = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float e = __builtin_amdgcn_exp2f(-a * a * 1.4426950408889634f);
  return copysignf(fmaf(-p, e, 1.f), x);
}
TURTLE_DEV float gelu_fast(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }

TURTLE_DEV float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }

// tanh-form GELU, x * sigmoid(1.5957691 (x + 0.044715 x^3)): |diff| to the erf form <= 5e-4,
// below the bf16 rounding step of any GELU output above 0.13; one exp2 + one rcp + 4 VALU
TURTLE_DEV float gelu_tanh(float x) {
  const float u = x * fmaf(-0.10294324f, x * x, -2.3022082f);   // -log2(e) * 1.5957691 (x + 0.044715 x^3)
  return x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(u));
}
// GELU of the bf16 kernels: the tanh form unless built with TURTLE_BF16_GELU_TANH=0 (the erf form,
// A&S 7.1.26, |error| <= 1.5e-7). Measured on MI355X at 1080p: the erf form leaves the bf16 - fp32
// PSNR delta where it was (0.0114 vs 0.0111 dB: the bf16 storage rounding dominates) and costs
// 6 % on the L1 GatedFFN fused kernel (855 -> 905 us)
#ifndef TURTLE_BF16_GELU_TANH
#define TURTLE_BF16_GELU_TANH 1
#endif
TURTLE_DEV float gelu_bf16(float x) {
#if TURTLE_BF16_GELU_TANH
  return gelu_tanh(x);
#else
  return gelu_fast(x);
#endif
}
// two tanh-form GELUs with the polynomial / scaling steps as packed f32 pairs (v_pk_mul / v_pk_fma,
// identical roundings to gelu_tanh per element); the bf16 kernels' GELU when TURTLE_BF16_GELU_TANH
TURTLE_DEV f32x2 gelu_tanh2(f32x2 x) {
  const f32x2 u = x * __builtin_elementwise_fma(f32x2{-0.10294324f, -0.10294324f}, x * x, f32x2{-2.3022082f, -2.3022082f});
  const f32x2 e = f32x2{__builtin_amdgcn_exp2f(u.x), __builtin_amdgcn_exp2f(u.y)} + f32x2{1.f, 1.f};
  return x * f32x2{__builtin_amdgcn_rcpf(e.x), __builtin_amdgcn_rcpf(e.y)};
}
TURTLE_DEV f32x2 gelu_bf16_2(f32x2 x) {
#if TURTLE_BF16_GELU_TANH
  return gelu_tanh2(x);
#else
  return f32x2{gelu_fast(x.x), gelu_fast(x.y)};
#endif
}
// GELU of a kernel computing in storage type T: gelu_bf16 for bf16 storage, libm erf for fp32
template <typename T>
TURTLE_DEV float gelu_t(float x) {
  if constexpr (sizeof(T) == 2) return gelu_bf16(x);
  else return gelu_erf(x);
}

TURTLE_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
TURTLE_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ------------------------------------------------------------------------------------------
// Host/device descriptors
// ------------------------------------------------------------------------------------------
#define TURTLE_MAX_SRC 6

// One operand source of a K-concatenated GEMM A matrix (pixel rows, channel columns).
// Row of output pixel m = (img, p):   src_img = img * img_mul + img_add
//   element (m, k) = base[(src_img * HW + p) * ld + off + k - kbeg]   for kbeg <= k < kbeg + K
struct SrcDesc {
  const void* base;
  int64_t ld;
  int off;
  int K;
  int img_mul;
  int img_add;
};

struct SrcList {
  SrcDesc s[TURTLE_MAX_SRC];
  int n;
  int Ktot;
  int64_t cb_px;   // > 0: the (single) source is channel-blocked [Ktot / 16][cb_px][16] (base, off 0), 2-D tiled GEMM only
};

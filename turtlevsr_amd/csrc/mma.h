// MFMA building blocks shared by the GEMM-shaped kernels (1x1 conv GEMM, SAB scores).
// Both operands are staged in LDS as [row][BK] tiles with ROWB bytes per row; one MFMA
// step multiplies a 16-row slice of each (i = A rows, j = B rows) over KSUB of K.
#pragma once
#include "common.h"

namespace turtle {

template <typename T> struct Mma;
template <> struct Mma<bf16> {
  static constexpr int BK = 64;    // elements per K tile (128 B per row)
  static constexpr int KSUB = 32;  // K per MFMA
  static constexpr int VEC = 8;
};
template <> struct Mma<float> {
  static constexpr int BK = 32;
  static constexpr int KSUB = 4;
  static constexpr int VEC = 4;
};

constexpr int ROWB = 144;  // LDS bytes per tile row: 128 data + 16 pad (spreads ds_read_b128 slots)

// acc[tm][tn] += A(rows wrow_n + 16 tn ..) x B(rows wrow_m + 16 tm ..)^T over K slice ks
template <typename T>
TURTLE_DEV void mma_step(const char* sW, const char* sX, int lane, int ks, f32x4 (&acc)[4][4],
                         int TM, int TN, int wrow_n, int wrow_m);

template <>
TURTLE_DEV void mma_step<bf16>(const char* sW, const char* sX, int lane, int ks, f32x4 (&acc)[4][4],
                               int TM, int TN, int wrow_n, int wrow_m) {
  const int r = lane & 15, kb = ks * 64 + (lane >> 4) * 16;   // byte offset within row
  bf16x8 a[4], b[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (t < TN) a[t] = *reinterpret_cast<const bf16x8*>(sW + (wrow_n + t * 16 + r) * ROWB + kb);
    if (t < TM) b[t] = *reinterpret_cast<const bf16x8*>(sX + (wrow_m + t * 16 + r) * ROWB + kb);
  }
#pragma unroll
  for (int tm = 0; tm < 4; ++tm)
#pragma unroll
    for (int tn = 0; tn < 4; ++tn)
      if (tm < TM && tn < TN)
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[tn], b[tm], acc[tm][tn], 0, 0, 0);
}

template <>
TURTLE_DEV void mma_step<float>(const char* sW, const char* sX, int lane, int ks, f32x4 (&acc)[4][4],
                                int TM, int TN, int wrow_n, int wrow_m) {
  const int r = lane & 15, kb = (ks * 4 + (lane >> 4)) * 4;
  float a[4], b[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (t < TN) a[t] = *reinterpret_cast<const float*>(sW + (wrow_n + t * 16 + r) * ROWB + kb);
    if (t < TM) b[t] = *reinterpret_cast<const float*>(sX + (wrow_m + t * 16 + r) * ROWB + kb);
  }
#pragma unroll
  for (int tm = 0; tm < 4; ++tm)
#pragma unroll
    for (int tn = 0; tn < 4; ++tn)
      if (tm < TM && tn < TN)
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[tn], b[tm], acc[tm][tn], 0, 0, 0);
}

// single-step MFMA operand fragments (A or B, 16 rows x one K step), per storage type
template <typename T> struct Frag;
template <> struct Frag<bf16> { typedef bf16x8 type; static constexpr int K = 32; };
template <> struct Frag<float> { typedef float type; static constexpr int K = 4; };

TURTLE_DEV f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
TURTLE_DEV f32x4 mfma(float a, float b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

// lane's fragment of one K step from a row-major [row][k] LDS image (row = lane & 15)
template <typename T>
TURTLE_DEV typename Frag<T>::type frag_at(const char* row0, int rowbytes, int k0, int lane) {
  const char* p = row0 + (lane & 15) * rowbytes;
  if constexpr (sizeof(T) == 2) return *reinterpret_cast<const bf16x8*>(p + (k0 + (lane >> 4) * 8) * 2);
  else return *reinterpret_cast<const float*>(p + (k0 + (lane >> 4)) * 4);
}

}  // namespace turtle

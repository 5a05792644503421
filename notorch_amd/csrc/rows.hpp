// Row-piece access for fp32 and bf16 feature rows: one lane moves N consecutive elements of a row
// (N = 4 fp32 or 8 bf16 = one 16-B piece, or N = 1 for rows that are not 16-B aligned), converting to
// and from fp32 registers.  Shared by the element-wise kernels that run on either storage dtype.
#pragma once

#include "common.hpp"

namespace nt {

typedef unsigned short bf16_raw;  // bf16 storage

template <typename T, bool VEC>
struct Piece;

template <>
struct Piece<float, true> {
  static constexpr int N = 4;
  __device__ __forceinline__ static void load(const float* p, float (&x)[N]) {
    const float4 v = *reinterpret_cast<const float4*>(p);
    x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
  }
  __device__ __forceinline__ static void store(float* p, const float (&x)[N]) {
    *reinterpret_cast<float4*>(p) = make_float4(x[0], x[1], x[2], x[3]);
  }
};

template <>
struct Piece<float, false> {
  static constexpr int N = 1;
  __device__ __forceinline__ static void load(const float* p, float (&x)[N]) { x[0] = *p; }
  __device__ __forceinline__ static void store(float* p, const float (&x)[N]) { *p = x[0]; }
};

template <>
struct Piece<bf16_raw, true> {
  static constexpr int N = 8;
  __device__ __forceinline__ static void load(const bf16_raw* p, float (&x)[N]) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    const unsigned u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      x[2 * i] = __uint_as_float(u[i] << 16);
      x[2 * i + 1] = __uint_as_float(u[i] & 0xffff0000u);
    }
  }
  __device__ __forceinline__ static void store(bf16_raw* p, const float (&x)[N]) {
    typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
    bf16x8 v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (__bf16)x[i];
    *reinterpret_cast<uint4*>(p) = __builtin_bit_cast(uint4, v);
  }
};

template <>
struct Piece<bf16_raw, false> {
  static constexpr int N = 1;
  __device__ __forceinline__ static void load(const bf16_raw* p, float (&x)[N]) {
    x[0] = __uint_as_float((unsigned)*p << 16);
  }
  __device__ __forceinline__ static void store(bf16_raw* p, const float (&x)[N]) {
    *p = __builtin_bit_cast(bf16_raw, (__bf16)x[0]);
  }
};

// the value an element of type T holds after a store (fp32: itself; bf16: rounded)
template <typename T>
__device__ __forceinline__ float as_stored(float x) {
  if constexpr (sizeof(T) == 2) return __uint_as_float((unsigned)__builtin_bit_cast(bf16_raw, (__bf16)x) << 16);
  else return x;
}

}  // namespace nt

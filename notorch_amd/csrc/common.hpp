// Shared helpers for the notorch_amd HIP kernels (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <float.h>

#include <string>

#include "../../include/notorch_amd.h"

namespace nt {

// ---- error plumbing (thread-local last error, returned through nt_last_error) ----
void set_error(const std::string& msg);
void clear_error();
// record the layer kernel variant a call launched (a static string), read by nt_last_kernel
void set_last_kernel(const char* name);

#define NT_REQUIRE(cond, code, msg)                      \
  do {                                                   \
    if (!(cond)) {                                       \
      ::nt::set_error(std::string(__func__) + ": " + (msg)); \
      return (code);                                     \
    }                                                    \
  } while (0)

#define NT_HIP(expr)                                                                    \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      ::nt::set_error(std::string(__func__) + ": " #expr " -> " + hipGetErrorString(_e)); \
      return NT_EHIP;                                                                   \
    }                                                                                   \
  } while (0)

// launch-error check (kernel launches are asynchronous; this catches bad configurations)
#define NT_LAUNCH_CHECK() NT_HIP(hipGetLastError())

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int kWave = 64;  // CDNA wavefront width

// ---- element-wise activations (torch formulas; nn.ReLU, nn.LeakyReLU, nn.ELU, nn.GELU, ...) ----
__device__ __forceinline__ float act_apply(float x, int act, float alpha) {
  switch (act) {
    case NT_ACT_RELU: return x > 0.f ? x : 0.f;
    case NT_ACT_LEAKY_RELU: return x > 0.f ? x : x * alpha;
    case NT_ACT_ELU: return x > 0.f ? x : alpha * expm1f(x);
    case NT_ACT_GELU: return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
    case NT_ACT_SILU: return x / (1.f + expf(-x));
    case NT_ACT_TANH: return tanhf(x);
    case NT_ACT_SIGMOID: return 1.f / (1.f + expf(-x));
    default: return x;
  }
}

// compile-time specialisation for the hot combinations (relu / identity) so the inner loops carry
// no switch; ACT < 0 means "runtime act".
template <int ACT>
__device__ __forceinline__ float act_t(float x, int act, float alpha) {
  if constexpr (ACT == NT_ACT_IDENTITY) return x;
  else if constexpr (ACT == NT_ACT_RELU) return x > 0.f ? x : 0.f;
  else return act_apply(x, act, alpha);
}

__device__ __forceinline__ float4 act4(float4 v, int act, float alpha) {
  return make_float4(act_apply(v.x, act, alpha), act_apply(v.y, act, alpha),
                     act_apply(v.z, act, alpha), act_apply(v.w, act, alpha));
}
template <int ACT>
__device__ __forceinline__ float4 act4_t(float4 v, int act, float alpha) {
  return make_float4(act_t<ACT>(v.x, act, alpha), act_t<ACT>(v.y, act, alpha),
                     act_t<ACT>(v.z, act, alpha), act_t<ACT>(v.w, act, alpha));
}

__device__ __forceinline__ float4 operator+(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 operator-(float4 a, float4 b) {
  return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w);
}

// ---- torch_scatter reduce semantics in fp32 (sum; mean = sum / max(n,1); max/min, empty -> 0) ----
template <int R>
struct Reducer {
  float acc;
  int n;
  __device__ __forceinline__ void init() {
    n = 0;
    if constexpr (R == NT_MAX) acc = -FLT_MAX;
    else if constexpr (R == NT_MIN) acc = FLT_MAX;
    else acc = 0.f;
  }
  __device__ __forceinline__ void push(float x) {
    ++n;
    if constexpr (R == NT_MAX) acc = (n == 1 || x > acc) ? x : acc;
    else if constexpr (R == NT_MIN) acc = (n == 1 || x < acc) ? x : acc;
    else acc += x;
  }
  __device__ __forceinline__ float result() const {
    if constexpr (R == NT_MEAN) return acc / (float)(n > 1 ? n : 1);
    else if constexpr (R == NT_MAX || R == NT_MIN) return n == 0 ? 0.f : acc;
    else return acc;
  }
};

template <int R>
struct Reducer4 {
  Reducer<R> x, y, z, w;
  __device__ __forceinline__ void init() { x.init(); y.init(); z.init(); w.init(); }
  __device__ __forceinline__ void push(float4 v) { x.push(v.x); y.push(v.y); z.push(v.z); w.push(v.w); }
  __device__ __forceinline__ float4 result() const {
    return make_float4(x.result(), y.result(), z.result(), w.result());
  }
};

// *p = max(*p, v) for non-negative floats (they order like their bit patterns).  The relaxed read
// first skips the atomic when it cannot raise the value, so the thousands of waves of a launch do not
// serialise on one L2 line (a stale read only costs an unneeded atomic: *p never decreases).
__device__ __forceinline__ void atomic_max_nonneg(float* p, float v) {
  if (!(v <= __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)))
    atomicMax(reinterpret_cast<unsigned int*>(p), __float_as_uint(v));
}

// Block-wide max of non-negative values into p[0] (and p[1]): wave shuffles, one LDS slot per wave,
// one atomic per block.  Every thread of the block must call it (it holds a barrier).
__device__ __forceinline__ void block_max_to(float* p, float a, float b = 0.f, bool two = false) {
  __shared__ float sm[2][16];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    a = fmaxf(a, __shfl_xor(a, o));
    b = fmaxf(b, __shfl_xor(b, o));
  }
  const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  if ((threadIdx.x & 63) == 0) {
    sm[0][w] = a;
    sm[1][w] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < nw; ++i) {
      a = fmaxf(a, sm[0][i]);
      b = fmaxf(b, sm[1][i]);
    }
    atomic_max_nonneg(p, a);
    if (two) atomic_max_nonneg(p + 1, b);
  }
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline int grid_for(int64_t work, int block, int cap = 256 * 16) {
  int64_t g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace nt

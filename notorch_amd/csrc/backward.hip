// Backward of the D-MPNN block: the gather/scatter/element-wise parts as HIP
// kernels; the two dense products per layer (dA = G W, dW = G^T A) are plain library GEMMs issued by
// the host on the same stream.
//
// Forward of layer l (chemprop.py:28-43, residual.py:27-28), per directed edge e:
//   M = act(H_l);  S_l[v] = R_{e->v} M[e];  A_l[e] = S_l[src e] - M[rev e];  H_{l+1} = H_l + A_l W^T + b
// Backward with G = dL/dH_{l+1} (R = sum or mean; c_v = max(in-degree v, 1) for mean, 1 for sum):
//   dA = G W;  dS[v] = sum_{e: src e = v} dA[e]                         (nt_segment_reduce, src CSR)
//   dL/dH_l[e] = (residual ? G[e] : 0)
//              + act'(H_l[e]) * (dS[dst e] / c_{dst e} - sum_{e': rev e' = e} dA[e'])   (this file)
// The rev term is a scatter by rev_index; the reference collate's rev_index is not a permutation
// (graph.py:200 offsets it by nodes), so it is read through the rev CSR (ascending e').
//
// Kernels (all HBM-bound streaming gathers, one lane per (row, 16-B column chunk) so every row is
// read as whole contiguous pieces):
//   nt_dmpnn_message        A[e] = S[src e] - act(H[rev e])                3 rows / edge
//   nt_dmpnn_edge_backward  the dL/dH_l line above                         5 rows / edge
//   nt_gather_rows          out[i] = base[i] + X[idx i] / c_{idx i}        3 rows / row
//                           (dnode[dst] into dL/dH_d, chemprop.py:86; readout backward, agg.py:23-38)
#include "common.hpp"
#include "rows.hpp"

namespace nt {

__device__ __forceinline__ float act_grad(float x, int act, float alpha) {
  switch (act) {
    case NT_ACT_RELU: return x > 0.f ? 1.f : 0.f;
    case NT_ACT_LEAKY_RELU: return x > 0.f ? 1.f : alpha;
    case NT_ACT_ELU: return x > 0.f ? 1.f : alpha * expf(x);
    case NT_ACT_GELU: {
      const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
      const float pdf = 0.39894228040143268f * expf(-0.5f * x * x);
      return cdf + x * pdf;
    }
    case NT_ACT_SILU: {
      const float s = 1.f / (1.f + expf(-x));
      return s * (1.f + x * (1.f - s));
    }
    case NT_ACT_TANH: {
      const float t = tanhf(x);
      return 1.f - t * t;
    }
    case NT_ACT_SIGMOID: {
      const float s = 1.f / (1.f + expf(-x));
      return s * (1.f - s);
    }
    default: return 1.f;
  }
}

template <int ACT>
__device__ __forceinline__ float act_grad_t(float x, int act, float alpha) {
  if constexpr (ACT == NT_ACT_IDENTITY) return 1.f;
  else if constexpr (ACT == NT_ACT_RELU) return x > 0.f ? 1.f : 0.f;
  else return act_grad(x, act, alpha);
}

// ---- element-type helpers: the same kernel body runs on float4 (h % 4 == 0) or float ----
__device__ __forceinline__ float4 vfill(float4, float s) { return make_float4(s, s, s, s); }
__device__ __forceinline__ float vfill(float, float s) { return s; }
__device__ __forceinline__ float4 vmul(float4 a, float4 b) {
  return make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w);
}
__device__ __forceinline__ float vmul(float a, float b) { return a * b; }
template <int ACT>
__device__ __forceinline__ float4 vact(float4 v, int act, float alpha) { return act4_t<ACT>(v, act, alpha); }
template <int ACT>
__device__ __forceinline__ float vact(float v, int act, float alpha) { return act_t<ACT>(v, act, alpha); }
template <int ACT>
__device__ __forceinline__ float4 vgrad(float4 v, int act, float alpha) {
  return make_float4(act_grad_t<ACT>(v.x, act, alpha), act_grad_t<ACT>(v.y, act, alpha),
                     act_grad_t<ACT>(v.z, act, alpha), act_grad_t<ACT>(v.w, act, alpha));
}
template <int ACT>
__device__ __forceinline__ float vgrad(float v, int act, float alpha) { return act_grad_t<ACT>(v, act, alpha); }

// ------------------------------------------------------------------------------ message
template <typename T, int ACT>
__global__ void __launch_bounds__(256) message_kernel(const T* __restrict__ H, const T* __restrict__ S,
                                                      const int64_t* __restrict__ src,
                                                      const int64_t* __restrict__ rev, int64_t E,
                                                      int64_t hw, int act, float alpha,
                                                      T* __restrict__ A) {
  const int64_t total = E * hw;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = t / hw, c = t - e * hw;
    A[t] = S[src[e] * hw + c] - vact<ACT>(H[rev[e] * hw + c], act, alpha);
  }
}

// max |x| over a value's components (the amax outputs: the backward's fp16-split scales)
__device__ __forceinline__ float vamax(float x) { return fabsf(x); }
__device__ __forceinline__ float vamax(float4 x) {
  return fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w)));
}

// ------------------------------------------------------------------------------ edge backward
template <typename T, int ACT, bool MEAN>
__global__ void __launch_bounds__(256) edge_backward_kernel(
    const T* __restrict__ G, const T* __restrict__ H, const T* __restrict__ dA,
    const T* __restrict__ dS, const int64_t* __restrict__ dst, const int32_t* __restrict__ rev_ptr,
    const int32_t* __restrict__ rev_perm, const int32_t* __restrict__ dst_ptr, int64_t E,
    int64_t hw, int residual, int act, float alpha, T* __restrict__ Gout, float* __restrict__ amax) {
  const int64_t total = E * hw;
  float m = 0.f;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = t / hw, c = t - e * hw;
    const int64_t v = dst[e];
    T dm = dS[v * hw + c];
    if constexpr (MEAN) {
      const int cnt = dst_ptr[v + 1] - dst_ptr[v];
      dm = vmul(dm, vfill(dm, 1.f / (float)(cnt > 1 ? cnt : 1)));
    }
    const int32_t b = rev_ptr[e], en = rev_ptr[e + 1];
    for (int32_t j = b; j < en; ++j) dm = dm - dA[(int64_t)rev_perm[j] * hw + c];
    T g = vmul(vgrad<ACT>(H[t], act, alpha), dm);
    if (residual) g = g + G[t];
    Gout[t] = g;
    m = fmaxf(m, vamax(g));
  }
  if (amax) block_max_to(amax, m);
}

// ------------------------------------------------------------------------------ gather rows
template <typename T, bool MEAN>
__global__ void __launch_bounds__(256) gather_rows_kernel(const T* __restrict__ base,
                                                          const T* __restrict__ X,
                                                          const int64_t* __restrict__ idx,
                                                          const int32_t* __restrict__ seg_ptr,
                                                          int64_t n, int64_t hw, T* __restrict__ out,
                                                          float* __restrict__ amax) {
  const int64_t total = n * hw;
  float m = 0.f;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t / hw, c = t - i * hw;
    const int64_t s = idx[i];
    T x = X[s * hw + c];
    if constexpr (MEAN) {
      const int cnt = seg_ptr[s + 1] - seg_ptr[s];
      x = vmul(x, vfill(x, 1.f / (float)(cnt > 1 ? cnt : 1)));
    }
    const T y = base ? base[t] + x : x;
    out[t] = y;
    m = fmaxf(m, vamax(y));
  }
  if (amax) block_max_to(amax, m);
}

// ------------------------------------------------------------------------------ max / min
// torch_scatter's scatter_max / scatter_min (chemprop.py:39,86; agg.py:45) send the whole gradient
// of an output element to its arg: the FIRST row of the segment, in the CSR's ascending-row order,
// whose value is the extreme (CPU reducer: strict > / <).  Empty segments have no arg (-1).
template <int ACT, bool MAXR>
__global__ void __launch_bounds__(256) segment_arg_kernel(const float* __restrict__ X,
                                                          const int32_t* __restrict__ seg_ptr,
                                                          const int32_t* __restrict__ perm,
                                                          int64_t nseg, int64_t h, int act, float alpha,
                                                          int32_t* __restrict__ arg) {
  const int64_t total = nseg * h;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = t / h, c = t - v * h;
    const int32_t b = seg_ptr[v], en = seg_ptr[v + 1];
    int32_t best_r = -1;
    float best = 0.f;
    for (int32_t j = b; j < en; ++j) {
      const int32_t r = perm ? perm[j] : j;
      const float x = act_t<ACT>(X[(int64_t)r * h + c], act, alpha);
      if (best_r < 0 || (MAXR ? x > best : x < best)) {
        best = x;
        best_r = r;
      }
    }
    arg[t] = best_r;
  }
}

__device__ __forceinline__ float4 arg_mask(float4 x, int4 a, int64_t e) {
  return make_float4(a.x == e ? x.x : 0.f, a.y == e ? x.y : 0.f, a.z == e ? x.z : 0.f, a.w == e ? x.w : 0.f);
}
__device__ __forceinline__ float arg_mask(float x, int a, int64_t e) { return a == e ? x : 0.f; }

// edge backward with the dS term routed through the arg: dS[dst e] reaches row e only where e is
// the arg of (dst e, column)
template <typename T, typename TI, int ACT>
__global__ void __launch_bounds__(256) edge_backward_arg_kernel(
    const T* __restrict__ G, const T* __restrict__ H, const T* __restrict__ dA,
    const T* __restrict__ dS, const TI* __restrict__ arg, const int64_t* __restrict__ dst,
    const int32_t* __restrict__ rev_ptr, const int32_t* __restrict__ rev_perm, int64_t E, int64_t hw,
    int residual, int act, float alpha, T* __restrict__ Gout, float* __restrict__ amax) {
  const int64_t total = E * hw;
  float m = 0.f;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = t / hw, c = t - e * hw;
    const int64_t v = dst[e];
    T dm = arg_mask(dS[v * hw + c], arg[v * hw + c], e);
    const int32_t b = rev_ptr[e], en = rev_ptr[e + 1];
    for (int32_t j = b; j < en; ++j) dm = dm - dA[(int64_t)rev_perm[j] * hw + c];
    T g = vmul(vgrad<ACT>(H[t], act, alpha), dm);
    if (residual) g = g + G[t];
    Gout[t] = g;
    m = fmaxf(m, vamax(g));
  }
  if (amax) block_max_to(amax, m);
}

// out[i] = (base ? base[i] : 0) + (arg[idx i] == i ? X[idx i] : 0): backward of a max/min scatter
// of rows i into segments idx i (the final node scatter, the Max / Min readout)
template <typename T, typename TI>
__global__ void __launch_bounds__(256) gather_rows_arg_kernel(const T* __restrict__ base,
                                                              const T* __restrict__ X,
                                                              const int64_t* __restrict__ idx,
                                                              const TI* __restrict__ arg, int64_t n,
                                                              int64_t hw, T* __restrict__ out,
                                                              float* __restrict__ amax) {
  const int64_t total = n * hw;
  float m = 0.f;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t / hw, c = t - i * hw;
    const int64_t s = idx[i];
    const T x = arg_mask(X[s * hw + c], arg[s * hw + c], i);
    const T y = base ? base[t] + x : x;
    out[t] = y;
    m = fmaxf(m, vamax(y));
  }
  if (amax) block_max_to(amax, m);
}

// ---- bf16 storage (bf16 training): same math in fp32 registers, one rounding per stored element ----
template <bool VEC, int ACT>
__global__ void __launch_bounds__(256) message_bf16(const bf16_raw* __restrict__ H,
                                                    const bf16_raw* __restrict__ S,
                                                    const int64_t* __restrict__ src,
                                                    const int64_t* __restrict__ rev, int64_t E,
                                                    int64_t h, int act, float alpha,
                                                    bf16_raw* __restrict__ A) {
  using P = Piece<bf16_raw, VEC>;
  constexpr int N = P::N;
  const int64_t hw = h / N, total = E * hw;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = t / hw, c = (t - e * hw) * N;
    float sv[N], qv[N];
    P::load(S + src[e] * h + c, sv);
    P::load(H + rev[e] * h + c, qv);
#pragma unroll
    for (int i = 0; i < N; ++i) sv[i] -= act_t<ACT>(qv[i], act, alpha);
    P::store(A + e * h + c, sv);
  }
}

template <bool VEC, int ACT, bool MEAN>
__global__ void __launch_bounds__(256) edge_backward_bf16(
    const bf16_raw* __restrict__ G, const bf16_raw* __restrict__ H, const bf16_raw* __restrict__ dA,
    const bf16_raw* __restrict__ dS, const int64_t* __restrict__ dst,
    const int32_t* __restrict__ rev_ptr, const int32_t* __restrict__ rev_perm,
    const int32_t* __restrict__ dst_ptr, int64_t E, int64_t h, int residual, int act, float alpha,
    bf16_raw* __restrict__ Gout) {
  using P = Piece<bf16_raw, VEC>;
  constexpr int N = P::N;
  const int64_t hw = h / N, total = E * hw;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = t / hw, c = (t - e * hw) * N;
    const int64_t v = dst[e];
    float dm[N], x[N];
    P::load(dS + v * h + c, dm);
    if constexpr (MEAN) {
      const int cnt = dst_ptr[v + 1] - dst_ptr[v];
      const float inv = 1.f / (float)(cnt > 1 ? cnt : 1);
#pragma unroll
      for (int i = 0; i < N; ++i) dm[i] *= inv;
    }
    for (int32_t j = rev_ptr[e]; j < rev_ptr[e + 1]; ++j) {
      P::load(dA + (int64_t)rev_perm[j] * h + c, x);
#pragma unroll
      for (int i = 0; i < N; ++i) dm[i] -= x[i];
    }
    P::load(H + e * h + c, x);
#pragma unroll
    for (int i = 0; i < N; ++i) dm[i] *= act_grad_t<ACT>(x[i], act, alpha);
    if (residual) {
      P::load(G + e * h + c, x);
#pragma unroll
      for (int i = 0; i < N; ++i) dm[i] += x[i];
    }
    P::store(Gout + e * h + c, dm);
  }
}

template <bool VEC, bool MEAN>
__global__ void __launch_bounds__(256) gather_rows_bf16(const bf16_raw* __restrict__ base,
                                                        const bf16_raw* __restrict__ X,
                                                        const int64_t* __restrict__ idx,
                                                        const int32_t* __restrict__ seg_ptr,
                                                        int64_t n, int64_t h,
                                                        bf16_raw* __restrict__ out) {
  using P = Piece<bf16_raw, VEC>;
  constexpr int N = P::N;
  const int64_t hw = h / N, total = n * hw;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t / hw, c = (t - i * hw) * N;
    const int64_t s = idx[i];
    float x[N], b[N];
    P::load(X + s * h + c, x);
    if constexpr (MEAN) {
      const int cnt = seg_ptr[s + 1] - seg_ptr[s];
      const float inv = 1.f / (float)(cnt > 1 ? cnt : 1);
#pragma unroll
      for (int q = 0; q < N; ++q) x[q] *= inv;
    }
    if (base) {
      P::load(base + i * h + c, b);
#pragma unroll
      for (int q = 0; q < N; ++q) x[q] += b[q];
    }
    P::store(out + i * h + c, x);
  }
}

// ---- bf16 max / min backward: the fp32 arg kernels' math on bf16 storage (one element per lane; the
// values are widened exactly, compared and masked in fp32, rounded once at the store) ----
__device__ __forceinline__ float bf_ld(const bf16_raw* p) { return __uint_as_float((unsigned)*p << 16); }
__device__ __forceinline__ bf16_raw bf_st(float x) { return __builtin_bit_cast(bf16_raw, (__bf16)x); }

template <int ACT, bool MAXR>
__global__ void __launch_bounds__(256) segment_arg_bf16(const bf16_raw* __restrict__ X,
                                                        const int32_t* __restrict__ seg_ptr,
                                                        const int32_t* __restrict__ perm, int64_t nseg,
                                                        int64_t h, int act, float alpha,
                                                        int32_t* __restrict__ arg) {
  const int64_t total = nseg * h;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = t / h, c = t - v * h;
    const int32_t b = seg_ptr[v], en = seg_ptr[v + 1];
    int32_t best_r = -1;
    float best = 0.f;
    for (int32_t j = b; j < en; ++j) {
      const int32_t r = perm ? perm[j] : j;
      // the forward aggregates act(H) of the stored (bf16) H; act evaluated in fp32 as there
      const float x = act_t<ACT>(bf_ld(X + (int64_t)r * h + c), act, alpha);
      if (best_r < 0 || (MAXR ? x > best : x < best)) {
        best = x;
        best_r = r;
      }
    }
    arg[t] = best_r;
  }
}

template <int ACT>
__global__ void __launch_bounds__(256) edge_backward_arg_bf16(
    const bf16_raw* __restrict__ G, const bf16_raw* __restrict__ H, const bf16_raw* __restrict__ dA,
    const bf16_raw* __restrict__ dS, const int32_t* __restrict__ arg, const int64_t* __restrict__ dst,
    const int32_t* __restrict__ rev_ptr, const int32_t* __restrict__ rev_perm, int64_t E, int64_t h,
    int residual, int act, float alpha, bf16_raw* __restrict__ Gout) {
  const int64_t total = E * h;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = t / h, c = t - e * h;
    const int64_t v = dst[e];
    float dm = arg[v * h + c] == e ? bf_ld(dS + v * h + c) : 0.f;
    for (int32_t j = rev_ptr[e]; j < rev_ptr[e + 1]; ++j) dm -= bf_ld(dA + (int64_t)rev_perm[j] * h + c);
    float g = act_grad_t<ACT>(bf_ld(H + t), act, alpha) * dm;
    if (residual) g += bf_ld(G + t);
    Gout[t] = bf_st(g);
  }
}

__global__ void __launch_bounds__(256) gather_rows_arg_bf16(const bf16_raw* __restrict__ base,
                                                            const bf16_raw* __restrict__ X,
                                                            const int64_t* __restrict__ idx,
                                                            const int32_t* __restrict__ arg, int64_t n,
                                                            int64_t h, bf16_raw* __restrict__ out) {
  const int64_t total = n * h;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t / h, c = t - i * h;
    const int64_t s = idx[i];
    const float x = arg[s * h + c] == i ? bf_ld(X + s * h + c) : 0.f;
    out[t] = bf_st(base ? bf_ld(base + t) + x : x);
  }
}

static bool valid_act(int a) { return a >= NT_ACT_IDENTITY && a <= NT_ACT_SIGMOID; }

#define NT_BW_DISPATCH_ACT(ACT, LAUNCH)                                          \
  do {                                                                           \
    if ((ACT) == NT_ACT_IDENTITY) { constexpr int A_ = NT_ACT_IDENTITY; LAUNCH; } \
    else if ((ACT) == NT_ACT_RELU) { constexpr int A_ = NT_ACT_RELU; LAUNCH; }    \
    else { constexpr int A_ = -1; LAUNCH; }                                      \
  } while (0)

}  // namespace nt

extern "C" int nt_dmpnn_message(const void* H, const void* S, const int64_t* src, const int64_t* rev,
                                int64_t V, int64_t E, int64_t h, int act, float act_alpha, int dtype,
                                void* A_out, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32 || dtype == NT_BF16, NT_EUNSUPPORTED, "dtype must be NT_F32 or NT_BF16");
  NT_REQUIRE(valid_act(act), NT_EINVAL, "bad act code");
  NT_REQUIRE(V >= 0 && E >= 0 && h > 0, NT_EINVAL, "bad sizes");
  if (E == 0) return NT_OK;
  NT_REQUIRE(H && S && src && rev && A_out, NT_EINVAL, "NULL pointer");
  hipStream_t stream = as_stream(stream_);
  if (dtype == NT_BF16) {
    const bool vec = h % 8 == 0 && aligned16(H) && aligned16(S) && aligned16(A_out);
    const int grid = grid_for(E * (vec ? h / 8 : h), 256, 256 * 32);
    if (vec)
      NT_BW_DISPATCH_ACT(act, (message_bf16<true, A_><<<grid, 256, 0, stream>>>(
                                  (const bf16_raw*)H, (const bf16_raw*)S, src, rev, E, h, act,
                                  act_alpha, (bf16_raw*)A_out)));
    else
      NT_BW_DISPATCH_ACT(act, (message_bf16<false, A_><<<grid, 256, 0, stream>>>(
                                  (const bf16_raw*)H, (const bf16_raw*)S, src, rev, E, h, act,
                                  act_alpha, (bf16_raw*)A_out)));
    NT_LAUNCH_CHECK();
    return NT_OK;
  }
  if (h % 4 == 0 && aligned16(H) && aligned16(S) && aligned16(A_out)) {
    const int64_t hw = h / 4;
    NT_BW_DISPATCH_ACT(act, (message_kernel<float4, A_><<<grid_for(E * hw, 256, 256 * 32), 256, 0, stream>>>(
                                (const float4*)H, (const float4*)S, src, rev, E, hw, act, act_alpha,
                                (float4*)A_out)));
  } else {
    NT_BW_DISPATCH_ACT(act, (message_kernel<float, A_><<<grid_for(E * h, 256, 256 * 32), 256, 0, stream>>>(
                                (const float*)H, (const float*)S, src, rev, E, h, act, act_alpha,
                                (float*)A_out)));
  }
  NT_LAUNCH_CHECK();
  return NT_OK;
}

extern "C" int nt_dmpnn_edge_backward(const void* G, const void* H, const void* dA, const void* dS,
                                      const int64_t* dst, const int32_t* rev_ptr,
                                      const int32_t* rev_perm, const int32_t* dst_ptr, int64_t V,
                                      int64_t E, int64_t h, int residual, int act, float act_alpha,
                                      int reduce, int dtype, void* G_out, float* amax_out, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32 || dtype == NT_BF16, NT_EUNSUPPORTED, "dtype must be NT_F32 or NT_BF16");
  NT_REQUIRE(valid_act(act), NT_EINVAL, "bad act code");
  NT_REQUIRE(reduce == NT_SUM || reduce == NT_MEAN, NT_EUNSUPPORTED,
             "edge backward covers reduce = sum | mean");
  NT_REQUIRE(V >= 0 && E >= 0 && h > 0, NT_EINVAL, "bad sizes");
  if (E == 0) return NT_OK;
  NT_REQUIRE(H && dA && dS && dst && rev_ptr && rev_perm && G_out, NT_EINVAL, "NULL pointer");
  NT_REQUIRE(!residual || G, NT_EINVAL, "residual needs G");
  NT_REQUIRE(reduce != NT_MEAN || dst_ptr, NT_EINVAL, "mean needs the dst CSR");
  hipStream_t stream = as_stream(stream_);
  const bool mean = reduce == NT_MEAN;
  if (dtype == NT_BF16) {
    const bool vec = h % 8 == 0 && aligned16(H) && aligned16(dA) && aligned16(dS) &&
                     aligned16(G_out) && (!residual || aligned16(G));
    const int grid = grid_for(E * (vec ? h / 8 : h), 256, 256 * 32);
#define NT_EB16(VEC_, MEAN_)                                                                        \
  NT_BW_DISPATCH_ACT(act, (edge_backward_bf16<VEC_, A_, MEAN_><<<grid, 256, 0, stream>>>(           \
                              (const bf16_raw*)G, (const bf16_raw*)H, (const bf16_raw*)dA,          \
                              (const bf16_raw*)dS, dst, rev_ptr, rev_perm, dst_ptr, E, h, residual, \
                              act, act_alpha, (bf16_raw*)G_out)))
    if (vec) { if (mean) NT_EB16(true, true); else NT_EB16(true, false); }
    else { if (mean) NT_EB16(false, true); else NT_EB16(false, false); }
#undef NT_EB16
    NT_LAUNCH_CHECK();
    return NT_OK;
  }
  if (h % 4 == 0 && aligned16(H) && aligned16(dA) && aligned16(dS) && aligned16(G_out) &&
      (!residual || aligned16(G))) {
    const int64_t hw = h / 4;
    const int grid = grid_for(E * hw, 256, 256 * 32);
#define NT_EB_LAUNCH(MEAN_)                                                                       \
  NT_BW_DISPATCH_ACT(act, (edge_backward_kernel<float4, A_, MEAN_><<<grid, 256, 0, stream>>>(     \
                              (const float4*)G, (const float4*)H, (const float4*)dA,              \
                              (const float4*)dS, dst, rev_ptr, rev_perm, dst_ptr, E, hw, residual, \
                              act, act_alpha, (float4*)G_out, amax_out)))
    if (mean) NT_EB_LAUNCH(true); else NT_EB_LAUNCH(false);
#undef NT_EB_LAUNCH
  } else {
    const int grid = grid_for(E * h, 256, 256 * 32);
#define NT_EB_LAUNCH(MEAN_)                                                                     \
  NT_BW_DISPATCH_ACT(act, (edge_backward_kernel<float, A_, MEAN_><<<grid, 256, 0, stream>>>(    \
                              (const float*)G, (const float*)H, (const float*)dA, (const float*)dS, \
                              dst, rev_ptr, rev_perm, dst_ptr, E, h, residual, act, act_alpha,   \
                              (float*)G_out, amax_out)))
    if (mean) NT_EB_LAUNCH(true); else NT_EB_LAUNCH(false);
#undef NT_EB_LAUNCH
  }
  NT_LAUNCH_CHECK();
  return NT_OK;
}

extern "C" int nt_gather_rows(const void* base, const void* X, const int64_t* idx,
                              const int32_t* seg_ptr, int64_t n, int64_t nseg, int64_t h, int dtype,
                              void* out, float* amax_out, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32 || dtype == NT_BF16, NT_EUNSUPPORTED, "dtype must be NT_F32 or NT_BF16");
  NT_REQUIRE(n >= 0 && nseg >= 0 && h > 0, NT_EINVAL, "bad sizes");
  if (n == 0) return NT_OK;
  NT_REQUIRE(X && idx && out, NT_EINVAL, "NULL pointer");
  hipStream_t stream = as_stream(stream_);
  const bool mean = seg_ptr != nullptr;
  if (dtype == NT_BF16) {
    const bool vec = h % 8 == 0 && aligned16(X) && aligned16(out) && (!base || aligned16(base));
    const int grid = grid_for(n * (vec ? h / 8 : h), 256, 256 * 32);
    const bf16_raw* b16 = (const bf16_raw*)base;
    const bf16_raw* x16 = (const bf16_raw*)X;
    bf16_raw* o16 = (bf16_raw*)out;
    if (vec && mean) gather_rows_bf16<true, true><<<grid, 256, 0, stream>>>(b16, x16, idx, seg_ptr, n, h, o16);
    else if (vec) gather_rows_bf16<true, false><<<grid, 256, 0, stream>>>(b16, x16, idx, seg_ptr, n, h, o16);
    else if (mean) gather_rows_bf16<false, true><<<grid, 256, 0, stream>>>(b16, x16, idx, seg_ptr, n, h, o16);
    else gather_rows_bf16<false, false><<<grid, 256, 0, stream>>>(b16, x16, idx, seg_ptr, n, h, o16);
    NT_LAUNCH_CHECK();
    return NT_OK;
  }
  if (h % 4 == 0 && aligned16(X) && aligned16(out) && (!base || aligned16(base))) {
    const int64_t hw = h / 4;
    const int grid = grid_for(n * hw, 256, 256 * 32);
    if (mean)
      gather_rows_kernel<float4, true><<<grid, 256, 0, stream>>>(
          (const float4*)base, (const float4*)X, idx, seg_ptr, n, hw, (float4*)out, amax_out);
    else
      gather_rows_kernel<float4, false><<<grid, 256, 0, stream>>>(
          (const float4*)base, (const float4*)X, idx, seg_ptr, n, hw, (float4*)out, amax_out);
  } else {
    const int grid = grid_for(n * h, 256, 256 * 32);
    if (mean)
      gather_rows_kernel<float, true><<<grid, 256, 0, stream>>>(
          (const float*)base, (const float*)X, idx, seg_ptr, n, h, (float*)out, amax_out);
    else
      gather_rows_kernel<float, false><<<grid, 256, 0, stream>>>(
          (const float*)base, (const float*)X, idx, seg_ptr, n, h, (float*)out, amax_out);
  }
  NT_LAUNCH_CHECK();
  return NT_OK;
}

extern "C" int nt_segment_arg(const void* X, const int32_t* seg_ptr, const int32_t* perm, int64_t nseg,
                              int64_t h, int reduce, int act, float act_alpha, int dtype, int32_t* arg,
                              void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32 || dtype == NT_BF16, NT_EUNSUPPORTED, "dtype must be NT_F32 or NT_BF16");
  NT_REQUIRE(reduce == NT_MAX || reduce == NT_MIN, NT_EINVAL, "nt_segment_arg: reduce must be max or min");
  NT_REQUIRE(valid_act(act), NT_EINVAL, "bad act code");
  NT_REQUIRE(nseg >= 0 && h > 0, NT_EINVAL, "bad sizes");
  if (nseg == 0) return NT_OK;
  NT_REQUIRE(X && seg_ptr && arg, NT_EINVAL, "NULL pointer");
  hipStream_t stream = as_stream(stream_);
  const int grid = grid_for(nseg * h, 256, 256 * 32);
  if (dtype == NT_BF16) {
#define NT_SA(MAXR_)                                                                          \
  NT_BW_DISPATCH_ACT(act, (segment_arg_bf16<A_, MAXR_><<<grid, 256, 0, stream>>>(             \
                              (const bf16_raw*)X, seg_ptr, perm, nseg, h, act, act_alpha, arg)))
    if (reduce == NT_MAX) NT_SA(true); else NT_SA(false);
#undef NT_SA
    NT_LAUNCH_CHECK();
    return NT_OK;
  }
#define NT_SA(MAXR_)                                                                          \
  NT_BW_DISPATCH_ACT(act, (segment_arg_kernel<A_, MAXR_><<<grid, 256, 0, stream>>>(           \
                              (const float*)X, seg_ptr, perm, nseg, h, act, act_alpha, arg)))
  if (reduce == NT_MAX) NT_SA(true); else NT_SA(false);
#undef NT_SA
  NT_LAUNCH_CHECK();
  return NT_OK;
}

extern "C" int nt_dmpnn_edge_backward_arg(const void* G, const void* H, const void* dA, const void* dS,
                                          const int32_t* arg, const int64_t* dst,
                                          const int32_t* rev_ptr, const int32_t* rev_perm, int64_t V,
                                          int64_t E, int64_t h, int residual, int act, float act_alpha,
                                          int dtype, void* G_out, float* amax_out, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32 || dtype == NT_BF16, NT_EUNSUPPORTED, "dtype must be NT_F32 or NT_BF16");
  NT_REQUIRE(valid_act(act), NT_EINVAL, "bad act code");
  NT_REQUIRE(V >= 0 && E >= 0 && h > 0, NT_EINVAL, "bad sizes");
  if (E == 0) return NT_OK;
  NT_REQUIRE(H && dA && dS && arg && dst && rev_ptr && rev_perm && G_out, NT_EINVAL, "NULL pointer");
  NT_REQUIRE(!residual || G, NT_EINVAL, "residual needs G");
  hipStream_t stream = as_stream(stream_);
  if (dtype == NT_BF16) {
    NT_REQUIRE(amax_out == nullptr, NT_EINVAL, "amax_out is fp32 only");
    const int grid = grid_for(E * h, 256, 256 * 32);
    NT_BW_DISPATCH_ACT(act, (edge_backward_arg_bf16<A_><<<grid, 256, 0, stream>>>(
                                (const bf16_raw*)G, (const bf16_raw*)H, (const bf16_raw*)dA,
                                (const bf16_raw*)dS, arg, dst, rev_ptr, rev_perm, E, h, residual, act,
                                act_alpha, (bf16_raw*)G_out)));
    NT_LAUNCH_CHECK();
    return NT_OK;
  }
  if (h % 4 == 0 && aligned16(H) && aligned16(dA) && aligned16(dS) && aligned16(G_out) &&
      aligned16(arg) && (!residual || aligned16(G))) {
    const int64_t hw = h / 4;
    const int grid = grid_for(E * hw, 256, 256 * 32);
    NT_BW_DISPATCH_ACT(act, (edge_backward_arg_kernel<float4, int4, A_><<<grid, 256, 0, stream>>>(
                                (const float4*)G, (const float4*)H, (const float4*)dA, (const float4*)dS,
                                (const int4*)arg, dst, rev_ptr, rev_perm, E, hw, residual, act,
                                act_alpha, (float4*)G_out, amax_out)));
  } else {
    const int grid = grid_for(E * h, 256, 256 * 32);
    NT_BW_DISPATCH_ACT(act, (edge_backward_arg_kernel<float, int, A_><<<grid, 256, 0, stream>>>(
                                (const float*)G, (const float*)H, (const float*)dA, (const float*)dS,
                                arg, dst, rev_ptr, rev_perm, E, h, residual, act, act_alpha,
                                (float*)G_out, amax_out)));
  }
  NT_LAUNCH_CHECK();
  return NT_OK;
}

extern "C" int nt_gather_rows_arg(const void* base, const void* X, const int64_t* idx, const int32_t* arg,
                                  int64_t n, int64_t h, int dtype, void* out, float* amax_out, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32 || dtype == NT_BF16, NT_EUNSUPPORTED, "dtype must be NT_F32 or NT_BF16");
  NT_REQUIRE(n >= 0 && h > 0, NT_EINVAL, "bad sizes");
  if (n == 0) return NT_OK;
  NT_REQUIRE(X && idx && arg && out, NT_EINVAL, "NULL pointer");
  hipStream_t stream = as_stream(stream_);
  if (dtype == NT_BF16) {
    NT_REQUIRE(amax_out == nullptr, NT_EINVAL, "amax_out is fp32 only");
    gather_rows_arg_bf16<<<grid_for(n * h, 256, 256 * 32), 256, 0, stream>>>(
        (const bf16_raw*)base, (const bf16_raw*)X, idx, arg, n, h, (bf16_raw*)out);
    NT_LAUNCH_CHECK();
    return NT_OK;
  }
  if (h % 4 == 0 && aligned16(X) && aligned16(out) && aligned16(arg) && (!base || aligned16(base))) {
    const int64_t hw = h / 4;
    gather_rows_arg_kernel<float4, int4><<<grid_for(n * hw, 256, 256 * 32), 256, 0, stream>>>(
        (const float4*)base, (const float4*)X, idx, (const int4*)arg, n, hw, (float4*)out, amax_out);
  } else {
    gather_rows_arg_kernel<float, int><<<grid_for(n * h, 256, 256 * 32), 256, 0, stream>>>(
        (const float*)base, (const float*)X, idx, arg, n, h, (float*)out, amax_out);
  }
  NT_LAUNCH_CHECK();
  return NT_OK;
}

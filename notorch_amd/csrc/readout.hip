// Attention readouts (notorch/nn/gnn/agg.py:50-86): a per-molecule softmax of
// node scores weighting a segmented sum of the node rows.
//
//   nt_node_scores        s[v] = X[v] . a + a_bias            (Gated.a = nn.Linear(d, 1), agg.py:53,59)
//                         s[v] = (Q[g(v)] . X[v]) / sqrt_key  (SDPAttention, agg.py:79-82)
//   nt_softmax_pool       out[g] = sum_{v in g} alpha[v] X[v],
//                         alpha = scatter_softmax(s, batch) (torch_scatter composite/softmax.py:
//                         exp(s - max_g) / sum_g exp(s - max_g); agg.py:60-61, :83-84)
//
// nt_node_scores: one wave per node row (lanes over 16-B pieces, butterfly reduction), rows are
// read once.  nt_softmax_pool: one lane per (molecule, column piece); the molecule's max and
// normaliser are recomputed per lane from the score vector (tiny, L1/L2-resident) in ascending node
// order, then alpha[v] * X[v] is accumulated in ascending node order — the CPU order of the
// reference's scatter_sum.  Both are HBM-bound on the V x h rows (read once each).
#include <math.h>

#include "rows.hpp"

namespace nt {
namespace {

template <typename T, bool VEC, bool SDPA>
__global__ void __launch_bounds__(256) node_scores_kernel(
    const T* __restrict__ X, const int32_t* __restrict__ seg_ptr, const int32_t* __restrict__ perm,
    const int64_t* __restrict__ node_seg, int64_t n, int64_t h, const T* __restrict__ a,
    const T* __restrict__ a_bias, const T* __restrict__ Q, float sqrt_key, float* __restrict__ s) {
  constexpr int N = Piece<T, VEC>::N;
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t v = wave; v < n; v += nwaves) {
    const T* q = a;
    if constexpr (SDPA) q = Q + node_seg[v] * h;
    float part = 0.f;
    for (int64_t c = (int64_t)lane * N; c < h; c += 64 * N) {
      float x[N], y[N];
      Piece<T, VEC>::load(X + v * h + c, x);
      Piece<T, VEC>::load(q + c, y);
#pragma unroll
      for (int i = 0; i < N; ++i) part = fmaf(x[i], y[i], part);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off);
    if (lane == 0) {
      float sc = part;
      if constexpr (SDPA) {
        sc = sc / sqrt_key;
      } else if (a_bias) {
        float bb[1];
        Piece<T, false>::load(a_bias, bb);
        sc += bb[0];
      }
      s[v] = sc;
    }
  }
}

template <typename T, bool VEC>
__global__ void __launch_bounds__(256) softmax_pool_kernel(
    const T* __restrict__ X, const float* __restrict__ s, const int32_t* __restrict__ seg_ptr,
    const int32_t* __restrict__ perm, int64_t nseg, int64_t h, T* __restrict__ out) {
  constexpr int N = Piece<T, VEC>::N;
  const int64_t hw = h / N;
  const int64_t total = nseg * hw;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t g = t / hw, c = (t - g * hw) * N;
    const int32_t b = seg_ptr[g], e = seg_ptr[g + 1];
    float m = -INFINITY;
    for (int32_t j = b; j < e; ++j) m = fmaxf(m, s[perm ? perm[j] : j]);
    float z = 0.f;
    for (int32_t j = b; j < e; ++j) z += expf(s[perm ? perm[j] : j] - m);
    float acc[N];
#pragma unroll
    for (int i = 0; i < N; ++i) acc[i] = 0.f;
    for (int32_t j = b; j < e; ++j) {
      const int64_t v = perm ? perm[j] : j;
      const float alpha = expf(s[v] - m) / z;
      float x[N];
      Piece<T, VEC>::load(X + v * h + c, x);
#pragma unroll
      for (int i = 0; i < N; ++i) acc[i] += alpha * x[i];
    }
    Piece<T, VEC>::store(out + g * h + c, acc);
  }
}

// ---- backward (agg.py:50-86 under autograd: the model's training_step, model.py:224-241) ----
// With alpha_v = softmax_g(s)_v and out[g] = sum_v alpha_v X[v], for dout[g]:
//   dalpha_v = <dout[g], X[v]>,  c_g = <dout[g], out[g]> = sum_v alpha_v dalpha_v
//   ds_v     = alpha_v (dalpha_v - c_g)                         (softmax backward)
//   dX[v]    = alpha_v dout[g] + ds_v key_v                      (key = a: Gated; Q[g] / sqrt_key: SDPA)
//   P[g]     = sum_{v in g} ds_v X[v]                            (Gated: da = sum_g P[g], db = sum_v ds_v;
//                                                                SDPA: dQ[g] = P[g] / sqrt_key)
// Three launches: per molecule (m_g, z_g, c_g) on one wave (m and z recomputed exactly as the
// forward's lanes do, so alpha is bit-identical); per node dX and ds on one wave; P as the forward's
// pool with the weights ds in place of alpha (ascending node order).
template <typename T, bool VEC>
__global__ void __launch_bounds__(256) pool_stats_kernel(
    const float* __restrict__ s, const int32_t* __restrict__ seg_ptr, const int32_t* __restrict__ perm,
    const T* __restrict__ out, const T* __restrict__ dout, int64_t nseg, int64_t h,
    float* __restrict__ stats) {
  constexpr int N = Piece<T, VEC>::N;
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t g = wave; g < nseg; g += nwaves) {
    const int32_t b = seg_ptr[g], e = seg_ptr[g + 1];
    float m = -INFINITY;
    for (int32_t j = b; j < e; ++j) m = fmaxf(m, s[perm ? perm[j] : j]);
    float z = 0.f;
    for (int32_t j = b; j < e; ++j) z += expf(s[perm ? perm[j] : j] - m);
    float part = 0.f;
    for (int64_t c = (int64_t)lane * N; c < h; c += 64 * N) {
      float x[N], y[N];
      Piece<T, VEC>::load(out + g * h + c, x);
      Piece<T, VEC>::load(dout + g * h + c, y);
#pragma unroll
      for (int i = 0; i < N; ++i) part = fmaf(x[i], y[i], part);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off);
    if (lane == 0) {
      stats[3 * g] = m;
      stats[3 * g + 1] = z;
      stats[3 * g + 2] = part;
    }
  }
}

template <typename T, bool VEC, bool SDPA>
__global__ void __launch_bounds__(256) pool_node_backward_kernel(
    const T* __restrict__ X, const float* __restrict__ s, const int64_t* __restrict__ node_seg,
    const float* __restrict__ stats, const T* __restrict__ dout, int64_t n, int64_t h,
    const T* __restrict__ a, const T* __restrict__ Q, float sqrt_key, T* __restrict__ dX,
    float* __restrict__ ds) {
  constexpr int N = Piece<T, VEC>::N;
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t v = wave; v < n; v += nwaves) {
    const int64_t g = node_seg[v];
    const float alpha = expf(s[v] - stats[3 * g]) / stats[3 * g + 1];
    float part = 0.f;
    for (int64_t c = (int64_t)lane * N; c < h; c += 64 * N) {
      float x[N], y[N];
      Piece<T, VEC>::load(X + v * h + c, x);
      Piece<T, VEC>::load(dout + g * h + c, y);
#pragma unroll
      for (int i = 0; i < N; ++i) part = fmaf(x[i], y[i], part);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off);
    const float dsv = alpha * (part - stats[3 * g + 2]);
    for (int64_t c = (int64_t)lane * N; c < h; c += 64 * N) {
      float k[N], y[N], o[N];
      Piece<T, VEC>::load(dout + g * h + c, y);
      if constexpr (SDPA) {
        Piece<T, VEC>::load(Q + g * h + c, k);
#pragma unroll
        for (int i = 0; i < N; ++i) k[i] /= sqrt_key;
      } else {
        Piece<T, VEC>::load(a + c, k);
      }
#pragma unroll
      for (int i = 0; i < N; ++i) o[i] = fmaf(alpha, y[i], dsv * k[i]);
      Piece<T, VEC>::store(dX + v * h + c, o);
    }
    if (lane == 0) ds[v] = dsv;
  }
}

// P[g] = sum_{v in g} w[v] X[v] (fp32 out), ascending node order
template <typename T, bool VEC>
__global__ void __launch_bounds__(256) weighted_pool_kernel(
    const T* __restrict__ X, const float* __restrict__ w, const int32_t* __restrict__ seg_ptr,
    const int32_t* __restrict__ perm, int64_t nseg, int64_t h, float* __restrict__ P) {
  constexpr int N = Piece<T, VEC>::N;
  const int64_t hw = h / N;
  const int64_t total = nseg * hw;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t g = t / hw, c = (t - g * hw) * N;
    float acc[N];
#pragma unroll
    for (int i = 0; i < N; ++i) acc[i] = 0.f;
    for (int32_t j = seg_ptr[g]; j < seg_ptr[g + 1]; ++j) {
      const int64_t v = perm ? perm[j] : j;
      float x[N];
      Piece<T, VEC>::load(X + v * h + c, x);
#pragma unroll
      for (int i = 0; i < N; ++i) acc[i] = fmaf(w[v], x[i], acc[i]);
    }
#pragma unroll
    for (int i = 0; i < N; ++i) P[g * h + c + i] = acc[i];
  }
}

template <typename T, bool VEC>
int launch_pool_backward(const void* X, const float* s, const int32_t* seg_ptr, const int32_t* perm,
                         const int64_t* node_seg, int64_t nseg, int64_t n, int64_t h, const void* out,
                         const void* dout, const void* a, const void* Q, float sqrt_key, float* stats,
                         void* dX, float* ds, float* P, hipStream_t stream) {
  constexpr int N = Piece<T, VEC>::N;
  pool_stats_kernel<T, VEC><<<grid_for(nseg * 64, 256, 256 * 32), 256, 0, stream>>>(
      s, seg_ptr, perm, (const T*)out, (const T*)dout, nseg, h, stats);
  NT_LAUNCH_CHECK();
  if (n > 0) {
    const int grid = grid_for(n * 64, 256, 256 * 32);
    if (Q)
      pool_node_backward_kernel<T, VEC, true><<<grid, 256, 0, stream>>>(
          (const T*)X, s, node_seg, stats, (const T*)dout, n, h, nullptr, (const T*)Q, sqrt_key, (T*)dX, ds);
    else
      pool_node_backward_kernel<T, VEC, false><<<grid, 256, 0, stream>>>(
          (const T*)X, s, node_seg, stats, (const T*)dout, n, h, (const T*)a, nullptr, 1.f, (T*)dX, ds);
    NT_LAUNCH_CHECK();
  }
  weighted_pool_kernel<T, VEC><<<grid_for(nseg * (h / N), 256, 256 * 32), 256, 0, stream>>>(
      (const T*)X, ds, seg_ptr, perm, nseg, h, P);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

template <typename T, bool VEC>
int launch_scores(const void* X, const int64_t* node_seg, int64_t n, int64_t h, const void* a,
                  const void* a_bias, const void* Q, float sqrt_key, float* s, hipStream_t stream) {
  const int grid = grid_for(n * 64, 256, 256 * 32);
  if (Q)
    node_scores_kernel<T, VEC, true><<<grid, 256, 0, stream>>>(
        (const T*)X, nullptr, nullptr, node_seg, n, h, nullptr, nullptr, (const T*)Q, sqrt_key, s);
  else
    node_scores_kernel<T, VEC, false><<<grid, 256, 0, stream>>>(
        (const T*)X, nullptr, nullptr, nullptr, n, h, (const T*)a, (const T*)a_bias, nullptr, 1.f, s);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

template <typename T, bool VEC>
int launch_pool(const void* X, const float* s, const int32_t* seg_ptr, const int32_t* perm,
                int64_t nseg, int64_t h, void* out, hipStream_t stream) {
  constexpr int N = Piece<T, VEC>::N;
  softmax_pool_kernel<T, VEC><<<grid_for(nseg * (h / N), 256, 256 * 32), 256, 0, stream>>>(
      (const T*)X, s, seg_ptr, perm, nseg, h, (T*)out);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

}  // namespace
}  // namespace nt

extern "C" int nt_node_scores(const void* X, int64_t n, int64_t h, const void* a, const void* a_bias,
                              const void* Q, const int64_t* node_seg, float sqrt_key, int dtype,
                              float* scores, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32 || dtype == NT_BF16, NT_EUNSUPPORTED, "dtype must be NT_F32 or NT_BF16");
  NT_REQUIRE(n >= 0 && h > 0, NT_EINVAL, "bad sizes");
  NT_REQUIRE((a == nullptr) != (Q == nullptr), NT_EINVAL, "exactly one of a (Gated) and Q (SDPA)");
  NT_REQUIRE(Q == nullptr || (node_seg && sqrt_key > 0.f), NT_EINVAL, "SDPA needs node_seg, sqrt_key > 0");
  if (n == 0) return NT_OK;
  NT_REQUIRE(X && scores, NT_EINVAL, "NULL pointer");
  hipStream_t stream = as_stream(stream_);
  const bool al = aligned16(X) && aligned16(a ? a : Q);
  if (dtype == NT_F32)
    return (h % 4 == 0 && al) ? launch_scores<float, true>(X, node_seg, n, h, a, a_bias, Q, sqrt_key, scores, stream)
                              : launch_scores<float, false>(X, node_seg, n, h, a, a_bias, Q, sqrt_key, scores, stream);
  return (h % 8 == 0 && al) ? launch_scores<bf16_raw, true>(X, node_seg, n, h, a, a_bias, Q, sqrt_key, scores, stream)
                            : launch_scores<bf16_raw, false>(X, node_seg, n, h, a, a_bias, Q, sqrt_key, scores, stream);
}

extern "C" int nt_softmax_pool(const void* X, const float* scores, const int32_t* seg_ptr,
                               const int32_t* perm, int64_t nseg, int64_t h, int dtype, void* out,
                               void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32 || dtype == NT_BF16, NT_EUNSUPPORTED, "dtype must be NT_F32 or NT_BF16");
  NT_REQUIRE(nseg >= 0 && h > 0, NT_EINVAL, "bad sizes");
  if (nseg == 0) return NT_OK;
  NT_REQUIRE(X && scores && seg_ptr && out, NT_EINVAL, "NULL pointer");
  hipStream_t stream = as_stream(stream_);
  const bool al = aligned16(X) && aligned16(out);
  if (dtype == NT_F32)
    return (h % 4 == 0 && al) ? launch_pool<float, true>(X, scores, seg_ptr, perm, nseg, h, out, stream)
                              : launch_pool<float, false>(X, scores, seg_ptr, perm, nseg, h, out, stream);
  return (h % 8 == 0 && al) ? launch_pool<bf16_raw, true>(X, scores, seg_ptr, perm, nseg, h, out, stream)
                            : launch_pool<bf16_raw, false>(X, scores, seg_ptr, perm, nseg, h, out, stream);
}

extern "C" int nt_softmax_pool_backward(const void* X, const float* scores, const int32_t* seg_ptr,
                                        const int32_t* perm, const int64_t* node_seg, int64_t nseg,
                                        int64_t n, int64_t h, const void* out, const void* dout,
                                        const void* a, const void* Q, float sqrt_key, int dtype,
                                        float* stats, void* dX, float* ds, float* P, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32 || dtype == NT_BF16, NT_EUNSUPPORTED, "dtype must be NT_F32 or NT_BF16");
  NT_REQUIRE(nseg >= 0 && n >= 0 && h > 0, NT_EINVAL, "bad sizes");
  NT_REQUIRE((a == nullptr) != (Q == nullptr), NT_EINVAL, "exactly one of a (Gated) and Q (SDPA)");
  NT_REQUIRE(Q == nullptr || sqrt_key > 0.f, NT_EINVAL, "SDPA needs sqrt_key > 0");
  if (nseg == 0) return NT_OK;
  NT_REQUIRE(X && scores && seg_ptr && node_seg && out && dout && stats && dX && ds && P, NT_EINVAL,
             "NULL pointer");
  hipStream_t stream = as_stream(stream_);
  const bool al = aligned16(X) && aligned16(out) && aligned16(dout) && aligned16(dX) && aligned16(a ? a : Q);
  if (dtype == NT_F32)
    return (h % 4 == 0 && al)
               ? launch_pool_backward<float, true>(X, scores, seg_ptr, perm, node_seg, nseg, n, h, out, dout, a, Q,
                                                   sqrt_key, stats, dX, ds, P, stream)
               : launch_pool_backward<float, false>(X, scores, seg_ptr, perm, node_seg, nseg, n, h, out, dout, a,
                                                    Q, sqrt_key, stats, dX, ds, P, stream);
  return (h % 8 == 0 && al)
             ? launch_pool_backward<bf16_raw, true>(X, scores, seg_ptr, perm, node_seg, nseg, n, h, out, dout, a,
                                                    Q, sqrt_key, stats, dX, ds, P, stream)
             : launch_pool_backward<bf16_raw, false>(X, scores, seg_ptr, perm, node_seg, nseg, n, h, out, dout, a,
                                                     Q, sqrt_key, stats, dX, ds, P, stream);
}

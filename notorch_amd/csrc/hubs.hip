// Hub nodes in the fused fp32 layer (polymer graphs, BASELINE config 5): nodes whose in-degree
// exceeds a hub degree (32) do not fit a node-aligned tile, so the tile plan cuts them at the stride
// (nt_dmpnn_tile_plan_hubs), the fused kernel stores their rows' H_out but no S_out
// (nt_dmpnn_mark_hub_rows turns off their rows' "last in-edge" flags), and one small launch per layer
// reduces the hubs' in-edges (nt_dmpnn_hub_aggregate).  Only tiles that touch a hub lose their
// fused aggregation; every other node keeps it (the rest of the layout still runs d + 1 launches).
//
//   S_out[v] = reduce_{e: dst[e] = v} act(X[e])     for the listed hub nodes v   (chemprop.py:37-39,
//                                                                                  :86; torch_scatter)
#include <float.h>

#include "common.hpp"

namespace nt {
namespace {

constexpr int kHubWaves = 16;  // waves per workgroup: each reduces a contiguous 1/16 of the in-edges
constexpr int kHubBatch = 8;  // rows in flight per lane

template <int R>
__device__ __forceinline__ float4 hub_identity() {
  if constexpr (R == NT_MAX) return make_float4(-FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX);
  else if constexpr (R == NT_MIN) return make_float4(FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX);
  else return make_float4(0.f, 0.f, 0.f, 0.f);
}

template <int R>
__device__ __forceinline__ float hub_op(float a, float x) {
  if constexpr (R == NT_MAX) return x > a ? x : a;
  else if constexpr (R == NT_MIN) return x < a ? x : a;
  else return a + x;
}

template <int R>
__device__ __forceinline__ float4 hub_op4(float4 a, float4 x) {
  return make_float4(hub_op<R>(a.x, x.x), hub_op<R>(a.y, x.y), hub_op<R>(a.z, x.z), hub_op<R>(a.w, x.w));
}

// grid (nhub, nslab), 1024 threads.  Slab j holds pieces [j P, (j + 1) P) of the hv 16-B pieces of a
// row (P = ceil(hv / nslab) <= 64, one per lane).  Wave w reduces rows [b + w n / 16, b + (w + 1) n / 16)
// of the hub's CSR range in ascending order with kHubBatch row loads in flight (indices clamped, the
// loads unconditional); the 16 partials combine in wave order through LDS (deterministic).
template <int R, int ACT>
__global__ void __launch_bounds__(kHubWaves * 64) hub_aggregate_kernel(
    const float4* __restrict__ X, const int32_t* __restrict__ perm, const int32_t* __restrict__ seg_ptr,
    const int32_t* __restrict__ hubs, int hv, int P, int act, float alpha, float4* __restrict__ out,
    float* __restrict__ amax, int ld) {  // ld: row pitch of X and out in 16-B pieces
  __shared__ float4 part[kHubWaves][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int s = hubs[blockIdx.x];
  const int32_t b = seg_ptr[s], n = seg_ptr[s + 1] - b;
  const int c = blockIdx.y * P + lane;
  const bool ok = lane < P && c < hv;
  const int cc = ok ? c : 0;
  const int32_t r0 = b + (int32_t)(((int64_t)n * w) / kHubWaves);
  const int32_t r1 = b + (int32_t)(((int64_t)n * (w + 1)) / kHubWaves);
  float4 acc = hub_identity<R>();
  for (int32_t j = r0; j < r1; j += kHubBatch) {
    float4 v[kHubBatch];
#pragma unroll
    for (int u = 0; u < kHubBatch; ++u) {
      const int32_t p = j + u < r1 ? j + u : r1 - 1;
      v[u] = X[(int64_t)perm[p] * ld + cc];
    }
#pragma unroll
    for (int u = 0; u < kHubBatch; ++u)
      if (j + u < r1) acc = hub_op4<R>(acc, act4_t<ACT>(v[u], act, alpha));
  }
  part[w][lane] = acc;
  __syncthreads();
  float m = 0.f;
  if (w == 0) {
    float4 r = part[0][lane];
#pragma unroll
    for (int k = 1; k < kHubWaves; ++k) {
      const float4 x = part[k][lane];
      // a wave with no rows holds the identity, which max / min / sum leave unchanged
      r = hub_op4<R>(r, x);
    }
    if constexpr (R == NT_MEAN) {
      const float inv = 1.f / (float)(n > 1 ? n : 1);
      r = make_float4(r.x * inv, r.y * inv, r.z * inv, r.w * inv);
    }
    if (n == 0) r = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ok) {
      out[(int64_t)s * ld + c] = r;
      m = fmaxf(fmaxf(fabsf(r.x), fabsf(r.y)), fmaxf(fabsf(r.z), fabsf(r.w)));
    }
  }
  if (amax != nullptr) block_max_to(amax, m);
}

// Row-table entries of hub nodes: {e, src, rev, (v << 2) | start} (no "last in-edge" flag, so the
// fused kernel's scan never stores S_out for them; every row its own segment start, so the scan's
// carry never crosses a hub row into a neighbour).
__global__ void __launch_bounds__(256) mark_hub_rows_kernel(int4* __restrict__ rt, int64_t E,
                                                            const int32_t* __restrict__ seg_ptr,
                                                            int hub_degree) {
  for (int64_t p = blockIdx.x * 256LL + threadIdx.x; p < E; p += (int64_t)gridDim.x * 256) {
    const int fl = rt[p].w;
    const int v = fl >> 2;
    if (seg_ptr[v + 1] - seg_ptr[v] > hub_degree) rt[p].w = (v << 2) | 1;
  }
}

template <int R>
int launch_hub(const float4* X, const int32_t* perm, const int32_t* seg_ptr, const int32_t* hubs,
               int64_t nhub, int hv, int act, float alpha, float4* out, float* amax, int ld, hipStream_t stream) {
  const int nslab = (hv + 63) / 64, P = (hv + nslab - 1) / nslab;
  const dim3 grid((unsigned)nhub, (unsigned)nslab);
  switch (act) {
    case NT_ACT_IDENTITY:
      hub_aggregate_kernel<R, NT_ACT_IDENTITY><<<grid, kHubWaves * 64, 0, stream>>>(X, perm, seg_ptr, hubs, hv, P,
                                                                                 act, alpha, out, amax, ld);
      break;
    case NT_ACT_RELU:
      hub_aggregate_kernel<R, NT_ACT_RELU><<<grid, kHubWaves * 64, 0, stream>>>(X, perm, seg_ptr, hubs, hv, P, act,
                                                                             alpha, out, amax, ld);
      break;
    default:
      hub_aggregate_kernel<R, -1><<<grid, kHubWaves * 64, 0, stream>>>(X, perm, seg_ptr, hubs, hv, P, act, alpha,
                                                                    out, amax, ld);
  }
  NT_LAUNCH_CHECK();
  return NT_OK;
}

}  // namespace
}  // namespace nt

extern "C" int nt_dmpnn_mark_hub_rows(void* row_table, int64_t E, const int32_t* dst_ptr, int64_t V,
                                      int hub_degree, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(E >= 0 && V >= 0 && E < (int64_t(1) << 31) && V < (int64_t(1) << 29), NT_EINVAL, "bad sizes");
  NT_REQUIRE(hub_degree >= 1, NT_EINVAL, "hub_degree must be >= 1");
  if (E == 0) return NT_OK;
  NT_REQUIRE(row_table && dst_ptr, NT_EINVAL, "NULL pointer");
  NT_REQUIRE(aligned16(row_table), NT_EINVAL, "row_table must be 16-byte aligned");
  mark_hub_rows_kernel<<<grid_for(E, 256, 256 * 16), 256, 0, as_stream(stream_)>>>((int4*)row_table, E, dst_ptr,
                                                                                   hub_degree);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

extern "C" int nt_dmpnn_hub_aggregate(const void* X, const int32_t* perm, const int32_t* seg_ptr,
                                      const int32_t* hubs, int64_t nhub, int64_t h, int reduce, int act,
                                      float act_alpha, int dtype, float* amax_out, void* out, int64_t ld,
                                      void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32, NT_EUNSUPPORTED, "nt_dmpnn_hub_aggregate: fp32 only");
  NT_REQUIRE(reduce >= NT_SUM && reduce <= NT_MIN, NT_EINVAL, "bad reduce code");
  NT_REQUIRE(act >= NT_ACT_IDENTITY && act <= NT_ACT_SIGMOID, NT_EINVAL, "bad act code");
  NT_REQUIRE(nhub >= 0 && nhub < (int64_t(1) << 31) && h > 0, NT_EINVAL, "bad sizes");
  NT_REQUIRE(h % 4 == 0 && h <= 4 * 65535 * 64, NT_EUNSUPPORTED, "nt_dmpnn_hub_aggregate needs h % 4 == 0");
  if (nhub == 0) return NT_OK;
  NT_REQUIRE(X && seg_ptr && hubs && out && perm, NT_EINVAL, "NULL pointer");
  NT_REQUIRE(aligned16(X) && aligned16(out), NT_EINVAL, "feature pointers must be 16-byte aligned");
  if (ld == 0) ld = h;
  NT_REQUIRE(ld >= h && ld % 4 == 0, NT_EINVAL, "row pitch must be >= h and a multiple of 4");
  const int hv = (int)(h / 4), ld4 = (int)(ld / 4);
  const float4* X4 = (const float4*)X;
  float4* O4 = (float4*)out;
  hipStream_t s = as_stream(stream_);
  switch (reduce) {
    case NT_SUM: return launch_hub<NT_SUM>(X4, perm, seg_ptr, hubs, nhub, hv, act, act_alpha, O4, amax_out, ld4, s);
    case NT_MEAN: return launch_hub<NT_MEAN>(X4, perm, seg_ptr, hubs, nhub, hv, act, act_alpha, O4, amax_out, ld4, s);
    case NT_MAX: return launch_hub<NT_MAX>(X4, perm, seg_ptr, hubs, nhub, hv, act, act_alpha, O4, amax_out, ld4, s);
    default: return launch_hub<NT_MIN>(X4, perm, seg_ptr, hubs, nhub, hv, act, act_alpha, O4, amax_out, ld4, s);
  }
}

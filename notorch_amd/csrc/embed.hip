// GraphEmbedding (notorch/nn/gnn/embed.py:11-36: two sum-mode nn.EmbeddingBag over the integer
// atom / bond type columns) on the device, alone and fused into the D-MPNN initial gather
// (SURVEY §8(f) row 2).
//
//   nt_embed_bag         out[i] = sum_j T[idx[i][j]]                                  (embed.py:29)
//   nt_dmpnn_init_embed  H0[e] = Xv[src e] + Xe[e] with Xv, Xe never materialised:
//                        Xv[s] = sum_j Tv[node_types[s][j]], Xe[e] = sum_j Te[edge_types[e][j]]
//                        fused with S[v] = R_{e->v} act(H0[e])                       (chemprop.py:82-83,
//                                                                                     :37-39, layer 0)
// Values are bit-identical to running the embedding, then nt_dmpnn_init: every bag is summed in
// ascending j from 0 in fp32 and rounded to the storage type where the unfused path stores it.
// Bytes: the tables are a few KiB (42 x h and 13 x h) and stay in L2, so the fused init reads
// (kv + ke) int64 type indices per edge instead of the Xv[src] and Xe rows (2 rows per edge), and
// the embedding's own V + E row writes disappear: (E + V) rows written in total instead of
// (2E + 2V) written + 2E read.
#include <algorithm>

#include "rows.hpp"

namespace nt {
int fk_absmax(const float* X, int64_t n, float* out, hipStream_t stream);  // update_pk.hip
}

namespace nt {
int cu_count();  // update_ps.hip

namespace {

template <typename T, bool VEC>
__device__ __forceinline__ void bag_sum(const T* __restrict__ table, int64_t ntypes,
                                        const int64_t* __restrict__ idx, int64_t k, int64_t h,
                                        int64_t c, float (&x)[Piece<T, VEC>::N]) {
  constexpr int N = Piece<T, VEC>::N;
#pragma unroll
  for (int i = 0; i < N; ++i) x[i] = 0.f;
  for (int64_t j = 0; j < k; ++j) {
    const int64_t t = idx[j];
    if (t < 0 || t >= ntypes) continue;  // validated on the host; never read out of bounds
    float y[N];
    Piece<T, VEC>::load(table + t * h + c, y);
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] += y[i];
  }
}

template <typename T, bool VEC>
__global__ void __launch_bounds__(256) embed_bag_kernel(const T* __restrict__ table, int64_t ntypes,
                                                        const int64_t* __restrict__ idx, int64_t n,
                                                        int64_t k, int64_t h, T* __restrict__ out) {
  constexpr int N = Piece<T, VEC>::N;
  const int64_t hw = h / N;
  const int64_t total = n * hw;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t / hw, c = (t - i * hw) * N;
    float x[N];
    bag_sum<T, VEC>(table, ntypes, idx + i * k, k, h, c, x);
    Piece<T, VEC>::store(out + i * h + c, x);
  }
}

struct EmbedArgs {
  const void* Tv;
  int64_t nv;
  const int64_t* vtypes;
  int64_t kv;
  const void* Te;
  int64_t ne;
  const int64_t* etypes;
  int64_t ke;
};

// H0 of edge e (the stored value), column piece c
template <typename T, bool VEC>
__device__ __forceinline__ void h0_piece(const EmbedArgs& a, const int64_t* __restrict__ src,
                                         int64_t e, int64_t h, int64_t c,
                                         float (&x)[Piece<T, VEC>::N]) {
  constexpr int N = Piece<T, VEC>::N;
  float xv[N], xe[N];
  bag_sum<T, VEC>((const T*)a.Tv, a.nv, a.vtypes + src[e] * a.kv, a.kv, h, c, xv);
  bag_sum<T, VEC>((const T*)a.Te, a.ne, a.etypes + e * a.ke, a.ke, h, c, xe);
#pragma unroll
  for (int i = 0; i < N; ++i) x[i] = as_stored<T>(as_stored<T>(xv[i]) + as_stored<T>(xe[i]));
}

template <typename T, bool VEC, int R, int ACT>
__global__ void __launch_bounds__(256) init_embed_aggregate(
    EmbedArgs a, const int64_t* __restrict__ src, const int32_t* __restrict__ seg_ptr,
    const int32_t* __restrict__ perm, int64_t V, int64_t h, int act, float alpha,
    T* __restrict__ H0, T* __restrict__ S) {
  constexpr int N = Piece<T, VEC>::N;
  const int64_t hw = h / N;
  const int64_t total = V * hw;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = t / hw, c = (t - v * hw) * N;
    const int32_t b = seg_ptr[v], en = seg_ptr[v + 1];
    Reducer<R> r[N];
#pragma unroll
    for (int i = 0; i < N; ++i) r[i].init();
    for (int32_t j = b; j < en; ++j) {
      const int64_t e = perm[j];
      float x[N];
      h0_piece<T, VEC>(a, src, e, h, c, x);
      Piece<T, VEC>::store(H0 + e * h + c, x);
#pragma unroll
      for (int i = 0; i < N; ++i) r[i].push(act_t<ACT>(x[i], act, alpha));
    }
    float y[N];
#pragma unroll
    for (int i = 0; i < N; ++i) y[i] = r[i].result();
    Piece<T, VEC>::store(S + v * h + c, y);
  }
}

// The same with the type-column counts known at compile time (the reference featurisation's 7 atom
// and 2 bond columns, transforms/graph.py:32-43): a node's in-edges are taken 4 at a time and every
// index load of the 4 (perm -> src -> type rows) is issued before the first table row is summed,
// so the three dependent index latencies are paid once per 4 edges instead of once per edge.
//
// LDS = true: both tables are first copied into LDS (a few tens of KiB: 42 x h and 13 x h), so the
// nine table-row reads per edge are LDS reads instead of L2 round trips (the tables do not fit the
// 32 KiB L1).  1024-thread workgroups, two per CU (kTabB of LDS each), grid-stride over the nodes.
constexpr int kTabB = 72 * 1024;
constexpr int kLdsThreads = 1024;

template <typename T, bool VEC, int R, int ACT, int KV, int KE, bool LDS = false>
__global__ void __launch_bounds__(LDS ? kLdsThreads : 256, LDS ? 2 : 1) init_embed_aggregate_k(
    EmbedArgs a, const int64_t* __restrict__ src, const int32_t* __restrict__ seg_ptr,
    const int32_t* __restrict__ perm, int64_t V, int64_t h, int act, float alpha,
    T* __restrict__ H0, T* __restrict__ S, float* __restrict__ amax, int64_t lo) {  // lo: H0 / S row pitch
  constexpr int N = Piece<T, VEC>::N;
  constexpr int U = LDS ? 2 : 4;  // LDS rows are cheap: fewer edges in flight, more waves
  float mh = 0.f, ms = 0.f;       // max |H0|, max |S| of this lane (amax != NULL)
  const T* Tv = (const T*)a.Tv;
  const T* Te = (const T*)a.Te;
  if constexpr (LDS) {
    __shared__ uint4 tab[kTabB / 16];
    const int64_t nvq = a.nv * h * (int64_t)sizeof(T) / 16, neq = a.ne * h * (int64_t)sizeof(T) / 16;
    const uint4* gv = (const uint4*)a.Tv;
    const uint4* ge = (const uint4*)a.Te;
    for (int64_t i = threadIdx.x; i < nvq + neq; i += blockDim.x) tab[i] = i < nvq ? gv[i] : ge[i - nvq];
    __syncthreads();
    Tv = (const T*)tab;
    Te = (const T*)(tab + nvq);
  }
  const int64_t hw = h / N;
  const int64_t total = V * hw;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = t / hw, c = (t - v * hw) * N;
    const int32_t b = seg_ptr[v], en = seg_ptr[v + 1];
    Reducer<R> r[N];
#pragma unroll
    for (int i = 0; i < N; ++i) r[i].init();
    for (int32_t j = b; j < en; j += U) {
      // type indices narrowed to int32 once in range-checked form (a type index is < 2^31 or it is
      // invalid anyway): half the registers of int64, so the kernel keeps 8 waves per SIMD
      int64_t e[U], sv[U];
      int tv[U][KV], te[U][KE];
#pragma unroll
      for (int u = 0; u < U; ++u) e[u] = j + u < en ? (int64_t)perm[j + u] : -1;
#pragma unroll
      for (int u = 0; u < U; ++u) sv[u] = e[u] >= 0 ? src[e[u]] : 0;
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int q = 0; q < KV; ++q) {
          const int64_t x = e[u] >= 0 ? a.vtypes[sv[u] * KV + q] : -1;
          tv[u][q] = (x >= 0 && x < a.nv) ? (int)x : -1;
        }
#pragma unroll
        for (int q = 0; q < KE; ++q) {
          const int64_t x = e[u] >= 0 ? a.etypes[e[u] * KE + q] : -1;
          te[u][q] = (x >= 0 && x < a.ne) ? (int)x : -1;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (e[u] < 0) break;
        float xv[N], xe[N], y[N];
#pragma unroll
        for (int i = 0; i < N; ++i) xv[i] = xe[i] = 0.f;
        // unconditional loads of clamped rows (no branch for the compiler to drain in front of);
        // an invalid index (the host validates, so never in practice) contributes +0.0f
#pragma unroll
        for (int q = 0; q < KV; ++q) {
          const bool ok = tv[u][q] >= 0;
          Piece<T, VEC>::load(Tv + (int64_t)(ok ? tv[u][q] : 0) * h + c, y);
#pragma unroll
          for (int i = 0; i < N; ++i) xv[i] += ok ? y[i] : 0.f;
        }
#pragma unroll
        for (int q = 0; q < KE; ++q) {
          const bool ok = te[u][q] >= 0;
          Piece<T, VEC>::load(Te + (int64_t)(ok ? te[u][q] : 0) * h + c, y);
#pragma unroll
          for (int i = 0; i < N; ++i) xe[i] += ok ? y[i] : 0.f;
        }
        float x[N];
#pragma unroll
        for (int i = 0; i < N; ++i) x[i] = as_stored<T>(as_stored<T>(xv[i]) + as_stored<T>(xe[i]));
        Piece<T, VEC>::store(H0 + e[u] * lo + c, x);
#pragma unroll
        for (int i = 0; i < N; ++i) {
          mh = fmaxf(mh, fabsf(x[i]));
          r[i].push(act_t<ACT>(x[i], act, alpha));
        }
      }
    }
    float y[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      y[i] = r[i].result();
      ms = fmaxf(ms, fabsf(y[i]));
    }
    Piece<T, VEC>::store(S + v * lo + c, y);
  }
  if (amax) block_max_to(amax, mh, ms, true);  // one atomic max per block
}

template <typename T, bool VEC>
__global__ void __launch_bounds__(256) init_embed_only(EmbedArgs a, const int64_t* __restrict__ src,
                                                       int64_t E, int64_t h, T* __restrict__ H0) {
  constexpr int N = Piece<T, VEC>::N;
  const int64_t hw = h / N;
  const int64_t total = E * hw;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = t / hw, c = (t - e * hw) * N;
    float x[N];
    h0_piece<T, VEC>(a, src, e, h, c, x);
    Piece<T, VEC>::store(H0 + e * h + c, x);
  }
}

template <typename T, bool VEC>
int launch_init_embed(const EmbedArgs& a, const int64_t* src, const int32_t* seg_ptr,
                      const int32_t* perm, int64_t V, int64_t E, int64_t h, int act, float alpha,
                      int reduce, void* H0, void* S, float* amax, int64_t lo, hipStream_t stream) {
  constexpr int N = Piece<T, VEC>::N;
  NT_REQUIRE(lo == h || (S != nullptr && a.kv == 7 && a.ke == 2), NT_EUNSUPPORTED,
             "padded rows: the fused 7 + 2 type-column init only");
  if (S == nullptr) {
    if (E == 0) return NT_OK;
    init_embed_only<T, VEC><<<grid_for(E * (h / N), 256, 256 * 32), 256, 0, stream>>>(
        a, src, E, h, (T*)H0);
    NT_LAUNCH_CHECK();
    if (amax) return fk_absmax((const float*)H0, E * h, amax, stream);
    return NT_OK;
  }
  if (V == 0) return NT_OK;
  const int grid = grid_for(V * (h / N), 256, 256 * 32);
  const bool k72 = a.kv == 7 && a.ke == 2;
  // tables in LDS when both fit (fp32 h <= 327, bf16 h <= 655 at the reference's 42 + 13 types)
  const bool lds = k72 && VEC && (a.nv + a.ne) * h * (int64_t)sizeof(T) <= kTabB &&
                   (a.nv * h * (int64_t)sizeof(T)) % 16 == 0;
  const int grid_lds = (int)std::min<int64_t>((V * (h / N) + kLdsThreads - 1) / kLdsThreads,
                                              2 * (int64_t)cu_count());
#define NT_IE(R_, A_)                                                                            \
  do {                                                                                           \
    if (lds)                                                                                     \
      init_embed_aggregate_k<T, VEC, R_, A_, 7, 2, true><<<grid_lds, kLdsThreads, 0, stream>>>(  \
          a, src, seg_ptr, perm, V, h, act, alpha, (T*)H0, (T*)S, amax, lo);                     \
    else if (k72)                                                                                \
      init_embed_aggregate_k<T, VEC, R_, A_, 7, 2><<<grid, 256, 0, stream>>>(                    \
          a, src, seg_ptr, perm, V, h, act, alpha, (T*)H0, (T*)S, amax, lo);                     \
    else                                                                                         \
      init_embed_aggregate<T, VEC, R_, A_><<<grid, 256, 0, stream>>>(a, src, seg_ptr, perm, V, h, \
                                                                     act, alpha, (T*)H0, (T*)S);  \
  } while (0)
#define NT_IE_A(R_)                                                \
  do {                                                             \
    if (act == NT_ACT_IDENTITY) NT_IE(R_, NT_ACT_IDENTITY);        \
    else if (act == NT_ACT_RELU) NT_IE(R_, NT_ACT_RELU);           \
    else NT_IE(R_, -1);                                            \
  } while (0)
  switch (reduce) {
    case NT_SUM: NT_IE_A(NT_SUM); break;
    case NT_MEAN: NT_IE_A(NT_MEAN); break;
    case NT_MAX: NT_IE_A(NT_MAX); break;
    default: NT_IE_A(NT_MIN); break;
  }
#undef NT_IE_A
#undef NT_IE
  NT_LAUNCH_CHECK();
  if (amax && !k72) {  // the generic variant: two max passes over the outputs
    int rc = fk_absmax((const float*)H0, E * h, amax, stream);
    if (rc == NT_OK) rc = fk_absmax((const float*)S, V * h, amax + 1, stream);
    return rc;
  }
  return NT_OK;
}

}  // namespace
}  // namespace nt

extern "C" int nt_embed_bag(const void* table, int64_t num_types, const int64_t* idx, int64_t n,
                            int64_t k, int64_t h, int dtype, void* out, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32 || dtype == NT_BF16, NT_EUNSUPPORTED, "dtype must be NT_F32 or NT_BF16");
  NT_REQUIRE(num_types >= 0 && n >= 0 && k >= 0 && h > 0, NT_EINVAL, "bad sizes");
  if (n == 0) return NT_OK;
  NT_REQUIRE(table && (idx || k == 0) && out, NT_EINVAL, "NULL pointer");
  hipStream_t stream = as_stream(stream_);
  const bool al = aligned16(table) && aligned16(out);
  if (dtype == NT_F32) {
    if (h % 4 == 0 && al)
      embed_bag_kernel<float, true><<<grid_for(n * (h / 4), 256, 256 * 32), 256, 0, stream>>>(
          (const float*)table, num_types, idx, n, k, h, (float*)out);
    else
      embed_bag_kernel<float, false><<<grid_for(n * h, 256, 256 * 32), 256, 0, stream>>>(
          (const float*)table, num_types, idx, n, k, h, (float*)out);
  } else {
    if (h % 8 == 0 && al)
      embed_bag_kernel<bf16_raw, true><<<grid_for(n * (h / 8), 256, 256 * 32), 256, 0, stream>>>(
          (const bf16_raw*)table, num_types, idx, n, k, h, (bf16_raw*)out);
    else
      embed_bag_kernel<bf16_raw, false><<<grid_for(n * h, 256, 256 * 32), 256, 0, stream>>>(
          (const bf16_raw*)table, num_types, idx, n, k, h, (bf16_raw*)out);
  }
  NT_LAUNCH_CHECK();
  return NT_OK;
}

extern "C" int nt_dmpnn_init_embed(const void* node_table, int64_t num_node_types,
                                   const int64_t* node_types, int64_t kv, const void* edge_table,
                                   int64_t num_edge_types, const int64_t* edge_types, int64_t ke,
                                   const int64_t* src, const int32_t* seg_ptr, const int32_t* perm,
                                   int64_t V, int64_t E, int64_t h, int act, float act_alpha,
                                   int reduce, int dtype, void* H0, void* S, float* amax_out,
                                   int64_t ld_out, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32 || dtype == NT_BF16, NT_EUNSUPPORTED, "dtype must be NT_F32 or NT_BF16");
  NT_REQUIRE(reduce >= NT_SUM && reduce <= NT_MIN, NT_EINVAL, "bad reduce code");
  NT_REQUIRE(act >= NT_ACT_IDENTITY && act <= NT_ACT_SIGMOID, NT_EINVAL, "bad act code");
  NT_REQUIRE(V >= 0 && E >= 0 && h > 0 && kv >= 0 && ke >= 0 && num_node_types >= 0 &&
                 num_edge_types >= 0,
             NT_EINVAL, "bad sizes");
  NT_REQUIRE(S == nullptr || (seg_ptr && (perm || E == 0)), NT_EINVAL, "fused aggregation needs the dst CSR");
  NT_REQUIRE(E == 0 || (node_table && edge_table && src && H0 && (node_types || kv == 0) &&
                        (edge_types || ke == 0)),
             NT_EINVAL, "NULL pointer");
  if (ld_out == 0) ld_out = h;
  NT_REQUIRE(ld_out == h || (dtype == NT_F32 && h % 4 == 0 && ld_out % 4 == 0 && ld_out > h), NT_EINVAL,
             "ld_out != h needs fp32, h % 4 == 0 and ld_out % 4 == 0");
  hipStream_t stream = as_stream(stream_);
  const EmbedArgs a{node_table, num_node_types, node_types, kv,
                    edge_table, num_edge_types, edge_types, ke};
  const bool al = aligned16(node_table) && aligned16(edge_table) && aligned16(H0) &&
                  (S == nullptr || aligned16(S));
  if (dtype == NT_F32) {
    if (h % 4 == 0 && al)
      return launch_init_embed<float, true>(a, src, seg_ptr, perm, V, E, h, act, act_alpha, reduce, H0, S,
                                            amax_out, ld_out, stream);
    return launch_init_embed<float, false>(a, src, seg_ptr, perm, V, E, h, act, act_alpha, reduce, H0, S,
                                           amax_out, ld_out, stream);
  }
  NT_REQUIRE(amax_out == nullptr, NT_EINVAL, "amax_out is fp32 only");
  if (h % 8 == 0 && al)
    return launch_init_embed<bf16_raw, true>(a, src, seg_ptr, perm, V, E, h, act, act_alpha, reduce, H0, S,
                                             nullptr, ld_out, stream);
  return launch_init_embed<bf16_raw, false>(a, src, seg_ptr, perm, V, E, h, act, act_alpha, reduce, H0, S,
                                            nullptr, ld_out, stream);
}

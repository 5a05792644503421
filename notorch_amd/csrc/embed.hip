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

// ---------------------------------------------------------------------- type records + wave init
// Per dst-sorted position p of the dst CSR, one 16-B record of the in-edge e = perm[p] with both bags'
// type indices as bytes (nt_embed_edge_records): {e, vt0..3, vt4..6 | et0 << 24, et1}, where vt are
// node_types[src e][0..6] and et edge_types[e][0..1]; an out-of-range index is stored as 255, which the
// init maps to a zero table row.  Built once per graph (7 + 2 type columns, < 255 types of each kind),
// it turns the init's dependent chain perm -> src -> 9 type loads into one load per in-edge.
__global__ void __launch_bounds__(256) edge_records_kernel(const int64_t* __restrict__ vtypes, int64_t nv,
                                                           const int64_t* __restrict__ etypes, int64_t ne,
                                                           const int64_t* __restrict__ src,
                                                           const int32_t* __restrict__ perm, int64_t V,
                                                           int64_t E, int4* __restrict__ out) {
  for (int64_t p = blockIdx.x * 256LL + threadIdx.x; p < E; p += (int64_t)gridDim.x * 256) {
    const int e = perm[p];
    const int64_t sv = src[e];
    const bool sok = sv >= 0 && sv < V;
    unsigned b[9];
#pragma unroll
    for (int q = 0; q < 7; ++q) {
      const int64_t t = sok ? vtypes[sv * 7 + q] : -1;
      b[q] = (t >= 0 && t < nv) ? (unsigned)t : 255u;
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int64_t t = etypes[(int64_t)e * 2 + q];
      b[7 + q] = (t >= 0 && t < ne) ? (unsigned)t : 255u;
    }
    out[p] = int4{e, (int)(b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24),
                  (int)(b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24), (int)b[8]};
  }
}

// One wave per node with both tables (plus a zero row each) in LDS: the node's range and its in-edge
// records are wave-uniform (scalar loads), 4 in-edges at a time; lane l takes row pieces l + 64 q, q <
// PPL (pieces past the row read piece 0 and are masked at the stores).  Same sums in the same order
// as init_embed_aggregate_k (each bag from +0.0 in ascending column, then xv + xe): the same bits.
constexpr int kWaveThreads = 512;  // 8 waves; two workgroups per CU (<= 128 VGPRs, 2 x 72 KiB LDS)
template <int R, int ACT, int PPL>
__global__ void __launch_bounds__(kWaveThreads, 2) init_embed_wave(
    const float* __restrict__ Tv_g, int64_t nv, const float* __restrict__ Te_g, int64_t ne,
    const int4* __restrict__ rec, const int32_t* __restrict__ seg_ptr, int64_t V, int64_t h, int act,
    float alpha, float4* __restrict__ H0, float4* __restrict__ S, float* __restrict__ amax, int64_t lo) {
  __shared__ uint4 tab[kTabB / 16];
  const int64_t hq = h / 4;  // 16-B pieces per row
  const int64_t nvq = nv * hq, neq = ne * hq;
  // [node table | zero row | edge table | zero row]
  for (int64_t i = threadIdx.x; i < nvq + neq + 2 * hq; i += blockDim.x) {
    uint4 x = uint4{0u, 0u, 0u, 0u};
    if (i < nvq) x = reinterpret_cast<const uint4*>(Tv_g)[i];
    else if (i >= nvq + hq && i < nvq + hq + neq) x = reinterpret_cast<const uint4*>(Te_g)[i - nvq - hq];
    tab[i] = x;
  }
  __syncthreads();
  const float4* Tv = reinterpret_cast<const float4*>(tab);
  const float4* Te = Tv + nvq + hq;
  const unsigned zv = (unsigned)nv, ze = (unsigned)ne;  // zero rows
  const int lane = threadIdx.x & 63;
  float mh = 0.f, ms = 0.f;
  int64_t cc[PPL];
  bool ok[PPL];
#pragma unroll
  for (int q = 0; q < PPL; ++q) {
    const int64_t c = lane + 64 * q;
    ok[q] = c < hq;
    cc[q] = ok[q] ? c : 0;
  }
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t v = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)));
       v < V; v += nwaves) {
    const int32_t b = seg_ptr[v], en = seg_ptr[v + 1];
    Reducer4<R> r[PPL];
#pragma unroll
    for (int q = 0; q < PPL; ++q) r[q].init();
    for (int32_t j = b; j < en; j += 4) {
      const int n = min(4, en - j);
      int4 rc[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) rc[u] = u < n ? rec[j + u] : int4{0, 0, 0, 0};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (u >= n) break;
        const unsigned w1 = (unsigned)rc[u].y, w2 = (unsigned)rc[u].z, w3 = (unsigned)rc[u].w;
        unsigned t[9] = {w1 & 255u, (w1 >> 8) & 255u, (w1 >> 16) & 255u, w1 >> 24,
                         w2 & 255u, (w2 >> 8) & 255u, (w2 >> 16) & 255u, w2 >> 24, w3 & 255u};
#pragma unroll
        for (int i = 0; i < 7; ++i) t[i] = t[i] < zv ? t[i] : zv;
#pragma unroll
        for (int i = 7; i < 9; ++i) t[i] = t[i] < ze ? t[i] : ze;
#pragma unroll
        for (int q = 0; q < PPL; ++q) {
          float4 xv = make_float4(0.f, 0.f, 0.f, 0.f), xe = xv;
#pragma unroll
          for (int i = 0; i < 7; ++i) xv = xv + Tv[t[i] * hq + cc[q]];
#pragma unroll
          for (int i = 7; i < 9; ++i) xe = xe + Te[t[i] * hq + cc[q]];
          const float4 h0 = xv + xe;
          if (ok[q]) {
            H0[(int64_t)rc[u].x * lo + cc[q]] = h0;
            mh = fmaxf(mh, fmaxf(fmaxf(fabsf(h0.x), fabsf(h0.y)), fmaxf(fabsf(h0.z), fabsf(h0.w))));
          }
          r[q].push(act4_t<ACT>(h0, act, alpha));
        }
      }
    }
#pragma unroll
    for (int q = 0; q < PPL; ++q) {
      if (ok[q]) {
        const float4 y = r[q].result();
        S[v * lo + cc[q]] = y;
        ms = fmaxf(ms, fmaxf(fmaxf(fabsf(y.x), fabsf(y.y)), fmaxf(fabsf(y.z), fabsf(y.w))));
      }
    }
  }
  if (amax) block_max_to(amax, mh, ms, true);  // one atomic max per block
}

// the wave init over records (fp32, 7 + 2 type columns, both tables + zero rows in LDS, h <= 256 PPL)
int launch_init_embed_wave(const EmbedArgs& a, const int4* rec, const int32_t* seg_ptr, int64_t V, int64_t h,
                           int act, float alpha, int reduce, float* H0, float* S, float* amax, int64_t lo,
                           hipStream_t stream) {
  const int grid = (int)std::min<int64_t>((V + kWaveThreads / 64 - 1) / (kWaveThreads / 64), 2 * (int64_t)cu_count());
  const int64_t hq = h / 4;
#define NT_IEW(R_, A_, P_)                                                                                  \
  init_embed_wave<R_, A_, P_><<<grid, kWaveThreads, 0, stream>>>((const float*)a.Tv, a.nv, (const float*)a.Te, \
                                                                 a.ne, rec, seg_ptr, V, h, act, alpha,       \
                                                                 (float4*)H0, (float4*)S, amax, lo / 4)
#define NT_IEW_P(R_, A_)              \
  do {                                \
    if (hq <= 64) NT_IEW(R_, A_, 1);  \
    else NT_IEW(R_, A_, 2);           \
  } while (0)
#define NT_IEW_A(R_)                                                   \
  do {                                                                 \
    if (act == NT_ACT_IDENTITY) NT_IEW_P(R_, NT_ACT_IDENTITY);         \
    else if (act == NT_ACT_RELU) NT_IEW_P(R_, NT_ACT_RELU);            \
    else NT_IEW_P(R_, -1);                                             \
  } while (0)
  switch (reduce) {
    case NT_SUM: NT_IEW_A(NT_SUM); break;
    case NT_MEAN: NT_IEW_A(NT_MEAN); break;
    case NT_MAX: NT_IEW_A(NT_MAX); break;
    default: NT_IEW_A(NT_MIN); break;
  }
#undef NT_IEW_A
#undef NT_IEW_P
#undef NT_IEW
  NT_LAUNCH_CHECK();
  return NT_OK;
}

// the record path applies: fp32 rows of whole 16-B pieces, h <= 512, 7 + 2 type columns, both tables
// plus their zero rows in kTabB of LDS
bool wave_embed_ok(const EmbedArgs& a, int64_t h) {
  return a.kv == 7 && a.ke == 2 && h % 4 == 0 && h <= 512 && a.nv < 255 && a.ne < 255 &&
         (a.nv + a.ne + 2) * h * 4 <= kTabB;
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

extern "C" int nt_embed_edge_records(const int64_t* node_types, int64_t num_node_types,
                                     const int64_t* edge_types, int64_t num_edge_types, const int64_t* src,
                                     const int32_t* perm, int64_t V, int64_t E, void* records,
                                     void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(V >= 0 && E >= 0 && E < (int64_t(1) << 31), NT_EINVAL, "bad sizes");
  NT_REQUIRE(num_node_types >= 0 && num_node_types < 255 && num_edge_types >= 0 && num_edge_types < 255,
             NT_EUNSUPPORTED, "type records hold fewer than 255 types of each kind");
  if (E == 0) return NT_OK;
  NT_REQUIRE(node_types && edge_types && src && perm && records, NT_EINVAL, "NULL pointer");
  NT_REQUIRE(aligned16(records), NT_EINVAL, "records must be 16-B aligned");
  hipStream_t stream = as_stream(stream_);
  edge_records_kernel<<<grid_for(E, 256), 256, 0, stream>>>(node_types, num_node_types, edge_types, num_edge_types,
                                                            src, perm, V, E, (int4*)records);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

extern "C" int nt_dmpnn_init_embed(const void* node_table, int64_t num_node_types,
                                   const int64_t* node_types, int64_t kv, const void* edge_table,
                                   int64_t num_edge_types, const int64_t* edge_types, int64_t ke,
                                   const int64_t* src, const int32_t* seg_ptr, const int32_t* perm,
                                   int64_t V, int64_t E, int64_t h, int act, float act_alpha,
                                   int reduce, int dtype, void* H0, void* S, float* amax_out,
                                   int64_t ld_out, const void* records, void* stream_) {
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
  if (records != nullptr) {
    NT_REQUIRE(dtype == NT_F32 && S != nullptr && al && wave_embed_ok(a, h) && aligned16(records), NT_EUNSUPPORTED,
               "records: fp32 with S, 16-B aligned rows, 7 + 2 type columns, h % 4 == 0, tables in LDS");
    if (V == 0) return NT_OK;
    return launch_init_embed_wave(a, (const int4*)records, seg_ptr, V, h, act, act_alpha, reduce, (float*)H0,
                                  (float*)S, amax_out, ld_out, stream);
  }
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

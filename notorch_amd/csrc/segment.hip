// Segmented reductions over a CSR view, and the fused initial-gather + first aggregation.
//
//   nt_segment_reduce : out[s] = R_{j in seg s} act(X[perm[j]])       (chemprop.py:37-39, :86;
//                                                                       agg.py:23-47)
//   nt_dmpnn_init     : H0[e] = Xv[src[e]] + Xe[e]; S[v] = R_{e->v} act(H0[e])   (chemprop.py:82-83
//                       fused with layer 0's chemprop.py:37-39)
//
// Mapping: one lane per (segment, 16-B column chunk).  Consecutive lanes walk one row, so every
// gathered row is read as whole 16-B-per-lane contiguous pieces (HBM-coalesced), and the sum over a
// segment is a sequential loop in ascending edge id — the CPU scatter_add_ order, so the only fp32
// difference left against the reference is none at all for the sum itself.
// These kernels are HBM-bound: bytes per segment = (rows read + 1 row written) * h * 4.
#include <float.h>

#include "bf16.hpp"
#include "common.hpp"

namespace nt {

// ---------------- segment reduce ----------------
#ifndef NT_SEG_WAVE
#define NT_SEG_WAVE 1  // A/B: 0 = the thread-per-piece kernel for every row width
#endif
template <int R, int ACT>
__global__ void __launch_bounds__(256) segment_reduce_vec4(
    const float4* __restrict__ X, const int32_t* __restrict__ seg_ptr,
    const int32_t* __restrict__ perm, int64_t nseg, int64_t hv, int act, float alpha,
    float4* __restrict__ out) {
  const int64_t total = nseg * hv;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = t / hv, c = t - s * hv;
    const int32_t b = seg_ptr[s], e = seg_ptr[s + 1];
    Reducer4<R> r;
    r.init();
    int32_t j = b;
    for (; j + 4 <= e; j += 4) {  // four rows in flight, pushed in order
      float4 x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) x[u] = X[(perm ? (int64_t)perm[j + u] : (int64_t)(j + u)) * hv + c];
#pragma unroll
      for (int u = 0; u < 4; ++u) r.push(act4_t<ACT>(x[u], act, alpha));
    }
    for (; j < e; ++j) {
      const int64_t row = perm ? perm[j] : j;
      r.push(act4_t<ACT>(X[row * hv + c], act, alpha));
    }
    out[t] = r.result();
  }
}

// One wave per segment (rows of >= 32 pieces): the segment bounds and the row indices are
// wave-uniform scalar loads, lane l takes row pieces l + 64 q (q < PPL), four rows in flight, pushed
// in ascending order -- the same bits as segment_reduce_vec4.  Pieces past the row load nothing.
template <int R, int ACT, int PPL>
__global__ void __launch_bounds__(256) segment_reduce_wave(
    const float4* __restrict__ X, const int32_t* __restrict__ seg_ptr, const int32_t* __restrict__ perm,
    int64_t nseg, int64_t hv, int act, float alpha, float4* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t s = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)));
       s < nseg; s += nwaves) {
    const int32_t b = seg_ptr[s], e = seg_ptr[s + 1];
    for (int64_t c0 = 0; c0 < hv; c0 += 64 * PPL) {
      int64_t cc[PPL];
      bool ok[PPL];
      Reducer4<R> r[PPL];
#pragma unroll
      for (int q = 0; q < PPL; ++q) {
        const int64_t c = c0 + lane + 64 * q;
        ok[q] = c < hv;
        cc[q] = ok[q] ? c : 0;
        r[q].init();
      }
      int32_t j = b;
      for (; j + 4 <= e; j += 4) {
        int64_t row[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) row[u] = perm ? (int64_t)perm[j + u] : (int64_t)(j + u);
        float4 x[4][PPL];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int q = 0; q < PPL; ++q)
            x[u][q] = ok[q] ? X[row[u] * hv + cc[q]] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int q = 0; q < PPL; ++q) r[q].push(act4_t<ACT>(x[u][q], act, alpha));
      }
      for (; j < e; ++j) {
        const int64_t row = perm ? (int64_t)perm[j] : (int64_t)j;
#pragma unroll
        for (int q = 0; q < PPL; ++q)
          r[q].push(act4_t<ACT>(ok[q] ? X[row * hv + cc[q]] : make_float4(0.f, 0.f, 0.f, 0.f), act, alpha));
      }
#pragma unroll
      for (int q = 0; q < PPL; ++q)
        if (ok[q]) out[s * hv + cc[q]] = r[q].result();
    }
  }
}

template <int R, int ACT>
__global__ void __launch_bounds__(256) segment_reduce_scalar(
    const float* __restrict__ X, const int32_t* __restrict__ seg_ptr,
    const int32_t* __restrict__ perm, int64_t nseg, int64_t h, int act, float alpha,
    float* __restrict__ out) {
  const int64_t total = nseg * h;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = t / h, c = t - s * h;
    const int32_t b = seg_ptr[s], e = seg_ptr[s + 1];
    Reducer<R> r;
    r.init();
    for (int32_t j = b; j < e; ++j) {
      const int64_t row = perm ? perm[j] : j;
      r.push(act_t<ACT>(X[row * h + c], act, alpha));
    }
    out[t] = r.result();
  }
}

// ---------------- fused init + first aggregation ----------------
#ifndef NT_INIT_BATCH
#define NT_INIT_BATCH 1
#endif
#ifndef NT_INIT_MASK
#define NT_INIT_MASK 1  // A/B: 0 = every lane loads every pass (pieces past the row read piece 0)
#endif

template <int R, int ACT>
__global__ void __launch_bounds__(256) init_aggregate_vec4(
    const float4* __restrict__ Xv, const float4* __restrict__ Xe, const int64_t* __restrict__ src,
    const int32_t* __restrict__ seg_ptr, const int32_t* __restrict__ perm, int64_t V, int64_t hv,
    int act, float alpha, float4* __restrict__ H0, float4* __restrict__ S, int64_t lo) {
  const int64_t total = V * hv;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = t / hv, c = t - v * hv;
    const int32_t b = seg_ptr[v], e = seg_ptr[v + 1];
    Reducer4<R> r;
    r.init();
    for (int32_t j = b; j < e; ++j) {
      const int64_t ed = perm[j];
      const float4 x = Xv[src[ed] * hv + c] + Xe[ed * hv + c];
      H0[ed * lo + c] = x;
      r.push(act4_t<ACT>(x, act, alpha));
    }
    S[v * lo + c] = r.result();
  }
}

// One wave per node (the node id is wave-uniform, so the index chain seg_ptr -> perm -> src runs on
// scalar loads once per wave instead of once per 16-B piece): lane l takes the row pieces
// p = l + 64 q (q < PPL, so one pass covers up to 64 PPL pieces, rows of h <= 256 PPL), and the
// in-edges go 4 at a time with all their row loads in flight (4 x 2 x PPL 16-B loads per lane).
// Lanes past the row read piece 0 and are masked at the stores.  Same order of operations per piece
// as init_aggregate_vec4, so the same bits.  Rows wider than one pass loop over passes.
template <int R, int ACT, int PPL>
__global__ void __launch_bounds__(1024) init_aggregate_wave(
    const float4* __restrict__ Xv, const float4* __restrict__ Xe, const int64_t* __restrict__ src,
    const int32_t* __restrict__ seg_ptr, const int32_t* __restrict__ perm, int64_t V, int64_t hv,
    int act, float alpha, float4* __restrict__ H0, float4* __restrict__ S, float* __restrict__ amax,
    int64_t lo, int skip_deg) {  // lo: output row pitch in 16-B pieces (H0, S); skip_deg: see nt_dmpnn_init
  const int lane = threadIdx.x & 63;
  float mh = 0.f, ms = 0.f;  // max |H0|, max |S| of this lane (amax != NULL)
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  auto amax4 = [](float m, float4 v) __attribute__((always_inline)) {
    return fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  };
  for (int64_t v = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)));
       v < V; v += nwaves) {
    const int32_t b = seg_ptr[v], en = seg_ptr[v + 1];
    if (skip_deg > 0 && en - b > skip_deg) continue;  // a hub: its rows and S row come from the chunked init
    for (int64_t c0 = 0; c0 < hv; c0 += 64 * PPL) {
      int64_t cc[PPL];
      bool ok[PPL];
      Reducer4<R> r[PPL];
#pragma unroll
      for (int q = 0; q < PPL; ++q) {
        const int64_t c = c0 + lane + 64 * q;
        ok[q] = c < hv;
        cc[q] = ok[q] ? c : 0;
        r[q].init();
      }
#if NT_INIT_BATCH
      // In-edges 4 at a time, the ragged last batch included (n < 4 under wave-uniform guards), so a
      // node of in-degree 1..4 issues its whole index chain and every row load before the first use.
      for (int32_t j = b; j < en; j += 4) {
        const int n = min(4, en - j);
        int64_t ed[4] = {0, 0, 0, 0}, sv[4] = {0, 0, 0, 0};
        float4 a[4][PPL], x[4][PPL];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (u < n) ed[u] = perm[j + u];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (u < n) sv[u] = src[ed[u]];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int q = 0; q < PPL; ++q) {
            if (u < n && (q == 0 || ok[q] || !NT_INIT_MASK)) {
              a[u][q] = Xv[sv[u] * hv + cc[q]];
              x[u][q] = Xe[ed[u] * hv + cc[q]];
            } else {
              a[u][q] = x[u][q] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
          }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (u >= n) break;
#pragma unroll
          for (int q = 0; q < PPL; ++q) {
            const float4 h0 = a[u][q] + x[u][q];
            if (ok[q]) {
              H0[ed[u] * lo + cc[q]] = h0;
              mh = amax4(mh, h0);
            }
            r[q].push(act4_t<ACT>(h0, act, alpha));
          }
        }
      }
#else
      int32_t j = b;
      for (; j + 4 <= en; j += 4) {
        int64_t ed[4], sv[4];
        float4 a[4][PPL], x[4][PPL];
#pragma unroll
        for (int u = 0; u < 4; ++u) ed[u] = perm[j + u];
#pragma unroll
        for (int u = 0; u < 4; ++u) sv[u] = src[ed[u]];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int q = 0; q < PPL; ++q) {
            if (q == 0 || ok[q] || !NT_INIT_MASK) {  // pieces past the row: no load (exec-masked)
              a[u][q] = Xv[sv[u] * hv + cc[q]];
              x[u][q] = Xe[ed[u] * hv + cc[q]];
            } else {
              a[u][q] = x[u][q] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
          }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int q = 0; q < PPL; ++q) {
            const float4 h0 = a[u][q] + x[u][q];
            if (ok[q]) {
              H0[ed[u] * lo + cc[q]] = h0;
              mh = amax4(mh, h0);
            }
            r[q].push(act4_t<ACT>(h0, act, alpha));
          }
      }
      for (; j < en; ++j) {
        const int64_t ed = perm[j], sv = src[ed];
#pragma unroll
        for (int q = 0; q < PPL; ++q) {
          const float4 h0 = Xv[sv * hv + cc[q]] + Xe[ed * hv + cc[q]];
          if (ok[q]) {
            H0[ed * lo + cc[q]] = h0;
            mh = amax4(mh, h0);
          }
          r[q].push(act4_t<ACT>(h0, act, alpha));
        }
      }
#endif
#pragma unroll
      for (int q = 0; q < PPL; ++q) {
        if (ok[q]) {
          const float4 s4 = r[q].result();
          S[v * lo + cc[q]] = s4;
          ms = amax4(ms, s4);
        }
      }
    }
  }
  if (amax) block_max_to(amax, mh, ms, true);  // one atomic max per block
}

template <int R, int ACT>
__global__ void __launch_bounds__(256) init_aggregate_scalar(
    const float* __restrict__ Xv, const float* __restrict__ Xe, const int64_t* __restrict__ src,
    const int32_t* __restrict__ seg_ptr, const int32_t* __restrict__ perm, int64_t V, int64_t h,
    int act, float alpha, float* __restrict__ H0, float* __restrict__ S) {
  const int64_t total = V * h;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = t / h, c = t - v * h;
    const int32_t b = seg_ptr[v], e = seg_ptr[v + 1];
    Reducer<R> r;
    r.init();
    for (int32_t j = b; j < e; ++j) {
      const int64_t ed = perm[j];
      const float x = Xv[src[ed] * h + c] + Xe[ed * h + c];
      H0[ed * h + c] = x;
      r.push(act_t<ACT>(x, act, alpha));
    }
    S[t] = r.result();
  }
}

// plain init (no aggregation): one lane per (edge, column chunk)
__global__ void __launch_bounds__(256) init_only_vec4(const float4* __restrict__ Xv,
                                                      const float4* __restrict__ Xe,
                                                      const int64_t* __restrict__ src, int64_t E,
                                                      int64_t hv, float4* __restrict__ H0,
                                                      float* __restrict__ amax, int64_t lo) {
  const int64_t total = E * hv;
  float m = 0.f;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = t / hv, c = t - e * hv;
    const float4 y = Xv[src[e] * hv + c] + Xe[t];
    H0[e * lo + c] = y;
    m = fmaxf(m, fmaxf(fmaxf(fabsf(y.x), fabsf(y.y)), fmaxf(fabsf(y.z), fabsf(y.w))));
  }
  if (amax) block_max_to(amax, m);
}
__global__ void __launch_bounds__(256) init_only_scalar(const float* __restrict__ Xv,
                                                        const float* __restrict__ Xe,
                                                        const int64_t* __restrict__ src, int64_t E,
                                                        int64_t h, float* __restrict__ H0,
                                                        float* __restrict__ amax) {
  const int64_t total = E * h;
  float m = 0.f;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = t / h, c = t - e * h;
    const float y = Xv[src[e] * h + c] + Xe[t];
    H0[t] = y;
    m = fmaxf(m, fabsf(y));
  }
  if (amax) block_max_to(amax, m);
}

// ---- dispatch helpers: (reduce, act) -> template instance ----
#define NT_DISPATCH_RA(REDUCE, ACT, LAUNCH)                                  \
  do {                                                                       \
    switch (REDUCE) {                                                        \
      case NT_SUM: { constexpr int R_ = NT_SUM; NT_DISPATCH_A(ACT, LAUNCH); } break;   \
      case NT_MEAN: { constexpr int R_ = NT_MEAN; NT_DISPATCH_A(ACT, LAUNCH); } break; \
      case NT_MAX: { constexpr int R_ = NT_MAX; NT_DISPATCH_A(ACT, LAUNCH); } break;   \
      case NT_MIN: { constexpr int R_ = NT_MIN; NT_DISPATCH_A(ACT, LAUNCH); } break;   \
    }                                                                        \
  } while (0)
#define NT_DISPATCH_A(ACT, LAUNCH)                                                      \
  do {                                                                                  \
    if ((ACT) == NT_ACT_IDENTITY) { constexpr int A_ = NT_ACT_IDENTITY; LAUNCH; }        \
    else if ((ACT) == NT_ACT_RELU) { constexpr int A_ = NT_ACT_RELU; LAUNCH; }           \
    else { constexpr int A_ = -1; LAUNCH; }                                             \
  } while (0)

static bool valid_reduce(int r) { return r >= NT_SUM && r <= NT_MIN; }
static bool valid_act(int a) { return a >= NT_ACT_IDENTITY && a <= NT_ACT_SIGMOID; }

}  // namespace nt

extern "C" int nt_segment_reduce(const void* X, const int32_t* seg_ptr, const int32_t* perm,
                                 int64_t nseg, int64_t h, int reduce, int act, float act_alpha,
                                 int dtype, void* out, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32 || dtype == NT_BF16, NT_EUNSUPPORTED, "dtype must be NT_F32 or NT_BF16");
  NT_REQUIRE(valid_reduce(reduce) && valid_act(act), NT_EINVAL, "bad reduce/act code");
  NT_REQUIRE(nseg >= 0 && h > 0, NT_EINVAL, "bad sizes");
  if (nseg == 0) return NT_OK;
  NT_REQUIRE(X && seg_ptr && out, NT_EINVAL, "NULL pointer");
  hipStream_t stream = as_stream(stream_);
  if (dtype == NT_BF16)
    return launch_segment_reduce_bf16(X, seg_ptr, perm, nseg, h, reduce, act, act_alpha, out, stream);
  const bool vec = (h % 4 == 0) && aligned16(X) && aligned16(out);
  if (vec && h / 4 >= 32 && NT_SEG_WAVE) {  // rows of >= 32 pieces: a wave per segment
    const int64_t hv = h / 4;
    const int grid = grid_for(nseg * 64, 256, 256 * 8);
    if (hv <= 64) {
      NT_DISPATCH_RA(reduce, act,
                     (segment_reduce_wave<R_, A_, 1><<<grid, 256, 0, stream>>>(
                         (const float4*)X, seg_ptr, perm, nseg, hv, act, act_alpha, (float4*)out)));
    } else {
      NT_DISPATCH_RA(reduce, act,
                     (segment_reduce_wave<R_, A_, 2><<<grid, 256, 0, stream>>>(
                         (const float4*)X, seg_ptr, perm, nseg, hv, act, act_alpha, (float4*)out)));
    }
  } else if (vec) {
    const int64_t hv = h / 4;
    const int grid = grid_for(nseg * hv, 256, 256 * 32);
    NT_DISPATCH_RA(reduce, act,
                   (segment_reduce_vec4<R_, A_><<<grid, 256, 0, stream>>>(
                       (const float4*)X, seg_ptr, perm, nseg, hv, act, act_alpha, (float4*)out)));
  } else {
    const int grid = grid_for(nseg * h, 256, 256 * 32);
    NT_DISPATCH_RA(reduce, act,
                   (segment_reduce_scalar<R_, A_><<<grid, 256, 0, stream>>>(
                       (const float*)X, seg_ptr, perm, nseg, h, act, act_alpha, (float*)out)));
  }
  NT_LAUNCH_CHECK();
  return NT_OK;
}

extern "C" int nt_dmpnn_aggregate(const void* H, const int32_t* row_ptr, const int32_t* perm, int64_t V,
                                  int64_t h, int reduce, int dtype, void* S_out, void* stream) {
  return nt_segment_reduce(H, row_ptr, perm, V, h, reduce, NT_ACT_RELU, 0.f, dtype, S_out, stream);
}

namespace nt {
int fk_absmax(const float* X, int64_t n, float* out, hipStream_t stream);  // update_pk.hip
}

extern "C" int nt_dmpnn_init(const void* Xv, const void* Xe, const int64_t* src,
                             const int32_t* seg_ptr, const int32_t* perm, int64_t V, int64_t E,
                             int64_t h, int act, float act_alpha, int reduce, int dtype, void* H0,
                             void* S, float* amax_out, int64_t ld_out, int skip_degree, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32 || dtype == NT_BF16, NT_EUNSUPPORTED, "dtype must be NT_F32 or NT_BF16");
  NT_REQUIRE(valid_reduce(reduce) && valid_act(act), NT_EINVAL, "bad reduce/act code");
  NT_REQUIRE(V >= 0 && E >= 0 && h > 0 && ld_out >= 0 && skip_degree >= 0, NT_EINVAL, "bad sizes");
  NT_REQUIRE(skip_degree == 0 || (dtype == NT_F32 && S != nullptr && h % 4 == 0 && h >= 128), NT_EUNSUPPORTED,
             "skip_degree needs fp32, the aggregation, h % 4 == 0 and h >= 128");
  if (ld_out == 0) ld_out = h;
  // padded output rows: the fp32 kernels that take them (the wave-per-node init, h >= 128, and the
  // plain init); every other variant writes dense rows
  NT_REQUIRE(ld_out == h || (dtype == NT_F32 && h % 4 == 0 && ld_out % 4 == 0 && ld_out > h &&
                             (S == nullptr || h >= 128)),
             NT_EUNSUPPORTED, "ld_out != h needs fp32, h % 4 == 0, ld_out % 4 == 0 and h >= 128 (with S)");
  const int64_t lo4 = ld_out / 4;
  hipStream_t stream = as_stream(stream_);
  if (dtype == NT_BF16) {
    NT_REQUIRE(amax_out == nullptr, NT_EINVAL, "amax_out is fp32 only");
    return launch_init_bf16(Xv, Xe, src, seg_ptr, perm, V, E, h, act, act_alpha, reduce, H0, S, stream);
  }
  const bool vec = (h % 4 == 0) && aligned16(Xv) && aligned16(Xe) && aligned16(H0) &&
                   (S == nullptr || aligned16(S));
  NT_REQUIRE((ld_out == h && skip_degree == 0) || vec, NT_EINVAL,
             "padded output rows and skip_degree need 16-byte aligned pointers");
  if (S != nullptr) {
    if (V == 0) return NT_OK;
    NT_REQUIRE(seg_ptr && (perm || E == 0), NT_EINVAL, "fused aggregation needs the dst CSR");
    NT_REQUIRE(E == 0 || (Xv && Xe && src && H0), NT_EINVAL, "NULL pointer");
    if (vec) {
      const int64_t hv = h / 4;
      if (hv >= 32) {  // rows of >= 32 pieces: a wave per node, every piece of the row in one pass
#ifndef NT_INIT_PPL1
#define NT_INIT_PPL1 0  // A/B: 1 = one 64-piece pass at a time (the round-3 kernel)
#endif
#ifndef NT_INIT_BLOCK
#define NT_INIT_BLOCK 1024  // A/B: threads per block (the amax chain: one atomic pair per block)
#endif
        const int grid = grid_for(V * 64, NT_INIT_BLOCK, 256 * 8 * 256 / NT_INIT_BLOCK);  // 32 waves per CU
        if (hv <= 64 || NT_INIT_PPL1) {
          NT_DISPATCH_RA(reduce, act,
                         (init_aggregate_wave<R_, A_, 1><<<grid, NT_INIT_BLOCK, 0, stream>>>(
                             (const float4*)Xv, (const float4*)Xe, src, seg_ptr, perm, V, hv, act,
                             act_alpha, (float4*)H0, (float4*)S, amax_out, lo4, skip_degree)));
        } else {
          NT_DISPATCH_RA(reduce, act,
                         (init_aggregate_wave<R_, A_, 2><<<grid, NT_INIT_BLOCK, 0, stream>>>(
                             (const float4*)Xv, (const float4*)Xe, src, seg_ptr, perm, V, hv, act,
                             act_alpha, (float4*)H0, (float4*)S, amax_out, lo4, skip_degree)));
        }
        NT_LAUNCH_CHECK();
        return NT_OK;
      } else {
        const int grid = grid_for(V * hv, 256, 256 * 32);
        NT_DISPATCH_RA(reduce, act,
                       (init_aggregate_vec4<R_, A_><<<grid, 256, 0, stream>>>(
                           (const float4*)Xv, (const float4*)Xe, src, seg_ptr, perm, V, hv, act,
                           act_alpha, (float4*)H0, (float4*)S, hv)));
      }
    } else {
      const int grid = grid_for(V * h, 256, 256 * 32);
      NT_DISPATCH_RA(reduce, act,
                     (init_aggregate_scalar<R_, A_><<<grid, 256, 0, stream>>>(
                         (const float*)Xv, (const float*)Xe, src, seg_ptr, perm, V, h, act,
                         act_alpha, (float*)H0, (float*)S)));
    }
    NT_LAUNCH_CHECK();
    if (amax_out) {  // the other init variants: two max passes over the outputs
      int rc = fk_absmax((const float*)H0, E * h, amax_out, stream);
      if (rc == NT_OK) rc = fk_absmax((const float*)S, V * h, amax_out + 1, stream);
      return rc;
    }
    return NT_OK;
  } else {
    if (E == 0) return NT_OK;
    NT_REQUIRE(Xv && Xe && src && H0, NT_EINVAL, "NULL pointer");
    if (vec) {
      const int64_t hv = h / 4;
      init_only_vec4<<<grid_for(E * hv, 256, 256 * 32), 256, 0, stream>>>(
          (const float4*)Xv, (const float4*)Xe, src, E, hv, (float4*)H0, amax_out, lo4);
    } else {
      init_only_scalar<<<grid_for(E * h, 256, 256 * 32), 256, 0, stream>>>(
          (const float*)Xv, (const float*)Xe, src, E, h, (float*)H0, amax_out);
    }
  }
  NT_LAUNCH_CHECK();
  return NT_OK;
}

// ------------------------------------------------------------------------------ long segments
// Load-balanced two-pass reduction for segments far longer than the rest (polymer hubs with
// in-degree ~512, readouts over 1k-10k-atom molecules: SURVEY §8(d) config 5).  The one-lane-per-
// (segment, piece) kernel above walks a whole segment serially, so one hub sets the kernel time.
// Here every segment is cut into chunks of at most kChunk rows (chunk_pos: monotone CSR positions,
// segment boundaries included); pass 1 reduces each chunk (one lane per (chunk, piece), 4 rows in
// flight): a chunk that is its segment's only one (chunk_seg[k] = s) is the segment's result and is
// stored to out[s] directly, the others go to the partial rows P[k]; pass 2 combines the chunk
// partials of the remaining segments (comb_seg: more than one chunk, or none) in chunk order.
// Deterministic; sums differ from the serial ascending order only by the regrouping (fp32
// reassociation at chunk boundaries, and at the 8 sub-ranges pass 2 splits a segment's chunks into).
#include "rows.hpp"

namespace nt {
namespace {

// reduce R's finishing step for one segment result held in accumulator form (the mean divides by the
// segment's row count n)
template <int R, int N>
__device__ __forceinline__ void seg_finish(float (&y)[N], int n) {
  if constexpr (R == NT_MEAN) {
#pragma unroll
    for (int i = 0; i < N; ++i) y[i] /= (float)(n > 1 ? n : 1);
  }
}

template <int N>
__device__ __forceinline__ float absmax_n(float m, const float (&y)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) m = fmaxf(m, fabsf(y[i]));
  return m;
}

#ifndef NT_SEG_PU
#define NT_SEG_PU 8
#endif
constexpr int kSegPU = NT_SEG_PU;  // rows in flight per lane in seg_chunk_partial (a chunk: <= 32 rows)

template <typename T, bool VEC, int R, int ACT>
__global__ void __launch_bounds__(256) seg_chunk_partial(const T* __restrict__ X,
                                                         const int32_t* __restrict__ perm,
                                                         const int32_t* __restrict__ chunk_pos,
                                                         const int32_t* __restrict__ chunk_seg,
                                                         int64_t nchunks, int64_t h, int act,
                                                         float alpha, float* __restrict__ P,
                                                         T* __restrict__ out, float* __restrict__ amax) {
  constexpr int N = Piece<T, VEC>::N;
  constexpr int RR = R == NT_MEAN ? NT_SUM : R;  // the mean divides at the end
  const int64_t hw = h / N;
  const int64_t total = nchunks * hw;
  float m = 0.f;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = t / hw, c = (t - k * hw) * N;
    const int32_t b = chunk_pos[k], e = chunk_pos[k + 1];
    Reducer<RR> r[N];
#pragma unroll
    for (int i = 0; i < N; ++i) r[i].init();
    for (int32_t j = b; j < e; j += kSegPU) {
      float x[kSegPU][N];
      int64_t row[kSegPU];
#pragma unroll
      for (int u = 0; u < kSegPU; ++u) row[u] = j + u < e ? (perm ? perm[j + u] : j + u) : (perm ? perm[b] : b);
#pragma unroll
      for (int u = 0; u < kSegPU; ++u) Piece<T, VEC>::load(X + row[u] * h + c, x[u]);
#pragma unroll
      for (int u = 0; u < kSegPU; ++u) {
        if (j + u >= e) break;
#pragma unroll
        for (int i = 0; i < N; ++i) r[i].push(act_t<ACT>(x[u][i], act, alpha));
      }
    }
    const int32_t sk = chunk_seg ? chunk_seg[k] : -1;
    float y[N];
#pragma unroll
    for (int i = 0; i < N; ++i) y[i] = r[i].acc;  // raw accumulator (chunk non-empty)
    if (sk >= 0) {  // the segment's only chunk: its result
      seg_finish<R>(y, e - b);
      Piece<T, VEC>::store(out + (int64_t)sk * h + c, y);
      m = absmax_n(m, y);
    } else {
#pragma unroll
      for (int i = 0; i < N; ++i) P[k * h + c + i] = y[i];
    }
  }
  if (amax) block_max_to(amax, m);  // fp32 callers: max|out| of the rows stored here
}

// The initial gather fused into pass 1 (hub graphs, fp32): the chunk's rows are computed, not read,
// H0[e] = Xv[src[e]] + Xe[e] (stored: every dst-sorted position lies in exactly one chunk) and reduced
// as act(H0) in the chunk's position order; amax[0] raised to max|H0|, amax[1] to max|S| of the
// segments finished here.  One lane per (chunk, piece), 4 rows in flight.
template <bool VEC, int R, int ACT>
__global__ void __launch_bounds__(256) init_chunk_partial(const float* __restrict__ Xv, const float* __restrict__ Xe,
                                                          const int64_t* __restrict__ src,
                                                          const int32_t* __restrict__ perm,
                                                          const int32_t* __restrict__ chunk_pos,
                                                          const int32_t* __restrict__ chunk_seg,
                                                          const int32_t* __restrict__ chunk_ids,
                                                          int64_t nchunks, int64_t h, int act, float alpha,
                                                          float* __restrict__ H0, float* __restrict__ P,
                                                          float* __restrict__ S, float* __restrict__ amax,
                                                          int64_t lo) {  // lo: row pitch of H0 and S
  // chunk_ids (may be NULL): the chunks to run (nchunks of them), else chunks 0 .. nchunks - 1
  constexpr int N = Piece<float, VEC>::N;
  constexpr int RR = R == NT_MEAN ? NT_SUM : R;  // the mean divides at the end
  const int64_t hw = h / N;
  const int64_t total = nchunks * hw;
  float m = 0.f, ms = 0.f;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t ki = t / hw, c = (t - ki * hw) * N;
    const int64_t k = chunk_ids ? chunk_ids[ki] : ki;
    const int32_t b = chunk_pos[k], e = chunk_pos[k + 1];
    Reducer<RR> r[N];
#pragma unroll
    for (int i = 0; i < N; ++i) r[i].init();
    for (int32_t j = b; j < e; j += 4) {
      int64_t ed[4], sv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) ed[u] = perm[j + u < e ? j + u : b];
#pragma unroll
      for (int u = 0; u < 4; ++u) sv[u] = src[ed[u]];
      float xv[4][N], xe[4][N];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        Piece<float, VEC>::load(Xv + sv[u] * h + c, xv[u]);
        Piece<float, VEC>::load(Xe + ed[u] * h + c, xe[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (j + u >= e) break;
        float y[N];
#pragma unroll
        for (int i = 0; i < N; ++i) {
          y[i] = xv[u][i] + xe[u][i];
          m = fmaxf(m, fabsf(y[i]));
          r[i].push(act_t<ACT>(y[i], act, alpha));
        }
        Piece<float, VEC>::store(H0 + ed[u] * lo + c, y);
      }
    }
    const int32_t sk = chunk_seg ? chunk_seg[k] : -1;
    float y[N];
#pragma unroll
    for (int i = 0; i < N; ++i) y[i] = r[i].acc;  // raw accumulator (chunk non-empty)
    if (sk >= 0) {
      seg_finish<R>(y, e - b);
      Piece<float, VEC>::store(S + (int64_t)sk * lo + c, y);
      ms = absmax_n(ms, y);
    } else {
#pragma unroll
      for (int i = 0; i < N; ++i) P[k * h + c + i] = y[i];
    }
  }
  if (amax) block_max_to(amax, m, ms, true);
}

// Pass 2: one block per (listed segment, 32-piece slab); the segment's chunks split into 32
// consecutive sub-ranges, each summed in chunk order (4 per 32-thread group in 256-thread blocks, 1
// in the 1024-thread blocks launched when the listed segments are few), then the sub-range results
// combined in order by group 0 (empty segment -> 0 for every reduction); the same bits at either
// block size.
constexpr int kCombSub = 32;  // a segment's chunks in 32 consecutive sub-ranges, whatever the block size
template <typename T, bool VEC, int R, int kCombG>
__global__ void __launch_bounds__(32 * kCombG) seg_chunk_combine(const float* __restrict__ P,
                                                         const int32_t* __restrict__ chunk_ptr,
                                                         const int32_t* __restrict__ seg_ptr,
                                                         const int32_t* __restrict__ comb_seg,
                                                         int64_t ncomb, int64_t h,
                                                         T* __restrict__ out, float* __restrict__ amax,
                                                         int64_t lo) {  // lo: row pitch of out
  constexpr int N = Piece<T, VEC>::N;
  constexpr int SPG = kCombSub / kCombG;  // sub-ranges per 32-thread group
  __shared__ float red[kCombSub][32][N];
  const int64_t hw = h / N, nslab = (hw + 31) / 32;
  const int g = threadIdx.x >> 5, cl = threadIdx.x & 31;
  float m = 0.f;
  for (int64_t blk = blockIdx.x; blk < ncomb * nslab; blk += gridDim.x) {
    const int64_t i = blk / nslab, pc = (blk - i * nslab) * 32 + cl;
    const int32_t sg = comb_seg ? comb_seg[i] : (int32_t)i;
    const int32_t b = chunk_ptr[sg], n = chunk_ptr[sg + 1] - b;
    const bool ok = pc < hw;
    const int64_t c = (ok ? pc : 0) * N;
    for (int sr = g * SPG; sr < (g + 1) * SPG; ++sr) {
      const int32_t kb = b + (int32_t)((int64_t)n * sr / kCombSub), ke = b + (int32_t)((int64_t)n * (sr + 1) / kCombSub);
      float y[N];
#pragma unroll
      for (int q = 0; q < N; ++q) y[q] = 0.f;
      for (int32_t k = kb; k < ke; k += 4) {
        float p[4][N];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int64_t kk = k + u < ke ? k + u : kb;
#pragma unroll
          for (int q = 0; q < N; ++q) p[u][q] = P[kk * h + c + q];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (k + u >= ke) break;
#pragma unroll
          for (int q = 0; q < N; ++q) {
            if constexpr (R == NT_MAX) y[q] = k + u == kb ? p[u][q] : fmaxf(y[q], p[u][q]);
            else if constexpr (R == NT_MIN) y[q] = k + u == kb ? p[u][q] : fminf(y[q], p[u][q]);
            else y[q] += p[u][q];
          }
        }
      }
#pragma unroll
      for (int q = 0; q < N; ++q) red[sr][cl][q] = y[q];
    }
    __syncthreads();
    if (g == 0 && ok) {
      float y[N];
      bool first = true;
      for (int sr = 0; sr < kCombSub; ++sr) {
        const int32_t gb = (int32_t)((int64_t)n * sr / kCombSub), ge = (int32_t)((int64_t)n * (sr + 1) / kCombSub);
        if (gb == ge) continue;  // an empty sub-range
#pragma unroll
        for (int q = 0; q < N; ++q) {
          const float v = red[sr][cl][q];
          if constexpr (R == NT_MAX) y[q] = first ? v : fmaxf(y[q], v);
          else if constexpr (R == NT_MIN) y[q] = first ? v : fminf(y[q], v);
          else y[q] = first ? v : y[q] + v;
        }
        first = false;
      }
      if (first) {  // no chunks: empty segment
#pragma unroll
        for (int q = 0; q < N; ++q) y[q] = 0.f;
      }
      seg_finish<R>(y, seg_ptr[sg + 1] - seg_ptr[sg]);
      Piece<T, VEC>::store(out + (int64_t)sg * lo + c, y);
      m = absmax_n(m, y);
    }
    __syncthreads();
  }
  if (amax) block_max_to(amax, m);  // fp32 callers: max|out| (the fp32 layer kernel's split scale)
}

#ifndef NT_COMB_WIDE
#define NT_COMB_WIDE 1
#endif
template <typename T, bool VEC, int R>
void launch_combine(const float* P, const int32_t* chunk_ptr, const int32_t* seg_ptr, const int32_t* comb_seg,
                    int64_t ncomb, int64_t h, T* out, float* amax, hipStream_t stream, int64_t lo = 0) {
  constexpr int N = Piece<T, VEC>::N;
  const int64_t blocks = ncomb * ((h / N + 31) / 32);
  if (blocks == 0) return;
  const int g = (int)(blocks < 256 * 16 ? blocks : 256 * 16);
  if (NT_COMB_WIDE && blocks < 1024) {  // few long segments (a readout over polymers): 32 sub-ranges
    seg_chunk_combine<T, VEC, R, 32><<<g, 1024, 0, stream>>>(P, chunk_ptr, seg_ptr, comb_seg, ncomb, h, out, amax,
                                                            lo ? lo : h);
    return;
  }
  seg_chunk_combine<T, VEC, R, 8><<<g, 256, 0, stream>>>(P, chunk_ptr, seg_ptr, comb_seg, ncomb, h, out, amax,
                                                         lo ? lo : h);
}

template <typename T, bool VEC>
void launch_combine_r(int reduce, const float* P, const int32_t* chunk_ptr, const int32_t* seg_ptr,
                      const int32_t* comb_seg, int64_t ncomb, int64_t h, T* out, float* amax, hipStream_t stream,
                      int64_t lo = 0) {
  switch (reduce) {
    case NT_SUM: launch_combine<T, VEC, NT_SUM>(P, chunk_ptr, seg_ptr, comb_seg, ncomb, h, out, amax, stream, lo); break;
    case NT_MEAN: launch_combine<T, VEC, NT_MEAN>(P, chunk_ptr, seg_ptr, comb_seg, ncomb, h, out, amax, stream, lo); break;
    case NT_MAX: launch_combine<T, VEC, NT_MAX>(P, chunk_ptr, seg_ptr, comb_seg, ncomb, h, out, amax, stream, lo); break;
    default: launch_combine<T, VEC, NT_MIN>(P, chunk_ptr, seg_ptr, comb_seg, ncomb, h, out, amax, stream, lo); break;
  }
}

template <bool VEC>
int launch_init_chunked(const float* Xv, const float* Xe, const int64_t* src, const int32_t* perm,
                        const int32_t* chunk_pos, int64_t nchunks, const int32_t* chunk_ptr,
                        const int32_t* chunk_seg, const int32_t* comb_seg, int64_t ncomb, const int32_t* seg_ptr,
                        int64_t nseg, int64_t h, int reduce, int act, float alpha, float* P, float* H0, float* S,
                        float* amax, int64_t lo, const int32_t* chunk_ids, int64_t nids, hipStream_t stream) {
  constexpr int N = Piece<float, VEC>::N;
  const int64_t nrun = chunk_ids ? nids : nchunks;
  if (nrun > 0) {
    const int g1 = grid_for(nrun * (h / N), 256, 256 * 32);
    NT_DISPATCH_RA(reduce, act,
                   (init_chunk_partial<VEC, R_, A_><<<g1, 256, 0, stream>>>(
                       Xv, Xe, src, perm, chunk_pos, chunk_seg, chunk_ids, nrun, h, act, alpha, H0, P, S, amax,
                       lo)));
    NT_LAUNCH_CHECK();
  }
  if (chunk_seg == nullptr) ncomb = nseg;  // every segment through pass 2
  launch_combine_r<float, VEC>(reduce, P, chunk_ptr, seg_ptr, chunk_seg ? comb_seg : nullptr, ncomb, h, S,
                               amax ? amax + 1 : nullptr, stream, lo);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

template <typename T, bool VEC>
int launch_chunked(const void* X, const int32_t* perm, const int32_t* chunk_pos, int64_t nchunks,
                   const int32_t* chunk_ptr, const int32_t* chunk_seg, const int32_t* comb_seg, int64_t ncomb,
                   const int32_t* seg_ptr, int64_t nseg, int64_t h, int reduce, int act, float alpha, float* P,
                   void* out, float* amax, hipStream_t stream) {
  constexpr int N = Piece<T, VEC>::N;
  if (nchunks > 0) {
    const int g1 = grid_for(nchunks * (h / N), 256, 256 * 32);
    NT_DISPATCH_RA(reduce, act,
                   (seg_chunk_partial<T, VEC, R_, A_><<<g1, 256, 0, stream>>>(
                       (const T*)X, perm, chunk_pos, chunk_seg, nchunks, h, act, alpha, P, (T*)out, amax)));
    NT_LAUNCH_CHECK();
  }
  if (chunk_seg == nullptr) ncomb = nseg;
  launch_combine_r<T, VEC>(reduce, P, chunk_ptr, seg_ptr, chunk_seg ? comb_seg : nullptr, ncomb, h, (T*)out, amax,
                           stream);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

}  // namespace
}  // namespace nt

extern "C" int nt_segment_reduce_chunked(const void* X, const int32_t* perm, const int32_t* chunk_pos,
                                         int64_t nchunks, const int32_t* chunk_ptr, const int32_t* chunk_seg,
                                         const int32_t* comb_seg, int64_t ncomb, const int32_t* seg_ptr,
                                         int64_t nseg, int64_t h, int reduce, int act, float act_alpha, int dtype,
                                         float* partial, void* out, float* amax_out, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32 || dtype == NT_BF16, NT_EUNSUPPORTED, "dtype must be NT_F32 or NT_BF16");
  NT_REQUIRE(valid_reduce(reduce) && valid_act(act), NT_EINVAL, "bad reduce/act code");
  NT_REQUIRE(nseg >= 0 && nchunks >= 0 && h > 0 && ncomb >= 0 && ncomb <= nseg, NT_EINVAL, "bad sizes");
  if (nseg == 0) return NT_OK;
  NT_REQUIRE(chunk_ptr && seg_ptr && out && (nchunks == 0 || (X && chunk_pos && partial)), NT_EINVAL,
             "NULL pointer");
  NT_REQUIRE(chunk_seg == nullptr || ncomb == 0 || comb_seg != nullptr, NT_EINVAL, "chunk_seg needs comb_seg");
  hipStream_t stream = as_stream(stream_);
  const bool al = aligned16(X) && aligned16(out) && aligned16(partial);
  if (dtype == NT_F32)
    return (h % 4 == 0 && al)
               ? launch_chunked<float, true>(X, perm, chunk_pos, nchunks, chunk_ptr, chunk_seg, comb_seg, ncomb,
                                             seg_ptr, nseg, h, reduce, act, act_alpha, partial, out, amax_out, stream)
               : launch_chunked<float, false>(X, perm, chunk_pos, nchunks, chunk_ptr, chunk_seg, comb_seg, ncomb,
                                              seg_ptr, nseg, h, reduce, act, act_alpha, partial, out, amax_out,
                                              stream);
  return (h % 8 == 0 && al)
             ? launch_chunked<bf16_raw, true>(X, perm, chunk_pos, nchunks, chunk_ptr, chunk_seg, comb_seg, ncomb,
                                              seg_ptr, nseg, h, reduce, act, act_alpha, partial, out, nullptr, stream)
             : launch_chunked<bf16_raw, false>(X, perm, chunk_pos, nchunks, chunk_ptr, chunk_seg, comb_seg, ncomb,
                                               seg_ptr, nseg, h, reduce, act, act_alpha, partial, out, nullptr,
                                               stream);
}

extern "C" int nt_dmpnn_init_chunked(const void* Xv, const void* Xe, const int64_t* src, const int32_t* perm,
                                     const int32_t* chunk_pos, int64_t nchunks, const int32_t* chunk_ptr,
                                     const int32_t* chunk_seg, const int32_t* comb_seg, int64_t ncomb,
                                     const int32_t* seg_ptr, int64_t V, int64_t E, int64_t h, int act,
                                     float act_alpha, int reduce, int dtype, float* partial, void* H0, void* S,
                                     float* amax_out, int64_t ld_out, const int32_t* chunk_ids, int64_t nids,
                                     void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32, NT_EUNSUPPORTED, "nt_dmpnn_init_chunked is fp32 only");
  NT_REQUIRE(valid_reduce(reduce) && valid_act(act), NT_EINVAL, "bad reduce/act code");
  NT_REQUIRE(V >= 0 && E >= 0 && nchunks >= 0 && h > 0 && ncomb >= 0 && ncomb <= V && nids >= 0 &&
                 nids <= nchunks, NT_EINVAL, "bad sizes");
  if (V == 0) return NT_OK;
  NT_REQUIRE(chunk_ptr && seg_ptr && S && (nchunks == 0 || (Xv && Xe && src && perm && chunk_pos && partial && H0)),
             NT_EINVAL, "NULL pointer");
  NT_REQUIRE(chunk_seg == nullptr || ncomb == 0 || comb_seg != nullptr, NT_EINVAL, "chunk_seg needs comb_seg");
  hipStream_t stream = as_stream(stream_);
  const bool al = aligned16(Xv) && aligned16(Xe) && aligned16(H0) && aligned16(S) && aligned16(partial);
  if (ld_out == 0) ld_out = h;
  NT_REQUIRE(ld_out == h || (h % 4 == 0 && ld_out % 4 == 0 && ld_out > h && al), NT_EINVAL,
             "padded rows need h % 4 == 0, ld_out % 4 == 0 and 16-byte aligned pointers");
  return (h % 4 == 0 && al)
             ? launch_init_chunked<true>((const float*)Xv, (const float*)Xe, src, perm, chunk_pos, nchunks, chunk_ptr,
                                         chunk_seg, comb_seg, ncomb, seg_ptr, V, h, reduce, act, act_alpha, partial,
                                         (float*)H0, (float*)S, amax_out, ld_out, chunk_ids, nids, stream)
             : launch_init_chunked<false>((const float*)Xv, (const float*)Xe, src, perm, chunk_pos, nchunks,
                                          chunk_ptr, chunk_seg, comb_seg, ncomb, seg_ptr, V, h, reduce, act,
                                          act_alpha, partial, (float*)H0, (float*)S, amax_out, ld_out, chunk_ids, nids,
                                          stream);
}

// The fused layer's hub sub-run partials combined per hub (nt_dmpnn_hub_combine): pass 2 of the
// chunked reduce with the hubs' slot ranges as the chunk CSR (slot_ptr[v] = slots before node v).
extern "C" int nt_dmpnn_hub_combine(const void* partial, const int32_t* hubs, const int32_t* slot_ptr, int64_t nhub,
                                    const int32_t* seg_ptr, int64_t V, int64_t h, int reduce, int dtype,
                                    float* amax_out, void* out, int64_t ld, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32, NT_EUNSUPPORTED, "nt_dmpnn_hub_combine: fp32 only");
  NT_REQUIRE(valid_reduce(reduce), NT_EINVAL, "bad reduce code");
  NT_REQUIRE(nhub >= 0 && nhub <= V && h > 0 && h % 4 == 0, NT_EINVAL, "bad sizes (h % 4 == 0)");
  if (ld == 0) ld = h;
  NT_REQUIRE(ld >= h && ld % 4 == 0, NT_EINVAL, "row pitch must be >= h and a multiple of 4");
  if (nhub == 0) return NT_OK;
  NT_REQUIRE(partial && hubs && slot_ptr && seg_ptr && out, NT_EINVAL, "NULL pointer");
  NT_REQUIRE(aligned16(partial) && aligned16(out), NT_EINVAL, "feature pointers must be 16-byte aligned");
  launch_combine_r<float, true>(reduce, (const float*)partial, slot_ptr, seg_ptr, hubs, nhub, h, (float*)out, amax_out,
                                as_stream(stream_), ld);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

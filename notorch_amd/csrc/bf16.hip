// bf16 storage path of the D-MPNN forward (BASELINE config 3: ZINC-shaped batches, depth 5,
// hidden 512, bf16).  Same math as the fp32 kernels (chemprop.py:28-43,81-88, residual.py:27-28,
// agg.py:23-47); feature rows, weights and bias are bf16 in HBM, every sum and product runs in fp32
// and each stored element is rounded to bf16 once (round-to-nearest-even, v_cvt_pk_bf16_f32).
//
//   init_bf16          H0[e] = Xv[src e] + Xe[e];  S[v] = R_{e->v} act(H0[e])          (3E+V rows)
//   segment_reduce     out[s] = R_{j in s} act(X[perm j])                                 (E+V rows)
//   update_bf16        H'[e] = H[e] + W (S[src e] - act(H[rev e])) + b                    (4 rows/edge)
//
// update_bf16 is a 64-edge-tile MFMA kernel (v_mfma_f32_16x16x32_bf16, fp32 accumulators):
//   1. gather: the four waves form A = S[src] - act(H[rev]) for the tile's 64 edges (one wave per
//      row, 16 B per lane, so a 512-wide bf16 row is one 1 KiB coalesced read) and store it as bf16
//      into LDS (row stride Kp*2 + 16 B: the fragment reads below are bank-conflict free);
//   2. MFMA: wave w owns column tiles w, w+4, ... (<= 8 of 16 columns) for all 64 rows: per 32-deep
//      k step it reads 4 A fragments from LDS and streams its B fragments from the packed weight
//      image (L2-resident: 512 KiB per layer at h = 512; one 1 KiB coalesced load per fragment,
//      prefetched one k step ahead);
//   3. epilogue: accumulators are staged through LDS (fp32, 256 columns per pass) and written as
//      whole 16-B row pieces with + bias + residual, rounded to bf16 once.
// Two workgroups per CU (66.5 KiB LDS each) overlap one tile's gather with the other's MFMAs.
// HBM bytes per edge: 4 rows x 2h (read H, gather S[src], gather H[rev], write H') + 16 B indices.
#include "bf16.hpp"

namespace nt {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short bf16_t;  // raw bf16 storage

__device__ __forceinline__ float bf2f(bf16_t u) { return __uint_as_float((unsigned)u << 16); }
__device__ __forceinline__ bf16_t f2bf(float x) { return __builtin_bit_cast(bf16_t, (__bf16)x); }

// W consecutive bf16 (W = 8: one 16-B piece, 16-B aligned; W = 1: one element) <-> fp32
template <int W>
__device__ __forceinline__ void load_chunk(const bf16_t* __restrict__ p, float (&x)[W]) {
  if constexpr (W == 8) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    const unsigned u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      x[2 * i] = __uint_as_float(u[i] << 16);
      x[2 * i + 1] = __uint_as_float(u[i] & 0xffff0000u);
    }
  } else {
    x[0] = bf2f(*p);
  }
}

template <int W>
__device__ __forceinline__ void store_chunk(bf16_t* __restrict__ p, const float (&x)[W]) {
  if constexpr (W == 8) {
    bf16x8 v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (__bf16)x[i];
    *reinterpret_cast<uint4*>(p) = __builtin_bit_cast(uint4, v);
  } else {
    *p = f2bf(x[0]);
  }
}

// round-trip through bf16 (the value a bf16 tensor would hold)
__device__ __forceinline__ float rbf(float x) { return bf2f(f2bf(x)); }

// ------------------------------------------------------------------------------ segment reduce
template <int R, int ACT, int W>
__global__ void __launch_bounds__(256) segment_reduce_bf16(
    const bf16_t* __restrict__ X, const int32_t* __restrict__ seg_ptr,
    const int32_t* __restrict__ perm, int64_t nseg, int64_t h, int act, float alpha,
    bf16_t* __restrict__ out) {
  const int64_t hw = h / W;
  const int64_t total = nseg * hw;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = t / hw, c = (t - s * hw) * W;
    const int32_t b = seg_ptr[s], e = seg_ptr[s + 1];
    Reducer<R> r[W];
#pragma unroll
    for (int i = 0; i < W; ++i) r[i].init();
    for (int32_t j = b; j < e; ++j) {
      const int64_t row = perm ? perm[j] : j;
      float x[W];
      load_chunk<W>(X + row * h + c, x);
#pragma unroll
      for (int i = 0; i < W; ++i) r[i].push(act_t<ACT>(x[i], act, alpha));
    }
    float y[W];
#pragma unroll
    for (int i = 0; i < W; ++i) y[i] = r[i].result();
    store_chunk<W>(out + s * h + c, y);
  }
}

// ------------------------------------------------------------------------------ init
template <int R, int ACT, int W>
__global__ void __launch_bounds__(256) init_aggregate_bf16(
    const bf16_t* __restrict__ Xv, const bf16_t* __restrict__ Xe, const int64_t* __restrict__ src,
    const int32_t* __restrict__ seg_ptr, const int32_t* __restrict__ perm, int64_t V, int64_t h,
    int act, float alpha, bf16_t* __restrict__ H0, bf16_t* __restrict__ S) {
  const int64_t hw = h / W;
  const int64_t total = V * hw;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = t / hw, c = (t - v * hw) * W;
    const int32_t b = seg_ptr[v], e = seg_ptr[v + 1];
    Reducer<R> r[W];
#pragma unroll
    for (int i = 0; i < W; ++i) r[i].init();
    for (int32_t j = b; j < e; ++j) {
      const int64_t ed = perm[j];
      float xv[W], xe[W], x[W];
      load_chunk<W>(Xv + src[ed] * h + c, xv);
      load_chunk<W>(Xe + ed * h + c, xe);
#pragma unroll
      for (int i = 0; i < W; ++i) x[i] = rbf(xv[i] + xe[i]);  // H0 as stored
      store_chunk<W>(H0 + ed * h + c, x);
#pragma unroll
      for (int i = 0; i < W; ++i) r[i].push(act_t<ACT>(x[i], act, alpha));
    }
    float y[W];
#pragma unroll
    for (int i = 0; i < W; ++i) y[i] = r[i].result();
    store_chunk<W>(S + v * h + c, y);
  }
}

template <int W>
__global__ void __launch_bounds__(256) init_only_bf16(const bf16_t* __restrict__ Xv,
                                                      const bf16_t* __restrict__ Xe,
                                                      const int64_t* __restrict__ src, int64_t E,
                                                      int64_t h, bf16_t* __restrict__ H0) {
  const int64_t hw = h / W;
  const int64_t total = E * hw;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = t / hw, c = (t - e * hw) * W;
    float xv[W], xe[W];
    load_chunk<W>(Xv + src[e] * h + c, xv);
    load_chunk<W>(Xe + e * h + c, xe);
#pragma unroll
    for (int i = 0; i < W; ++i) xv[i] += xe[i];
    store_chunk<W>(H0 + e * h + c, xv);
  }
}

// ------------------------------------------------------------------------------ weight image
// Wp[ks][nt][lane] = 8 bf16: W[n][k], n = 16 nt + (lane & 15), k = 32 ks + 8 (lane >> 4) + j
// (zero outside [0, h)) — exactly the B fragment of v_mfma_f32_16x16x32_bf16 for out = A W^T.
__global__ void __launch_bounds__(256) pack_bf16(const bf16_t* __restrict__ W, int64_t nlayers,
                                                 int64_t h, int KS, int NTn, int64_t layer_stride16,
                                                 uint4* __restrict__ Wp) {
  const int64_t per_layer = (int64_t)KS * NTn * 64;
  const int64_t total = nlayers * per_layer;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t l = t / per_layer;
    int64_t r = t - l * per_layer;
    const int lane = (int)(r & 63);
    r >>= 6;
    const int nt = (int)(r % NTn);
    const int ks = (int)(r / NTn);
    const int64_t n = 16 * nt + (lane & 15);
    const int64_t k0 = 32 * ks + 8 * (lane >> 4);
    const bf16_t* Wl = W + l * h * h;
    unsigned short v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (n < h && k0 + j < h) ? Wl[n * h + k0 + j] : (bf16_t)0;
    uint4 o;
    o.x = v[0] | ((unsigned)v[1] << 16);
    o.y = v[2] | ((unsigned)v[3] << 16);
    o.z = v[4] | ((unsigned)v[5] << 16);
    o.w = v[6] | ((unsigned)v[7] << 16);
    Wp[l * layer_stride16 + ((int64_t)ks * NTn + nt) * 64 + lane] = o;
  }
}

// ------------------------------------------------------------------------------ update
constexpr int kM = 64;        // edges per tile
constexpr int kThreads = 256;  // 4 waves
constexpr int kNWMax = 8;     // column tiles per wave at h = 512 (NW = ceil(ceil(h/16) / 4))
constexpr int kSO = 260;      // staging row stride (floats): 256 columns + 4 (conflict-free writes)
constexpr int kStageB = kM * kSO * 4;  // 66,560 B

__host__ __device__ constexpr int a_row_bytes(int KS) { return KS * 64 + 16; }
inline int lds_bytes_bf16(int KS) {
  const int a = kM * a_row_bytes(KS);
  return a > kStageB ? a : kStageB;
}

template <int ACT, int W, int NW>
__global__ void __launch_bounds__(kThreads, 2) update_bf16_kernel(
    const bf16_t* __restrict__ H, const bf16_t* __restrict__ S, const int64_t* __restrict__ src,
    const int64_t* __restrict__ rev, const uint4* __restrict__ Wp, const bf16_t* __restrict__ bias,
    int64_t V, int64_t E, int h, int KS, int NTn, int residual, int act, float alpha,
    bf16_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  __shared__ int64_t soff[kM], qoff[kM];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t e0 = (int64_t)blockIdx.x * kM;
  const int lda = a_row_bytes(KS);

  if (tid < kM) {
    const int64_t e = e0 + tid;
    int64_t so = -1, qo = -1;
    if (e < E) {
      const int64_t s = src[e], q = rev[e];
      if (s >= 0 && s < V) so = s * h;
      if (q >= 0 && q < E) qo = q * h;
    }
    soff[tid] = so;
    qoff[tid] = qo;
  }
  // Column tile j of this wave is nt = w + 4 j, j < NW.  A wave's last tile may lie past NTn (h not
  // a multiple of 64): its loads are clamped to a valid fragment and its result is never stored,
  // so every load and MFMA below is unconditional (no branch for hipcc to drain vmcnt in front of).
  int boff[NW];
#pragma unroll
  for (int j = 0; j < NW; ++j) boff[j] = (w + 4 * j < NTn ? w + 4 * j : NTn - 1) * 64 + lane;
  const int64_t kstride = (int64_t)NTn * 64;
  // B fragments of the first k step, in flight during the gather
  uint4 bcur[NW];
#pragma unroll
  for (int j = 0; j < NW; ++j) bcur[j] = Wp[boff[j]];
  __syncthreads();

  // ---- 1. gather A = S[src] - act(H[rev]) (fp32) -> bf16 LDS tile [64][Kp] ----
  {
    const int chunks = KS * 4;  // 8-element pieces per padded row
    constexpr int kRU = 4;      // rows in flight per wave
    for (int r0 = w * kRU; r0 < kM; r0 += 4 * kRU) {
      for (int c = lane; c < chunks; c += 64) {
        const int k0 = c * 8;
        float sv[kRU][8], qv[kRU][8];
#pragma unroll
        for (int u = 0; u < kRU; ++u) {
          const int64_t so = soff[r0 + u], qo = qoff[r0 + u];
          if constexpr (W == 8) {
            // clamped, unconditional loads; out-of-range pieces are zeroed after the load
            const int kc = k0 < h ? k0 : h - 8;
            load_chunk<8>(S + (so >= 0 ? so : 0) + kc, sv[u]);
            load_chunk<8>(H + (qo >= 0 ? qo : 0) + kc, qv[u]);
            const bool sok = so >= 0 && k0 < h, qok = qo >= 0 && k0 < h;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              sv[u][i] = sok ? sv[u][i] : 0.f;
              qv[u][i] = qok ? qv[u][i] : 0.f;
            }
          } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              const bool in = k0 + i < h;
              sv[u][i] = (in && so >= 0) ? bf2f(S[so + k0 + i]) : 0.f;
              qv[u][i] = (in && qo >= 0) ? bf2f(H[qo + k0 + i]) : 0.f;
            }
          }
        }
#pragma unroll
        for (int u = 0; u < kRU; ++u) {
          bf16x8 a;
#pragma unroll
          for (int i = 0; i < 8; ++i) a[i] = (__bf16)(sv[u][i] - act_t<ACT>(qv[u][i], act, alpha));
          *reinterpret_cast<uint4*>(lds + (r0 + u) * lda + c * 16) = __builtin_bit_cast(uint4, a);
        }
      }
    }
  }
  __syncthreads();

  // ---- 2. MFMA over k: acc[mt][j] = rows 16 mt.., columns of tile w + 4 j ----
  f32x4 acc[4][NW];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int j = 0; j < NW; ++j) acc[mt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const char* arow = lds + (lane & 15) * lda + 16 * (lane >> 4);
  for (int ks = 0; ks < KS; ++ks) {
    // next step's fragments (the last step re-reads its own: no branch, no drain)
    const int64_t kn = (ks + 1 < KS ? ks + 1 : ks) * kstride;
    uint4 bnext[NW];
#pragma unroll
    for (int j = 0; j < NW; ++j) bnext[j] = Wp[kn + boff[j]];
    bf16x8 a[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
      a[mt] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(arow + 16 * mt * lda + 64 * ks));
#pragma unroll
    for (int j = 0; j < NW; ++j) {
      const bf16x8 b = __builtin_bit_cast(bf16x8, bcur[j]);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], b, acc[mt][j], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NW; ++j) bcur[j] = bnext[j];
  }
  __syncthreads();  // every wave is done with the A tile: its LDS becomes the staging tile

  // ---- 3. epilogue: 256 columns per pass through LDS, + bias + residual, bf16 rows ----
  float* stage = reinterpret_cast<float*>(lds);
  const int Np = NTn * 16;
  // p and jj fully unrolled: acc[][j] must only ever be indexed by constants, or it lands in scratch
#pragma unroll
  for (int p = 0; p < (NW + 3) / 4; ++p) {
    if (p * 256 >= Np) break;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int j = 4 * p + jj;
      if (j < NW && w + 4 * j < NTn) {
        const int sc = 16 * w + 64 * jj + (lane & 15);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) stage[(16 * mt + 4 * (lane >> 4) + r) * kSO + sc] = acc[mt][j][r];
      }
    }
    __syncthreads();
    const int n0 = 256 * p;
    const int ncols = h - n0 < 256 ? h - n0 : 256;
    if constexpr (W == 8) {
      for (int i = tid; i < kM * 32; i += kThreads) {
        const int r = i >> 5, c = (i & 31) * 8;
        const int64_t e = e0 + r;
        if (c < ncols && e < E) {
          float y[8], hres[8], bb[8];
          const float* st = stage + r * kSO + c;
#pragma unroll
          for (int q = 0; q < 8; ++q) y[q] = st[q];
          if (bias) {
            load_chunk<8>(bias + n0 + c, bb);
#pragma unroll
            for (int q = 0; q < 8; ++q) y[q] += bb[q];
          }
          if (residual) {
            load_chunk<8>(H + e * h + n0 + c, hres);
#pragma unroll
            for (int q = 0; q < 8; ++q) y[q] += hres[q];
          }
          store_chunk<8>(out + e * h + n0 + c, y);
        }
      }
    } else {
      for (int i = tid; i < kM * 256; i += kThreads) {
        const int r = i >> 8, c = i & 255;
        const int64_t e = e0 + r;
        if (c < ncols && e < E) {
          float y = stage[r * kSO + c];
          if (bias) y += bf2f(bias[n0 + c]);
          if (residual) y += bf2f(H[e * h + n0 + c]);
          out[e * h + n0 + c] = f2bf(y);
        }
      }
    }
    __syncthreads();
  }
}

static bool valid_reduce(int r) { return r >= NT_SUM && r <= NT_MIN; }

#define NT_BF_DISPATCH_A(ACT, LAUNCH)                                            \
  do {                                                                           \
    if ((ACT) == NT_ACT_IDENTITY) { constexpr int A_ = NT_ACT_IDENTITY; LAUNCH; } \
    else if ((ACT) == NT_ACT_RELU) { constexpr int A_ = NT_ACT_RELU; LAUNCH; }    \
    else { constexpr int A_ = -1; LAUNCH; }                                      \
  } while (0)
#define NT_BF_DISPATCH_RA(REDUCE, ACT, LAUNCH)                                                  \
  do {                                                                                          \
    switch (REDUCE) {                                                                           \
      case NT_SUM: { constexpr int R_ = NT_SUM; NT_BF_DISPATCH_A(ACT, LAUNCH); } break;   \
      case NT_MEAN: { constexpr int R_ = NT_MEAN; NT_BF_DISPATCH_A(ACT, LAUNCH); } break; \
      case NT_MAX: { constexpr int R_ = NT_MAX; NT_BF_DISPATCH_A(ACT, LAUNCH); } break;   \
      case NT_MIN: { constexpr int R_ = NT_MIN; NT_BF_DISPATCH_A(ACT, LAUNCH); } break;   \
    }                                                                                           \
  } while (0)

template <int ACT, int W, int NW>
int launch_upd(const void* H, const void* S, const int64_t* src, const int64_t* rev, const void* Wp,
               const void* b, int64_t V, int64_t E, int64_t h, int residual, int act, float alpha,
               void* H_out, hipStream_t stream) {
  const int KS = (int)((h + 31) / 32), NTn = (int)((h + 15) / 16);
  const int64_t grid = (E + kM - 1) / kM;
  const int lds = lds_bytes_bf16(KS);
  auto kern = update_bf16_kernel<ACT, W, NW>;
  if (lds > 64 * 1024)
    NT_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  kern<<<(unsigned)grid, kThreads, lds, stream>>>(
      (const bf16_t*)H, (const bf16_t*)S, src, rev, (const uint4*)Wp, (const bf16_t*)b, V, E, (int)h,
      KS, NTn, residual, act, alpha, (bf16_t*)H_out);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

}  // namespace

int launch_segment_reduce_bf16(const void* X, const int32_t* seg_ptr, const int32_t* perm,
                               int64_t nseg, int64_t h, int reduce, int act, float alpha, void* out,
                               hipStream_t stream) {
  NT_REQUIRE(valid_reduce(reduce), NT_EINVAL, "bad reduce code");
  const bool vec = h % 8 == 0 && aligned16(X) && aligned16(out);
  if (vec) {
    const int grid = grid_for(nseg * (h / 8), 256, 256 * 32);
    NT_BF_DISPATCH_RA(reduce, act,
                      (segment_reduce_bf16<R_, A_, 8><<<grid, 256, 0, stream>>>(
                          (const bf16_t*)X, seg_ptr, perm, nseg, h, act, alpha, (bf16_t*)out)));
  } else {
    const int grid = grid_for(nseg * h, 256, 256 * 32);
    NT_BF_DISPATCH_RA(reduce, act,
                      (segment_reduce_bf16<R_, A_, 1><<<grid, 256, 0, stream>>>(
                          (const bf16_t*)X, seg_ptr, perm, nseg, h, act, alpha, (bf16_t*)out)));
  }
  NT_LAUNCH_CHECK();
  return NT_OK;
}

int launch_init_bf16(const void* Xv, const void* Xe, const int64_t* src, const int32_t* seg_ptr,
                     const int32_t* perm, int64_t V, int64_t E, int64_t h, int act, float alpha,
                     int reduce, void* H0, void* S, hipStream_t stream) {
  NT_REQUIRE(valid_reduce(reduce), NT_EINVAL, "bad reduce code");
  const bool vec = h % 8 == 0 && aligned16(Xv) && aligned16(Xe) && aligned16(H0) &&
                   (S == nullptr || aligned16(S));
  if (S != nullptr) {
    if (V == 0) return NT_OK;
    NT_REQUIRE(seg_ptr && perm, NT_EINVAL, "fused aggregation needs the dst CSR");
    NT_REQUIRE(E == 0 || (Xv && Xe && src && H0), NT_EINVAL, "NULL pointer");
    if (vec) {
      const int grid = grid_for(V * (h / 8), 256, 256 * 32);
      NT_BF_DISPATCH_RA(reduce, act,
                        (init_aggregate_bf16<R_, A_, 8><<<grid, 256, 0, stream>>>(
                            (const bf16_t*)Xv, (const bf16_t*)Xe, src, seg_ptr, perm, V, h, act,
                            alpha, (bf16_t*)H0, (bf16_t*)S)));
    } else {
      const int grid = grid_for(V * h, 256, 256 * 32);
      NT_BF_DISPATCH_RA(reduce, act,
                        (init_aggregate_bf16<R_, A_, 1><<<grid, 256, 0, stream>>>(
                            (const bf16_t*)Xv, (const bf16_t*)Xe, src, seg_ptr, perm, V, h, act,
                            alpha, (bf16_t*)H0, (bf16_t*)S)));
    }
  } else {
    if (E == 0) return NT_OK;
    NT_REQUIRE(Xv && Xe && src && H0, NT_EINVAL, "NULL pointer");
    if (vec)
      init_only_bf16<8><<<grid_for(E * (h / 8), 256, 256 * 32), 256, 0, stream>>>(
          (const bf16_t*)Xv, (const bf16_t*)Xe, src, E, h, (bf16_t*)H0);
    else
      init_only_bf16<1><<<grid_for(E * h, 256, 256 * 32), 256, 0, stream>>>(
          (const bf16_t*)Xv, (const bf16_t*)Xe, src, E, h, (bf16_t*)H0);
  }
  NT_LAUNCH_CHECK();
  return NT_OK;
}

size_t bf16_image_bytes(int64_t h) {
  const int64_t KS = (h + 31) / 32, NTn = (h + 15) / 16;
  return (size_t)KS * NTn * 64 * 16;
}

int pack_weight_bf16(const void* W, int64_t nlayers, int64_t h, int64_t layer_stride_bytes, void* Wp,
                     hipStream_t stream) {
  NT_REQUIRE(layer_stride_bytes % 16 == 0, NT_EINVAL, "internal: layer stride");
  const int KS = (int)((h + 31) / 32), NTn = (int)((h + 15) / 16);
  const int64_t total = nlayers * KS * NTn * 64;
  pack_bf16<<<grid_for(total, 256), 256, 0, stream>>>((const bf16_t*)W, nlayers, h, KS, NTn,
                                                      layer_stride_bytes / 16, (uint4*)Wp);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

template <int ACT, int W>
static int launch_upd_nw(const void* H, const void* S, const int64_t* src, const int64_t* rev,
                  const void* Wp, const void* b, int64_t V, int64_t E, int64_t h, int residual,
                  int act, float alpha, void* H_out, hipStream_t stream) {
  const int nw = (int)(((h + 15) / 16 + 3) / 4);
  switch (nw) {
#define NT_NW(N) \
  case N: return launch_upd<ACT, W, N>(H, S, src, rev, Wp, b, V, E, h, residual, act, alpha, H_out, stream);
    NT_NW(1) NT_NW(2) NT_NW(3) NT_NW(4) NT_NW(5) NT_NW(6) NT_NW(7) NT_NW(8)
#undef NT_NW
  }
  set_error("bf16 update: no kernel for this hidden size");
  return NT_EUNSUPPORTED;
}

int launch_update_bf16(const void* H, const void* S, const int64_t* src, const int64_t* rev,
                       const void* Wp, const void* b, int64_t V, int64_t E, int64_t h, int residual,
                       int act, float alpha, void* H_out, hipStream_t stream) {
  NT_REQUIRE(h <= 4 * kNWMax * 16, NT_EUNSUPPORTED, "bf16 update supports h <= 512");
  NT_REQUIRE((E + kM - 1) / kM < (int64_t(1) << 31), NT_EINVAL, "too many edges");
  const bool vec = h % 8 == 0 && aligned16(H) && aligned16(S) && aligned16(H_out) &&
                   (b == nullptr || aligned16(b));
  if (vec)
    NT_BF_DISPATCH_A(act, return (launch_upd_nw<A_, 8>(H, S, src, rev, Wp, b, V, E, h, residual,
                                                       act, alpha, H_out, stream)));
  else
    NT_BF_DISPATCH_A(act, return (launch_upd_nw<A_, 1>(H, S, src, rev, Wp, b, V, E, h, residual,
                                                       act, alpha, H_out, stream)));
  return NT_OK;
}

}  // namespace nt

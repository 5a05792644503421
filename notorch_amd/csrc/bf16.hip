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

int cu_count();   // update_ps.hip
int xcd_count();  // update_ps.hip

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
// BF_ABL (variant builds only, tools/r5_bf16_abl.sh): 1 = gathers read row 0, 2 = W fragments of
// k step 0 only, 4 = no H' / S' stores, 8 = no residual loads, 16 = no MFMA.  Results are wrong.
#ifndef BF_ABL
#define BF_ABL 0
#endif
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

// Fused aggregation of the layer output (nt_dmpnn_update_fused): tiles are the tile plan's cuts of
// the dst-sorted edge order, so every node's in-edges are consecutive rows of one tile.
struct BfAgg {
  const int* tile_ptr;   // ntiles + 1 positions
  const int* perm;       // dst CSR permutation: position -> edge
  const int* dsts;       // position -> destination node
  int reduce, aact;
  float aalpha;
  bf16_t* S_out;         // V x h, rows of in-degree-0 nodes pre-zeroed by the caller
};

// S_out[node] piece = R over rows [r0, r1) of the staged values (already aact(stored H'))
template <int R>
__device__ __forceinline__ void reduce_rows(const float* stage, int r0, int r1, int c, float (&y)[8]) {
  Reducer<R> red[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) red[q].init();
  for (int r = r0; r < r1; ++r) {
    const float* st = stage + r * kSO + c;
#pragma unroll
    for (int q = 0; q < 8; ++q) red[q].push(st[q]);
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) y[q] = red[q].result();
}

// AGG: 0 = no aggregation; 1 = fused aggregation of the stored H' (final node scatter, identity);
// 2 = fused aggregation of act(H') (the next layer's chemprop.py:37-39, same act as this layer)
template <int ACT, int W, int NW, int AGG>
__global__ void __launch_bounds__(kThreads, 2) update_bf16_kernel(
    const bf16_t* __restrict__ H, const bf16_t* __restrict__ S, const int64_t* __restrict__ src,
    const int64_t* __restrict__ rev, const uint4* __restrict__ Wp, const bf16_t* __restrict__ bias,
    int64_t V, int64_t E, int h, int KS, int NTn, int residual, int act, float alpha,
    bf16_t* __restrict__ out, BfAgg agg, int ntiles, int nxcd) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  __shared__ int64_t soff[kM], qoff[kM], erow[kM];
  __shared__ int nstart[kM + 1], nnode[kM], nseg;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lda = a_row_bytes(KS);
  const int G = gridDim.x;
  // Column tile j of this wave is nt = w + 4 j, j < NW.  A wave's last tile may lie past NTn (h not
  // a multiple of 64): its loads are clamped to a valid fragment and its result is never stored,
  // so every load and MFMA below is unconditional (no branch for hipcc to drain vmcnt in front of).
  // (recomputed where used, not kept in registers: the column tile of fragment j, clamped)
  auto boff = [&](int j) { return (w + 4 * j < NTn ? w + 4 * j : NTn - 1) * 64 + lane; };
  const int64_t kstride = (int64_t)NTn * 64;

  // Persistent loop over tiles t = blockIdx.x + i G.  Wave 0 lane r holds row r's indices of the
  // NEXT tile, fetched in three dependent stages spread over the current tile (tile bounds before
  // the gather, edge / node ids before the MFMAs, src / rev before the epilogue) so the index
  // chain tile_ptr -> perm -> src, rev never stalls the pipeline.
  int cT = 0, cn = 0;           // stage A: tile start position and size
  int ce = -1;                  // stage B: edge of row `lane` (E < 2^31)
  int cnode = -1, cprev = -2;   // stage B: its destination node, and that of the row before
  int cs = -1, cq = -1;         // stage C: src / rev of that edge (-1 when out of range)
  auto stage_a = [&](int t) {
    if constexpr (AGG != 0) {
      cT = agg.tile_ptr[t];
      cn = agg.tile_ptr[t + 1] - cT;
    } else {
      cT = t * kM;
      cn = E - (int64_t)cT < kM ? (int)(E - cT) : kM;
    }
  };
  auto stage_b = [&]() {
    ce = -1;
    cnode = -1;
    cprev = -2;
    if (lane < cn) {
      if constexpr (AGG != 0) {
        ce = agg.perm[cT + lane];
        cnode = agg.dsts[cT + lane];
        cprev = lane > 0 ? agg.dsts[cT + lane - 1] : -2;
      } else {
        ce = cT + lane;
      }
    }
  };
  auto stage_c = [&]() {
    // dense mode (src = rev = NULL, nt_dmpnn_dense_matmul): row e of A is S[e]
    const int64_t s = ce >= 0 ? (src ? src[ce] : (int64_t)ce) : -1, q = (ce >= 0 && rev) ? rev[ce] : -1;
    cs = (s >= 0 && s < V) ? (int)s : -1;
    cq = (q >= 0 && q < E) ? (int)q : -1;
  };
  // XCD-aware walk (as update_pk.hip): blocks b and b + nxcd share an XCD; each XCD takes one
  // contiguous 1/nxcd of the tiles, so rows shared by neighbouring tiles stay in its L2.
  int t_first = blockIdx.x, t_step = G, t_end = ntiles;
  if (nxcd > 1 && G % nxcd == 0) {
    const int x = (int)blockIdx.x % nxcd, chunk = (ntiles + nxcd - 1) / nxcd;
    t_first = x * chunk + (int)blockIdx.x / nxcd;
    t_step = G / nxcd;
    t_end = min(ntiles, x * chunk + chunk);
  }
  if (w == 0 && t_first < t_end) {
    stage_a(t_first);
    stage_b();
    stage_c();
  }

  for (int t = t_first; t < t_end; t += t_step) {
    const bool has_next = t + t_step < t_end;
    if (w == 0) {  // publish this tile's indices (the previous tile's epilogue ended with a barrier)
      erow[lane] = ce;
      soff[lane] = cs >= 0 ? (int64_t)cs * h : -1;
      qoff[lane] = cq >= 0 ? (int64_t)cq * h : -1;
      if constexpr (AGG != 0) {  // segment starts of the tile's nodes (ballot + prefix popcount)
        const bool first = lane < cn && cnode != cprev;
        const unsigned long long m = __ballot(first);
        const int k = __popcll(m & ((1ull << lane) - 1ull));
        if (first) {
          nstart[k] = lane;
          nnode[k] = cnode;
        }
        if (lane == 0) {
          nseg = __popcll(m);
          nstart[__popcll(m)] = cn;
        }
      }
      if (has_next) stage_a(t + t_step);
    }
    // B fragments of the first k step, in flight during the gather
    uint4 bcur[NW];
#pragma unroll
    for (int j = 0; j < NW; ++j) bcur[j] = Wp[boff(j)];
    __syncthreads();

  // ---- 1. gather A = S[src] - act(H[rev]) (fp32) -> bf16 LDS tile [64][Kp] ----
  if constexpr (W == 8) {
    // wave w owns rows 16 w .. 16 w + 15; lane c takes the c-th 16-B piece of each row, and all 32
    // loads of the wave are issued before the first is consumed (latency hidden by depth)
    const int chunks = KS * 4;
    constexpr int kRG = 8;  // rows in flight per round (2 rounds of 8: 64 VGPRs of raw pieces)
    for (int idx = lane; idx < chunks * (16 / kRG); idx += 64) {
      const int c = idx % chunks, r0 = 16 * w + kRG * (idx / chunks);
      const int k0 = c * 8;
      const int kc = k0 < h ? k0 : h - 8;  // clamped, unconditional loads
      uint4 sraw[kRG], qraw[kRG];
#pragma unroll
      for (int u = 0; u < kRG; ++u) {
        const int64_t so = (BF_ABL & 1) ? 0 : soff[r0 + u], qo = (BF_ABL & 1) ? 0 : qoff[r0 + u];
        sraw[u] = *reinterpret_cast<const uint4*>(S + (so >= 0 ? so : 0) + kc);
        qraw[u] = *reinterpret_cast<const uint4*>(H + (qo >= 0 ? qo : 0) + kc);
      }
#pragma unroll
      for (int u = 0; u < kRG; ++u) {
        const int r = r0 + u;
        const bool sok = soff[r] >= 0 && k0 < h, qok = qoff[r] >= 0 && k0 < h;
        const unsigned su[4] = {sraw[u].x, sraw[u].y, sraw[u].z, sraw[u].w};
        const unsigned qu[4] = {qraw[u].x, qraw[u].y, qraw[u].z, qraw[u].w};
        bf16x8 a;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const unsigned sb = (i & 1) ? (su[i >> 1] & 0xffff0000u) : (su[i >> 1] << 16);
          const unsigned qb = (i & 1) ? (qu[i >> 1] & 0xffff0000u) : (qu[i >> 1] << 16);
          const float sv = sok ? __uint_as_float(sb) : 0.f;
          const float qv = qok ? __uint_as_float(qb) : 0.f;
          a[i] = (__bf16)(sv - act_t<ACT>(qv, act, alpha));
        }
        *reinterpret_cast<uint4*>(lds + r * lda + c * 16) = __builtin_bit_cast(uint4, a);
      }
    }
  } else {
    const int chunks = KS * 4;  // 8-element pieces per padded row
    constexpr int kRU = 4;      // rows in flight per wave
    for (int r0 = w * kRU; r0 < kM; r0 += 4 * kRU) {
      for (int c = lane; c < chunks; c += 64) {
        const int k0 = c * 8;
        float sv[kRU][8], qv[kRU][8];
#pragma unroll
        for (int u = 0; u < kRU; ++u) {
          const int64_t so = soff[r0 + u], qo = qoff[r0 + u];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const bool in = k0 + i < h;
            sv[u][i] = (in && so >= 0) ? bf2f(S[so + k0 + i]) : 0.f;
            qv[u][i] = (in && qo >= 0) ? bf2f(H[qo + k0 + i]) : 0.f;
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

    if (w == 0 && has_next) stage_b();

  // ---- 2. MFMA over k: acc[mt][j] = rows 16 mt.., columns of tile w + 4 j ----
  f32x4 acc[4][NW];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int j = 0; j < NW; ++j) acc[mt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const char* arow = lds + (lane & 15) * lda + 16 * (lane >> 4);
  for (int ks = 0; ks < KS; ++ks) {
    // next step's fragments (the last step re-reads its own: no branch, no drain)
    const int64_t kn = (BF_ABL & 2) ? 0 : (ks + 1 < KS ? ks + 1 : ks) * kstride;
    uint4 bnext[NW];
#pragma unroll
    for (int j = 0; j < NW; ++j) bnext[j] = Wp[kn + boff(j)];
    bf16x8 a[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
      a[mt] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(arow + 16 * mt * lda + 64 * ks));
#pragma unroll
    for (int j = 0; j < NW; ++j) {
      const bf16x8 b = __builtin_bit_cast(bf16x8, bcur[j]);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        if constexpr ((BF_ABL & 16) != 0) {
          acc[mt][j][0] += (float)a[mt][0] * (float)b[0];
        } else {
          acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], b, acc[mt][j], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < NW; ++j) bcur[j] = bnext[j];
  }
    if (w == 0 && has_next) stage_c();
  __syncthreads();  // every wave is done with the A tile: its LDS becomes the staging tile

  // ---- 3. epilogue: 256 columns per pass through LDS, + bias + residual, bf16 rows ----
  float* stage = reinterpret_cast<float*>(lds);
  const int Np = NTn * 16;
  // p and jj fully unrolled: acc[][j] must only ever be indexed by constants, or it lands in scratch
#pragma unroll
  for (int p = 0; p < (NW + 3) / 4; ++p) {
    if (p * 256 >= Np) break;
    const int n0 = 256 * p;
    const int ncols = h - n0 < 256 ? h - n0 : 256;
    // W == 8: thread (tid) owns column piece c = 8 (tid & 31) of rows (tid >> 5) + 8 it, it < 8;
    // its residual pieces are loaded before the staging round trip so their latency overlaps it
    constexpr int kIt = kM * 32 / kThreads;
    const int cpiece = 8 * (tid & 31);
    const bool cok = cpiece < ncols;
    // all residual pieces are in flight across the staging round trip (halving that for the fused
    // aggregation did not remove its spill and cost ~5% at config 3)
    constexpr int kPre = kIt;
    auto load_res = [&](int it) {
      const int64_t e = erow[(tid >> 5) + 8 * it];
      const bool ok = cok && e >= 0 && residual && (BF_ABL & 8) == 0;
      return *reinterpret_cast<const uint4*>(H + (ok ? e * h + n0 + cpiece : 0));
    };
    uint4 hres[kPre];
    if constexpr (W == 8) {
#pragma unroll
      for (int it = 0; it < kPre; ++it) hres[it] = load_res(it);
    }
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
    if constexpr (W == 8) {
      float bb[8];
      if (bias && cok) load_chunk<8>(bias + n0 + cpiece, bb);
      else for (int q = 0; q < 8; ++q) bb[q] = 0.f;
#pragma unroll
      for (int it = 0; it < kIt; ++it) {
        const int r = (tid >> 5) + 8 * it;
        const int64_t e = erow[r];
        if (cok && e >= 0) {
          float* st = stage + r * kSO + cpiece;
          const uint4 hr = it < kPre ? hres[it < kPre ? it : 0] : load_res(it);
          const unsigned hu[4] = {hr.x, hr.y, hr.z, hr.w};
          float y[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const unsigned hb = (q & 1) ? (hu[q >> 1] & 0xffff0000u) : (hu[q >> 1] << 16);
            y[q] = st[q] + bb[q] + (residual ? __uint_as_float(hb) : 0.f);
          }
          if constexpr ((BF_ABL & 4) == 0) store_chunk<8>(out + e * h + n0 + cpiece, y);
          if constexpr (AGG != 0) {  // the aggregation reads the stored (bf16) value, as unfused
#pragma unroll
            for (int q = 0; q < 8; ++q) st[q] = AGG == 2 ? act_t<ACT>(rbf(y[q]), act, alpha) : rbf(y[q]);
          }
        }
      }
      if constexpr (AGG != 0) {
        __syncthreads();
        for (int k = tid >> 5; k < nseg; k += kThreads / 32) {
          if (!cok) continue;
          float y[8];
          switch (agg.reduce) {
            case NT_SUM: reduce_rows<NT_SUM>(stage, nstart[k], nstart[k + 1], cpiece, y); break;
            case NT_MEAN: reduce_rows<NT_MEAN>(stage, nstart[k], nstart[k + 1], cpiece, y); break;
            case NT_MAX: reduce_rows<NT_MAX>(stage, nstart[k], nstart[k + 1], cpiece, y); break;
            default: reduce_rows<NT_MIN>(stage, nstart[k], nstart[k + 1], cpiece, y); break;
          }
          if constexpr ((BF_ABL & 4) == 0) store_chunk<8>(agg.S_out + (int64_t)nnode[k] * h + n0 + cpiece, y);
        }
      }
    } else {
      for (int i = tid; i < kM * 256; i += kThreads) {
        const int r = i >> 8, c = i & 255;
        const int64_t e = erow[r];
        if (c < ncols && e >= 0) {
          float y = stage[r * kSO + c];
          if (bias) y += bf2f(bias[n0 + c]);
          if (residual) y += bf2f(H[e * h + n0 + c]);
          out[e * h + n0 + c] = f2bf(y);
        }
      }
    }
    __syncthreads();
  }
  }  // tile loop
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

template <int ACT, int W, int NW, int AGG>
int launch_upd(const void* H, const void* S, const int64_t* src, const int64_t* rev, const void* Wp,
               const void* b, int64_t V, int64_t E, int64_t h, int residual, int act, float alpha,
               void* H_out, int64_t grid, const BfAgg& agg, hipStream_t stream) {
  const int KS = (int)((h + 31) / 32), NTn = (int)((h + 15) / 16);
  const int lds = lds_bytes_bf16(KS);
  auto kern = update_bf16_kernel<ACT, W, NW, AGG>;
  if (lds > 64 * 1024)
    NT_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  const int64_t slots = 2 * (int64_t)cu_count();  // two resident workgroups per CU (LDS-bound)
  const int64_t g = grid < slots ? grid : slots;
  set_last_kernel("update_bf16_kernel: two 4-wave workgroups per CU, 64-edge tiles");
  kern<<<(unsigned)g, kThreads, lds, stream>>>(
      (const bf16_t*)H, (const bf16_t*)S, src, rev, (const uint4*)Wp, (const bf16_t*)b, V, E, (int)h,
      KS, NTn, residual, act, alpha, (bf16_t*)H_out, agg, (int)grid, xcd_count());
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
    NT_REQUIRE(seg_ptr && (perm || E == 0), NT_EINVAL, "fused aggregation needs the dst CSR");
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

template <int ACT, int W, int AGG>
static int launch_upd_nw(const void* H, const void* S, const int64_t* src, const int64_t* rev,
                         const void* Wp, const void* b, int64_t V, int64_t E, int64_t h, int residual,
                         int act, float alpha, void* H_out, int64_t grid, const BfAgg& agg,
                         hipStream_t stream) {
  const int nw = (int)(((h + 15) / 16 + 3) / 4);
  switch (nw) {
#define NT_NW(N)                                                                                  \
  case N:                                                                                         \
    return launch_upd<ACT, W, N, AGG>(H, S, src, rev, Wp, b, V, E, h, residual, act, alpha, H_out, \
                                      grid, agg, stream);
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
  const int64_t grid = (E + kM - 1) / kM;
  NT_REQUIRE(grid < (int64_t(1) << 31), NT_EINVAL, "too many edges");
  const bool vec = h % 8 == 0 && aligned16(H) && aligned16(S) && aligned16(H_out) &&
                   (b == nullptr || aligned16(b));
  const BfAgg none{nullptr, nullptr, nullptr, 0, 0, 0.f, nullptr};
  if (vec)
    NT_BF_DISPATCH_A(act, return (launch_upd_nw<A_, 8, 0>(H, S, src, rev, Wp, b, V, E, h, residual,
                                                              act, alpha, H_out, grid, none, stream)));
  else
    NT_BF_DISPATCH_A(act, return (launch_upd_nw<A_, 1, 0>(H, S, src, rev, Wp, b, V, E, h, residual,
                                                              act, alpha, H_out, grid, none, stream)));
  return NT_OK;
}

bool bf16_fused_supported(int64_t h) { return h % 8 == 0 && h <= 4 * kNWMax * 16; }

int launch_update_bf16_fused(const void* H, const void* S, const int64_t* src, const int64_t* rev,
                             const void* Wp, const void* b, int64_t V, int64_t E, int64_t h,
                             int residual, int act, float alpha, const int32_t* tile_ptr,
                             int64_t ntiles, const int32_t* perm, const int32_t* dsts, int reduce,
                             int aact, float aalpha, void* H_out, void* S_out, hipStream_t stream) {
  if (tile_ptr == nullptr)  // no plan: the plain (unfused) kernel computes H_out only
    return launch_update_bf16(H, S, src, rev, Wp, b, V, E, h, residual, act, alpha, H_out, stream);
  NT_REQUIRE(bf16_fused_supported(h), NT_EUNSUPPORTED, "bf16 update_fused needs h % 8 == 0, h <= 512");
  NT_REQUIRE(perm && dsts && S_out && aligned16(S_out), NT_EINVAL, "fused aggregation needs perm, "
             "dst_sorted and a 16-byte aligned S_out");
  NT_REQUIRE(ntiles > 0 && ntiles < (int64_t(1) << 31), NT_EINVAL, "bad ntiles");
  // the kernel applies either identity (final node scatter) or this layer's own act (the next
  // layer's aggregation, which ChempropBlock guarantees uses the same activation)
  NT_REQUIRE(aact == NT_ACT_IDENTITY || (aact == act && aalpha == alpha), NT_EUNSUPPORTED,
             "bf16 update_fused: agg_act must be identity or equal to act");
  const BfAgg agg{tile_ptr, perm, dsts, reduce, aact, aalpha, (bf16_t*)S_out};
  if (aact == NT_ACT_IDENTITY)
    NT_BF_DISPATCH_A(act, return (launch_upd_nw<A_, 8, 1>(H, S, src, rev, Wp, b, V, E, h, residual,
                                                          act, alpha, H_out, ntiles, agg, stream)));
  else
    NT_BF_DISPATCH_A(act, return (launch_upd_nw<A_, 8, 2>(H, S, src, rev, Wp, b, V, E, h, residual,
                                                          act, alpha, H_out, ntiles, agg, stream)));
  return NT_OK;
}

}  // namespace nt

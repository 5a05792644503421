// Persistent producer/consumer D-MPNN layer update, optionally fused with the next aggregation
// ("ps"):
//
//   H_out[e] = (residual ? H[e] : 0) + W (S[src[e]] - act(H[rev[e]])) + b        (chemprop.py:36-43,
//                                                                                 residual.py:27-28)
//   S_out[v] = reduce_{e: dst[e] = v} aact(H_out[e])   (fused mode: the next layer's chemprop.py:37-39
//                                                        aggregation, or with aact = identity the
//                                                        final node scatter of chemprop.py:86)
//
// Numerics: update_x6.hip's bf16x6 fp32 emulation (six bf16 products of three-way splits, fp32
// accumulation) on v_mfma_f32_16x16x32_bf16; the aggregation sums in ascending edge id like the
// CPU scatter_add_ (positions come from the stable dst CSR).
//
// Why.  The per-layer work is ~370 MB of gathers/stores (HBM or Infinity Cache) plus 38 us of
// MFMA at h = 300; only a CU that keeps its memory pipe AND its matrix cores busy at the same time
// approaches that bound.  One workgroup per CU (persistent over tiles t = blockIdx, +grid, ...):
//   * waves 0-3 (consumers) run the MFMA loop of tile i out of LDS buffer i & 1: wave w owns the
//     16-column tiles w, w+4, ... of all 64 rows; W fragments stream from L2 straight into VGPRs
//     (pre-split image, next K step's tile j loaded as soon as this step's tile j is issued);
//   * waves 4-7 (producers) meanwhile finish tile i-1 (staged accumulators + bias + residual ->
//     H_out rows, and in fused mode the segmented reduction of those rows into S_out) and gather
//     tile i+1 (A = S[src] - act(H[rev]), fp32) into the other buffer.
// Tiles are ranges of positions of the dst-sorted edge order (row r <-> edge perm[T + r]) cut at
// node boundaries (nt_dmpnn_tile_plan), so every node's in-edges lie in one tile and S_out rows are
// complete when the tile's epilogue runs.  Without a plan (tile_ptr = NULL) tiles are 64
// consecutive edges and nothing is aggregated.
//
// LDS: two 64 x 76 x 16-B A buffers (155,648 B).  Piece p of row r lives in slot p ^ ((r >> 3) & 1)
// of a 76-piece row: conflict-free ds_read_b128 fragment reads (searched exhaustively for the
// gfx950 lane groups).  After the MFMA loop a buffer is reused as the [64][304] fp32 staging tile.
//
// Barriers per tile (all 512 threads): B3 after K step `kmid` (~70 % of the K loop; producers have finished reading the
// staging of tile i-1, so the gather may overwrite that buffer), B1 after the MFMA loop (tile i+1
//
// Diagnostic library only (make DIAG=1): moved out of update_ps.hip, which keeps the tile planner.
#include <stdlib.h>

#include <type_traits>

#include "../common.hpp"
#include "../update.hpp"

namespace nt {
int cu_count();  // update_ps.hip
// Diagnostic build (NT_PS_ABL=16): cycles summed over waves.  Producers: [0] finish, [1] wait B3,
// [2] gather, [3] wait B1+B2; consumers: [4] steps before B3, [5] wait B3, [6] steps after,
// [7] wait B1, [8] staging + B2; [9] producer waves, [10] consumer waves.
__device__ unsigned long long g_ps_stamps[12];

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kRows = 64;                 // rows (edges) per tile
constexpr int kPieces = 76;               // 16-B pieces per LDS A row (304 floats)
constexpr int kBufF4 = kRows * kPieces;   // 4864 float4 = 77,824 B per buffer
constexpr int kSO = 304;                  // staging row stride (floats)
constexpr int kThreads = 512;             // 4 consumer + 4 producer waves
static_assert(kRows * kSO <= 4 * kBufF4, "staging tile must fit an A buffer");

__device__ __forceinline__ int a_slot(int r, int p) { return r * kPieces + (p ^ ((r >> 3) & 1)); }

__device__ __forceinline__ void split3(const float (&x)[8], bf16x8& p0, bf16x8& p1, bf16x8& p2) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h0 = (__bf16)x[j];
    const float r1 = x[j] - (float)h0;
    const __bf16 h1 = (__bf16)r1;
    const float r2 = r1 - (float)h1;
    p0[j] = h0;
    p1[j] = h1;
    p2[j] = (__bf16)r2;
  }
}

__device__ __forceinline__ bf16x8 as_bf16x8(uint4 v) { return __builtin_bit_cast(bf16x8, v); }

struct TileRange {
  int T, n;  // first position, rows
};

__device__ __forceinline__ TileRange tile_range(const int* __restrict__ tile_ptr, int t, int64_t E) {
  if (tile_ptr) {
    const int a = tile_ptr[t], b = tile_ptr[t + 1];
    return {a, b - a};
  }
  const int64_t a = (int64_t)t * kRows;
  const int64_t n = E - a < kRows ? E - a : kRows;
  return {(int)a, (int)n};
}

struct Args {
  const float4* H4;
  const float4* S4;
  const int64_t* src;
  const int64_t* rev;
  const uint4* Wb;
  const float4* b4;
  int64_t V, E;
  int hv, nt16, residual, act;
  float alpha;
  const int* tile_ptr;  // NULL: 64-edge tiles in edge order, no aggregation
  int ntiles;
  const int* perm;      // dst CSR permutation (position -> edge), fused mode
  const int* dsts;      // node of every position, fused mode
  int reduce, aact;
  float aalpha;
  int kmid;
  float4* O4;
  float4* SO4;          // NULL: no aggregation
};

// ------------------------------------------------------------------------------------ producer
// Row edges of tile t for producer wave pw: lane l < 16 <-> row r = 4 l + pw (position T + r);
// -1 past the tile.  Issued one phase before the gather needs it.
__device__ __forceinline__ int gather_rows(const Args& a, int t, int pw, int lane) {
  int e = -1;
  if (lane < 16) {
    const TileRange tr = tile_range(a.tile_ptr, t, a.E);
    const int r = 4 * lane + pw;
    if (r < tr.n) e = a.perm ? a.perm[tr.T + r] : tr.T + r;
  }
  return e;
}

// Gather tile t into buffer `buf`: A[r][k] = S[src[e_r]][k] - act(H[rev[e_r]][k]) (rows >= n and
// pieces >= hv are zero).  Producer wave pw owns rows 4m + pw (m < 16); the wave's 16 x 76 row
// pieces are flattened over its lanes (19 per lane), every load issued before the first use, so
// the tile costs one index round trip and one data round trip.
template <int ACT>
__device__ __forceinline__ void gather_tile(const Args& a, int erow, float4* __restrict__ buf,
                                            int pw, int lane) {
  int soff = -1, qoff = -1;
  if (erow >= 0) {
    const int64_t s = a.src[erow], q = a.rev[erow];
    soff = (s >= 0 && s < a.V) ? (int)s * a.hv : -1;
    qoff = (q >= 0 && q < a.E) ? (int)q * a.hv : -1;
  }
  const int hv = a.hv;
  constexpr int NP = 16 * kPieces / 64;  // 19 pieces per lane, in two batches
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  auto batch = [&](auto k0_tag, auto nk_tag) {
    constexpr int K0 = decltype(k0_tag)::value, NK = decltype(nk_tag)::value;
    float4 sv[NK], qv[NK];
    int so[NK], qo[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int i = lane + 64 * (K0 + k);
      const int m = i / kPieces, pc = i - m * kPieces;
      so[k] = __shfl(soff, m);
      qo[k] = __shfl(qoff, m);
      const int cc = pc < hv ? pc : 0;
      sv[k] = a.S4[(so[k] >= 0 ? so[k] : 0) + cc];
      qv[k] = a.H4[(qo[k] >= 0 ? qo[k] : 0) + cc];
    }
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int i = lane + 64 * (K0 + k);
      const int m = i / kPieces, pc = i - m * kPieces;
      const bool in = pc < hv;
      const float4 mq = (in && qo[k] >= 0) ? act4_t<ACT>(qv[k], a.act, a.alpha) : z;
      buf[a_slot(4 * m + pw, pc)] = ((in && so[k] >= 0) ? sv[k] : z) - mq;
    }
  };
  batch(std::integral_constant<int, 0>{}, std::integral_constant<int, 10>{});
  batch(std::integral_constant<int, 10>{}, std::integral_constant<int, NP - 10>{});
}

__device__ __forceinline__ float reduce_step(float acc, float x, int reduce, bool first) {
  if (reduce == NT_MAX) return first ? x : fmaxf(acc, x);
  if (reduce == NT_MIN) return first ? x : fminf(acc, x);
  return acc + x;  // sum / mean
}

// First node boundary >= x among the tile's rows (fused mode), found by one wave: lane l looks
// at row x + l - 1 vs x + l; a ballot picks the first change.  Serial tail only past 63 rows.
__device__ __forceinline__ int align_row(const Args& a, const TileRange& tr, int x, int lane) {
  if (x <= 0) return 0;
  if (x >= tr.n) return tr.n;
  const int y = x + lane;
  const int yc = y < tr.n ? y : tr.n - 1;
  const int d1 = a.dsts[tr.T + yc], d0 = a.dsts[tr.T + yc - 1];
  const unsigned long long m = __ballot(y >= tr.n || d1 != d0);
  if (m) return x + (int)__builtin_ctzll(m) < tr.n ? x + (int)__builtin_ctzll(m) : tr.n;
  int z = x + 64;
  while (z < tr.n && a.dsts[tr.T + z] == a.dsts[tr.T + z - 1]) ++z;
  return z;
}

// Finish tile t from the staged accumulators in `so` ([64][kSO] fp32): H_out rows (+ bias
// + residual) and, in fused mode, the segmented reduction of those rows into S_out.  Producer
// wave pw owns a node-aligned quarter of the rows (every node's rows in one wave, so one lane
// reduces each S_out piece, in ascending position = ascending edge id order); lane l owns pieces l
// and l + 64 of every row.  Row edges and nodes are read once per wave (lane = row), broadcast with
// readlane; residual rows are loaded 8 rows ahead.
template <int AACT, bool SUMONLY, int FABL = 0>
__device__ __forceinline__ void finish_tile(const Args& a, int t, const float* __restrict__ so,
                                            int pw, int lane) {
  const TileRange tr = tile_range(a.tile_ptr, t, a.E);
  const int hv = a.hv;
  const bool fused = a.SO4 != nullptr;
  const int x0 = (pw * tr.n) >> 2, x1 = ((pw + 1) * tr.n) >> 2;
  const int rs = fused ? align_row(a, tr, x0, lane) : x0;
  const int re = pw == 3 ? tr.n : (fused ? align_row(a, tr, x1, lane) : x1);
  const int nr = re - rs;
  if (nr <= 0) return;
  int ev = tr.T + rs, vv = -1;
  if (lane < nr) {
    ev = a.perm ? a.perm[tr.T + rs + lane] : tr.T + rs + lane;
    if (fused) vv = a.dsts[tr.T + rs + lane];
  }
  const int c0 = lane, c1 = lane + 64;
  const bool in0 = c0 < hv, in1 = c1 < hv;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 b0 = (a.b4 && in0) ? a.b4[c0] : z, b1 = (a.b4 && in1) ? a.b4[c1] : z;
  float4 acc0 = z, acc1 = z;
  int cnt = 0;
  constexpr int U = 16;  // a wave's rows in one chunk for tiles up to 64 rows (all loads in flight)
  for (int r0 = 0; r0 < nr; r0 += U) {
    float4 h0[U], h1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = r0 + u < nr ? r0 + u : nr - 1;
      const int64_t e = __builtin_amdgcn_readlane(ev, r);
      if constexpr ((FABL & 32) != 0) {
        h0[u] = make_float4((float)e, 0.f, 0.f, 0.f);
        h1[u] = h0[u];
      } else {
        h0[u] = (a.residual && in0) ? a.H4[e * hv + c0] : z;
        h1[u] = (a.residual && in1) ? a.H4[e * hv + c1] : z;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = r0 + u;
      if (r < nr) {
        const int64_t e = __builtin_amdgcn_readlane(ev, r);
        const float* srow = so + (rs + r) * kSO;
        float4 o0 = z, o1 = z;
        if (in0) {
          o0 = (*reinterpret_cast<const float4*>(srow + 4 * c0) + b0) + h0[u];
          if constexpr ((FABL & 64) == 0) a.O4[e * hv + c0] = o0;
        }
        if (in1) {
          o1 = (*reinterpret_cast<const float4*>(srow + 4 * c1) + b1) + h1[u];
          if constexpr ((FABL & 64) == 0) a.O4[e * hv + c1] = o1;
        }
        if constexpr ((FABL & 64) != 0) {
          if (o0.x == 123.f && o1.y == 7.f) a.O4[0] = o0;  // keep the math live
        }
        if (fused) {
          const int v = __builtin_amdgcn_readlane(vv, r);
          const int vn = r + 1 < nr ? __builtin_amdgcn_readlane(vv, r + 1) : -1;
          const float4 m0 = act4_t<AACT>(o0, a.aact, a.aalpha);
          const float4 m1 = act4_t<AACT>(o1, a.aact, a.aalpha);
          if constexpr (SUMONLY) {
            acc0 = acc0 + m0;
            acc1 = acc1 + m1;
          } else {
            const bool first = cnt == 0;
            acc0.x = reduce_step(acc0.x, m0.x, a.reduce, first);
            acc0.y = reduce_step(acc0.y, m0.y, a.reduce, first);
            acc0.z = reduce_step(acc0.z, m0.z, a.reduce, first);
            acc0.w = reduce_step(acc0.w, m0.w, a.reduce, first);
            acc1.x = reduce_step(acc1.x, m1.x, a.reduce, first);
            acc1.y = reduce_step(acc1.y, m1.y, a.reduce, first);
            acc1.z = reduce_step(acc1.z, m1.z, a.reduce, first);
            acc1.w = reduce_step(acc1.w, m1.w, a.reduce, first);
          }
          ++cnt;
          if (vn != v) {  // wave-uniform
            if (!SUMONLY && a.reduce == NT_MEAN) {
              const float inv = (float)cnt;
              acc0 = make_float4(acc0.x / inv, acc0.y / inv, acc0.z / inv, acc0.w / inv);
              acc1 = make_float4(acc1.x / inv, acc1.y / inv, acc1.z / inv, acc1.w / inv);
            }
            if (in0) a.SO4[(int64_t)v * hv + c0] = acc0;
            if (in1) a.SO4[(int64_t)v * hv + c1] = acc1;
            acc0 = z;
            acc1 = z;
            cnt = 0;
          }
        }
      }
    }
  }
}

__device__ __forceinline__ unsigned long long ps_now() {
  unsigned long long t = 0;
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
#endif
  return t;
}

// ------------------------------------------------------------------------------------ kernel
// ABL (timing-only ablation builds, outputs wrong; NT_PS_ABL): 1 = producers idle, 2 = no MFMA,
// 4 = no W loads, 8 = no split VALU (A fragments used raw); 16 = phase stamps (outputs right)
template <int KS, int ACT, int AACT, bool SUMONLY, int ABL = 0>
__global__ void __launch_bounds__(kThreads, 1) update_ps_kernel(Args a) {
  constexpr int CT = (KS + 1) / 2;
  __shared__ __attribute__((aligned(16))) float4 lds[2 * kBufF4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nt = (a.ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  if (nt <= 0) return;  // uniform over the workgroup
  auto tile_of = [&](int i) { return (int)blockIdx.x + i * (int)gridDim.x; };

  if (wave >= 4) {
    // ================================================================ producers
    const int pw = wave - 4;
    if constexpr ((ABL & 1) != 0) {
      __syncthreads();
      for (int i = 0; i < nt; ++i) {
        __syncthreads();
        __syncthreads();
        __syncthreads();
      }
      return;
    }
    constexpr bool D = (ABL & 16) != 0;
    unsigned long long st[4] = {0, 0, 0, 0}, t0 = 0, t1 = 0;
    gather_tile<ACT>(a, gather_rows(a, tile_of(0), pw, lane), lds, pw, lane);
    __syncthreads();  // B0
    for (int i = 0; i < nt; ++i) {
      if constexpr (D) t0 = ps_now();
      const int erow = i + 1 < nt ? gather_rows(a, tile_of(i + 1), pw, lane) : -1;
      if (i > 0)
        finish_tile<AACT, SUMONLY, (ABL & 96)>(a, tile_of(i - 1),
                          reinterpret_cast<const float*>(lds + ((i - 1) & 1) * kBufF4), pw, lane);
      if constexpr (D) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        t1 = ps_now();
        st[0] += t1 - t0;
      }
      __syncthreads();  // B3
      if constexpr (D) {
        t0 = ps_now();
        st[1] += t0 - t1;
      }
      if (i + 1 < nt) gather_tile<ACT>(a, erow, lds + ((i + 1) & 1) * kBufF4, pw, lane);
      if constexpr (D) {
        t1 = ps_now();
        st[2] += t1 - t0;
      }
      __syncthreads();  // B1
      __syncthreads();  // B2
      if constexpr (D) st[3] += ps_now() - t1;
    }
    if constexpr (D) {
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) atomicAdd(&g_ps_stamps[k], st[k]);
        atomicAdd(&g_ps_stamps[9], 1ull);
      }
    }
    finish_tile<AACT, SUMONLY, (ABL & 96)>(a, tile_of(nt - 1),
                      reinterpret_cast<const float*>(lds + ((nt - 1) & 1) * kBufF4), pw, lane);
    return;
  }

  // ================================================================== consumers
  // Per K step (32 deep) and row tile rt ("unit"): 6 NC MFMAs with the split A fragment of this
  // unit, while the next unit's raw fragment is read from LDS and split (VALU hidden under the
  // MFMAs); the whole next step's W fragments are loaded one step ahead (double-buffered).
  const int g = lane >> 4, fr = lane & 15;
  const int nc = (a.nt16 - wave + 3) / 4;  // valid 16-column tiles of this wave
  // W fragments through a buffer descriptor: one voffset VGPR (lane * 16) for every load, the
  // (step, tile, part) offset in an SGPR -- flat loads would need a 64-bit address per load
  const int wbytes = KS * a.nt16 * 3 * 1024;
  const auto wrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)a.Wb, (short)0, wbytes, 0x00020000);
  const int wvoff = lane * 16;
  const int step_bytes = a.nt16 * 3 * 1024;
  __syncthreads();  // B0

  auto run = [&](auto nc_tag) {
    constexpr int NC = decltype(nc_tag)::value;
    unsigned long long cst[5] = {0, 0, 0, 0, 0};
    f32x4 acc[4][CT];
    uint4 bw[NC][3];
    float4 xa[4][2];
    auto load_w = [&](int ks, int j) {
      const int base = __builtin_amdgcn_readfirstlane(ks * step_bytes + wave * 3 * 1024);
#pragma unroll
      for (int p = 0; p < 3; ++p)
        bw[j][p] = __builtin_bit_cast(
            uint4, __builtin_amdgcn_raw_buffer_load_b128(wrsrc, wvoff, base + (4 * j * 3 + p) * 1024, 0));
    };
#pragma unroll
    for (int j = 0; j < NC; ++j) load_w(0, j);
    for (int i = 0; i < nt; ++i) {
      const float4* A = lds + (i & 1) * kBufF4;
#pragma unroll
      for (int rt = 0; rt < 4; ++rt)
#pragma unroll
        for (int j = 0; j < CT; ++j) acc[rt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      auto read_a = [&](int ks) {
        const int p = 8 * ks + 2 * g;
        const bool ok = p < kPieces;  // p even, kPieces even: p + 1 < kPieces too
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int rt = 0; rt < 4; ++rt) {
          const int r = 16 * rt + fr;
          const float4 v0 = A[a_slot(r, ok ? p : 0)], v1 = A[a_slot(r, ok ? p + 1 : 1)];
          xa[rt][0] = ok ? v0 : z;
          xa[rt][1] = ok ? v1 : z;
        }
      };
      // Per 32-deep K step: split this step's A fragments (read from LDS during the previous
      // step), issue the next step's fragment reads, then per column tile j: 24 MFMAs and the
      // next step's 3 W loads of tile j into the freed registers (sched_barriers pin this order;
      // hipcc otherwise sinks the W prefetches next to their use).
      auto step = [&](int ks) {
        bf16x8 af[4][3];
#pragma unroll
        for (int rt = 0; rt < 4; ++rt) {
          if constexpr ((ABL & 8) != 0) {
            af[rt][0] = __builtin_bit_cast(bf16x8, xa[rt][0]);
            af[rt][1] = __builtin_bit_cast(bf16x8, xa[rt][1]);
            af[rt][2] = af[rt][0];
          } else {
            const float x[8] = {xa[rt][0].x, xa[rt][0].y, xa[rt][0].z, xa[rt][0].w,
                                xa[rt][1].x, xa[rt][1].y, xa[rt][1].z, xa[rt][1].w};
            split3(x, af[rt][0], af[rt][1], af[rt][2]);
          }
        }
        const int kn = ks + 1 < KS ? ks + 1 : 0;  // W of step 0 serves the next tile
        __builtin_amdgcn_sched_barrier(0);
        read_a(ks + 1 < KS ? ks + 1 : ks);
#pragma unroll
        for (int j = 0; j < NC; ++j) {
          __builtin_amdgcn_sched_barrier(0);
          const bf16x8 w0 = as_bf16x8(bw[j][0]), w1 = as_bf16x8(bw[j][1]),
                       w2 = as_bf16x8(bw[j][2]);
#pragma unroll
          for (int rt = 0; rt < 4; ++rt) {
            if constexpr ((ABL & 2) != 0) {
              acc[rt][j] += f32x4{(float)w0[0], (float)w1[0], (float)w2[0], (float)af[rt][2][0]};
              continue;
            }
            f32x4 c = acc[rt][j];
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[rt][2], w0, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[rt][1], w1, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[rt][0], w2, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[rt][1], w0, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[rt][0], w1, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[rt][0], w0, c, 0, 0, 0);
            acc[rt][j] = c;
          }
          __builtin_amdgcn_sched_barrier(0);
          if constexpr ((ABL & 4) == 0) load_w(kn, j);
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      constexpr bool D = (ABL & 16) != 0;
      unsigned long long c0 = 0, c1 = 0;
      if constexpr (D) c0 = ps_now();
      read_a(0);
      int ks = 0;
      for (; ks < a.kmid; ++ks) step(ks);
      if constexpr (D) {
        c1 = ps_now();
        cst[0] += c1 - c0;
      }
      __syncthreads();  // B3
      if constexpr (D) {
        c0 = ps_now();
        cst[1] += c0 - c1;
      }
      for (; ks < KS; ++ks) step(ks);
      if constexpr (D) {
        c1 = ps_now();
        cst[2] += c1 - c0;
      }
      __syncthreads();  // B1: every consumer is done with buffer i & 1
      if constexpr (D) {
        c0 = ps_now();
        cst[3] += c0 - c1;
      }
      float* so = reinterpret_cast<float*>(lds + (i & 1) * kBufF4);
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        const int col = 16 * (wave + 4 * j) + fr;
#pragma unroll
        for (int rt = 0; rt < 4; ++rt)
#pragma unroll
          for (int q = 0; q < 4; ++q) so[(16 * rt + 4 * g + q) * kSO + col] = acc[rt][j][q];
      }
      __syncthreads();  // B2
      if constexpr (D) cst[4] += ps_now() - c0;
    }
    if constexpr ((ABL & 16) != 0) {
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 5; ++k) atomicAdd(&g_ps_stamps[4 + k], cst[k]);
        atomicAdd(&g_ps_stamps[10], 1ull);
      }
    }
  };
  if (nc >= CT) {
    run(std::integral_constant<int, CT>{});
  } else if constexpr (CT > 1) {
    run(std::integral_constant<int, CT - 1>{});
  } else {
    // a wave with no column tile still takes part in every barrier
    for (int i = 0; i < nt; ++i) {
      __syncthreads();
      __syncthreads();
      __syncthreads();
    }
  }
}

}  // namespace
namespace {
template <int KS, int ACT, int AACT, bool SUMONLY>
int launch_ps(const Args& a, hipStream_t stream) {
  const int grid = a.ntiles < cu_count() ? a.ntiles : cu_count();
  auto kern = update_ps_kernel<KS, ACT, AACT, SUMONLY>;
  if constexpr (KS == 10 && ACT == NT_ACT_RELU && SUMONLY) {
    const char* ab = getenv("NT_PS_ABL");
    const int m = ab && ab[0] ? atoi(ab) : 0;
    if (m == 1) kern = update_ps_kernel<KS, ACT, AACT, SUMONLY, 1>;
    if (m == 2) kern = update_ps_kernel<KS, ACT, AACT, SUMONLY, 2>;
    if (m == 3) kern = update_ps_kernel<KS, ACT, AACT, SUMONLY, 3>;
    if (m == 4) kern = update_ps_kernel<KS, ACT, AACT, SUMONLY, 4>;
    if (m == 5) kern = update_ps_kernel<KS, ACT, AACT, SUMONLY, 5>;
    if (m == 6) kern = update_ps_kernel<KS, ACT, AACT, SUMONLY, 6>;
    if (m == 8) kern = update_ps_kernel<KS, ACT, AACT, SUMONLY, 8>;
    if (m == 9) kern = update_ps_kernel<KS, ACT, AACT, SUMONLY, 9>;
    if (m == 13) kern = update_ps_kernel<KS, ACT, AACT, SUMONLY, 13>;
    if (m == 16) kern = update_ps_kernel<KS, ACT, AACT, SUMONLY, 16>;
    if (m == 32) kern = update_ps_kernel<KS, ACT, AACT, SUMONLY, 32>;
    if (m == 64) kern = update_ps_kernel<KS, ACT, AACT, SUMONLY, 64>;
    if (m == 96) kern = update_ps_kernel<KS, ACT, AACT, SUMONLY, 96>;
    if (m == 34) kern = update_ps_kernel<KS, ACT, AACT, SUMONLY, 34>;
    if (m == 98) kern = update_ps_kernel<KS, ACT, AACT, SUMONLY, 98>;
  }
  kern<<<grid, kThreads, 0, stream>>>(a);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

template <int ACT, int AACT, bool SUMONLY, int... Ks>
int dispatch_ps(const Args& a, int ks, hipStream_t stream, std::integer_sequence<int, Ks...>) {
  int rc = NT_EUNSUPPORTED;
  bool done = false;
  ((ks == Ks + 1 ? (rc = launch_ps<Ks + 1, ACT, AACT, SUMONLY>(a, stream), done = true) : false), ...);
  if (!done) set_error("nt_dmpnn_update_fused: no kernel for this hidden size");
  return rc;
}

}  // namespace
}  // namespace nt

namespace nt {
// A/B only: the persistent producer/consumer ps kernel (NT_FUSED_KERNEL=ps) or the pk kernel.
int launch_update_ps(const UpdateArgs& u, const int32_t* tile_ptr, int64_t ntiles,
                     const int32_t* perm, const int32_t* dsts, int reduce, int aact, float aalpha,
                     float* S_out) {
  NT_REQUIRE(ps_supported(u.h), NT_EUNSUPPORTED, "fused update needs h % 4 == 0 and h <= 304");
  NT_REQUIRE((u.E * u.h) / 4 < (int64_t(1) << 31) && (u.V * u.h) / 4 < (int64_t(1) << 31),
             NT_EUNSUPPORTED, "fused update: E*h and V*h must stay below 2^33");
  const bool fused = tile_ptr != nullptr;
  NT_REQUIRE(fused == (S_out != nullptr), NT_EINVAL, "S_out must be given exactly with a tile plan");
  NT_REQUIRE(!fused || (perm && dsts), NT_EINVAL, "fused mode needs perm and dst_sorted");
#ifdef NT_DIAG
  // kernel choice (A/B): NT_FUSED_KERNEL = pk (default: K-slice ring of pre-split A) | ps
  const char* fk = getenv("NT_FUSED_KERNEL");
  if (!(fk && fk[0] == 'p' && fk[1] == 's'))
    return launch_update_pk(u, tile_ptr, ntiles, perm, dsts, reduce, aact, aalpha, S_out);
  Args a;
  a.H4 = (const float4*)u.H;
  a.S4 = (const float4*)u.S;
  a.src = u.src;
  a.rev = u.rev;
  a.Wb = (const uint4*)u.Wp;
  a.b4 = (const float4*)u.b;
  a.V = u.V;
  a.E = u.E;
  a.hv = (int)(u.h / 4);
  a.nt16 = (int)((u.h + 15) / 16);
  a.residual = u.residual;
  a.act = u.act;
  a.alpha = u.alpha;
  a.tile_ptr = tile_ptr;
  a.ntiles = fused ? (int)ntiles : (int)((u.E + kRows - 1) / kRows);
  a.perm = perm;
  a.dsts = dsts;
  a.reduce = reduce;
  a.aact = aact;
  a.aalpha = aalpha;
  const int KS = (int)((u.h + 31) / 32);
  const char* km = getenv("NT_PS_KMID");
  a.kmid = km && km[0] ? atoi(km) : (7 * KS + 5) / 10;  // B3 at 70 % of the K loop (measured)
  if (a.kmid < 0) a.kmid = 0;
  if (a.kmid > KS) a.kmid = KS;
  a.O4 = (float4*)u.H_out;
  a.SO4 = (float4*)S_out;
  if (a.ntiles == 0) return NT_OK;
  using Seq = std::make_integer_sequence<int, 10>;  // KS = 1 .. 10
  const bool relu = u.act == NT_ACT_RELU;
  const bool sum = !fused || reduce == NT_SUM;
  if (relu && sum && (!fused || aact == NT_ACT_RELU))
    return dispatch_ps<NT_ACT_RELU, NT_ACT_RELU, true>(a, KS, u.stream, Seq{});
  if (relu && sum && aact == NT_ACT_IDENTITY)
    return dispatch_ps<NT_ACT_RELU, NT_ACT_IDENTITY, true>(a, KS, u.stream, Seq{});
  return dispatch_ps<-1, -1, false>(a, KS, u.stream, Seq{});
#else
  return launch_update_pk(u, tile_ptr, ntiles, perm, dsts, reduce, aact, aalpha, S_out);
#endif
}
}  // namespace nt

// Debug-only (not part of include/notorch_amd.h): read (and optionally reset) the stamp sums of the
// diagnostic ps build (NT_PS_ABL=16).
extern "C" __attribute__((visibility("default"))) int nt_debug_ps_stamps(unsigned long long* out11,
                                                                         int reset) {
  if (hipMemcpyFromSymbol(out11, HIP_SYMBOL(nt::g_ps_stamps), 11 * sizeof(unsigned long long), 0,
                          hipMemcpyDeviceToHost) != hipSuccess)
    return 2;
  if (reset) {
    unsigned long long z[12] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(nt::g_ps_stamps), z, sizeof(z), 0, hipMemcpyHostToDevice) !=
        hipSuccess)
      return 2;
  }
  return 0;
}

// Persistent D-MPNN layer kernel with a K-slice ring ("pk"): same math and outputs as
// update_ps.hip (one layer, optionally fused with the aggregation its output feeds):
//
//   H_out[e] = (residual ? H[e] : 0) + W (S[src[e]] - act(H[rev[e]])) + b        (chemprop.py:36-43,
//                                                                                 residual.py:27-28)
//   S_out[v] = reduce_{e: dst[e] = v} aact(H_out[e])                               (chemprop.py:37-39,
//                                                                                 :86 with identity)
//
// Difference to "ps": the A operand reaches the MFMA waves already split.  Producers (waves 4-7)
// gather one 64-row x 32-k slice at a time, form A = S[src] - act(H[rev]) in fp32, split it into
// the three bf16 parts (once per element; in "ps" every consumer wave re-split the same fragments)
// and write the parts into a ring of kR LDS slots.  Consumers (waves 0-3) read ready-made
// fragments (12 ds_read_b128 per step, next step's read ahead), so their VALU is nearly free for
// the MFMA stream.  Producer and consumers are decoupled through LDS counters (ready / freed per
// slot, stage_ready / stage_free for the [64][304] fp32 staging tile); every spin is bounded
// (g_pk_timeout records a give-up).  The producers finish tile f (H_out rows, fused aggregation)
// just before they produce slice (f + 1) KS + kR - 1, i.e. with up to kR - 1 slices of the next
// tile buffered for the consumers while they do.
//
// LDS: ring kR x 12 KiB (part p, row r, k-group kg at 16-B slot r * 4 + (kg ^ 2 ((r >> 3) & 1)),
// conflict-free for the consumer's fragment reads) + staging 77,824 B + counters.
//
// Diagnostic library only (make DIAG=1), moved out of update_pk.hip (which keeps the shipping fp32
// layer kernel's launchers).
#include <stdlib.h>

#include <atomic>

#include <type_traits>

#include "../common.hpp"
#include "../update.hpp"

namespace nt {
// the ring's give-up word (set when a bounded spin gave up, read by nt_debug_pk_timeouts)
__device__ unsigned int g_pk_timeout;
// NT_PK_DIAG=1: per-wave cycle sums.  Consumers: [0] ready waits, [1] stage_free waits, [2] whole
// loop; producers: [3] freed waits, [4] stage_ready waits, [5] finish, [6] whole loop; [7] consumer
// waves, [8] producer waves.
__device__ unsigned long long g_pkr_stamps[10];
int cu_count();   // update_ps.hip
int xcd_count();  // update_ps.hip
}  // namespace nt

// ------------------------------------------------------------------------------ pk (A/B only)
// The persistent bf16x6 K-slice-ring kernel: superseded by update_fk_kernel, kept in the diagnostic
// library for A/B runs.
namespace nt {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kRows = 64;
constexpr int kPW = 4;                        // producer waves (the last kPW waves)
__host__ __device__ constexpr int threads_for(int cw) { return (cw + kPW) * 64; }
constexpr int kR = 6;                         // ring slots
constexpr int kLCap = 6;                      // slices a producer keeps loading ahead (4 before)
constexpr int kPartB = kRows * 4 * 16;        // one bf16 part of a slice: 4096 B
constexpr int kSliceB = 3 * kPartB;           // 12,288 B
constexpr int kSO = 304;                      // staging row stride (floats)
constexpr int kStageB = kRows * kSO * 4;      // 77,824 B
constexpr int kFlagInts = 16;
constexpr int kEmaps = 8;                     // row -> edge maps of the last 8 tiles (64 ints each)
constexpr int kLdsB = kR * kSliceB + kStageB + 4 * kFlagInts + 4 * 64 * kEmaps;
static_assert(kLdsB <= 160 * 1024, "LDS budget");
// counter words: [0, kR) ready, [kR, 2 kR) freed, 2 kR stage_ready, 2 kR + 1 stage_free
constexpr int kReady = 0, kFreed = kR, kStageReady = 2 * kR, kStageFree = 2 * kR + 1;

__device__ __forceinline__ int pslot(int r, int kg) { return r * 4 + (kg ^ (((r >> 3) & 1) << 1)); }

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
  int T, n;
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
  const int* tile_ptr;
  int ntiles;
  const int* perm;
  const int* dsts;
  int reduce, aact;
  float aalpha;
  float4* O4;
  float4* SO4;
  int prio;  // 1 = producers at s_setprio 1 (default), 2 = consumers, 0 = none (NT_PK_PRIO, DIAG)
  int nxcd;  // XCDs of the device (xcd_count()): blocks b and b + nxcd share an L2
};

// ------------------------------------------------------------------------------ LDS counters
__device__ __forceinline__ int lds_load(const int* p) {
  return __atomic_load_n(p, __ATOMIC_RELAXED);
}

__device__ __forceinline__ unsigned long long pk_now() {
  unsigned long long t = 0;
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
#endif
  return t;
}

// wait until counter >= target; bounded.  A give-up is only counted here (no memory op inside the
// spin: a VMEM op on that path would make hipcc drain vmcnt(0) after every wait) and recorded in
// g_pk_timeout when the wave ends.
template <bool D = false>
__device__ __forceinline__ void wait_ge(const int* p, int target, int& gave_up,
                                        unsigned long long* acc = nullptr) {
  if constexpr (D) {
    const unsigned long long t0 = pk_now();
    wait_ge<false>(p, target, gave_up);
    *acc += pk_now() - t0;
    return;
  }
  if (lds_load(p) >= target) return;
  for (int it = 0; it < (1 << 20); ++it) {  // ~40 ms; a legitimate wait is microseconds
    __builtin_amdgcn_s_sleep(1);
    if (lds_load(p) >= target) return;
  }
  gave_up = 1;
}

// publish this wave's LDS writes: every ds op retired, then one lane bumps the counter
__device__ __forceinline__ void signal(int* p, int lane) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_fetch_add(p, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// ------------------------------------------------------------------------------ producer
// One lane = one (row, k-group) of a slice: row 16 pw + (lane >> 2), k-group lane & 3.
struct RowSrc {
  int soff, qoff;  // float4 offsets of S[src[e]] and H[rev[e]] rows, -1 = none
};

__device__ __forceinline__ int row_edge(const Args& a, int t, int row) {
  const TileRange tr = tile_range(a.tile_ptr, t, a.E);
  if (row >= tr.n) return -1;
  const int pos = tr.T + row;
  return a.perm ? a.perm[pos] : pos;
}

__device__ __forceinline__ RowSrc row_src(const Args& a, int e) {
  RowSrc rs{-1, -1};
  if (e >= 0) {
    // dense mode (nt_dmpnn_dense_matmul): no src -> row e itself, no rev -> nothing subtracted
    const int64_t s = a.src ? a.src[e] : e, q = a.rev ? a.rev[e] : -1;
    rs.soff = (s >= 0 && s < a.V) ? (int)s * a.hv : -1;
    rs.qoff = (q >= 0 && q < a.E) ? (int)q * a.hv : -1;
  }
  return rs;
}

// select by value, field by field: `c ? a : b` on the structs themselves made hipcc take their
// addresses and keep both in scratch memory (a dependent scratch load in front of every gather)
__device__ __forceinline__ RowSrc pick_src(bool c, const RowSrc& x, const RowSrc& y) {
  return RowSrc{c ? x.soff : y.soff, c ? x.qoff : y.qoff};
}

struct SliceRegs {
  float4 s0, s1, q0, q1;
  int p0;  // first piece
  RowSrc rs;
};

__device__ __forceinline__ void load_slice(const Args& a, const RowSrc& rs, int ks, int kg,
                                           SliceRegs& o) {
  const int p0 = 8 * ks + 2 * kg, hv = a.hv;
  const int c0 = p0 < hv ? p0 : 0, c1 = p0 + 1 < hv ? p0 + 1 : 0;
  const int sb = rs.soff >= 0 ? rs.soff : 0, qb = rs.qoff >= 0 ? rs.qoff : 0;
  o.s0 = a.S4[sb + c0];
  o.s1 = a.S4[sb + c1];
  o.q0 = a.H4[qb + c0];
  o.q1 = a.H4[qb + c1];
  o.p0 = p0;
  o.rs = rs;
}

template <int ACT>
__device__ __forceinline__ void write_slice(const Args& a, const SliceRegs& x, char* slot_base,
                                            int row, int kg) {
  const int hv = a.hv;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  const bool in0 = x.p0 < hv, in1 = x.p0 + 1 < hv;
  const bool sok = x.rs.soff >= 0, qok = x.rs.qoff >= 0;
  const float4 a0 = ((sok && in0) ? x.s0 : z) - ((qok && in0) ? act4_t<ACT>(x.q0, a.act, a.alpha) : z);
  const float4 a1 = ((sok && in1) ? x.s1 : z) - ((qok && in1) ? act4_t<ACT>(x.q1, a.act, a.alpha) : z);
  const float v[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  bf16x8 p0, p1, p2;
  split3(v, p0, p1, p2);
  const int off = pslot(row, kg) * 16;
  *reinterpret_cast<bf16x8*>(slot_base + off) = p0;
  *reinterpret_cast<bf16x8*>(slot_base + kPartB + off) = p1;
  *reinterpret_cast<bf16x8*>(slot_base + 2 * kPartB + off) = p2;
}

__device__ __forceinline__ float reduce_step(float acc, float x, int reduce, bool first) {
  if (reduce == NT_MAX) return first ? x : fmaxf(acc, x);
  if (reduce == NT_MIN) return first ? x : fminf(acc, x);
  return acc + x;
}

// Finish tile t from the staging tile (the consumers staged final rows: residual + W A + bias):
// H_out rows and, fused, S_out.  Wave pw owns a node-aligned quarter of the rows; lane l owns
// pieces l and l + 64 of each row.
template <int AACT, bool SUMONLY, bool CWR, int FU = 4>
__device__ __forceinline__ void finish_tile(const Args& a, int t, const float* __restrict__ so,
                                            int pw, int lane) {
  const TileRange tr = tile_range(a.tile_ptr, t, a.E);
  const int hv = a.hv;
  const bool fused = a.SO4 != nullptr;
  // lane = row: edge and node of every row of the tile (n <= 64)
  int ev = 0, vv = -1;
  if (lane < tr.n) {
    ev = a.perm ? a.perm[tr.T + lane] : tr.T + lane;
    if (fused) vv = a.dsts[tr.T + lane];
  }
  int rs, re;
  {
    const int x0 = (pw * tr.n) >> 2, x1 = ((pw + 1) * tr.n) >> 2;
    if (fused) {
      const int vprev = __shfl_up(vv, 1);
      const bool start = lane >= tr.n || lane == 0 || vprev != vv;  // a node's first row (or past n)
      const unsigned long long m0 = __ballot(start && lane >= x0);
      const unsigned long long m1 = __ballot(start && lane >= x1);
      rs = m0 ? (int)__builtin_ctzll(m0) : tr.n;
      re = pw == 3 ? tr.n : (m1 ? (int)__builtin_ctzll(m1) : tr.n);
      rs = rs < tr.n ? rs : tr.n;
      re = re < tr.n ? re : tr.n;
    } else {
      rs = x0;
      re = pw == 3 ? tr.n : x1;
    }
  }
  const int nr = re - rs;
  if (nr <= 0) return;
  const int c0 = lane, c1 = lane + 64;
  const bool in0 = c0 < hv, in1 = c1 < hv;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 acc0 = z, acc1 = z;
  int cnt = 0;
  auto row_vals = [&](int r, float4& o0, float4& o1) {
    const float* srow = so + (rs + r) * kSO;
    o0 = in0 ? *reinterpret_cast<const float4*>(srow + 4 * c0) : z;
    o1 = in1 ? *reinterpret_cast<const float4*>(srow + 4 * c1) : z;
  };
  auto process = [&](int r, const float4& o0, const float4& o1) {
    const int64_t e = __builtin_amdgcn_readlane(ev, rs + r);
    if constexpr (!CWR) {
      if (in0) a.O4[e * hv + c0] = o0;
      if (in1) a.O4[e * hv + c1] = o1;
    }
    if (fused) {
      const int v = __builtin_amdgcn_readlane(vv, rs + r);
      const int vn = r + 1 < nr ? __builtin_amdgcn_readlane(vv, rs + r + 1) : -1;
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
  };
  // rows four at a time: their eight staged-piece LDS reads are in flight together
  int r = 0;
  if constexpr (FU > 1) {
    for (; r + FU <= nr; r += FU) {
      float4 p0[FU], p1[FU];
#pragma unroll
      for (int u = 0; u < FU; ++u) row_vals(r + u, p0[u], p1[u]);
#pragma unroll
      for (int u = 0; u < FU; ++u) process(r + u, p0[u], p1[u]);
    }
  }
  for (; r < nr; ++r) {
    float4 o0, o1;
    row_vals(r, o0, o1);
    process(r, o0, o1);
  }
}

// ------------------------------------------------------------------------------ kernel
// ABL (timing-only builds, outputs wrong; NT_PK_ABL): 1 = producers skip gathers and finishes
// (protocol only), 2 = no W loads, 4 = no residual loads, 8 = no MFMA
// CWR: the consumers store the finished H' rows straight from their accumulators (16-B row pieces)
// and the producers' finish only runs the fused aggregation from the staged tile.
// PF: rows of the next step's A fragments prefetched during the current step (of 4); the other rows
// are read after the step's MFMAs.  PF = 2 frees 24 VGPRs, which removes the scratch spills the
// full prefetch (PF = 4) caused inside the consumers' MFMA loop.
// CW: consumer (MFMA) waves, 4 (one per SIMD) or 8 (two per SIMD: one wave's MFMAs cover its
// partner's ring waits, fragment reads and W / residual load latency; consumer-only time at
// config 2 108 -> 87 us).  PF = 0 and 5 producer slices in flight keep 3 waves per SIMD (168 VGPRs).
template <int KS, int ACT, int AACT, bool SUMONLY, bool D = false, int ABL = 0, bool CWR = false,
          int PF = 0, int CW = 8>
__global__ void __launch_bounds__(threads_for(CW), 1) update_pk_kernel(Args a) {
  unsigned long long st[4] = {0, 0, 0, 0};
  const unsigned long long t_begin = D ? pk_now() : 0;
  int gave_up = 0;
  auto report = [&]() {
    if (gave_up && (threadIdx.x & 63) == 0) atomicOr(&g_pk_timeout, 1u);
  };
  constexpr int CT = (2 * KS + CW - 1) / CW;  // column tiles of the busiest consumer wave
  __shared__ __attribute__((aligned(16))) uint4 smem[kLdsB / 16];
  char* ring = reinterpret_cast<char*>(smem);
  float* stage = reinterpret_cast<float*>(ring + kR * kSliceB);
  int* flags = reinterpret_cast<int*>(ring + kR * kSliceB + kStageB);
  int* emap = flags + kFlagInts;  // [kEmaps][64]: edge of every row of tile i in emap[i % kEmaps]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware tile walk: workgroups are dispatched round-robin over the nxcd XCDs (blocks b and
  // b + nxcd share one), so give each XCD one contiguous 1/nxcd of the tile plan.  Neighbouring
  // tiles share S / H rows (molecules straddle tile cuts), which then stay in that XCD's L2.
  int t0 = (int)blockIdx.x, tstride = (int)gridDim.x, nt;
  const int nx = a.nxcd;
  if (nx > 1 && (int)gridDim.x % nx == 0) {
    const int x = (int)blockIdx.x % nx, chunk = (a.ntiles + nx - 1) / nx;
    const int lo = x * chunk, hi = min(a.ntiles, lo + chunk);
    t0 = lo + (int)blockIdx.x / nx;
    tstride = (int)gridDim.x / nx;
    nt = hi > t0 ? (hi - t0 + tstride - 1) / tstride : 0;
  } else {
    nt = (a.ntiles - t0 + tstride - 1) / tstride;
  }
  if (nt <= 0) return;
  if (tid < kFlagInts) flags[tid] = 0;
  __syncthreads();  // the only barrier: counters zeroed
  auto tile_of = [&](int i) { return t0 + i * tstride; };
  const int G = nt * KS;

  if (a.prio == 1 && wave >= CW) __builtin_amdgcn_s_setprio(1);
  if (a.prio == 2 && wave < CW) __builtin_amdgcn_s_setprio(1);
  if (wave >= CW) {
    // =============================================================== producers
    const int pw = wave - CW;
    const int row = 16 * pw + (lane >> 2), kg = lane & 3;
    // Slice loads run L slices ahead of the LDS writes (a register ring, loop unrolled by L), so
    // each slice's gather latency overlaps L consumer steps.  Slice g + L belongs to the tile of
    // slice g or the next one (L < KS): rs_cur / rs_nxt, rotated when slice g starts a tile.
    constexpr int LC = CW == 8 ? 5 : kLCap;  // 3 waves per SIMD: a 168-VGPR budget
    constexpr int L = KS == 1 ? 1 : (KS - 1 < LC ? KS - 1 : LC);
    int e_cur = row_edge(a, tile_of(0), row);
    int e_nxt = nt > 1 ? row_edge(a, tile_of(1), row) : -1;
    RowSrc rs_cur = row_src(a, e_cur);
    RowSrc rs_nxt = row_src(a, e_nxt);
    SliceRegs q[L];
#pragma unroll
    for (int u = 0; u < L; ++u)
      if (u < G) load_slice(a, pick_src(u / KS == 0, rs_cur, rs_nxt), u % KS, kg, q[u]);
    int fin = 0;  // next tile to finish: before slice (fin + 1) KS + kR - 1 is produced
    auto finish_next = [&]() {
      wait_ge<D>(flags + kStageReady, CW * (fin + 1), gave_up, &st[1]);  // consumers staged tile fin
      const unsigned long long tf = D ? pk_now() : 0;
      if constexpr ((ABL & 1) == 0) {
        if (!CWR || a.SO4 != nullptr) finish_tile<AACT, SUMONLY, CWR>(a, tile_of(fin), stage, pw, lane);
      }
      if constexpr (D) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st[2] += pk_now() - tf;
      }
      signal(flags + kStageFree, lane);
      ++fin;
    };
    for (int g0 = 0; g0 < G; g0 += L) {
#pragma unroll
      for (int u = 0; u < L; ++u) {
        const int g = g0 + u;
        if (g < G) {
          const int i = g / KS, s = g - i * KS;
          if (s == 0 && g > 0) {  // slice g opens tile i: rotate the row sources
            rs_cur = rs_nxt;
            e_cur = e_nxt;
            e_nxt = i + 1 < nt ? row_edge(a, tile_of(i + 1), row) : -1;
          }
          if (s == (KS > 1 ? 1 : 0) && g > 0 && i + 1 < nt) rs_nxt = row_src(a, e_nxt);
          // the consumers read tile i's row -> edge map once slice (i, 0) is published
          if (s == 0 && kg == 0) emap[(i % kEmaps) * 64 + row] = e_cur;
          while (fin < nt && (fin + 1) * KS + (kR - 1) <= g) finish_next();
          const int slot = g % kR;
          wait_ge<D>(flags + kFreed + slot, CW * (g / kR), gave_up, &st[0]);
          write_slice<ACT>(a, q[u], ring + slot * kSliceB, row, kg);
          signal(flags + kReady + slot, lane);
          const int gl = g + L;  // refill this register slot with slice g + L
          if ((ABL & 1) == 0 && gl < G) {
            const int il = gl / KS;
            load_slice(a, pick_src(il == i, rs_cur, rs_nxt), gl - il * KS, kg, q[u]);
          }
        }
      }
    }
    while (fin < nt) finish_next();
    report();
    if constexpr (D) {
      if (lane == 0) {
        atomicAdd(&g_pkr_stamps[3], st[0]);
        atomicAdd(&g_pkr_stamps[4], st[1]);
        atomicAdd(&g_pkr_stamps[5], st[2]);
        atomicAdd(&g_pkr_stamps[6], pk_now() - t_begin);
        atomicAdd(&g_pkr_stamps[8], 1ull);
      }
    }
    return;
  }

  // ================================================================= consumers
  const int g16 = lane >> 4, fr = lane & 15;
  const int nc = (a.nt16 - wave + CW - 1) / CW;
  const int wbytes = KS * a.nt16 * 3 * 1024;
  const auto wrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)a.Wb, (short)0, wbytes, 0x00020000);
  const int wvoff = lane * 16;
  const int step_bytes = a.nt16 * 3 * 1024;

  auto run = [&](auto nc_tag) {
    constexpr int NC = decltype(nc_tag)::value;
    f32x4 acc[4][CT];
    uint4 bw[NC][3];
    bf16x8 af[4][3], an[PF > 0 ? PF : 1][3];
    auto load_w = [&](int ks, int j) {
      const int base = __builtin_amdgcn_readfirstlane(ks * step_bytes + wave * 3 * 1024);
#pragma unroll
      for (int p = 0; p < 3; ++p)
        bw[j][p] = __builtin_bit_cast(
            uint4, __builtin_amdgcn_raw_buffer_load_b128(wrsrc, wvoff, base + (CW * j * 3 + p) * 1024, 0));
    };
    auto read_row = [&](int g, int rt, bf16x8 (&dst)[3]) {
      const char* base = ring + (g % kR) * kSliceB;
      const int off = pslot(16 * rt + fr, g16) * 16;
#pragma unroll
      for (int p = 0; p < 3; ++p) dst[p] = *reinterpret_cast<const bf16x8*>(base + p * kPartB + off);
    };
    auto read_frags = [&](int g, bf16x8 (&dst)[4][3]) {
#pragma unroll
      for (int rt = 0; rt < 4; ++rt) read_row(g, rt, dst[rt]);
    };
    wait_ge(flags + kReady + 0, 4, gave_up);
    read_frags(0, af);
    signal(flags + kFreed + 0, lane);
    for (int i = 0; i < nt; ++i) {
      // The MFMA runs transposed (A operand = W fragment, B operand = edge fragment), so an
      // accumulator holds 4 consecutive output columns of one edge: C/D lane (fr, g16), register q
      // = edge row 16 rt + fr, column 16 (wave + CW j) + 4 g16 + q.  They start at the residual row
      // pieces H[e] (one 16-B load each; rows past the tile read row 0 and are never stored);
      // slice (i, 0) is published, so tile i's row -> edge map is visible.
      const int hh = 4 * a.hv;
      {
        const int* em = emap + (i % kEmaps) * 64;
        const float* Hf = reinterpret_cast<const float*>(a.H4);
#pragma unroll
        for (int rt = 0; rt < 4; ++rt) {
          const int er = em[16 * rt + fr];
          const int64_t e = er >= 0 ? er : 0;
#pragma unroll
          for (int j = 0; j < CT; ++j) {
            int col = 16 * (wave + CW * j) + 4 * g16;
            col = col < hh ? col : 0;
            if constexpr ((ABL & 4) != 0) {
              acc[rt][j] = f32x4{(float)e, 0.f, 0.f, 0.f};
            } else if (a.residual) {
              const float4 hv4 = *reinterpret_cast<const float4*>(Hf + e * hh + col);
              acc[rt][j] = f32x4{hv4.x, hv4.y, hv4.z, hv4.w};
            } else {
              acc[rt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
          }
        }
      }
      // W of step 0 (after the residual loads, so the first step waits for both with one count)
#pragma unroll
      for (int j = 0; j < NC; ++j)
        if constexpr ((ABL & 2) == 0) load_w(0, j);
      auto step = [&](int s) {
        const int g = i * KS + s;
        const bool more = g + 1 < G;
        const int gn = more ? g + 1 : g;  // the last step re-reads its own slice (no branch)
        wait_ge<D>(flags + kReady + gn % kR, more ? 4 * (gn / kR + 1) : 0, gave_up, &st[0]);
#pragma unroll
        for (int rt = 0; rt < PF; ++rt) read_row(gn, rt, an[rt]);
        const bool reload = s + 1 < KS;  // the next tile's step-0 W is loaded at its start
#pragma unroll
        for (int j = 0; j < NC; ++j) {
          __builtin_amdgcn_sched_barrier(0);
          const bf16x8 w0 = as_bf16x8(bw[j][0]), w1 = as_bf16x8(bw[j][1]), w2 = as_bf16x8(bw[j][2]);
#pragma unroll
          for (int rt = 0; rt < 4; ++rt) {
            if constexpr ((ABL & 8) != 0) {
              acc[rt][j] += f32x4{(float)af[rt][2][0], (float)w0[0], (float)w1[0], (float)w2[0]};
              continue;
            }
            f32x4 c = acc[rt][j];
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, af[rt][2], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, af[rt][1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2, af[rt][0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, af[rt][1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, af[rt][0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, af[rt][0], c, 0, 0, 0);
            acc[rt][j] = c;
          }
          __builtin_amdgcn_sched_barrier(0);
          if constexpr ((ABL & 2) == 0) {
            if (reload) load_w(s + 1, j);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int rt = PF; rt < 4; ++rt) read_row(gn, rt, af[rt]);  // late rows: af[rt] is free now
        if (more) signal(flags + kFreed + (g + 1) % kR, lane);       // (waits for those reads)
#pragma unroll
        for (int rt = 0; rt < PF; ++rt)
#pragma unroll
          for (int p = 0; p < 3; ++p) af[rt][p] = an[rt][p];
      };
      step(0);  // peeled: its waits cover the residual loads; the loop's waits only the W ring
      for (int s = 1; s < KS; ++s) step(s);
      // stage the tile for the producers (after they finished reading the previous one)
      if (i > 0) wait_ge<D>(flags + kStageFree, 4 * i, gave_up, &st[1]);
      {
        const float* bf = reinterpret_cast<const float*>(a.b4);
        const int* em = emap + (i % kEmaps) * 64;
        float* Of = reinterpret_cast<float*>(a.O4);
        const bool stage_it = !CWR || a.SO4 != nullptr;
#pragma unroll
        for (int j = 0; j < NC; ++j) {
          const int col = 16 * (wave + CW * j) + 4 * g16;
          const float4 bj = (bf && col < hh) ? *reinterpret_cast<const float4*>(bf + col)
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int rt = 0; rt < 4; ++rt) {
            const float4 o = make_float4(acc[rt][j][0] + bj.x, acc[rt][j][1] + bj.y,
                                         acc[rt][j][2] + bj.z, acc[rt][j][3] + bj.w);
            if (stage_it) *reinterpret_cast<float4*>(stage + (16 * rt + fr) * kSO + col) = o;
            if constexpr (CWR) {
              const int er = em[16 * rt + fr];  // re-read from LDS: no registers held across the tile
              if (er >= 0 && col < hh) *reinterpret_cast<float4*>(Of + (int64_t)er * hh + col) = o;
            }
          }
        }
      }
      signal(flags + kStageReady, lane);
    }
    report();
    if constexpr (D) {
      if (lane == 0) {
        atomicAdd(&g_pkr_stamps[0], st[0]);
        atomicAdd(&g_pkr_stamps[1], st[1]);
        atomicAdd(&g_pkr_stamps[2], pk_now() - t_begin);
        atomicAdd(&g_pkr_stamps[7], 1ull);
      }
    }
  };
  if (nc >= CT) {
    run(std::integral_constant<int, CT>{});
  } else if constexpr (CT > 1) {
    run(std::integral_constant<int, CT - 1>{});
  } else {
    // a wave with no column tile still releases every slot and stages (nothing) every tile
    for (int g = 0; g < G; ++g) {
      wait_ge(flags + kReady + g % kR, 4 * (g / kR + 1), gave_up);
      signal(flags + kFreed + g % kR, lane);
      if (g % KS == KS - 1) {
        const int i = g / KS;
        if (i > 0) wait_ge(flags + kStageFree, 4 * i, gave_up);
        signal(flags + kStageReady, lane);
      }
    }
    report();
  }
}

template <int KS, int ACT, int AACT, bool SUMONLY>
int launch_pk(const Args& a, int grid, hipStream_t stream) {
  auto kern = update_pk_kernel<KS, ACT, AACT, SUMONLY>;
  int threads = threads_for(8);
#ifdef NT_DIAG
  // NT_PK_NCW=4: one consumer wave per SIMD (the round-1 layout), for A/B
  const char* ncw = getenv("NT_PK_NCW");
  if (ncw && ncw[0] == '4') {
    kern = update_pk_kernel<KS, ACT, AACT, SUMONLY, false, 0, false, 2, 4>;
    threads = threads_for(4);
  }
  // A/B builds (make DIAG=1): NT_PK_CW=1 consumers store H' (measured slower at config 2: 157 vs
  // 143 us), NT_PK_PF=4 the full next-step prefetch, NT_PK_DIAG=1 stamps, NT_PK_ABL=m ablations
  // (timing only: outputs are wrong)
  const char* cw = getenv("NT_PK_CW");
  if (cw && cw[0] == '1') kern = update_pk_kernel<KS, ACT, AACT, SUMONLY, false, 0, true>;
  const char* pf = getenv("NT_PK_PF");
  if (pf && pf[0] == '4') kern = update_pk_kernel<KS, ACT, AACT, SUMONLY, false, 0, false, 4>;
  if constexpr (KS == 10 && ACT == NT_ACT_RELU && SUMONLY) {
    const char* d = getenv("NT_PK_DIAG");
    if (d && d[0] == '1') kern = update_pk_kernel<KS, ACT, AACT, SUMONLY, true>;
    const char* ab = getenv("NT_PK_ABL");
    const int m = ab && ab[0] ? atoi(ab) : 0;
    if (m == 1) kern = update_pk_kernel<KS, ACT, AACT, SUMONLY, false, 1>;
    if (m == 3) kern = update_pk_kernel<KS, ACT, AACT, SUMONLY, false, 3>;
    if (m == 5) kern = update_pk_kernel<KS, ACT, AACT, SUMONLY, false, 5>;
    if (m == 7) kern = update_pk_kernel<KS, ACT, AACT, SUMONLY, false, 7>;
    if (m == 9) kern = update_pk_kernel<KS, ACT, AACT, SUMONLY, false, 9>;
    if (m == 15) kern = update_pk_kernel<KS, ACT, AACT, SUMONLY, false, 15>;
  }
#endif
  kern<<<grid, threads, 0, stream>>>(a);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

template <int ACT, int AACT, bool SUMONLY, int... Ks>
int dispatch_pk(const Args& a, int ks, int grid, hipStream_t stream,
                std::integer_sequence<int, Ks...>) {
  int rc = NT_EUNSUPPORTED;
  bool done = false;
  ((ks == Ks + 1 ? (rc = launch_pk<Ks + 1, ACT, AACT, SUMONLY>(a, grid, stream), done = true) : false),
   ...);
  if (!done) set_error("nt_dmpnn_update_fused: no pk kernel for this hidden size");
  return rc;
}

}  // namespace

int launch_update_pk(const UpdateArgs& u, const int32_t* tile_ptr, int64_t ntiles,
                     const int32_t* perm, const int32_t* dsts, int reduce, int aact, float aalpha,
                     float* S_out) {
  const bool fused = tile_ptr != nullptr;
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
  a.O4 = (float4*)u.H_out;
  a.SO4 = (float4*)S_out;
  a.nxcd = xcd_count();
  // producers at s_setprio 1: with two consumer waves per SIMD the producers bound the kernel, and
  // winning issue arbitration takes 4 % off a launch (133.7 -> 128.6 us at config 2; consumer
  // priority: 134.6)
  a.prio = 1;
#ifdef NT_DIAG
  {
    const char* pr = getenv("NT_PK_PRIO");
    if (pr && pr[0]) a.prio = atoi(pr);
  }
#endif
  if (a.ntiles == 0) return NT_OK;
  const int grid = a.ntiles < cu_count() ? a.ntiles : cu_count();
  const int KS = (int)((u.h + 31) / 32);
  using Seq = std::make_integer_sequence<int, 10>;
  const bool relu = u.act == NT_ACT_RELU;
  const bool sum = !fused || reduce == NT_SUM;
  if (relu && sum && (!fused || aact == NT_ACT_RELU))
    return dispatch_pk<NT_ACT_RELU, NT_ACT_RELU, true>(a, KS, grid, u.stream, Seq{});
  if (relu && sum && aact == NT_ACT_IDENTITY)
    return dispatch_pk<NT_ACT_RELU, NT_ACT_IDENTITY, true>(a, KS, grid, u.stream, Seq{});
  if (u.act == NT_ACT_IDENTITY && !fused)  // dense mode (the backward's dA) and identity layers
    return dispatch_pk<NT_ACT_IDENTITY, NT_ACT_IDENTITY, true>(a, KS, grid, u.stream, Seq{});
  return dispatch_pk<-1, -1, false>(a, KS, grid, u.stream, Seq{});
}
}  // namespace nt

// Debug-only (diagnostic library, not part of include/notorch_amd.h): bounded-spin give-ups of the pk
// kernel.
extern "C" __attribute__((visibility("default"))) int nt_debug_pk_timeouts(unsigned* out,
                                                                           int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(nt::g_pk_timeout), sizeof(unsigned), 0,
                          hipMemcpyDeviceToHost) != hipSuccess)
    return 2;
  if (reset) {  // 1: clear; 2: set (tests of the wrapper's status check)
    unsigned z = reset == 2 ? 1u : 0u;
    if (hipMemcpyToSymbol(HIP_SYMBOL(nt::g_pk_timeout), &z, sizeof(z), 0, hipMemcpyHostToDevice) !=
        hipSuccess)
      return 2;
  }
  return 0;
}

extern "C" __attribute__((visibility("default"))) int nt_debug_pkr_stamps(unsigned long long* out9,
                                                                         int reset) {
  if (hipMemcpyFromSymbol(out9, HIP_SYMBOL(nt::g_pkr_stamps), 9 * sizeof(unsigned long long), 0,
                          hipMemcpyDeviceToHost) != hipSuccess)
    return 2;
  if (reset) {
    unsigned long long z[10] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(nt::g_pkr_stamps), z, sizeof(z), 0, hipMemcpyHostToDevice) !=
        hipSuccess)
      return 2;
  }
  return 0;
}

// fp32 D-MPNN layer kernel, two-part fp16 split on fp16 MFMA, with the output tile staged in LDS and
// written back while the NEXT tile's K loop runs ("fk2").  Included by update_pk.hip after
// update_fk.hpp (it reuses that kernel's per-thread state, gathers, W loads and MFMA step).
//
//   H_out[e] = (residual ? H[e] : 0) + W (S[src[e]] - act(H[rev[e]])) + b        (chemprop.py:36-43,
//                                                                                 residual.py:27-28)
//   S_out[v] = reduce_{e: dst[e] = v} aact(H_out[e])                               (chemprop.py:37-39)
//
// Why a second kernel: in update_fk_kernel every CU ends a tile with a burst of H_out / S_out stores
// (231 KB per 128-row tile) and the next tile's first waits (vmcnt counts loads and stores in issue
// order) sit behind that burst; with all CUs bursting at once the store drain, not the K loop, set the
// time (no-store ablation 43 us vs 131 us at config 2).  Here the epilogue only writes acc / s + b
// into an LDS stage (64 rows x h fp32, <= 97 KiB); during the next tile's KS k-steps the workgroup
// finishes the staged tile node by node, one batch of nodes per k-step, between the split and the
// barrier: for each (node, 16-B column piece) item, over the node's rows in ascending order,
//   x = stage[row] + H[e] (residual rows prefetched one step ahead) -> H_out[e],
//   S_out[v] = reduce of aact(x) in the same left-to-right order as CPU scatter_add_ (same bits).
// The stores of one tile are spread over the next tile's K loop (about 12 KB per k-step per CU),
// interleaved with its gathers instead of piling up in front of them.
//
// Gathers: thread t stages row t / 8 of the tile, 16-B piece t % 8 of the k-step: each wave-load covers
// 8 rows x one 128-B row segment (a 32-deep fp32 k-slice), the split scatters the fp16 parts into
// the MFMA B-fragment slots.
//
// Tiles: 64 rows (4 row tiles), node-aligned (nt_dmpnn_tile_plan with 64-row capacity), 8 waves x 3
// column tiles (h <= 384, one chunk).  Numerics as update_fk_kernel, except that the residual enters
// after the K loop (x = (acc / (s_A s_W) + b) + H[e]) instead of in the accumulator.
#pragma once

#include "../update_fk.hpp"

namespace nt {
namespace fk {

constexpr int kStageV = 97;  // float4 per staged row: odd row stride >= hv (h <= 384)
constexpr int kFk2MaxH = 384;
constexpr int kNodeInfo = 68;  // ints per tile: [0] node count, [1 + k] first row of node k, then n
constexpr int kPre = 3;        // residual rows prefetched per item (nodes with more rows load the rest inline)

template <int CT, int GD>
struct State2 : State<4, CT, GD> {
  f32x4 rres[kPre];  // residual pieces of the thread's first item of the next batch
  int it_e[kPre];    // ... its rows' edges (first kPre rows), node, float4 column, first row, row count
  int it_v, it_p, it_r0, it_n;
  f32x4* stage;      // 64 x hsv float4
  f32x4* sbias;      // bias (zeros without one), hv float4
  int* ninfo;        // kEmaps x kNodeInfo
  int hsv, tid, KS;
  float rhv;
};

// item q of a batch -> (node within the batch, float4 column); q < 1024, hv <= 96
__device__ __forceinline__ void fk2_item(int q, int hv, float rhv, int& k, int& p) {
  int t = (int)((float)q * rhv);
  t = t * hv > q ? t - 1 : ((t + 1) * hv <= q ? t + 1 : t);
  k = t;
  p = q - t * hv;
}

// nodes [k0, k0 + cnt) of batch b of a tile's node list
__device__ __forceinline__ void fk2_batch(const int* ni, int KS, int b, int& k0, int& cnt) {
  const int nn = ni[0];
  const int nb = (nn + KS - 1) / KS;
  k0 = b * nb;
  const int c = nn - k0;
  cnt = c < 0 ? 0 : (c < nb ? c : nb);
}

// node list of the tile in an emap slot (one wave; the emap entries were written before a barrier):
// first rows of its nodes in ascending order, then the tile's row count
__device__ __forceinline__ void fk2_node_list(const int4* emap, int* ni, int lane) {
  const int4 ri = emap[lane];
  const bool valid = ri.x >= 0;
  const bool start = valid && (ri.z & kFlagStart);
  const unsigned long long vm = __ballot(valid);
  const unsigned long long sm = __ballot(start);
  const int nn = __popcll(sm);
  if (start) ni[1 + __popcll(sm & ((1ull << lane) - 1ull))] = lane;
  if (lane == 0) {
    ni[0] = nn;
    ni[1 + nn] = __popcll(vm);
  }
}

// the thread's first item of batch b of the staged tile (slot x, nn nodes): its rows' edges, node,
// column and residual pieces (unconditional loads: rows past the node read S's first row)
template <int CT, int GD>
__device__ __forceinline__ void fk2_prefetch(State2<CT, GD>& st, const Args& a, bool resid, int x, int nn, int b) {
  const int* ni = st.ninfo + x * kNodeInfo;
  const int4* em = st.emap + x * 64;
  const int nb = (nn + st.KS - 1) / st.KS, k0 = b * nb;
  const int cnt = nn - k0 < 0 ? 0 : (nn - k0 < nb ? nn - k0 : nb);
  const bool ok = st.tid < cnt * st.hv;
  int k, p;
  fk2_item(ok ? st.tid : 0, st.hv, st.rhv, k, p);
  const int kk = ok ? k0 + k : 0;
  const int r0 = ok ? ni[1 + kk] : 0, r1 = ok ? ni[2 + kk] : 0;
  const f32x4* R4 = reinterpret_cast<const f32x4*>(resid ? a.H : a.S);
#pragma unroll
  for (int u = 0; u < kPre; ++u) {
    const int r = r0 + u < 64 ? r0 + u : 63;
    const int4 ri = em[r];
    if (u == 0) st.it_v = ri.y;
    st.it_e[u] = ri.x;
    const int64_t off = (resid && r0 + u < r1 && ri.x >= 0) ? (int64_t)ri.x * st.hv + p : 0;
    st.rres[u] = R4[off];
  }
  st.it_p = p;
  st.it_r0 = r0;
  st.it_n = r1 - r0;  // 0: no item
}

// one row of an item: x = stage + residual -> H_out, folded into the node's reduction
template <int AACT, bool SUMONLY, bool FUSED, bool STORE>
__device__ __forceinline__ void fk2_row(const Args& a, const f32x4& sx, const f32x4& rv, bool resid, int e, int hv,
                                        int p, bool first, f32x4& acc, float& cnt, float& mxH) {
  f32x4 x = sx;
  if (resid) x = x + rv;
  if constexpr (STORE) reinterpret_cast<f32x4*>(a.O)[(int64_t)e * hv + p] = x;
  mxH = fmaxf(mxH, fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])), fmaxf(fabsf(x[2]), fabsf(x[3]))));
  if constexpr (FUSED) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float v = act_t<AACT>(x[c], a.aact, a.aalpha);
      float y;
      if constexpr (SUMONLY) y = acc[c] + v;
      else y = a.reduce == NT_MAX ? fmaxf(acc[c], v) : (a.reduce == NT_MIN ? fminf(acc[c], v) : acc[c] + v);
      acc[c] = first ? v : y;
    }
    cnt = first ? 1.f : cnt + 1.f;
  }
}

// batch b of the staged tile (slot x, nn nodes): H_out of its nodes' rows, S_out of its nodes.  The
// thread's first item comes from the prefetch; a second one (batches of more than 512 items) is
// looked up here
template <int AACT, bool SUMONLY, bool FUSED, bool STORE = true, int CT, int GD>
__device__ __forceinline__ void fk2_trickle(State2<CT, GD>& st, const Args& a, bool resid, int x, int nn, int b) {
  const int4* em = st.emap + x * 64;
  const f32x4* H4 = reinterpret_cast<const f32x4*>(a.H);
  const f32x4 z4 = f32x4{0.f, 0.f, 0.f, 0.f};
  if (st.it_n > 0) {
    const int p = st.it_p, r0 = st.it_r0, n = st.it_n;
    f32x4 acc = z4;
    float c = 0.f;
    f32x4 sx[kPre];
#pragma unroll
    for (int u = 0; u < kPre; ++u) sx[u] = st.stage[(u < n ? r0 + u : r0) * st.hsv + p];
#pragma unroll
    for (int u = 0; u < kPre; ++u)
      if (u < n) fk2_row<AACT, SUMONLY, FUSED, STORE>(a, sx[u], st.rres[u], resid, st.it_e[u], st.hv, p, u == 0, acc, c, st.mxH);
    for (int r = r0 + kPre; r < r0 + n; ++r) {  // rows past the prefetched ones (in-degree > kPre)
      const int er = em[r].x;
      const f32x4 rv = resid ? H4[(int64_t)er * st.hv + p] : z4;
      fk2_row<AACT, SUMONLY, FUSED, STORE>(a, st.stage[r * st.hsv + p], rv, resid, er, st.hv, p, false, acc, c, st.mxH);
    }
    if constexpr (FUSED) {
      if (!SUMONLY && a.reduce == NT_MEAN) acc = acc / c;
      if constexpr (STORE) reinterpret_cast<f32x4*>(a.SO)[(int64_t)st.it_v * st.hv + p] = acc;
      st.mxS = fmaxf(st.mxS, fmaxf(fmaxf(fabsf(acc[0]), fabsf(acc[1])), fmaxf(fabsf(acc[2]), fabsf(acc[3]))));
    }
  }
  // second item (q = tid + 512)
  const int nb = (nn + st.KS - 1) / st.KS, k0 = b * nb;
  const int cnt = nn - k0 < 0 ? 0 : (nn - k0 < nb ? nn - k0 : nb);
  const int q = st.tid + 512;
  if (q < cnt * st.hv) {
    const int* ni = st.ninfo + x * kNodeInfo;
    int k, p;
    fk2_item(q, st.hv, st.rhv, k, p);
    const int r0 = ni[1 + k0 + k], r1 = ni[2 + k0 + k];
    f32x4 acc = z4;
    float c = 0.f;
    for (int r = r0; r < r1; ++r) {
      const int er = em[r].x;
      const f32x4 rv = resid ? H4[(int64_t)er * st.hv + p] : z4;
      fk2_row<AACT, SUMONLY, FUSED, STORE>(a, st.stage[r * st.hsv + p], rv, resid, er, st.hv, p, r == r0, acc, c,
                                           st.mxH);
    }
    if constexpr (FUSED) {
      if (!SUMONLY && a.reduce == NT_MEAN) acc = acc / c;
      if constexpr (STORE) reinterpret_cast<f32x4*>(a.SO)[(int64_t)em[r0].y * st.hv + p] = acc;
      st.mxS = fmaxf(st.mxS, fmaxf(fmaxf(fabsf(acc[0]), fabsf(acc[1])), fmaxf(fabsf(acc[2]), fabsf(acc[3]))));
    }
  }
}

// A = S[src] - act(H[rev]) of the thread's staged piece (row t / 8, piece t % 8 of the k-step), scaled
// by s_A, split into two fp16 parts written to their MFMA B-fragment slots of LDS buffer BUF
template <int CT, int ACT, int P, int BUF, int GD>
__device__ __forceinline__ void fk2_split(State2<CT, GD>& st, const Args& a, int s) {
  constexpr int kBufB = State<4, CT, GD>::kBufB, kPartB = State<4, CT, GD>::kPartB;
  const bool sok = st.gso[P] >= 0, qok = st.gqo[P] >= 0;
  const bool in = 8 * s + st.kp0 < st.hv;
  const f32x4 sv = st.gs[P][0];
  const f32x4 qv = st.gq[P][0];
  f16x4 h0, h1;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float q = act_t<ACT>(qv[c], a.act, a.alpha);
    const float x = ((sok && in ? sv[c] : 0.f) - (qok && in ? q : 0.f)) * st.sA;
    const _Float16 t0 = (_Float16)x;
    h0[c] = t0;
    h1[c] = (_Float16)(x - (float)t0);
  }
  // row tile grow / 16, fragment lane (grow % 16) + 16 (piece / 2), half piece % 2
  char* base = st.abuf + BUF * kBufB + (st.grow >> 4) * 1024 + ((st.grow & 15) + 16 * (st.kp0 >> 1)) * 16 +
               8 * (st.kp0 & 1);
  *reinterpret_cast<f16x4*>(base) = h0;
  *reinterpret_cast<f16x4*>(base + kPartB) = h1;
}

// epilogue of the K loop: stage = acc / (s_A s_W) + b (rows past the tile are staged and never read);
// the accumulators restart at zero
template <int J, int RTI, int CT, int GD>
__device__ __forceinline__ void fk2_stage_one(State2<CT, GD>& st) {
  const int ct = st.wave + 8 * J;
  const int pc = 4 * ct + st.g16;
  if (ct < st.NT && pc < st.hv) {
    const f32x4 bj = st.sbias[pc];
    f32x4 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = fmaf(st.acc[RTI][J][q], st.inv, bj[q]);
    st.stage[(16 * RTI + st.fr) * st.hsv + pc] = o;
  }
  st.acc[RTI][J] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (RTI + 1 < 4) fk2_stage_one<J, RTI + 1, CT, GD>(st);
  else if constexpr (J + 1 < CT) fk2_stage_one<J + 1, 0, CT, GD>(st);
}

// ABL (diagnostic builds only, 0 in the shipping library): timing ablations, results invalid --
// 1 gathers read row 0, 2 no MFMA, 4 no split, 8 no trickle stores, 16 no residual prefetch,
// 32 no W loads, 64 no trickle at all, 128 per-phase cycle stamps summed into g_pk_stamps
// ([0] W + gather issue, [1] MFMA, [2] split, [3] trickle + prefetch, [4] barrier, [5] tile end,
// [6] whole loop, [7] waves).
// TABLE: fused (rows from the row table, S_out) or plain / dense (fixed 64-row tiles in edge order)
template <int CT, int ACT, int AACT, bool SUMONLY, bool TABLE, int GD = 2, int ABL = 0>
__global__ void __launch_bounds__(kThreads, 2) update_fk2_kernel(Args a) {
  using St = State2<CT, GD>;
  constexpr int RT = 4;
  constexpr int ROWS = 64;
  constexpr int kBufB = State<RT, CT, GD>::kBufB;
  constexpr int kEmapB = kEmaps * ROWS * 16;
  constexpr int kStageB = ROWS * kStageV * 16;
  constexpr int kBiasB = kStageV * 16;
  constexpr int kInfoB = kEmaps * kNodeInfo * 4;
  __shared__ __attribute__((aligned(16))) uint4 smem[(2 * kBufB + kEmapB + kStageB + kBiasB + kInfoB) / 16];

  // XCD-aware persistent walk (as update_fk_kernel)
  int t0 = (int)blockIdx.x, tstride = (int)gridDim.x, ntl;
  const int nx = a.nxcd;
  if (nx > 1 && (int)gridDim.x % nx == 0) {
    const int x = (int)blockIdx.x % nx, chunk = (a.ntiles + nx - 1) / nx;
    const int lo = x * chunk, hi = min(a.ntiles, lo + chunk);
    t0 = lo + (int)blockIdx.x / nx;
    tstride = (int)gridDim.x / nx;
    ntl = hi > t0 ? (hi - t0 + tstride - 1) / tstride : 0;
  } else {
    ntl = (a.ntiles - t0 + tstride - 1) / tstride;
  }
  if (ntl <= 0) return;
  auto tile = [&](int i) __attribute__((always_inline)) { return t0 + (i < ntl ? i : ntl - 1) * tstride; };

  St st;
  const int tid = threadIdx.x;
  st.tid = tid;
  st.lane = tid & 63;
  st.wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  st.fr = st.lane & 15;
  st.g16 = st.lane >> 4;
  st.grow = tid >> 3;  // gather row of the thread (8 threads per row)
  st.grt = st.grow >> 4;
  st.kp0 = tid & 7;    // its 16-B piece of the 32-deep k-step
  st.hv = a.hv;
  st.hc = a.hv;
  st.NT = a.NT;
  st.CTC = 8 * CT;
  st.KS = a.KS;
  st.abuf = reinterpret_cast<char*>(smem);
  st.emap = reinterpret_cast<int4*>(st.abuf + 2 * kBufB);
  st.stage = reinterpret_cast<f32x4*>(st.abuf + 2 * kBufB + kEmapB);
  st.sbias = reinterpret_cast<f32x4*>(st.abuf + 2 * kBufB + kEmapB + kStageB);
  st.ninfo = reinterpret_cast<int*>(st.abuf + 2 * kBufB + kEmapB + kStageB + kBiasB);
  st.hsv = a.hv | 1;
  st.rhv = 1.f / (float)a.hv;
  st.wrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)a.Wimg, (short)0, (int)image_bytes(a.h), 0x00020000);
  st.mxH = 0.f;
  st.mxS = 0.f;
  const float bound = a.src ? a.amax_in[1] + (a.rev ? act_bound(a.amax_in[0], a.act, a.alpha) : 0.f)
                            : a.amax_in[1];
  st.sA = ldexpf(1.f, scale_exp(bound));
  const float sW = *reinterpret_cast<const float*>(a.Wimg);
  st.sAW = st.sA * sW;
  st.inv = 1.f / st.sAW;  // exact: a power of two
  const bool resid = a.residual && a.H != nullptr;
  const bool info_writer = st.kp0 == 0;
  const int KS = a.KS;
  const int G = ntl * KS;

  // ---- tile info: cur (tile i) and nxt (i + 1) row offsets, raw row of tile i + 2 in flight
  int2 cur, nxt;
  int n_cur, n_nxt;
  int4 raw2;
  TileHead h2, h3;
  {
    const TileHead h0 = tile_head<RT, TABLE>(a, tile(0));
    const int4 r0 = row_raw<RT, TABLE>(a, h0, st.grow);
    const TileHead h1 = tile_head<RT, TABLE>(a, tile(1));
    const int4 r1 = row_raw<RT, TABLE>(a, h1, st.grow);
    h2 = tile_head<RT, TABLE>(a, tile(2));
    raw2 = row_raw<RT, TABLE>(a, h2, st.grow);
    h3 = tile_head<RT, TABLE>(a, tile(3));
    const bool v0 = st.grow < h0.n, v1 = st.grow < h1.n;
    cur = row_offsets(a, r0, v0);
    nxt = row_offsets(a, r1, v1);
    if (info_writer) {
      st.emap[0 * ROWS + st.grow] = row_entry(r0, v0);
      st.emap[1 * ROWS + st.grow] = row_entry(r1, v1);
    }
    n_cur = h0.n < ROWS ? h0.n : ROWS;
    n_nxt = h1.n < ROWS ? h1.n : ROWS;
  }
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int j = 0; j < CT; ++j) st.acc[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (tid < a.hv) st.sbias[tid] = a.bias ? reinterpret_cast<const f32x4*>(a.bias)[tid] : f32x4{0.f, 0.f, 0.f, 0.f};
  // node lists: slot 3's stays empty until a tile is announced into it, and stands for "no staged
  // tile yet" during tile 0
  if (tid < kEmaps) st.ninfo[tid * kNodeInfo] = 0;
#pragma unroll
  for (int u = 0; u < kPre; ++u) {
    st.rres[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    st.it_e[u] = 0;
  }
  st.it_v = st.it_p = st.it_r0 = st.it_n = 0;
  int x_prv = kEmaps - 1, nn_prv = 0;  // staged tile: emap slot, node count

  // ---- prologue: node lists of tiles 0 and 1, steps 0 and 1 staged, W of step 0, slice 0 split
  __syncthreads();  // emap of tiles 0 and 1
  if (st.wave == 0) {
    fk2_node_list(st.emap, st.ninfo, st.lane);
    fk2_node_list(st.emap + ROWS, st.ninfo + kNodeInfo, st.lane);
  }
  fk_gather<RT, CT, ACT, 0>(st, a, cur.x, cur.y, 0);
  if constexpr (GD == 2) fk_gather<RT, CT, ACT, 1>(st, a, cur.x, cur.y, 1);  // KS >= 2
  fk_load_w<RT, CT, 0>(st, 0, 0);
  fk2_split<CT, ACT, 0, 0>(st, a, 0);
  fk_barrier();

  // ---- main loop: one 32-deep k-step per iteration, two iterations per trip (register parity)
  constexpr bool STAMP = (ABL & 128) != 0;
  unsigned long long tacc[6] = {0, 0, 0, 0, 0, 0}, tp = 0, tb = 0;
  if constexpr (STAMP) tb = tp = __builtin_amdgcn_s_memtime();
  auto stamp = [&](int slot) __attribute__((always_inline)) {
    if constexpr (STAMP) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      tacc[slot] += t - tp;
      tp = t;
    }
  };
  int g = 0, i = 0, k = 0;
  while (g < G) {
#pragma unroll
    for (int P = 0; P < 2; ++P) {
      if (P == 0 || g < G) {
        const int s = k;
        // (1) W fragments of step g + 1
        const int s1 = k + 1 < KS ? k + 1 : 0;
        if constexpr ((ABL & 32) == 0) {
          if (P == 0) fk_load_w<RT, CT, 1>(st, 0, s1);
          else fk_load_w<RT, CT, 0>(st, 0, s1);
        }
        // (2) stage step g + GD (tile i or i + 1)
        {
          const int k2 = k + GD;
          const int adv = k2 >= KS ? 1 : 0;
          const int s2 = k2 - adv * KS;
          int so = adv == 0 ? cur.x : nxt.x, qo = adv == 0 ? cur.y : nxt.y;
          if constexpr ((ABL & 1) != 0) so = qo = 0;
          if (GD == 1 || P == 0) fk_gather<RT, CT, ACT, 0>(st, a, so, qo, s2);
          else fk_gather<RT, CT, ACT, GD - 1>(st, a, so, qo, s2);
        }
        stamp(0);
        // (3) MFMAs of step g
        if constexpr ((ABL & 2) == 0) {
          if (P == 0) fk_mfma<RT, CT, 0>(st, 0, (n_cur + 15) >> 4);
          else fk_mfma<RT, CT, 1>(st, 0, (n_cur + 15) >> 4);
        }
        stamp(1);
        // (4) split step g + 1's staged piece into the other buffer
        if constexpr ((ABL & 4) == 0) {
          if (P == 0) fk2_split<CT, ACT, GD - 1, 1>(st, a, s1);
          else fk2_split<CT, ACT, 0, 0>(st, a, s1);
        }
        stamp(2);
        // (5) batch s of the staged tile; then the residual rows of the next batch (batch s + 1, or
        // batch 0 of this tile, which is staged at this step's end)
        if constexpr ((ABL & 64) == 0) {
          fk2_trickle<AACT, SUMONLY, TABLE, (ABL & 8) == 0>(st, a, resid, x_prv, nn_prv, s);
          if constexpr ((ABL & 16) == 0) {
            const bool last = s + 1 == KS;
            const int xc = i % kEmaps;
            const int nn_c = last ? __builtin_amdgcn_readfirstlane(st.ninfo[xc * kNodeInfo]) : nn_prv;
            fk2_prefetch(st, a, resid, last ? xc : x_prv, nn_c, last ? 0 : s + 1);
          }
        }
        // node list of tile i + 1 (its emap was written at the last advance, before a barrier)
        if (s == 1 && st.wave == 0)
          fk2_node_list(st.emap + ((i + 1) % kEmaps) * ROWS, st.ninfo + ((i + 1) % kEmaps) * kNodeInfo, st.lane);
        stamp(3);
        fk_barrier();
        stamp(4);
        // (6) end of the tile's K loop: stage this tile (the previous one is finished)
        ++g;
        if (++k == KS) {
          fk2_stage_one<0, 0, CT, GD>(st);
          x_prv = i % kEmaps;
          nn_prv = __builtin_amdgcn_readfirstlane(st.ninfo[x_prv * kNodeInfo]);
          fk_barrier();
          // advance: tile i + 1 becomes current, tile i + 2's row (loaded a tile ago) is published
          k = 0;
          ++i;
          cur = nxt;
          n_cur = n_nxt;
          const bool v2 = st.grow < h2.n;
          nxt = row_offsets(a, raw2, v2);
          if (info_writer) st.emap[((i + 1) % kEmaps) * ROWS + st.grow] = row_entry(raw2, v2);
          n_nxt = h2.n < ROWS ? h2.n : ROWS;
          h2 = h3;
          raw2 = row_raw<RT, TABLE>(a, h2, st.grow);
          h3 = tile_head<RT, TABLE>(a, tile(i + 3));
          stamp(5);
        }
      }
    }
  }
  if constexpr (STAMP) {
    if (st.lane == 0) {
#pragma unroll
      for (int q = 0; q < 6; ++q) atomicAdd(&g_pk_stamps[q], tacc[q]);
      atomicAdd(&g_pk_stamps[6], __builtin_amdgcn_s_memtime() - tb);
      atomicAdd(&g_pk_stamps[7], 1ull);
    }
  }
  // ---- tail: finish the last staged tile (batches 0 .. KS - 1, one barrier each)
  for (int s = 0; s < KS; ++s) {
    fk2_trickle<AACT, SUMONLY, TABLE>(st, a, resid, x_prv, nn_prv, s);
    fk2_prefetch(st, a, resid, x_prv, nn_prv, s + 1);
    fk_barrier();
  }
  if (a.amax_out) {
    const float mh = wave_max(st.mxH), ms = wave_max(st.mxS);
    if (st.lane == 0) {
      atomic_max_abs(a.amax_out, mh);
      if (a.SO) atomic_max_abs(a.amax_out + 1, ms);
    }
  }
}

}  // namespace fk
}  // namespace nt

// fp32 D-MPNN layer kernel on fp16 MFMA with a two-part split ("fk"), optionally fused with the
// aggregation its output feeds.  Included by update_pk.hip.  Tiles hold at most 16 RT rows: the plan
// builders guarantee it and check it when they build a plan (kernels.tile_plan, host_tile_plan); the
// kernel clamps a larger tile to its capacity (memory-safe) and keeps no device status word.
//
//   H_out[e] = (residual ? H[e] : 0) + W (S[src[e]] - act(H[rev[e]])) + b        (chemprop.py:36-43,
//                                                                                 residual.py:27-28)
//   S_out[v] = reduce_{e: dst[e] = v} aact(H_out[e])                               (chemprop.py:37-39,
//                                                                                 :86 with identity)
//
// Numerics (fp32 contract).  Every operand is split into two fp16 parts, x = x0 + x1 with
// x0 = fp16(x), x1 = fp16(x - x0), after a power-of-two scale that puts the operand's magnitude
// bound at 2^14: the A rows by s_A (from amax_in = max|H|, max|S| of the inputs, written by the
// kernels that produced them), W by s_W (stored in the image header by the pack kernel).  Three
// v_mfma_f32_16x16x32_f16 products per k-step, W1 A0 + W0 A1 + W0 A0, accumulate in fp32; the
// dropped W1 A1 term and the two split roundings are ~2^-22 relative: 8.6e-7 normalised from fp64 at
// config 2, 2.7x the fp32 CPU oracle's 3.2e-7 (tests/test_gpu_numerics.py).  The scale is per tensor,
// but the low part is stored x 2^11 (lo_part; its product takes W0 x 2^-11), so rows down to 2^-28 of
// the scaled max keep both parts normal: per-row fp32 accuracy.  Half the MFMA work of a bf16x6 split and
// two thirds of its operand bytes.  The residual row enters the accumulator scaled by s_A s_W while
// the K loop runs; the epilogue multiplies by the exact inverse and adds the bias.
//
// Structure: persistent, one 512-thread workgroup (8 waves, two per SIMD) per CU over a tile plan
// of up to 16 RT rows per tile, cut at node boundaries (nt_dmpnn_tile_plan) and balanced to a
// whole number of tiles per CU.  Each XCD walks one contiguous 1/nxcd of the plan (rows of
// neighbouring tiles stay in that XCD's L2).  Per 32-deep k-step every thread gathers its
// (row, 8-k) piece of S[src] and H[rev] two steps ahead into registers, forms A, splits it and
// writes both fp16 parts straight into MFMA fragment order in an LDS double buffer; all 8 waves
// then read the whole A slice (16 ds_read_b128 per wave) and run the MFMAs for their own output
// column tiles (wave w: tiles w, w + 8, w + 16 of the chunk) with W fragments prefetched one step
// ahead from the L2-resident image.  One barrier per k-step.  The tile's W image is read once per
// 16 RT rows (128 at h <= 384), so W bytes per edge are a quarter of the 64-row bf16x6 kernel's.
// Epilogue per wave and output column tile: scale + bias, H_out as 16-B row pieces from the
// accumulators, and the fused aggregation as a left-to-right segmented scan over the tile's rows
// (DPP row shifts within 16 lanes, carries between row tiles): the node sums come out in ascending
// edge order, bit-identical to CPU scatter_add_ of the same H_out.  Hidden sizes beyond one chunk
// of 128 columns x CT (h > 384 / 512) loop over column chunks, re-gathering A per chunk.
#pragma once

#include <type_traits>

#include "common.hpp"

namespace nt {
namespace fk {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// bf16 storage (PREC = 1): the two bf16 halves of a 32-bit word, widened exactly
__device__ __forceinline__ float bf_lo(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }
// four consecutive bf16 (8 B, the low two words of v) widened to fp32
__device__ __forceinline__ float4 bf4_widen(uint4 v) {
  return float4{bf_lo(v.x), bf_hi(v.x), bf_lo(v.y), bf_hi(v.y)};
}
// fp32 -> four bf16 (round to nearest even), packed in 8 B
__device__ __forceinline__ uint2 bf4_pack(float a, float b, float c, float d) {
  const bf16x4 v = bf16x4{(__bf16)a, (__bf16)b, (__bf16)c, (__bf16)d};
  return __builtin_bit_cast(uint2, v);
}

constexpr int kThreads = 512;
constexpr int kWaves = 8;
constexpr int kImgHdr = 256;  // image header bytes (float s_W at 0, max|W| partials at 1..32); fragments follow
constexpr int kEmaps = 4;     // row-info buffers (tile index mod 4)
// row flags: first / last row of a segment; kFlagPart: a hub sub-run whose sum goes to the partial rows
// a.SP (row-table entries of hub rows are negative: -((slot << 2) | start | end << 1) - 1)
constexpr int kFlagStart = 1, kFlagEnd = 2, kFlagPart = 4;

__host__ __device__ constexpr int ks_for(int64_t h) { return (int)((h + 31) / 32); }
__host__ __device__ constexpr int nt_for(int64_t h) { return (int)((h + 15) / 16); }
// image bytes of one layer: header + KS x NT x 2 parts x 1 KiB fragment blocks
__host__ __device__ constexpr int64_t image_bytes(int64_t h) {
  return kImgHdr + (int64_t)ks_for(h) * nt_for(h) * 2 * 1024;
}

struct Args {
  const float* H;     // E x h (NULL in dense mode)
  const float* S;     // V x h (dense mode: the M x h operand X)
  const int64_t* src;  // NULL: dense mode (A[e] = S[e])
  const int64_t* rev;  // NULL: nothing subtracted
  const char* Wimg;   // fk image of one layer
  const float* bias;  // may be NULL
  const float* amax_in;  // [0] max|H| (unused in dense mode), [1] max|S|
  float* amax_out;       // may be NULL: [0] max over H_out, [1] max over S_out (atomic max)
  int64_t V, E;
  int h, hv, KS, NT, nchunks;
  // row pitches: ldiv = 16-B gather pieces per input row of H and S (fp32 ld / 4, bf16 ld / 8); ldic /
  // ldoc = 4-column pieces per input (H residual) / output (H_out, S_out) row.  = hv, h / 4 for dense rows
  int ldiv, ldic, ldoc;
  int residual, act;
  float alpha;
  const int* tile_ptr;  // NULL: fixed tiles of 16 RT rows in edge order (no aggregation)
  int ntiles;
  const int4* rows;  // fused mode: row table {edge, src, rev, (node << 2) | start | end << 1} per
                     // dst-sorted position (nt_dmpnn_row_table)
  int reduce, aact;
  float aalpha;
  float* O;
  float* SO;  // NULL: no aggregation
  float* SP = nullptr;  // hub partial rows (slots x h fp32), written at the end rows of kFlagPart sub-runs
  int nxcd;
  int stagger;  // diagnostic: start delay of workgroup b = stagger * ((b / nxcd) % 4) x 8k cycles (0)
#ifdef NT_DIAG
  int rtabl = 0;  // diagnostic library: the fw walk's timing ablations (NT_FK_RTABL, results invalid)
#endif
};

// power-of-two scale that maps a magnitude bound to < 2^14 (exponent at most 24; every finite
// bound < 2^128 gets s >= -114, so no finite operand overflows fp16 after scaling).  A zero bound
// leaves the operand unscaled; so does a non-finite one (an inf / NaN in H or S): the rows holding it
// come out inf / NaN as in fp32, and finite entries above 65504 of that tensor overflow too (the
// contract covers finite inputs).
__host__ __device__ inline int scale_exp(float bound) {
  if (!(bound > 0.f) || !(bound <= 3.4028235e38f)) return 0;
  int e;
  frexpf(bound, &e);  // bound < 2^e, e <= 128
  int s = 14 - e;
  return s > 24 ? 24 : s;
}

// upper bound of |act(x)| for |x| <= m (every act code: relu / identity / gelu / silu <= m + 1,
// leaky <= max(1, |alpha|) m, elu <= max(m, |alpha|), tanh / sigmoid <= 1)
__device__ __forceinline__ float act_bound(float m, int act, float alpha) {
  if (act == NT_ACT_RELU || act == NT_ACT_IDENTITY) return m;
  const float a = fabsf(alpha) > 1.f ? fabsf(alpha) : 1.f;
  return a * m + a;
}

__device__ __forceinline__ void atomic_max_abs(float* p, float v) {
  // non-negative floats order like their bit patterns
  atomic_max_nonneg(p, v);
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

__device__ __forceinline__ f16x8 as_f16x8(uint4 v) { return __builtin_bit_cast(f16x8, v); }

// Low fp16 part of the split x = x0 + x1 (x0 = fp16(x)), stored as x1 x 2^11 so that it stays a
// normal fp16 for every x down to fp16's normal range (|x| >= 2^-14, 2^-28 of the scaled max 2^14):
// unscaled, x1 ~ 2^-11 x fell into fp16's subnormals for |x| < 2^-3, so rows far below the tensor's
// max (one split scale per tensor) lost their low part.  x - x0 and the x 2^11 are exact in fp32.
constexpr float kLoScale = 2048.f;
__device__ __forceinline__ _Float16 lo_part(float x, _Float16 x0) { return (_Float16)((x - (float)x0) * kLoScale); }

// compile-time loop: f(integral_constant<int, 0>) ... f(integral_constant<int, N - 1>), so register
// arrays are only ever indexed by constants (a dynamic index would put them in scratch)
template <typename F, int... Is>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}

// DPP: y[lane] = x[lane - 1] within each row of 16 lanes; lane 0 of a row keeps `old`
__device__ __forceinline__ float dpp_shr1(float old, float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old),
                                                               __builtin_bit_cast(int, x), 0x111, 0xf,
                                                               0xf, false));
}
// DPP with bound control: y[lane] = x[lane - 1] within each row of 16 lanes, lane 0 of a row reads 0
__device__ __forceinline__ float dpp_shr1_bc(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x111, 0xf, 0xf, true));
}
// DPP: y[lane] = x[lane + 15 mod 16] within each row (lane 0 gets lane 15)
__device__ __forceinline__ float dpp_ror1(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x121,
                                                               0xf, 0xf, false));
}

// --------------------------------------------------------------------------- per-row tile info
struct TileHead {  // tile bounds (uniform: scalar loads)
  int T, n;
};

template <int RT, bool PLAN>
__device__ __forceinline__ TileHead tile_head(const Args& a, int t) {
  if constexpr (PLAN) {
    const int T = a.tile_ptr[t], n = a.tile_ptr[t + 1] - T;
    return {T, n};
  }
  const int64_t T = (int64_t)t * (16 * RT);
  const int64_t n = a.E - T < 16 * RT ? a.E - T : 16 * RT;
  return {(int)T, (int)n};
}

// The thread's row of a tile in one dependent step: the row-table entry (fused mode) or
// {edge, src, rev} of the edge-ordered position (plain / dense mode).  Rows past the tile read the
// tile's first row (valid memory, no branch) and are masked by row < n at use.
template <int RT, bool TABLE>
__device__ __forceinline__ int4 row_raw(const Args& a, TileHead th, int row) {
  const int pos = th.T + (row < th.n ? row : 0);
  if constexpr (TABLE) return a.rows[pos];
  const int s = a.src ? (int)a.src[pos] : pos;
  const int q = a.rev ? (int)a.rev[pos] : -1;
  return int4{pos, s, q, kFlagStart | kFlagEnd};
}

// float4 offsets of the S[src] and H[rev] rows (-1: none / row past the tile)
__device__ __forceinline__ int2 row_offsets(const Args& a, int4 raw, bool valid) {
  const bool sok = valid && raw.y >= 0 && raw.y < a.V, qok = valid && raw.z >= 0 && raw.z < a.E;
  return int2{sok ? raw.y * a.ldiv : -1, qok ? raw.z * a.ldiv : -1};
}

// emap entry {edge (-1 past the tile), node, flags, 0}
__device__ __forceinline__ int4 row_entry(int4 raw, bool valid) {
  if (!valid) return int4{-1, -1, kFlagStart | kFlagEnd, 0};
  if (raw.w >= 0) return int4{raw.x, raw.w >> 2, raw.w & 3, 0};
  const int wv = -raw.w - 1;  // a hub sub-run row: {edge, partial slot, flags | kFlagPart}
  return int4{raw.x, wv >> 2, (wv & 3) | kFlagPart, 0};
}

// --------------------------------------------------------------------------- kernel
// Per-thread state of the kernel.  Plain members + force-inlined free functions taking it by
// reference (no lambdas: closures holding pointers to these arrays kept them in scratch).
template <int RT, int CT, int GD = 2, int PREC = 0, int NW = 8>
struct State {
  static constexpr int ROWS = 16 * RT;
  static constexpr int PPT = 2 * RT / NW;   // 16-B pieces per thread per tensor per k-step (2 or 1)
  static constexpr int kPartB = RT * 1024;  // one fp16 part of a k-slice
  static constexpr int kBufB = 2 * kPartB;  // both parts
  f32x4 acc[RT][CT];
  f32x4 bias[CT];      // bias of the thread's 4 columns per column tile, for the next epilogue
  uint4 wb[2][CT][2];  // W fragments (parity, column tile, part)
  f32x4 gs[GD][PPT], gq[GD][PPT];  // staged pieces, GD k-steps ahead
  int gso[GD], gqo[GD];  // their row sources
  float mxH, mxS;
  // constants of the thread / launch
  int lane, wave, fr, g16, grt, grow, kp0, hv, hc, NT, CTC;  // hv: 16-B gather pieces per row,
                                                           // hc: 4-column output pieces per row
  int li, lo;  // row pitches in 4-column pieces: input (residual H), output (H_out, S_out)
  float sA, sAW, inv;
  char* abuf;
  float* lbias;  // 4-wave workgroups: the bias in fp32 (h floats) in LDS, loaded once
  int4* emap;
  __amdgpu_buffer_rsrc_t wrsrc;
};

template <int RT, int CT, int ACT, int P, int GD, int PREC, int NW>
__device__ __forceinline__ void fk_gather(State<RT, CT, GD, PREC, NW>& st, const Args& a, int soff, int qoff, int s) {
  st.gso[P] = soff;
  st.gqo[P] = qoff;
  const int sb = soff >= 0 ? soff : 0, qb = qoff >= 0 ? qoff : 0;
  const f32x4* S4 = reinterpret_cast<const f32x4*>(a.S);
  // no H (dense mode): read S's first rows instead (qoff is -1, the piece is masked at the split),
  // so the load is unconditional and the compiler's vmcnt waits stay counted
  const f32x4* H4 = reinterpret_cast<const f32x4*>(a.H ? a.H : a.S);
  // fp32: PPT pieces of 4 values; bf16: one piece of 8 values (128-row tiles), the same 8 k
  constexpr int NP = PREC ? 1 : State<RT, CT, GD, PREC, NW>::PPT;
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    int p = PREC ? 4 * s + st.g16 : 8 * s + st.kp0 + u;
    p = p < st.hv ? p : 0;
    st.gs[P][u] = S4[sb + p];
    st.gq[P][u] = H4[qb + p];
  }
}

// A = S[src] - act(H[rev]) of the staged piece, scaled by s_A, split into two fp16 parts written in
// MFMA B-fragment order (row tile grt, lane (k-group, row): 16 B per part) into LDS buffer P
template <int RT, int CT, int ACT, int P, int BUF, int GD, int PREC, int NW>
__device__ __forceinline__ void fk_split(State<RT, CT, GD, PREC, NW>& st, const Args& a, int s) {
  using St = State<RT, CT, GD, PREC, NW>;
  const bool sok = st.gso[P] >= 0, qok = st.gqo[P] >= 0;
  if constexpr (PREC == 1) {
    // bf16 storage: A in fp32 from the widened pieces, one rounding to bf16, one fragment part
    static_assert(RT == NW, "bf16 fk tiles: one row tile per wave");
    const bool in = 4 * s + st.g16 < st.hv;
    const uint4 su = __builtin_bit_cast(uint4, st.gs[P][0]), qu = __builtin_bit_cast(uint4, st.gq[P][0]);
    const unsigned sw[4] = {su.x, su.y, su.z, su.w}, qw[4] = {qu.x, qu.y, qu.z, qu.w};
    bf16x8 h0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float q0 = act_t<ACT>(bf_lo(qw[c]), a.act, a.alpha), q1 = act_t<ACT>(bf_hi(qw[c]), a.act, a.alpha);
      h0[2 * c] = (__bf16)((sok && in ? bf_lo(sw[c]) : 0.f) - (qok && in ? q0 : 0.f));
      h0[2 * c + 1] = (__bf16)((sok && in ? bf_hi(sw[c]) : 0.f) - (qok && in ? q1 : 0.f));
    }
    *reinterpret_cast<bf16x8*>(st.abuf + BUF * St::kBufB + st.grt * 1024 + st.lane * 16) = h0;
    return;
  }
  float x[4 * St::PPT];
#pragma unroll
  for (int u = 0; u < St::PPT; ++u) {
    const bool in = 8 * s + st.kp0 + u < st.hv;
    const f32x4 sv = st.gs[P][u];
    const f32x4 qv = st.gq[P][u];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float q = act_t<ACT>(qv[c], a.act, a.alpha);
      const float av = (sok && in ? sv[c] : 0.f) - (qok && in ? q : 0.f);
      x[4 * u + c] = av * st.sA;
    }
  }
  char* base = st.abuf + BUF * St::kBufB + st.grt * 1024 + st.lane * 16 +
               (RT == NW ? 0 : 8 * (st.wave >> 2));
  if constexpr (St::PPT == 2) {
    f16x8 h0, h1;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const _Float16 t0 = (_Float16)x[c];
      h0[c] = t0;
      h1[c] = lo_part(x[c], t0);
    }
    *reinterpret_cast<f16x8*>(base) = h0;
    *reinterpret_cast<f16x8*>(base + St::kPartB) = h1;
  } else {
    f16x4 h0, h1;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const _Float16 t0 = (_Float16)x[c];
      h0[c] = t0;
      h1[c] = lo_part(x[c], t0);
    }
    *reinterpret_cast<f16x4*>(base) = h0;
    *reinterpret_cast<f16x4*>(base + St::kPartB) = h1;
  }
}

template <int RT, int CT, int P, int GD, int PREC, int NW>
__device__ __forceinline__ void fk_load_w(State<RT, CT, GD, PREC, NW>& st, int c, int s) {
#pragma unroll
  for (int j = 0; j < CT; ++j) {
    // unconditional (no branch around vector-memory ops keeps the compiler's vmcnt waits counted):
    // a column tile past NT reads beyond the buffer's range, which returns zeros
    const int ct = c * st.CTC + st.wave + NW * j;
    // fp32: two parts per block behind the scale header; bf16: the plain bf16 image (one part)
    const int blk = PREC ? (s * st.NT + ct) * 1024 : kImgHdr + ((s * st.NT + ct) * 2) * 1024;
    const int soff = __builtin_amdgcn_readfirstlane(ct < st.NT ? blk : 0x7fff0000);
    st.wb[P][j][0] = __builtin_bit_cast(
        uint4, __builtin_amdgcn_raw_buffer_load_b128(st.wrsrc, st.lane * 16, soff, 0));
    if constexpr (PREC == 0)
      st.wb[P][j][1] = __builtin_bit_cast(
          uint4, __builtin_amdgcn_raw_buffer_load_b128(st.wrsrc, st.lane * 16, soff + 1024, 0));
  }
}

// W0 x 2^-11 in fp16 (exact unless the product is subnormal, i.e. |W0| < 2^-17 of the scaled max:
// such a weight's error term is below 2^-36 of the row's own scale): the operand of the scaled low
// part of A.  Volatile asm: one copy per use, so the compiler neither merges the (row tile, column
// tile) copies nor keeps 4 more registers per column tile live across the row tiles.
__device__ __forceinline__ f16x8 w0_lo_scaled(uint4 w) {
  const unsigned k = 0x10001000u;  // two fp16 2^-11
  uint4 r;
  asm volatile("v_pk_mul_f16 %0, %1, %2" : "=v"(r.x) : "v"(w.x), "s"(k));
  asm volatile("v_pk_mul_f16 %0, %1, %2" : "=v"(r.y) : "v"(w.y), "s"(k));
  asm volatile("v_pk_mul_f16 %0, %1, %2" : "=v"(r.z) : "v"(w.z), "s"(k));
  asm volatile("v_pk_mul_f16 %0, %1, %2" : "=v"(r.w) : "v"(w.w), "s"(k));
  return as_f16x8(r);
}

// one (row tile, column tile) k-step: fp32 = the three split products, bf16 = one bf16 MFMA.  a1 is
// the scaled low part A1 x 2^11 (lo_part), so its product takes W0 x 2^-11: W1 A0 + W0 A1 + W0 A0.
template <int PREC>
__device__ __forceinline__ f32x4 fk_mac(uint4 w0r, uint4 w1r, f16x8 a0, f16x8 a1, f32x4 t) {
  if constexpr (PREC == 1) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, w0r), __builtin_bit_cast(bf16x8, a0),
                                                   t, 0, 0, 0);
  } else {
    const f16x8 w0 = as_f16x8(w0r), w1 = as_f16x8(w1r);
    t = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1, a0, t, 0, 0, 0);
    t = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0_lo_scaled(w0r), a1, t, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(w0, a0, t, 0, 0, 0);
  }
}

template <int RT, int CT, int P, int GD, int PREC, int NW>
__device__ __forceinline__ void fk_mfma(State<RT, CT, GD, PREC, NW>& st, int c, int nrt) {
  using St = State<RT, CT, GD, PREC, NW>;
  const char* bb = st.abuf + P * St::kBufB + st.lane * 16;
  // A fragments one row tile ahead; the schedule barriers keep the compiler from hoisting every row
  // tile's fragments (64 VGPRs) above the MFMAs
  f16x8 a0 = *reinterpret_cast<const f16x8*>(bb);
  f16x8 a1 = PREC ? a0 : *reinterpret_cast<const f16x8*>(bb + St::kPartB);
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    if (rt < nrt) {
      f16x8 n0 = a0, n1 = a1;
      if (rt + 1 < RT) {
        n0 = *reinterpret_cast<const f16x8*>(bb + (rt + 1) * 1024);
        n1 = PREC ? n0 : *reinterpret_cast<const f16x8*>(bb + St::kPartB + (rt + 1) * 1024);
      }
#pragma unroll
      for (int j = 0; j < CT; ++j) {
        if (c * st.CTC + st.wave + NW * j < st.NT) {
          st.acc[rt][j] = fk_mac<PREC>(st.wb[P][j][0], st.wb[P][j][1], a0, a1, st.acc[rt][j]);
        }
      }
      a0 = n0;
      a1 = n1;
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// Residual rows H[e] of (tile i, chunk c), column tile j, loaded straight into the accumulators:
// issued by the epilogue of the previous (tile, chunk) as soon as it has stored column tile j, so
// they land during the rest of that epilogue; fk_resid_scale multiplies them by s_A s_W before the
// first MFMA of the K loop (48 packed multiplies per tile, no staging registers).
template <int RT, int CT, int GD, int PREC, int NW>
__device__ __forceinline__ void fk_resid_load(State<RT, CT, GD, PREC, NW>& st, const Args& a, int i, int c, int j) {
  using St = State<RT, CT, GD, PREC, NW>;
  int pc = 4 * (c * st.CTC + st.wave + NW * j) + st.g16;
  pc = pc < st.hc ? pc : 0;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int e = st.emap[(i % kEmaps) * St::ROWS + 16 * rt + st.fr].x;
    const int64_t r = (int64_t)(e >= 0 ? e : 0) * st.li + pc;
    if constexpr (PREC == 1) {  // 4 bf16 (8 B), widened by fk_resid_scale once they have landed
      const uint2 v = reinterpret_cast<const uint2*>(a.H)[r];
      st.acc[rt][j] = __builtin_bit_cast(f32x4, uint4{v.x, v.y, 0u, 0u});
    } else {
      st.acc[rt][j] = reinterpret_cast<const f32x4*>(a.H)[r];
    }
  }
}

// Bias of chunk c, column tile j: an unconditional load (no bias: S's first row, zeroed at use),
// issued a whole chunk before the epilogue that uses it.
template <int RT, int CT, int GD, int PREC, int NW>
__device__ __forceinline__ void fk_bias_load(State<RT, CT, GD, PREC, NW>& st, const Args& a, int c, int j) {
  int pc = 4 * (c * st.CTC + st.wave + NW * j) + st.g16;
  pc = (pc < st.hc && a.bias) ? pc : 0;
  if constexpr (PREC == 1) {  // raw 8 B, widened at use
    const uint2 v = reinterpret_cast<const uint2*>(a.bias ? a.bias : a.S)[pc];
    st.bias[j] = __builtin_bit_cast(f32x4, uint4{v.x, v.y, 0u, 0u});
  } else {
    st.bias[j] = reinterpret_cast<const f32x4*>(a.bias ? a.bias : a.S)[pc];
  }
}

template <int RT, int CT, int GD, int PREC, int NW>
__device__ __forceinline__ void fk_resid_scale(State<RT, CT, GD, PREC, NW>& st) {
  if constexpr (PREC == 1) {  // bf16: widen the raw residual pieces (no scale)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int j = 0; j < CT; ++j) {
        const float4 w = bf4_widen(__builtin_bit_cast(uint4, st.acc[rt][j]));
        st.acc[rt][j] = f32x4{w.x, w.y, w.z, w.w};
      }
    return;
  }
  const f32x4 s4 = f32x4{st.sAW, st.sAW, st.sAW, st.sAW};
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int j = 0; j < CT; ++j) st.acc[rt][j] = st.acc[rt][j] * s4;
}

// epilogue of (tile i, chunk c): scale + bias, H_out from the accumulators, fused aggregation as a
// left-to-right segmented scan over each row tile's 16 rows (rows on lanes fr, carries between row
// tiles): after L rounds the last row of every node holds ((m_first + m_2) + ...) + m_last.
// Column tiles and row tiles are compile-time (template recursion: the loops hold convergent DPP /
// ballot operations that the unroller leaves alone, and a runtime index puts the accumulators in
// scratch).
// 4-wave workgroups keep the bias in LDS instead of CT registers per thread (their 5 column tiles
// per wave leave no registers for it)
constexpr bool fk_lds_bias(int NW) { return NW == 4; }

struct EpiCtx {
  const f32x4* b4;
  f32x4* O4;
  f32x4* SO4;
  const int4* em;
  int n;
};

template <int RTI, int J, int RT, int CT, int AACT, bool SUMONLY, int MAXL, int GD, int ABL, int PREC, int NW>
__device__ __forceinline__ void fk_epi_row(State<RT, CT, GD, PREC, NW>& st, const Args& a, const EpiCtx& x0, int pc,
                                           bool pok, const f32x4& bj, f32x4& carry, float& ccnt) {
  if (16 * RTI < x0.n) {
    const int lo = st.lo;
    const int4 ri = x0.em[16 * RTI + st.fr];
    f32x4 o;
    uint2 ob = uint2{0u, 0u};  // bf16: the stored (rounded) H_out piece
    if constexpr (PREC == 1) {
      // bf16: acc + bias in fp32, one rounding; the aggregation below reads the stored value
      ob = bf4_pack(st.acc[RTI][J][0] + bj[0], st.acc[RTI][J][1] + bj[1], st.acc[RTI][J][2] + bj[2],
                    st.acc[RTI][J][3] + bj[3]);
      const float4 w = bf4_widen(uint4{ob.x, ob.y, 0u, 0u});
      o = f32x4{w.x, w.y, w.z, w.w};
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = fmaf(st.acc[RTI][J][q], st.inv, bj[q]);
    }
    const bool rok = ri.x >= 0 && pok;
    if (rok && (ABL & 64) == 0) {
      if constexpr (PREC == 1) {
        reinterpret_cast<uint2*>(x0.O4)[(int64_t)ri.x * lo + pc] = ob;
      } else {
        x0.O4[(int64_t)ri.x * lo + pc] = o;
        st.mxH = fmaxf(st.mxH, fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3]))));
      }
    }
    if (x0.SO4 != nullptr) {
      // MAXL rounds of x[r] = start[r] ? m[r] : x[r - 1] + m[r] (the carry enters at row 0): a
      // row's value is final once the rounds cover its distance from its node's first row, at
      // most max in-degree - 1 (<= 16 within a row tile); extra rounds leave converged rows as they
      // are.  Straight-line code: a branch around the rounds costs the kernel its registers.
      const bool start = (ri.z & kFlagStart) != 0;
      f32x4 m;
#pragma unroll
      for (int q = 0; q < 4; ++q) m[q] = act_t<AACT>(o[q], a.aact, a.aalpha);
      f32x4 x = m, cin;
#pragma unroll
      for (int q = 0; q < 4; ++q) cin[q] = dpp_ror1(carry[q]);
      float cnt = 1.f;
      const float cinc = SUMONLY ? 0.f : dpp_ror1(ccnt);
#pragma unroll
      for (int it = 0; it < MAXL; ++it) {
        f32x4 y;
#pragma unroll
        for (int q = 0; q < 4; ++q) y[q] = dpp_shr1(cin[q], x[q]);
        if constexpr (SUMONLY) {
          x = start ? m : y + m;
        } else {
          const float yc = dpp_shr1(cinc, cnt);
          f32x4 z;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float mx = fmaxf(y[q], m[q]), mn = fminf(y[q], m[q]), sm = y[q] + m[q];
            z[q] = a.reduce == NT_MAX ? mx : (a.reduce == NT_MIN ? mn : sm);
          }
          x = start ? m : z;
          cnt = start ? 1.f : yc + 1.f;
        }
      }
      if ((ri.z & kFlagPart) && (ri.z & kFlagEnd) && rok) {  // a hub sub-run: its raw partial
        if constexpr (PREC == 0) reinterpret_cast<f32x4*>(a.SP)[(int64_t)ri.y * st.hc + pc] = x;
      } else if ((ri.z & kFlagEnd) && rok && (ABL & 128) == 0) {
        f32x4 r = x;
        if (!SUMONLY && a.reduce == NT_MEAN) r = x / cnt;
        if constexpr (PREC == 1) {
          reinterpret_cast<uint2*>(x0.SO4)[(int64_t)ri.y * lo + pc] = bf4_pack(r[0], r[1], r[2], r[3]);
        } else {
          x0.SO4[(int64_t)ri.y * lo + pc] = r;
          st.mxS = fmaxf(st.mxS, fmaxf(fmaxf(fabsf(r[0]), fabsf(r[1])), fmaxf(fabsf(r[2]), fabsf(r[3]))));
        }
      }
      carry = x;
      ccnt = cnt;
    }
  }
  if constexpr (RTI + 1 < RT)
    fk_epi_row<RTI + 1, J, RT, CT, AACT, SUMONLY, MAXL, GD, ABL>(st, a, x0, pc, pok, bj, carry, ccnt);
}

template <int J, int RT, int CT, int AACT, bool SUMONLY, int MAXL, int GD, int ABL, int PREC, int NW>
__device__ __forceinline__ void fk_epi_col(State<RT, CT, GD, PREC, NW>& st, const Args& a, const EpiCtx& x0, int i, int c,
                                           bool load_next, int i_next, int c_next) {
  const int ct = c * st.CTC + st.wave + NW * J;
  if (ct < st.NT) {
    const int pc = 4 * ct + st.g16;
    const bool pok = pc < st.hc;
    f32x4 bj = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (fk_lds_bias(NW)) {  // the bias from LDS (copied once per workgroup): no registers
      if (x0.b4 && pok) bj = *reinterpret_cast<const f32x4*>(st.lbias + 4 * pc);
    } else {
      if (x0.b4 && pok) bj = st.bias[J];
    }
    if constexpr (PREC == 1 && !fk_lds_bias(NW)) {  // the raw bf16 bias piece (zero bits stay zero)
      const float4 w = bf4_widen(__builtin_bit_cast(uint4, bj));
      bj = f32x4{w.x, w.y, w.z, w.w};
    }
    f32x4 carry = f32x4{0.f, 0.f, 0.f, 0.f};
    float ccnt = 0.f;
    fk_epi_row<0, J, RT, CT, AACT, SUMONLY, MAXL, GD, ABL>(st, a, x0, pc, pok, bj, carry, ccnt);
  }
  // column tile J is stored: its accumulators start the next (tile, chunk) (after the last tile the
  // loads re-read this tile's rows and go unused)
  if (!fk_lds_bias(NW) && c_next != c) fk_bias_load(st, a, c_next, J);  // column chunks: the next chunk's bias
  if (load_next) {
    fk_resid_load(st, a, i_next, c_next, J);
  } else {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) st.acc[rt][J] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if constexpr (J + 1 < CT)
    fk_epi_col<J + 1, RT, CT, AACT, SUMONLY, MAXL, GD, ABL>(st, a, x0, i, c, load_next, i_next, c_next);
}

template <int RT, int CT, int AACT, bool SUMONLY, int MAXL, int GD, int ABL, int PREC, int NW>
__device__ __forceinline__ void fk_epilogue(State<RT, CT, GD, PREC, NW>& st, const Args& a, int i, int c, int n,
                                            bool load_next, int i_next, int c_next) {
  EpiCtx x0;
  x0.b4 = reinterpret_cast<const f32x4*>(a.bias);
  x0.O4 = reinterpret_cast<f32x4*>(a.O);
  x0.SO4 = reinterpret_cast<f32x4*>(a.SO);
  x0.em = st.emap + (i % kEmaps) * State<RT, CT, GD, PREC, NW>::ROWS;
  x0.n = n;
  fk_epi_col<0, RT, CT, AACT, SUMONLY, MAXL, GD, ABL>(st, a, x0, i, c, load_next, i_next, c_next);
}

constexpr int kLbiasB = 512 * 4;  // the bias in LDS (4-wave workgroups, h <= 512)

__device__ __forceinline__ void fk_barrier() {
  // LDS writes of this step retired, then the workgroup barrier (vector-memory loads stay in flight)
  __syncthreads();
}

// ABL (diagnostic builds only, 0 in the shipping library): timing ablations, results invalid --
// 1 gathers read row 0, 2 no MFMA, 4 no split, 8 no epilogue, 16 no per-step barrier, 32 no residual,
// 64 no H_out stores, 128 no S_out stores; 256 (results valid): per-phase s_memtime cycle sums into
// g_pk_stamps (0 residual scale + MFMAs, 1 W issue, 2 split + gather issue, 3 barrier, 4 epilogue,
// 6 whole loop, 7 waves).
template <int RT, int CT, int ACT, int AACT, bool SUMONLY, int MAXL, int GD = 2, int ABL = 0, int PREC = 0,
          int NW = 8>
__global__ void __launch_bounds__(64 * NW, 2) update_fk_kernel(Args a) {
  // fused variants (MAXL > 1) read their rows from the row table, plain ones from src / rev
  constexpr bool TABLE = MAXL > 1;
  using St = State<RT, CT, GD, PREC, NW>;
  constexpr int ROWS = St::ROWS;
  constexpr int kEmapB = kEmaps * ROWS * 16;
  static_assert(RT == NW || (RT == 4 && NW == 8), "row tiles per wave mapping");
  constexpr bool LB = fk_lds_bias(NW);
  constexpr int kExtraB = LB ? kLbiasB : 0;
  __shared__ __attribute__((aligned(16))) uint4 smem[(2 * St::kBufB + kEmapB + kExtraB) / 16];

  // XCD-aware persistent walk (blocks b and b + nxcd share an L2): each XCD one contiguous chunk
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
  if constexpr (NW == 4) {
    // two workgroups per CU: the second half of the grid (the second workgroup of each CU, which the
    // XCD walk also gives the smaller tile count) starts `stagger` x 8k cycles late, so the pair's
    // K loops and epilogues start out of phase (A/B: NT_FK_STAGGER)
    for (int q = (int)blockIdx.x >= (int)gridDim.x / 2 ? a.stagger : 0; q > 0; --q) __builtin_amdgcn_s_sleep(127);
  } else {
    for (int q = a.stagger * (((int)blockIdx.x / (nx > 0 ? nx : 1)) & 3); q > 0; --q) __builtin_amdgcn_s_sleep(127);
  }

  St st;
  const int tid = threadIdx.x;
  st.lane = tid & 63;
  st.wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  st.fr = st.lane & 15;
  st.g16 = st.lane >> 4;
  // one row tile per wave when the waves are as many as the row tiles (128 rows / 8 waves, 64 / 4),
  // else (64 rows / 8 waves) two waves per row tile, each half the k-pieces
  st.grt = RT == NW ? st.wave : (st.wave & 3);
  st.grow = 16 * st.grt + st.fr;
  st.kp0 = RT == NW ? 2 * st.g16 : 2 * st.g16 + (st.wave >> 2);
  st.hv = a.hv;       // fp32: h / 4 (16-B pieces of 4 floats); bf16: h / 8 (of 8 bf16)
  st.hc = a.h / 4;    // 4-column output pieces per row
  st.li = a.ldic;
  st.lo = a.ldoc;
  st.NT = a.NT;
  st.CTC = NW * CT;
  st.abuf = reinterpret_cast<char*>(smem);
  st.emap = reinterpret_cast<int4*>(st.abuf + 2 * St::kBufB);
  st.lbias = reinterpret_cast<float*>(st.abuf + 2 * St::kBufB + kEmapB);

  if constexpr (LB) {  // the bias in fp32, once (h <= 512)
    for (int q = tid; q < a.h; q += 64 * NW) {
      float b = 0.f;
      if (a.bias) {
        if constexpr (PREC == 1) b = __uint_as_float((unsigned)reinterpret_cast<const unsigned short*>(a.bias)[q] << 16);
        else b = a.bias[q];
      }
      st.lbias[q] = b;
    }
  }
  st.wrsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.Wimg, (short)0, PREC ? ks_for(a.h) * nt_for(a.h) * 1024 : (int)image_bytes(a.h), 0x00020000);
  st.mxH = 0.f;
  st.mxS = 0.f;
  // scales: s_A from the bound of |A| = |S[src] - act(H[rev])|, s_W from the image header
  if constexpr (PREC == 1) {  // bf16: no split, no scales
    st.sA = st.sAW = st.inv = 1.f;
  } else {
    const float bound = a.src ? a.amax_in[1] + (a.rev ? act_bound(a.amax_in[0], a.act, a.alpha) : 0.f)
                              : a.amax_in[1];
    st.sA = ldexpf(1.f, scale_exp(bound));
    const float sW = *reinterpret_cast<const float*>(a.Wimg);
    st.sAW = st.sA * sW;
    st.inv = 1.f / st.sAW;  // exact: a power of two
  }
  const bool resid = (ABL & 32) == 0 && a.residual && a.H != nullptr;
  const bool info_writer = st.g16 == 0 && st.wave < RT;
  const int SPT = a.nchunks * a.KS;  // steps per tile

  // ---- tile info: cur (tile i) and nxt (i + 1) row offsets, raw row of tile i + 2 in flight
  int2 cur, nxt;
  int n_cur, n_nxt;
  int4 raw2;
  TileHead h2, h3;  // h3: bounds of tile i + 3, loaded a tile before its row is
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

  // ---- prologue: steps 0 and 1 staged, W of step 0, slice 0 split into buffer 0
  __syncthreads();  // emap of tiles 0 and 1
  if (resid) {
#pragma unroll
    for (int j = 0; j < CT; ++j) fk_resid_load(st, a, 0, 0, j);
  }
#pragma unroll
  for (int j = 0; j < CT; ++j)
    if constexpr (!LB) fk_bias_load(st, a, 0, j);
  auto kcs = [&](int kk, int& cc, int& ss) __attribute__((always_inline)) {  // step in a tile -> chunk, k-step
    cc = kk / a.KS;
    ss = kk - cc * a.KS;
  };
  {  // steps 0, 1, 2 gathered, W of steps 0 and 1, slice 0 split (the launcher keeps SPT >= 3)
    int c1, s1;
    kcs(1, c1, s1);
    fk_gather<RT, CT, ACT, 0>(st, a, cur.x, cur.y, 0);
    fk_gather<RT, CT, ACT, 1>(st, a, cur.x, cur.y, 1 % a.KS);
    fk_load_w<RT, CT, 0>(st, 0, 0);
    fk_load_w<RT, CT, 1>(st, c1, s1);
    fk_split<RT, CT, ACT, 0, 0>(st, a, 0);
    fk_gather<RT, CT, ACT, 0>(st, a, cur.x, cur.y, 2 % a.KS);
  }
  fk_barrier();

  // ---- main loop: per (tile, column chunk) unit, the residual scale, then the unit's KS k-steps as
  // an inner loop of two steps per trip (register parity P: A buffer and W fragments of steps k and
  // k + 2, gather slot of steps k + 1 and k + 3; KS is even, so every unit starts at parity 0), then
  // the epilogue.  The epilogue loads the next unit's residual rows into the accumulators; they are
  // consumed (the residual scale) before the inner loop starts, so inside the inner loop no
  // accumulator is a pending load and the compiler's vmcnt waits count only the W fragments and
  // gathers each step really needs: W two steps ahead and gathers three steps ahead stay in flight
  // across the MFMAs.  Every vector-memory op is unconditional.
  int i = 0, c = 0;  // tile-local index, column chunk
  const int U = ntl * a.nchunks;
  [[maybe_unused]] unsigned long long tacc[5] = {0, 0, 0, 0, 0}, tp = 0, tb = 0;
  if constexpr ((ABL & 256) != 0) tb = tp = __builtin_amdgcn_s_memtime();
  auto stamp = [&](int slot) __attribute__((always_inline)) {
    if constexpr ((ABL & 256) != 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      tacc[slot] += t - tp;
      tp = t;
    }
  };
  for (int u = 0; u < U; ++u) {
    // (1) residual rows (loaded by the previous epilogue) into the accumulators' scale; without a
    // residual the accumulators are zero and the scale leaves them so.  Unconditional, so that no
    // path into the inner loop carries an accumulator load still pending.
    fk_resid_scale(st);
    const int nrt = (n_cur + 15) >> 4;
    const int kb = c * a.KS;
    for (int s0 = 0; s0 < a.KS; s0 += 2) {
#pragma unroll
      for (int P = 0; P < 2; ++P) {
        const int k = kb + s0 + P;
        auto phase_mfma = [&]() __attribute__((always_inline)) {
          // (2) MFMAs of step k
          if constexpr ((ABL & 2) == 0) {
            if (P == 0) fk_mfma<RT, CT, 0>(st, c, nrt);
            else fk_mfma<RT, CT, 1>(st, c, nrt);
          }
          stamp(0);
          // (3) W fragments of step k + 2 into the registers step k used
          {
            int c2, s2;
            kcs(k + 2 < SPT ? k + 2 : k + 2 - SPT, c2, s2);
            if (P == 0) fk_load_w<RT, CT, 0>(st, c2, s2);
            else fk_load_w<RT, CT, 1>(st, c2, s2);
          }
          stamp(1);
        };
        auto phase_split = [&]() __attribute__((always_inline)) {
          // (4) split step k + 1's staged piece into the other buffer, then gather step k + 3 into the
          // freed slot (tile i or i + 1)
          const int k1 = k + 1 < SPT ? k + 1 : k + 1 - SPT;
          const int s1 = k1 - (k1 / a.KS) * a.KS;
          if constexpr ((ABL & 4) == 0) {
            if (P == 0) fk_split<RT, CT, ACT, 1, 1>(st, a, s1);
            else fk_split<RT, CT, ACT, 0, 0>(st, a, s1);
          }
          const int k3 = k + 3;
          const int adv = k3 >= SPT ? 1 : 0;
          const int s3 = (k3 - adv * SPT) % a.KS;
          int so = adv == 0 ? cur.x : nxt.x, qo = adv == 0 ? cur.y : nxt.y;
          if constexpr ((ABL & 1) != 0) so = qo = 0;
          if (P == 0) fk_gather<RT, CT, ACT, 1>(st, a, so, qo, s3);
          else fk_gather<RT, CT, ACT, 0>(st, a, so, qo, s3);
          stamp(2);
        };
        phase_mfma();
        phase_split();
        if constexpr ((ABL & 16) == 0) fk_barrier();
        stamp(3);
      }
    }
    // (5) epilogue of the unit; it starts the next (tile, chunk)'s residual loads
    const bool last_c = c + 1 == a.nchunks;
    const int i_next = last_c ? (i + 1 < ntl ? i + 1 : i) : i, c_next = last_c ? 0 : c + 1;
    if constexpr ((ABL & 8) == 0) {
      fk_epilogue<RT, CT, AACT, SUMONLY, MAXL, GD, ABL>(st, a, i, c, n_cur, resid, i_next, c_next);
      stamp(4);
    }
    // (6) advance: tile i + 1 becomes current, tile i + 2's row (loaded a tile ago) is published
    c = c_next;
    if (last_c) {
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
    }
  }
  if (a.amax_out) {
    const float mh = wave_max(st.mxH), ms = wave_max(st.mxS);
    // one atomic pair per workgroup (the waves' maxima through LDS): every wave of the workgroup ran
    // the same persistent loop, so all reach this barrier
    __shared__ float amx[2][NW];
    if (st.lane == 0) {
      amx[0][st.wave] = mh;
      amx[1][st.wave] = ms;
    }
    __syncthreads();
    if (tid == 0) {
      float bh = amx[0][0], bs = amx[1][0];
#pragma unroll
      for (int w = 1; w < NW; ++w) {
        bh = fmaxf(bh, amx[0][w]);
        bs = fmaxf(bs, amx[1][w]);
      }
      atomic_max_abs(a.amax_out, bh);
      if (a.SO) atomic_max_abs(a.amax_out + 1, bs);
    }
  }
#ifdef NT_DIAG
  if constexpr ((ABL & 256) != 0) {
    if (st.lane == 0) {
      for (int q = 0; q < 5; ++q) atomicAdd(&g_pk_stamps[q], tacc[q]);
      atomicAdd(&g_pk_stamps[6], __builtin_amdgcn_s_memtime() - tb);
      atomicAdd(&g_pk_stamps[7], 1ull);
    }
  }
#endif
}

// Row table of a fused plan (one 16-B entry per dst-sorted position, so the layer kernel reaches a
// tile's rows in one dependent load): {edge, src[edge] (-1 if out of range), rev[edge] (-1 if out of
// range), (node << 2) | start | end << 1} with start / end = first / last in-edge of its node.
__global__ void __launch_bounds__(256) row_table_kernel(const int32_t* __restrict__ perm,
                                                        const int32_t* __restrict__ dsts,
                                                        const int64_t* __restrict__ src,
                                                        const int64_t* __restrict__ rev, int64_t V,
                                                        int64_t E, int4* __restrict__ out) {
  for (int64_t p = blockIdx.x * 256LL + threadIdx.x; p < E; p += (int64_t)gridDim.x * 256) {
    const int e = perm[p];
    const int64_t s = src[e], q = rev[e];
    const int v = dsts[p];
    const bool start = p == 0 || dsts[p - 1] != v, end = p + 1 == E || dsts[p + 1] != v;
    out[p] = int4{e, (s >= 0 && s < V) ? (int)s : -1, (q >= 0 && q < E) ? (int)q : -1,
                  (v << 2) | (start ? kFlagStart : 0) | (end ? kFlagEnd : 0)};
  }
}

// --------------------------------------------------------------------------- packing
// Two launches: the layer scales, then one thread per 16-B fragment slot: image block
// ((s NT + ct) 2 + p), lane l holds W[16 ct + (l & 15)][32 s + 8 (l >> 4) + j], j < 8, part p of the
// scaled two-part fp16 split.
// max|W| of every layer in kScaleParts partial maxima (header floats 1 .. kScaleParts): grid
// (kScaleParts, layers) of 256-thread blocks, each over a 1/kScaleParts slice of the layer
constexpr int kScaleParts = 32;
__global__ void __launch_bounds__(256) pack_fk_scale_kernel(const float* __restrict__ W, int64_t h,
                                                            int64_t w_stride, int64_t img_stride,
                                                            char* __restrict__ img) {
  const float* Wl = W + blockIdx.y * w_stride;
  const int64_t n = h * h, per = (n + kScaleParts - 1) / kScaleParts;
  const int64_t lo = blockIdx.x * per, hi = lo + per < n ? lo + per : n;
  __shared__ float red[4];
  float m = 0.f;
  for (int64_t q = lo + threadIdx.x; q < hi; q += 256) m = fmaxf(m, fabsf(Wl[q]));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0)
    reinterpret_cast<float*>(img + blockIdx.y * img_stride)[1 + blockIdx.x] =
        fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// fragment slots of every layer (after pack_fk_scale_kernel wrote the layer's partial maxima); block 0
// stores s_W in the header
__global__ void __launch_bounds__(256) pack_fk_kernel(const float* __restrict__ W, int64_t h, int KS,
                                                      int NT, int64_t w_stride, int64_t img_stride,
                                                      char* __restrict__ img) {
  const int layer = blockIdx.y;
  const float* Wl = W + layer * w_stride;
  char* out = img + layer * img_stride;
  float mw = 0.f;
#pragma unroll
  for (int i = 1; i <= kScaleParts; ++i) mw = fmaxf(mw, reinterpret_cast<const float*>(out)[i]);
  const float sW = ldexpf(1.f, scale_exp(mw));
  if (blockIdx.x == 0 && threadIdx.x == 0) *reinterpret_cast<float*>(out) = sW;
  const int64_t slots = (int64_t)KS * NT * 2 * 64;
  const int64_t q = blockIdx.x * 256LL + threadIdx.x;
  if (q >= slots) return;
  const int l = (int)(q & 63);
  const int64_t blk = q >> 6;
  const int p = (int)(blk & 1);
  const int64_t sc = blk >> 1;
  const int ct = (int)(sc % NT), s = (int)(sc / NT);
  const int col = 16 * ct + (l & 15);
  f16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 32 * s + 8 * (l >> 4) + j;
    const float w = (col < h && k < h) ? Wl[(int64_t)col * h + k] * sW : 0.f;
    const _Float16 w0 = (_Float16)w;
    v[j] = p == 0 ? w0 : (_Float16)(w - (float)w0);
  }
  *reinterpret_cast<f16x8*>(out + kImgHdr + q * 16) = v;
}

// Multi-layer pack: the fk images of up to kPackMax layer weights (separate tensors) and, optionally,
// the images of their transposes (the backward's dA = G W), in one launch pair: the scale partials
// of layer l (max|W| = max|W^T|) go into both headers; a fragment slot of the W^T image reads W
// transposed (no transposed copy of W).  Same values as pack_fk_{scale_,}kernel on W and on
// W.t().contiguous().
constexpr int kPackMax = 16;
struct PackPtrs {
  const float* W[kPackMax];
  char* img[kPackMax];
  char* imgT[kPackMax];  // may be NULL
};

__global__ void __launch_bounds__(256) pack_fk_scale_multi(PackPtrs p, int64_t h) {
  const float* Wl = p.W[blockIdx.y];
  const int64_t n = h * h, per = (n + kScaleParts - 1) / kScaleParts;
  const int64_t lo = blockIdx.x * per, hi = lo + per < n ? lo + per : n;
  __shared__ float red[4];
  float m = 0.f;
  for (int64_t q = lo + threadIdx.x; q < hi; q += 256) m = fmaxf(m, fabsf(Wl[q]));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float r = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    reinterpret_cast<float*>(p.img[blockIdx.y])[1 + blockIdx.x] = r;
    if (p.imgT[blockIdx.y]) reinterpret_cast<float*>(p.imgT[blockIdx.y])[1 + blockIdx.x] = r;
  }
}

__global__ void __launch_bounds__(256) pack_fk_multi(PackPtrs p, int64_t h, int KS, int NT) {
  const int layer = blockIdx.y;
  const float* Wl = p.W[layer];
  char* out = p.img[layer];
  char* outT = p.imgT[layer];
  float mw = 0.f;
#pragma unroll
  for (int i = 1; i <= kScaleParts; ++i) mw = fmaxf(mw, reinterpret_cast<const float*>(out)[i]);
  const float sW = ldexpf(1.f, scale_exp(mw));
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *reinterpret_cast<float*>(out) = sW;
    if (outT) *reinterpret_cast<float*>(outT) = sW;
  }
  const int64_t slots = (int64_t)KS * NT * 2 * 64;
  const int64_t q = blockIdx.x * 256LL + threadIdx.x;
  if (q >= slots) return;
  const int l = (int)(q & 63);
  const int64_t blk = q >> 6;
  const int part = (int)(blk & 1);
  const int64_t sc = blk >> 1;
  const int ct = (int)(sc % NT), s = (int)(sc / NT);
  const int col = 16 * ct + (l & 15);
  f16x8 v, vt;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 32 * s + 8 * (l >> 4) + j;
    const bool in = col < h && k < h;
    const float w = in ? Wl[(int64_t)col * h + k] * sW : 0.f;
    const _Float16 w0 = (_Float16)w;
    v[j] = part == 0 ? w0 : (_Float16)(w - (float)w0);
    if (outT) {  // W^T[col][k] = W[k][col]
      const float wt = in ? Wl[(int64_t)k * h + col] * sW : 0.f;
      const _Float16 t0 = (_Float16)wt;
      vt[j] = part == 0 ? t0 : (_Float16)(wt - (float)t0);
    }
  }
  *reinterpret_cast<f16x8*>(out + kImgHdr + q * 16) = v;
  if (outT) *reinterpret_cast<f16x8*>(outT + kImgHdr + q * 16) = vt;
}

// atomically max |X| over n elements into *out (non-negative float bit order)
__global__ void __launch_bounds__(256) absmax_kernel(const float* __restrict__ X, int64_t n,
                                                     float* __restrict__ out) {
  float m = 0.f;
  const int64_t n4 = (reinterpret_cast<uintptr_t>(X) & 15) == 0 ? n / 4 : 0;
  const float4* X4 = reinterpret_cast<const float4*>(X);
  for (int64_t q = blockIdx.x * 256LL + threadIdx.x; q < n4; q += (int64_t)gridDim.x * 256) {
    const float4 v = X4[q];
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  }
  for (int64_t q = 4 * n4 + blockIdx.x * 256LL + threadIdx.x; q < n; q += (int64_t)gridDim.x * 256)
    m = fmaxf(m, fabsf(X[q]));
  block_max_to(out, m);
}

}  // namespace fk
}  // namespace nt

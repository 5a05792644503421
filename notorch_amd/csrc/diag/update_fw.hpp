// fp32 D-MPNN layer kernel at ONE wave per SIMD ("fw"), fused with the sum aggregation its output
// feeds.  Included by update_pk.hip after update_fk.hpp (same numerics, image, tile plan and row
// table as update_fk_kernel; it reuses that header's helpers).
//
//   H_out[e] = (residual ? H[e] : 0) + W (S[src[e]] - act(H[rev[e]])) + b        (chemprop.py:36-43,
//                                                                                 residual.py:27-28)
//   S_out[v] = sum_{e: dst[e] = v} aact(H_out[e])                                  (chemprop.py:37-39,
//                                                                                 :86 with identity)
//
// Why a second skeleton.  update_fk_kernel runs two waves per SIMD that meet at one workgroup barrier
// per k-step, so both waves of a SIMD issue their MFMAs in the same window and then their split VALU
// in the same window: the matrix pipe idles while the split runs (MFMA busy 17 % at config 2).  Here
// a 256-thread workgroup (4 waves, one per SIMD, up to 512 registers each) walks 128-row tiles, and
// each wave issues its step's MFMAs (all 8 row tiles x its NCT column tiles x 3 split products)
// with the side work of the same step placed between them: the W fragments of the next step, the
// split of the next step's gathered A slice into the other LDS buffer, and the gathers of the step
// after that.  The single wave keeps the MFMA stream and the VALU stream in one instruction stream,
// so the split rides in the MFMA issue gaps instead of after them.
//
// Numerics are update_fk_kernel's bit for bit (same split, same s_A / s_W, same product order
// W1 A0 + W0 A1 + W0 A0 per k-step in ascending k, the residual entering the accumulator scaled by
// s_A s_W, the same epilogue rounding and the same left-to-right segmented node sums), so either
// kernel may run any layer of a forward.
//
// Thread roles.  Gather / split: thread (wave w, lane l) stages row 32 w + (l & 31) of the tile,
// k-groups 2 q and 2 q + 1 (q = l >> 5) of each 32-deep k-step: four 16-B pieces of S[src] and of
// H[rev] per step (lanes l and l + 32 read the two halves of one 128-B row segment).  MFMA /
// epilogue: wave w owns column tiles w, w + 4, ... (NCT of them, compile time) for all 8 row tiles;
// lane l holds row l & 15 of a row tile, columns 4 (l >> 4) .. + 3 of a column tile.
#pragma once

#include "../update_fk.hpp"

#ifndef FW_ONE_PATH
#define FW_ONE_PATH 0
#endif
#ifndef FW_EPI_FENCE
#define FW_EPI_FENCE 0
#endif
// FW_EPI_RT: the row-tile-outer epilogue (fw_epilogue_rt); 0: column-tile-outer (fw_epi_col)
#ifndef FW_EPI_RT
#define FW_EPI_RT 1
#endif
// FW_EPI_LDS: the node sums from an LDS stage per column tile (fw_epilogue_lds; overrides FW_EPI_RT)
#ifndef FW_EPI_LDS
#define FW_EPI_LDS 1
#endif
// FW_STAMP (A/B builds): s_memtime sums per wave into g_pk_stamps: [0] K loops, [1] epilogues,
// [2] first step pair of each tile (the tile-start wait), [3] tiles, [4] waves, [5] whole walk
#ifndef FW_STAMP
#define FW_STAMP 0
#endif
// FW_ABL (A/B builds, timing ablations, results invalid): Args::rtabl bits (NT_FK_RTABL) -- 1 gathers
// read row 0, 4 no H_out / S_out stores, 8 residual rows read row 0, 32 no aggregation scan, 64 no
// epilogue at all, 128 no MFMA, 256 no split, 512 no per-step barrier, 2 W reads block 0, 1024 no W
// loads in the K loop, 2048 no gathers in the K loop
#ifndef FW_ABL
#define FW_ABL 0
#endif

namespace nt {
namespace fw {

using fk::Args;
using fk::f16x4;
using fk::f16x8;
using fk::f32x4;

constexpr int kThreads = 256;
constexpr int kRT = 8;                // row tiles per tile
constexpr int kRows = 16 * kRT;       // 128
constexpr int kPartB = kRT * 1024;    // one fp16 / bf16 part of a k-slice (8 KiB)
constexpr int kEmaps = 4;             // row-info buffers (tile index mod 4)
constexpr int kEmapB = kEmaps * kRows * 16;
constexpr int kBiasB = 512 * 4;
constexpr int kMaxNT = 20;            // fp32: h <= 320
constexpr int kMaxNTb = 32;           // bf16: h <= 512
// PREC 0: fp32 storage, two fp16 parts per k-slice; 1: bf16 storage, one bf16 part
constexpr int buf_bytes(int PREC) { return PREC ? kPartB : 2 * kPartB; }
// FW_EPI_LDS: per-wave stage of one column tile (128 rows x 16 columns, pitch 20 floats: conflict-free
// 16-B row writes) for the node reduction, and the tile's node list (start rows, count)
constexpr int kStagePitch = 20;
constexpr int kStageB = kRows * kStagePitch * 4;  // 10 KiB per wave
constexpr int kNodeListN = kRows + 4;             // start rows [0, ns], ns at [kRows + 2]
constexpr int kNodeListB = kNodeListN * 4;
constexpr int lds_bytes(int PREC) {
  return 2 * buf_bytes(PREC) + kEmapB + kBiasB + (FW_EPI_LDS ? 4 * (kStageB + kNodeListB) : 0);
}

template <int NCT, int PREC>
struct St {
  static constexpr int NPART = PREC ? 1 : 2;  // operand parts per fragment
  static constexpr int NPC = PREC ? 2 : 4;    // 16-B gather pieces per thread, tensor and k-step
  f32x4 acc[kRT][NCT];
  uint4 wb[2][NCT][NPART];     // W fragments (parity, column tile, part)
  f32x4 gs[2][NPC], gq[2][NPC];  // gathered pieces of two k-steps (slot, piece)
  int gso[2], gqo[2];          // their row sources (16-B piece offsets, -1: none)
  float mxH, mxS;
  int lane, wave, fr, g16, grow, q, hv, hc, NT;
  int rtabl;  // FW_ABL builds: Args::rtabl
  float sA, sAW, inv;
  char* abuf;
  int4* emap;
  float* lbias;
  float* stage;  // FW_EPI_LDS: this wave's column-tile stage
  int* nlist;    // FW_EPI_LDS: this wave's copy of the tile's node list
  __amdgpu_buffer_rsrc_t wrsrc;
};

// the thread's pieces of k-step s (fp32: 8 s + 4 q + u, u < 4; bf16: 4 s + 2 q + u, u < 2) of its
// row of S[src] and H[rev] into slot P
template <int NCT, int PREC, int P>
__device__ __forceinline__ void fw_gather(St<NCT, PREC>& st, const Args& a, int soff, int qoff, int s) {
  using S_ = St<NCT, PREC>;
  st.gso[P] = soff;
  st.gqo[P] = qoff;
  int sb = soff >= 0 ? soff : 0, qb = qoff >= 0 ? qoff : 0;
#if FW_ABL
  if (a.rtabl & 1) sb = qb = 0;
#endif
  const f32x4* S4 = reinterpret_cast<const f32x4*>(a.S);
  const f32x4* H4 = reinterpret_cast<const f32x4*>(a.H ? a.H : a.S);
#pragma unroll
  for (int u = 0; u < S_::NPC; ++u) {
    int p = 2 * S_::NPC * s + S_::NPC * st.q + u;
    p = p < st.hv ? p : 0;
    st.gs[P][u] = S4[sb + p];
    st.gq[P][u] = H4[qb + p];
  }
}

// item v (k-group 2 q + v) of slot P: A = S[src] - act(H[rev]) scaled by s_A, split into two fp16
// parts written in MFMA B-fragment order into LDS buffer BUF
template <int NCT, int PREC, int ACT, int P, int BUF>
__device__ __forceinline__ void fw_split(St<NCT, PREC>& st, const Args& a, int s, int v) {
  const bool sok = st.gso[P] >= 0, qok = st.gqo[P] >= 0;
  char* base = st.abuf + BUF * buf_bytes(PREC) + (st.grow >> 4) * 1024 + ((2 * st.q + v) * 16 + (st.grow & 15)) * 16;
  if constexpr (PREC == 1) {
    // bf16: piece v holds k-group 2 q + v (8 values); A in fp32 from the widened values, rounded to
    // bf16 once (as update_bf16_kernel)
    const bool in = 4 * s + 2 * st.q + v < st.hv;
    const uint4 su = __builtin_bit_cast(uint4, st.gs[P][v]), qu = __builtin_bit_cast(uint4, st.gq[P][v]);
    const unsigned sw[4] = {su.x, su.y, su.z, su.w}, qw[4] = {qu.x, qu.y, qu.z, qu.w};
    fk::bf16x8 hb;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float q0 = act_t<ACT>(fk::bf_lo(qw[c]), a.act, a.alpha), q1 = act_t<ACT>(fk::bf_hi(qw[c]), a.act, a.alpha);
      hb[2 * c] = (__bf16)((sok && in ? fk::bf_lo(sw[c]) : 0.f) - (qok && in ? q0 : 0.f));
      hb[2 * c + 1] = (__bf16)((sok && in ? fk::bf_hi(sw[c]) : 0.f) - (qok && in ? q1 : 0.f));
    }
    *reinterpret_cast<fk::bf16x8*>(base) = hb;
    return;
  }
  f16x8 h0, h1;
#pragma unroll
  for (int uu = 0; uu < 2; ++uu) {
    const int u = 2 * v + uu;
    const bool in = 8 * s + 4 * st.q + u < st.hv;
    const f32x4 sv = st.gs[P][u];
    const f32x4 qv = st.gq[P][u];
    // per piece: the scale s_A, or 0 for a masked operand (a row past the tile, k past h, no src /
    // rev); x = fma(s, fs, -act(q) fq) rounds once, = fp32(s - act(q)) s_A exactly (power of two);
    // relu(q) fq = max(q fq, 0) as fq >= 0.  A masked read is of valid memory (row 0 / piece 0):
    // finite by the contract, so its product with 0 is 0.
    const float fs = sok && in ? st.sA : 0.f, fq = qok && in ? st.sA : 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float qs;
      if constexpr (ACT == NT_ACT_RELU) qs = fmaxf(qv[c] * fq, 0.f);
      else qs = act_t<ACT>(qv[c], a.act, a.alpha) * fq;
      float x = fmaf(sv[c], fs, -qs);
      // x is the fp32 value of A s_A: keep hipcc from fusing the fma into the fp16 conversion
      // (v_fma_mix* would round the exact product to fp16 once, not fp32 x to fp16)
      asm volatile("" : "+v"(x));
      const _Float16 t0 = (_Float16)x;
      h0[4 * uu + c] = t0;
      h1[4 * uu + c] = fk::lo_part(x, t0);
    }
  }
  *reinterpret_cast<f16x8*>(base) = h0;
  *reinterpret_cast<f16x8*>(base + kPartB) = h1;
}

// W fragments of k-step s, column tiles [J0, J1) of this wave, into parity P
template <int NCT, int PREC, int P, int J0, int J1>
__device__ __forceinline__ void fw_load_w(St<NCT, PREC>& st, int s) {
#pragma unroll
  for (int j = J0; j < J1; ++j) {
    const int ct = st.wave + 4 * j;
    // fp32: two parts per block behind the scale header; bf16: the plain bf16 image (one part)
    int blk = PREC ? (s * st.NT + ct) * 1024 : fk::kImgHdr + ((s * st.NT + ct) * 2) * 1024;
#if FW_ABL
    if (st.rtabl & 2) blk = PREC ? 0 : fk::kImgHdr;
#endif
    const int soff = __builtin_amdgcn_readfirstlane(blk);
    st.wb[P][j][0] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(st.wrsrc, st.lane * 16, soff, 0));
    if constexpr (PREC == 0)
      st.wb[P][j][1] =
          __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(st.wrsrc, st.lane * 16, soff + 1024, 0));
  }
}

// residual rows of tile i, column tile j, straight into the accumulators (scaled before the K loop)
template <int NCT, int PREC>
__device__ __forceinline__ void fw_resid_load(St<NCT, PREC>& st, const Args& a, int i, int j) {
  int pc = 4 * (st.wave + 4 * j) + st.g16;
  pc = pc < st.hc ? pc : 0;
#pragma unroll
  for (int rt = 0; rt < kRT; ++rt) {
    int e = st.emap[(i % kEmaps) * kRows + 16 * rt + st.fr].x;
#if FW_ABL
    if (a.rtabl & 8) e = 0;
#endif
    st.acc[rt][j] = reinterpret_cast<const f32x4*>(a.H)[(int64_t)(e >= 0 ? e : 0) * st.hc + pc];
  }
}

// One k-step: MFMAs of step k (LDS buffer P, W parity P) with the side work of the step between
// the row tiles: W of step k + 1 into parity 1 - P, the split of the staged step k + 1 (slot 1 - P)
// into buffer 1 - P, then the gathers of step k + 3 into the freed slot.  Row tiles past the tile's
// rows (nrt) are skipped as a whole (wave-uniform).
template <int NCT, int PREC, int ACT, int P>
__device__ __forceinline__ void fw_step(St<NCT, PREC>& st, const Args& a, int s_w1, int s_split, int s_g, int g_soff,
                                        int g_qoff, int nrt) {
  const char* bb = st.abuf + P * buf_bytes(PREC) + st.lane * 16;
  f16x8 a0 = *reinterpret_cast<const f16x8*>(bb);
  f16x8 a1 = PREC ? a0 : *reinterpret_cast<const f16x8*>(bb + kPartB);
  fk::sfor<kRT>([&](auto RTc) {
    constexpr int rt = decltype(RTc)::value;
    f16x8 n0 = a0, n1 = a1;
    if constexpr (rt + 1 < kRT) {
      n0 = *reinterpret_cast<const f16x8*>(bb + (rt + 1) * 1024);
      if constexpr (PREC == 0) n1 = *reinterpret_cast<const f16x8*>(bb + kPartB + (rt + 1) * 1024);
    }
#if FW_ABL
    if (!(a.rtabl & 128))
#endif
    if (rt < 6 || rt < nrt) {
#pragma unroll
      for (int j = 0; j < NCT; ++j)
        st.acc[rt][j] = fk::fk_mac<PREC>(st.wb[P][j][0], st.wb[P][j][PREC ? 0 : 1], a0, a1, st.acc[rt][j]);
    }
    // side work of this row tile
#if FW_ABL
    if (!(a.rtabl & 1024)) {
#endif
    if constexpr (rt == 0) fw_load_w<NCT, PREC, 1 - P, 0, (NCT + 1) / 2>(st, s_w1);
    if constexpr (rt == 1) fw_load_w<NCT, PREC, 1 - P, (NCT + 1) / 2, NCT>(st, s_w1);
#if FW_ABL
    }
#endif
#if FW_ABL
    if (!(a.rtabl & 256)) {
#endif
    if constexpr (rt == 2) fw_split<NCT, PREC, ACT, 1 - P, 1 - P>(st, a, s_split, 0);
    if constexpr (rt == 3) fw_split<NCT, PREC, ACT, 1 - P, 1 - P>(st, a, s_split, 1);
#if FW_ABL
    }
#endif
#if FW_ABL
    if (!(a.rtabl & 2048))
#endif
    if constexpr (rt == 4) fw_gather<NCT, PREC, 1 - P>(st, a, g_soff, g_qoff, s_g);
    a0 = n0;
    a1 = n1;
    __builtin_amdgcn_sched_barrier(0);
  });
#if FW_ABL
  if (a.rtabl & 512) return;  // no barrier (results invalid)
#endif
  __syncthreads();
}

// bf16 residual pieces of column tile J (8 B = 4 bf16 per row tile), issued a column tile ahead
template <int NCT, int PREC>
__device__ __forceinline__ void fw_resid_bf(St<NCT, PREC>& st, const Args& a, const int4* em, int J, uint2 (&rr)[kRT]) {
  int pc = 4 * (st.wave + 4 * J) + st.g16;
  pc = pc < st.hc ? pc : 0;
#pragma unroll
  for (int rt = 0; rt < kRT; ++rt) {
    const int e = em[16 * rt + st.fr].x;
    rr[rt] = reinterpret_cast<const uint2*>(a.H)[(int64_t)(e >= 0 ? e : 0) * st.hc + pc];
  }
}

// epilogue unit (row tile RTI, column tile J): H_out piece, the segmented node scan (MAXL rounds,
// carries between row tiles) and S_out at node ends.  As fk_epi_row (SUMONLY).  fp32: H_out =
// acc / (s_A s_W) + b (the residual is in acc).  bf16: H_out = bf16((acc + b) + H[e]) as
// update_bf16_kernel, the scan over the stored (rounded) values.
template <int RTI, int J, int NCT, int PREC, int AACT, int MAXL>
__device__ __forceinline__ void fw_epi_row(St<NCT, PREC>& st, const Args& a, const int4* em, int n, int pc, bool pok,
                                           const f32x4& bj, f32x4& carry, const uint2 (&rr)[kRT], bool resid) {
  if (16 * RTI < n) {
    const int hc = st.hc;
    const int4 ri = em[16 * RTI + st.fr];
    f32x4 o;
    uint2 ob = uint2{0u, 0u};
    if constexpr (PREC == 1) {
      const float4 r = resid ? fk::bf4_widen(uint4{rr[RTI].x, rr[RTI].y, 0u, 0u}) : float4{0.f, 0.f, 0.f, 0.f};
      ob = fk::bf4_pack((st.acc[RTI][J][0] + bj[0]) + r.x, (st.acc[RTI][J][1] + bj[1]) + r.y,
                        (st.acc[RTI][J][2] + bj[2]) + r.z, (st.acc[RTI][J][3] + bj[3]) + r.w);
      const float4 w = fk::bf4_widen(uint4{ob.x, ob.y, 0u, 0u});
      o = f32x4{w.x, w.y, w.z, w.w};
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = fmaf(st.acc[RTI][J][q], st.inv, bj[q]);
    }
    bool rok = ri.x >= 0 && pok;
#if FW_ABL
    if (a.rtabl & 4) rok = false;
#endif
    if (rok) {
      if constexpr (PREC == 1) {
        reinterpret_cast<uint2*>(a.O)[(int64_t)ri.x * hc + pc] = ob;
      } else {
        reinterpret_cast<f32x4*>(a.O)[(int64_t)ri.x * hc + pc] = o;
        st.mxH = fmaxf(st.mxH, fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3]))));
      }
    }
    const bool start = (ri.z & fk::kFlagStart) != 0;
    f32x4 m;
#pragma unroll
    for (int q = 0; q < 4; ++q) m[q] = act_t<AACT>(o[q], a.aact, a.aalpha);
    f32x4 x = m, cin;
#pragma unroll
    for (int q = 0; q < 4; ++q) cin[q] = fk::dpp_ror1(carry[q]);
#if FW_ABL
    if (!(a.rtabl & 32))
#endif
#pragma unroll
    for (int it = 0; it < MAXL; ++it) {
      f32x4 y;
#pragma unroll
      for (int q = 0; q < 4; ++q) y[q] = fk::dpp_shr1(cin[q], x[q]);
      x = start ? m : y + m;
    }
    if ((ri.z & fk::kFlagEnd) && rok) {
      if constexpr (PREC == 1) {
        reinterpret_cast<uint2*>(a.SO)[(int64_t)ri.y * hc + pc] = fk::bf4_pack(x[0], x[1], x[2], x[3]);
      } else {
        reinterpret_cast<f32x4*>(a.SO)[(int64_t)ri.y * hc + pc] = x;
        st.mxS = fmaxf(st.mxS, fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])), fmaxf(fabsf(x[2]), fabsf(x[3]))));
      }
    }
    carry = x;
  }
#if FW_EPI_FENCE
  __builtin_amdgcn_sched_barrier(0);
#endif
  if constexpr (RTI + 1 < kRT) fw_epi_row<RTI + 1, J, NCT, PREC, AACT, MAXL>(st, a, em, n, pc, pok, bj, carry, rr, resid);
}

template <int J, int NCT, int PREC, int AACT, int MAXL>
__device__ __forceinline__ void fw_epi_col(St<NCT, PREC>& st, const Args& a, const int4* em, int n, bool resid,
                                           bool load_next, int i_next, uint2 (&rr0)[kRT], uint2 (&rr1)[kRT]) {
  uint2(&rr)[kRT] = (J & 1) ? rr1 : rr0;
  if constexpr (PREC == 1) {  // the next column tile's residual pieces, in flight across this one
    if (J + 1 < NCT && resid) fw_resid_bf(st, a, em, J + 1, (J & 1) ? rr0 : rr1);
  }
  const int pc = 4 * (st.wave + 4 * J) + st.g16;
  const bool pok = pc < st.hc;
  f32x4 bj = f32x4{0.f, 0.f, 0.f, 0.f};
  if (a.bias && pok) bj = *reinterpret_cast<const f32x4*>(st.lbias + 4 * pc);
  f32x4 carry = f32x4{0.f, 0.f, 0.f, 0.f};
  fw_epi_row<0, J, NCT, PREC, AACT, MAXL>(st, a, em, n, pc, pok, bj, carry, rr, resid);
  // column tile J is stored: fp32 -- its accumulators take the next tile's residual rows; bf16 --
  // they restart at zero (the residual enters in the epilogue)
  if (PREC == 0 && load_next) {
    fw_resid_load(st, a, i_next, J);
  } else {
#pragma unroll
    for (int rt = 0; rt < kRT; ++rt) st.acc[rt][J] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if constexpr (J + 1 < NCT) fw_epi_col<J + 1, NCT, PREC, AACT, MAXL>(st, a, em, n, resid, load_next, i_next, rr0, rr1);
}

// Row-tile-outer epilogue (FW_EPI_RT): per row tile, its row entry (read once, the next one in
// flight), then the NCT column tiles of the wave as independent units (their scans interleave, the
// node carries of all column tiles live across row tiles), H_out / S_out at one row address per row
// tile plus immediate column offsets, and then the next tile's residual rows of this row tile into
// its dead accumulators (fp32) -- the loads spread over the epilogue.  Same values as fw_epi_col.
template <int NCT, int PREC, int AACT, int MAXL>
__device__ __forceinline__ void fw_epilogue_rt(St<NCT, PREC>& st, const Args& a, const int4* em, int n, bool resid,
                                               bool load_next, const int4* em_next) {
  const int hc = st.hc;
  f32x4 carry[NCT], bj[NCT];
  bool pok[NCT];
  const int pc0 = 4 * st.wave + st.g16;  // column tile J: piece pc0 + 16 J
#pragma unroll
  for (int J = 0; J < NCT; ++J) {
    carry[J] = f32x4{0.f, 0.f, 0.f, 0.f};
    pok[J] = pc0 + 16 * J < hc;
    bj[J] = (a.bias && pok[J]) ? *reinterpret_cast<const f32x4*>(st.lbias + 4 * (pc0 + 16 * J)) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  int4 ri_n = em[st.fr];
  int en_n = load_next ? em_next[st.fr].x : 0;
  uint2 rr[NCT], rr_n[NCT];
  if constexpr (PREC == 1) {
#pragma unroll
    for (int J = 0; J < NCT; ++J) {
      const int pc = pok[J] ? pc0 + 16 * J : 0;
      rr_n[J] = resid ? reinterpret_cast<const uint2*>(a.H)[(int64_t)(ri_n.x >= 0 ? ri_n.x : 0) * hc + pc] : uint2{0u, 0u};
    }
  }
  fk::sfor<kRT>([&](auto RTc) {
    constexpr int rt = decltype(RTc)::value;
    const int4 ri = ri_n;
    const int en = en_n;
    if constexpr (rt + 1 < kRT) {
      ri_n = em[16 * (rt + 1) + st.fr];
      en_n = load_next ? em_next[16 * (rt + 1) + st.fr].x : 0;
    }
    if constexpr (PREC == 1) {
#pragma unroll
      for (int J = 0; J < NCT; ++J) rr[J] = rr_n[J];
      if constexpr (rt + 1 < kRT) {  // the next row tile's residual pieces, in flight across this one
#pragma unroll
        for (int J = 0; J < NCT; ++J) {
          const int pc = pok[J] ? pc0 + 16 * J : 0;
          rr_n[J] = resid ? reinterpret_cast<const uint2*>(a.H)[(int64_t)(ri_n.x >= 0 ? ri_n.x : 0) * hc + pc]
                          : uint2{0u, 0u};
        }
      }
    }
    if (16 * rt < n) {
      const bool rowok = ri.x >= 0;
      bool endok = (ri.z & fk::kFlagEnd) && rowok;
#if FW_ABL
      const bool st_ok = !(a.rtabl & 4);
#else
      constexpr bool st_ok = true;
#endif
      const bool start = (ri.z & fk::kFlagStart) != 0;
      const int64_t obase = (int64_t)(rowok ? ri.x : 0) * hc + pc0;
      const int64_t sbase = (int64_t)(ri.y >= 0 ? ri.y : 0) * hc + pc0;
#pragma unroll
      for (int J = 0; J < NCT; ++J) {
        f32x4 o;
        uint2 ob = uint2{0u, 0u};
        if constexpr (PREC == 1) {
          const float4 r = fk::bf4_widen(uint4{rr[J].x, rr[J].y, 0u, 0u});
          ob = fk::bf4_pack((st.acc[rt][J][0] + bj[J][0]) + r.x, (st.acc[rt][J][1] + bj[J][1]) + r.y,
                            (st.acc[rt][J][2] + bj[J][2]) + r.z, (st.acc[rt][J][3] + bj[J][3]) + r.w);
          const float4 w = fk::bf4_widen(uint4{ob.x, ob.y, 0u, 0u});
          o = f32x4{w.x, w.y, w.z, w.w};
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) o[q] = fmaf(st.acc[rt][J][q], st.inv, bj[J][q]);
        }
        if (rowok && pok[J] && st_ok) {
          if constexpr (PREC == 1) {
            reinterpret_cast<uint2*>(a.O)[obase + 16 * J] = ob;
          } else {
            reinterpret_cast<f32x4*>(a.O)[obase + 16 * J] = o;
            st.mxH = fmaxf(st.mxH, fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3]))));
          }
        }
        f32x4 m;
#pragma unroll
        for (int q = 0; q < 4; ++q) m[q] = act_t<AACT>(o[q], a.aact, a.aalpha);
        f32x4 x = m, cin;
#pragma unroll
        for (int q = 0; q < 4; ++q) cin[q] = fk::dpp_ror1(carry[J][q]);
#if FW_ABL
        if (!(a.rtabl & 32))
#endif
#pragma unroll
          for (int it = 0; it < MAXL; ++it) {
            f32x4 y;
#pragma unroll
            for (int q = 0; q < 4; ++q) y[q] = fk::dpp_shr1(cin[q], x[q]);
            x = start ? m : y + m;
          }
        if (endok && pok[J] && st_ok) {
          if constexpr (PREC == 1) {
            reinterpret_cast<uint2*>(a.SO)[sbase + 16 * J] = fk::bf4_pack(x[0], x[1], x[2], x[3]);
          } else {
            reinterpret_cast<f32x4*>(a.SO)[sbase + 16 * J] = x;
            st.mxS = fmaxf(st.mxS, fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])), fmaxf(fabsf(x[2]), fabsf(x[3]))));
          }
        }
        carry[J] = x;
      }
    }
    // row tile rt is stored: fp32 -- its accumulators take the next tile's residual rows; bf16 --
    // they restart at zero
    if constexpr (PREC == 0) {
      if (load_next) {
        int e = en;
#if FW_ABL
        if (a.rtabl & 8) e = 0;
#endif
        const int64_t rb = (int64_t)(e >= 0 ? e : 0) * hc;
#pragma unroll
        for (int J = 0; J < NCT; ++J)
          st.acc[rt][J] = reinterpret_cast<const f32x4*>(a.H)[rb + (pok[J] ? pc0 + 16 * J : 0)];
      } else {
#pragma unroll
        for (int J = 0; J < NCT; ++J) st.acc[rt][J] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    } else {
#pragma unroll
      for (int J = 0; J < NCT; ++J) st.acc[rt][J] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  });
}

// LDS-staged epilogue (FW_EPI_LDS).  Per column tile J of the wave: every row tile's unit computes
// H_out (stored as a 16-B row piece) and writes aact(H_out) into the wave's stage (128 rows x 16
// columns); then lanes take (node, 4-column piece) items -- 16 nodes x 4 pieces per round -- and sum
// the node's consecutive rows left to right from the stage (the order of CPU scatter_add_, so the
// same bits as the scan), S_out as 16-B pieces (4 lanes: one 64-B segment of the node row).  No
// cross-wave sync: each wave owns its stage and its copy of the tile's node list.  Per unit this is
// ~12 VALU + one ds_write instead of the scan's ~40 VALU.
template <int NCT, int PREC, int AACT>
__device__ __forceinline__ void fw_epilogue_lds(St<NCT, PREC>& st, const Args& a, const int4* em, int n, bool resid,
                                                bool load_next, const int4* em_next) {
  const int hc = st.hc;
  const int pc0 = 4 * st.wave + st.g16;  // column tile J: piece pc0 + 16 J
  // the tile's node list: start rows of its nodes (ascending), ns = count, start[ns] = n
  {
    const int l = st.lane;
    const bool s0 = l < n && (em[l].z & fk::kFlagStart), s1 = l + 64 < n && (em[l + 64].z & fk::kFlagStart);
    const unsigned long long m0 = __ballot(s0), m1 = __ballot(s1);
    const unsigned long long below = (1ull << l) - 1ull;
    const int c0 = __popcll(m0);
    if (s0) st.nlist[__popcll(m0 & below)] = l;
    if (s1) st.nlist[c0 + __popcll(m1 & below)] = l + 64;
    if (l == 0) {
      const int ns = c0 + __popcll(m1);
      st.nlist[ns] = n;
      st.nlist[kRows + 2] = ns;
    }
  }
  // the rows' edges (this tile) and the next tile's, one per row tile
  int e_row[kRT], e_nxt[kRT];
#pragma unroll
  for (int rt = 0; rt < kRT; ++rt) {
    e_row[rt] = em[16 * rt + st.fr].x;
    e_nxt[rt] = load_next ? em_next[16 * rt + st.fr].x : 0;
  }
  uint2 rr[kRT], rr_n[kRT];
  if constexpr (PREC == 1) {
#pragma unroll
    for (int rt = 0; rt < kRT; ++rt)
      rr_n[rt] = resid ? reinterpret_cast<const uint2*>(a.H)[(int64_t)(e_row[rt] >= 0 ? e_row[rt] : 0) * hc + pc0]
                       : uint2{0u, 0u};
  }
  const int ns = st.nlist[kRows + 2];
  fk::sfor<NCT>([&](auto Jc) {
    constexpr int J = decltype(Jc)::value;
    const int pc = pc0 + 16 * J;
    const bool pok = pc < hc;
    const f32x4 bj = (a.bias && pok) ? *reinterpret_cast<const f32x4*>(st.lbias + 4 * pc) : f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (PREC == 1) {
#pragma unroll
      for (int rt = 0; rt < kRT; ++rt) rr[rt] = rr_n[rt];
      if constexpr (J + 1 < NCT) {  // the next column tile's residual pieces, in flight across this one
        const int pn = pc + 16 < hc ? pc + 16 : 0;
#pragma unroll
        for (int rt = 0; rt < kRT; ++rt)
          rr_n[rt] = resid ? reinterpret_cast<const uint2*>(a.H)[(int64_t)(e_row[rt] >= 0 ? e_row[rt] : 0) * hc + pn]
                           : uint2{0u, 0u};
      }
    }
#if FW_ABL
    const bool st_ok = !(a.rtabl & 4);
#else
    constexpr bool st_ok = true;
#endif
    // (1) units: H_out, aact(H_out) into the stage
#pragma unroll
    for (int rt = 0; rt < kRT; ++rt) {
      if (16 * rt < n) {
        f32x4 o;
        uint2 ob = uint2{0u, 0u};
        if constexpr (PREC == 1) {
          const float4 r = fk::bf4_widen(uint4{rr[rt].x, rr[rt].y, 0u, 0u});
          ob = fk::bf4_pack((st.acc[rt][J][0] + bj[0]) + r.x, (st.acc[rt][J][1] + bj[1]) + r.y,
                            (st.acc[rt][J][2] + bj[2]) + r.z, (st.acc[rt][J][3] + bj[3]) + r.w);
          const float4 w = fk::bf4_widen(uint4{ob.x, ob.y, 0u, 0u});
          o = f32x4{w.x, w.y, w.z, w.w};
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) o[q] = fmaf(st.acc[rt][J][q], st.inv, bj[q]);
        }
        const int e = e_row[rt];
        if (e >= 0 && pok && st_ok) {
          if constexpr (PREC == 1) {
            reinterpret_cast<uint2*>(a.O)[(int64_t)e * hc + pc] = ob;
          } else {
            reinterpret_cast<f32x4*>(a.O)[(int64_t)e * hc + pc] = o;
            st.mxH = fmaxf(st.mxH, fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3]))));
          }
        }
        f32x4 m;
#pragma unroll
        for (int q = 0; q < 4; ++q) m[q] = act_t<AACT>(o[q], a.aact, a.aalpha);
        *reinterpret_cast<f32x4*>(st.stage + (16 * rt + st.fr) * kStagePitch + 4 * st.g16) = m;
      }
      // row tile rt of column tile J is out: fp32 -- the accumulators take the next tile's residual
      // rows; bf16 -- they restart at zero
      if constexpr (PREC == 0) {
        if (load_next) {
          int en = e_nxt[rt];
#if FW_ABL
          if (a.rtabl & 8) en = 0;
#endif
          st.acc[rt][J] = reinterpret_cast<const f32x4*>(a.H)[(int64_t)(en >= 0 ? en : 0) * hc + (pok ? pc : 0)];
        } else {
          st.acc[rt][J] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      } else {
        st.acc[rt][J] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    // (2) nodes: lane = (node 16 r + (lane >> 2), piece lane & 3), rows summed left to right (the
    // stage rows were written by other lanes of this wave: LDS keeps a wave's operations in order)
    __builtin_amdgcn_wave_barrier();
    const int p4 = st.lane & 3;
    const int pcn = 4 * (st.wave + 4 * J) + p4;  // the item's 4-column piece of the row
    for (int k = st.lane >> 2; k < ns; k += 16) {
      const int r0 = st.nlist[k], r1 = st.nlist[k + 1];
      f32x4 x = *reinterpret_cast<const f32x4*>(st.stage + r0 * kStagePitch + 4 * p4);
      for (int r = r0 + 1; r < r1; ++r) x = x + *reinterpret_cast<const f32x4*>(st.stage + r * kStagePitch + 4 * p4);
      const int4 re = em[r1 - 1];  // the node's last row: its id and end flag (hub rows carry none)
      if ((re.z & fk::kFlagEnd) && re.x >= 0 && pcn < hc && st_ok) {
        if constexpr (PREC == 1) {
          reinterpret_cast<uint2*>(a.SO)[(int64_t)re.y * hc + pcn] = fk::bf4_pack(x[0], x[1], x[2], x[3]);
        } else {
          reinterpret_cast<f32x4*>(a.SO)[(int64_t)re.y * hc + pcn] = x;
          st.mxS = fmaxf(st.mxS, fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])), fmaxf(fabsf(x[2]), fabsf(x[3]))));
        }
      }
    }
    __builtin_amdgcn_wave_barrier();  // the next column tile rewrites the stage
  });
}

template <int NCT, int PREC, int ACT, int AACT, int MAXL>
__device__ __forceinline__ void fw_run(const Args& a, char* smem, int t0, int tstride, int ntl) {
  auto tile = [&](int i) __attribute__((always_inline)) { return t0 + (i < ntl ? i : ntl - 1) * tstride; };
  St<NCT, PREC> st;
  const int tid = threadIdx.x;
  st.lane = tid & 63;
  st.wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  st.fr = st.lane & 15;
  st.g16 = st.lane >> 4;
  st.grow = 32 * st.wave + (st.lane & 31);
  st.q = st.lane >> 5;
  st.hv = a.hv;
  st.hc = a.h / 4;
  st.NT = a.NT;
  st.rtabl = a.rtabl;
  st.abuf = smem;
  st.emap = reinterpret_cast<int4*>(smem + 2 * buf_bytes(PREC));
  st.lbias = reinterpret_cast<float*>(smem + 2 * buf_bytes(PREC) + kEmapB);
  st.stage = reinterpret_cast<float*>(smem + 2 * buf_bytes(PREC) + kEmapB + kBiasB + st.wave * kStageB);
  st.nlist = reinterpret_cast<int*>(smem + 2 * buf_bytes(PREC) + kEmapB + kBiasB + 4 * kStageB) + st.wave * kNodeListN;
  for (int c = tid; c < a.h; c += kThreads) {
    float b = 0.f;
    if (a.bias) {
      if constexpr (PREC == 1) b = __uint_as_float((unsigned)reinterpret_cast<const unsigned short*>(a.bias)[c] << 16);
      else b = a.bias[c];
    }
    st.lbias[c] = b;
  }
  st.wrsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.Wimg, (short)0, PREC ? fk::ks_for(a.h) * fk::nt_for(a.h) * 1024 : (int)fk::image_bytes(a.h), 0x00020000);
  st.mxH = 0.f;
  st.mxS = 0.f;
  if constexpr (PREC == 1) {
    st.sA = st.sAW = st.inv = 1.f;
  } else {
    const float bound = a.amax_in[1] + (a.rev ? fk::act_bound(a.amax_in[0], a.act, a.alpha) : 0.f);
    st.sA = ldexpf(1.f, fk::scale_exp(bound));
    const float sW = *reinterpret_cast<const float*>(a.Wimg);
    st.sAW = st.sA * sW;
    st.inv = 1.f / st.sAW;
  }
  const bool resid = a.residual && a.H != nullptr;
  const bool info_writer = st.q == 0;
  const int SPT = a.KS;

  // ---- tile info: cur (tile i) and nxt (i + 1) row offsets, raw row of tile i + 2 in flight
  int2 cur, nxt;
  int n_cur, n_nxt;
  int4 raw2;
  fk::TileHead h2, h3;
  {
    const fk::TileHead h0 = fk::tile_head<kRT, true>(a, tile(0));
    const int4 r0 = fk::row_raw<kRT, true>(a, h0, st.grow);
    const fk::TileHead h1 = fk::tile_head<kRT, true>(a, tile(1));
    const int4 r1 = fk::row_raw<kRT, true>(a, h1, st.grow);
    h2 = fk::tile_head<kRT, true>(a, tile(2));
    raw2 = fk::row_raw<kRT, true>(a, h2, st.grow);
    h3 = fk::tile_head<kRT, true>(a, tile(3));
    const bool v0 = st.grow < h0.n, v1 = st.grow < h1.n;
    cur = fk::row_offsets(a, r0, v0);
    nxt = fk::row_offsets(a, r1, v1);
    if (info_writer) {
      st.emap[0 * kRows + st.grow] = fk::row_entry(r0, v0);
      st.emap[1 * kRows + st.grow] = fk::row_entry(r1, v1);
    }
    n_cur = h0.n < kRows ? h0.n : kRows;
    n_nxt = h1.n < kRows ? h1.n : kRows;
  }
#pragma unroll
  for (int r = 0; r < kRT; ++r)
#pragma unroll
    for (int j = 0; j < NCT; ++j) st.acc[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();  // emap of tiles 0 and 1, the bias
  if (PREC == 0 && resid) {
#pragma unroll
    for (int j = 0; j < NCT; ++j) fw_resid_load(st, a, 0, j);
  }
  // steps 0 and 1 gathered, W of step 0, step 0 split into buffer 0, step 2 gathered
  fw_gather<NCT, PREC, 0>(st, a, cur.x, cur.y, 0);
  fw_gather<NCT, PREC, 1>(st, a, cur.x, cur.y, 1);
  fw_load_w<NCT, PREC, 0, 0, NCT>(st, 0);
  fw_split<NCT, PREC, ACT, 0, 0>(st, a, 0, 0);
  fw_split<NCT, PREC, ACT, 0, 0>(st, a, 0, 1);
  fw_gather<NCT, PREC, 0>(st, a, cur.x, cur.y, 2 % SPT);
  __syncthreads();

  uint2 rr0[kRT], rr1[kRT];
  [[maybe_unused]] unsigned long long ts_k = 0, ts_e = 0, ts_f = 0, ts_0 = 0, ts_1 = 0, ts_w = 0;
#if FW_STAMP
  ts_w = __builtin_amdgcn_s_memtime();
#endif
  for (int i = 0; i < ntl; ++i) {
#if FW_STAMP
    ts_0 = __builtin_amdgcn_s_memtime();
#endif
    if constexpr (PREC == 0) {  // residual rows (loaded by the previous epilogue) into the accumulators' scale
      const f32x4 s4 = f32x4{st.sAW, st.sAW, st.sAW, st.sAW};
#pragma unroll
      for (int rt = 0; rt < kRT; ++rt)
#pragma unroll
        for (int j = 0; j < NCT; ++j) st.acc[rt][j] = st.acc[rt][j] * s4;
    }
    const int nrt = (n_cur + 15) >> 4;
    for (int k = 0; k < SPT; k += 2) {
      // step k (parity 0) and k + 1 (parity 1); W one step ahead (the next tile's step 0 after the
      // last), split one step ahead, gathers three steps ahead (into the next tile at the end)
      {
        const int k3 = k + 3, adv = k3 >= SPT ? 1 : 0;
        fw_step<NCT, PREC, ACT, 0>(st, a, k + 1, k + 1, k3 - adv * SPT, adv ? nxt.x : cur.x, adv ? nxt.y : cur.y, nrt);
      }
      {
        const int k1 = k + 2 < SPT ? k + 2 : 0;
        const int k3 = k + 4, adv = k3 >= SPT ? 1 : 0;
        fw_step<NCT, PREC, ACT, 1>(st, a, k1, k1, k3 - adv * SPT, adv ? nxt.x : cur.x, adv ? nxt.y : cur.y, nrt);
      }
#if FW_STAMP
      if (k == 0) ts_f += __builtin_amdgcn_s_memtime() - ts_0;
#endif
    }
#if FW_STAMP
    ts_1 = __builtin_amdgcn_s_memtime();
    ts_k += ts_1 - ts_0;
#endif
    const bool more = i + 1 < ntl;
    const int4* em = st.emap + (i % kEmaps) * kRows;
#if FW_ABL
    if (a.rtabl & 64) {  // no epilogue: the K loops alone (accumulators restart at zero)
#pragma unroll
      for (int rt = 0; rt < kRT; ++rt)
#pragma unroll
        for (int j = 0; j < NCT; ++j) st.acc[rt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    } else
#endif
#if FW_EPI_LDS
    fw_epilogue_lds<NCT, PREC, AACT>(st, a, em, n_cur, resid, resid && more, st.emap + ((i + 1) % kEmaps) * kRows);
#elif FW_EPI_RT
    fw_epilogue_rt<NCT, PREC, AACT, MAXL>(st, a, em, n_cur, resid, resid && more, st.emap + ((i + 1) % kEmaps) * kRows);
#else
    if (PREC == 1 && resid) fw_resid_bf(st, a, em, 0, rr0);
    fw_epi_col<0, NCT, PREC, AACT, MAXL>(st, a, em, n_cur, resid, resid && more, i + 1, rr0, rr1);
#endif
#if FW_STAMP
    ts_e += __builtin_amdgcn_s_memtime() - ts_1;
#endif
    // advance: tile i + 1 becomes current, tile i + 2's row (loaded a tile ago) is published
    cur = nxt;
    n_cur = n_nxt;
    const bool v2 = st.grow < h2.n;
    nxt = fk::row_offsets(a, raw2, v2);
    if (info_writer) st.emap[((i + 2) % kEmaps) * kRows + st.grow] = fk::row_entry(raw2, v2);
    n_nxt = h2.n < kRows ? h2.n : kRows;
    h2 = h3;
    raw2 = fk::row_raw<kRT, true>(a, h2, st.grow);
    h3 = fk::tile_head<kRT, true>(a, tile(i + 4));
  }
  if (a.amax_out) {
    const float mh = fk::wave_max(st.mxH), ms = fk::wave_max(st.mxS);
    if (st.lane == 0) {
      fk::atomic_max_abs(a.amax_out, mh);
      fk::atomic_max_abs(a.amax_out + 1, ms);
    }
  }
#if FW_STAMP
  if (st.lane == 0) {
    atomicAdd(&g_pk_stamps[0], ts_k);
    atomicAdd(&g_pk_stamps[1], ts_e);
    atomicAdd(&g_pk_stamps[2], ts_f);
    atomicAdd(&g_pk_stamps[3], (unsigned long long)ntl);
    atomicAdd(&g_pk_stamps[4], 1ull);
    atomicAdd(&g_pk_stamps[5], __builtin_amdgcn_s_memtime() - ts_w);
  }
#endif
}

// Fused relu / sum layers, tiles of <= 128 rows; fp32 (PREC 0) h <= 320 (NT <= 20), bf16 (PREC 1)
// h <= 512 (NT <= 32): waves with ceil(NT / 4) column tiles run fw_run<CTM>, the others
// (NT % 4 != 0) fw_run<CTM - 1>.
template <int CTM, int PREC, int ACT, int AACT, int MAXL>
__global__ void __launch_bounds__(kThreads, 1) update_fw_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) char smem[lds_bytes(PREC)];
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
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int nct = (a.NT - wave + 3) / 4;
  if constexpr (CTM > 1 && !FW_ONE_PATH) {
    if (nct < CTM) {
      fw_run<CTM - 1, PREC, ACT, AACT, MAXL>(a, smem, t0, tstride, ntl);
      return;
    }
  }
  fw_run<CTM, PREC, ACT, AACT, MAXL>(a, smem, t0, tstride, ntl);
}

}  // namespace fw
}  // namespace nt

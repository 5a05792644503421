// Launchers of the fp32 D-MPNN layer kernel (update_fk.hpp: the two-part fp16 split on fp16 MFMA,
// optionally fused with the aggregation its output feeds) and of its bf16 instance:
//
//   H_out[e] = (residual ? H[e] : 0) + W (S[src[e]] - act(H[rev[e]])) + b        (chemprop.py:36-43,
//                                                                                 residual.py:27-28)
//   S_out[v] = reduce_{e: dst[e] = v} aact(H_out[e])                               (chemprop.py:37-39,
//                                                                                 :86 with identity)
//
// The persistent K-slice-ring ("pk") kernel that used to live here is an A/B variant of the diagnostic
// library: csrc/diag/update_pk_ring.hip.
// Supports h % 4 == 0, h <= 304, E * h / 4 < 2^31, V * h / 4 < 2^31.
#include <stdlib.h>

#include <atomic>

#include <type_traits>

#include "common.hpp"
#include "update.hpp"

namespace nt {

#ifdef NT_DIAG
// diagnostic builds only (the shipping library holds no device state): stamp sums of the fk (ABL 256)
// and fw (FW_STAMP) walks, read by nt_debug_fw_stamps
__device__ unsigned long long g_pk_stamps[10];
#endif

}  // namespace nt

// the fp32 layer kernel (two-part fp16 split)
#include "update_fk.hpp"
#ifdef NT_DIAG
#include "diag/update_fk2.hpp"  // A/B: LDS-staged output variant (NT_FK=2)
#include "diag/update_fw.hpp"   // A/B: one-wave-per-SIMD walk of the fused layer (NT_FK_FW=1)
#endif

namespace nt {
int cu_count();   // update_ps.hip
int xcd_count();  // update_ps.hip
}  // namespace nt


namespace nt {
// ------------------------------------------------------------------------------ fk launcher
namespace {
template <int RT, int CT, int ACT, int AACT, bool SUMONLY, int MAXL>
int launch_fk_t(const fk::Args& a, int grid, hipStream_t stream) {
  set_last_kernel(RT == 8 ? "update_fk_kernel: one 8-wave workgroup per CU, 128-row tiles"
                          : "update_fk_kernel: one 8-wave workgroup per CU, 64-row tiles");
  fk::update_fk_kernel<RT, CT, ACT, AACT, SUMONLY, MAXL><<<grid, fk::kThreads, 0, stream>>>(a);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

// 128-row tiles: relu layers with a sum aggregation whose act is relu / identity, or no aggregation
template <int CT>
int launch_fk_wide(const fk::Args& a, int maxl, int grid, hipStream_t stream) {
  const bool fused = a.SO != nullptr;
  const bool relu = a.act == NT_ACT_RELU;
  if (!fused) {  // plain update / dense mode: no aggregation
    if (relu) return launch_fk_t<8, CT, NT_ACT_RELU, NT_ACT_IDENTITY, true, 1>(a, grid, stream);
    if (a.act == NT_ACT_IDENTITY)
      return launch_fk_t<8, CT, NT_ACT_IDENTITY, NT_ACT_IDENTITY, true, 1>(a, grid, stream);
    return launch_fk_t<8, CT, -1, NT_ACT_IDENTITY, true, 1>(a, grid, stream);
  }
  // fused (fk_tile_rows: act = relu): scan rounds 3 cover in-degree <= 4 (molecules), 8 in-degree <= 9
  // (the non-hub nodes of hub graphs, cut at HUB_CUT_DEGREE), 16 every plan
#ifdef NT_DIAG
  {  // per-phase stamps of the config-2 instance (tools/stamps_fk.py)
    const char* e = getenv("NT_FK_ABL");
    if (e && atoi(e) == 256 && maxl <= 3 && a.aact == NT_ACT_RELU) {
      fk::update_fk_kernel<8, CT, NT_ACT_RELU, NT_ACT_RELU, true, 3, 2, 256><<<grid, fk::kThreads, 0, stream>>>(a);
      NT_LAUNCH_CHECK();
      return NT_OK;
    }
  }
#endif
  if (a.aact == NT_ACT_RELU)
    return maxl <= 3   ? launch_fk_t<8, CT, NT_ACT_RELU, NT_ACT_RELU, true, 3>(a, grid, stream)
           : maxl <= 8 ? launch_fk_t<8, CT, NT_ACT_RELU, NT_ACT_RELU, true, 8>(a, grid, stream)
                       : launch_fk_t<8, CT, NT_ACT_RELU, NT_ACT_RELU, true, 16>(a, grid, stream);
  return maxl <= 3   ? launch_fk_t<8, CT, NT_ACT_RELU, NT_ACT_IDENTITY, true, 3>(a, grid, stream)
         : maxl <= 8 ? launch_fk_t<8, CT, NT_ACT_RELU, NT_ACT_IDENTITY, true, 8>(a, grid, stream)
                     : launch_fk_t<8, CT, NT_ACT_RELU, NT_ACT_IDENTITY, true, 16>(a, grid, stream);
}

#ifdef NT_DIAG
// fk2 (64-row tiles, output staged in LDS and written during the next tile): h <= 384, any layer
template <int ACT, int AACT, bool SUMONLY, bool TABLE>
int launch_fk2_t(const fk::Args& a, int grid, hipStream_t stream) {
  fk::update_fk2_kernel<3, ACT, AACT, SUMONLY, TABLE><<<grid, fk::kThreads, 0, stream>>>(a);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

int launch_fk2(const fk::Args& a, int grid, hipStream_t stream) {
  const bool relu = a.act == NT_ACT_RELU, ident = a.act == NT_ACT_IDENTITY;
  if (a.SO == nullptr) {  // plain / dense: no aggregation
    if (relu) return launch_fk2_t<NT_ACT_RELU, NT_ACT_IDENTITY, true, false>(a, grid, stream);
    if (ident) return launch_fk2_t<NT_ACT_IDENTITY, NT_ACT_IDENTITY, true, false>(a, grid, stream);
    return launch_fk2_t<-1, NT_ACT_IDENTITY, true, false>(a, grid, stream);
  }
  const bool sum = a.reduce == NT_SUM;
#ifdef NT_DIAG
  if (relu && sum && a.aact == NT_ACT_RELU) {
    const char* e = getenv("NT_FK_ABL");
    switch (e ? atoi(e) : 0) {
#define NT_FK2_ABL_CASE(n)                                                                                  \
  case n:                                                                                                   \
    fk::update_fk2_kernel<3, NT_ACT_RELU, NT_ACT_RELU, true, true, 2, n><<<grid, fk::kThreads, 0, stream>>>(a); \
    NT_LAUNCH_CHECK();                                                                                      \
    return NT_OK;
      NT_FK2_ABL_CASE(1)
      NT_FK2_ABL_CASE(2)
      NT_FK2_ABL_CASE(6)
      NT_FK2_ABL_CASE(8)
      NT_FK2_ABL_CASE(16)
      NT_FK2_ABL_CASE(32)
      NT_FK2_ABL_CASE(64)
      NT_FK2_ABL_CASE(70)
      NT_FK2_ABL_CASE(102)
      NT_FK2_ABL_CASE(71)
      NT_FK2_ABL_CASE(24)
      NT_FK2_ABL_CASE(128)
      NT_FK2_ABL_CASE(198)
#undef NT_FK2_ABL_CASE
      default:
        break;
    }
  }
#endif
  if (relu && sum && a.aact == NT_ACT_RELU) return launch_fk2_t<NT_ACT_RELU, NT_ACT_RELU, true, true>(a, grid, stream);
  if (relu && sum && a.aact == NT_ACT_IDENTITY)
    return launch_fk2_t<NT_ACT_RELU, NT_ACT_IDENTITY, true, true>(a, grid, stream);
  return launch_fk2_t<-1, -1, false, true>(a, grid, stream);
}

#endif  // NT_DIAG

// which fp32 layer kernel runs: update_fk_kernel; diagnostic builds: NT_FK=2 selects the LDS-staged
// update_fk2_kernel for h <= 384
bool fk2_selected(int64_t h) {
#ifdef NT_DIAG
  const char* e = getenv("NT_FK");
  return e && e[0] == '2' && h <= fk::kFk2MaxH;
#else
  (void)h;
  return false;
#endif
}

// Fused relu / sum layers given a plan of <= 64-row tiles (h <= 320): two independent 4-wave
// workgroups per CU (5 column tiles per wave, the bias in LDS), so one workgroup's epilogue runs
// beside the other's K loop instead of every CU's epilogue bursting at once.  Faster than the
// 128-row walk on small batches (config 2: 115 vs 125 us), slower on large ones (qm9-32k: 905 vs
// 894, polymer-16: 720 vs 691): the caller picks the plan rows (_engine.NW4_MAX_EDGES).
// NT_FK_NW=8 turns it off, NT_FK_NW=4 makes it the tile capacity (tests).
// NT_FK_NW (A/B, read once per process): 8 = never the two-workgroup walk, 4 = always its 64-row plans
int fk_nw_env() {
  static const int v = [] {
    const char* e = getenv("NT_FK_NW");
    return e ? atoi(e) : 0;
  }();
  return v;
}
bool fk_nw4(int64_t h, bool fused, int act, int reduce, int aact) {
  return fk_nw_env() != 8 && fused && act == NT_ACT_RELU && reduce == NT_SUM &&
         (aact == NT_ACT_RELU || aact == NT_ACT_IDENTITY) && fk::nt_for(h) <= 20;
}
bool fk_nw4_forced() { return fk_nw_env() == 4; }

template <int AACT, int MAXL>
int launch_fk_nw4_t(const fk::Args& a, int grid, hipStream_t stream) {
  set_last_kernel("update_fk_kernel: two 4-wave workgroups per CU, 64-row tiles");
  fk::update_fk_kernel<4, 5, NT_ACT_RELU, AACT, true, MAXL, 2, 0, 0, 4><<<grid, 256, 0, stream>>>(a);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

int launch_fk_nw4(const fk::Args& a, int maxl, int grid, hipStream_t stream) {
  if (a.aact == NT_ACT_RELU)
    return maxl <= 3   ? launch_fk_nw4_t<NT_ACT_RELU, 3>(a, grid, stream)
           : maxl <= 8 ? launch_fk_nw4_t<NT_ACT_RELU, 8>(a, grid, stream)
                       : launch_fk_nw4_t<NT_ACT_RELU, 16>(a, grid, stream);
  return maxl <= 3   ? launch_fk_nw4_t<NT_ACT_IDENTITY, 3>(a, grid, stream)
         : maxl <= 8 ? launch_fk_nw4_t<NT_ACT_IDENTITY, 8>(a, grid, stream)
                     : launch_fk_nw4_t<NT_ACT_IDENTITY, 16>(a, grid, stream);
}

#ifdef NT_DIAG
// A/B switch: NT_FK_FW=1 / 0 (read once per process) selects update_fw_kernel where it applies;
// nt_debug_set_fw overrides it (tests and kernel benches switch within one process)
int g_fw_override = -1;
bool fw_selected() {
  static const int v = [] {
    const char* e = getenv("NT_FK_FW");
    return e && e[0] == '1' ? 1 : 0;
  }();
  return (g_fw_override >= 0 ? g_fw_override : v) != 0;
}

template <int AACT, int MAXL>
int launch_fw_t(const fk::Args& a, int grid, hipStream_t stream) {
  set_last_kernel("update_fw_kernel: one 4-wave workgroup per CU (one wave per SIMD), 128-row tiles");
  fw::update_fw_kernel<5, 0, NT_ACT_RELU, AACT, MAXL><<<grid, fw::kThreads, 0, stream>>>(a);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

template <int AACT, int MAXL>
int launch_fwb_t(const fk::Args& a, int grid, hipStream_t stream) {
  set_last_kernel("update_fw_kernel (bf16): one 4-wave workgroup per CU (one wave per SIMD), 128-row tiles");
  fw::update_fw_kernel<8, 1, NT_ACT_RELU, AACT, MAXL><<<grid, fw::kThreads, 0, stream>>>(a);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

int launch_fwb(const fk::Args& a, int maxl, int grid, hipStream_t stream) {
  if (a.aact == NT_ACT_RELU)
    return maxl <= 3   ? launch_fwb_t<NT_ACT_RELU, 3>(a, grid, stream)
           : maxl <= 8 ? launch_fwb_t<NT_ACT_RELU, 8>(a, grid, stream)
                       : launch_fwb_t<NT_ACT_RELU, 16>(a, grid, stream);
  return maxl <= 3   ? launch_fwb_t<NT_ACT_IDENTITY, 3>(a, grid, stream)
         : maxl <= 8 ? launch_fwb_t<NT_ACT_IDENTITY, 8>(a, grid, stream)
                     : launch_fwb_t<NT_ACT_IDENTITY, 16>(a, grid, stream);
}

int launch_fw(const fk::Args& a, int maxl, int grid, hipStream_t stream) {
  if (a.aact == NT_ACT_RELU)
    return maxl <= 3   ? launch_fw_t<NT_ACT_RELU, 3>(a, grid, stream)
           : maxl <= 8 ? launch_fw_t<NT_ACT_RELU, 8>(a, grid, stream)
                       : launch_fw_t<NT_ACT_RELU, 16>(a, grid, stream);
  return maxl <= 3   ? launch_fw_t<NT_ACT_IDENTITY, 3>(a, grid, stream)
         : maxl <= 8 ? launch_fw_t<NT_ACT_IDENTITY, 8>(a, grid, stream)
                     : launch_fw_t<NT_ACT_IDENTITY, 16>(a, grid, stream);
}

#endif  // NT_DIAG

// 64-row tiles: every other combination (any reduce, any aggregation act) and h > 384
template <int CT>
int launch_fk_narrow(const fk::Args& a, int maxl, int grid, hipStream_t stream) {
  const bool fused = a.SO != nullptr;
  const bool relu = a.act == NT_ACT_RELU;
  const bool fast = !fused || (a.reduce == NT_SUM && (a.aact == NT_ACT_RELU || a.aact == NT_ACT_IDENTITY));
  if (fast) {
    if (!fused)
      return relu ? launch_fk_t<4, CT, NT_ACT_RELU, NT_ACT_IDENTITY, true, 1>(a, grid, stream)
                  : launch_fk_t<4, CT, -1, NT_ACT_IDENTITY, true, 1>(a, grid, stream);
    if (a.aact == NT_ACT_RELU)
      return relu ? launch_fk_t<4, CT, NT_ACT_RELU, NT_ACT_RELU, true, 16>(a, grid, stream)
                  : launch_fk_t<4, CT, -1, NT_ACT_RELU, true, 16>(a, grid, stream);
    return relu ? launch_fk_t<4, CT, NT_ACT_RELU, NT_ACT_IDENTITY, true, 16>(a, grid, stream)
                : launch_fk_t<4, CT, -1, NT_ACT_IDENTITY, true, 16>(a, grid, stream);
  }
  (void)maxl;
  return launch_fk_t<4, CT, -1, -1, false, 16>(a, grid, stream);
}
}  // namespace

// Row capacity of the fk tiles for a layer: 128 for h <= 384 with act = relu and a sum aggregation
// whose act is relu / identity, or with no aggregation (fused < 0); else 64.  (The other variants
// need more registers than two waves per SIMD hold at 128 rows.)
int fk_tile_rows(int64_t h, int act, int reduce, int aact, bool fused) {
  if (fk2_selected(h) || (fk_nw4_forced() && fk_nw4(h, fused, act, reduce, aact))) return 64;
  const bool wide_ok =
      !fused || (act == NT_ACT_RELU && reduce == NT_SUM && (aact == NT_ACT_RELU || aact == NT_ACT_IDENTITY));
  return (fk::nt_for(h) <= 24 && wide_ok) ? 128 : 64;
}

// the one-wave-per-SIMD walk for this fused layer (A/B switch fw_selected): fp32 257 <= h <= 320,
// bf16 449 <= h <= 512 (eight column tiles per wave), relu layers with a relu / identity sum
bool fw_active(int64_t h, int dtype, int act, int reduce, int aact) {
#ifdef NT_DIAG
  if (!fw_selected() || act != NT_ACT_RELU || reduce != NT_SUM || !(aact == NT_ACT_RELU || aact == NT_ACT_IDENTITY))
    return false;
  const int nt = fk::nt_for(h);
  return dtype == NT_BF16 ? (h % 8 == 0 && nt > 28 && nt <= fw::kMaxNTb) : (nt > 16 && nt <= fw::kMaxNT);
#else
  (void)h, (void)dtype, (void)act, (void)reduce, (void)aact;
  return false;  // the fw walk is an A/B of the diagnostic library only
#endif
}

int launch_update_fk(const UpdateArgs& u, const void* Wimg, const float* amax_in, float* amax_out,
                     const int32_t* tile_ptr, int64_t ntiles, int tile_rows, int max_in_degree,
                     const void* row_table, int reduce, int aact, float aalpha, float* S_out) {
  const bool fused = tile_ptr != nullptr;
  NT_REQUIRE(fused == (S_out != nullptr), NT_EINVAL, "S_out must be given exactly with a tile plan");
  NT_REQUIRE(!fused || row_table, NT_EINVAL, "fp32 fused mode needs the row table (nt_dmpnn_row_table)");
  NT_REQUIRE(amax_in != nullptr, NT_EINVAL, "fp32 update needs amax_in (max|H|, max|S| on the device)");
  NT_REQUIRE(u.h % 4 == 0, NT_EUNSUPPORTED, "fp32 update needs h % 4 == 0");
  NT_REQUIRE((u.E * u.h) / 4 < (int64_t(1) << 31) && (u.V * u.h) / 4 < (int64_t(1) << 31),
             NT_EUNSUPPORTED, "fp32 update: E*h and V*h must stay below 2^33");
  const int cap = fk_tile_rows(u.h, u.act, reduce, aact, fused);
  NT_REQUIRE(!fused || (tile_rows >= 1 && tile_rows <= cap), NT_EUNSUPPORTED,
             "tile plan rows exceed nt_dmpnn_fused_tile_rows for this layer");
  NT_REQUIRE(!fused || (max_in_degree >= 0 && max_in_degree <= 32), NT_EUNSUPPORTED,
             "fused aggregation needs max_in_degree <= 32");
  fk::Args a;
  a.H = u.H;
  a.S = u.S;
  a.src = u.src;
  a.rev = u.rev;
  a.Wimg = (const char*)Wimg;
  a.bias = u.b;
  a.amax_in = amax_in;
  a.amax_out = amax_out;
  a.V = u.V;
  a.E = u.E;
  a.h = (int)u.h;
  a.hv = (int)(u.h / 4);
  {
    const int64_t ldi = u.ldi ? u.ldi : u.h, ldo = u.ldo ? u.ldo : u.h;
    NT_REQUIRE(ldi >= u.h && ldo >= u.h && ldi % 4 == 0 && ldo % 4 == 0, NT_EINVAL,
               "row pitches must be >= h and multiples of 4");
    NT_REQUIRE((u.E * ldi) / 4 < (int64_t(1) << 31) && (u.V * ldi) / 4 < (int64_t(1) << 31) &&
                   (u.E * ldo) / 4 < (int64_t(1) << 31) && (u.V * ldo) / 4 < (int64_t(1) << 31),
               NT_EUNSUPPORTED, "fp32 update: E*ld and V*ld must stay below 2^33");
    a.ldiv = a.ldic = (int)(ldi / 4);
    a.ldoc = (int)(ldo / 4);
#ifdef NT_DIAG
    NT_REQUIRE((ldi == u.h && ldo == u.h && u.S_part == nullptr) ||
                   !(fk2_selected(u.h) || fw_active(u.h, NT_F32, u.act, reduce, aact)),
               NT_EUNSUPPORTED, "diagnostic walks take dense rows and no hub partials only");
#endif
  }
  // an even number of k-steps, at least four, per tile (update_fk_kernel runs two steps per inner
  // trip and gathers three steps ahead, within the next tile at most); a k-step past the image reads
  // zeros (buffer range) and masked-off pieces
  a.KS = fk::ks_for(u.h) < 4 ? 4 : (fk::ks_for(u.h) + 1) / 2 * 2;
  a.NT = fk::nt_for(u.h);
  a.residual = u.residual;
  a.act = u.act;
  a.alpha = u.alpha;
  a.tile_ptr = tile_ptr;
  a.rows = fused ? (const int4*)row_table : nullptr;
  a.reduce = reduce;
  a.aact = aact;
  a.aalpha = aalpha;
  a.O = u.H_out;
  a.SO = S_out;
  a.SP = u.S_part;
  a.nxcd = xcd_count();
  {
    // timing experiments only, read once per process: NT_FK_STAGGER (start delay of half the grid)
    static const int stagger = [] {
      const char* e = getenv("NT_FK_STAGGER");
      return e ? atoi(e) : 0;
    }();
    a.stagger = stagger;
#ifdef NT_DIAG
    static const int rtabl = [] {
      const char* e = getenv("NT_FK_RTABL");
      return e ? atoi(e) : 0;
    }();
    a.rtabl = rtabl;
#endif
  }
  a.ntiles = fused ? (int)ntiles : (int)((u.E + cap - 1) / cap);
  if (a.ntiles == 0) return NT_OK;
  const int grid = a.ntiles < cu_count() ? a.ntiles : cu_count();
  const int maxl = max_in_degree - 1;  // scan rounds needed within a 16-row tile
#ifdef NT_DIAG
  if (fk2_selected(u.h)) {
    a.nchunks = 1;
    return launch_fk2(a, grid, u.stream);
  }
#endif
#ifdef NT_DIAG
  if (fused && fw_active(u.h, NT_F32, u.act, reduce, aact)) {
    a.nchunks = 1;
    return launch_fw(a, maxl, grid, u.stream);
  }
#endif
  if (fused && tile_rows <= 64 && fk_nw4(u.h, true, u.act, reduce, aact)) {
    a.nchunks = 1;
    const int g4 = a.ntiles < 2 * cu_count() ? a.ntiles : 2 * cu_count();
    return launch_fk_nw4(a, maxl, g4, u.stream);
  }
  // up to 3 column tiles per wave (NT <= 24, one chunk); waves past NT skip theirs at run time
  if (cap == 128) {
    a.nchunks = 1;
    return launch_fk_wide<3>(a, maxl, grid, u.stream);
  }
  if (a.NT <= 24) {
    a.nchunks = 1;
    return launch_fk_narrow<3>(a, maxl, grid, u.stream);
  }
  a.nchunks = (a.NT + 31) / 32;
  return launch_fk_narrow<4>(a, maxl, grid, u.stream);
}

// ------------------------------------------------------------------------------ bf16 on the fk skeleton
// bf16 storage (PREC = 1): the same persistent kernel with 128-row tiles and 4 column tiles per wave
// (h <= 512), one bf16 MFMA per (row tile, column tile) and k-step, no split and no scales; W is the
// plain bf16 fragment image (nt_dmpnn_pack_weight, bf16).
namespace {
template <int ACT, int AACT, bool SUMONLY, int MAXL>
int launch_fkb_t(const fk::Args& a, int grid, hipStream_t stream) {
  set_last_kernel("update_fk_kernel (bf16): one 8-wave workgroup per CU, 128-row tiles");
  fk::update_fk_kernel<8, 4, ACT, AACT, SUMONLY, MAXL, 2, 0, 1><<<grid, fk::kThreads, 0, stream>>>(a);
  NT_LAUNCH_CHECK();
  return NT_OK;
}
// A/B (NT_BF16_KERNEL=fk4): 64-row bf16 tiles walked by two 4-wave workgroups per CU, 8 column tiles
// per wave (h <= 512), the bias in LDS
template <int AACT, int MAXL>
int launch_fkb4_t(const fk::Args& a, int grid, hipStream_t stream) {
  set_last_kernel("update_fk_kernel (bf16): two 4-wave workgroups per CU, 64-row tiles");
  fk::update_fk_kernel<4, 8, NT_ACT_RELU, AACT, true, MAXL, 2, 0, 1, 4><<<grid, 256, 0, stream>>>(a);
  NT_LAUNCH_CHECK();
  return NT_OK;
}
}  // namespace

bool fkb_supported(int64_t h) { return h % 8 == 0 && h >= 8 && h <= 512; }

// NT_BF16_KERNEL (A/B, read once per process): 0 = the 64-row bf16 kernel (default), 1 = "fk" (the
// fk skeleton, 128-row tiles), 2 = "fk4" (its two-workgroup 64-row walk)
int bf16_kernel_env() {
  static const int v = [] {
    const char* e = getenv("NT_BF16_KERNEL");
    if (!(e && e[0] == 'f' && e[1] == 'k')) return 0;
    return e[2] == '4' ? 2 : 1;
  }();
  return v;
}

int launch_update_fk_bf16(const UpdateArgs& u, const void* Wimg, const int32_t* tile_ptr, int64_t ntiles,
                          int tile_rows, int max_in_degree, const void* row_table, int reduce, int aact,
                          float aalpha, void* S_out) {
  const bool fused = tile_ptr != nullptr;
  NT_REQUIRE(fkb_supported(u.h), NT_EUNSUPPORTED, "bf16 layer kernel needs h % 8 == 0 and h <= 512");
  NT_REQUIRE(fused == (S_out != nullptr), NT_EINVAL, "S_out must be given exactly with a tile plan");
  NT_REQUIRE(!fused || row_table, NT_EINVAL, "bf16 fused mode needs the row table (nt_dmpnn_row_table)");
  NT_REQUIRE(!fused || (tile_rows >= 1 && tile_rows <= 128), NT_EUNSUPPORTED, "bf16 tiles hold at most 128 rows");
  NT_REQUIRE(!fused || (max_in_degree >= 0 && max_in_degree <= 32), NT_EUNSUPPORTED,
             "fused aggregation needs max_in_degree <= 32");
  NT_REQUIRE((u.E * u.h) / 4 < (int64_t(1) << 31) && (u.V * u.h) / 4 < (int64_t(1) << 31), NT_EUNSUPPORTED,
             "bf16 update: E*h and V*h must stay below 2^33");
  fk::Args a;
  a.H = u.H;
  a.S = u.S;
  a.src = u.src;
  a.rev = u.rev;
  a.Wimg = (const char*)Wimg;
  a.bias = u.b;
  a.amax_in = nullptr;
  a.amax_out = nullptr;
  a.V = u.V;
  a.E = u.E;
  a.h = (int)u.h;
  a.hv = (int)(u.h / 8);  // 16-B gather pieces of 8 bf16
  a.ldiv = a.hv;
  a.ldic = a.ldoc = (int)(u.h / 4);
  a.KS = fk::ks_for(u.h) < 4 ? 4 : (fk::ks_for(u.h) + 1) / 2 * 2;
  a.NT = fk::nt_for(u.h);
  a.nchunks = 1;
  a.residual = u.residual;
  a.act = u.act;
  a.alpha = u.alpha;
  a.tile_ptr = tile_ptr;
  a.rows = fused ? (const int4*)row_table : nullptr;
  a.reduce = reduce;
  a.aact = aact;
  a.aalpha = aalpha;
  a.O = u.H_out;
  a.SO = (float*)S_out;
  a.nxcd = xcd_count();
  a.stagger = 0;
  a.ntiles = fused ? (int)ntiles : (int)((u.E + 127) / 128);
  if (a.ntiles == 0) return NT_OK;
  const int grid = a.ntiles < cu_count() ? a.ntiles : cu_count();
  const bool relu = u.act == NT_ACT_RELU;
  if (!fused) {
    if (relu) return launch_fkb_t<NT_ACT_RELU, NT_ACT_IDENTITY, true, 1>(a, grid, u.stream);
    if (u.act == NT_ACT_IDENTITY) return launch_fkb_t<NT_ACT_IDENTITY, NT_ACT_IDENTITY, true, 1>(a, grid, u.stream);
    return launch_fkb_t<-1, NT_ACT_IDENTITY, true, 1>(a, grid, u.stream);
  }
  const int maxl = max_in_degree - 1;
#ifdef NT_DIAG
  if (fw_active(u.h, NT_BF16, u.act, reduce, aact)) return launch_fwb(a, maxl, grid, u.stream);
#endif
  {
    if (bf16_kernel_env() == 2 && tile_rows <= 64 && relu && reduce == NT_SUM &&
        (aact == NT_ACT_RELU || aact == NT_ACT_IDENTITY)) {
      const int g4 = a.ntiles < 2 * cu_count() ? a.ntiles : 2 * cu_count();
      if (aact == NT_ACT_RELU)
        return maxl <= 3 ? launch_fkb4_t<NT_ACT_RELU, 3>(a, g4, u.stream)
                         : launch_fkb4_t<NT_ACT_RELU, 16>(a, g4, u.stream);
      return maxl <= 3 ? launch_fkb4_t<NT_ACT_IDENTITY, 3>(a, g4, u.stream)
                       : launch_fkb4_t<NT_ACT_IDENTITY, 16>(a, g4, u.stream);
    }
  }
  if (relu && reduce == NT_SUM && aact == NT_ACT_RELU)
    return maxl <= 3   ? launch_fkb_t<NT_ACT_RELU, NT_ACT_RELU, true, 3>(a, grid, u.stream)
           : maxl <= 8 ? launch_fkb_t<NT_ACT_RELU, NT_ACT_RELU, true, 8>(a, grid, u.stream)
                       : launch_fkb_t<NT_ACT_RELU, NT_ACT_RELU, true, 16>(a, grid, u.stream);
  if (relu && reduce == NT_SUM && aact == NT_ACT_IDENTITY)
    return maxl <= 3   ? launch_fkb_t<NT_ACT_RELU, NT_ACT_IDENTITY, true, 3>(a, grid, u.stream)
           : maxl <= 8 ? launch_fkb_t<NT_ACT_RELU, NT_ACT_IDENTITY, true, 8>(a, grid, u.stream)
                       : launch_fkb_t<NT_ACT_RELU, NT_ACT_IDENTITY, true, 16>(a, grid, u.stream);
  return launch_fkb_t<-1, -1, false, 16>(a, grid, u.stream);
}

int fk_pack(const float* W, int64_t nlayers, int64_t h, int64_t w_stride, int64_t img_stride, void* img,
            hipStream_t stream) {
  const int KS = fk::ks_for(h), NT = fk::nt_for(h);
  const int64_t slots = (int64_t)KS * NT * 2 * 64;
  fk::pack_fk_scale_kernel<<<dim3(fk::kScaleParts, (unsigned)nlayers), 256, 0, stream>>>(W, h, w_stride, img_stride,
                                                                                         (char*)img);
  NT_LAUNCH_CHECK();
  dim3 grid((unsigned)((slots + 255) / 256), (unsigned)nlayers);
  fk::pack_fk_kernel<<<grid, 256, 0, stream>>>(W, h, KS, NT, w_stride, img_stride, (char*)img);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

int fk_pack_multi(const float* const* W, int64_t nlayers, int64_t h, char* const* img, char* const* imgT,
                  hipStream_t stream) {
  const int KS = fk::ks_for(h), NT = fk::nt_for(h);
  const int64_t slots = (int64_t)KS * NT * 2 * 64;
  fk::PackPtrs p;
  for (int l = 0; l < fk::kPackMax; ++l) {
    p.W[l] = l < nlayers ? W[l] : nullptr;
    p.img[l] = l < nlayers ? img[l] : nullptr;
    p.imgT[l] = (l < nlayers && imgT) ? imgT[l] : nullptr;
  }
  fk::pack_fk_scale_multi<<<dim3(fk::kScaleParts, (unsigned)nlayers), 256, 0, stream>>>(p, h);
  NT_LAUNCH_CHECK();
  fk::pack_fk_multi<<<dim3((unsigned)((slots + 255) / 256), (unsigned)nlayers), 256, 0, stream>>>(p, h, KS, NT);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

int fk_row_table(const int32_t* perm, const int32_t* dsts, const int64_t* src, const int64_t* rev, int64_t V,
                 int64_t E, void* out, hipStream_t stream) {
  if (E <= 0) return NT_OK;
  fk::row_table_kernel<<<grid_for(E, 256, 256 * 16), 256, 0, stream>>>(perm, dsts, src, rev, V, E, (int4*)out);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

int fk_absmax(const float* X, int64_t n, float* out, hipStream_t stream) {
  if (n <= 0) return NT_OK;
  fk::absmax_kernel<<<grid_for(n / 4 + 1, 256, 256 * 8), 256, 0, stream>>>(X, n, out);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

// Split scales for the C ABI entry points that carry no amax (nt_dmpnn_update, nt_dmpnn_dense_matmul
// without amax_in): the caller's 2-float device workspace, zeroed and filled on the call's stream, so
// every use is ordered by the stream like the layer kernel that reads it.
int amax_fill(float* ws, const float* H, int64_t nh, const float* S, int64_t ns, hipStream_t stream) {
  NT_HIP(hipMemsetAsync(ws, 0, 2 * sizeof(float), stream));
  int rc = H ? fk_absmax(H, nh, ws, stream) : NT_OK;
  if (rc == NT_OK && S) rc = fk_absmax(S, ns, ws + 1, stream);
  return rc;
}

}  // namespace nt

#if defined(NT_DIAG) && FW_STAMP
// A/B builds only (FW_STAMP): read and reset the fw kernel's stamp sums (6 values)
extern "C" __attribute__((visibility("default"))) int nt_debug_fw_stamps(unsigned long long* out6) {
  if (hipMemcpyFromSymbol(out6, HIP_SYMBOL(nt::g_pk_stamps), 6 * sizeof(unsigned long long), 0,
                          hipMemcpyDeviceToHost) != hipSuccess)
    return 2;
  unsigned long long z[10] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(nt::g_pk_stamps), z, sizeof(z), 0, hipMemcpyHostToDevice) == hipSuccess ? 0 : 2;
}
#endif

#ifdef NT_DIAG
// Debug-only (diagnostic library, not part of include/notorch_amd.h): select the fp32 fused layer
// walk (-1: the default, 0: update_fk_kernel, 1: update_fw_kernel where it applies)
extern "C" __attribute__((visibility("default"))) int nt_debug_set_fw(int v) {
  nt::g_fw_override = v;
  return 0;
}
#endif

// Fused D-MPNN layer update, LDS-DMA streamed fp32 MFMA kernel (default for h % 4 == 0, h <= 512):
//
//   H_out[e] = (residual ? H[e] : 0) + W (S[src[e]] - act(H[rev[e]])) + b     (chemprop.py:36-43,
//                                                                               residual.py:27-28)
// Structure (one workgroup = 4 waves = 64 edges x all h output columns):
//   * K advances in 16-deep chunks through a 2-slot LDS ring.  Every load of the K loop is an
//     LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave-instruction, per-lane source address):
//       - S rows:  64 rows x 64 B  (row r of the tile gathers S[src[e0+r]])    4 instructions
//       - H rows:  64 rows x 64 B  (row r gathers H[rev[e0+r]])                 4 instructions
//       - W tiles: NT x 1 KiB from the packed fragment image (L2-resident)     NT instructions
//     Chunk k+1 is issued at the top of step k and retired by the barrier that ends step k, so
//     its latency hides behind step k's MFMAs.  No VGPR-destination load exists in the loop, so
//     the compiler's waitcnt placement cannot drain or sink the stream.
//   * Wave w owns rows 16w..16w+15 and ALL NT column tiles (acc = 4*NT VGPRs); the W tiles in
//     LDS are shared by the 4 waves (4x reuse).  The A fragment a = S - act(H) is formed in
//     registers from two ds_read_b128 (row validity / k < h masks applied here).
//   * Epilogue: accumulators staged per wave through LDS in column groups of <= 10 tiles, then
//     bias + residual + store as 16-B row pieces.
// Roofline: MFMA-bound (2 h^2 flop per edge vs ~16 h bytes per edge, 51 flop/B at h = 300).
// A/B-only kernel: compiled into the diagnostic library (make DIAG=1) only.
#ifdef NT_DIAG
#include "common.hpp"
#include "update.hpp"

#include <type_traits>

namespace nt {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

constexpr int kRows = 64;     // edges per workgroup
constexpr int kEpiGroup = 10; // column tiles per epilogue group

template <int NT>
struct GldsLds {
  static constexpr int kS = 0;                       // [64][16] floats
  static constexpr int kH = kRows * 16;              // [64][16] floats
  static constexpr int kB = 2 * kRows * 16;          // [NT][64 lanes][4] floats
  static constexpr int kSlot = kB + NT * 256;        // floats per ring slot
  static constexpr int kRing = 2 * kSlot;
  static constexpr int kEpiTiles = NT < kEpiGroup ? NT : kEpiGroup;
  static constexpr int kLDE = 16 * kEpiTiles + 4;    // == 4 (mod 8): conflict-free C writes
  static constexpr int kEpi = 4 * 16 * kLDE;
  static constexpr int kIdx = kRing > kEpi ? kRing : kEpi;  // then 2 x 64 int64 row offsets
  static constexpr int kFloats = kIdx + 4 * kRows;
};

__device__ __forceinline__ void glds16(const void* g, float* l) {
  __builtin_amdgcn_global_load_lds((gbl_void*)g, (lds_void*)l, 16, 0, 0);
}

template <int NT, int ACT>
__global__ void __launch_bounds__(256, 2) update_glds_kernel(
    const float4* __restrict__ H4, const float4* __restrict__ S4, const int64_t* __restrict__ src,
    const int64_t* __restrict__ rev, const float4* __restrict__ Wp, const float4* __restrict__ b4,
    int64_t V, int64_t E, int hv, int KB, int residual, int act, float alpha,
    float4* __restrict__ O4) {
  using L = GldsLds<NT>;
  // ONE __shared__ array for everything: a second __shared__ object makes hipcc wait vmcnt(0)
  // (drain the LDS-DMA stream) before the first ds_read of every step.
  __shared__ __attribute__((aligned(16))) float smem[L::kFloats];
  int64_t* s_src = reinterpret_cast<int64_t*>(smem + L::kIdx);
  int64_t* s_rev = s_src + kRows;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (scalar) index
  const int64_t e0 = (int64_t)blockIdx.x * kRows;

  if (tid < kRows) {
    const int64_t e = e0 + tid;
    int64_t s = -1, q = -1;
    if (e < E) {
      s = src[e];
      q = rev[e];
      s = (s >= 0 && s < V) ? s * hv : -1;  // float4 row offsets, -1 = invalid (zero row)
      q = (q >= 0 && q < E) ? q * hv : -1;
    }
    s_src[tid] = s;
    s_rev[tid] = q;
  }
  __syncthreads();

  // ---- LDS-DMA roles: this lane gathers piece (lane & 3) of tile row 16*wave + lane/4 ----
  const int lrow = 16 * wave + (lane >> 2), lpiece = lane & 3;
  const int64_t ls = s_src[lrow], lq = s_rev[lrow];
  const float4* s_row = S4 + (ls >= 0 ? ls : 0);  // invalid rows read row 0, masked at use
  const float4* h_row = H4 + (lq >= 0 ? lq : 0);
  auto issue_chunk = [&](int kb) {
    float* slot = smem + (kb & 1) * L::kSlot;
    int c = 4 * kb + lpiece;
    c = c < hv ? c : hv - 1;  // columns past h read a valid piece, masked at use
    glds16(s_row + c, slot + L::kS + 16 * 16 * wave);
    glds16(h_row + c, slot + L::kH + 16 * 16 * wave);
    const float4* wk = Wp + (int64_t)kb * NT * 64 + lane;
    for (int t = wave; t < NT; t += 4) glds16(wk + t * 64, slot + L::kB + 256 * t);
  };

  // ---- MFMA roles: this lane's A fragment is row 16*wave + (lane & 15), k-piece lane >> 4 ----
  const int frow = 16 * wave + (lane & 15), fg = lane >> 4;
  const bool fs_ok = s_src[frow] >= 0, fq_ok = s_rev[frow] >= 0;

  f32x4 acc[NT];
#pragma unroll
  for (int ct = 0; ct < NT; ++ct) acc[ct] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto mfma_pair = [&](int ct, const float4& a, const float4& b0, const float4& b1) {
    acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b0.x, acc[ct], 0, 0, 0);
    acc[ct + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b1.x, acc[ct + 1], 0, 0, 0);
    acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b0.y, acc[ct], 0, 0, 0);
    acc[ct + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b1.y, acc[ct + 1], 0, 0, 0);
    acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b0.z, acc[ct], 0, 0, 0);
    acc[ct + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b1.z, acc[ct + 1], 0, 0, 0);
    acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b0.w, acc[ct], 0, 0, 0);
    acc[ct + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b1.w, acc[ct + 1], 0, 0, 0);
  };
  auto mfma_one = [&](int ct, const float4& a, const float4& b0) {
    acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b0.x, acc[ct], 0, 0, 0);
    acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b0.y, acc[ct], 0, 0, 0);
    acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b0.z, acc[ct], 0, 0, 0);
    acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b0.w, acc[ct], 0, 0, 0);
  };
  auto make_a = [&](int kb, const float4& sv, const float4& hq) {
    const bool kin = 4 * kb + fg < hv;
    const float4 mq = act4_t<ACT>(hq, act, alpha);  // branch-free masking (selects only)
    const bool use_s = kin && fs_ok, use_q = kin && fq_ok;
    float4 a;
    a.x = (use_s ? sv.x : 0.f) - (use_q ? mq.x : 0.f);
    a.y = (use_s ? sv.y : 0.f) - (use_q ? mq.y : 0.f);
    a.z = (use_s ? sv.z : 0.f) - (use_q ? mq.z : 0.f);
    a.w = (use_s ? sv.w : 0.f) - (use_q ? mq.w : 0.f);
    return a;
  };

  issue_chunk(0);
  __syncthreads();
  for (int kb = 0; kb < KB; ++kb) {
    const float* slot = smem + (kb & 1) * L::kSlot;
    const float4 sv = *reinterpret_cast<const float4*>(slot + L::kS + frow * 16 + 4 * fg);
    const float4 hq = *reinterpret_cast<const float4*>(slot + L::kH + frow * 16 + 4 * fg);
    const float4* bl = reinterpret_cast<const float4*>(slot + L::kB) + lane;
    if constexpr (NT <= 24) {
      // Read every fragment of this step BEFORE issuing the next chunk's LDS-DMA: hipcc cannot
      // prove the DMA into the other slot does not alias these reads and would otherwise put a
      // vmcnt(0) (a full drain of the prefetch) in front of them.
      float4 bf[NT];
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) bf[ct] = bl[64 * ct];
      if (kb + 1 < KB) issue_chunk(kb + 1);
      const float4 a = make_a(kb, sv, hq);
#pragma unroll
      for (int ct = 0; ct + 1 < NT; ct += 2) mfma_pair(ct, a, bf[ct], bf[ct + 1]);
      if constexpr (NT & 1) mfma_one(NT - 1, a, bf[NT - 1]);
    } else {
      if (kb + 1 < KB) issue_chunk(kb + 1);
      const float4 a = make_a(kb, sv, hq);
#pragma unroll
      for (int ct = 0; ct + 1 < NT; ct += 2) mfma_pair(ct, a, bl[64 * ct], bl[64 * (ct + 1)]);
      if constexpr (NT & 1) mfma_one(NT - 1, a, bl[64 * (NT - 1)]);
    }
    // keep every MFMA of this step above the barrier: MFMAs touch no memory, so without this
    // fence the scheduler hoists the barrier (and its vmcnt(0) on the just-issued DMA) over them.
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();  // retires chunk kb+1's LDS-DMA (vmcnt(0)) and this step's ring reads
  }

  // ---- epilogue: column groups of <= kEpiGroup tiles through a wave-private LDS slab ----
  float* slab = smem + wave * 16 * L::kLDE;
#pragma unroll
  for (int g0 = 0; g0 < NT; g0 += kEpiGroup) {
    constexpr int kG = L::kEpiTiles;
#pragma unroll
    for (int i = 0; i < kG; ++i) {
      const int ct = g0 + i;
      if (ct < NT) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          slab[(4 * (lane >> 4) + j) * L::kLDE + 16 * i + (lane & 15)] = acc[ct][j];
      }
    }
    __syncthreads();
    const int ntiles = (NT - g0) < kG ? (NT - g0) : kG;
    const int nc4 = ntiles * 4;
    for (int i = lane; i < 16 * nc4; i += 64) {
      const int r = i / nc4, c = i - r * nc4;
      const int64_t e = e0 + 16 * wave + r;
      const int col4 = 4 * g0 + c;
      if (e < E && col4 < hv) {
        float4 o = *reinterpret_cast<const float4*>(&slab[r * L::kLDE + 4 * c]);
        if (b4) o = o + b4[col4];
        if (residual) o = H4[e * hv + col4] + o;
        O4[e * hv + col4] = o;
      }
    }
    __syncthreads();
  }
}

template <int NT, int ACT>
int launch_nt(const UpdateArgs& a) {
  const int64_t grid = (a.E + kRows - 1) / kRows;
  NT_REQUIRE(grid < (int64_t(1) << 31), NT_EINVAL, "too many edges");
  update_glds_kernel<NT, ACT><<<(unsigned)grid, 256, 0, a.stream>>>(
      (const float4*)a.H, (const float4*)a.S, a.src, a.rev, (const float4*)a.Wp,
      (const float4*)a.b, a.V, a.E, (int)(a.h / 4), a.KB, a.residual, a.act, a.alpha,
      (float4*)a.H_out);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

template <int ACT, int... NTs>
int dispatch_nt(const UpdateArgs& a, std::integer_sequence<int, NTs...>) {
  int rc = NT_EUNSUPPORTED;
  bool done = false;
  ((a.NT == NTs + 1 ? (rc = launch_nt<NTs + 1, ACT>(a), done = true) : false), ...);
  if (!done) set_error("nt_dmpnn_update: no LDS-DMA kernel for this hidden size");
  return rc;
}


// ------------------------------------------------------------------------------------------
// Ring variant: S/H pieces 2 chunks ahead (3-slot ring), W tiles 1 chunk ahead (2-slot ring).
// Every ring slot is its OWN __shared__ array and the K loop is unrolled over the ring period
// (lcm(3,2) = 6 steps), so each step's slots are compile-time objects: hipcc then knows the
// outstanding LDS-DMA targets other objects and puts no vmcnt wait in front of the reads.  The
// step ends with a counted `s_waitcnt vmcnt(2)` (only this step's two S/H DMAs may stay in flight)
// and a raw s_barrier (a __syncthreads() would drain the prefetch with vmcnt(0)).
// ------------------------------------------------------------------------------------------
constexpr int kRingEpiG = 3;  // epilogue column group: 2 waves x 16 x (16*3+4) floats fit 8 KiB

template <int NT, int ACT>
__global__ void __launch_bounds__(256, 2) update_ring_kernel(
    const float4* __restrict__ H4, const float4* __restrict__ S4, const int64_t* __restrict__ src,
    const int64_t* __restrict__ rev, const float4* __restrict__ Wp, const float4* __restrict__ b4,
    int64_t V, int64_t E, int hv, int KB, int residual, int act, float alpha,
    float4* __restrict__ O4) {
  __shared__ __attribute__((aligned(16))) float sh0[2 * kRows * 16];  // S [64][16] | H [64][16]
  __shared__ __attribute__((aligned(16))) float sh1[2 * kRows * 16];
  __shared__ __attribute__((aligned(16))) float sh2[2 * kRows * 16];
  __shared__ __attribute__((aligned(16))) float wb0[NT * 256];        // [NT][64 lanes][4]
  __shared__ __attribute__((aligned(16))) float wb1[NT * 256];
  __shared__ int64_t s_idx[2 * kRows];
  int64_t* s_src = s_idx;
  int64_t* s_rev = s_idx + kRows;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t e0 = (int64_t)blockIdx.x * kRows;

  if (tid < kRows) {
    const int64_t e = e0 + tid;
    int64_t s = -1, q = -1;
    if (e < E) {
      s = src[e];
      q = rev[e];
      s = (s >= 0 && s < V) ? s * hv : -1;
      q = (q >= 0 && q < E) ? q * hv : -1;
    }
    s_src[tid] = s;
    s_rev[tid] = q;
  }
  __syncthreads();

  const int lrow = 16 * wave + (lane >> 2), lpiece = lane & 3;
  const int64_t ls = s_src[lrow], lq = s_rev[lrow];
  const float4* s_row = S4 + (ls >= 0 ? ls : 0);
  const float4* h_row = H4 + (lq >= 0 ? lq : 0);
  const int frow = 16 * wave + (lane & 15), fg = lane >> 4;
  const bool fs_ok = s_src[frow] >= 0, fq_ok = s_rev[frow] >= 0;

  auto sh_slot = [&](auto tag) -> float* {
    constexpr int k = decltype(tag)::value;
    if constexpr (k == 0) return sh0;
    else if constexpr (k == 1) return sh1;
    else return sh2;
  };
  auto wb_slot = [&](auto tag) -> float* {
    constexpr int k = decltype(tag)::value;
    if constexpr (k == 0) return wb0;
    else return wb1;
  };
  auto issue_sh = [&](int kb, float* slot) {
    int c = 4 * kb + lpiece;
    c = c < hv ? c : hv - 1;
    glds16(s_row + c, slot + 16 * 16 * wave);
    glds16(h_row + c, slot + kRows * 16 + 16 * 16 * wave);
  };
  auto issue_w = [&](int kb, float* slot) {
    const float4* wk = Wp + (int64_t)kb * NT * 64 + lane;
    for (int t = wave; t < NT; t += 4) glds16(wk + t * 64, slot + 256 * t);
  };

  f32x4 acc[NT];
#pragma unroll
  for (int ct = 0; ct < NT; ++ct) acc[ct] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one K step reading S/H slot RS and W slot RW (compile-time), prefetching ahead
  auto step = [&](int kb, auto rs_tag, auto rw_tag) {
    constexpr int RS = decltype(rs_tag)::value, RW = decltype(rw_tag)::value;
    const float* shs = sh_slot(std::integral_constant<int, RS>{});
    const float* wbs = wb_slot(std::integral_constant<int, RW>{});
    const float4 sv = *reinterpret_cast<const float4*>(shs + frow * 16 + 4 * fg);
    const float4 hq = *reinterpret_cast<const float4*>(shs + kRows * 16 + frow * 16 + 4 * fg);
    const float4* bl = reinterpret_cast<const float4*>(wbs) + lane;
    float4 bf[NT];
#pragma unroll
    for (int ct = 0; ct < NT; ++ct) bf[ct] = bl[64 * ct];
    // prefetch: W(kb+1) first, then S/H(kb+2), so a counted vmcnt(2) leaves only the latter
    if (kb + 1 < KB) issue_w(kb + 1, wb_slot(std::integral_constant<int, (RW + 1) % 2>{}));
    const bool sh_issued = kb + 2 < KB;
    if (sh_issued) issue_sh(kb + 2, sh_slot(std::integral_constant<int, (RS + 2) % 3>{}));
    const bool kin = 4 * kb + fg < hv;
    const float4 mq = act4_t<ACT>(hq, act, alpha);
    const bool use_s = kin && fs_ok, use_q = kin && fq_ok;
    float4 a;
    a.x = (use_s ? sv.x : 0.f) - (use_q ? mq.x : 0.f);
    a.y = (use_s ? sv.y : 0.f) - (use_q ? mq.y : 0.f);
    a.z = (use_s ? sv.z : 0.f) - (use_q ? mq.z : 0.f);
    a.w = (use_s ? sv.w : 0.f) - (use_q ? mq.w : 0.f);
#pragma unroll
    for (int ct = 0; ct + 1 < NT; ct += 2) {
      acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, bf[ct].x, acc[ct], 0, 0, 0);
      acc[ct + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, bf[ct + 1].x, acc[ct + 1], 0, 0, 0);
      acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, bf[ct].y, acc[ct], 0, 0, 0);
      acc[ct + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, bf[ct + 1].y, acc[ct + 1], 0, 0, 0);
      acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, bf[ct].z, acc[ct], 0, 0, 0);
      acc[ct + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, bf[ct + 1].z, acc[ct + 1], 0, 0, 0);
      acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, bf[ct].w, acc[ct], 0, 0, 0);
      acc[ct + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, bf[ct + 1].w, acc[ct + 1], 0, 0, 0);
    }
    if constexpr (NT & 1) {
      acc[NT - 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, bf[NT - 1].x, acc[NT - 1], 0, 0, 0);
      acc[NT - 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, bf[NT - 1].y, acc[NT - 1], 0, 0, 0);
      acc[NT - 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, bf[NT - 1].z, acc[NT - 1], 0, 0, 0);
      acc[NT - 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, bf[NT - 1].w, acc[NT - 1], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (sh_issued) asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  // prologue: W(0), S/H(0), S/H(1); wait all but S/H(1)
  issue_w(0, wb0);
  issue_sh(0, sh0);
  if (KB > 1) {
    issue_sh(1, sh1);
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  int kb = 0;
  for (; kb + 6 <= KB; kb += 6) {
    step(kb, I0{}, I0{});
    step(kb + 1, I1{}, I1{});
    step(kb + 2, I2{}, I0{});
    step(kb + 3, I0{}, I1{});
    step(kb + 4, I1{}, I0{});
    step(kb + 5, I2{}, I1{});
  }
  const int rem = KB - kb;  // 0..5, the period restarts at slots (0, 0)
  if (rem > 0) step(kb, I0{}, I0{});
  if (rem > 1) step(kb + 1, I1{}, I1{});
  if (rem > 2) step(kb + 2, I2{}, I0{});
  if (rem > 3) step(kb + 3, I0{}, I1{});
  if (rem > 4) step(kb + 4, I1{}, I0{});

  // ---- epilogue: groups of 3 column tiles, slabs in sh0 (waves 0,1) and sh1 (waves 2,3) ----
  constexpr int kLDE = 16 * kRingEpiG + 4;
  float* slab = (wave < 2 ? sh0 : sh1) + (wave & 1) * 16 * kLDE;
  __syncthreads();
#pragma unroll
  for (int g0 = 0; g0 < NT; g0 += kRingEpiG) {
#pragma unroll
    for (int i = 0; i < kRingEpiG; ++i) {
      const int ct = g0 + i;
      if (ct < NT) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          slab[(4 * (lane >> 4) + j) * kLDE + 16 * i + (lane & 15)] = acc[ct][j];
      }
    }
    __syncthreads();
    const int ntiles = (NT - g0) < kRingEpiG ? (NT - g0) : kRingEpiG;
    const int nc4 = ntiles * 4;
    for (int i = lane; i < 16 * nc4; i += 64) {
      const int r = i / nc4, c = i - r * nc4;
      const int64_t e = e0 + 16 * wave + r;
      const int col4 = 4 * g0 + c;
      if (e < E && col4 < hv) {
        float4 o = *reinterpret_cast<const float4*>(&slab[r * kLDE + 4 * c]);
        if (b4) o = o + b4[col4];
        if (residual) o = H4[e * hv + col4] + o;
        O4[e * hv + col4] = o;
      }
    }
    __syncthreads();
  }
}

template <int NT, int ACT>
int launch_ring(const UpdateArgs& a) {
  const int64_t grid = (a.E + kRows - 1) / kRows;
  NT_REQUIRE(grid < (int64_t(1) << 31), NT_EINVAL, "too many edges");
  update_ring_kernel<NT, ACT><<<(unsigned)grid, 256, 0, a.stream>>>(
      (const float4*)a.H, (const float4*)a.S, a.src, a.rev, (const float4*)a.Wp,
      (const float4*)a.b, a.V, a.E, (int)(a.h / 4), a.KB, a.residual, a.act, a.alpha,
      (float4*)a.H_out);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

template <int ACT, int... NTs>
int dispatch_ring(const UpdateArgs& a, std::integer_sequence<int, NTs...>) {
  int rc = NT_EUNSUPPORTED;
  bool done = false;
  ((a.NT == NTs + 1 ? (rc = launch_ring<NTs + 1, ACT>(a), done = true) : false), ...);
  if (!done) set_error("nt_dmpnn_update: no ring kernel for this hidden size");
  return rc;
}
}  // namespace

int launch_update_ring(const UpdateArgs& a) {
  using Seq = std::make_integer_sequence<int, 24>;  // NT <= 24: all W fragments held in VGPRs
  if (a.act == NT_ACT_RELU) return dispatch_ring<NT_ACT_RELU>(a, Seq{});
  return dispatch_ring<-1>(a, Seq{});
}

int launch_update_glds(const UpdateArgs& a) {
  using Seq = std::make_integer_sequence<int, 32>;
  if (a.act == NT_ACT_RELU) return dispatch_nt<NT_ACT_RELU>(a, Seq{});
  return dispatch_nt<-1>(a, Seq{});
}

}  // namespace nt
#endif  // NT_DIAG

// Fused D-MPNN layer update, bf16x6 fp32 emulation, warp-specialised producer/consumer kernel
// (default for h % 4 == 0, 97 <= h <= 320):
//
//   H_out[e] = (residual ? H[e] : 0) + W (S[src[e]] - act(H[rev[e]])) + b     (chemprop.py:36-43,
//                                                                               residual.py:27-28)
// Why: in-kernel s_memtime stamps of the single-role kernel (update_x6.hip) showed each MFMA wave
// spending ~1000 cycles per K-step just ISSUING LDS-DMA (~100 cycles per global_load_lds) and
// ~700 on the A read + bf16 split, against ~1000 cycles of MFMA.  Here those jobs move to
// dedicated waves:
//   * 4 producer waves: issue every LDS-DMA (S/H row pieces and the W chunk 2 chunks ahead),
//     and turn the landed S/H pieces of their own 32 rows into the A operand, split into three
//     bf16 parts, written as MFMA-ready fragments (an "A-parts" ring).  A producer only reads
//     rows it DMA'd itself, so its own counted vmcnt orders DMA -> split (no barrier needed).
//   * 8 consumer waves: per step 3 ds_read_b128 (A parts) + 3 per column tile (W parts) and 6
//     v_mfma_f32_32x32x16_bf16 per tile; nothing else.  Wave c owns 32-row tile (c % 4) x
//     column half (c / 4).
//   * one workgroup barrier per K-step; every ring slot is its own __shared__ object so hipcc
//     places no vmcnt drain in front of reads of the current slot.
// Workgroup = 12 waves (768 lanes), 128 edges x all h columns, 1 workgroup per CU (3 waves/SIMD).
// A/B-only kernel: compiled into the diagnostic library (make DIAG=1) only.
#ifdef NT_DIAG
#include <stdlib.h>

#include <type_traits>

#include "common.hpp"
#include "update.hpp"

namespace nt {

// Diagnostic stamp sums (STAMP builds only): [0] consumer compute, [1] consumer barrier,
// [2] producer DMA issue, [3] producer vmcnt wait, [4] producer split, [5] producer barrier,
// [6] consumer steps, [7] producer steps.
__device__ unsigned long long g_pc_stamps[9];

namespace {

__device__ __forceinline__ unsigned long long stamp_now() {
  unsigned long long t = 0;
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
#endif
  return t;
}

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

constexpr int kRows = 128;   // edges per workgroup (4 row tiles of 32)
constexpr int kCons = 8;     // consumer waves
constexpr int kProd = 4;     // producer waves
constexpr int kThreads = 64 * (kCons + kProd);
constexpr int kAP = 3 * 4 * 64 * 4;  // floats per A-parts slot: [part][rt][lane] x 16 B
constexpr int kLDE = 32 + 4;         // epilogue slab row stride (one 32-col tile), == 4 mod 8
constexpr int kSlab = 32 * kLDE;
constexpr int kWDist = 3;            // W chunk DMA'd this many steps ahead (ring of kWDist + 1)
constexpr int kRD = 4;               // producer register ring: S/H chunk loaded kRD-1 steps ahead

template <int NT32>
struct PCGeom {
  static constexpr int kWT = NT32 * 3;                    // W tiles (1 KiB) per chunk
  static constexpr int kWPC = (kWT + kCons - 1) / kCons;  // W DMAs per consumer per step
  static constexpr int kW = kWPC * kCons * 256;           // floats per W slot (incl. padding)
  static constexpr int kLdsBytes = 4 * (2 * kAP + (kWDist + 1) * kW) + 16 * kRows;
  static constexpr bool kFits = kLdsBytes <= 160 * 1024 && kCons * kSlab <= 2 * kW;
};

__device__ __forceinline__ void glds16(const void* g, float* l) {
  __builtin_amdgcn_global_load_lds((gbl_void*)g, (lds_void*)l, 16, 0, 0);
}

// The same DMA issued from inline asm.  hipcc's waitcnt pass does not see it, so it cannot put a
// vmcnt(0) drain in front of LDS reads it fails to prove disjoint from the DMA (it does so at the
// loop head of a 4-slot ring).  The issuing wave orders completion itself with counted vmcnt.
__device__ __forceinline__ void glds16_asm(const void* g, float* l) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef __attribute__((address_space(3))) float lds_float;
  const unsigned m = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_float*)l);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m)
               : "memory", "m0");
#endif
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
#endif
}

// Raw workgroup barrier: LDS operations retired, then s_barrier.  A __syncthreads() would add
// vmcnt(0) and drain the loads / DMA that are meant to stay in flight across it.
__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_sched_barrier(0);
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int K>
using IC = std::integral_constant<int, K>;

// MODE (diagnostic builds only): 1 stamps.
template <int NT32, int ACT, int MODE = 0>
__global__ void __launch_bounds__(kThreads, 3) update_pc_kernel(
    const float4* __restrict__ H4, const float4* __restrict__ S4, const int64_t* __restrict__ src,
    const int64_t* __restrict__ rev, const uint4* __restrict__ Wx, const float4* __restrict__ b4,
    int64_t V, int64_t E, int hv, int KB, int residual, int act, float alpha,
    float4* __restrict__ O4) {
  using G = PCGeom<NT32>;
  constexpr int kWT = G::kWT, kWPC = G::kWPC, kW = G::kW;
  constexpr bool STAMP = MODE & 1;
  // rings: A-parts (2 slots, written by producers one step ahead), W (4 slots, DMA'd by the
  // consumers three steps ahead).  Every slot is its own object: reads of the current slot do not
  // alias the DMA in flight into the others, so hipcc puts no vmcnt drain in front of them.
  __shared__ __attribute__((aligned(16))) float ap0[kAP];
  __shared__ __attribute__((aligned(16))) float ap1[kAP];
  __shared__ __attribute__((aligned(16))) float wb0[kW];
  __shared__ __attribute__((aligned(16))) float wb1[kW];
  __shared__ __attribute__((aligned(16))) float wb2[kW];
  __shared__ __attribute__((aligned(16))) float wb3[kW];
  __shared__ int64_t s_idx[2 * kRows];
  int64_t* s_src = s_idx;
  int64_t* s_rev = s_idx + kRows;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t e0 = (int64_t)blockIdx.x * kRows;
  unsigned long long st[4] = {0, 0, 0, 0};
  auto stamp = [&]() -> unsigned long long {
    if constexpr (STAMP) return stamp_now();
    else return 0;
  };

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

  auto ap_slot = [&](auto tag) -> float* {
    if constexpr (decltype(tag)::value == 0) return ap0;
    else return ap1;
  };
  auto wb_slot = [&](auto tag) -> float* {
    constexpr int k = decltype(tag)::value;
    if constexpr (k == 0) return wb0;
    else if constexpr (k == 1) return wb1;
    else if constexpr (k == 2) return wb2;
    else return wb3;
  };

  if (wave >= kCons) {
    // =============================== producer waves ===============================
    // Wave p owns row tile p (rows 32p .. 32p+31).  Lane: fragment row 32p + (lane & 31), k group
    // fk = lane >> 5 (k = 8 fk + j of the 16-wide chunk).  Per chunk a lane loads its 2 + 2 float4
    // of S[src] and H[rev] straight into registers, kRD - 1 chunks ahead of the split.
    const int p = wave - kCons;
    const int frow = 32 * p + (lane & 31), fk = lane >> 5;
    const int64_t ls = s_src[frow], lq = s_rev[frow];
    const bool fs_ok = ls >= 0, fq_ok = lq >= 0;
    const float4* sp = S4 + (fs_ok ? ls : 0);
    const float4* hp = H4 + (fq_ok ? lq : 0);
    float4 R[kRD][4];
    auto load_chunk = [&](int kb, auto slot) {
      constexpr int r = decltype(slot)::value;
      const int c = 4 * kb + 2 * fk;
      const int ca = c < hv ? c : hv - 1;  // past h (or past the last chunk): a valid piece,
      const int cb = c + 1 < hv ? c + 1 : hv - 1;  // masked in the split or never used
      R[r][0] = sp[ca];
      R[r][1] = sp[cb];
      R[r][2] = hp[ca];
      R[r][3] = hp[cb];
    };
    auto split_chunk = [&](int kb, auto slot, float* aps) {
      constexpr int r = decltype(slot)::value;
      const int col4 = 4 * kb + 2 * fk;
      const bool k0 = col4 < hv, k1 = col4 + 1 < hv;
      const float4 s0 = R[r][0], s1 = R[r][1];
      const float4 m0 = act4_t<ACT>(R[r][2], act, alpha), m1 = act4_t<ACT>(R[r][3], act, alpha);
      const bool us0 = k0 && fs_ok, uq0 = k0 && fq_ok, us1 = k1 && fs_ok, uq1 = k1 && fq_ok;
      float x[8];
      x[0] = (us0 ? s0.x : 0.f) - (uq0 ? m0.x : 0.f);
      x[1] = (us0 ? s0.y : 0.f) - (uq0 ? m0.y : 0.f);
      x[2] = (us0 ? s0.z : 0.f) - (uq0 ? m0.z : 0.f);
      x[3] = (us0 ? s0.w : 0.f) - (uq0 ? m0.w : 0.f);
      x[4] = (us1 ? s1.x : 0.f) - (uq1 ? m1.x : 0.f);
      x[5] = (us1 ? s1.y : 0.f) - (uq1 ? m1.y : 0.f);
      x[6] = (us1 ? s1.z : 0.f) - (uq1 ? m1.z : 0.f);
      x[7] = (us1 ? s1.w : 0.f) - (uq1 ? m1.w : 0.f);
      bf16x8 a[3];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const __bf16 h0 = (__bf16)x[j];
        const float r1 = x[j] - (float)h0;
        const __bf16 h1 = (__bf16)r1;
        a[0][j] = h0;
        a[1][j] = h1;
        a[2][j] = (__bf16)(r1 - (float)h1);
      }
      bf16x8* dst = reinterpret_cast<bf16x8*>(aps) + p * 64 + lane;  // [part][rt][lane]
#pragma unroll
      for (int part = 0; part < 3; ++part) dst[part * 4 * 64] = a[part];
    };

    // prologue: chunks 0 .. kRD-1 in flight, split chunk 0 -> ap0
    load_chunk(0, IC<0>{});
    load_chunk(1, IC<1>{});
    load_chunk(2, IC<2>{});
    load_chunk(3, IC<3>{});
    split_chunk(0, IC<0>{}, ap0);
    raw_barrier();

    // step kb (consumers read A-parts slot kb%2): load chunk kb+kRD into register set kb%kRD
    // (chunk kb's, split a step ago), split chunk kb+1 (set (kb+1)%kRD) -> A-parts slot (kb+1)%2.
    auto pstep = [&](int kb, auto rr) {
      constexpr int RR = decltype(rr)::value;  // kb % 4
      const unsigned long long t0 = stamp();
      load_chunk(kb + kRD, IC<RR>{});
      const unsigned long long t1 = stamp();
      if (kb + 1 < KB) split_chunk(kb + 1, IC<(RR + 1) % kRD>{}, ap_slot(IC<(RR + 1) % 2>{}));
      const unsigned long long t2 = stamp();
      raw_barrier();
      if constexpr (STAMP) {
        const unsigned long long t3 = stamp();
        st[0] += t1 - t0;
        st[2] += t2 - t1;
        st[3] += t3 - t2;
      }
    };
    int kb = 0;
    for (; kb + 4 <= KB; kb += 4) {  // ring period lcm(kRD, 2)
      pstep(kb, IC<0>{});
      pstep(kb + 1, IC<1>{});
      pstep(kb + 2, IC<2>{});
      pstep(kb + 3, IC<3>{});
    }
    const int rem = KB - kb;
    if (rem > 0) pstep(kb, IC<0>{});
    if (rem > 1) pstep(kb + 1, IC<1>{});
    if (rem > 2) pstep(kb + 2, IC<2>{});
    raw_barrier();  // matches the consumers' pre-epilogue barrier
    if constexpr (STAMP) {
      if (lane == 0) {
        for (int i = 0; i < 4; ++i) atomicAdd(&g_pc_stamps[2 + i], st[i]);
        atomicAdd(&g_pc_stamps[7], (unsigned long long)KB);
      }
    }
    return;  // outstanding prefetch loads past the last chunk are harmless (registers only)
  }

  // =============================== consumer waves ===============================
  const int rt = wave % 4, ch = wave / 4;
  constexpr int CW = (NT32 + 1) / 2;
  const int ncol = ch == 0 ? CW : NT32 - CW;
  const int c0 = ch == 0 ? 0 : CW;
  // W DMA role: wave `wave` moves W tiles wave + kCons*i of each chunk (tiles past kWT: a padding
  // copy of tile 0 into the slot's tail, so every consumer issues the same count -> counted vmcnt)
  const uint4* wsrc = Wx + lane;
  auto issue_w = [&](int kb, float* wbs) {
    const uint4* wk = wsrc + (int64_t)kb * kWT * 64;
#pragma unroll
    for (int i = 0; i < kWPC; ++i) {
      const int t = wave + kCons * i;
      glds16_asm(wk + (t < kWT ? t : 0) * 64, wbs + 256 * t);
    }
  };
  f32x16 acc[CW];
#pragma unroll
  for (int i = 0; i < CW; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;

  // prologue: W(0..2) in flight, W(0) landed before the barrier (KB >= 7 for this kernel)
  issue_w(0, wb0);
  issue_w(1, wb1);
  issue_w(2, wb2);
  wait_vmcnt<2 * kWPC>();
  raw_barrier();

  auto body = [&](auto nc_tag) {
    constexpr int NC = decltype(nc_tag)::value;
    auto cstep = [&](int kb, auto rw) {
      constexpr int RW = decltype(rw)::value;  // kb % 4; A-parts slot kb % 2
      const unsigned long long t0 = stamp();
      const int n_after = KB - 2 - kb;  // W chunks issued after W(kb+1) once this step issued
      if (kb + kWDist < KB) issue_w(kb + kWDist, wb_slot(IC<(RW + kWDist) % 4>{}));
      const bf16x8* apl = reinterpret_cast<const bf16x8*>(ap_slot(IC<RW % 2>{})) + rt * 64 + lane;
      const bf16x8 a0 = apl[0], a1 = apl[4 * 64], a2 = apl[8 * 64];
      const bf16x8* wl = reinterpret_cast<const bf16x8*>(wb_slot(rw)) + lane;
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        const int t = c0 + i;
        const bf16x8 w0 = wl[(3 * t + 0) * 64], w1 = wl[(3 * t + 1) * 64], w2 = wl[(3 * t + 2) * 64];
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, w0, acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, w1, acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, w2, acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, w0, acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, w1, acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, w0, acc[i], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the MFMAs above the wait + barrier
#if defined(__HIP_DEVICE_COMPILE__)
      if constexpr (STAMP) {
#pragma unroll
        for (int i = 0; i < NC; ++i) asm volatile("" ::"v"(acc[i]));
      }
#endif
      const unsigned long long t1 = stamp();
      // own W(kb+1) DMA landed (leave W(kb+2), W(kb+3) in flight), then publish
      if (n_after >= 2) wait_vmcnt<2 * kWPC>();
      else if (n_after == 1) wait_vmcnt<kWPC>();
      else wait_vmcnt<0>();
      raw_barrier();
      if constexpr (STAMP) {
        const unsigned long long t2 = stamp();
        st[0] += t1 - t0;
        st[1] += t2 - t1;
      }
    };
    int kb = 0;
    for (; kb + 4 <= KB; kb += 4) {
      cstep(kb, IC<0>{});
      cstep(kb + 1, IC<1>{});
      cstep(kb + 2, IC<2>{});
      cstep(kb + 3, IC<3>{});
    }
    const int rem = KB - kb;
    if (rem > 0) cstep(kb, IC<0>{});
    if (rem > 1) cstep(kb + 1, IC<1>{});
    if (rem > 2) cstep(kb + 2, IC<2>{});
  };
  if (ncol == CW) body(IC<CW>{});
  else body(IC<NT32 - CW>{});
  wait_vmcnt<0>();
  raw_barrier();  // every wave is past its last W-slot read: the W ring becomes slab space
  if constexpr (STAMP) {
    if (lane == 0) {
      atomicAdd(&g_pc_stamps[0], st[0]);
      atomicAdd(&g_pc_stamps[1], st[1]);
      atomicAdd(&g_pc_stamps[6], (unsigned long long)KB);
    }
  }

  // ---- epilogue: per 32-col tile, a wave-private slab (in-order LDS within a wave: no
  // barrier between the C-fragment writes and the row-piece reads) -> +bias +residual -> store
  // C/D map of 32x32 MFMA: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
  float* slab = (wave < 4 ? wb0 : wb1) + (wave & 3) * kSlab;  // W ring is free after the loop
#pragma unroll
  for (int i = 0; i < CW; ++i) {
    if (i < ncol) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        slab[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * kLDE + (lane & 31)] = acc[i][r];
      // 32 rows x 8 float4 = 4 pieces per lane: issue every load first, then one wait
      float4 o[4], hr[4], bb[4];
      bool ok[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int j = lane + 64 * u, r = j >> 3, c = j & 7;
        const int64_t e = e0 + 32 * rt + r;
        const int col4 = 8 * (c0 + i) + c;
        ok[u] = e < E && col4 < hv;
        const int64_t off = ok[u] ? e * hv + col4 : 0;
        hr[u] = residual ? H4[off] : make_float4(0.f, 0.f, 0.f, 0.f);
        bb[u] = b4 ? b4[ok[u] ? col4 : 0] : make_float4(0.f, 0.f, 0.f, 0.f);
        o[u] = *reinterpret_cast<const float4*>(&slab[r * kLDE + 4 * c]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int j = lane + 64 * u, r = j >> 3, c = j & 7;
        if (ok[u]) O4[(e0 + 32 * rt + r) * hv + 8 * (c0 + i) + c] = hr[u] + (o[u] + bb[u]);
      }
    }
  }
}

template <int NT32, int ACT, int MODE = 0>
int launch_pc(const UpdateArgs& a) {
  const int64_t grid = (a.E + kRows - 1) / kRows;
  NT_REQUIRE(grid < (int64_t(1) << 31), NT_EINVAL, "too many edges");
  update_pc_kernel<NT32, ACT, MODE><<<(unsigned)grid, kThreads, 0, a.stream>>>(
      (const float4*)a.H, (const float4*)a.S, a.src, a.rev, (const uint4*)a.Wp,
      (const float4*)a.b, a.V, a.E, (int)(a.h / 4), (int)((a.h + 15) / 16), a.residual, a.act,
      a.alpha, (float4*)a.H_out);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

template <int NT32, int ACT>
int launch_pc_if_fits(const UpdateArgs& a) {
  if constexpr (PCGeom<NT32>::kFits) {
    if constexpr (NT32 == 10 && ACT == NT_ACT_RELU) {  // diagnostic stamp build (A/B only)
      const char* v = getenv("NT_PC_MODE");
      const int m = v ? atoi(v) : 0;
      if (m == 1) return launch_pc<NT32, ACT, 1>(a);
    }
    return launch_pc<NT32, ACT>(a);
  } else {
    return NT_EUNSUPPORTED;
  }
}

template <int ACT, int... Ns>
int dispatch_pc(const UpdateArgs& a, int nt32, std::integer_sequence<int, Ns...>) {
  int rc = NT_EUNSUPPORTED;
  bool done = false;
  ((nt32 == Ns + 4 && PCGeom<Ns + 4>::kFits ? (rc = launch_pc_if_fits<Ns + 4, ACT>(a), done = true)
                                            : false),
   ...);
  if (!done) set_error("nt_dmpnn_update: no producer/consumer kernel for this hidden size");
  return rc;
}

template <int... Ns>
constexpr bool any_fits(int nt32, std::integer_sequence<int, Ns...>) {
  return ((nt32 == Ns + 4 && PCGeom<Ns + 4>::kFits) || ...);
}

}  // namespace

bool pc_supported(int64_t h) {
  const int nt32 = (int)((h + 31) / 32);
  return h % 4 == 0 && any_fits(nt32, std::make_integer_sequence<int, 13>{});
}

int launch_update_pc(const UpdateArgs& a) {
  using Seq = std::make_integer_sequence<int, 13>;  // NT32 = 4 .. 16 where the LDS fits
  const int nt32 = (int)((a.h + 31) / 32);
  if (a.act == NT_ACT_RELU) return dispatch_pc<NT_ACT_RELU>(a, nt32, Seq{});
  return dispatch_pc<-1>(a, nt32, Seq{});
}

}  // namespace nt

// Debug-only (not in include/notorch_amd.h): read/reset the producer/consumer stamp sums.
extern "C" __attribute__((visibility("default"))) int nt_debug_pc_stamps(unsigned long long* out8,
                                                                         int reset) {
  if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(nt::g_pc_stamps), 9 * sizeof(unsigned long long), 0,
                          hipMemcpyDeviceToHost) != hipSuccess)
    return 2;
  if (reset) {
    unsigned long long z[9] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(nt::g_pc_stamps), z, sizeof(z), 0, hipMemcpyHostToDevice) !=
        hipSuccess)
      return 2;
  }
  return 0;
}
#endif  // NT_DIAG

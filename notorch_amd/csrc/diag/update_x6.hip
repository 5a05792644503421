// Fused D-MPNN layer update on bf16 MFMA with fp32 emulation ("bf16x6"):
//
//   H_out[e] = (residual ? H[e] : 0) + W (S[src[e]] - act(H[rev[e]])) + b     (chemprop.py:36-43,
//                                                                               residual.py:27-28)
// Numerics.  Every fp32 operand x is split exactly into three bf16 parts x = x0 + x1 + x2
// (x0 = rne(x), x1 = rne(x - x0), x2 = rne(x - x0 - x1); 3 x 8 = 24 significant bits), and
//   a.w ~= a0.w0 + a0.w1 + a1.w0 + a0.w2 + a1.w1 + a2.w0
// is accumulated in fp32 by six v_mfma_f32_32x32x16_bf16.  Each bf16 x bf16 product is exact in
// fp32; the dropped terms (a1.w2, a2.w1, a2.w2) are < 2^-24 relative, so the result carries fp32
// GEMM accuracy (tests: <= 1e-5 normalised vs the fp32 oracle, typically ~3e-7 vs fp64) at
// 6 x 16 = 96 MFMA cycles per 32x32x16 block instead of the 256 of fp32 MFMA (2.7x).
//
// Structure (one workgroup = 4 waves = 64 edges x all h output columns, K in 16-deep chunks):
//   * 2-slot LDS rings, each slot its own __shared__ array (compile-time slot per step, loop
//     unrolled by 2, so hipcc puts no vmcnt wait on reads of the current slot while the next
//     slot's LDS-DMA is in flight):
//       - S/H pieces: 64 rows x 64 B each (S[src[e]], H[rev[e]]), global_load_lds_dwordx4
//       - W chunk:   NT32 x 3 parts x 1 KiB of the pre-split fragment image (L2-resident)
//   * wave w computes the 32-row tile (w & 1) x column half (w >> 1): acc = 16 VGPR per 32x32
//     tile.  The A fragment (8 k per lane) is formed as S - act(H), masked, split in registers.
//   * epilogue: accumulators staged through LDS (reusing the W ring) in 2-tile column groups,
//     then + bias + residual and 16-B row-piece stores.
#include <stdlib.h>

#include <type_traits>

#include "../common.hpp"
#include "../update.hpp"

#ifdef NT_DIAG  // A/B variant: superseded by update_fk_kernel in the shipping library
namespace nt {

// Diagnostic-build stamp accumulators (cycles summed over waves): issue, A read+split, MFMA
// (incl. B reads), barrier/vmcnt wait, steps.  Only the ABL == 8 instantiation writes them.
__device__ unsigned long long g_x6_stamps[8];

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

// Geometry: MW 32-row tiles per workgroup (2 column halves -> 2*MW waves), S/H gather ring of
// SHR slots (SHR = 3: gathers run two K-chunks ahead), W ring of 2 slots.
template <int NT32, int MW>
struct X6Geom {
  static constexpr int kWaves = 2 * MW;
  static constexpr int kThreads = 64 * kWaves;
  static constexpr int kRows = 32 * MW;
  static constexpr int kSH = 2 * kRows * 16;           // floats per S/H slot: S [rows][16] | H
  static constexpr int kW = NT32 * 3 * 256;            // floats per W slot ([nt][part][lane] 16 B)
  // epilogue: column tiles per group kG, slab row stride (== 4 mod 8); kWaves/2 slabs per W slot
  static constexpr int kG = ((kWaves / 2) * 32 * (32 * 2 + 4) <= kW) ? 2 : 1;
  static constexpr int kLDE = 32 * kG + 4;
  static constexpr int kSlab = 32 * kLDE;
  static constexpr bool kFits = (kWaves / 2) * kSlab <= kW;
};

__device__ __forceinline__ void glds16(const void* g, float* l) {
  __builtin_amdgcn_global_load_lds((gbl_void*)g, (lds_void*)l, 16, 0, 0);
}

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

// ABL (timing-only ablation builds, outputs wrong): 1 = no W DMA, 2 = no S/H DMA, 4 = no MFMA;
// ABL == 8: diagnostic stamp build (outputs right, slower; phase cycles -> g_x6_stamps)
// RESACC: residual + bias preloaded into the accumulators (else added in the epilogue)
template <int NT32, int MW, int SHR, int WR, int ACT, int ABL = 0, bool RESACC = false>
__global__ void __launch_bounds__(128 * MW, 2) update_x6_kernel(
    const float4* __restrict__ H4, const float4* __restrict__ S4, const int64_t* __restrict__ src,
    const int64_t* __restrict__ rev, const uint4* __restrict__ Wx, const float4* __restrict__ b4,
    int64_t V, int64_t E, int hv, int KB, int residual, int act, float alpha,
    float4* __restrict__ O4) {
  using G = X6Geom<NT32, MW>;
  constexpr int kRows = G::kRows, kW = G::kW, kSH = G::kSH;
  constexpr int kEpiG = G::kG, kLDE = G::kLDE, kSlab = G::kSlab;
  static_assert(G::kFits, "epilogue slabs must fit the W ring");
  static_assert(SHR == 2 || SHR == 3, "S/H ring depth");
  static_assert(WR == 2 || (WR == 3 && SHR == 3), "W ring depth");
  // W tiles per wave per step: every wave issues the same count (kWPW); padding loads re-read
  // tile 0 into the spare tail of the slot, so a counted vmcnt is wave-uniform
  constexpr int kWT = NT32 * 3;
  constexpr int kWPW = (kWT + G::kWaves - 1) / G::kWaves;
  // every ring slot is its own __shared__ object (see file header)
  __shared__ __attribute__((aligned(16))) float sh0[kSH];
  __shared__ __attribute__((aligned(16))) float sh1[kSH];
  __shared__ __attribute__((aligned(16))) float sh2[SHR > 2 ? kSH : 4];
  constexpr int kWS = WR == 3 ? kWPW * G::kWaves * 256 : kW;  // W slot incl. padding tiles
  __shared__ __attribute__((aligned(16))) float wb0[kWS];
  __shared__ __attribute__((aligned(16))) float wb1[kWS];
  __shared__ __attribute__((aligned(16))) float wb2[WR > 2 ? kWS : 4];
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

  auto sh_slot = [&](auto tag) -> float* {
    constexpr int k = decltype(tag)::value;
    if constexpr (k == 0) return sh0;
    else if constexpr (k == 1) return sh1;
    else return sh2;
  };
  auto wb_slot = [&](auto tag) -> float* {
    constexpr int k = decltype(tag)::value;
    if constexpr (k == 0) return wb0;
    else if constexpr (k == 1) return wb1;
    else return wb2;
  };

  // LDS-DMA roles: S/H piece (lane & 3) of tile row 16*wave + lane/4; W tiles wave, wave+NW, ...
  const int lrow = 16 * wave + (lane >> 2), lpiece = lane & 3;
  const int64_t ls = s_src[lrow], lq = s_rev[lrow];
  const float4* s_row = S4 + (ls >= 0 ? ls : 0);
  const float4* h_row = H4 + (lq >= 0 ? lq : 0);
  // LDS slot q of a 64-B row holds logical piece q ^ f(row), f(row) = (row >> 2) & 3: the swizzle
  // (applied on the DMA source address; the DMA destination stays lane-linear) makes the
  // ds_read_b128 fragment reads conflict-free.  For DMA lanes f(row) = (lane >> 4) & 3.
  const int lsrc_piece = lpiece ^ ((lane >> 4) & 3);
  auto issue_sh = [&](int kb, float* shs) {
    if constexpr ((ABL & 2) != 0) return;
    int c = 4 * kb + lsrc_piece;
    c = c < hv ? c : hv - 1;
    glds16(s_row + c, shs + 16 * 16 * wave);
    glds16(h_row + c, shs + kRows * 16 + 16 * 16 * wave);
  };
  auto issue_w = [&](int kb, float* wbs) {
    if constexpr ((ABL & 1) != 0) return;
    const uint4* wk = Wx + (int64_t)kb * NT32 * 3 * 64 + lane;
    if constexpr (WR == 3) {
#pragma unroll
      for (int i = 0; i < kWPW; ++i) {
        const int t = wave + i * G::kWaves;
        glds16(wk + (t < kWT ? t : 0) * 64, wbs + 256 * t);  // t >= kWT: padding slot tail
      }
    } else {
      for (int t = wave; t < kWT; t += G::kWaves) glds16(wk + t * 64, wbs + 256 * t);
    }
  };

  // MFMA role: 32-row tile rt, column tiles [c0, c0 + ncol)
  const int rt = wave % MW, ch = wave / MW;
  constexpr int CW = (NT32 + 1) / 2;
  const int ncol = ch == 0 ? CW : NT32 - CW;
  const int c0 = ch == 0 ? 0 : CW;
  const int frow = 32 * rt + (lane & 31), fk = lane >> 5;  // fragment: k = 8 fk + j
  const bool fs_ok = s_src[frow] >= 0, fq_ok = s_rev[frow] >= 0;
  const int fsw = (frow >> 2) & 3;                        // swizzle of this fragment row
  const int fslot0 = 4 * ((2 * fk) ^ fsw), fslot1 = 4 * ((2 * fk + 1) ^ fsw);  // float offsets

  f32x16 acc[CW];

  unsigned long long st[5] = {0, 0, 0, 0, 0};  // diagnostic stamp sums (ABL == 8)
  auto body = [&](auto nc_tag) {
    constexpr int NC = decltype(nc_tag)::value;
    // RESACC: accumulators start at residual + bias (C/D layout: row = (r&3) + 8(r>>2) +
    // 4(lane>>5), col = lane & 31), read here and overlapped with the K loop; each load is two
    // full 128-B row segments.  Otherwise they start at 0 and the epilogue adds both.
    if constexpr (!RESACC) {
#pragma unroll
      for (int i = 0; i < CW; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    } else {
      const float* Hf = reinterpret_cast<const float*>(H4);
      const float* bf = reinterpret_cast<const float*>(b4);
      const int h = 4 * hv;
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        int col = 32 * (c0 + i) + (lane & 31);
        col = col < h ? col : h - 1;  // padding columns: any finite value, never stored
        const float bv = bf ? bf[col] : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          int64_t e = e0 + 32 * rt + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          e = e < E ? e : E - 1;
          acc[i][r] = residual ? Hf[e * h + col] + bv : bv;
        }
      }
#pragma unroll
      for (int i = NC; i < CW; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    }
    auto stamp = [&]() -> unsigned long long {
      if constexpr (ABL == 8) {
        unsigned long long t = 0;
#if defined(__HIP_DEVICE_COMPILE__)
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
        __builtin_amdgcn_sched_barrier(0);
#endif
        return t;
      } else {
        return 0;
      }
    };
    auto step = [&](int kb, auto rs_tag, auto rw_tag) {
      constexpr int RS = decltype(rs_tag)::value, RW = decltype(rw_tag)::value;
      const unsigned long long t0 = stamp();
      const float* shs = sh_slot(rs_tag);
      const float* wbs = wb_slot(rw_tag);
      // prefetch: W first, then S/H, so a counted vmcnt can leave the newest DMAs in flight
      bool sh_ahead = false;
      if constexpr (WR == 3) {
        sh_ahead = kb + 2 < KB;
        if (sh_ahead) {
          issue_w(kb + 2, wb_slot(std::integral_constant<int, (RW + 2) % 3>{}));
          issue_sh(kb + 2, sh_slot(std::integral_constant<int, (RS + 2) % 3>{}));
        }
      } else {
        if (kb + 1 < KB) issue_w(kb + 1, wb_slot(std::integral_constant<int, (RW + 1) % 2>{}));
        if constexpr (SHR == 3) {
          sh_ahead = kb + 2 < KB;
          if (sh_ahead) issue_sh(kb + 2, sh_slot(std::integral_constant<int, (RS + 2) % 3>{}));
        } else {
          if (kb + 1 < KB) issue_sh(kb + 1, sh_slot(std::integral_constant<int, (RS + 1) % 2>{}));
        }
      }
      const unsigned long long t1 = stamp();
      // A fragment: row frow, k = 16kb + 8fk + j  (two 16-B pieces of S and of H)
      const float* sp = shs + frow * 16;
      const float* hp = shs + kRows * 16 + frow * 16;
      const float4 s0 = *reinterpret_cast<const float4*>(sp + fslot0);
      const float4 s1 = *reinterpret_cast<const float4*>(sp + fslot1);
      const float4 q0 = *reinterpret_cast<const float4*>(hp + fslot0);
      const float4 q1 = *reinterpret_cast<const float4*>(hp + fslot1);
      const int col4 = 4 * kb + 2 * fk;
      const bool k0 = col4 < hv, k1 = col4 + 1 < hv;
      const float4 m0 = act4_t<ACT>(q0, act, alpha), m1 = act4_t<ACT>(q1, act, alpha);
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
      bf16x8 a0, a1, a2;
      split3(x, a0, a1, a2);
#if defined(__HIP_DEVICE_COMPILE__)
      if constexpr (ABL == 8) asm volatile("" ::"v"(a0), "v"(a1), "v"(a2));
#endif
      const unsigned long long t2 = stamp();
      const bf16x8* wl = reinterpret_cast<const bf16x8*>(wbs) + lane;
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        const int t = c0 + i;
        const bf16x8 w0 = wl[(3 * t + 0) * 64], w1 = wl[(3 * t + 1) * 64], w2 = wl[(3 * t + 2) * 64];
        if constexpr ((ABL & 4) != 0) {  // keep operands live, skip the MFMAs
          asm volatile("" ::"v"(a0), "v"(a1), "v"(a2), "v"(w0), "v"(w1), "v"(w2));
          continue;
        }
        // smallest terms first
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, w0, acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, w1, acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, w2, acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, w0, acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, w1, acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, w0, acc[i], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the MFMAs above the barrier's wait
#if defined(__HIP_DEVICE_COMPILE__)
      if constexpr (ABL == 8) {
#pragma unroll
        for (int i = 0; i < NC; ++i) asm volatile("" ::"v"(acc[i]));
      }
#endif
      const unsigned long long t3 = stamp();
      if constexpr (WR == 3) {
        // only this step's DMAs (kWPW W + 2 S/H) may stay in flight
        if (sh_ahead) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(kWPW + 2) : "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      } else if constexpr (SHR == 3) {
        // only this step's two S/H DMAs may stay in flight (a __syncthreads() would drain them)
        if (sh_ahead) asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      } else {
        __syncthreads();  // retires chunk kb+1's LDS-DMA; frees slot kb
      }
      if constexpr (ABL == 8) {
        const unsigned long long t4 = stamp();
        st[0] += t1 - t0;
        st[1] += t2 - t1;
        st[2] += t3 - t2;
        st[3] += t4 - t3;
        st[4] += 1;
      }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    int kb = 0;
    if constexpr (WR == 3) {  // both rings of depth 3: period 3
      for (; kb + 3 <= KB; kb += 3) {
        step(kb, I0{}, I0{});
        step(kb + 1, I1{}, I1{});
        step(kb + 2, I2{}, I2{});
      }
      const int rem = KB - kb;
      if (rem > 0) step(kb, I0{}, I0{});
      if (rem > 1) step(kb + 1, I1{}, I1{});
    } else if constexpr (SHR == 3) {  // ring period lcm(3, 2) = 6
      for (; kb + 6 <= KB; kb += 6) {
        step(kb, I0{}, I0{});
        step(kb + 1, I1{}, I1{});
        step(kb + 2, I2{}, I0{});
        step(kb + 3, I0{}, I1{});
        step(kb + 4, I1{}, I0{});
        step(kb + 5, I2{}, I1{});
      }
      const int rem = KB - kb;
      if (rem > 0) step(kb, I0{}, I0{});
      if (rem > 1) step(kb + 1, I1{}, I1{});
      if (rem > 2) step(kb + 2, I2{}, I0{});
      if (rem > 3) step(kb + 3, I0{}, I1{});
      if (rem > 4) step(kb + 4, I1{}, I0{});
    } else {
      for (; kb + 2 <= KB; kb += 2) {
        step(kb, I0{}, I0{});
        step(kb + 1, I1{}, I1{});
      }
      if (kb < KB) step(kb, I0{}, I0{});
    }
  };

  issue_w(0, wb0);
  issue_sh(0, sh0);
  if constexpr (WR == 3) {
    if (KB > 1) {
      issue_w(1, wb1);
      issue_sh(1, sh1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kWPW + 2) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  } else if constexpr (SHR == 3) {
    if (KB > 1) {
      issue_sh(1, sh1);
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  } else {
    __syncthreads();
  }
  if (ncol == CW) body(std::integral_constant<int, CW>{});
  else body(std::integral_constant<int, NT32 - CW>{});

  // ---- epilogue: kEpiG-tile column groups through a wave-private slab (W ring is free now) ----
  // C/D map of 32x32 MFMA: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
  __syncthreads();
  float* slab = (wave < G::kWaves / 2 ? wb0 : wb1) + (wave % (G::kWaves / 2)) * kSlab;
#pragma unroll
  for (int g = 0; g < CW; g += kEpiG) {
#pragma unroll
    for (int i = 0; i < kEpiG; ++i) {
      if (g + i < ncol) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          slab[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * kLDE + 32 * i + (lane & 31)] = acc[g + i][r];
      }
    }
    __syncthreads();
    const int ntiles = (ncol - g) < kEpiG ? (ncol - g) : kEpiG;
    const int nc4 = ntiles > 0 ? ntiles * 8 : 0;  // float4 columns in this group
    for (int i = lane; i < 32 * nc4; i += 64) {
      const int r = i / nc4, c = i - r * nc4;
      const int64_t e = e0 + 32 * rt + r;
      const int col4 = 8 * (c0 + g) + c;
      if (e < E && col4 < hv) {
        float4 o = *reinterpret_cast<const float4*>(&slab[r * kLDE + 4 * c]);
        if constexpr (!RESACC) {
          if (b4) o = o + b4[col4];
          if (residual) o = H4[e * hv + col4] + o;
        }
        O4[e * hv + col4] = o;
      }
    }
    __syncthreads();
  }
  if constexpr (ABL == 8) {
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < 5; ++i) atomicAdd(&g_x6_stamps[i], st[i]);
    }
  }
}

// Pre-split weight image: Wx[kb][nt][part][lane] = 8 bf16 (16 B), element j holding part `part`
// of W[n][k] with n = 32 nt + (lane & 31), k = 16 kb + 8 (lane >> 5) + j (zero outside [0,h)).
__global__ void __launch_bounds__(256) pack_x6(const float* __restrict__ W, int64_t nlayers,
                                               int64_t h, int KB, int NT32, int64_t layer_stride16,
                                               uint4* __restrict__ Wx) {
  const int64_t per_layer = (int64_t)KB * NT32 * 64;  // (kb, nt, lane) triples
  const int64_t total = nlayers * per_layer;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t l = t / per_layer;
    int64_t r = t - l * per_layer;
    const int lane = (int)(r & 63);
    r >>= 6;
    const int nt = (int)(r % NT32);
    const int kb = (int)(r / NT32);
    const int64_t n = 32 * nt + (lane & 31);
    const int64_t k0 = 16 * kb + 8 * (lane >> 5);
    const float* Wl = W + l * h * h;
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = (n < h && k0 + j < h) ? Wl[n * h + k0 + j] : 0.f;
    bf16x8 p[3];
    split3(x, p[0], p[1], p[2]);
    uint4* out = Wx + l * layer_stride16 + (((int64_t)kb * NT32 + nt) * 3) * 64 + lane;
#pragma unroll
    for (int part = 0; part < 3; ++part) out[part * 64] = *reinterpret_cast<const uint4*>(&p[part]);
  }
}

template <int NT32, int MW, int SHR, int WR, int ACT, int ABL = 0, bool RESACC = false>
int launch_x6(const UpdateArgs& a) {
  using G = X6Geom<NT32, MW>;
  const int64_t grid = (a.E + G::kRows - 1) / G::kRows;
  NT_REQUIRE(grid < (int64_t(1) << 31), NT_EINVAL, "too many edges");
  update_x6_kernel<NT32, MW, SHR, WR, ACT, ABL, RESACC><<<(unsigned)grid, G::kThreads, 0, a.stream>>>(
      (const float4*)a.H, (const float4*)a.S, a.src, a.rev, (const uint4*)a.Wp,
      (const float4*)a.b, a.V, a.E, (int)(a.h / 4), (int)((a.h + 15) / 16), a.residual, a.act,
      a.alpha, (float4*)a.H_out);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

// x6 configuration (rows per workgroup / gather ring depth); NT_X6_CFG overrides for A/B runs:
//   "a" = 64 rows, 2-slot rings   "b" = 128 rows, 2-slot rings
//   "c" = 128 rows, 3-slot S/H ring   "d" = 128 rows, 3-slot S/H and W rings
static char x6_cfg() {
#ifdef NT_DIAG
  const char* v = getenv("NT_X6_CFG");
  return (v && v[0]) ? v[0] : 'a';
#else
  return 'a';
#endif
}

// static LDS bytes of a configuration (must stay <= 160 KiB)
template <int NT32, int MW, int SHR, int WR>
constexpr int x6_lds_bytes() {
  using G = X6Geom<NT32, MW>;
  constexpr int wpw = (NT32 * 3 + G::kWaves - 1) / G::kWaves;
  constexpr int ws = WR == 3 ? wpw * G::kWaves * 256 : G::kW;
  return 4 * (SHR * G::kSH + WR * ws) + 16 * G::kRows;
}

template <int NT32, int ACT>
int launch_x6_cfg(const UpdateArgs& a) {
#ifdef NT_DIAG
  if constexpr (ACT == NT_ACT_RELU && X6Geom<NT32, 4>::kFits) {
    const char c = x6_cfg();
    if (c == 'b') return launch_x6<NT32, 4, 2, 2, ACT>(a);
    if (c == 'c') return launch_x6<NT32, 4, 3, 2, ACT>(a);
    if constexpr (x6_lds_bytes<NT32, 4, 3, 3>() <= 160 * 1024) {
      if (c == 'd') return launch_x6<NT32, 4, 3, 3, ACT>(a);
    }
    if constexpr (NT32 == 10) {  // ablation builds (timing only) of config 'a'
      if (c == '1') return launch_x6<NT32, 2, 2, 2, ACT, 1>(a);
      if (c == '2') return launch_x6<NT32, 2, 2, 2, ACT, 2>(a);
      if (c == '3') return launch_x6<NT32, 2, 2, 2, ACT, 3>(a);
      if (c == '4') return launch_x6<NT32, 2, 2, 2, ACT, 4>(a);
      if (c == '7') return launch_x6<NT32, 2, 2, 2, ACT, 7>(a);
      if (c == 'r') return launch_x6<NT32, 2, 2, 2, ACT, 0, true>(a);
      if (c == 's') return launch_x6<NT32, 2, 2, 2, ACT, 8>(a);
    }
  }
#endif
  return launch_x6<NT32, 2, 2, 2, ACT>(a);
}

template <int ACT, int... Ns>
int dispatch_x6(const UpdateArgs& a, int nt32, std::integer_sequence<int, Ns...>) {
  int rc = NT_EUNSUPPORTED;
  bool done = false;
  ((nt32 == Ns + 4 ? (rc = launch_x6_cfg<Ns + 4, ACT>(a), done = true) : false), ...);
  if (!done) set_error("nt_dmpnn_update: no bf16x6 kernel for this hidden size");
  return rc;
}

}  // namespace

int x6_nt32(int64_t h) { return (int)((h + 31) / 32); }

bool x6_supported(int64_t h) { return h % 4 == 0 && x6_nt32(h) >= 4 && x6_nt32(h) <= 16; }

size_t x6_image_bytes(int64_t h) {
  return (size_t)((h + 15) / 16) * x6_nt32(h) * 3 * 64 * 16;
}

int pack_weight_x6(const float* W, int64_t nlayers, int64_t h, int64_t layer_stride_bytes,
                   void* Wx, hipStream_t stream) {
  const int KB = (int)((h + 15) / 16), NT32 = x6_nt32(h);
  const int64_t total = nlayers * KB * NT32 * 64;
  pack_x6<<<grid_for(total, 256), 256, 0, stream>>>(W, nlayers, h, KB, NT32,
                                                    layer_stride_bytes / 16, (uint4*)Wx);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

int launch_update_x6(const UpdateArgs& a) {
  using Seq = std::make_integer_sequence<int, 13>;  // NT32 = 4 .. 16  (97 <= h <= 512)
  const int nt32 = x6_nt32(a.h);
  if (a.act == NT_ACT_RELU) return dispatch_x6<NT_ACT_RELU>(a, nt32, Seq{});
  return dispatch_x6<-1>(a, nt32, Seq{});
}

}  // namespace nt
#endif  // NT_DIAG

// Debug-only (not part of include/notorch_amd.h): read (and optionally reset) the stamp sums of the
#ifdef NT_DIAG
// diagnostic x6 build selected with NT_UPDATE_KERNEL=x6 NT_X6_CFG=s.
extern "C" __attribute__((visibility("default"))) int nt_debug_x6_stamps(unsigned long long* out5,
                                                                         int reset) {
  if (hipMemcpyFromSymbol(out5, HIP_SYMBOL(nt::g_x6_stamps), 5 * sizeof(unsigned long long), 0,
                          hipMemcpyDeviceToHost) != hipSuccess)
    return 2;
  if (reset) {
    unsigned long long z[8] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(nt::g_x6_stamps), z, sizeof(z), 0, hipMemcpyHostToDevice) !=
        hipSuccess)
      return 2;
  }
  return 0;
}
#endif  // NT_DIAG

// A-stationary D-MPNN layer update on bf16 MFMA with fp32 emulation ("as16"):
//
//   H_out[e] = (residual ? H[e] : 0) + W (S[src[e]] - act(H[rev[e]])) + b     (chemprop.py:36-43,
//                                                                               residual.py:27-28)
// Numerics are those of update_x6.hip (three-way bf16 split of both operands, six products
// a2.w0 + a1.w1 + a0.w2 + a1.w0 + a0.w1 + a0.w0 accumulated in fp32), on v_mfma_f32_16x16x32_bf16.
//
// Why a second design.  update_x6 streams S/H pieces and W chunks through LDS rings in 16-deep K
// chunks with a workgroup barrier per chunk; only 16 KiB of gathers are in flight per CU and the
// waves spend most of the launch parked on the barrier.  Here one workgroup (4 waves, 64 edges)
// runs three barrier-separated phases:
//   1. gather: the whole A tile, A[r][k] = S[src][k] - act(H[rev][k]) for 64 rows x 32*KS k, is
//      gathered with 16-B loads (all 64 rows in flight at once) and written to LDS in fp32.
//      The tile is 80 KiB, so two workgroups share a CU and one's gather overlaps the other's
//      MFMA phase.
//   2. MFMA: no barrier and no LDS traffic for W.  Wave w owns the 16-column tiles w, w+4, ...
//      (5 tiles at h = 300) for all 64 rows (20 accumulators); its W fragments come straight from
//      L2 into VGPRs (pre-split image, one 1 KiB coalesced load per tile x part x 32-deep step),
//      tile j of step ks+1 loaded as soon as tile j of step ks has issued its MFMAs.  A fragments
//      are read from LDS (conflict-free: 16-B piece p of row r lives in slot p ^ (r & 15)) and
//      split in registers.
//   3. epilogue: accumulators staged through the (now free) LDS tile, then + bias + residual and
//      row-contiguous 16-B stores.
// Supports h % 4 == 0, h <= 304 (the staging tile must fit the 80 KiB A tile).
#include <stdlib.h>

#include <type_traits>

#include "../common.hpp"
#include "../update.hpp"

#ifdef NT_DIAG  // A/B variant: superseded by update_fk_kernel in the shipping library
namespace nt {

// Diagnostic build (NT_AS_DIAG=1): per-wave phase cycles summed over waves: gather (incl. barrier),
// MFMA loop, staging (incl. barriers), stores; [4] = waves; [5]/[6] = min start / max end stamp.
__device__ unsigned long long g_as_stamps[8];

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kRows = 64;                   // edges per workgroup
constexpr int kThreads = 256;               // 4 waves
constexpr int kPieces = 80;                 // 16-B pieces per LDS A row (320 floats)
constexpr int kLdsF4 = kRows * kPieces;     // 5120 float4 = 80 KiB -> 2 workgroups per CU
constexpr int kSO = 308;                    // epilogue staging row stride (floats), == 4 mod 8
static_assert(kRows * kSO <= 4 * kLdsF4, "staging tile must fit the A tile");

__device__ __forceinline__ int a_slot(int r, int p) { return r * kPieces + (p ^ (r & 15)); }

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

// KS: 32-deep K steps (h <= 32 KS); CT: 16-column tiles per wave (tile ct = wave + 4 j).
__device__ __forceinline__ unsigned long long stamp_now() {
  unsigned long long t = 0;
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
#endif
  return t;
}

template <int KS, int ACT, bool DIAG = false>
__global__ void __launch_bounds__(kThreads, 2) update_as_kernel(
    const float4* __restrict__ H4, const float4* __restrict__ S4, const int64_t* __restrict__ src,
    const int64_t* __restrict__ rev, const uint4* __restrict__ Wb, const float4* __restrict__ b4,
    int64_t V, int64_t E, int hv, int nt16, int residual, int act, float alpha,
    float4* __restrict__ O4) {
  constexpr int CT = (KS + 1) / 2;
  constexpr int PR = 8 * KS;                 // pieces per row gathered (zero beyond hv)
  constexpr int NIT = kRows * PR / kThreads; // gather iterations per thread (PR % 4 == 0)
  static_assert(kRows * PR % kThreads == 0, "gather tiling");
  __shared__ __attribute__((aligned(16))) float4 lds[kLdsF4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t e0 = (int64_t)blockIdx.x * kRows;
  unsigned long long ts[5] = {0, 0, 0, 0, 0};
  if constexpr (DIAG) ts[0] = stamp_now();

  // ---- phase 1: gather the A tile into LDS (two batches bound the live registers) ----
  // Loads are unconditional (out-of-range rows/pieces read row 0 / piece 0 and are masked), so the
  // batch issues back to back without branches.
  constexpr int NB = (NIT + 1) / 2;
#pragma unroll
  for (int b0 = 0; b0 < NIT; b0 += NB) {
    float4 sv[NB], qv[NB];
    int fl[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (b0 + j < NIT) {
        const int i = tid + kThreads * (b0 + j);
        const int r = i / PR, c = i - r * PR;
        const int64_t e = e0 + r;
        const bool live = e < E && c < hv;
        const int64_t ec = live ? e : 0;
        const int64_t s = src[ec], q = rev[ec];
        const bool sok = live && s >= 0 && s < V, qok = live && q >= 0 && q < E;
        const int cc = live ? c : 0;
        sv[j] = S4[(sok ? s : 0) * hv + cc];
        qv[j] = H4[(qok ? q : 0) * hv + cc];
        fl[j] = (sok ? 1 : 0) | (qok ? 2 : 0);
      }
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (b0 + j < NIT) {
        const int i = tid + kThreads * (b0 + j);
        const int r = i / PR, c = i - r * PR;
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 m = (fl[j] & 2) ? act4_t<ACT>(qv[j], act, alpha) : z;
        lds[a_slot(r, c)] = ((fl[j] & 1) ? sv[j] : z) - m;
      }
    }
  }
  __syncthreads();
  if constexpr (DIAG) ts[1] = stamp_now();

  // ---- phase 2: 64 x (16 NC) accumulators per wave over 32-deep K steps ----
  f32x4 acc[4][CT];
#pragma unroll
  for (int rt = 0; rt < 4; ++rt)
#pragma unroll
    for (int j = 0; j < CT; ++j) acc[rt][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, fr = lane & 15;
  // image: Wb[ks][ct][part][lane]; this wave's tile j of step ks at ((ks nt16 + wave + 4j) 3 + p) 64
  const uint4* wl = Wb + (int64_t)wave * 3 * 64 + lane;
  const int64_t step_stride = (int64_t)nt16 * 3 * 64;

  auto body = [&](auto nc_tag) {
    constexpr int NC = decltype(nc_tag)::value;
    // Software pipeline per K step (sched_barriers pin the order; hipcc otherwise sinks the W
    // prefetches next to their use and waits on them inside the step):
    //   split this step's A fragments (read from LDS during the previous step)
    //   -> issue next step's A fragment reads
    //   -> per tile j: 24 MFMAs, then next step's 3 W loads of tile j into the freed registers
    uint4 bw[NC][3];
    float4 xa[4][2];
#pragma unroll
    for (int j = 0; j < NC; ++j)
#pragma unroll
      for (int p = 0; p < 3; ++p) bw[j][p] = wl[(4 * j * 3 + p) * 64];
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) {
      const int r = 16 * rt + fr, p = 2 * g;
      xa[rt][0] = lds[a_slot(r, p)];
      xa[rt][1] = lds[a_slot(r, p + 1)];
    }
#pragma unroll 1
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 a[4][3];
#pragma unroll
      for (int rt = 0; rt < 4; ++rt) {
        const float x[8] = {xa[rt][0].x, xa[rt][0].y, xa[rt][0].z, xa[rt][0].w,
                            xa[rt][1].x, xa[rt][1].y, xa[rt][1].z, xa[rt][1].w};
        split3(x, a[rt][0], a[rt][1], a[rt][2]);
      }
      const int kn = ks + 1 < KS ? ks + 1 : ks;  // last step re-reads its own (no branch)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int rt = 0; rt < 4; ++rt) {
        const int r = 16 * rt + fr, p = 8 * kn + 2 * g;
        xa[rt][0] = lds[a_slot(r, p)];
        xa[rt][1] = lds[a_slot(r, p + 1)];
      }
      const uint4* wn = wl + kn * step_stride;
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        __builtin_amdgcn_sched_barrier(0);
        const bf16x8 w0 = as_bf16x8(bw[j][0]), w1 = as_bf16x8(bw[j][1]), w2 = as_bf16x8(bw[j][2]);
#pragma unroll
        for (int rt = 0; rt < 4; ++rt) {
          f32x4 c = acc[rt][j];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rt][2], w0, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rt][1], w1, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rt][0], w2, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rt][1], w0, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rt][0], w1, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rt][0], w0, c, 0, 0, 0);
          acc[rt][j] = c;
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int p = 0; p < 3; ++p) bw[j][p] = wn[(4 * j * 3 + p) * 64];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  const int nc = (nt16 - wave + 3) / 4;  // valid tiles of this wave (wave-uniform)
  if (nc >= CT) body(std::integral_constant<int, CT>{});
  else if constexpr (CT > 1) body(std::integral_constant<int, CT - 1>{});

  // ---- phase 3: stage through LDS, + bias + residual, row-contiguous stores ----
  if constexpr (DIAG) ts[2] = stamp_now();
  __syncthreads();  // every wave is done reading the A tile
  float* so = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int j = 0; j < CT; ++j) {
    if (j < nc) {
      const int col = 16 * (wave + 4 * j) + fr;
#pragma unroll
      for (int rt = 0; rt < 4; ++rt)
#pragma unroll
        for (int i = 0; i < 4; ++i) so[(16 * rt + 4 * g + i) * kSO + col] = acc[rt][j][i];
    }
  }
  __syncthreads();
  if constexpr (DIAG) ts[3] = stamp_now();
#pragma unroll 2
  for (int it = 0; it < NIT; ++it) {
    const int i = tid + kThreads * it;
    const int r = i / PR, c = i - r * PR;
    const int64_t e = e0 + r;
    if (e < E && c < hv) {
      float4 o = *reinterpret_cast<const float4*>(&so[r * kSO + 4 * c]);
      if (b4) o = o + b4[c];
      if (residual) o = H4[e * hv + c] + o;
      O4[e * hv + c] = o;
    }
  }
  if constexpr (DIAG) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ts[4] = stamp_now();
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) atomicAdd(&g_as_stamps[i], ts[i + 1] - ts[i]);
      atomicAdd(&g_as_stamps[4], 1ull);
      atomicMin(&g_as_stamps[5], ts[0]);
      atomicMax(&g_as_stamps[6], ts[4]);
    }
  }
}

// Pre-split weight image: Wb[kstep][ct][part][lane] = 8 bf16 (16 B), element j holding part `part`
// of W[n][k] with n = 16 ct + (lane & 15), k = 32 kstep + 8 (lane >> 4) + j (zero outside [0,h)).
__global__ void __launch_bounds__(256) pack_as(const float* __restrict__ W, int64_t nlayers,
                                               int64_t h, int KS, int NT16, int64_t layer_stride16,
                                               uint4* __restrict__ Wb) {
  const int64_t per_layer = (int64_t)KS * NT16 * 64;
  const int64_t total = nlayers * per_layer;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t l = t / per_layer;
    int64_t r = t - l * per_layer;
    const int lane = (int)(r & 63);
    r >>= 6;
    const int ct = (int)(r % NT16);
    const int ks = (int)(r / NT16);
    const int64_t n = 16 * ct + (lane & 15);
    const int64_t k0 = 32 * ks + 8 * (lane >> 4);
    const float* Wl = W + l * h * h;
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = (n < h && k0 + j < h) ? Wl[n * h + k0 + j] : 0.f;
    bf16x8 p[3];
    split3(x, p[0], p[1], p[2]);
    uint4* out = Wb + l * layer_stride16 + (((int64_t)ks * NT16 + ct) * 3) * 64 + lane;
#pragma unroll
    for (int part = 0; part < 3; ++part) out[part * 64] = __builtin_bit_cast(uint4, p[part]);
  }
}

template <int KS, int ACT>
int launch_as(const UpdateArgs& a) {
  const int64_t grid = (a.E + kRows - 1) / kRows;
  NT_REQUIRE(grid < (int64_t(1) << 31), NT_EINVAL, "too many edges");
  auto kern = update_as_kernel<KS, ACT>;
#ifdef NT_DIAG
  const char* dg = getenv("NT_AS_DIAG");
  if (dg && dg[0] == '1') kern = update_as_kernel<KS, ACT, true>;
#endif
  kern<<<(unsigned)grid, kThreads, 0, a.stream>>>(
      (const float4*)a.H, (const float4*)a.S, a.src, a.rev, (const uint4*)a.Wp,
      (const float4*)a.b, a.V, a.E, (int)(a.h / 4), (int)((a.h + 15) / 16), a.residual, a.act,
      a.alpha, (float4*)a.H_out);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

template <int ACT, int... Ks>
int dispatch_as(const UpdateArgs& a, int ks, std::integer_sequence<int, Ks...>) {
  int rc = NT_EUNSUPPORTED;
  bool done = false;
  ((ks == Ks + 1 ? (rc = launch_as<Ks + 1, ACT>(a), done = true) : false), ...);
  if (!done) set_error("nt_dmpnn_update: no as16 kernel for this hidden size");
  return rc;
}

}  // namespace

bool as_supported(int64_t h) { return h % 4 == 0 && h >= 4 && h <= 304; }

size_t as_image_bytes(int64_t h) {
  const int64_t ks = (h + 31) / 32, nt16 = (h + 15) / 16;
  return (size_t)(ks * nt16 * 3 * 64 * 16);
}

int pack_weight_as(const float* W, int64_t nlayers, int64_t h, int64_t layer_stride_bytes,
                   void* Wb, hipStream_t stream) {
  const int KS = (int)((h + 31) / 32), NT16 = (int)((h + 15) / 16);
  const int64_t total = nlayers * KS * NT16 * 64;
  pack_as<<<grid_for(total, 256), 256, 0, stream>>>(W, nlayers, h, KS, NT16,
                                                    layer_stride_bytes / 16, (uint4*)Wb);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

int launch_update_as(const UpdateArgs& a) {
  using Seq = std::make_integer_sequence<int, 10>;  // KS = 1 .. 10  (h <= 304)
  const int ks = (int)((a.h + 31) / 32);
  if (a.act == NT_ACT_RELU) return dispatch_as<NT_ACT_RELU>(a, ks, Seq{});
  return dispatch_as<-1>(a, ks, Seq{});
}

}  // namespace nt
#endif  // NT_DIAG

// Debug-only (not part of include/notorch_amd.h): read (and optionally reset) the stamp sums of the
#ifdef NT_DIAG
// diagnostic as16 build (NT_AS_DIAG=1).
extern "C" __attribute__((visibility("default"))) int nt_debug_as_stamps(unsigned long long* out7,
                                                                         int reset) {
  if (hipMemcpyFromSymbol(out7, HIP_SYMBOL(nt::g_as_stamps), 7 * sizeof(unsigned long long), 0,
                          hipMemcpyDeviceToHost) != hipSuccess)
    return 2;
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, ~0ull, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(nt::g_as_stamps), z, sizeof(z), 0, hipMemcpyHostToDevice) !=
        hipSuccess)
      return 2;
  }
  return 0;
}
#endif  // NT_DIAG

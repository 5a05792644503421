// Fused D-MPNN layer update on fp32 MFMA (v_mfma_f32_16x16x4_f32, exact f32 fma chain):
//
//   H_out[e] = (residual ? H[e] : 0) + W (S[src[e]] - act(H[rev[e]])) + b
//
// = ChempropLayer.forward (notorch/nn/gnn/chemprop.py:36-43: gather-sub at :40, nn.Linear at :41)
//   wrapped in Residual (notorch/nn/residual.py:27-28).  One launch per layer replaces the
//   reference's two gathers, a subtract, an addmm, a bias add and the residual add.
//
// Tiling (one workgroup = 4 waves = 256 lanes, BM edges x all h output columns):
//   1. gather: the BM rows A[r] = S[src[e0+r]] - act(H[rev[e0+r]]) are formed in registers from
//      16-B-per-lane coalesced row reads and written to an LDS tile [BM][Kpad+8] (the +8 float pad
//      makes the ds_read_b128 fragment reads bank-conflict-free).  rev is an
//      arbitrary gather index (the reference collate does not produce rev = e^1, graph.py:200).
//   2. MFMA: wave w owns output column tiles [w*CPW, (w+1)*CPW) x all BM rows.  Per 16-deep k
//      block a lane reads its A fragments with one ds_read_b128 per 16-row tile and its B
//      fragments with one global_load_dwordx4 per column tile from the pre-packed weight image
//      (L2-resident, 1 KiB per wave-instruction, prefetched one k-block ahead).  The 16-deep k
//      block is consumed as 4 MFMAs whose k-lanes are permuted identically in A and B (lane group
//      g = lane>>4 takes k = 16kb + 4g + s at step s), which lets both operands be 16-B vectors.
//   3. epilogue: the accumulators go through LDS (reusing the A tile) so that bias, residual and
//      the store are done with 16-B coalesced row accesses.
//
// Roofline: 2*h^2 flop per edge (MFMA) against (3 rows read + 1 row written) * 4h bytes per edge;
// at h = 300 that is 51 flop/B > the fp32 ridge (~20), i.e. bound by the 157 TF fp32 MFMA peak.
#include <stdlib.h>

#include <type_traits>

#include "common.hpp"
#include "bf16.hpp"
#include <string.h>

#include "update.hpp"

namespace nt {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kWaves = 4;

// kernel selection for A/B runs (read per call):
//   NT_UPDATE_KERNEL = as (default: A-stationary bf16x6) | x6 (LDS-ring bf16x6)
//                      | stream | tile (exact fp32 MFMA)
#ifdef NT_DIAG
static char update_kernel_choice() {
#ifdef NT_DIAG
  const char* v = getenv("NT_UPDATE_KERNEL");
  return (v && v[0]) ? v[0] : 'a';
#else
  return 'a';
#endif
}
#endif

struct UpdateGeom {
  int KB;   // 16-deep k blocks (Kpad = 16*KB >= h)
  int NT;   // 16-wide output column tiles (Npad = 16*NT >= h)
  int CPW;  // column tiles per wave = ceil(NT / 4)
  int LDA;  // LDS row stride of the A tile (floats)
  int LDO;  // LDS row stride of the output tile (floats)
};

static UpdateGeom geom_for(int64_t h) {
  UpdateGeom g;
  g.KB = (int)((h + 15) / 16);
  g.NT = g.KB;
  g.CPW = (g.NT + kWaves - 1) / kWaves;
  g.LDA = g.KB * 16 + 8;  // == 8 (mod 16): conflict-free ds_read_b128 fragment reads
  g.LDO = g.NT * 16 + 4;  // == 4 (mod 8): conflict-free ds_write_b32 of the 16x16 C layout
  return g;
}

template <int BM>
static size_t lds_bytes(const UpdateGeom& g) {
  size_t tile = (size_t)BM * (size_t)(g.LDA > g.LDO ? g.LDA : g.LDO) * sizeof(float);
  return tile + (size_t)BM * 2 * sizeof(int64_t);
}

// Packed weight image: Wp[kb][nt][lane] is a float4 whose element j is W[n][k] with
// n = 16nt + (lane & 15), k = 16kb + 4(lane >> 4) + j (zero outside [0,h)).  nn.Linear stores
// W as [out][in] (chemprop.py:26), so y = A W^T means B[k][n] = W[n][k].
__global__ void __launch_bounds__(256) pack_weight_f32(const float* __restrict__ W, int64_t nlayers,
                                                       int64_t h, int KB, int NT,
                                                       float4* __restrict__ Wp) {
  const int64_t per_layer = (int64_t)KB * NT * 64;
  const int64_t total = nlayers * per_layer;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t l = t / per_layer;
    int64_t r = t - l * per_layer;
    const int lane = (int)(r & 63);
    r >>= 6;
    const int nt = (int)(r % NT);
    const int kb = (int)(r / NT);
    const int64_t n = 16 * nt + (lane & 15);
    const int64_t k0 = 16 * kb + 4 * (lane >> 4);
    const float* Wl = W + l * h * h;
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = (n < h && k0 + j < h) ? Wl[n * h + k0 + j] : 0.f;
    Wp[t] = make_float4(v[0], v[1], v[2], v[3]);
  }
}

template <int BM, int CPW, int ACT, bool VEC>
__global__ void __launch_bounds__(kThreads, 2) dmpnn_update_f32(
    const float* __restrict__ H, const float* __restrict__ S, const int64_t* __restrict__ src,
    const int64_t* __restrict__ rev, const float4* __restrict__ Wp, const float* __restrict__ bias,
    int64_t V, int64_t E, int h, int KB, int NT, int LDA, int LDO, int residual, int act,
    float alpha, float* __restrict__ H_out) {
  constexpr int MT = BM / 16;  // 16-row tiles per workgroup
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int64_t e0 = (int64_t)blockIdx.x * BM;
  const int tile_floats = BM * (LDA > LDO ? LDA : LDO);
  int64_t* s_src = reinterpret_cast<int64_t*>(smem + tile_floats);
  int64_t* s_rev = s_src + BM;

  // ---- 0. edge indices of this tile -> LDS (out-of-range indices become -1 = zero row) ----
  if (tid < BM) {
    const int64_t e = e0 + tid;
    int64_t s = -1, q = -1;
    if (e < E) {
      s = src[e];
      q = rev[e];
      if (s < 0 || s >= V) s = -1;
      if (q < 0 || q >= E) q = -1;
    }
    s_src[tid] = s;
    s_rev[tid] = q;
  }
  __syncthreads();

  // ---- 1. gather A = S[src] - act(H[rev]) into the LDS tile (k padded with zeros to 16*KB) ----
  if constexpr (VEC) {
    const int kv = KB * 4;  // float4 chunks per padded row
    const int hv = h >> 2;
    const float4* S4 = reinterpret_cast<const float4*>(S);
    const float4* H4 = reinterpret_cast<const float4*>(H);
    for (int i = tid; i < BM * kv; i += kThreads) {
      const int r = i / kv;
      const int c = i - r * kv;
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
      if (c < hv) {
        const int64_t s = s_src[r], q = s_rev[r];
        const float4 sv = s >= 0 ? S4[s * hv + c] : a;
        const float4 mv = q >= 0 ? act4_t<ACT>(H4[q * hv + c], act, alpha) : a;
        a = sv - mv;
      }
      *reinterpret_cast<float4*>(&smem[r * LDA + 4 * c]) = a;
    }
  } else {
    const int kp = KB * 16;
    for (int i = tid; i < BM * kp; i += kThreads) {
      const int r = i / kp;
      const int c = i - r * kp;
      float a = 0.f;
      if (c < h) {
        const int64_t s = s_src[r], q = s_rev[r];
        const float sv = s >= 0 ? S[s * h + c] : 0.f;
        const float mv = q >= 0 ? act_t<ACT>(H[q * h + c], act, alpha) : 0.f;
        a = sv - mv;
      }
      smem[r * LDA + c] = a;
    }
  }
  __syncthreads();

  // ---- 2. MFMA: acc[mt][ct] += A[16mt.., k] * B[k, 16(nt0+ct)..] ----
  const int nt0 = wave * CPW;
  f32x4 acc[MT][CPW];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int ct = 0; ct < CPW; ++ct) acc[mt][ct] = f32x4{0.f, 0.f, 0.f, 0.f};

  float4 bcur[CPW], bnext[CPW];
#pragma unroll
  for (int ct = 0; ct < CPW; ++ct) {
    const int nt = nt0 + ct;
    bcur[ct] = nt < NT ? Wp[(int64_t)nt * 64 + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const float* a_base = smem + (lane & 15) * LDA + 4 * (lane >> 4);
  for (int kb = 0; kb < KB; ++kb) {
    if (kb + 1 < KB) {
#pragma unroll
      for (int ct = 0; ct < CPW; ++ct) {
        const int nt = nt0 + ct;
        bnext[ct] = nt < NT ? Wp[((int64_t)(kb + 1) * NT + nt) * 64 + lane]
                            : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    float4 a[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
      a[mt] = *reinterpret_cast<const float4*>(a_base + mt * 16 * LDA + 16 * kb);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const float av = s == 0 ? a[mt].x : s == 1 ? a[mt].y : s == 2 ? a[mt].z : a[mt].w;
#pragma unroll
        for (int ct = 0; ct < CPW; ++ct) {
          const float bv = s == 0 ? bcur[ct].x : s == 1 ? bcur[ct].y : s == 2 ? bcur[ct].z : bcur[ct].w;
          acc[mt][ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[mt][ct], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int ct = 0; ct < CPW; ++ct) bcur[ct] = bnext[ct];
  }
  __syncthreads();  // every wave is done reading the A tile

  // ---- 3. epilogue: C fragments -> LDS (C/D map: col = lane&15, row = 4*(lane>>4) + j) ----
#pragma unroll
  for (int ct = 0; ct < CPW; ++ct) {
    const int nt = nt0 + ct;
    if (nt < NT) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = 16 * mt + 4 * (lane >> 4) + j;
          smem[row * LDO + 16 * nt + (lane & 15)] = acc[mt][ct][j];
        }
      }
    }
  }
  __syncthreads();

  if constexpr (VEC) {
    const int hv = h >> 2;
    const float4* H4 = reinterpret_cast<const float4*>(H);
    const float4* b4 = reinterpret_cast<const float4*>(bias);
    float4* O4 = reinterpret_cast<float4*>(H_out);
    for (int i = tid; i < BM * hv; i += kThreads) {
      const int r = i / hv;
      const int c = i - r * hv;
      const int64_t e = e0 + r;
      if (e < E) {
        float4 o = *reinterpret_cast<const float4*>(&smem[r * LDO + 4 * c]);
        if (bias) o = o + b4[c];
        if (residual) o = H4[e * hv + c] + o;
        O4[e * hv + c] = o;
      }
    }
  } else {
    for (int i = tid; i < BM * h; i += kThreads) {
      const int r = i / h;
      const int c = i - r * h;
      const int64_t e = e0 + r;
      if (e < E) {
        float o = smem[r * LDO + c];
        if (bias) o = o + bias[c];
        if (residual) o = H[e * h + c] + o;
        H_out[e * h + c] = o;
      }
    }
  }
}


// ------------------------------------------------------------------------------------------
// Streamed variant (h % 4 == 0): the A tile is never materialised whole.  K advances in 16-deep
// chunks through a 2-slot LDS ring (64 rows x 16 k, 6 KiB per slot); while the MFMAs consume
// chunk k, the gathered S/H pieces of chunk k+1 wait in registers to be combined and written, and
// the loads of chunk k+2 are in flight.  One workgroup barrier per chunk.  ~23 KiB of LDS and
// <= 168 VGPRs give 3 workgroups per CU, so a CU interleaves several tiles' gathers and MFMAs.
// Column tiles are dealt to waves as evenly as possible (ceil / floor), and a wave only issues
// MFMAs for real tiles (no padding tiles).  Epilogue: per 16-row tile, each wave stages its
// C fragments in a wave-private LDS slab and stores whole 16-B row pieces (+bias +residual).
// ------------------------------------------------------------------------------------------
#ifdef NT_DIAG  // A/B-only streamed variant (make DIAG=1)
#ifndef NT_STREAM_WAVES
#define NT_STREAM_WAVES 2  // min waves per SIMD the streamed kernel is register-allocated for
#endif
constexpr int kBM2 = 64;   // edges per workgroup
constexpr int kLDA2 = 24;  // ring row stride (floats): == 8 (mod 16) -> conflict-free b128 reads

template <int CPW>
struct Stream2Lds {
  static constexpr int kRing = 2 * kBM2 * kLDA2;                 // floats
  static constexpr int kLDE = 16 * CPW + 4;                      // == 4 (mod 8)
  static constexpr int kEpi = kWaves * 16 * kLDE;                // floats
  static constexpr int kFloats = (kRing > kEpi ? kRing : kEpi);
};

template <int NC, int CPW>
__device__ __forceinline__ void mfma_chunk(f32x4 (&acc)[4][CPW], const float4 (&a)[4],
                                           const float4* b) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const float av = s == 0 ? a[mt].x : s == 1 ? a[mt].y : s == 2 ? a[mt].z : a[mt].w;
#pragma unroll
      for (int ct = 0; ct < NC; ++ct) {
        const float bv = s == 0 ? b[ct].x : s == 1 ? b[ct].y : s == 2 ? b[ct].z : b[ct].w;
        acc[mt][ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[mt][ct], 0, 0, 0);
      }
    }
  }
}

template <int CPW, int ACT>
__global__ void __launch_bounds__(kThreads, NT_STREAM_WAVES) dmpnn_update_f32_stream(
    const float4* __restrict__ H4, const float4* __restrict__ S4, const int64_t* __restrict__ src,
    const int64_t* __restrict__ rev, const float4* __restrict__ Wp, const float4* __restrict__ b4,
    int64_t V, int64_t E, int hv, int KB, int NT, int residual, int act, float alpha,
    float4* __restrict__ O4) {
  using L = Stream2Lds<CPW>;
  __shared__ __attribute__((aligned(16))) float smem[L::kFloats];
  __shared__ int64_t s_src[kBM2], s_rev[kBM2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t e0 = (int64_t)blockIdx.x * kBM2;

  if (tid < kBM2) {
    const int64_t e = e0 + tid;
    int64_t s = -1, q = -1;
    if (e < E) {
      s = src[e];
      q = rev[e];
      s = (s >= 0 && s < V) ? s * hv : -1;  // store float4 row offsets
      q = (q >= 0 && q < E) ? q * hv : -1;
    }
    s_src[tid] = s;
    s_rev[tid] = q;
  }
  // column tiles of this wave: ceil/floor split of NT over the 4 waves
  const int base = NT >> 2, rem = NT & 3;
  const int ncol = base + (wave < rem ? 1 : 0);
  const int nt0 = wave * base + (wave < rem ? wave : rem);
  __syncthreads();

  // gather role of this lane: row gr, 16-B piece gc of the 64-B chunk row.  Loads are issued
  // unconditionally from a clamped (always valid) address and masked afterwards, so the compiler
  // emits plain global_load_dwordx4 with no exec-mask branches around them.
  const int gr = tid >> 2, gc = tid & 3;
  const int64_t gs_raw = s_src[gr], gq_raw = s_rev[gr];
  const bool gs_ok = gs_raw >= 0, gq_ok = gq_raw >= 0;
  const int64_t gs = gs_ok ? gs_raw : 0, gq = gq_ok ? gq_raw : 0;
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
  // validity masks are applied when the chunk is consumed (put_chunk), never right after the
  // load: a select on freshly loaded registers forces an early s_waitcnt and kills the prefetch.
  auto load_chunk = [&](int kb, float4& sv, float4& hq) {
    const int c = kb * 4 + gc;
    const int cc = c < hv ? c : hv - 1;
    sv = S4[gs + cc];
    hq = H4[gq + cc];
  };
  auto put_chunk = [&](int kb, const float4& sv, const float4& hq) {
    const bool in = kb * 4 + gc < hv;
    float4 a = (in && gs_ok ? sv : zero4) - (in && gq_ok ? act4_t<ACT>(hq, act, alpha) : zero4);
    *reinterpret_cast<float4*>(&smem[(kb & 1) * kBM2 * kLDA2 + gr * kLDA2 + 4 * gc]) = a;
  };

  f32x4 acc[4][CPW];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int ct = 0; ct < CPW; ++ct) acc[mt][ct] = f32x4{0.f, 0.f, 0.f, 0.f};

  float4 sv, hq;
  load_chunk(0, sv, hq);
  put_chunk(0, sv, hq);
  if (KB > 1) load_chunk(1, sv, hq);
  __syncthreads();

  const float* a_base = smem + (lane & 15) * kLDA2 + 4 * (lane >> 4);
  const float4* wp_lane = Wp + (int64_t)nt0 * 64 + lane;
  // main loop, specialised on this wave's (wave-uniform) column-tile count NC
  auto main_loop = [&](auto nc_tag) {
    constexpr int NC = decltype(nc_tag)::value;
    float4 b0[NC > 0 ? NC : 1], b1[NC > 0 ? NC : 1];
    auto load_b = [&](int kb, float4(&b)[NC > 0 ? NC : 1]) {
#pragma unroll
      for (int ct = 0; ct < NC; ++ct) b[ct] = wp_lane[((int64_t)kb * NT + ct) * 64];
    };
    // one k-chunk: prefetch B(kb+1) into bn, MFMA on chunk kb with bc, restage the ring
    auto step = [&](int kb, float4(&bc)[NC > 0 ? NC : 1], float4(&bn)[NC > 0 ? NC : 1]) {
      if (kb + 1 < KB) load_b(kb + 1, bn);
      const float* ab = a_base + (kb & 1) * kBM2 * kLDA2;
      float4 a[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) a[mt] = *reinterpret_cast<const float4*>(ab + mt * 16 * kLDA2);
      if constexpr (NC > 0) mfma_chunk<NC, CPW>(acc, a, bc);
      if (kb + 1 < KB) {
        put_chunk(kb + 1, sv, hq);
        if (kb + 2 < KB) load_chunk(kb + 2, sv, hq);
      }
      __syncthreads();
    };
    load_b(0, b0);
    int kb = 0;
    for (; kb + 1 < KB; kb += 2) {  // unrolled by two: B registers ping-pong, no copies
      step(kb, b0, b1);
      step(kb + 1, b1, b0);
    }
    if (kb < KB) step(kb, b0, b1);
  };
  if (ncol == CPW) main_loop(std::integral_constant<int, CPW>{});
  else main_loop(std::integral_constant<int, (CPW > 0 ? CPW - 1 : 0)>{});

  // ---- epilogue: per 16-row tile, wave-private LDS slab -> 16-B row pieces ----
  float* slab = smem + wave * 16 * L::kLDE;
  const int nc4 = ncol * 4;  // float4 columns of this wave
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
    for (int ct = 0; ct < CPW; ++ct) {
      if (ct < ncol) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          slab[(4 * (lane >> 4) + j) * L::kLDE + 16 * ct + (lane & 15)] = acc[mt][ct][j];
      }
    }
    __syncthreads();
    for (int i = lane; i < 16 * nc4; i += 64) {
      const int r = i / nc4, c = i - r * nc4;
      const int64_t e = e0 + 16 * mt + r;
      const int col4 = nt0 * 4 + c;
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

template <int CPW, int ACT>
static int launch_stream(const float* H, const float* S, const int64_t* src, const int64_t* rev,
                         const float4* Wp, const float* b, int64_t V, int64_t E, int h,
                         const UpdateGeom& g, int residual, int act, float alpha, float* H_out,
                         hipStream_t stream) {
  const int64_t grid = (E + kBM2 - 1) / kBM2;
  NT_REQUIRE(grid < (int64_t(1) << 31), NT_EINVAL, "too many edges");
  dmpnn_update_f32_stream<CPW, ACT><<<(unsigned)grid, kThreads, 0, stream>>>(
      (const float4*)H, (const float4*)S, src, rev, Wp, (const float4*)b, V, E, h / 4, g.KB, g.NT,
      residual, act, alpha, (float4*)H_out);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

#endif  // NT_DIAG

template <int BM, int CPW, int ACT, bool VEC>
static int launch_update(const float* H, const float* S, const int64_t* src, const int64_t* rev,
                         const float4* Wp, const float* b, int64_t V, int64_t E, int h,
                         const UpdateGeom& g, int residual, int act, float alpha, float* H_out,
                         hipStream_t stream) {
  const size_t lds = lds_bytes<BM>(g);
  NT_REQUIRE(lds <= 160 * 1024, NT_EUNSUPPORTED, "hidden size too large for the LDS tile");
  auto kern = dmpnn_update_f32<BM, CPW, ACT, VEC>;
  if (lds > 64 * 1024) NT_HIP(hipFuncSetAttribute((const void*)kern,
                                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                                  (int)lds));
  const int64_t grid = (E + BM - 1) / BM;
  NT_REQUIRE(grid < (int64_t(1) << 31), NT_EINVAL, "too many edges");
  kern<<<(unsigned)grid, kThreads, lds, stream>>>(H, S, src, rev, Wp, b, V, E, h, g.KB, g.NT,
                                                  g.LDA, g.LDO, residual, act, alpha, H_out);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

template <int BM, int CPW>
static int dispatch_act_vec(const float* H, const float* S, const int64_t* src, const int64_t* rev,
                            const float4* Wp, const float* b, int64_t V, int64_t E, int h,
                            const UpdateGeom& g, int residual, int act, float alpha, float* H_out,
                            bool vec, hipStream_t stream) {
#ifdef NT_DIAG
  if (vec && update_kernel_choice() == 's') {
    return act == NT_ACT_RELU
               ? launch_stream<CPW, NT_ACT_RELU>(H, S, src, rev, Wp, b, V, E, h, g, residual, act,
                                                 alpha, H_out, stream)
               : launch_stream<CPW, -1>(H, S, src, rev, Wp, b, V, E, h, g, residual, act, alpha,
                                        H_out, stream);
  }
#endif
  if (act == NT_ACT_RELU) {
    return vec ? launch_update<BM, CPW, NT_ACT_RELU, true>(H, S, src, rev, Wp, b, V, E, h, g,
                                                           residual, act, alpha, H_out, stream)
               : launch_update<BM, CPW, NT_ACT_RELU, false>(H, S, src, rev, Wp, b, V, E, h, g,
                                                            residual, act, alpha, H_out, stream);
  }
  return vec ? launch_update<BM, CPW, -1, true>(H, S, src, rev, Wp, b, V, E, h, g, residual, act,
                                                alpha, H_out, stream)
             : launch_update<BM, CPW, -1, false>(H, S, src, rev, Wp, b, V, E, h, g, residual, act,
                                                 alpha, H_out, stream);
}

template <int BM>
static int dispatch_cpw(const float* H, const float* S, const int64_t* src, const int64_t* rev,
                        const float4* Wp, const float* b, int64_t V, int64_t E, int h,
                        const UpdateGeom& g, int residual, int act, float alpha, float* H_out,
                        bool vec, hipStream_t stream) {
  set_last_kernel("update_f32_tile_kernel: exact fp32 MFMA tiles (h % 4 != 0)");
#define NT_CASE(C)                                                                          \
  case C:                                                                                   \
    return dispatch_act_vec<BM, C>(H, S, src, rev, Wp, b, V, E, h, g, residual, act, alpha, \
                                   H_out, vec, stream);
  switch (g.CPW) {
    NT_CASE(1) NT_CASE(2) NT_CASE(3) NT_CASE(4) NT_CASE(5) NT_CASE(6) NT_CASE(7) NT_CASE(8)
    default:
      set_error("nt_dmpnn_update: hidden size > 512 is not supported by the fp32 MFMA kernel");
      return NT_EUNSUPPORTED;
  }
#undef NT_CASE
}

}  // namespace nt

// Packed image per layer (fp32 weights).  Shipping library: h % 4 == 0 (or h > 512) carries only the
// fk image (two-part fp16, 16x16x32 MFMA, scale header: every fp32 update, fused or not, and the
// backward's dense dA run on update_fk_kernel); other h <= 512 carry only the fp32 fragment image of
// the exact fp32 tile kernel (16x16x4 MFMA; the one kernel for h % 4 != 0).  Diagnostic library (A/B
// variants): [fp32 fragment image][bf16x6 image (32x32x16)][bf16x6 image (16x16x32)][fk image], each
// part 256-B aligned; the variant picks the part it consumes.
static bool has_fk_image(int64_t h) {
#ifdef NT_DIAG
  (void)h;
  return true;
#else
  return h % 4 == 0 || h > 512;
#endif
}
static size_t f32_image_bytes(int64_t h) {
  if (h > 512) return 0;
#ifndef NT_DIAG
  if (h % 4 == 0) return 0;
#endif
  const nt::UpdateGeom g = nt::geom_for(h);
  return ((size_t)g.KB * g.NT * 64 * sizeof(float4) + 255) & ~size_t(255);
}
#ifdef NT_DIAG
static size_t x6_part_bytes(int64_t h) {
  return nt::x6_supported(h) ? ((nt::x6_image_bytes(h) + 255) & ~size_t(255)) : 0;
}

static size_t as_part_bytes(int64_t h) {
  return nt::as_supported(h) ? ((nt::as_image_bytes(h) + 255) & ~size_t(255)) : 0;
}
#else
static size_t x6_part_bytes(int64_t) { return 0; }
static size_t as_part_bytes(int64_t) { return 0; }
#endif

static size_t fk_offset(int64_t h) { return f32_image_bytes(h) + x6_part_bytes(h) + as_part_bytes(h); }

// bf16 layer kernel: the fk skeleton (NT_BF16_KERNEL=fk / fk4, read once) or the 64-row bf16 kernel
static bool bf16_fk(int64_t h) { return nt::bf16_kernel_env() != 0 && nt::fkb_supported(h); }

extern "C" size_t nt_dmpnn_packed_weight_bytes(int64_t h, int dtype) {
  if (h <= 0) return 0;
  if (dtype == NT_BF16) return (nt::bf16_image_bytes(h) + 255) & ~size_t(255);
  return fk_offset(h) + (has_fk_image(h) ? (((size_t)nt::fk_image_bytes(h) + 255) & ~size_t(255)) : 0);
}

extern "C" int nt_dmpnn_pack_weight(const void* W, int64_t nlayers, int64_t h, int dtype, void* Wp,
                                    void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32 || dtype == NT_BF16, NT_EUNSUPPORTED, "dtype must be NT_F32 or NT_BF16");
  NT_REQUIRE(nlayers >= 0 && h > 0 && (dtype == NT_F32 || h <= 512) && h <= 8192, NT_EINVAL,
             "bad sizes (1 <= h <= 512 for bf16, <= 8192 for fp32)");
  if (nlayers == 0) return NT_OK;
  NT_REQUIRE(W && Wp && aligned16(Wp), NT_EINVAL, "NULL or misaligned pointer");
  if (dtype == NT_BF16)
    return pack_weight_bf16(W, nlayers, h, (int64_t)nt_dmpnn_packed_weight_bytes(h, dtype), Wp,
                            as_stream(stream_));
  const size_t per_layer = nt_dmpnn_packed_weight_bytes(h, dtype);
  NT_REQUIRE(per_layer % 16 == 0, NT_EINVAL, "internal: packed layer size");
  hipStream_t stream = as_stream(stream_);
  if (f32_image_bytes(h) > 0) {
    const UpdateGeom g = geom_for(h);
    // fp32 image of every layer (layer stride = per_layer bytes)
    for (int64_t l = 0; l < nlayers; ++l) {
      const int64_t total = (int64_t)g.KB * g.NT * 64;
      pack_weight_f32<<<grid_for(total, 256), 256, 0, stream>>>(
          (const float*)W + l * h * h, 1, h, g.KB, g.NT,
          (float4*)((char*)Wp + l * per_layer));
      NT_LAUNCH_CHECK();
    }
  }
#ifdef NT_DIAG
  if (x6_supported(h)) {
    int rc = pack_weight_x6((const float*)W, nlayers, h, (int64_t)per_layer,
                            (char*)Wp + f32_image_bytes(h), stream);
    if (rc != NT_OK) return rc;
  }
  if (as_supported(h)) {
    int rc = pack_weight_as((const float*)W, nlayers, h, (int64_t)per_layer,
                            (char*)Wp + f32_image_bytes(h) + x6_part_bytes(h), stream);
    if (rc != NT_OK) return rc;
  }
#endif
  if (!has_fk_image(h)) return NT_OK;
  return fk_pack((const float*)W, nlayers, h, h * h, (int64_t)per_layer, (char*)Wp + fk_offset(h), stream);
}

extern "C" int nt_dmpnn_pack_weight_fk(const void* W, int64_t nlayers, int64_t h, void* Wp, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(nlayers >= 0 && h > 0 && h <= 8192, NT_EINVAL, "bad sizes (1 <= h <= 8192)");
  if (nlayers == 0) return NT_OK;
  NT_REQUIRE(W && Wp && aligned16(Wp), NT_EINVAL, "NULL or misaligned pointer");
  NT_REQUIRE(has_fk_image(h), NT_EUNSUPPORTED, "the fk image needs h % 4 == 0 (or h > 512)");
  const size_t per_layer = nt_dmpnn_packed_weight_bytes(h, NT_F32);
  return fk_pack((const float*)W, nlayers, h, h * h, (int64_t)per_layer, (char*)Wp + fk_offset(h),
                 as_stream(stream_));
}

extern "C" int nt_dmpnn_pack_weights_fk(const void* const* W, int64_t nlayers, int64_t h, void* const* Wp,
                                        void* const* WpT, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(nlayers >= 0 && nlayers <= 16 && h > 0 && h <= 8192, NT_EINVAL, "bad sizes (nlayers <= 16, h <= 8192)");
  if (nlayers == 0) return NT_OK;
  NT_REQUIRE(W && Wp, NT_EINVAL, "NULL pointer array");
  NT_REQUIRE(has_fk_image(h), NT_EUNSUPPORTED, "the fk image needs h % 4 == 0 (or h > 512)");
  const float* w[16];
  char* img[16];
  char* imgT[16];
  for (int64_t l = 0; l < nlayers; ++l) {
    NT_REQUIRE(W[l] && Wp[l] && aligned16(Wp[l]) && (WpT == nullptr || (WpT[l] && aligned16(WpT[l]))), NT_EINVAL,
               "NULL or misaligned pointer");
    w[l] = (const float*)W[l];
    img[l] = (char*)Wp[l] + fk_offset(h);
    imgT[l] = WpT ? (char*)WpT[l] + fk_offset(h) : nullptr;
  }
  return fk_pack_multi(w, nlayers, h, img, WpT ? imgT : nullptr, as_stream(stream_));
}

extern "C" int nt_dmpnn_fused_tile_rows(int64_t h, int dtype, int act, int reduce, int agg_act) {
  if (h <= 0) return 0;
  if (dtype == NT_BF16) {
    if (nt::fw_active(h, NT_BF16, act, reduce, agg_act)) return 128;
    return bf16_fk(h) && nt::bf16_kernel_env() != 2 ? 128 : 64;  // fk4 (A/B): 64-row tiles, two workgroups per CU
  }
  return nt::fk_tile_rows(h, act, reduce, agg_act, true);
}

extern "C" int nt_dmpnn_row_table(const int32_t* perm, const int32_t* dst_sorted, const int64_t* src,
                                  const int64_t* rev, int64_t V, int64_t E, void* out, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(V >= 0 && E >= 0 && E < (int64_t(1) << 31) && V < (int64_t(1) << 29), NT_EINVAL,
             "bad sizes (E < 2^31, V < 2^29)");
  if (E == 0) return NT_OK;
  NT_REQUIRE(perm && dst_sorted && src && rev && out, NT_EINVAL, "NULL pointer");
  NT_REQUIRE(aligned16(out), NT_EINVAL, "out must be 16-byte aligned");
  return fk_row_table(perm, dst_sorted, src, rev, V, E, out, as_stream(stream_));
}

extern "C" int nt_absmax(const void* X, int64_t n, int dtype, float* out, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32, NT_EUNSUPPORTED, "nt_absmax: fp32 only");
  NT_REQUIRE(n >= 0, NT_EINVAL, "bad size");
  NT_REQUIRE(out != nullptr && (n == 0 || X != nullptr), NT_EINVAL, "NULL pointer");
  return fk_absmax((const float*)X, n, out, as_stream(stream_));
}

extern "C" int nt_dmpnn_update(const void* H, const void* S, const int64_t* src,
                               const int64_t* rev, const void* Wp, const void* b, int64_t V,
                               int64_t E, int64_t h, int residual, int act, float act_alpha,
                               int dtype, float* amax_ws, void* H_out, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32 || dtype == NT_BF16, NT_EUNSUPPORTED, "dtype must be NT_F32 or NT_BF16");
  NT_REQUIRE(act >= NT_ACT_IDENTITY && act <= NT_ACT_SIGMOID, NT_EINVAL, "bad act code");
  NT_REQUIRE(V >= 0 && E >= 0 && h > 0 && h <= 512, NT_EINVAL, "bad sizes (1 <= h <= 512)");
  if (E == 0) return NT_OK;
  NT_REQUIRE(H && S && src && rev && Wp && H_out, NT_EINVAL, "NULL pointer");
  NT_REQUIRE(H != H_out, NT_EINVAL, "H_out must not alias H");
  NT_REQUIRE(aligned16(Wp), NT_EINVAL, "Wp must be 16-byte aligned");
  if (dtype == NT_BF16) {
    if (bf16_fk(h) && aligned16(H) && aligned16(S) && aligned16(H_out) && (b == nullptr || aligned16(b))) {
      UpdateArgs a{(const float*)H, (const float*)S, src, rev, Wp, (const float*)b, V, E, h,
                   0, 0, residual, act, act_alpha, (float*)H_out, as_stream(stream_)};
      return launch_update_fk_bf16(a, Wp, nullptr, 0, 0, 0, nullptr, NT_SUM, NT_ACT_IDENTITY, 0.f, nullptr);
    }
    return launch_update_bf16(H, S, src, rev, Wp, b, V, E, h, residual, act, act_alpha, H_out,
                              as_stream(stream_));
  }
  const UpdateGeom g = geom_for(h);
  hipStream_t stream = as_stream(stream_);
#ifdef NT_DIAG
  const bool vec = (h % 4 == 0) && aligned16(H) && aligned16(S) && aligned16(H_out) &&
                   (b == nullptr || aligned16(b));
  const char choice = update_kernel_choice();
  if (vec && choice == 'a' && as_supported(h)) {
    UpdateArgs a{(const float*)H, (const float*)S, src, rev,
                 (const char*)Wp + f32_image_bytes(h) + x6_part_bytes(h), (const float*)b, V, E, h,
                 g.KB, g.NT, residual, act, act_alpha, (float*)H_out, stream};
    return launch_update_as(a);
  }
  if (vec && (choice == 'x' || choice == 'a') && x6_supported(h)) {
    UpdateArgs a{(const float*)H, (const float*)S, src, rev, (const char*)Wp + f32_image_bytes(h),
                 (const float*)b, V, E, h, g.KB, g.NT, residual, act, act_alpha, (float*)H_out,
                 stream};
    return launch_update_x6(a);
  }
#else
  // h % 4 == 0: update_fk_kernel in its plain mode (no aggregation); the split scales come from a
  // max|H|, max|S| pass into the caller's workspace (the C ABI call carries no amax)
  if (h % 4 == 0) {
    NT_REQUIRE(aligned16(H) && aligned16(S) && aligned16(H_out) && (b == nullptr || aligned16(b)), NT_EINVAL,
               "fp32 with h % 4 == 0 needs 16-byte aligned feature pointers");
    NT_REQUIRE(amax_ws != nullptr, NT_EINVAL, "fp32 with h % 4 == 0 needs amax_ws (2 device floats)");
    float* amax = amax_ws;
    int rc = amax_fill(amax, (const float*)H, E * h, (const float*)S, V * h, stream);
    if (rc != NT_OK) return rc;
    UpdateArgs a{(const float*)H, (const float*)S, src, rev, Wp, (const float*)b, V, E, h,
                 0, 0, residual, act, act_alpha, (float*)H_out, stream};
    return launch_update_fk(a, (const char*)Wp + fk_offset(h), amax, nullptr, nullptr, 0, 0, 0, nullptr,
                            NT_SUM, NT_ACT_IDENTITY, 0.f, nullptr);
  }
  const bool vec = false;  // h % 4 != 0: the exact fp32 tile kernel's scalar rows
#endif
  // 64-edge tiles while two workgroups still fit one CU's LDS (h <= 304), else 32-edge tiles.
  if (lds_bytes<64>(g) <= 80 * 1024)
    return dispatch_cpw<64>((const float*)H, (const float*)S, src, rev, (const float4*)Wp,
                            (const float*)b, V, E, (int)h, g, residual, act, act_alpha,
                            (float*)H_out, vec, stream);
  return dispatch_cpw<32>((const float*)H, (const float*)S, src, rev, (const float4*)Wp,
                          (const float*)b, V, E, (int)h, g, residual, act, act_alpha,
                          (float*)H_out, vec, stream);
}

extern "C" int nt_dmpnn_update_fused(const void* H, const void* S, const int64_t* src,
                                     const int64_t* rev, const void* Wp, const void* b, int64_t V,
                                     int64_t E, int64_t h, int residual, int act, float act_alpha,
                                     const int32_t* tile_ptr, int64_t ntiles, int tile_rows,
                                     int max_in_degree, const int32_t* perm,
                                     const int32_t* dst_sorted, const void* row_table, int reduce,
                                     int agg_act, float agg_alpha, int dtype, const float* amax_in,
                                     float* amax_out, void* H_out, void* S_out, void* S_part, int64_t ld_in,
                                     int64_t ld_out, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(ld_in >= 0 && ld_out >= 0, NT_EINVAL, "bad row pitch");
  NT_REQUIRE(dtype == NT_F32 || ((ld_in == 0 || ld_in == h) && (ld_out == 0 || ld_out == h) && S_part == nullptr),
             NT_EUNSUPPORTED, "row pitches other than h and hub partials are fp32 only");
  NT_REQUIRE(dtype == NT_F32 || dtype == NT_BF16, NT_EUNSUPPORTED, "dtype must be NT_F32 or NT_BF16");
  NT_REQUIRE(act >= NT_ACT_IDENTITY && act <= NT_ACT_SIGMOID, NT_EINVAL, "bad act code");
  NT_REQUIRE(agg_act >= NT_ACT_IDENTITY && agg_act <= NT_ACT_SIGMOID, NT_EINVAL, "bad agg_act code");
  NT_REQUIRE(reduce >= NT_SUM && reduce <= NT_MIN, NT_EINVAL, "bad reduce code");
  NT_REQUIRE(V >= 0 && E >= 0 && E < (int64_t(1) << 31) && V < (int64_t(1) << 31) && h > 0, NT_EINVAL,
             "bad sizes");
  NT_REQUIRE(dtype == NT_BF16 ? bf16_fused_supported(h) : (h % 4 == 0 && h <= 8192), NT_EUNSUPPORTED,
             "update_fused needs h % 4 == 0 (fp32), h % 8 == 0 and h <= 512 (bf16)");
  if (E == 0) return NT_OK;
  NT_REQUIRE(H && S && src && rev && Wp && H_out, NT_EINVAL, "NULL pointer");
  NT_REQUIRE(H != H_out && (S_out == nullptr || S_out != S), NT_EINVAL, "outputs alias inputs");
  NT_REQUIRE(aligned16(H) && aligned16(S) && aligned16(H_out) && aligned16(Wp) &&
                 (b == nullptr || aligned16(b)) && (S_out == nullptr || aligned16(S_out)),
             NT_EINVAL, "feature pointers must be 16-byte aligned");
  if (dtype == NT_BF16) {
    // the fk skeleton (128-row tiles) when the plan comes with its row table, else the 64-row kernel;
    // the one-wave-per-SIMD walk for fused relu / sum layers whose plan has a row table
    const bool fwb = tile_ptr != nullptr && row_table != nullptr && fw_active(h, NT_BF16, act, reduce, agg_act);
    if ((bf16_fk(h) || fwb) && (tile_ptr == nullptr || row_table != nullptr)) {
      NT_REQUIRE(row_table == nullptr || aligned16(row_table), NT_EINVAL, "row_table must be 16-byte aligned");
      UpdateArgs a{(const float*)H, (const float*)S, src, rev, Wp, (const float*)b, V, E, h,
                   0, 0, residual, act, act_alpha, (float*)H_out, as_stream(stream_)};
      return launch_update_fk_bf16(a, Wp, tile_ptr, ntiles, tile_rows, max_in_degree, row_table, reduce, agg_act,
                                   agg_alpha, S_out);
    }
    NT_REQUIRE(tile_ptr == nullptr || tile_rows <= 64, NT_EUNSUPPORTED, "bf16 tiles hold at most 64 rows");
    return launch_update_bf16_fused(H, S, src, rev, Wp, b, V, E, h, residual, act, act_alpha,
                                    tile_ptr, ntiles, perm, dst_sorted, reduce, agg_act, agg_alpha,
                                    H_out, S_out, as_stream(stream_));
  }
  UpdateArgs a{(const float*)H, (const float*)S, src, rev, Wp, (const float*)b, V, E, h,
               0, 0, residual, act, act_alpha, (float*)H_out, as_stream(stream_), ld_in, ld_out, (float*)S_part};
  NT_REQUIRE(row_table == nullptr || aligned16(row_table), NT_EINVAL, "row_table must be 16-byte aligned");
  NT_REQUIRE(S_part == nullptr || (tile_ptr != nullptr && aligned16(S_part)), NT_EINVAL,
             "S_part needs a tile plan and 16-byte alignment");
  return launch_update_fk(a, (const char*)Wp + fk_offset(h), amax_in, amax_out, tile_ptr, ntiles,
                          tile_rows, max_in_degree, row_table, reduce, agg_act, agg_alpha, (float*)S_out);
}

// out = X W^T (the layer GEMM alone: no gathers, no residual, no bias); the backward's dA = G W passes
// the packed image of W^T.  amax_in = (unused, max|X|) on the device: the fp16x3 fk kernel in its
// dense mode (row e of A is X[e]), any h % 4 == 0; amax_in = NULL: the persistent bf16x6 pk kernel
// (h <= 304).
extern "C" int nt_dmpnn_dense_matmul(const void* X, int64_t M, int64_t h, const void* Wp, int dtype,
                                     const float* amax_in, float* amax_ws, void* out, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32 || dtype == NT_BF16, NT_EUNSUPPORTED, "nt_dmpnn_dense_matmul: fp32 or bf16");
  NT_REQUIRE(M >= 0 && M < (int64_t(1) << 31) && h > 0, NT_EINVAL, "bad sizes");
  if (dtype == NT_BF16) {  // the bf16 layer kernel without gathers, residual or bias (h <= 512)
    NT_REQUIRE(h <= 512, NT_EUNSUPPORTED, "nt_dmpnn_dense_matmul: bf16 needs h <= 512");
    if (M == 0) return NT_OK;
    NT_REQUIRE(X && Wp && out && X != out, NT_EINVAL, "NULL pointer or out aliases X");
    if (bf16_fk(h) && aligned16(X) && aligned16(out)) {  // the bf16 layer kernel's dense mode
      UpdateArgs a{nullptr, (const float*)X, nullptr, nullptr, Wp, nullptr, M, M, h,
                   0, 0, 0, NT_ACT_IDENTITY, 0.f, (float*)out, as_stream(stream_)};
      return launch_update_fk_bf16(a, Wp, nullptr, 0, 0, 0, nullptr, NT_SUM, NT_ACT_IDENTITY, 0.f, nullptr);
    }
    return launch_update_bf16(X, X, nullptr, nullptr, Wp, nullptr, M, M, h, 0, NT_ACT_IDENTITY, 0.f, out,
                              as_stream(stream_));
  }
#ifdef NT_DIAG
  NT_REQUIRE(amax_in ? (h % 4 == 0 && h <= 8192) : ps_supported(h), NT_EUNSUPPORTED,
             "nt_dmpnn_dense_matmul needs h % 4 == 0 (and h <= 304 without amax_in)");
#else
  NT_REQUIRE(h % 4 == 0 && h <= 8192, NT_EUNSUPPORTED, "nt_dmpnn_dense_matmul needs h % 4 == 0 (fp32)");
#endif
  if (M == 0) return NT_OK;
  NT_REQUIRE(X && Wp && out, NT_EINVAL, "NULL pointer");
  NT_REQUIRE(X != out, NT_EINVAL, "out aliases X");
  NT_REQUIRE(aligned16(X) && aligned16(out) && aligned16(Wp), NT_EINVAL, "pointers must be 16-byte aligned");
#ifndef NT_DIAG
  if (!amax_in) {  // max|X| into the caller's workspace
    NT_REQUIRE(amax_ws != nullptr, NT_EINVAL, "fp32 without amax_in needs amax_ws (2 device floats)");
    int rc = amax_fill(amax_ws, nullptr, 0, (const float*)X, M * h, as_stream(stream_));
    if (rc != NT_OK) return rc;
    amax_in = amax_ws;
  }
#endif
  if (amax_in) {
    UpdateArgs a{nullptr, (const float*)X, nullptr, nullptr, Wp, nullptr, M, M, h,
                 0, 0, 0, NT_ACT_IDENTITY, 0.f, (float*)out, as_stream(stream_)};
    return launch_update_fk(a, (const char*)Wp + fk_offset(h), amax_in, nullptr, nullptr, 0, 0, 0, nullptr,
                            NT_SUM, NT_ACT_IDENTITY, 0.f, nullptr);
  }
#ifdef NT_DIAG
  const UpdateGeom g = geom_for(h);
  UpdateArgs a{(const float*)X, (const float*)X, nullptr, nullptr,
               (const char*)Wp + f32_image_bytes(h) + x6_part_bytes(h), nullptr, M, M, h,
               g.KB, g.NT, 0, NT_ACT_IDENTITY, 0.f, (float*)out, as_stream(stream_)};
  return launch_update_pk(a, nullptr, 0, nullptr, nullptr, NT_SUM, NT_ACT_IDENTITY, 0.f, nullptr);
#else
  return NT_OK;  // not reached: amax_in is set above
#endif
}

// Weight and bias gradient of one D-MPNN layer (backward of nn.Linear at
// chemprop.py:26,41, trained through lightning_models/model.py:224-241), with the layer message
// formed while staging so it is never written to HBM:
//   A[e]  = S[src e] - act(H[rev e])                           (chemprop.py:40; src/rev NULL: A = S)
//   dW    = G^T A          (h x h, reduced over all E edges)
//   db    = sum_e G[e]
//
// Split-K over edges: a 1-D grid of (64 x 64 output tile, edge chunk) workgroups.  Each workgroup
// walks its chunk 32 edges at a time: 256 threads load the 32 x 64 slab of G and of A (thread =
// one column, 8 consecutive edges; each load instruction reads 64 consecutive floats of one row),
// split every fp32 value into three bf16 parts once, and store them to a double-buffered LDS slab
// laid out [part][edge group][column] in 16-B units, so both the writes and the MFMA fragment reads
// are contiguous 1 KiB runs (no bank conflicts).  Wave w owns a 32 x 32 quadrant: 4 MFMA tiles x 6
// bf16 products (the bf16x6 split of csrc/update_pk.hip: fp32-accurate) per 32 edges.
// Partials (and the bias partials of the j-tile-0 workgroups) go to a workspace, reduced by a
// second kernel in fixed order, so the result is deterministic.
//
// XCD-aware: all output tiles of one edge chunk run on one XCD (blocks b, b + n share an XCD), so
// the chunk's G / S / H rows are fetched into that XCD's L2 once and read from there by the 25
// (at h = 300) tiles.
//
// Algorithmic bytes per call: G and A operands E*h*4 each (+ the gathers S[src], H[rev] replace A:
// 3 rows per edge), partial writes ksplit*h*h*4; flops 2*E*h^2.
#include "common.hpp"

namespace nt {
int cu_count();   // csrc/update_ps.hip: the current device's CU count, queried once per device
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kT = 64;              // output tile edge
constexpr int kK = 32;              // edges per step
constexpr int kPartB = 4 * 64 * 16; // one bf16 part of a 32 x 64 slab: 4 groups x 64 cols x 16 B
constexpr int kSlabB = 3 * kPartB;  // 12 KiB
constexpr int kBufs = 1;           // LDS slabs: one (24 KiB, two barriers per step) -> 4 workgroups
                                   // per CU (VGPR-bound) instead of 3 with a double buffer
constexpr int kWgPerCu = 4;

__device__ __forceinline__ void split3(const float (&x)[8], bf16x8& p0, bf16x8& p1, bf16x8& p2) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h0 = (__bf16)x[j];
    const float r1 = x[j] - (float)h0;
    const __bf16 h1 = (__bf16)r1;
    p0[j] = h0;
    p1[j] = h1;
    p2[j] = (__bf16)(r1 - (float)h1);
  }
}

struct WgArgs {
  const float* G;
  const float* H;
  const float* S;
  const int64_t* src;
  const int64_t* rev;
  int64_t E, h;
  int tiles, ksplit, chunk_steps, xcds;
  float alpha;
  int act;
  float* part;     // [ksplit][h][h]
  float* part_db;  // [ksplit][h] or NULL
};

template <int ACT, bool GATHER>
__global__ void __launch_bounds__(256) wgrad_kernel(WgArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  // XCD-aware work id: consecutive work ids (the tiles of one chunk) on one XCD
  const int nb = gridDim.x;
  int w = blockIdx.x;
  if (a.xcds > 1 && nb % a.xcds == 0) w = (w % a.xcds) * (nb / a.xcds) + w / a.xcds;
  const int y = w / a.tiles, tile = w - y * a.tiles;
  const int tpr = (int)((a.h + kT - 1) / kT);
  const int ti = tile / tpr, tj = tile - ti * tpr;
  const int64_t i0 = (int64_t)ti * kT, j0 = (int64_t)tj * kT, h = a.h;
  const int64_t e_beg = (int64_t)y * a.chunk_steps * kK;
  const int64_t e_end0 = e_beg + (int64_t)a.chunk_steps * kK;
  const int64_t e_end = e_end0 < a.E ? e_end0 : a.E;
  const int nsteps = e_end > e_beg ? (int)((e_end - e_beg + kK - 1) / kK) : 0;

  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int c = lane;          // staging: my column
  const int g = wave;          // staging: my edge group (8 edges)
  const bool ci = i0 + c < h, cj = j0 + c < h;
  const bool want_db = a.part_db != nullptr && tj == 0;
  float dbacc = 0.f;

  // The 8 edges' (src, rev) of a wave's group are fetched one step ahead as one vector load (lane r:
  // src of edge r, lane 8 + r: its rev) and broadcast with readlane, so no scalar-load round trip
  // sits in front of the row gathers.  Every load is unconditional (rows clamped to the chunk,
  // columns to the row) and masked afterwards.
  auto load_idx = [&](int s) -> int {
    int64_t e = e_beg + (int64_t)s * kK + 8 * g + (lane & 7);
    e = e < e_end ? e : e_end - 1;
    if (!GATHER || lane >= 16) return 0;
    return (int)(lane < 8 ? a.src[e] : a.rev[e]);
  };
  // masks instead of branches: a load whose value is only used under a condition gets sunk into a
  // branch by the compiler, with a vmcnt(0) wait right behind it (every gather serialised)
  const int64_t ic = ci ? i0 + c : 0, jc = cj ? j0 + c : 0;
  const unsigned mi = ci ? ~0u : 0u, mj = cj ? ~0u : 0u;
  // raw rows of the step in flight (consumed by store(), after the MFMAs of the previous step)
  float xg[8], xs[8], xh[8];
  int64_t eb_next = 0;
  auto load = [&](int s, int idxv) {
    const int64_t eb = e_beg + (int64_t)s * kK + 8 * g;
    eb_next = eb;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int64_t e = eb + r;
      const int64_t ec = e < e_end ? e : e_end - 1;
      xg[r] = a.G[ec * h + ic];
      if constexpr (GATHER) {
        const int64_t se = __builtin_amdgcn_readlane(idxv, r), re = __builtin_amdgcn_readlane(idxv, 8 + r);
        xs[r] = a.S[se * h + jc];
        xh[r] = a.H[re * h + jc];
      } else {
        xs[r] = a.S[ec * h + jc];
      }
    }
  };
  auto store = [&](int buf) {
    float gv[8], av[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const unsigned ok = eb_next + r < e_end ? ~0u : 0u;
      gv[r] = __uint_as_float(__float_as_uint(xg[r]) & (ok & mi));
      float v = xs[r];
      if constexpr (GATHER) v -= act_t<ACT>(xh[r], a.act, a.alpha);
      av[r] = __uint_as_float(__float_as_uint(v) & (ok & mj));
    }
    char* base = lds + (kBufs > 1 ? buf : 0) * 2 * kSlabB;
    const int off = (g * 64 + c) * 16;
    bf16x8 p0, p1, p2;
    split3(gv, p0, p1, p2);
    *reinterpret_cast<bf16x8*>(base + off) = p0;
    *reinterpret_cast<bf16x8*>(base + kPartB + off) = p1;
    *reinterpret_cast<bf16x8*>(base + 2 * kPartB + off) = p2;
    split3(av, p0, p1, p2);
    base += kSlabB;
    *reinterpret_cast<bf16x8*>(base + off) = p0;
    *reinterpret_cast<bf16x8*>(base + kPartB + off) = p1;
    *reinterpret_cast<bf16x8*>(base + 2 * kPartB + off) = p2;
    if (want_db) {
#pragma unroll
      for (int r = 0; r < 8; ++r) dbacc += gv[r];
    }
  };

  // MFMA roles: wave (wi, wj) owns rows 32 wi.. and columns 32 wj.. of the tile
  const int fr = lane & 15, g16 = lane >> 4;
  const int wi = wave & 1, wj = wave >> 1;
  f32x4 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int z = 0; z < 2; ++z) acc[x][z] = f32x4{0.f, 0.f, 0.f, 0.f};

  int idx_next = 0;
  if (nsteps > 0) {
    load(0, load_idx(0));
    if (nsteps > 1) idx_next = load_idx(1);
    store(0);
  }
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    const bool more = s + 1 < nsteps;
    if (more) {
      load(s + 1, idx_next);
      if (s + 2 < nsteps) idx_next = load_idx(s + 2);
    }
    const char* gb = lds + (kBufs > 1 ? buf : 0) * 2 * kSlabB;
    const char* ab = gb + kSlabB;
    bf16x8 fa[2][3], fb[2][3];
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      const int off_a = (g16 * 64 + 32 * wi + 16 * x + fr) * 16;
      const int off_b = (g16 * 64 + 32 * wj + 16 * x + fr) * 16;
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        fa[x][p] = *reinterpret_cast<const bf16x8*>(gb + p * kPartB + off_a);
        fb[x][p] = *reinterpret_cast<const bf16x8*>(ab + p * kPartB + off_b);
      }
    }
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int z = 0; z < 2; ++z) {
        f32x4 cc = acc[x][z];
        cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[x][0], fb[z][2], cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[x][1], fb[z][1], cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[x][2], fb[z][0], cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[x][0], fb[z][1], cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[x][1], fb[z][0], cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[x][0], fb[z][0], cc, 0, 0, 0);
        acc[x][z] = cc;
      }
    if (more) {
      if constexpr (kBufs == 1) __syncthreads();  // every wave has read the slab
      store(buf ^ 1);
    }
    __syncthreads();
  }

  // D lane (fr, g16), register q = tile row 4 g16 + q (A operand: G column = dW row), column fr
  float* P = a.part + (int64_t)y * h * h;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int z = 0; z < 2; ++z) {
      const int64_t col = j0 + 32 * wj + 16 * z + fr;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t row = i0 + 32 * wi + 16 * x + 4 * g16 + q;
        if (row < h && col < h) P[row * h + col] = acc[x][z][q];
      }
    }
  if (want_db) {
    float* red = reinterpret_cast<float*>(lds);  // slabs are dead after the last barrier
    red[g * 64 + c] = dbacc;
    __syncthreads();
    if (wave == 0 && ci) a.part_db[(int64_t)y * h + i0 + c] = red[c] + red[64 + c] + red[128 + c] + red[192 + c];
  }
}

// ---------------------------------------------------------------------------------------------
// wgrad_wide_kernel (h <= 320, gathered A): one 512-thread workgroup computes dW[:, j0:j0+128] of
// an edge chunk, i.e. every output row (all of G's columns) against a 128-column block of A, so the
// chunk's G rows are read by ceil(h / 128) workgroups instead of 25 and A's by one (5h floats per
// edge from L2 instead of 16h).  Per 32-edge step the workgroup stages G[32][NI * 16] and
// A[32][128] (three bf16 parts each, [part][edge group][column] 16-B runs, as wgrad_kernel); wave w
// owns i-tiles 5 (w % 4) .. +5 and j-tiles 4 (w / 4) .. +4 (20 accumulators).
constexpr int kWI = 320;            // max rows (G columns) of the wide kernel
constexpr int kWJ = 128;            // A columns per workgroup
constexpr int kWGPart = 4 * kWI * 16;   // one bf16 part of the G slab
constexpr int kWAPart = 4 * kWJ * 16;   // one bf16 part of the A slab
constexpr int kWLds = 3 * (kWGPart + kWAPart);  // 84 KiB

struct WwArgs {
  const float* G;
  const float* H;
  const float* S;
  const int64_t* src;
  const int64_t* rev;
  int64_t E, h;
  int jblocks, ksplit, chunk_steps, xcds;
  float alpha;
  int act;
  float* part;     // [ksplit][h][h]
  float* part_db;  // [ksplit][h] or NULL
};

template <int ACT>
__global__ void __launch_bounds__(512, 1) wgrad_wide_kernel(WwArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int nb = gridDim.x;
  int w = blockIdx.x;
  if (a.xcds > 1 && nb % a.xcds == 0) w = (w % a.xcds) * (nb / a.xcds) + w / a.xcds;
  const int y = w / a.jblocks, jb = w - y * a.jblocks;
  const int64_t h = a.h, j0 = (int64_t)jb * kWJ;
  const int64_t e_beg = (int64_t)y * a.chunk_steps * kK;
  const int64_t e_end0 = e_beg + (int64_t)a.chunk_steps * kK;
  const int64_t e_end = e_end0 < a.E ? e_end0 : a.E;
  const int nsteps = e_end > e_beg ? (int)((e_end - e_beg + kK - 1) / kK) : 0;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int ni16 = (int)((h + 15) / 16) * 16;  // G columns staged (multiple of 16, <= 320)
  const bool want_db = a.part_db != nullptr && jb == 0;

  // staging items: G (column cg, group gg) for q = t + 512 m < 4 ni16; A (column ca, group ga) = t
  int cg[3], gg[3];
  bool okg[3];
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    const int q = t + 512 * m;
    okg[m] = q < 4 * ni16;
    const int qq = okg[m] ? q : 0;
    gg[m] = qq / ni16;
    cg[m] = qq - gg[m] * ni16;
  }
  const int ca = t & (kWJ - 1), ga = t >> 7;  // 128 columns x 4 groups = 512
  const int64_t jc = j0 + ca < h ? j0 + ca : 0;
  const unsigned mj = j0 + ca < h ? ~0u : 0u;
  float dbacc[3] = {0.f, 0.f, 0.f};

  // (src, rev) of the wave's 8 A edges (every wave's items share one edge group), fetched a step
  // ahead as one vector load (lane r: src of edge r, lane 8 + r: its rev) and broadcast with readlane,
  // so no index round trip sits in front of the row gathers
  auto load_idx = [&](int s) __attribute__((always_inline)) -> int {
    int64_t e = e_beg + (int64_t)s * kK + 8 * ga + (lane & 7);
    e = e < e_end ? e : e_end - 1;
    return lane >= 16 ? 0 : (int)(lane < 8 ? a.src[e] : a.rev[e]);
  };
  float xg[3][8], xs[8], xh[8];
  int64_t eb_cur = 0;
  auto load = [&](int s, int idxv) __attribute__((always_inline)) {
    const int64_t eb = e_beg + (int64_t)s * kK;
    eb_cur = eb;
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      const int64_t col = cg[m] < h ? cg[m] : 0;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        int64_t e = eb + 8 * gg[m] + r;
        e = e < e_end ? e : e_end - 1;
        xg[m][r] = a.G[e * h + col];
      }
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int64_t se = __builtin_amdgcn_readlane(idxv, r), re = __builtin_amdgcn_readlane(idxv, 8 + r);
      xs[r] = a.S[se * h + jc];
      xh[r] = a.H[re * h + jc];
    }
  };
  auto store = [&]() __attribute__((always_inline)) {
    char* gbase = lds;
    char* abase = lds + 3 * kWGPart;
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      float gv[8];
      const unsigned mc = (okg[m] && cg[m] < h) ? ~0u : 0u;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const unsigned ok = eb_cur + 8 * gg[m] + r < e_end ? ~0u : 0u;
        gv[r] = __uint_as_float(__float_as_uint(xg[m][r]) & (ok & mc));
      }
      if (want_db) {
#pragma unroll
        for (int r = 0; r < 8; ++r) dbacc[m] += gv[r];
      }
      if (okg[m]) {
        bf16x8 p0, p1, p2;
        split3(gv, p0, p1, p2);
        const int off = (gg[m] * kWI + cg[m]) * 16;
        *reinterpret_cast<bf16x8*>(gbase + off) = p0;
        *reinterpret_cast<bf16x8*>(gbase + kWGPart + off) = p1;
        *reinterpret_cast<bf16x8*>(gbase + 2 * kWGPart + off) = p2;
      }
    }
    float av[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const unsigned ok = eb_cur + 8 * ga + r < e_end ? ~0u : 0u;
      const float v = xs[r] - act_t<ACT>(xh[r], a.act, a.alpha);
      av[r] = __uint_as_float(__float_as_uint(v) & (ok & mj));
    }
    bf16x8 p0, p1, p2;
    split3(av, p0, p1, p2);
    const int off = (ga * kWJ + ca) * 16;
    *reinterpret_cast<bf16x8*>(abase + off) = p0;
    *reinterpret_cast<bf16x8*>(abase + kWAPart + off) = p1;
    *reinterpret_cast<bf16x8*>(abase + 2 * kWAPart + off) = p2;
  };

  const int fr = lane & 15, g16 = lane >> 4;
  const int wi = wave & 3, wj = wave >> 2;  // i-tiles 5 wi .. 5 wi + 4, j-tiles 4 wj .. 4 wj + 3
  f32x4 acc[5][4];
#pragma unroll
  for (int x = 0; x < 5; ++x)
#pragma unroll
    for (int z = 0; z < 4; ++z) acc[x][z] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool iact = 16 * 5 * wi < ni16;  // waves whose i-tiles are all past h skip the MFMAs

  int idx_next = 0;
  if (nsteps > 0) {
    load(0, load_idx(0));
    if (nsteps > 1) idx_next = load_idx(1);
    store();
  }
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const bool more = s + 1 < nsteps;
    if (more) {
      load(s + 1, idx_next);
      if (s + 2 < nsteps) idx_next = load_idx(s + 2);
    }
    if (iact) {
      const char* gb = lds;
      const char* ab = lds + 3 * kWGPart;
      bf16x8 fb[4][3];
#pragma unroll
      for (int z = 0; z < 4; ++z) {
        const int off_b = (g16 * kWJ + 16 * (4 * wj + z) + fr) * 16;
#pragma unroll
        for (int p = 0; p < 3; ++p) fb[z][p] = *reinterpret_cast<const bf16x8*>(ab + p * kWAPart + off_b);
      }
#pragma unroll
      for (int x = 0; x < 5; ++x) {
        const int off_a = (g16 * kWI + 16 * (5 * wi + x) + fr) * 16;
        bf16x8 fa[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) fa[p] = *reinterpret_cast<const bf16x8*>(gb + p * kWGPart + off_a);
#pragma unroll
        for (int z = 0; z < 4; ++z) {
          f32x4 cc = acc[x][z];
          cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[z][2], cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], fb[z][1], cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[2], fb[z][0], cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[z][1], cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], fb[z][0], cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[z][0], cc, 0, 0, 0);
          acc[x][z] = cc;
        }
      }
    }
    if (more) {
      __syncthreads();  // every wave has read the slab
      store();
    }
    __syncthreads();
  }

  float* P = a.part + (int64_t)y * h * h;
#pragma unroll
  for (int x = 0; x < 5; ++x)
#pragma unroll
    for (int z = 0; z < 4; ++z) {
      const int64_t col = j0 + 16 * (4 * wj + z) + fr;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t row = 16 * (5 * wi + x) + 4 * g16 + q;
        if (row < h && col < h) P[row * h + col] = acc[x][z][q];
      }
    }
  if (want_db) {  // fixed-order column sums over the 4 edge groups (deterministic)
    float* red = reinterpret_cast<float*>(lds);  // the slabs are dead after the last barrier
#pragma unroll
    for (int m = 0; m < 3; ++m)
      if (okg[m]) red[gg[m] * kWI + cg[m]] = dbacc[m];
    __syncthreads();
    if (t < h) a.part_db[(int64_t)y * h + t] = ((red[t] + red[kWI + t]) + red[2 * kWI + t]) + red[3 * kWI + t];
  }
}

// wgrad_fk_kernel (h <= 320, gathered A): the wide kernel's work split on the fp32 layer kernel's
// numerics (csrc/update_fk.hpp): G scaled by s_G = 2^(14 - e(max|G|)), A by s_A = 2^(14 - e(bound
// of |S[src] - act(H[rev])|)) (device amax values the caller already has: the forward's amax chain
// and the max|G| the backward's dA takes), each split into two fp16 parts, and three
// v_mfma_f32_16x16x32_f16 products G1 A0 + G0 A1 + G0 A0 per tile (the dropped G1 A1 and the split
// roundings are ~2^-22 relative: fp32 accuracy).  Against the bf16x6 wide kernel: half the MFMAs,
// two thirds of the LDS bytes and of the split arithmetic, and a double-buffered LDS slab (112 KiB,
// one barrier per step instead of two).  Same work split: one 512-thread workgroup per (edge chunk,
// 128-column block of A), wave w owns i-tiles 5 (w % 4) .. +5 and j-tiles 4 (w / 4) .. +4.
constexpr int kFJ = 128;                     // A columns per workgroup
constexpr int kFGPart = 4 * kWI * 16;        // one fp16 part of the G slab (20 KiB)
constexpr int kFAPart = 4 * kFJ * 16;        // one fp16 part of the A slab (10 KiB)
constexpr int kFBuf = 2 * (kFGPart + kFAPart);
constexpr int kFLds = 2 * kFBuf;             // 112 KiB: two slabs

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split2s(const float (&x)[8], float s, f16x8& p0, f16x8& p1) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float v = x[j] * s;
    const _Float16 h0 = (_Float16)v;
    p0[j] = h0;
    p1[j] = (_Float16)(v - (float)h0);
  }
}

// 2^(14 - e): the power-of-two scale that maps |x| <= bound below 2^14 (update_fk.hpp scale_exp, but
// up to 2^120: tiny gradients are scaled up all the way, and the result is unscaled in two steps)
__device__ __forceinline__ int wg_scale_exp(float bound) {
  if (!(bound > 0.f) || !(bound <= 3.4028235e38f)) return 0;
  int e;
  frexpf(bound, &e);  // e <= 128 for every finite bound, so s >= -114 keeps it below 2^14
  const int s = 14 - e;
  return s > 120 ? 120 : s;
}
__device__ __forceinline__ float wg_act_bound(float m, int act, float alpha) {
  if (act == NT_ACT_RELU || act == NT_ACT_IDENTITY) return m;
  const float b = fabsf(alpha) > 1.f ? fabsf(alpha) : 1.f;
  return b * m + b;
}

struct WfArgs {
  const float* G;
  const float* H;
  const float* S;
  const int64_t* src;
  const int64_t* rev;
  const float* amax_G;   // [0] >= max|G|
  const float* amax_HS;  // [0] >= max|H|, [1] >= max|S|
  int64_t E, h;
  int jblocks, ksplit, chunk_steps, xcds;
  float alpha;
  int act;
  float* part;     // [ksplit][h][h]
  float* part_db;  // [ksplit][h] or NULL
};

template <int ACT>
__global__ void __launch_bounds__(512, 1) wgrad_fk_kernel(WfArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int nb = gridDim.x;
  int w = blockIdx.x;
  if (a.xcds > 1 && nb % a.xcds == 0) w = (w % a.xcds) * (nb / a.xcds) + w / a.xcds;
  const int y = w / a.jblocks, jb = w - y * a.jblocks;
  const int64_t h = a.h, j0 = (int64_t)jb * kFJ;
  const int64_t e_beg = (int64_t)y * a.chunk_steps * kK;
  const int64_t e_end0 = e_beg + (int64_t)a.chunk_steps * kK;
  const int64_t e_end = e_end0 < a.E ? e_end0 : a.E;
  const int nsteps = e_end > e_beg ? (int)((e_end - e_beg + kK - 1) / kK) : 0;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int ni16 = (int)((h + 15) / 16) * 16;
  const bool want_db = a.part_db != nullptr && jb == 0;
  const int eG = wg_scale_exp(a.amax_G[0]);
  const int eA = wg_scale_exp(a.amax_HS[1] + wg_act_bound(a.amax_HS[0], a.act, a.alpha));
  const float sG = ldexpf(1.f, eG), sA = ldexpf(1.f, eA);

  int cg[3], gg[3];
  bool okg[3];
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    const int q = t + 512 * m;
    okg[m] = q < 4 * ni16;
    const int qq = okg[m] ? q : 0;
    gg[m] = qq / ni16;
    cg[m] = qq - gg[m] * ni16;
  }
  const int c1 = t & (kFJ - 1), ga = t >> 7;  // 128 columns x 4 groups = 512: one edge group per wave
  const int64_t jc1 = j0 + c1 < h ? j0 + c1 : 0;
  const unsigned mj1 = j0 + c1 < h ? ~0u : 0u;
  float dbacc[3] = {0.f, 0.f, 0.f};

  auto load_idx = [&](int s) __attribute__((always_inline)) -> int {
    int64_t e = e_beg + (int64_t)s * kK + 8 * ga + (lane & 7);
    e = e < e_end ? e : e_end - 1;
    return lane >= 16 ? 0 : (int)(lane < 8 ? a.src[e] : a.rev[e]);
  };
  float xg[3][8], xs[8], xh[8];
  int64_t eb_cur = 0;
  auto load = [&](int s, int idxv) __attribute__((always_inline)) {
    const int64_t eb = e_beg + (int64_t)s * kK;
    eb_cur = eb;
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      const int64_t col = cg[m] < h ? cg[m] : 0;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        int64_t e = eb + 8 * gg[m] + r;
        e = e < e_end ? e : e_end - 1;
        xg[m][r] = a.G[e * h + col];
      }
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int64_t se = __builtin_amdgcn_readlane(idxv, r), re = __builtin_amdgcn_readlane(idxv, 8 + r);
      xs[r] = a.S[se * h + jc1];
      xh[r] = a.H[re * h + jc1];
    }
  };
  auto store = [&](char* buf) __attribute__((always_inline)) {
    char* gbase = buf;
    char* abase = buf + 2 * kFGPart;
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      float gv[8];
      const unsigned mc = (okg[m] && cg[m] < h) ? ~0u : 0u;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const unsigned ok = eb_cur + 8 * gg[m] + r < e_end ? ~0u : 0u;
        gv[r] = __uint_as_float(__float_as_uint(xg[m][r]) & (ok & mc));
      }
      if (want_db) {
#pragma unroll
        for (int r = 0; r < 8; ++r) dbacc[m] += gv[r];
      }
      if (okg[m]) {
        f16x8 p0, p1;
        split2s(gv, sG, p0, p1);
        const int off = (gg[m] * kWI + cg[m]) * 16;
        *reinterpret_cast<f16x8*>(gbase + off) = p0;
        *reinterpret_cast<f16x8*>(gbase + kFGPart + off) = p1;
      }
    }
    float av[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const unsigned ok = eb_cur + 8 * ga + r < e_end ? ~0u : 0u;
      const float v = xs[r] - act_t<ACT>(xh[r], a.act, a.alpha);
      av[r] = __uint_as_float(__float_as_uint(v) & (ok & mj1));
    }
    f16x8 p0, p1;
    split2s(av, sA, p0, p1);
    const int off = (ga * kFJ + c1) * 16;
    *reinterpret_cast<f16x8*>(abase + off) = p0;
    *reinterpret_cast<f16x8*>(abase + kFAPart + off) = p1;
  };

  const int fr = lane & 15, g16 = lane >> 4;
  const int wi = wave & 3, wj = wave >> 2;  // i-tiles 5 wi .. 5 wi + 4, j-tiles 4 wj .. 4 wj + 3
  f32x4 acc[5][4];
#pragma unroll
  for (int x = 0; x < 5; ++x)
#pragma unroll
    for (int z = 0; z < 4; ++z) acc[x][z] = f32x4{0.f, 0.f, 0.f, 0.f};
  // waves whose i-tiles or j-tiles all lie past h skip the MFMAs
  const bool active = 16 * 5 * wi < ni16 && j0 + 16 * 4 * wj < h;

  int idx_next = 0;
  if (nsteps > 0) {
    load(0, load_idx(0));
    if (nsteps > 1) idx_next = load_idx(1);
    store(lds);
  }
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const bool more = s + 1 < nsteps;
    if (more) {
      load(s + 1, idx_next);
      if (s + 2 < nsteps) idx_next = load_idx(s + 2);
    }
    if (active) {
      const char* gb = lds + (s & 1) * kFBuf;
      const char* ab = gb + 2 * kFGPart;
      f16x8 fb[4][2];
#pragma unroll
      for (int z = 0; z < 4; ++z) {
        const int off_b = (g16 * kFJ + 16 * (4 * wj + z) + fr) * 16;
        fb[z][0] = *reinterpret_cast<const f16x8*>(ab + off_b);
        fb[z][1] = *reinterpret_cast<const f16x8*>(ab + kFAPart + off_b);
      }
#pragma unroll
      for (int x = 0; x < 5; ++x) {
        const int off_a = (g16 * kWI + 16 * (5 * wi + x) + fr) * 16;
        const f16x8 fa0 = *reinterpret_cast<const f16x8*>(gb + off_a);
        const f16x8 fa1 = *reinterpret_cast<const f16x8*>(gb + kFGPart + off_a);
#pragma unroll
        for (int z = 0; z < 4; ++z) {
          f32x4 cc = acc[x][z];
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa1, fb[z][0], cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa0, fb[z][1], cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa0, fb[z][0], cc, 0, 0, 0);
          acc[x][z] = cc;
        }
      }
    }
    if (more) store(lds + ((s + 1) & 1) * kFBuf);
    __syncthreads();  // one barrier: the next slab is written, this one is read by every wave
  }

  // unscale by 2^-eG 2^-eA (two exact steps: their product may leave the fp32 range)
  const float iG = ldexpf(1.f, -eG), iA = ldexpf(1.f, -eA);
  float* P = a.part + (int64_t)y * h * h;
#pragma unroll
  for (int x = 0; x < 5; ++x)
#pragma unroll
    for (int z = 0; z < 4; ++z) {
      const int64_t col = j0 + 16 * (4 * wj + z) + fr;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t row = 16 * (5 * wi + x) + 4 * g16 + q;
        if (row < h && col < h) P[row * h + col] = (acc[x][z][q] * iG) * iA;
      }
    }
  if (want_db) {  // fixed-order column sums over the 4 edge groups (deterministic)
    float* red = reinterpret_cast<float*>(lds);  // the slabs are dead after the last barrier
#pragma unroll
    for (int m = 0; m < 3; ++m)
      if (okg[m]) red[gg[m] * kWI + cg[m]] = dbacc[m];
    __syncthreads();
    if (t < h) a.part_db[(int64_t)y * h + t] = ((red[t] + red[kWI + t]) + red[2 * kWI + t]) + red[3 * kWI + t];
  }
}

// wgrad_bf16_kernel (bf16 storage, h <= 512, gathered A): dW = G^T A and db = colsum G of a bf16
// layer (BASELINE config 3) with the message A = S[src] - act(H[rev]) formed in fp32 and rounded to
// bf16 once, as the bf16 forward's message is (chemprop.py:40), never written.  The operands are
// exact bf16 values, so one v_mfma_f32_16x16x32_bf16 per tile and fp32 partials (the library path
// rounded every split-K partial to bf16).  One 512-thread workgroup per (edge chunk, 128-column
// block of A) stages all of G's columns (<= 512; each thread loads column pairs as 4-B words) and
// the block's A columns per 32-edge step into a double-buffered LDS slab (80 KiB, one barrier per
// step); wave w owns i-tiles 8 (w % 4) .. +8 and j-tiles 4 (w / 4) .. +4 (32 accumulators).
constexpr int kBI = 512;                // max G columns
constexpr int kBGPart = 4 * kBI * 16;   // G slab (32 KiB)
constexpr int kBAPart = 4 * kWJ * 16;   // A slab (8 KiB)
constexpr int kBBuf = kBGPart + kBAPart;
constexpr int kBLds = 2 * kBBuf;

struct WbArgs {
  const uint16_t* G;
  const uint16_t* H;
  const uint16_t* S;
  const int64_t* src;
  const int64_t* rev;
  int64_t E, h;
  int jblocks, ksplit, chunk_steps, xcds;
  float alpha;
  int act;
  float* part;     // [ksplit][h][h]
  float* part_db;  // [ksplit][h] or NULL
};

__device__ __forceinline__ float bfu(uint32_t u16) { return __uint_as_float(u16 << 16); }

template <int ACT>
__global__ void __launch_bounds__(512, 1) wgrad_bf16_kernel(WbArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int nb = gridDim.x;
  int w = blockIdx.x;
  if (a.xcds > 1 && nb % a.xcds == 0) w = (w % a.xcds) * (nb / a.xcds) + w / a.xcds;
  const int y = w / a.jblocks, jb = w - y * a.jblocks;
  const int64_t h = a.h, j0 = (int64_t)jb * kWJ;
  const int64_t e_beg = (int64_t)y * a.chunk_steps * kK;
  const int64_t e_end0 = e_beg + (int64_t)a.chunk_steps * kK;
  const int64_t e_end = e_end0 < a.E ? e_end0 : a.E;
  const int nsteps = e_end > e_beg ? (int)((e_end - e_beg + kK - 1) / kK) : 0;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int ni16 = (int)((h + 15) / 16) * 16;
  const int np = ni16 / 2;  // column pairs staged per edge group
  const bool want_db = a.part_db != nullptr && jb == 0;

  // G items: (column pair cp, group gg) for q = t + 512 m < 4 np
  int cp[2], gg[2];
  bool okg[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int q = t + 512 * m;
    okg[m] = q < 4 * np;
    const int qq = okg[m] ? q : 0;
    gg[m] = qq / np;
    cp[m] = qq - gg[m] * np;
  }
  const int c1 = t & (kWJ - 1), ga = t >> 7;
  const int64_t jc1 = j0 + c1 < h ? j0 + c1 : 0;
  const bool okj = j0 + c1 < h;
  float dbacc[2][2] = {{0.f, 0.f}, {0.f, 0.f}};

  auto load_idx = [&](int s) __attribute__((always_inline)) -> int {
    int64_t e = e_beg + (int64_t)s * kK + 8 * ga + (lane & 7);
    e = e < e_end ? e : e_end - 1;
    return lane >= 16 ? 0 : (int)(lane < 8 ? a.src[e] : a.rev[e]);
  };
  uint32_t xg[2][8], xs[8], xh[8];
  int64_t eb_cur = 0;
  const uint32_t* G32 = reinterpret_cast<const uint32_t*>(a.G);  // h even: column pairs are aligned words
  auto load = [&](int s, int idxv) __attribute__((always_inline)) {
    const int64_t eb = e_beg + (int64_t)s * kK;
    eb_cur = eb;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int64_t col = 2 * cp[m] < h ? 2 * cp[m] : 0;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        int64_t e = eb + 8 * gg[m] + r;
        e = e < e_end ? e : e_end - 1;
        xg[m][r] = G32[(e * h + col) >> 1];
      }
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int64_t se = __builtin_amdgcn_readlane(idxv, r), re = __builtin_amdgcn_readlane(idxv, 8 + r);
      xs[r] = a.S[se * h + jc1];
      xh[r] = a.H[re * h + jc1];
    }
  };
  auto store = [&](char* buf) __attribute__((always_inline)) {
    char* gbase = buf;
    char* abase = buf + kBGPart;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      uint32_t lo[8], hi[8];
      const bool in0 = okg[m] && 2 * cp[m] < h, in1 = okg[m] && 2 * cp[m] + 1 < h;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const bool ok = eb_cur + 8 * gg[m] + r < e_end;
        lo[r] = (ok && in0) ? (xg[m][r] & 0xffffu) : 0u;
        hi[r] = (ok && in1) ? (xg[m][r] >> 16) : 0u;
      }
      if (want_db) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          dbacc[m][0] += bfu(lo[r]);
          dbacc[m][1] += bfu(hi[r]);
        }
      }
      if (okg[m]) {
        uint4 v0, v1;
        v0.x = lo[0] | (lo[1] << 16); v0.y = lo[2] | (lo[3] << 16); v0.z = lo[4] | (lo[5] << 16); v0.w = lo[6] | (lo[7] << 16);
        v1.x = hi[0] | (hi[1] << 16); v1.y = hi[2] | (hi[3] << 16); v1.z = hi[4] | (hi[5] << 16); v1.w = hi[6] | (hi[7] << 16);
        const int off = (gg[m] * kBI + 2 * cp[m]) * 16;
        *reinterpret_cast<uint4*>(gbase + off) = v0;
        *reinterpret_cast<uint4*>(gbase + off + 16) = v1;
      }
    }
    bf16x8 av;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const bool ok = okj && eb_cur + 8 * ga + r < e_end;
      const float v = bfu(xs[r] & 0xffffu) - act_t<ACT>(bfu(xh[r] & 0xffffu), a.act, a.alpha);
      av[r] = (__bf16)(ok ? v : 0.f);
    }
    *reinterpret_cast<bf16x8*>(abase + (ga * kWJ + c1) * 16) = av;
  };

  const int fr = lane & 15, g16 = lane >> 4;
  const int wi = wave & 3, wj = wave >> 2;  // i-tiles 8 wi .. 8 wi + 7, j-tiles 4 wj .. 4 wj + 3
  f32x4 acc[8][4];
#pragma unroll
  for (int x = 0; x < 8; ++x)
#pragma unroll
    for (int z = 0; z < 4; ++z) acc[x][z] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool active = 16 * 8 * wi < ni16 && j0 + 16 * 4 * wj < h;

  int idx_next = 0;
  if (nsteps > 0) {
    load(0, load_idx(0));
    if (nsteps > 1) idx_next = load_idx(1);
    store(lds);
  }
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const bool more = s + 1 < nsteps;
    if (more) {
      load(s + 1, idx_next);
      if (s + 2 < nsteps) idx_next = load_idx(s + 2);
    }
    if (active) {
      const char* gb = lds + (s & 1) * kBBuf;
      const char* ab = gb + kBGPart;
      bf16x8 fb[4];
#pragma unroll
      for (int z = 0; z < 4; ++z)
        fb[z] = *reinterpret_cast<const bf16x8*>(ab + (g16 * kWJ + 16 * (4 * wj + z) + fr) * 16);
#pragma unroll
      for (int x = 0; x < 8; ++x) {
        const bf16x8 fa = *reinterpret_cast<const bf16x8*>(gb + (g16 * kBI + 16 * (8 * wi + x) + fr) * 16);
#pragma unroll
        for (int z = 0; z < 4; ++z) acc[x][z] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[z], acc[x][z], 0, 0, 0);
      }
    }
    if (more) store(lds + ((s + 1) & 1) * kBBuf);
    __syncthreads();
  }

  float* P = a.part + (int64_t)y * h * h;
#pragma unroll
  for (int x = 0; x < 8; ++x)
#pragma unroll
    for (int z = 0; z < 4; ++z) {
      const int64_t col = j0 + 16 * (4 * wj + z) + fr;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t row = 16 * (8 * wi + x) + 4 * g16 + q;
        if (row < h && col < h) P[row * h + col] = acc[x][z][q];
      }
    }
  if (want_db) {  // fixed-order column sums over the 4 edge groups (deterministic)
    float* red = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int m = 0; m < 2; ++m)
      if (okg[m]) {
        red[gg[m] * kBI + 2 * cp[m]] = dbacc[m][0];
        red[gg[m] * kBI + 2 * cp[m] + 1] = dbacc[m][1];
      }
    __syncthreads();
    for (int c = t; c < h; c += 512)
      a.part_db[(int64_t)y * h + c] = ((red[c] + red[kBI + c]) + red[2 * kBI + c]) + red[3 * kBI + c];
  }
}

// dW and db partials reduced in one launch: index i < n1 sums part[y][i] into out1[i], the rest sums
// part_db[y][i - n1] into out2, each in ascending y (fixed order: deterministic)
__global__ void __launch_bounds__(256) wgrad_reduce2_kernel(const float* __restrict__ part, int64_t n1,
                                                            const float* __restrict__ part_db, int64_t n2,
                                                            int ksplit, float* __restrict__ out1,
                                                            float* __restrict__ out2) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n1 + n2; i += (int64_t)gridDim.x * blockDim.x) {
    const bool first = i < n1;
    const float* src = first ? part + i : part_db + (i - n1);
    const int64_t stride = first ? n1 : n2;
    float s = 0.f;
    int y = 0;
    for (; y + 8 <= ksplit; y += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = src[(int64_t)(y + u) * stride];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; y < ksplit; ++y) s += src[(int64_t)y * stride];
    if (first) out1[i] = s;
    else out2[i - n1] = s;
  }
}

int reduce_partials(const float* part, const float* part_db, int64_t h, int ksplit, float* dW, float* db,
                    hipStream_t stream) {
  const int64_t n2 = db ? h : 0;
  wgrad_reduce2_kernel<<<grid_for(h * h + n2, 256, 256 * 8), 256, 0, stream>>>(part, h * h, part_db, n2, ksplit,
                                                                               dW, db);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

struct Plan {
  int tiles, ksplit, chunk_steps;
};

Plan make_plan(int64_t E, int64_t h) {
  Plan p;
  const int tpr = (int)((h + kT - 1) / kT);
  p.tiles = tpr * tpr;
  const int64_t steps = (E + kK - 1) / kK;
  // one round of workgroups: ksplit = the largest multiple of 8 with tiles * ksplit <= resident slots
  const int slots = kWgPerCu * (cu_count() > 0 ? cu_count() : 256);
  int64_t ks = slots / p.tiles / 8 * 8;
  if (ks < 8) ks = 8;
  if (ks > steps) ks = steps > 0 ? steps : 1;
  p.chunk_steps = (int)((steps + ks - 1) / ks);
  if (p.chunk_steps < 1) p.chunk_steps = 1;
  p.ksplit = (int)((steps + p.chunk_steps - 1) / p.chunk_steps);
  if (p.ksplit < 1) p.ksplit = 1;
  return p;
}

struct WPlan {
  int ksplit, chunk_steps;
};

// one workgroup per CU: ksplit = CUs / jblocks chunks of the edge range (jcols: A columns per block)
WPlan make_wide_plan(int64_t E, int64_t h, int jcols = kWJ) {
  WPlan p;
  const int jblocks = (int)((h + jcols - 1) / jcols);
  const int64_t steps = (E + kK - 1) / kK;
  int64_t ks = (cu_count() > 0 ? cu_count() : 256) / jblocks;
  if (ks < 1) ks = 1;
  if (ks > steps) ks = steps > 0 ? steps : 1;
  p.chunk_steps = (int)((steps + ks - 1) / ks);
  if (p.chunk_steps < 1) p.chunk_steps = 1;
  p.ksplit = (int)((steps + p.chunk_steps - 1) / p.chunk_steps);
  if (p.ksplit < 1) p.ksplit = 1;
  return p;
}

}  // namespace

int xcd_count();  // csrc/update_ps.hip: the current device's XCD count, queried once per device
}  // namespace nt

extern "C" int64_t nt_dmpnn_weight_grad_workspace(int64_t E, int64_t h) {
  if (E < 0 || h <= 0) return -1;
  const nt::Plan p = nt::make_plan(E, h);
  const nt::WPlan q = nt::make_wide_plan(E, h), f = nt::make_wide_plan(E, h, nt::kFJ);
  int64_t ks = p.ksplit > q.ksplit ? p.ksplit : q.ksplit;  // every kernel fits
  ks = ks > f.ksplit ? ks : f.ksplit;
  return ks * (h * h + h) * (int64_t)sizeof(float);
}

extern "C" int nt_dmpnn_weight_grad(const void* G, const void* H, const void* S, const int64_t* src,
                                    const int64_t* rev, int64_t V, int64_t E, int64_t h, int act,
                                    float act_alpha, int dtype, void* workspace, int64_t workspace_bytes,
                                    void* dW_out, void* db_out, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32 || dtype == NT_BF16, NT_EUNSUPPORTED, "nt_dmpnn_weight_grad: fp32 or bf16");
  NT_REQUIRE(act >= NT_ACT_IDENTITY && act <= NT_ACT_SIGMOID, NT_EINVAL, "bad act code");
  NT_REQUIRE(V >= 0 && E >= 0 && h > 0, NT_EINVAL, "bad sizes");
  NT_REQUIRE(dtype == NT_F32 || (h <= kBI && h % 2 == 0 && src && rev), NT_EUNSUPPORTED,
             "nt_dmpnn_weight_grad: bf16 needs h <= 512, h even, src and rev");
  // row indices are narrowed to int for the lane broadcasts
  NT_REQUIRE(V < ((int64_t)1 << 31) && E < ((int64_t)1 << 31), NT_EUNSUPPORTED,
             "nt_dmpnn_weight_grad: V and E must be < 2^31");
  NT_REQUIRE((src == nullptr) == (rev == nullptr), NT_EINVAL, "src and rev: both or neither");
  NT_REQUIRE(dW_out, NT_EINVAL, "NULL dW_out");
  hipStream_t stream = as_stream(stream_);
  if (E == 0) {
    NT_HIP(hipMemsetAsync(dW_out, 0, h * h * sizeof(float), stream));
    if (db_out) NT_HIP(hipMemsetAsync(db_out, 0, h * sizeof(float), stream));
    return NT_OK;
  }
  NT_REQUIRE(G && S && (src == nullptr || H), NT_EINVAL, "NULL pointer");
  const Plan p = make_plan(E, h);
  NT_REQUIRE(workspace && workspace_bytes >= nt_dmpnn_weight_grad_workspace(E, h), NT_EINVAL,
             "workspace too small (nt_dmpnn_weight_grad_workspace)");
  WgArgs a;
  a.G = (const float*)G;
  a.H = (const float*)H;
  a.S = (const float*)S;
  a.src = src;
  a.rev = rev;
  a.E = E;
  a.h = h;
  a.tiles = p.tiles;
  a.ksplit = p.ksplit;
  a.chunk_steps = p.chunk_steps;
  a.xcds = xcd_count();
  a.alpha = act_alpha;
  a.act = act;
  a.part = (float*)workspace;
  a.part_db = db_out ? a.part + (int64_t)p.ksplit * h * h : nullptr;
  if (dtype == NT_BF16) {
    const WPlan q = make_wide_plan(E, h);
    WbArgs b;
    b.G = (const uint16_t*)G;
    b.H = (const uint16_t*)H;
    b.S = (const uint16_t*)S;
    b.src = src;
    b.rev = rev;
    b.E = E;
    b.h = h;
    b.jblocks = (int)((h + kWJ - 1) / kWJ);
    b.ksplit = q.ksplit;
    b.chunk_steps = q.chunk_steps;
    b.xcds = xcd_count();
    b.alpha = act_alpha;
    b.act = act;
    b.part = (float*)workspace;
    b.part_db = db_out ? b.part + (int64_t)q.ksplit * h * h : nullptr;
    const int grid = b.jblocks * q.ksplit;
    auto kern = act == NT_ACT_IDENTITY ? wgrad_bf16_kernel<NT_ACT_IDENTITY>
                : act == NT_ACT_RELU   ? wgrad_bf16_kernel<NT_ACT_RELU>
                                       : wgrad_bf16_kernel<-1>;
    NT_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, kBLds));
    kern<<<grid, 512, kBLds, stream>>>(b);
    NT_LAUNCH_CHECK();
    return reduce_partials(b.part, b.part_db, h, q.ksplit, (float*)dW_out, (float*)db_out, stream);
  }
  if (src && h <= kWI) {  // the wide kernel: 128-column blocks of A against all of G
    const int jblocks = (int)((h + kWJ - 1) / kWJ);
    const WPlan q = make_wide_plan(E, h);
    WwArgs b;
    b.G = (const float*)G;
    b.H = (const float*)H;
    b.S = (const float*)S;
    b.src = src;
    b.rev = rev;
    b.E = E;
    b.h = h;
    b.jblocks = jblocks;
    b.ksplit = q.ksplit;
    b.chunk_steps = q.chunk_steps;
    b.xcds = xcd_count();
    b.alpha = act_alpha;
    b.act = act;
    b.part = (float*)workspace;
    b.part_db = db_out ? b.part + (int64_t)q.ksplit * h * h : nullptr;
    const int grid = jblocks * q.ksplit;
    if (act == NT_ACT_IDENTITY)
      wgrad_wide_kernel<NT_ACT_IDENTITY><<<grid, 512, kWLds, stream>>>(b);
    else if (act == NT_ACT_RELU)
      wgrad_wide_kernel<NT_ACT_RELU><<<grid, 512, kWLds, stream>>>(b);
    else
      wgrad_wide_kernel<-1><<<grid, 512, kWLds, stream>>>(b);
    NT_LAUNCH_CHECK();
    return reduce_partials(b.part, b.part_db, h, q.ksplit, (float*)dW_out, (float*)db_out, stream);
  }
  const int grid = p.tiles * p.ksplit;
  const size_t lds = kBufs * 2 * kSlabB;
  if (!src)
    wgrad_kernel<NT_ACT_IDENTITY, false><<<grid, 256, lds, stream>>>(a);
  else if (act == NT_ACT_IDENTITY)
    wgrad_kernel<NT_ACT_IDENTITY, true><<<grid, 256, lds, stream>>>(a);
  else if (act == NT_ACT_RELU)
    wgrad_kernel<NT_ACT_RELU, true><<<grid, 256, lds, stream>>>(a);
  else
    wgrad_kernel<-1, true><<<grid, 256, lds, stream>>>(a);
  NT_LAUNCH_CHECK();
  return reduce_partials(a.part, a.part_db, h, p.ksplit, (float*)dW_out, (float*)db_out, stream);
}

extern "C" int nt_dmpnn_weight_grad_fk(const void* G, const void* H, const void* S, const int64_t* src,
                                       const int64_t* rev, int64_t V, int64_t E, int64_t h, int act,
                                       float act_alpha, const float* amax_G, const float* amax_HS, int dtype,
                                       void* workspace, int64_t workspace_bytes, void* dW_out, void* db_out,
                                       void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(dtype == NT_F32, NT_EUNSUPPORTED, "nt_dmpnn_weight_grad_fk: fp32 only");
  NT_REQUIRE(act >= NT_ACT_IDENTITY && act <= NT_ACT_SIGMOID, NT_EINVAL, "bad act code");
  NT_REQUIRE(V >= 0 && E >= 0 && h > 0, NT_EINVAL, "bad sizes");
  NT_REQUIRE(h <= kWI, NT_EUNSUPPORTED, "nt_dmpnn_weight_grad_fk: h <= 320 (use nt_dmpnn_weight_grad)");
  NT_REQUIRE(V < ((int64_t)1 << 31) && E < ((int64_t)1 << 31), NT_EUNSUPPORTED,
             "nt_dmpnn_weight_grad_fk: V and E must be < 2^31");
  NT_REQUIRE(dW_out, NT_EINVAL, "NULL dW_out");
  hipStream_t stream = as_stream(stream_);
  if (E == 0) {
    NT_HIP(hipMemsetAsync(dW_out, 0, h * h * sizeof(float), stream));
    if (db_out) NT_HIP(hipMemsetAsync(db_out, 0, h * sizeof(float), stream));
    return NT_OK;
  }
  NT_REQUIRE(G && S && H && src && rev && amax_G && amax_HS, NT_EINVAL, "NULL pointer");
  NT_REQUIRE(workspace && workspace_bytes >= nt_dmpnn_weight_grad_workspace(E, h), NT_EINVAL,
             "workspace too small (nt_dmpnn_weight_grad_workspace)");
  const WPlan q = make_wide_plan(E, h, kFJ);
  WfArgs b;
  b.G = (const float*)G;
  b.H = (const float*)H;
  b.S = (const float*)S;
  b.src = src;
  b.rev = rev;
  b.amax_G = amax_G;
  b.amax_HS = amax_HS;
  b.E = E;
  b.h = h;
  b.jblocks = (int)((h + kFJ - 1) / kFJ);
  b.ksplit = q.ksplit;
  b.chunk_steps = q.chunk_steps;
  b.xcds = xcd_count();
  b.alpha = act_alpha;
  b.act = act;
  b.part = (float*)workspace;
  b.part_db = db_out ? b.part + (int64_t)q.ksplit * h * h : nullptr;
  const int grid = b.jblocks * q.ksplit;
  auto kern = act == NT_ACT_IDENTITY ? wgrad_fk_kernel<NT_ACT_IDENTITY>
              : act == NT_ACT_RELU   ? wgrad_fk_kernel<NT_ACT_RELU>
                                     : wgrad_fk_kernel<-1>;
  NT_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, kFLds));
  kern<<<grid, 512, kFLds, stream>>>(b);
  NT_LAUNCH_CHECK();
  return reduce_partials(b.part, b.part_db, h, q.ksplit, (float*)dW_out, (float*)db_out, stream);
}

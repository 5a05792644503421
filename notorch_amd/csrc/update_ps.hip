// Tile planner of the fused layer kernels: node-aligned tiles of the dst-sorted edge order
// (nt_dmpnn_tile_plan, nt_dmpnn_tile_plan_hubs), their balanced stride (nt_dmpnn_tile_stride), and the
// device's CU / XCD counts the launchers size their grids by.  (The persistent producer/consumer "ps"
// layer kernel that used to live here is an A/B variant of the diagnostic library:
// csrc/diag/update_ps_ring.hip.)
#include <stdlib.h>

#include <type_traits>

#include "common.hpp"
#include "update.hpp"

namespace nt {

namespace {

// tile_ptr[k] = dst_ptr[first v with dst_ptr[v] >= k L], k < ntiles; tile_ptr[ntiles] = E: the
// target k L rounded up to the next node start, except inside a hub (a node with more than
// hub_degree in-edges), where the tile is cut at k L itself.
__global__ void tile_plan_kernel(const int32_t* __restrict__ dst_ptr, int64_t V, int64_t E, int L,
                                 int ntiles, int hub_degree, int32_t* __restrict__ tile_ptr) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k > ntiles) return;
  if (k == ntiles) {
    tile_ptr[k] = (int32_t)E;
    return;
  }
  const int64_t target = (int64_t)k * L;  // < E
  int64_t lo = 0, hi = V;  // first v in [0, V] with dst_ptr[v] > target (exists: dst_ptr[V] = E)
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (dst_ptr[mid] > target) hi = mid;
    else lo = mid + 1;
  }
  const int64_t v = lo - 1;  // the node whose in-edges hold position target
  const int32_t b = dst_ptr[v], e = dst_ptr[v + 1];
  tile_ptr[k] = (b == target || e - b > hub_degree) ? (int32_t)target : e;
}

// dsts[p] = v for every position p in [dst_ptr[v], dst_ptr[v+1])
__global__ void dst_sorted_kernel(const int32_t* __restrict__ dst_ptr, int64_t V,
                                  int32_t* __restrict__ dsts) {
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < V;
       v += (int64_t)gridDim.x * blockDim.x)
    for (int p = dst_ptr[v]; p < dst_ptr[v + 1]; ++p) dsts[p] = (int32_t)v;
}

}  // namespace

// XCDs (XCCs) of the current device: blocks b and b + xcd_count() share an XCD's L2 (dispatch is
// round-robin over the XCDs, MI355X_MICROARCH.md); 1 on a part or partition mode with one XCD.
int xcd_count() {
  static int n[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 1;
  if (n[dev] == 0) {
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeNumberOfXccs, dev) != hipSuccess || c <= 0) c = 1;
    n[dev] = c;
  }
  return n[dev];
}

int cu_count() {
  static int n[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (n[dev] == 0) {
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
      c = 256;
    n[dev] = c;
  }
  return n[dev];
}

bool ps_supported(int64_t h) { return h % 4 == 0 && h >= 4 && h <= 304; }

}  // namespace nt

extern "C" int64_t nt_dmpnn_tile_stride(int64_t E, int max_in_degree, int rows, int ncu) {
  if (E <= 0 || rows < 1 || max_in_degree > rows) return 0;
  const int64_t lmax = rows + 1 - (max_in_degree > 1 ? max_in_degree : 1);  // every tile <= rows
  if (ncu <= 0) return lmax;
  // balance: the fewest rounds of ncu tiles at stride <= lmax, then the stride that fills them evenly
  const int64_t rounds = (E + ncu * lmax - 1) / (ncu * lmax);
  int64_t L = (E + rounds * ncu - 1) / (rounds * ncu);
  return L < 1 ? 1 : (L > lmax ? lmax : L);
}

extern "C" int64_t nt_dmpnn_tile_count(int64_t E, int64_t stride) {
  if (E <= 0 || stride <= 0) return 0;
  return (E + stride - 1) / stride;
}

extern "C" int nt_dmpnn_tile_plan_hubs(const int32_t* dst_ptr, int64_t V, int64_t E, int64_t stride,
                                       int hub_degree, int32_t* tile_ptr, int64_t ntiles,
                                       int32_t* dst_sorted, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(hub_degree >= 1, NT_EINVAL, "hub_degree must be >= 1");
  NT_REQUIRE(V >= 0 && E >= 0 && E < (int64_t(1) << 31), NT_EINVAL, "bad sizes");
  NT_REQUIRE(E == 0 || (stride >= 1 && stride < (int64_t(1) << 30)), NT_EINVAL, "bad stride");
  NT_REQUIRE(ntiles == nt_dmpnn_tile_count(E, stride), NT_EINVAL,
             "ntiles != nt_dmpnn_tile_count(E, stride)");
  NT_REQUIRE(dst_ptr && tile_ptr && (E == 0 || dst_sorted), NT_EINVAL, "NULL pointer");
  hipStream_t stream = as_stream(stream_);
  tile_plan_kernel<<<(unsigned)((ntiles + 1 + 255) / 256), 256, 0, stream>>>(
      dst_ptr, V, E, (int)stride, (int)ntiles, hub_degree, tile_ptr);
  NT_LAUNCH_CHECK();
  if (E > 0 && V > 0) {
    dst_sorted_kernel<<<grid_for(V, 256), 256, 0, stream>>>(dst_ptr, V, dst_sorted);
    NT_LAUNCH_CHECK();
  }
  return NT_OK;
}

extern "C" int nt_dmpnn_tile_plan(const int32_t* dst_ptr, int64_t V, int64_t E, int64_t stride,
                                  int32_t* tile_ptr, int64_t ntiles, int32_t* dst_sorted,
                                  void* stream_) {
  return nt_dmpnn_tile_plan_hubs(dst_ptr, V, E, stride, INT32_MAX, tile_ptr, ntiles, dst_sorted, stream_);
}


// CSR (segment) construction for scatter-by-index: a stable LSD radix sort of the int64 index
// vector (hipCUB, key range clipped to ceil(log2(nseg+1)) bits), then a boundary kernel that
// writes seg_ptr.  Stability gives ascending source index inside every segment, i.e. the order
// in which the reference's CPU scatter_add_ accumulates (torch_scatter.scatter_sum ->
// zeros().scatter_add_, called from notorch/nn/gnn/chemprop.py:39,86 and agg.py:27,36,45).
//
// This runs once per batched graph (the collate normally ships the CSR already), never inside the
// per-layer loop, so it is not a roofline kernel.
#include <hipcub/hipcub.hpp>

#include "common.hpp"

namespace nt {

// idx (int64) -> uint32 key; out-of-range indices map to the sentinel nseg (sorted last, dropped).
__global__ void csr_keys_kernel(const int64_t* __restrict__ idx, int64_t n, int64_t nseg,
                                uint32_t* __restrict__ keys, int32_t* __restrict__ vals,
                                int32_t* __restrict__ err) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t k = idx[i];
    bool ok = (k >= 0) && (k < nseg);
    if (!ok && err) *err = 1;
    keys[i] = ok ? (uint32_t)k : (uint32_t)nseg;
    vals[i] = (int32_t)i;
  }
}

// seg_ptr[s] = first position p with keys[p] >= s  (lower bound), for s in [0, nseg]: one thread
// per segment, binary search in the sorted keys.  (A thread per position filling the empty
// segments after it was serial in the length of an empty run: the rev_index CSR of a compat-mode
// batch has tens of thousands of empty segments in one run, 264 us per build.)
__global__ void csr_bounds_kernel(const uint32_t* __restrict__ keys, int64_t n, int64_t nseg,
                                  int32_t* __restrict__ seg_ptr) {
  for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s <= nseg;
       s += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = n;  // first p in [0, n] with keys[p] >= s
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if ((int64_t)keys[mid] < s) lo = mid + 1;
      else hi = mid;
    }
    seg_ptr[s] = (int32_t)lo;
  }
}

static size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

static size_t cub_temp_bytes(int64_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                     (const int32_t*)nullptr, (int32_t*)nullptr, (int)n, 0, 32,
                                     (hipStream_t)0);
  return bytes;
}

}  // namespace nt

extern "C" size_t nt_csr_workspace_bytes(int64_t n, int64_t nseg) {
  (void)nseg;
  size_t nn = (size_t)(n > 0 ? n : 1);
  return 2 * nt::align_up(nn * 4) + nt::align_up(nn * 4) + nt::align_up(nt::cub_temp_bytes(n > 0 ? n : 1));
}

extern "C" int nt_csr_build(const int64_t* idx, int64_t n, int64_t nseg, int32_t* seg_ptr,
                            int32_t* perm, void* workspace, size_t workspace_bytes,
                            int32_t* err_flag, void* stream_) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(n >= 0 && nseg >= 0, NT_EINVAL, "negative size");
  NT_REQUIRE(n < (int64_t(1) << 31) && nseg < (int64_t(1) << 31) - 1, NT_EINVAL,
             "n and nseg must fit int32");
  NT_REQUIRE(seg_ptr != nullptr, NT_EINVAL, "seg_ptr is NULL");
  hipStream_t stream = as_stream(stream_);
  if (n == 0) {
    NT_HIP(hipMemsetAsync(seg_ptr, 0, sizeof(int32_t) * (nseg + 1), stream));
    return NT_OK;
  }
  NT_REQUIRE(idx && perm && workspace, NT_EINVAL, "NULL pointer");
  NT_REQUIRE(workspace_bytes >= nt_csr_workspace_bytes(n, nseg), NT_EINVAL,
             "workspace too small (see nt_csr_workspace_bytes)");
  char* ws = static_cast<char*>(workspace);
  uint32_t* keys_in = reinterpret_cast<uint32_t*>(ws);
  ws += align_up(n * 4);
  uint32_t* keys_out = reinterpret_cast<uint32_t*>(ws);
  ws += align_up(n * 4);
  int32_t* vals_in = reinterpret_cast<int32_t*>(ws);
  ws += align_up(n * 4);
  size_t temp_bytes = cub_temp_bytes(n);

  csr_keys_kernel<<<grid_for(n, 256), 256, 0, stream>>>(idx, n, nseg, keys_in, vals_in, err_flag);
  NT_LAUNCH_CHECK();
  int end_bit = 1;
  while (end_bit < 32 && ((uint64_t)nseg >> end_bit) != 0) ++end_bit;  // bits to hold sentinel nseg
  NT_HIP(hipcub::DeviceRadixSort::SortPairs(ws, temp_bytes, keys_in, keys_out, vals_in, perm, (int)n,
                                            0, end_bit, stream));
  csr_bounds_kernel<<<grid_for(nseg + 1, 256), 256, 0, stream>>>(keys_out, n, nseg, seg_ptr);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

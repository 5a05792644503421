// Dropout of the layer update fused with its residual add (the training path of
// chemprop.py:26 `update = Sequential(Linear, Dropout(p))` under residual.py:28 `H + module(H)`):
//
//   out[i] = (base ? base[i] : 0) + keep(seed, offset + i) * Y[i] / (1 - p)
//
// keep() is a counter-based hash of (seed, element index): the mask is never stored, the backward
// regenerates it from the same (seed, offset) (dY = keep * G / (1 - p) is this kernel with
// base = NULL).  The hash is the splitmix64 finaliser of seed + (i + 1) * golden-ratio; an element
// is kept when its top 32 bits are >= p * 2^32, i.e. with probability 1 - p (p = 1 drops all,
// out = base, like torch.nn.Dropout(1.0)).  HBM-bound: 2-3 rows of traffic per row.
#include "common.hpp"
#include "rows.hpp"

namespace nt {

namespace {

__device__ __forceinline__ uint32_t drop_hash(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}

template <typename T, bool VEC>
__global__ void __launch_bounds__(256) dropout_residual_kernel(const T* __restrict__ base,
                                                               const T* __restrict__ Y, int64_t n,
                                                               uint32_t thr, int drop_all,
                                                               float scale, uint64_t seed,
                                                               uint64_t offset, T* __restrict__ out) {
  using P = Piece<T, VEC>;
  constexpr int N = P::N;
  const int64_t pieces = n / N;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < pieces;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i0 = t * N;
    float y[N], b[N];
    P::load(Y + i0, y);
    if (base) P::load(base + i0, b);
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const bool keep = !drop_all && drop_hash(seed, offset + (uint64_t)(i0 + k)) >= thr;
      const float v = keep ? y[k] * scale : 0.f;
      y[k] = base ? b[k] + v : v;
    }
    P::store(out + i0, y);
  }
}

template <typename T>
void launch_dropout(const void* base, const void* Y, int64_t n, float p, uint64_t seed,
                    uint64_t offset, void* out, hipStream_t stream) {
  const bool drop_all = p >= 1.f;
  const double t = (double)p * 4294967296.0;
  const uint32_t thr = drop_all ? 0u : (uint32_t)(t >= 4294967295.0 ? 4294967295.0 : t);
  const float scale = drop_all ? 0.f : 1.f / (1.f - p);
  constexpr int NV = 16 / sizeof(T);
  const bool vec = n % NV == 0 && aligned16(Y) && aligned16(out) && (!base || aligned16(base));
  const int grid = grid_for(vec ? n / NV : n, 256, 256 * 32);
  if (vec)
    dropout_residual_kernel<T, true><<<grid, 256, 0, stream>>>(
        (const T*)base, (const T*)Y, n, thr, drop_all, scale, seed, offset, (T*)out);
  else
    dropout_residual_kernel<T, false><<<grid, 256, 0, stream>>>(
        (const T*)base, (const T*)Y, n, thr, drop_all, scale, seed, offset, (T*)out);
}

}  // namespace

}  // namespace nt

using namespace nt;

extern "C" int nt_dropout_residual(const void* base, const void* Y, int64_t n, float p,
                                   uint64_t seed, uint64_t offset, int dtype, void* out,
                                   void* stream_) {
  clear_error();
  NT_REQUIRE(dtype == NT_F32 || dtype == NT_BF16, NT_EUNSUPPORTED, "dtype must be NT_F32 or NT_BF16");
  NT_REQUIRE(n >= 0, NT_EINVAL, "bad sizes");
  NT_REQUIRE(p >= 0.f && p <= 1.f, NT_EINVAL, "dropout probability must be in [0, 1]");
  if (n == 0) return NT_OK;
  NT_REQUIRE(Y && out, NT_EINVAL, "NULL pointer");
  hipStream_t stream = as_stream(stream_);
  if (dtype == NT_BF16)
    launch_dropout<bf16_raw>(base, Y, n, p, seed, offset, out, stream);
  else
    launch_dropout<float>(base, Y, n, p, seed, offset, out, stream);
  NT_LAUNCH_CHECK();
  return NT_OK;
}

// Micro-benchmark: cycles per v_mfma_f32_16x16x32_f16 in the fw K-loop shape (one wave per SIMD,
// 8 row tiles x 5 column tiles x 3 split products per step), with the A fragments re-read from LDS
// (as the fw walk does) or kept in registers.  Prints cycles per MFMA per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <int MODE>  // 0: operands in registers; 1: A fragments from LDS each row tile (1 ahead);
                     // 2: as 1 plus the 3 products of one (rt, j) back to back (chain order)
__global__ void __launch_bounds__(256, 1) mb(const uint4* __restrict__ w, float* out, unsigned long long* cyc,
                                             int steps) {
  __shared__ __attribute__((aligned(16))) char lds[16384];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 1024; i += 256) reinterpret_cast<uint4*>(lds)[i] = w[i];
  __syncthreads();
  f32x4 acc[8][5];
  for (int r = 0; r < 8; ++r)
    for (int j = 0; j < 5; ++j) acc[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f16x8 w0[5], w1[5];
  for (int j = 0; j < 5; ++j) {
    w0[j] = __builtin_bit_cast(f16x8, w[j * 64 + lane]);
    w1[j] = __builtin_bit_cast(f16x8, w[(j + 5) * 64 + lane]);
  }
  f16x8 ar0 = __builtin_bit_cast(f16x8, w[lane + 640]), ar1 = __builtin_bit_cast(f16x8, w[lane + 704]);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int s = 0; s < steps; ++s) {
    const char* bb = lds + (s & 1) * 8192 + lane * 16;
    f16x8 a0 = MODE ? *reinterpret_cast<const f16x8*>(bb) : ar0;
    f16x8 a1 = MODE ? *reinterpret_cast<const f16x8*>(bb + 4096) : ar1;
#pragma unroll
    for (int rt = 0; rt < 8; ++rt) {
      f16x8 n0 = a0, n1 = a1;
      if (MODE && rt + 1 < 8) {
        n0 = *reinterpret_cast<const f16x8*>(bb + ((rt + 1) & 3) * 1024);
        n1 = *reinterpret_cast<const f16x8*>(bb + 4096 + ((rt + 1) & 3) * 1024);
      }
      if (MODE == 2) {
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[j], a0, acc[rt][j], 0, 0, 0);
          acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0[j], a1, acc[rt][j], 0, 0, 0);
          acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0[j], a0, acc[rt][j], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[j], a0, acc[rt][j], 0, 0, 0);
          acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0[j], a1, acc[rt][j], 0, 0, 0);
          acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0[j], a0, acc[rt][j], 0, 0, 0);
        }
      }
      a0 = n0;
      a1 = n1;
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float sum = 0.f;
  for (int r = 0; r < 8; ++r)
    for (int j = 0; j < 5; ++j) sum += acc[r][j][0] + acc[r][j][1] + acc[r][j][2] + acc[r][j][3];
  out[blockIdx.x * 256 + threadIdx.x] = sum;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
void run(const uint4* w, float* out, unsigned long long* cyc, int grid, int steps) {
  mb<MODE><<<grid, 256>>>(w, out, cyc, steps);
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  mb<MODE><<<grid, 256>>>(w, out, cyc, steps);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  std::vector<unsigned long long> h(grid);
  hipMemcpy(h.data(), cyc, grid * 8, hipMemcpyDeviceToHost);
  double avg = 0;
  for (auto v : h) avg += v;
  avg /= grid;
  const double mfma = 120.0 * steps;
  printf("mode %d grid %d: %.1f cycles per MFMA per wave (s_memtime), wall %.1f us -> %.1f ns per MFMA\n", MODE,
         grid, avg / mfma, ms * 1e3, ms * 1e6 / mfma);
}

int main() {
  uint4* w;
  float* out;
  unsigned long long* cyc;
  hipMalloc(&w, 1024 * 16);
  hipMemset(w, 0x11, 1024 * 16);  // small fp16 values (0x1111 = 6.5e-4) stay finite
  hipMalloc(&out, 1024 * 256 * 4);
  hipMalloc(&cyc, 1024 * 8);
  for (int g : {256, 1024}) {
    run<0>(w, out, cyc, g, 2000);
    run<1>(w, out, cyc, g, 2000);
    run<2>(w, out, cyc, g, 2000);
  }
  return 0;
}

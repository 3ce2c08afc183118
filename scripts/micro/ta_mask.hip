// Microbenchmark: does the texture-address path cost scale with active lanes / active quads?
// Gather 16 B per lane from an L2-resident table; variants mask lanes in different patterns.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void gather(const float* __restrict__ tab, float* __restrict__ out, int iters,
                                              unsigned mask_n) {
  const int lane = threadIdx.x & 63;
  bool act = true;
  if (MODE == 1) act = ((lane >> 2) & 1) == 0;  // half the quads fully inactive
  if (MODE == 2) act = (lane & 1) == 0;         // half the lanes, every quad partially active
  if (MODE == 3) act = ((lane >> 2) & 3) == 0;  // a quarter of the quads
  const bool oob = (MODE == 4 && (lane & 1)) || (MODE == 5 && ((lane >> 2) & 1));  // out-of-range offset instead of exec mask
  __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void*)tab, (short)0, (int)(mask_n * 16u), 0x00020000);
  unsigned idx = (blockIdx.x * 256 + threadIdx.x) * 2654435761u;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < iters; ++i) {
    idx = idx * 1664525u + 1013904223u;
    const unsigned off = oob ? 0x80000000u : ((idx >> 8) % mask_n) * 16u;
    if (act) {
      floatx4 v = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
      acc += v;
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

template <int MODE>
float run(const float* tab, float* out, int blocks, int iters, unsigned n) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(gather<MODE>, dim3(blocks), dim3(256), 0, 0, tab, out, iters, n);
  hipEventRecord(a);
  for (int k = 0; k < 5; ++k) hipLaunchKernelGGL(gather<MODE>, dim3(blocks), dim3(256), 0, 0, tab, out, iters, n);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  const unsigned n = 1u << 16;  // 1 MiB table: L2 resident
  const int blocks = 256 * 8, iters = 256;
  float *tab, *out;
  hipMalloc(&tab, n * 16);
  hipMalloc(&out, blocks * 256 * 4);
  hipMemset(tab, 0, n * 16);
  const double loads = (double)blocks * 4 * iters;  // wave-level load instructions
  float t0 = run<0>(tab, out, blocks, iters, n), t1 = run<1>(tab, out, blocks, iters, n);
  float t2 = run<2>(tab, out, blocks, iters, n), t3 = run<3>(tab, out, blocks, iters, n);
  float t4 = run<4>(tab, out, blocks, iters, n), t5 = run<5>(tab, out, blocks, iters, n);
  printf("all lanes        : %.3f ms  %.2f cycles/instr/CU\n", t0, t0 * 1e-3 * 2.4e9 * 256 / loads);
  printf("half quads       : %.3f ms  %.2f\n", t1, t1 * 1e-3 * 2.4e9 * 256 / loads);
  printf("half lanes (odd) : %.3f ms  %.2f\n", t2, t2 * 1e-3 * 2.4e9 * 256 / loads);
  printf("quarter quads    : %.3f ms  %.2f\n", t3, t3 * 1e-3 * 2.4e9 * 256 / loads);
  printf("half lanes OOB   : %.3f ms  %.2f\n", t4, t4 * 1e-3 * 2.4e9 * 256 / loads);
  printf("half quads OOB   : %.3f ms  %.2f\n", t5, t5 * 1e-3 * 2.4e9 * 256 / loads);
  return 0;
}

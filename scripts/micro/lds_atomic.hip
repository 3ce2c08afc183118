// Microbenchmark: LDS atomic add rate on gfx950 against plain LDS stores, by address pattern.
// Reports LDS-unit cycles per wave-instruction per CU (2.4 GHz), 4 blocks x 4 waves per CU.
//   hipcc -O3 --offload-arch=gfx950 scripts/micro/lds_atomic.hip -o /tmp/lds_atomic && /tmp/lds_atomic
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kCells = 585 * 8;

template <int MODE>
__global__ __launch_bounds__(256) void lds_kernel(float* __restrict__ out, int iters) {
  __shared__ float win[kCells];
  __shared__ unsigned wu[kCells];
  for (int i = threadIdx.x; i < kCells; i += 256) win[i] = 0.f, wu[i] = 0u;
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  unsigned h = (blockIdx.x * 256 + threadIdx.x) * 2654435761u;
  float v = 1.f + lane;
  for (int i = 0; i < iters; ++i) {
    const int c = i & 7;
    int a;
    if (MODE == 0 || MODE == 1 || MODE == 4) a = c * 585 + wv * 64 + lane;       // distinct, consecutive
    else if (MODE == 2) a = c * 585 + wv * 64 + (lane >> 1);                     // 2 lanes per address
    else if (MODE == 3) { h = h * 1664525u + 1013904223u; a = c * 585 + (int)((h >> 8) % 585u); }  // random
    else if (MODE == 5) a = c * 585 + 0;                                          // one address
    else if (MODE == 6) a = c * 585 + 2 * lane;                                   // stride 2 (bank pairs)
    else a = (wv * 64 + lane) * 8 + c;                                            // cell-major, stride 8
    if (MODE == 0) win[a] = v;
    else if (MODE == 4) atomicAdd(&wu[a], 1u);
    else atomicAdd(&win[a], v);
    v += 1.f;
  }
  __syncthreads();
  float s = 0.f;
  for (int i = threadIdx.x; i < kCells; i += 256) s += win[i] + (float)wu[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE>
void run(const char* name, float* out) {
  const int blocks = 256 * 4, iters = 4096;
  hipLaunchKernelGGL(lds_kernel<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  for (int k = 0; k < 5; ++k) hipLaunchKernelGGL(lds_kernel<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  ms /= 5;
  const double instr_per_cu = (double)blocks * 4 * iters / 256;
  printf("%-34s %8.3f ms  %7.1f cycles per wave-instruction per CU\n", name, ms, ms * 1e-3 * 2.4e9 / instr_per_cu);
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 4 * 256 * 4);
  run<0>("ds_write_b32 consecutive", out);
  run<1>("ds_add_f32 consecutive", out);
  run<2>("ds_add_f32 2 lanes/address", out);
  run<3>("ds_add_f32 random in 585", out);
  run<4>("ds_add_u32 consecutive", out);
  run<5>("ds_add_f32 one address", out);
  run<6>("ds_add_f32 stride 2", out);
  run<7>("ds_add_f32 stride 8", out);
  hipFree(out);
  return 0;
}

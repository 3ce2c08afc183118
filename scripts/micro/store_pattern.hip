// Microbenchmark: HBM write rate for the store patterns of the full-resolution VALU convs.
// Each wave writes 8 "planes" x 2 KiB (64 voxels x 32 B), planes PLANE bytes apart, 256 MiB total.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float fx4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void store(float* __restrict__ y, long plane_floats, int rows) {
  const int lane = threadIdx.x & 63;
  const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wave >= rows) return;
  __shared__ float4 stage[4][128];
  float4* st = stage[threadIdx.x >> 6];
  float4 v0 = make_float4(lane, 1.f, 2.f, 3.f), v1 = make_float4(4.f, 5.f, 6.f, (float)wave);
  for (int d = 0; d < 8; ++d) {
    float* base = y + (MODE == 3 ? (wave * 8 + d) * 512 : d * plane_floats + wave * (MODE == 2 || MODE == 7 ? 496 : 512));
    float4* q = reinterpret_cast<float4*>(base);
    if (MODE == 0) {  // lane-contiguous: each instruction 1 KiB contiguous
      q[lane] = v0;
      q[lane + 64] = v1;
    } else if (MODE == 1 || MODE == 3) {  // 32 B per lane, two 16 B stores at a 32 B lane stride
      q[2 * lane] = v0;
      q[2 * lane + 1] = v1;
    } else if (MODE == 4) {  // 32 B lane stride, nontemporal
      fx4* r = reinterpret_cast<fx4*>(q);
      __builtin_nontemporal_store(fx4{v0.x, v0.y, v0.z, v0.w}, &r[2 * lane]);
      __builtin_nontemporal_store(fx4{v1.x, v1.y, v1.z, v1.w}, &r[2 * lane + 1]);
    } else if (MODE == 5) {  // lane-contiguous, nontemporal
      fx4* r = reinterpret_cast<fx4*>(q);
      __builtin_nontemporal_store(fx4{v0.x, v0.y, v0.z, v0.w}, &r[lane]);
      __builtin_nontemporal_store(fx4{v1.x, v1.y, v1.z, v1.w}, &r[lane + 64]);
    } else if (MODE == 7) {  // lane-contiguous chunks of a 62-voxel misaligned row
      if (lane >= 2) q[lane - 2] = v0;
      if (lane < 62) q[lane + 62] = v1;
    } else if (MODE == 8) {  // per-voxel 32 B through LDS, then lane-contiguous stores
      st[2 * lane] = v0;
      st[2 * lane + 1] = v1;
      __builtin_amdgcn_wave_barrier();
      const float4 a = st[lane], b = st[lane + 64];
      __builtin_amdgcn_wave_barrier();
      q[lane] = a;
      q[lane + 64] = b;
    } else {  // conv0: 62 of 64 lanes, rows 62 voxels apart (misaligned)
      if (lane >= 1 && lane <= 62) {
        q[2 * lane - 2] = v0;
        q[2 * lane - 1] = v1;
      }
    }
    v0.y += 1.f;
  }
}

template <int MODE>
float run(float* y, long plane_floats, int rows) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int blocks = (rows + 3) / 4;
  hipLaunchKernelGGL(store<MODE>, dim3(blocks), dim3(256), 0, 0, y, plane_floats, rows);
  hipEventRecord(a);
  for (int k = 0; k < 10; ++k) hipLaunchKernelGGL(store<MODE>, dim3(blocks), dim3(256), 0, 0, y, plane_floats, rows);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 10;
}

int main() {
  const long total = 256l << 20;                // bytes
  const int rows = (int)(total / (8 * 2048));   // waves
  const long plane_floats = (long)rows * 512;   // one plane = all waves' rows
  float* y;
  hipMalloc(&y, total + (1 << 20));
  const char* names[] = {"lane-contiguous", "32B lane stride", "conv0 62-lane misaligned", "wave-contiguous planes",
                         "32B lane stride, nt", "lane-contiguous, nt", "lane-contig 62 misaligned", "LDS staged"};
  float t[8] = {run<0>(y, plane_floats, rows), run<1>(y, plane_floats, rows), run<6>(y, plane_floats, rows),
                run<3>(y, plane_floats, rows), run<4>(y, plane_floats, rows), run<5>(y, plane_floats, rows), run<7>(y, plane_floats, rows), run<8>(y, plane_floats, rows)};
  for (int m = 0; m < 8; ++m) printf("%-26s %7.1f us  %6.0f GB/s\n", names[m], t[m] * 1e3, total / (t[m] * 1e-3) / 1e9);
  return 0;
}

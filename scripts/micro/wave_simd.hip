// Which SIMD each wave of a 1024-thread workgroup runs on (HW_ID.SIMD_ID, bits 5:4 of hwreg 4 on gfx9-family
// parts): decides how the fused conv11 + prob kernel's MFMA / walk wave roles should alternate so that every
// SIMD holds both roles. One workgroup per CU (LDS-limited, as that kernel).
//   hipcc --offload-arch=gfx950 -O2 scripts/micro/wave_simd.hip -o /tmp/wave_simd && /tmp/wave_simd
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(1024) void wave_simd(unsigned* out) {
  __shared__ float pad[27000];  // 108 KB: one workgroup per CU
  pad[threadIdx.x] = 0.f;
  __syncthreads();
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_REG_HW_ID, offset 0, 32 bits
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + (threadIdx.x >> 6)] = hw + (pad[threadIdx.x] != 0.f);
}

int main() {
  const int nb = 8;
  unsigned* d;
  hipMalloc(&d, nb * 16 * sizeof(unsigned));
  hipLaunchKernelGGL(wave_simd, dim3(nb), dim3(1024), 0, 0, d);
  unsigned h[nb * 16];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int b = 0; b < nb; ++b) {
    printf("block %d SIMD of waves 0..15:", b);
    for (int w = 0; w < 16; ++w) printf(" %u", (h[b * 16 + w] >> 4) & 3);
    printf("   (wave slot:");
    for (int w = 0; w < 16; ++w) printf(" %u", h[b * 16 + w] & 15);
    printf(")\n");
  }
  hipFree(d);
  return 0;
}

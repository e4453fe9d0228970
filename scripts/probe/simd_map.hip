// Which SIMD does each wave of a 512-thread workgroup run on?  (HW_REG_HW_ID bits 5:4 on gfx9.)
// Workgroups of 8 waves with 160 KB of LDS (one per CU, as the wave-specialised dgrad).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(512) void probe(int* out, int lds_kb) {
  extern __shared__ int sm[];
  const int w = threadIdx.x >> 6;
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_ID, all 32 bits
  if ((threadIdx.x & 63) == 0) {
    sm[w] = (int)hw;
    out[blockIdx.x * 8 + w] = (int)hw;
  }
  (void)lds_kb;
}
int main() {
  int* d;
  const int nb = 512;
  hipMalloc(&d, nb * 8 * sizeof(int));
  hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int kb : {160, 16}) {
    hipLaunchKernelGGL(probe, dim3(nb), dim3(512), kb * 1024, 0, d, kb);
    hipDeviceSynchronize();
    int h[nb * 8];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int hist[8][4] = {};
    for (int b = 0; b < nb; ++b)
      for (int w = 0; w < 8; ++w) hist[w][(h[b * 8 + w] >> 4) & 3]++;
    printf("LDS %d KB: wave -> SIMD histogram over %d workgroups\n", kb, nb);
    for (int w = 0; w < 8; ++w) printf("  wave %d: %d %d %d %d\n", w, hist[w][0], hist[w][1], hist[w][2], hist[w][3]);
    printf("  block 0 raw:");
    for (int w = 0; w < 8; ++w) printf(" %08x", h[w]);
    printf("\n");
  }
  hipFree(d);
  return 0;
}

// probe: does an out-of-range buffer_load ... lds (LDS-DMA) write zeros into LDS, or leave it?
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef short s16x4 __attribute__((ext_vector_type(4)));
__global__ void k(const float* g, float* out, int nbytes) {
  __shared__ __attribute__((aligned(16))) float lds[256 * 4];
  for (int i = threadIdx.x; i < 1024; i += 64) lds[i] = -7.f;   // stale marker
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)g, (short)0, nbytes, 0x00020000);
  const unsigned off = (threadIdx.x & 1) ? 0x80000000u : threadIdx.x * 16u;   // odd lanes OOB
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, off, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += 64) out[i] = lds[i];
  // tr read check: 4 rows x 16 cols of 16-bit values laid out row-major with 32-B rows
  __shared__ __attribute__((aligned(16))) unsigned short t[64 * 16];
  for (int i = threadIdx.x; i < 64 * 16; i += 64) t[i] = (unsigned short)i;
  __syncthreads();
  const int g16 = threadIdx.x >> 4, l = threadIdx.x & 15, q = l >> 2, p = l & 3;
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(t + (g16 * 4 + q) * 16 + 4 * p));
  for (int e = 0; e < 4; ++e) out[256 + threadIdx.x * 4 + e] = (float)(unsigned short)v[e];
}
int main() {
  float *g, *o;
  hipMalloc(&g, 4096); hipMalloc(&o, 4096 * 4);
  float h[1024]; for (int i = 0; i < 1024; ++i) h[i] = (float)(i + 1);
  hipMemcpy(g, h, 4096, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, g, o, 4096);
  float r[512]; hipMemcpy(r, o, 512 * 4, hipMemcpyDeviceToHost);
  printf("glds lanes 0..3 (16B each):");
  for (int i = 0; i < 16; ++i) printf(" %g", r[i]);
  printf("\ntr16 lane0: %g %g %g %g  lane1: %g %g %g %g  lane16: %g %g %g %g\n", r[256], r[257], r[258], r[259],
         r[260], r[261], r[262], r[263], r[256 + 64], r[257 + 64], r[258 + 64], r[259 + 64]);
  return 0;
}

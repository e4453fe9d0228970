// Shared helpers for libtmr (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define TMR_API extern "C" __attribute__((visibility("default")))

// Thread-local last-error message (tmr_last_error in api.cpp).
void tmr_set_error(const char* fmt, ...);

#define TMR_CHECK_ARG(cond, ...)            \
  do {                                      \
    if (!(cond)) {                          \
      tmr_set_error(__VA_ARGS__);           \
      return 1;                             \
    }                                       \
  } while (0)

#define TMR_CHECK_LAUNCH(name)                                                \
  do {                                                                        \
    hipError_t e_ = hipGetLastError();                                        \
    if (e_ != hipSuccess) {                                                   \
      tmr_set_error("%s: launch failed: %s", name, hipGetErrorString(e_));    \
      return 2;                                                               \
    }                                                                         \
  } while (0)

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

// Unsigned division by a runtime-invariant divisor (n < 2^31).
struct FastDiv {
  uint32_t d, m, s;
};
static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
  if (d == 1) { f.m = 0; f.s = 0; }
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (__umulhi(n, f.m) + n) >> f.s;
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double warp_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// Gradient reaching input pixel (nn, iy, ix), channel quad cq, through MaxPool2d(3, 2, 1): the
// gather form of its backward (each input pixel sits in at most 2x2 windows; a window passes its
// gradient to the input its argmax -- the first maximum in scan order, 0..8 -- points at).
__device__ __forceinline__ float4 maxpool_grad4(const float* __restrict__ dy,
                                                const uchar4* __restrict__ am, int nn, int iy,
                                                int ix, int cq, int c4, int ho, int wo) {
  float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
  const int oy0 = iy / 2, oy1 = min((iy + 1) / 2, ho - 1);
  const int ox0 = ix / 2, ox1 = min((ix + 1) / 2, wo - 1);
  for (int oy = oy0; oy <= oy1; ++oy) {
    for (int ox = ox0; ox <= ox1; ++ox) {
      const long o = (((long)nn * ho + oy) * wo + ox) * c4 + cq;
      const unsigned char id = (unsigned char)((iy - (oy * 2 - 1)) * 3 + (ix - (ox * 2 - 1)));
      const uchar4 a = am[o];
      const float4 d = reinterpret_cast<const float4*>(dy)[o];
      if (a.x == id) g.x += d.x;
      if (a.y == id) g.y += d.y;
      if (a.z == id) g.z += d.z;
      if (a.w == id) g.w += d.w;
    }
  }
  return g;
}

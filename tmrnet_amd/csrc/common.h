// Shared helpers for libtmr (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
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

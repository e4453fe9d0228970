// Pooling, layout conversion and the input transform (HBM-bound kernels).
//
//  * MaxPool2d(3,2,1) / AdaptiveAvgPool2d(1) of torchvision resnet50 as used by
//    the `share` trunk (code/Training TMRNet/train_only_non-local_pretrained.py:207,:214)
//  * per-clip RandomCrop + ToTensor + Normalize of the train transform
//    (train_only_non-local_pretrained.py:101-126 crop with per-clip seed,
//    :335-341 Normalize constants), producing the NHWC4 layout the stem conv reads.
#include "common.h"
#include <type_traits>
#include "tmr.h"

namespace {
constexpr int NT = 256;

int ew_blocks(long n) {
  long b = (n + NT - 1) / NT;
  if (b > 8192) b = 8192;
  return (int)(b > 0 ? b : 1);
}

__device__ __forceinline__ float4 ldx4(const float* p, long i4) {
  return reinterpret_cast<const float4*>(p)[i4];
}
__device__ __forceinline__ float4 ldx4(const __bf16* p, long i4) {   // bf16 -> fp32, exact
  const uint2 u = reinterpret_cast<const uint2*>(p)[i4];
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                     __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
}

// BN: the input is the stem conv's pre-BN output; relu(x*scale + shift) is applied per loaded
// element (the stem's BN+ReLU output is never materialised; same fmaf/max as bn_apply).
template <bool BN, typename TY = float, typename TX = float>
__global__ __launch_bounds__(NT) void maxpool_fwd_k(const TX* __restrict__ x, TY* __restrict__ y,
                                                    uchar4* __restrict__ am, int n, int h, int w,
                                                    int c4, int ho, int wo,
                                                    const float* __restrict__ scale,
                                                    const float* __restrict__ shift) {
  const long total = (long)n * ho * wo * c4;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int cq = (int)(i % c4);
    long p = i / c4;
    const int ox = (int)(p % wo);
    p /= wo;
    const int oy = (int)(p % ho);
    const int nn = (int)(p / ho);
    float4 best = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    uchar4 bi = make_uchar4(0, 0, 0, 0);
    float4 sc = make_float4(1.f, 1.f, 1.f, 1.f), sf = make_float4(0.f, 0.f, 0.f, 0.f);
    if (BN) {
      sc = reinterpret_cast<const float4*>(scale)[cq];
      sf = reinterpret_cast<const float4*>(shift)[cq];
    }
    for (int dy = 0; dy < 3; ++dy) {
      const int iy = oy * 2 - 1 + dy;
      if (iy < 0 || iy >= h) continue;
      for (int dx = 0; dx < 3; ++dx) {
        const int ix = ox * 2 - 1 + dx;
        if (ix < 0 || ix >= w) continue;
        float4 v = ldx4(x, (((long)nn * h + iy) * w + ix) * c4 + cq);
        if (BN) {
          v.x = fmaxf(fmaf(v.x, sc.x, sf.x), 0.f);
          v.y = fmaxf(fmaf(v.y, sc.y, sf.y), 0.f);
          v.z = fmaxf(fmaf(v.z, sc.z, sf.z), 0.f);
          v.w = fmaxf(fmaf(v.w, sc.w, sf.w), 0.f);
        }
        const unsigned char id = (unsigned char)(dy * 3 + dx);
        // first maximum in scan order wins (PyTorch: val > max || isnan(val))
        if (v.x > best.x || isnan(v.x)) { best.x = v.x; bi.x = id; }
        if (v.y > best.y || isnan(v.y)) { best.y = v.y; bi.y = id; }
        if (v.z > best.z || isnan(v.z)) { best.z = v.z; bi.z = id; }
        if (v.w > best.w || isnan(v.w)) { best.w = v.w; bi.w = id; }
      }
    }
    if constexpr (std::is_same<TY, float>::value) {
      reinterpret_cast<float4*>(y)[i] = best;
    } else {   // bf16 (RNE): a tensor consumed only as a bf16-math conv operand
      typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
      const bf16x2_t lo = {(__bf16)best.x, (__bf16)best.y}, hi = {(__bf16)best.z, (__bf16)best.w};
      reinterpret_cast<uint2*>(y)[i] =
          make_uint2(__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi));
    }
    am[i] = bi;
  }
}

// 8 consecutive values (index i in units of 8) of an fp32 / bf16 tensor as raw words, and their
// fp32 values
struct Raw8 { uint4 a, b; };
__device__ __forceinline__ Raw8 ld_raw8(const float* p, int i) {
  // 64-bit element offset: the host guard bounds i (< 2^31), not 2 i
  const long j = 2 * (long)i;
  return {reinterpret_cast<const uint4*>(p)[j], reinterpret_cast<const uint4*>(p)[j + 1]};
}
__device__ __forceinline__ Raw8 ld_raw8(const __bf16* p, int i) {
  return {reinterpret_cast<const uint4*>(p)[i], make_uint4(0u, 0u, 0u, 0u)};
}
template <typename T>
__device__ __forceinline__ float raw_val(const Raw8& r, int e) {
  if constexpr (std::is_same<T, float>::value) {
    const uint4 q = e < 4 ? r.a : r.b;
    const uint32_t w4[4] = {q.x, q.y, q.z, q.w};
    return __uint_as_float(w4[e & 3]);
  } else {
    const uint32_t w4[4] = {r.a.x, r.a.y, r.a.z, r.a.w};
    return __uint_as_float((e & 1) ? (w4[e >> 1] & 0xffff0000u) : (w4[e >> 1] << 16));
  }
}

// The 8-channel form (the bf16-activation step's bf16 pre-BN input and bf16 output; round 5: the
// fp32 step's fp32 input too), 8 channels per thread: 32-bit magic-number index division instead
// of maxpool_fwd_k's 64-bit divides, the 9 window loads issued before any is consumed, 16-B
// stores of y and 8-B argmax stores.  Same BN+ReLU arithmetic and scan order as maxpool_fwd_k:
// identical outputs.  total = n*ho*wo*c/8 < 2^31, c / 8 a power of two (lc8 = log2), both
// checked on the host.
template <typename TX, typename TY>
__global__ __launch_bounds__(NT) void maxpool_fwd_bn8(const TX* __restrict__ x, TY* __restrict__ y,
                                                     uint2* __restrict__ am, int total, int h,
                                                     int w, int lc8, FastDiv dHWo, FastDiv dWo,
                                                     const float* __restrict__ scale,
                                                     const float* __restrict__ shift) {
  const int c8 = 1 << lc8;
  for (int i = blockIdx.x * NT + threadIdx.x; i < total; i += gridDim.x * NT) {
    const int cq = i & (c8 - 1);
    const uint32_t p = (uint32_t)i >> lc8;
    const uint32_t nn = fdiv(p, dHWo);
    const uint32_t rem = p - nn * dHWo.d;
    const int oy = (int)fdiv(rem, dWo), ox = (int)(rem - (uint32_t)oy * dWo.d);
    Raw8 u[9];
    bool ok[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int iy = oy * 2 - 1 + k / 3, ix = ox * 2 - 1 + k % 3;
      ok[k] = iy >= 0 && iy < h && ix >= 0 && ix < w;
      const int src = ok[k] ? (((int)nn * h + iy) * w + ix) * c8 + cq : i;
      u[k] = ld_raw8(x, src);
    }
    float sc[8], sf[8];
    {
      const float4 s0 = reinterpret_cast<const float4*>(scale)[2 * cq];
      const float4 s1 = reinterpret_cast<const float4*>(scale)[2 * cq + 1];
      const float4 f0 = reinterpret_cast<const float4*>(shift)[2 * cq];
      const float4 f1 = reinterpret_cast<const float4*>(shift)[2 * cq + 1];
      const float a[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      const float b[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) { sc[e] = a[e]; sf[e] = b[e]; }
    }
    float best[8];
    uint32_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; bi[e] = 0u; }
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      if (!ok[k]) continue;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float raw = raw_val<TX>(u[k], e);
        const float v = fmaxf(fmaf(raw, sc[e], sf[e]), 0.f);
        // first maximum in scan order wins (PyTorch: val > max || isnan(val))
        if (v > best[e] || isnan(v)) { best[e] = v; bi[e] = (uint32_t)k; }
      }
    }
    if constexpr (std::is_same<TY, float>::value) {
      const long j = 2 * (long)i;
      reinterpret_cast<float4*>(y)[j] = make_float4(best[0], best[1], best[2], best[3]);
      reinterpret_cast<float4*>(y)[j + 1] = make_float4(best[4], best[5], best[6], best[7]);
    } else {
      typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
      uint32_t ow[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bf16x2_t pr = {(__bf16)best[2 * e], (__bf16)best[2 * e + 1]};
        ow[e] = __builtin_bit_cast(uint32_t, pr);
      }
      reinterpret_cast<uint4*>(y)[i] = make_uint4(ow[0], ow[1], ow[2], ow[3]);
    }
    am[i] = make_uint2(bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24),
                       bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24));
  }
}

__global__ __launch_bounds__(NT) void maxpool_bwd_k(const float* __restrict__ dy, const uchar4* __restrict__ am,
                                                    float* __restrict__ dx, int n, int h, int w,
                                                    int c4, int ho, int wo) {
  const long total = (long)n * h * w * c4;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int cq = (int)(i % c4);
    long p = i / c4;
    const int ix = (int)(p % w);
    p /= w;
    const int iy = (int)(p % h);
    const int nn = (int)(p / h);
    const float4 g = maxpool_grad4(dy, am, nn, iy, ix, cq, c4, ho, wo);
    reinterpret_cast<float4*>(dx)[i] = g;
  }
}

template <typename TX = float>
__global__ __launch_bounds__(NT) void avgpool_fwd_k(const TX* __restrict__ x, float* __restrict__ y, int n,
                                                    int hw, int c4) {
  const long total = (long)n * c4;
  const float inv = 1.0f / (float)hw;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int cq = (int)(i % c4);
    const long nn = i / c4;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    const long base = nn * hw * c4 + cq;
    for (int p = 0; p < hw; ++p) {
      const float4 v = ldx4(x, base + (long)p * c4);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    s.x *= inv; s.y *= inv; s.z *= inv; s.w *= inv;
    reinterpret_cast<float4*>(y)[i] = s;
  }
}

__global__ __launch_bounds__(NT) void avgpool_bwd_k(const float* __restrict__ dy, float* __restrict__ dx, int n,
                                                    int hw, int c4) {
  const long total = (long)n * hw * c4;
  const float inv = 1.0f / (float)hw;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int cq = (int)(i % c4);
    const long nn = i / ((long)hw * c4);
    float4 d = reinterpret_cast<const float4*>(dy)[nn * c4 + cq];
    d.x *= inv; d.y *= inv; d.z *= inv; d.w *= inv;
    reinterpret_cast<float4*>(dx)[i] = d;
  }
}

template <typename TO>
__global__ void oihw_to_krsc_k(const float* __restrict__ w, TO* __restrict__ wk, int k, int c,
                               int rs, int cpad) {
  const long total = (long)k * rs * cpad;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int ci = (int)(i % cpad);
    const long t = i / cpad;
    const int tap = (int)(t % rs);
    const int ko = (int)(t / rs);
    wk[i] = (TO)(ci < c ? w[((long)ko * c + ci) * rs + tap] : 0.f);   // bf16: RNE
  }
}

// OIHW -> [Cin][R][S][Cout] (the transposed weights of the dgrad view, TMR_IO_WT_BF16); writes
// along co are strided, the weights are small (<= 9.4 MB per tensor)
template <typename TO>
__global__ void oihw_to_crsk_k(const float* __restrict__ w, TO* __restrict__ wt, int k, int c,
                               int rs) {
  const long total = (long)k * rs * c;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int ko = (int)(i % k);
    const long t = i / k;
    const int tap = (int)(t % rs);
    const int ci = (int)(t / rs);
    wt[i] = (TO)w[((long)ko * c + ci) * rs + tap];   // bf16: RNE
  }
}

__global__ void nchw_to_nhwc_k(const float* __restrict__ x, float* __restrict__ y, int n, int c,
                               int h, int w, int cpad) {
  const long total = (long)n * h * w * cpad;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int ci = (int)(i % cpad);
    const long p = i / cpad;
    const long hw = p % ((long)h * w);
    const long nn = p / ((long)h * w);
    y[i] = ci < c ? x[(nn * c + ci) * h * w + hw] : 0.f;
  }
}

__global__ void nhwc_to_nchw_k(const float* __restrict__ x, float* __restrict__ y, int n, int c,
                               int cs, int h, int w) {
  const long total = (long)n * c * h * w;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long hw = i % ((long)h * w);
    const long t = i / ((long)h * w);
    const int ci = (int)(t % c);
    const long nn = t / c;
    y[i] = x[(nn * h * w + hw) * cs + ci];
  }
}

__global__ __launch_bounds__(NT) void crop_normalize_k(const uint8_t* __restrict__ fr,
                                                       const int32_t* __restrict__ off,
                                                       float4* __restrict__ out, int f, int hin,
                                                       int win, int seq, int crop, float m0,
                                                       float m1, float m2, float s0, float s1,
                                                       float s2) {
  const long total = (long)f * crop * crop;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int x = (int)(i % crop);
    const long t = i / crop;
    const int y = (int)(t % crop);
    const int fi = (int)(t / crop);
    const int clip = fi / seq;
    // clamp keeps a bad offset from reading outside the frame
    const int x1 = min(max(off[2 * clip], 0), win - crop);
    const int y1 = min(max(off[2 * clip + 1], 0), hin - crop);
    const uint8_t* px = fr + (((long)fi * hin + (y + y1)) * win + (x + x1)) * 3;
    // ToTensor: u8 -> float / 255; Normalize: (v - mean) / std
    const float r = (float)px[0] / 255.0f, g = (float)px[1] / 255.0f, b = (float)px[2] / 255.0f;
    out[i] = make_float4((r - m0) / s0, (g - m1) / s1, (b - m2) / s2, 0.f);
  }
}

}  // namespace

TMR_API int tmr_maxpool2d_fwd(const float* x, float* y, uint8_t* argmax, int n, int h, int w,
                              int c, int ho, int wo, hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0, "tmr_maxpool2d_fwd: channels %d must be a multiple of 4", c);
  const long total = (long)n * ho * wo * (c / 4);
  hipLaunchKernelGGL(maxpool_fwd_k<false>, dim3(ew_blocks(total)), dim3(NT), 0, stream, x, y,
                     (uchar4*)argmax, n, h, w, c / 4, ho, wo, nullptr, nullptr);
  TMR_CHECK_LAUNCH("maxpool_fwd");
  return 0;
}

TMR_API int tmr_maxpool2d_fwd_bn(const float* x, const float* scale, const float* shift, float* y,
                                 uint8_t* argmax, int n, int h, int w, int c, int ho, int wo,
                                 hipStream_t stream) {
  return tmr_maxpool2d_fwd_bn_x(x, scale, shift, y, argmax, n, h, w, c, ho, wo, 0, stream);
}

TMR_API int tmr_maxpool2d_fwd_bn_x(const float* x, const float* scale, const float* shift, void* y,
                                   uint8_t* argmax, int n, int h, int w, int c, int ho, int wo,
                                   int out_bf16, hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0, "tmr_maxpool2d_fwd_bn: channels %d must be a multiple of 4", c);
  TMR_CHECK_ARG(scale && shift, "tmr_maxpool2d_fwd_bn: null BatchNorm scale/shift");
  const long total = (long)n * ho * wo * (c / 4);
  const int c8 = c / 8;
  // 8 channels per thread (maxpool_fwd_bn8, as the bf16 step's stem; round 5), else 4-wide
  if (c % 8 == 0 && (c8 & (c8 - 1)) == 0 && (long)n * h * w * c8 < 0x7fffffffL &&
      (((uintptr_t)x | (uintptr_t)y) & 15) == 0 && ((uintptr_t)argmax & 7) == 0) {
    const int t8 = (int)(total / 2);
    const FastDiv dhwo = make_fastdiv((uint32_t)(ho * wo)), dwo = make_fastdiv((uint32_t)wo);
    if (out_bf16)
      hipLaunchKernelGGL((maxpool_fwd_bn8<float, __bf16>), dim3(ew_blocks(t8)), dim3(NT), 0, stream,
                         x, (__bf16*)y, (uint2*)argmax, t8, h, w, __builtin_ctz(c8), dhwo, dwo,
                         scale, shift);
    else
      hipLaunchKernelGGL((maxpool_fwd_bn8<float, float>), dim3(ew_blocks(t8)), dim3(NT), 0, stream,
                         x, (float*)y, (uint2*)argmax, t8, h, w, __builtin_ctz(c8), dhwo, dwo,
                         scale, shift);
  } else if (out_bf16)
    hipLaunchKernelGGL((maxpool_fwd_k<true, __bf16>), dim3(ew_blocks(total)), dim3(NT), 0, stream, x,
                       (__bf16*)y, (uchar4*)argmax, n, h, w, c / 4, ho, wo, scale, shift);
  else
    hipLaunchKernelGGL((maxpool_fwd_k<true>), dim3(ew_blocks(total)), dim3(NT), 0, stream, x,
                       (float*)y, (uchar4*)argmax, n, h, w, c / 4, ho, wo, scale, shift);
  TMR_CHECK_LAUNCH("maxpool_fwd_bn");
  return 0;
}

TMR_API int tmr_maxpool2d_fwd_bn_a16(const void* x, const float* scale, const float* shift, void* y,
                                     uint8_t* argmax, int n, int h, int w, int c, int ho, int wo,
                                     hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0, "tmr_maxpool2d_fwd_bn_a16: channels %d must be a multiple of 4", c);
  TMR_CHECK_ARG(scale && shift, "tmr_maxpool2d_fwd_bn_a16: null BatchNorm scale/shift");
  const long total = (long)n * ho * wo * (c / 4);
  const int c8 = c / 8;
  // 8 channels per thread (else the 4-wide form)
  if (c % 8 == 0 && (c8 & (c8 - 1)) == 0 &&
      (long)n * h * w * c8 < 0x7fffffffL &&
      (((uintptr_t)x | (uintptr_t)y) & 15) == 0 && ((uintptr_t)argmax & 7) == 0) {
    const int t8 = (int)(total / 2);
    hipLaunchKernelGGL((maxpool_fwd_bn8<__bf16, __bf16>), dim3(ew_blocks(t8)), dim3(NT), 0, stream,
                       (const __bf16*)x, (__bf16*)y, (uint2*)argmax, t8, h, w, __builtin_ctz(c8),
                       make_fastdiv((uint32_t)(ho * wo)), make_fastdiv((uint32_t)wo), scale, shift);
  } else {
    hipLaunchKernelGGL((maxpool_fwd_k<true, __bf16, __bf16>), dim3(ew_blocks(total)), dim3(NT), 0,
                       stream, (const __bf16*)x, (__bf16*)y, (uchar4*)argmax, n, h, w, c / 4, ho, wo,
                       scale, shift);
  }
  TMR_CHECK_LAUNCH("maxpool_fwd_bn_a16");
  return 0;
}

TMR_API int tmr_maxpool2d_bwd(const float* dy, const uint8_t* argmax, float* dx, int n, int h,
                              int w, int c, int ho, int wo, hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0, "tmr_maxpool2d_bwd: channels %d must be a multiple of 4", c);
  const long total = (long)n * h * w * (c / 4);
  hipLaunchKernelGGL(maxpool_bwd_k, dim3(ew_blocks(total)), dim3(NT), 0, stream, dy,
                     (const uchar4*)argmax, dx, n, h, w, c / 4, ho, wo);
  TMR_CHECK_LAUNCH("maxpool_bwd");
  return 0;
}

TMR_API int tmr_avgpool_fwd(const float* x, float* y, int n, int hw, int c, hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0, "tmr_avgpool_fwd: channels %d must be a multiple of 4", c);
  hipLaunchKernelGGL(avgpool_fwd_k<float>, dim3(ew_blocks((long)n * c / 4)), dim3(NT), 0, stream, x, y, n,
                     hw, c / 4);
  TMR_CHECK_LAUNCH("avgpool_fwd");
  return 0;
}

TMR_API int tmr_avgpool_fwd_a16(const void* x, float* y, int n, int hw, int c, hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0, "tmr_avgpool_fwd_a16: channels %d must be a multiple of 4", c);
  hipLaunchKernelGGL(avgpool_fwd_k<__bf16>, dim3(ew_blocks((long)n * c / 4)), dim3(NT), 0, stream,
                     (const __bf16*)x, y, n, hw, c / 4);
  TMR_CHECK_LAUNCH("avgpool_fwd_a16");
  return 0;
}

TMR_API int tmr_avgpool_bwd(const float* dy, float* dx, int n, int hw, int c, hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0, "tmr_avgpool_bwd: channels %d must be a multiple of 4", c);
  hipLaunchKernelGGL(avgpool_bwd_k, dim3(ew_blocks((long)n * hw * c / 4)), dim3(NT), 0, stream, dy,
                     dx, n, hw, c / 4);
  TMR_CHECK_LAUNCH("avgpool_bwd");
  return 0;
}

TMR_API int tmr_weight_oihw_to_krsc(const float* w, float* wk, int k, int c, int r, int s,
                                    int cpad, hipStream_t stream) {
  return tmr_weight_oihw_to_krsc_x(w, wk, k, c, r, s, cpad, 0, stream);
}

TMR_API int tmr_weight_oihw_to_krsc_x(const float* w, void* wk, int k, int c, int r, int s,
                                      int cpad, int out_bf16, hipStream_t stream) {
  TMR_CHECK_ARG(cpad >= c, "tmr_weight_oihw_to_krsc: cpad < c");
  if (out_bf16)
    hipLaunchKernelGGL(oihw_to_krsc_k<__bf16>, dim3(ew_blocks((long)k * r * s * cpad)), dim3(NT), 0,
                       stream, w, (__bf16*)wk, k, c, r * s, cpad);
  else
    hipLaunchKernelGGL(oihw_to_krsc_k<float>, dim3(ew_blocks((long)k * r * s * cpad)), dim3(NT), 0,
                       stream, w, (float*)wk, k, c, r * s, cpad);
  TMR_CHECK_LAUNCH("oihw_to_krsc");
  return 0;
}

TMR_API int tmr_weight_oihw_to_crsk_x(const float* w, void* wt, int k, int c, int r, int s,
                                      int out_bf16, hipStream_t stream) {
  TMR_CHECK_ARG(w && wt && k > 0 && c > 0 && r > 0 && s > 0, "tmr_weight_oihw_to_crsk_x: bad arguments");
  if (out_bf16)
    hipLaunchKernelGGL(oihw_to_crsk_k<__bf16>, dim3(ew_blocks((long)k * r * s * c)), dim3(NT), 0,
                       stream, w, (__bf16*)wt, k, c, r * s);
  else
    hipLaunchKernelGGL(oihw_to_crsk_k<float>, dim3(ew_blocks((long)k * r * s * c)), dim3(NT), 0,
                       stream, w, (float*)wt, k, c, r * s);
  TMR_CHECK_LAUNCH("oihw_to_crsk");
  return 0;
}

// Every weight layout of a train step in one launch (tmr_weight_layouts_multi): block b converts
// elements [ (b - block0) * NT * WL_EPB, ... ) of the entry whose block range holds it (binary
// search over block0); the element mapping and rounding of oihw_to_krsc_k / oihw_to_crsk_k.
constexpr int WL_EPB = 8;
__global__ __launch_bounds__(NT) void wlayout_multi_k(const tmr_wlayout* __restrict__ tab, int n) {
  int lo = 0, hi = n - 1;
  const long long b = blockIdx.x;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tab[mid].block0 <= b) lo = mid; else hi = mid - 1;
  }
  const tmr_wlayout e = tab[lo];
  const long long base = (b - e.block0) * (long long)NT * WL_EPB;
#pragma unroll
  for (int j = 0; j < WL_EPB; ++j) {
    const long long i = base + (long long)j * NT + threadIdx.x;
    if (i >= e.n) break;
    float v;
    if (e.kind == 0) {   // KRSC, channels zero-padded to cpad
      const int ci = (int)(i % e.cpad);
      const long long t = i / e.cpad;
      const int tap = (int)(t % e.rs);
      const int ko = (int)(t / e.rs);
      v = ci < e.c ? e.w[((long long)ko * e.c + ci) * e.rs + tap] : 0.f;
    } else {             // CRSK
      const int ko = (int)(i % e.k);
      const long long t = i / e.k;
      const int tap = (int)(t % e.rs);
      const int ci = (int)(t / e.rs);
      v = e.w[((long long)ko * e.c + ci) * e.rs + tap];
    }
    if (e.bf16) reinterpret_cast<__bf16*>(e.out)[i] = (__bf16)v;   // RNE
    else reinterpret_cast<float*>(e.out)[i] = v;
  }
}

TMR_API int tmr_weight_layouts_multi(const tmr_wlayout* tab_dev, int n, int total_blocks,
                                     hipStream_t stream) {
  TMR_CHECK_ARG(tab_dev && n > 0 && total_blocks > 0, "tmr_weight_layouts_multi: empty table");
  hipLaunchKernelGGL(wlayout_multi_k, dim3(total_blocks), dim3(NT), 0, stream, tab_dev, n);
  TMR_CHECK_LAUNCH("weight_layouts_multi");
  return 0;
}

TMR_API int tmr_weight_layouts_epb(void) { return NT * WL_EPB; }

// fp32 -> bf16 (RNE) copy: the bf16 conv operand of a tensor produced in fp32 (ResNeSt split-
// attention / pool outputs), 8 elements per thread
__global__ __launch_bounds__(NT) void cast_bf16_k(const float* __restrict__ x, __bf16* __restrict__ y,
                                                  long n8) {
  typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
    const float4 a = reinterpret_cast<const float4*>(x)[2 * i];
    const float4 b = reinterpret_cast<const float4*>(x)[2 * i + 1];
    const bf16x8_t v = {(__bf16)a.x, (__bf16)a.y, (__bf16)a.z, (__bf16)a.w,
                        (__bf16)b.x, (__bf16)b.y, (__bf16)b.z, (__bf16)b.w};
    reinterpret_cast<bf16x8_t*>(y)[i] = v;
  }
}

TMR_API int tmr_cast_f32_bf16(const float* x, void* y, long n, hipStream_t stream) {
  TMR_CHECK_ARG(x && y && n >= 0 && n % 8 == 0, "tmr_cast_f32_bf16: n %ld must be a multiple of 8", n);
  if (n == 0) return 0;
  hipLaunchKernelGGL(cast_bf16_k, dim3(ew_blocks(n / 8)), dim3(NT), 0, stream, x, (__bf16*)y, n / 8);
  TMR_CHECK_LAUNCH("cast_bf16");
  return 0;
}

// stem input of the bf16 step: fp32 NHWC4 pixel (3 colours + zero) -> 8 bf16 (RNE; channels 4-7
// zero), one 16-B read and one 16-B write per pixel
__global__ __launch_bounds__(NT) void nhwc4_bf16x8_k(const float4* __restrict__ x,
                                                     uint4* __restrict__ y, long npix) {
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < npix; i += (long)gridDim.x * NT) {
    const float4 a = x[i];
    const uint32_t w0 = (uint32_t)__builtin_bit_cast(unsigned short, (__bf16)a.x) |
                        ((uint32_t)__builtin_bit_cast(unsigned short, (__bf16)a.y) << 16);
    const uint32_t w1 = (uint32_t)__builtin_bit_cast(unsigned short, (__bf16)a.z) |
                        ((uint32_t)__builtin_bit_cast(unsigned short, (__bf16)a.w) << 16);
    y[i] = make_uint4(w0, w1, 0u, 0u);
  }
}

TMR_API int tmr_nhwc4_to_bf16x8(const float* x4, void* y8, long npix, hipStream_t stream) {
  TMR_CHECK_ARG(x4 && y8 && npix >= 0, "tmr_nhwc4_to_bf16x8: bad arguments");
  TMR_CHECK_ARG((((uintptr_t)x4 | (uintptr_t)y8) & 15) == 0, "tmr_nhwc4_to_bf16x8: 16-B aligned pixels");
  if (npix == 0) return 0;
  hipLaunchKernelGGL(nhwc4_bf16x8_k, dim3(ew_blocks(npix)), dim3(NT), 0, stream,
                     (const float4*)x4, (uint4*)y8, npix);
  TMR_CHECK_LAUNCH("nhwc4_bf16x8");
  return 0;
}

TMR_API int tmr_nchw_to_nhwc(const float* x, float* y, int n, int c, int h, int w, int cpad,
                             hipStream_t stream) {
  TMR_CHECK_ARG(cpad >= c, "tmr_nchw_to_nhwc: cpad < c");
  hipLaunchKernelGGL(nchw_to_nhwc_k, dim3(ew_blocks((long)n * h * w * cpad)), dim3(NT), 0, stream,
                     x, y, n, c, h, w, cpad);
  TMR_CHECK_LAUNCH("nchw_to_nhwc");
  return 0;
}

TMR_API int tmr_nhwc_to_nchw(const float* x, float* y, int n, int c, int cstore, int h, int w,
                             hipStream_t stream) {
  hipLaunchKernelGGL(nhwc_to_nchw_k, dim3(ew_blocks((long)n * h * w * c)), dim3(NT), 0, stream, x,
                     y, n, c, cstore, h, w);
  TMR_CHECK_LAUNCH("nhwc_to_nchw");
  return 0;
}

TMR_API int tmr_crop_normalize(const uint8_t* frames, const int32_t* offsets, float* out, int f,
                               int hin, int win, int seq_len, int crop, float m0, float m1,
                               float m2, float s0, float s1, float s2, hipStream_t stream) {
  TMR_CHECK_ARG(seq_len > 0 && f % seq_len == 0, "tmr_crop_normalize: frames %d not a multiple of seq_len %d", f, seq_len);
  TMR_CHECK_ARG(crop <= hin && crop <= win, "tmr_crop_normalize: crop larger than frame");
  hipLaunchKernelGGL(crop_normalize_k, dim3(ew_blocks((long)f * crop * crop)), dim3(NT), 0, stream,
                     frames, offsets, (float4*)out, f, hin, win, seq_len, crop, m0, m1, m2, s0, s1,
                     s2);
  TMR_CHECK_LAUNCH("crop_normalize");
  return 0;
}

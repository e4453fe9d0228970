// ResNeSt-50 building blocks that are not convolutions (NHWC fp32, HBM-bound):
//  * split-attention core of SplAtConv2d (radix 2, cardinality 1): the radix-summed global
//    average pool, the r-softmax + weighted sum of the splits, and their backward passes
//  * AvgPool2d (avd layer: 3x3/s2/p1, count_include_pad=True; avg_down: 2x2/s2,
//    ceil_mode=True, count_include_pad=False) forward/backward
// Reference: the `resnest50()` trunk built at code/Training TMRNet/
// train_non-local_mutiConv_resnest.py:210-220 (third-party `resnest` package,
// docker/Dockerfile:24; restated in oracle/tmrnet_ref.py).
#include "common.h"
#include "tmr.h"

namespace {
constexpr int NT = 256;
// per-channel reductions over frames: 64 columns x 16 row groups per block
constexpr int CC_COLS = 64, CC_RG = 16;

int blocks_for(long n) {
  long b = (n + NT - 1) / NT;
  if (b > 8192) b = 8192;
  return (int)(b > 0 ? b : 1);
}

// block shape of the per-frame reductions: `cols` float4 columns (power of two <= 64) x NT/cols rows
void red_shape(int c4, int& cols, int& chunks) {
  cols = 1;
  while (cols * 2 <= c4 && cols < 64) cols *= 2;
  chunks = (c4 + cols - 1) / cols;
}

// Per-frame channel reductions over hw pixels.  One block per (frame, chunk of up to 64
// float4 channel columns): thread (col, row) walks pixels row, row+R, ... with coalesced float4
// loads and double accumulators, then an LDS tree over the R rows.  The sums feed a BatchNorm
// over N frames whose inputs differ by ~1% of their magnitude, so fp32 sequential sums
// (error ~ hw*eps) would be amplified ~100x; double keeps them exact to fp32 rounding.
struct Red4 { double x, y, z, w; };

__device__ __forceinline__ void red_add(Red4& a, float4 v) { a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w; }

__device__ __forceinline__ void red_fma(Red4& a, float4 g, float4 v) {
  a.x = fma((double)g.x, (double)v.x, a.x); a.y = fma((double)g.y, (double)v.y, a.y);
  a.z = fma((double)g.z, (double)v.z, a.z); a.w = fma((double)g.w, (double)v.w, a.w);
}

// tree-reduce `nacc` Red4 accumulators per thread over the block's rows; result in rows 0
template <int NACC>
__device__ __forceinline__ void red_rows(Red4 (&acc)[NACC], Red4* lds, int col, int row, int cols, int rows) {
  for (int k = 0; k < NACC; ++k) lds[(k * rows + row) * cols + col] = acc[k];
  __syncthreads();
  for (int half = rows >> 1; half > 0; half >>= 1) {
    if (row < half)
      for (int k = 0; k < NACC; ++k) {
        Red4& d = lds[(k * rows + row) * cols + col];
        const Red4 o = lds[(k * rows + row + half) * cols + col];
        d.x += o.x; d.y += o.y; d.z += o.z; d.w += o.w;
      }
    __syncthreads();
  }
  for (int k = 0; k < NACC; ++k) acc[k] = lds[(k * rows) * cols + col];
}

// gap[n][c] = mean_hw (x[n,hw,c] + x[n,hw,C+c]),  x: [n][hw][2C]
__global__ __launch_bounds__(NT) void splat_gap_k(const float* __restrict__ x, float* __restrict__ gap,
                                                  int hw, int c4, int cols, int chunks) {
  __shared__ Red4 lds[NT];
  const int nn = blockIdx.x / chunks, cq = (blockIdx.x % chunks) * cols + threadIdx.x % cols;
  const int col = threadIdx.x % cols, row = threadIdx.x / cols, rows = NT / cols;
  const bool live = cq < c4;
  Red4 acc[1] = {{0.0, 0.0, 0.0, 0.0}};
  const float4* px = reinterpret_cast<const float4*>(x) + (long)nn * hw * 2 * c4;
  if (live)
    for (int p = row; p < hw; p += rows) {
      red_add(acc[0], px[(long)p * 2 * c4 + cq]);
      red_add(acc[0], px[(long)p * 2 * c4 + c4 + cq]);
    }
  red_rows<1>(acc, lds, col, row, cols, rows);
  if (row == 0 && live) {
    const double inv = 1.0 / (double)hw;
    reinterpret_cast<float4*>(gap)[(long)nn * c4 + cq] =
        make_float4((float)(acc[0].x * inv), (float)(acc[0].y * inv), (float)(acc[0].z * inv),
                    (float)(acc[0].w * inv));
  }
}

__device__ __forceinline__ void rsoft2(float z0, float z1, float& a0, float& a1) {
  const float m = fmaxf(z0, z1);
  const float e0 = expf(z0 - m), e1 = expf(z1 - m);
  const float inv = 1.0f / (e0 + e1);
  a0 = e0 * inv;
  a1 = e1 * inv;
}

// att[n][r*C+c] = softmax_r(z[n][r*C+c]);  out[n,hw,c] = sum_r att_r * x[n,hw,r*C+c]
__global__ __launch_bounds__(NT) void splat_combine_k(const float* __restrict__ x, const float* __restrict__ z,
                                                      float* __restrict__ att, float* __restrict__ out,
                                                      int n, int hw, int C) {
  const long total = (long)n * hw * C;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int c = (int)(i % C);
    const long p = i / C;           // pixel index n*hw + q
    const long nn = p / hw;
    float a0, a1;
    rsoft2(z[nn * 2 * C + c], z[nn * 2 * C + C + c], a0, a1);
    if (att && p % hw == 0) { att[nn * 2 * C + c] = a0; att[nn * 2 * C + C + c] = a1; }
    out[i] = a0 * x[p * 2 * C + c] + a1 * x[p * 2 * C + C + c];
  }
}

// dz[n][r*C+c] from da_r = sum_hw dout * x_r  (softmax backward over the radix pair)
__global__ __launch_bounds__(NT) void splat_bwd_reduce_k(const float* __restrict__ dout, const float* __restrict__ x,
                                                         const float* __restrict__ att, float* __restrict__ dz,
                                                         int hw, int c4, int cols, int chunks) {
  __shared__ Red4 lds[2 * NT];
  const int nn = blockIdx.x / chunks, cq = (blockIdx.x % chunks) * cols + threadIdx.x % cols;
  const int col = threadIdx.x % cols, row = threadIdx.x / cols, rows = NT / cols;
  const bool live = cq < c4;
  Red4 acc[2] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
  const float4* g = reinterpret_cast<const float4*>(dout) + (long)nn * hw * c4;
  const float4* px = reinterpret_cast<const float4*>(x) + (long)nn * hw * 2 * c4;
  if (live)
    for (int p = row; p < hw; p += rows) {
      const float4 gv = g[(long)p * c4 + cq];
      red_fma(acc[0], gv, px[(long)p * 2 * c4 + cq]);
      red_fma(acc[1], gv, px[(long)p * 2 * c4 + c4 + cq]);
    }
  red_rows<2>(acc, lds, col, row, cols, rows);
  if (row == 0 && live) {
    const int C = c4 * 4;
    const double d0[4] = {acc[0].x, acc[0].y, acc[0].z, acc[0].w};
    const double d1[4] = {acc[1].x, acc[1].y, acc[1].z, acc[1].w};
    for (int j = 0; j < 4; ++j) {
      const long i0 = (long)nn * 2 * C + cq * 4 + j;
      const double a0 = att[i0], a1 = att[i0 + C];
      const double dot = a0 * d0[j] + a1 * d1[j];
      dz[i0] = (float)(a0 * (d0[j] - dot));
      dz[i0 + C] = (float)(a1 * (d1[j] - dot));
    }
  }
}

// dx[n,hw,r*C+c] = att_r * dout[n,hw,c] + dgap[n][c] / hw
__global__ __launch_bounds__(NT) void splat_bwd_apply_k(const float* __restrict__ dout, const float* __restrict__ att,
                                                        const float* __restrict__ dgap, float* __restrict__ dx,
                                                        int n, int hw, int C) {
  const long total = (long)n * hw * 2 * C;
  const float inv = 1.0f / (float)hw;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int rc = (int)(i % (2 * C));
    const long p = i / (2 * C);
    const long nn = p / hw;
    const int c = rc % C;
    dx[i] = att[nn * 2 * C + rc] * dout[p * C + c] + dgap[nn * C + c] * inv;
  }
}

// general AvgPool2d on NHWC: divisor = k*k (count_include_pad) or #valid input cells
// IT: index type (uint32_t when the element groups fit 31 bits: 64-bit divisions cost
// ~100 instructions per element; tmr_avgpool2d_* pick it)
template <typename IT>
__global__ __launch_bounds__(NT) void avgpool2d_fwd_k(const float* __restrict__ x, float* __restrict__ y,
                                                      int n, int h, int w, int c4, int ho, int wo,
                                                      int k, int s, int p, int incl) {
  const IT total = (IT) (long)n * ho * wo * c4;
  for (IT i = (IT)blockIdx.x * NT + threadIdx.x; i < total; i += (IT)gridDim.x * NT) {
    const int cq = (int)(i % (IT)c4);
    IT t = i / (IT)c4;
    const int ox = (int)(t % (IT)wo);
    t /= (IT)wo;
    const int oy = (int)(t % (IT)ho);
    const int nn = (int)(t / (IT)ho);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int cnt = 0;
    for (int dy = 0; dy < k; ++dy) {
      const int iy = oy * s - p + dy;
      if (iy < 0 || iy >= h) continue;
      for (int dx = 0; dx < k; ++dx) {
        const int ix = ox * s - p + dx;
        if (ix < 0 || ix >= w) continue;
        const float4 v = reinterpret_cast<const float4*>(x)[(((long)nn * h + iy) * w + ix) * c4 + cq];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        ++cnt;
      }
    }
    const float inv = 1.0f / (float)(incl ? k * k : (cnt > 0 ? cnt : 1));
    acc.x *= inv; acc.y *= inv; acc.z *= inv; acc.w *= inv;
    reinterpret_cast<float4*>(y)[i] = acc;
  }
}

// IT: index type (uint32_t when the element groups fit 31 bits: 64-bit divisions cost
// ~100 instructions per element; tmr_avgpool2d_* pick it)
template <typename IT>
__global__ __launch_bounds__(NT) void avgpool2d_bwd_k(const float* __restrict__ dy, float* __restrict__ dx,
                                                      int n, int h, int w, int c4, int ho, int wo,
                                                      int k, int s, int p, int incl) {
  const IT total = (IT) (long)n * h * w * c4;
  for (IT i = (IT)blockIdx.x * NT + threadIdx.x; i < total; i += (IT)gridDim.x * NT) {
    const int cq = (int)(i % (IT)c4);
    IT t = i / (IT)c4;
    const int ix = (int)(t % (IT)w);
    t /= (IT)w;
    const int iy = (int)(t % (IT)h);
    const int nn = (int)(t / (IT)h);
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    // outputs oy with oy*s - p <= iy <= oy*s - p + k - 1
    const int oy0 = max(0, (iy + p - k + s) / s), oy1 = min(ho - 1, (iy + p) / s);
    const int ox0 = max(0, (ix + p - k + s) / s), ox1 = min(wo - 1, (ix + p) / s);
    for (int oy = oy0; oy <= oy1; ++oy) {
      if (iy < oy * s - p || iy > oy * s - p + k - 1) continue;
      for (int ox = ox0; ox <= ox1; ++ox) {
        if (ix < ox * s - p || ix > ox * s - p + k - 1) continue;
        int cnt = k * k;
        if (!incl) {
          const int y0 = max(0, oy * s - p), y1 = min(h, oy * s - p + k);
          const int x0 = max(0, ox * s - p), x1 = min(w, ox * s - p + k);
          cnt = (y1 - y0) * (x1 - x0);
        }
        const float inv = 1.0f / (float)cnt;
        const float4 d = reinterpret_cast<const float4*>(dy)[(((long)nn * ho + oy) * wo + ox) * c4 + cq];
        g.x += d.x * inv; g.y += d.y * inv; g.z += d.z * inv; g.w += d.w * inv;
      }
    }
    reinterpret_cast<float4*>(dx)[i] = g;
  }
}

// The same with the pixel / channel indices by magic-number division (the element-group count
// fits 32 bits, checked on the host): the generic form's three 32-bit divisions per 4 elements
// made it instruction-bound (~2 TB/s).  Same sums in the same order.  KK / SS / PP: ResNeSt's two
// pools as compile-time windows (the avd 3x3/2 pad 1 and the avg_down 2x2/2), so the window
// bounds divide by a constant; 0: the runtime k / s / p.
template <int KK, int SS, int PP>
__global__ __launch_bounds__(NT) void avgpool2d_bwd_fd_k(const float* __restrict__ dy,
                                                         float* __restrict__ dx, uint32_t total,
                                                         FastDiv dc4, FastDiv dw, FastDiv dh,
                                                         int ho, int wo, int k_, int s_, int p_,
                                                         int incl) {
  const int k = KK ? KK : k_, s = KK ? SS : s_, p = KK ? PP : p_;
  const uint32_t c4 = dc4.d, w = dw.d, h = dh.d;
  for (uint32_t i = blockIdx.x * NT + threadIdx.x; i < total; i += gridDim.x * NT) {
    const uint32_t t0 = fdiv(i, dc4);
    const int cq = (int)(i - t0 * c4);
    const uint32_t t1 = fdiv(t0, dw);
    const int ix = (int)(t0 - t1 * w);
    const uint32_t nn = fdiv(t1, dh);
    const int iy = (int)(t1 - nn * h);
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    const int oy0 = max(0, (iy + p - k + s) / s), oy1 = min(ho - 1, (iy + p) / s);
    const int ox0 = max(0, (ix + p - k + s) / s), ox1 = min(wo - 1, (ix + p) / s);
    for (int oy = oy0; oy <= oy1; ++oy) {
      if (iy < oy * s - p || iy > oy * s - p + k - 1) continue;
      for (int ox = ox0; ox <= ox1; ++ox) {
        if (ix < ox * s - p || ix > ox * s - p + k - 1) continue;
        int cnt = k * k;
        if (!incl) {
          const int y0 = max(0, oy * s - p), y1 = min((int)h, oy * s - p + k);
          const int x0 = max(0, ox * s - p), x1 = min((int)w, ox * s - p + k);
          cnt = (y1 - y0) * (x1 - x0);
        }
        const float inv = 1.0f / (float)cnt;
        const float4 d = reinterpret_cast<const float4*>(dy)[(((long)nn * ho + oy) * wo + ox) * c4 + cq];
        g.x += d.x * inv; g.y += d.y * inv; g.z += d.z * inv; g.w += d.w * inv;
      }
    }
    reinterpret_cast<float4*>(dx)[i] = g;
  }
}

// ---------------------------------------------------------------------------------------------
// Split attention with bn0 + ReLU applied on load (the whole-trunk ResNeSt node, resnest.py).
// The grouped conv's pre-BN output y2 [n][hw][2C] (bf16 under the bf16-activation contract, else
// fp32) is the only stored tensor of the SplAtConv2d: x_r = relu(y2_r * scale + shift) -- rounded
// to bf16 under act16, the value a stored bf16 activation would hold -- is recomputed wherever the
// split attention reads it (GAP, weighted sum, both backward passes), so the post-BN tensor x is
// never written and its backward (dx of the weighted sum, the ReLU mask, the BatchNorm backward of
// bn0) runs as one reduction pass and one apply pass.
template <typename T> struct Act;
template <> struct Act<float> {
  static __device__ __forceinline__ float4 ld(const float* p, long i4) {
    return reinterpret_cast<const float4*>(p)[i4];
  }
  static __device__ __forceinline__ void st(float* p, long i4, float4 v) {
    reinterpret_cast<float4*>(p)[i4] = v;
  }
  static __device__ __forceinline__ float rnd(float v) { return v; }
};
template <> struct Act<__bf16> {
  static __device__ __forceinline__ float4 ld(const __bf16* p, long i4) {
    const uint2 w = reinterpret_cast<const uint2*>(p)[i4];
    return make_float4(__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                       __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u));
  }
  static __device__ __forceinline__ void st(__bf16* p, long i4, float4 v) {
    typedef __bf16 b2 __attribute__((ext_vector_type(2)));
    const b2 lo = {(__bf16)v.x, (__bf16)v.y}, hi = {(__bf16)v.z, (__bf16)v.w};
    reinterpret_cast<uint2*>(p)[i4] = make_uint2(__builtin_bit_cast(uint32_t, lo),
                                                 __builtin_bit_cast(uint32_t, hi));
  }
  static __device__ __forceinline__ float rnd(float v) { return (float)(__bf16)v; }
};

// x = rnd(relu(y * sc + sh)) per element of a channel quad
template <typename T>
__device__ __forceinline__ float4 bnrelu4(float4 y, float4 sc, float4 sh) {
  return make_float4(Act<T>::rnd(fmaxf(fmaf(y.x, sc.x, sh.x), 0.f)), Act<T>::rnd(fmaxf(fmaf(y.y, sc.y, sh.y), 0.f)),
                     Act<T>::rnd(fmaxf(fmaf(y.z, sc.z, sh.z), 0.f)), Act<T>::rnd(fmaxf(fmaf(y.w, sc.w, sh.w), 0.f)));
}
__device__ __forceinline__ float4 ld4f(const float* p, long i4) { return reinterpret_cast<const float4*>(p)[i4]; }

// gap[n][c] = mean_hw (x0[n,hw,c] + x1[n,hw,c]) with x_r recomputed from y2 (splat_gap_k's block shape)
// (BT threads per block: the bf16 step launches 1024 -- one block per frame and channel chunk is
// too few blocks at 256 threads to keep enough loads in flight)
template <typename T, int BT = NT>
__global__ __launch_bounds__(BT) void splat_gap_bn_k(const T* __restrict__ y, const float* __restrict__ sc,
                                                     const float* __restrict__ sh, float* __restrict__ gap,
                                                     int hw, int c4, int cols, int chunks) {
  __shared__ Red4 lds[BT];
  const int nn = blockIdx.x / chunks, cq = (blockIdx.x % chunks) * cols + threadIdx.x % cols;
  const int col = threadIdx.x % cols, row = threadIdx.x / cols, rows = BT / cols;
  const bool live = cq < c4;
  Red4 acc[1] = {{0.0, 0.0, 0.0, 0.0}};
  if (live) {
    const float4 s0 = ld4f(sc, cq), s1 = ld4f(sc, c4 + cq), h0 = ld4f(sh, cq), h1 = ld4f(sh, c4 + cq);
    const long base = (long)nn * hw * 2 * c4;
    for (int p = row; p < hw; p += rows) {
      const long i = base + (long)p * 2 * c4;
      red_add(acc[0], bnrelu4<T>(Act<T>::ld(y, i + cq), s0, h0));
      red_add(acc[0], bnrelu4<T>(Act<T>::ld(y, i + c4 + cq), s1, h1));
    }
  }
  red_rows<1>(acc, lds, col, row, cols, rows);
  if (row == 0 && live) {
    const double inv = 1.0 / (double)hw;
    reinterpret_cast<float4*>(gap)[(long)nn * c4 + cq] =
        make_float4((float)(acc[0].x * inv), (float)(acc[0].y * inv), (float)(acc[0].z * inv),
                    (float)(acc[0].w * inv));
  }
}

// att[n][r*C+c] = softmax over the radix pair of the fc2 logits zl
__global__ __launch_bounds__(NT) void splat_att_k(const float* __restrict__ zl, float* __restrict__ att,
                                                  int n, int C) {
  const long total = (long)n * C;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const long nn = i / C;
    const int c = (int)(i - nn * C);
    float a0, a1;
    rsoft2(zl[nn * 2 * C + c], zl[nn * 2 * C + C + c], a0, a1);
    att[nn * 2 * C + c] = a0;
    att[nn * 2 * C + C + c] = a1;
  }
}

// out[n,hw,c] = rnd(att0 * x0 + att1 * x1).  32-bit index math with magic-number division (the
// host checks the element count; 64-bit divisions cost ~100 instructions per element)
template <typename T>
__global__ __launch_bounds__(NT) void splat_combine_bn_k(const T* __restrict__ y, const float* __restrict__ sc,
                                                         const float* __restrict__ sh, const float* __restrict__ att,
                                                         T* __restrict__ out, uint32_t total, FastDiv dc4,
                                                         FastDiv dhw) {
  const uint32_t c4 = dc4.d;
  for (uint32_t i = blockIdx.x * NT + threadIdx.x; i < total; i += gridDim.x * NT) {
    const uint32_t p = fdiv(i, dc4);
    const uint32_t cq = i - p * c4;
    const uint32_t nn = fdiv(p, dhw);
    const float4 x0 = bnrelu4<T>(Act<T>::ld(y, (long)p * 2 * c4 + cq), ld4f(sc, cq), ld4f(sh, cq));
    const float4 x1 = bnrelu4<T>(Act<T>::ld(y, (long)p * 2 * c4 + c4 + cq), ld4f(sc, c4 + cq), ld4f(sh, c4 + cq));
    const float4 a0 = ld4f(att, (long)nn * 2 * c4 + cq), a1 = ld4f(att, (long)nn * 2 * c4 + c4 + cq);
    Act<T>::st(out, i, make_float4(fmaf(a1.x, x1.x, a0.x * x0.x), fmaf(a1.y, x1.y, a0.y * x0.y),
                                   fmaf(a1.z, x1.z, a0.z * x0.z), fmaf(a1.w, x1.w, a0.w * x0.w)));
  }
}

// The bf16 form with 8 channels per thread (splat_bwd_apply_bn8_k's layout: the octet fixed per
// thread, both radix halves' BN coefficients in registers, att once per frame, 16-B accesses); the
// same arithmetic per element as splat_combine_bn_k.
__global__ __launch_bounds__(NT) void splat_combine_bn8_k(const __bf16* __restrict__ y,
                                                          const float* __restrict__ sc,
                                                          const float* __restrict__ sh,
                                                          const float* __restrict__ att,
                                                          __bf16* __restrict__ out, uint32_t npix,
                                                          int C, FastDiv dhw) {
  const int c8 = C / 8;
  const uint32_t t = blockIdx.x * NT + threadIdx.x;
  const int q = (int)(t % (uint32_t)c8);
  const uint32_t pstride = gridDim.x * NT / c8;
  float s[2][8], h[2][8];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s[r][e] = sc[r * C + 8 * q + e];
      h[r][e] = sh[r * C + 8 * q + e];
    }
  float a[2][8];
  uint32_t cur = 0xffffffffu;
  for (uint32_t p = t / c8; p < npix; p += pstride) {
    const uint32_t nn = fdiv(p, dhw);
    if (nn != cur) {
      cur = nn;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        a[0][e] = att[(long)nn * 2 * C + 8 * q + e];
        a[1][e] = att[(long)nn * 2 * C + C + 8 * q + e];
      }
    }
    const uint4 w0 = *reinterpret_cast<const uint4*>(y + (long)p * 2 * C + 8 * q);
    const uint4 w1 = *reinterpret_cast<const uint4*>(y + (long)p * 2 * C + C + 8 * q);
    const uint32_t u0[4] = {w0.x, w0.y, w0.z, w0.w}, u1[4] = {w1.x, w1.y, w1.z, w1.w};
    uint32_t o[4];
#pragma unroll
    for (int e2 = 0; e2 < 4; ++e2) {
      float v[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int e = 2 * e2 + b;
        const float y0 = b ? __uint_as_float(u0[e2] & 0xffff0000u) : __uint_as_float(u0[e2] << 16);
        const float y1 = b ? __uint_as_float(u1[e2] & 0xffff0000u) : __uint_as_float(u1[e2] << 16);
        const float x0 = Act<__bf16>::rnd(fmaxf(fmaf(y0, s[0][e], h[0][e]), 0.f));
        const float x1 = Act<__bf16>::rnd(fmaxf(fmaf(y1, s[1][e], h[1][e]), 0.f));
        v[b] = fmaf(a[1][e], x1, a[0][e] * x0);
      }
      typedef __bf16 b2 __attribute__((ext_vector_type(2)));
      const b2 pr = {(__bf16)v[0], (__bf16)v[1]};
      o[e2] = __builtin_bit_cast(uint32_t, pr);
    }
    *reinterpret_cast<uint4*>(out + (long)p * C + 8 * q) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// Backward reduction pass, per (frame, channel): for each radix r (x_r recomputed, m_r its ReLU
// mask, d_r = y_r - mean_r)
//   P_r = sum dout*x_r        -> dzl = softmax backward over the radix pair (weighted-sum -> att)
//   S1 = sum m_r*dout, S2 = sum m_r, S3 = sum m_r*dout*d_r, S4 = sum m_r*d_r
// The bn0 input gradient is g_r = m_r*(att_r*dout + dgap/hw) with dgap known only after the fc
// backward; its BatchNorm sums over the frame are att_r*S1 + dgap/hw*S2 and att_r*S3 + dgap/hw*S4,
// so one pass over (dout, y2) serves the attention and the BatchNorm backward.
// sums: float [4][n][2C].
template <typename T, int BT = NT>
__global__ __launch_bounds__(BT) void splat_bwd_reduce_bn_k(
    const float* __restrict__ dout, const T* __restrict__ y, const float* __restrict__ sc,
    const float* __restrict__ sh, const float* __restrict__ mean, const float* __restrict__ att,
    float* __restrict__ dzl, float* __restrict__ sums, int n, int hw, int c4, int cols, int chunks) {
  __shared__ Red4 lds[BT];
  const int nn = blockIdx.x / chunks, cq = (blockIdx.x % chunks) * cols + threadIdx.x % cols;
  const int col = threadIdx.x % cols, row = threadIdx.x / cols, rows = BT / cols;
  const bool live = cq < c4;
  Red4 acc[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) acc[k] = {0.0, 0.0, 0.0, 0.0};
  if (live) {
    float4 s[2], h[2], mu[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      s[r] = ld4f(sc, r * c4 + cq); h[r] = ld4f(sh, r * c4 + cq); mu[r] = ld4f(mean, r * c4 + cq);
    }
    const long base = (long)nn * hw;
    for (int p = row; p < hw; p += rows) {
      const float4 g = ld4f(dout, (base + p) * c4 + cq);
      const float gv[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const float4 yv = Act<T>::ld(y, (base + p) * 2 * c4 + r * c4 + cq);
        const float ya[4] = {yv.x, yv.y, yv.z, yv.w};
        const float sa[4] = {s[r].x, s[r].y, s[r].z, s[r].w}, ha[4] = {h[r].x, h[r].y, h[r].z, h[r].w};
        const float ma[4] = {mu[r].x, mu[r].y, mu[r].z, mu[r].w};
        double* a = &acc[5 * r].x;   // Red4 = 4 doubles: acc[5r + k].(x..w) = a[4k + e]
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = fmaf(ya[e], sa[e], ha[e]);
          const bool m = v > 0.f;
          const float x = Act<T>::rnd(fmaxf(v, 0.f));
          const double d = m ? (double)(ya[e] - ma[e]) : 0.0;
          const double gm = m ? (double)gv[e] : 0.0;
          a[e] = fma((double)gv[e], (double)x, a[e]);   // P
          a[4 + e] += gm;                                // S1
          a[8 + e] += m ? 1.0 : 0.0;                     // S2
          a[12 + e] = fma(gm, (double)(ya[e] - ma[e]), a[12 + e]);   // S3
          a[16 + e] += d;                                // S4
        }
      }
    }
  }
  // tree-reduce the ten accumulators over the block's rows, one at a time through one LDS buffer
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    Red4 one[1] = {acc[k]};
    red_rows<1>(one, lds, col, row, cols, rows);
    acc[k] = one[0];
    __syncthreads();
  }
  if (row == 0 && live) {
    const int C = 4 * c4;
    const long plane = (long)n * 2 * C;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = 4 * cq + e;
      const long i0 = (long)nn * 2 * C + c;
      const double p0 = (&acc[0].x)[e], p1 = (&acc[5].x)[e];
      const double a0 = att[i0], a1 = att[i0 + C];
      const double dot = a0 * p0 + a1 * p1;
      dzl[i0] = (float)(a0 * (p0 - dot));
      dzl[i0 + C] = (float)(a1 * (p1 - dot));
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          sums[k * plane + i0 + r * C] = (float)(&acc[5 * r + 1 + k].x)[e];
    }
  }
}

// per channel j of the 2C bn0 channels (r = j / C, c = j % C), frames summed in order:
//   sg = sum_n att*S1 + dgap/hw*S2 = sum g,  sgx = sum_n att*S3 + dgap/hw*S4 = sum g*(y - mean)
// -> dbeta = sg, dgamma = sgx*invstd, coef[3][2C] = (gamma*invstd, sg/N, invstd^2*sgx/N):
//   dy = coef0 * (g - coef1 - (y - mean) * coef2)   (nn.BatchNorm2d's batch-statistics backward)
__global__ __launch_bounds__(CC_COLS * CC_RG) void splat_bn0_coefs_k(
    const float* __restrict__ att, const float* __restrict__ dgap, const float* __restrict__ sums,
    const float* __restrict__ mean, const float* __restrict__ invstd, const float* __restrict__ gamma,
    float* __restrict__ coef, float* __restrict__ dgamma, float* __restrict__ dbeta, int n, int hw,
    int C) {
  __shared__ double part[2][CC_RG][CC_COLS];
  const int cl = threadIdx.x % CC_COLS, rg = threadIdx.x / CC_COLS;
  const int j = blockIdx.x * CC_COLS + cl;
  const long plane = (long)n * 2 * C;
  const double ihw = 1.0 / (double)hw;
  double sg = 0.0, sgx = 0.0;
  if (j < 2 * C) {
    const int c = j % C;
    for (int nn = rg; nn < n; nn += CC_RG) {
      const long i = (long)nn * 2 * C + j;
      const double a = att[i], dg = (double)dgap[(long)nn * C + c] * ihw;
      sg += a * sums[i] + dg * sums[plane + i];                    // att*S1 + dgap/hw*S2
      sgx += a * sums[2 * plane + i] + dg * sums[3 * plane + i];   // att*S3 + dgap/hw*S4
    }
  }
  part[0][rg][cl] = sg;
  part[1][rg][cl] = sgx;
  __syncthreads();
  if (rg != 0 || j >= 2 * C) return;
  sg = 0.0; sgx = 0.0;
  for (int q = 0; q < CC_RG; ++q) { sg += part[0][q][cl]; sgx += part[1][q][cl]; }
  (void)mean;
  const double inv = invstd[j], N = (double)n * hw;
  dbeta[j] = (float)sg;
  dgamma[j] = (float)(sgx * inv);
  coef[j] = (float)((double)gamma[j] * inv);
  coef[2 * C + j] = (float)(sg / N);
  coef[4 * C + j] = (float)(inv * inv * sgx / N);
}

// dy[n,hw,j] = coef0 * (g - coef1 - (y - mean) * coef2), g = m*(att*dout + dgap/hw)
template <typename T>
__global__ __launch_bounds__(NT) void splat_bwd_apply_bn_k(
    const float* __restrict__ dout, const T* __restrict__ y, const float* __restrict__ sc,
    const float* __restrict__ sh, const float* __restrict__ mean, const float* __restrict__ att,
    const float* __restrict__ dgap, const float* __restrict__ coef, T* __restrict__ dy,
    uint32_t total, FastDiv dj4, FastDiv dhw) {
  const uint32_t j4 = dj4.d, c4 = j4 / 2;
  const float ihw = 1.0f / (float)dhw.d;
  for (uint32_t i = blockIdx.x * NT + threadIdx.x; i < total; i += gridDim.x * NT) {
    const uint32_t p = fdiv(i, dj4);
    const uint32_t jq = i - p * j4;
    const uint32_t cq = jq < c4 ? jq : jq - c4;
    const uint32_t nn = fdiv(p, dhw);
    const float4 yv = Act<T>::ld(y, i);
    const float4 g0 = ld4f(dout, (long)p * c4 + cq);
    const float4 a = ld4f(att, (long)nn * j4 + jq);
    const float4 dg = ld4f(dgap, (long)nn * c4 + cq);
    const float4 s = ld4f(sc, jq), h = ld4f(sh, jq), mu = ld4f(mean, jq);
    const float4 k0 = ld4f(coef, jq), k1 = ld4f(coef, j4 + jq), k2 = ld4f(coef, 2 * j4 + jq);
    auto one = [&](float yv_, float s_, float h_, float mu_, float g_, float a_, float dg_, float k0_,
                   float k1_, float k2_) {
      const float gg = fmaf(yv_, s_, h_) > 0.f ? fmaf(a_, g_, dg_ * ihw) : 0.f;
      return k0_ * (gg - k1_ - (yv_ - mu_) * k2_);
    };
    Act<T>::st(dy, i, make_float4(one(yv.x, s.x, h.x, mu.x, g0.x, a.x, dg.x, k0.x, k1.x, k2.x),
                                  one(yv.y, s.y, h.y, mu.y, g0.y, a.y, dg.y, k0.y, k1.y, k2.y),
                                  one(yv.z, s.z, h.z, mu.z, g0.z, a.z, dg.z, k0.z, k1.z, k2.z),
                                  one(yv.w, s.w, h.w, mu.w, g0.w, a.w, dg.w, k0.w, k1.w, k2.w)));
  }
}

// The bf16 form with 8 channels of both radix halves per thread (C a multiple of 8, 256 / (C/8)
// whole): the channel octet is fixed per thread (the grid is a multiple of C/8 threads), so the
// per-channel coefficients stay in registers, dout is read once for both halves (it was read per
// half), att / dgap once per frame, every access 16 B.  The same arithmetic per element as
// splat_bwd_apply_bn_k (dgap/hw rounded once per channel, as there per element).
__global__ __launch_bounds__(NT) void splat_bwd_apply_bn8_k(
    const float* __restrict__ dout, const __bf16* __restrict__ y, const float* __restrict__ sc,
    const float* __restrict__ sh, const float* __restrict__ mean, const float* __restrict__ att,
    const float* __restrict__ dgap, const float* __restrict__ coef, __bf16* __restrict__ dy,
    uint32_t npix, int C, FastDiv dhw) {
  const int c8 = C / 8;
  const uint32_t t = blockIdx.x * NT + threadIdx.x;
  const int q = (int)(t % (uint32_t)c8);
  const uint32_t pstride = gridDim.x * NT / c8;
  const float ihw = 1.0f / (float)dhw.d;
  float s[2][8], h[2][8], mu[2][8], k0[2][8], k1[2][8], k2[2][8];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int j = r * C + 8 * q + e;
      s[r][e] = sc[j]; h[r][e] = sh[j]; mu[r][e] = mean[j];
      k0[r][e] = coef[j]; k1[r][e] = coef[2 * C + j]; k2[r][e] = coef[4 * C + j];
    }
  float a[2][8], dg[8];
  uint32_t cur = 0xffffffffu;
  for (uint32_t p = t / c8; p < npix; p += pstride) {
    const uint32_t nn = fdiv(p, dhw);
    if (nn != cur) {
      cur = nn;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        a[0][e] = att[(long)nn * 2 * C + 8 * q + e];
        a[1][e] = att[(long)nn * 2 * C + C + 8 * q + e];
        dg[e] = dgap[(long)nn * C + 8 * q + e] * ihw;
      }
    }
    const float4* gp = reinterpret_cast<const float4*>(dout + (long)p * C + 8 * q);
    const float4 g0 = gp[0], g1 = gp[1];
    const float gv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const long off = (long)p * 2 * C + r * C + 8 * q;   // elements
      const uint4 yw = *reinterpret_cast<const uint4*>(y + off);
      const uint32_t yu[4] = {yw.x, yw.y, yw.z, yw.w};
      uint32_t o[4];
#pragma unroll
      for (int e2 = 0; e2 < 4; ++e2) {
        float v[2];
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int e = 2 * e2 + b;
          const float yv = b ? __uint_as_float(yu[e2] & 0xffff0000u) : __uint_as_float(yu[e2] << 16);
          const float gg = fmaf(yv, s[r][e], h[r][e]) > 0.f ? fmaf(a[r][e], gv[e], dg[e]) : 0.f;
          v[b] = k0[r][e] * (gg - k1[r][e] - (yv - mu[r][e]) * k2[r][e]);
        }
        typedef __bf16 b2 __attribute__((ext_vector_type(2)));
        const b2 pr = {(__bf16)v[0], (__bf16)v[1]};
        o[e2] = __builtin_bit_cast(uint32_t, pr);
      }
      *reinterpret_cast<uint4*>(dy + off) = make_uint4(o[0], o[1], o[2], o[3]);
    }
  }
}

// AvgPool2d of bf16 activations (avd layer, avg_down): fp32 sums of the bf16 inputs, output rounded
// IT: index type (uint32_t when the element groups fit 31 bits: 64-bit divisions cost
// ~100 instructions per element; tmr_avgpool2d_* pick it)
template <typename IT>
__global__ __launch_bounds__(NT) void avgpool2d_fwd_a16_k(const __bf16* __restrict__ x, __bf16* __restrict__ y,
                                                          int n, int h, int w, int c4, int ho, int wo,
                                                          int k, int s, int p, int incl) {
  const IT total = (IT) (long)n * ho * wo * c4;
  for (IT i = (IT)blockIdx.x * NT + threadIdx.x; i < total; i += (IT)gridDim.x * NT) {
    const int cq = (int)(i % (IT)c4);
    IT t = i / (IT)c4;
    const int ox = (int)(t % (IT)wo);
    t /= (IT)wo;
    const int oy = (int)(t % (IT)ho);
    const int nn = (int)(t / (IT)ho);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int cnt = 0;
    for (int dy = 0; dy < k; ++dy) {
      const int iy = oy * s - p + dy;
      if (iy < 0 || iy >= h) continue;
      for (int dx = 0; dx < k; ++dx) {
        const int ix = ox * s - p + dx;
        if (ix < 0 || ix >= w) continue;
        const float4 v = Act<__bf16>::ld(x, (((long)nn * h + iy) * w + ix) * c4 + cq);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        ++cnt;
      }
    }
    const float inv = 1.0f / (float)(incl ? k * k : (cnt > 0 ? cnt : 1));
    acc.x *= inv; acc.y *= inv; acc.z *= inv; acc.w *= inv;
    Act<__bf16>::st(y, i, acc);
  }
}

// The same with magic-number index division (the output element-group count fits 32 bits) for
// ResNeSt's two windows at compile time (the avd 3x3/2 pad 1, the avg_down 2x2/2): same sums,
// same order
template <int KK, int SS, int PP>
__global__ __launch_bounds__(NT) void avgpool2d_fwd_a16_fd_k(const __bf16* __restrict__ x,
                                                             __bf16* __restrict__ y, uint32_t total,
                                                             FastDiv dc4, FastDiv dwo, FastDiv dho,
                                                             int h, int w, int incl) {
  static_assert(KK > 0 && SS > 0, "compile-time window");
  constexpr int k = KK, s = SS, p = PP;
  const uint32_t c4 = dc4.d, wo = dwo.d, ho = dho.d;
  for (uint32_t i = blockIdx.x * NT + threadIdx.x; i < total; i += gridDim.x * NT) {
    const uint32_t t0 = fdiv(i, dc4);
    const int cq = (int)(i - t0 * c4);
    const uint32_t t1 = fdiv(t0, dwo);
    const int ox = (int)(t0 - t1 * wo);
    const uint32_t nn = fdiv(t1, dho);
    const int oy = (int)(t1 - nn * ho);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int cnt = 0;
#pragma unroll
    for (int dy = 0; dy < k; ++dy) {
      const int iy = oy * s - p + dy;
      if (iy < 0 || iy >= h) continue;
#pragma unroll
      for (int dx = 0; dx < k; ++dx) {
        const int ix = ox * s - p + dx;
        if (ix < 0 || ix >= w) continue;
        const float4 v = Act<__bf16>::ld(x, (((long)nn * h + iy) * w + ix) * c4 + cq);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        ++cnt;
      }
    }
    const float inv = 1.0f / (float)(incl ? k * k : (cnt > 0 ? cnt : 1));
    acc.x *= inv; acc.y *= inv; acc.z *= inv; acc.w *= inv;
    Act<__bf16>::st(y, i, acc);
  }
}

// Column means over the frames: block = 64 columns x 16 row groups (1024 threads), each thread
// sums its rows in double, the 16 partial sums are added in a fixed order (deterministic).
__global__ __launch_bounds__(CC_COLS * CC_RG) void center_cols_k(const float* __restrict__ x, int rows, int cols,
                                                                 float* __restrict__ center, float* __restrict__ xc) {
  __shared__ double part[CC_RG][CC_COLS];
  __shared__ float mean_s[CC_COLS];
  const int cl = threadIdx.x % CC_COLS, rg = threadIdx.x / CC_COLS;
  const int j = blockIdx.x * CC_COLS + cl;
  double s = 0.0;
  if (j < cols)
    for (int i = rg; i < rows; i += CC_RG) s += x[(long)i * cols + j];
  part[rg][cl] = s;
  __syncthreads();
  if (rg == 0) {
    double t = 0.0;
    for (int q = 0; q < CC_RG; ++q) t += part[q][cl];
    const float m = (float)(t / (double)rows);
    mean_s[cl] = m;
    if (j < cols) center[j] = m;
  }
  __syncthreads();
  if (j < cols) {
    const float m = mean_s[cl];
    for (int i = rg; i < rows; i += CC_RG) xc[(long)i * cols + j] = x[(long)i * cols + j] - m;
  }
}

__global__ __launch_bounds__(NT) void axpy_k(int n, float alpha, const float* __restrict__ x,
                                             float* __restrict__ y) {
  for (int i = blockIdx.x * NT + threadIdx.x; i < n; i += gridDim.x * NT) y[i] = fmaf(alpha, x[i], y[i]);
}

}  // namespace

TMR_API int tmr_center_cols(const float* x, int rows, int cols, float* center, float* xc,
                            hipStream_t stream) {
  TMR_CHECK_ARG(rows > 0 && cols > 0, "tmr_center_cols: bad shape %dx%d", rows, cols);
  hipLaunchKernelGGL(center_cols_k, dim3(cdiv(cols, CC_COLS)), dim3(CC_COLS * CC_RG), 0, stream, x,
                     rows, cols, center, xc);
  TMR_CHECK_LAUNCH("center_cols");
  return 0;
}

TMR_API int tmr_axpy(int n, float alpha, const float* x, float* y, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(axpy_k, dim3(blocks_for(n)), dim3(NT), 0, stream, n, alpha, x, y);
  TMR_CHECK_LAUNCH("axpy");
  return 0;
}

TMR_API int tmr_splat_gap(const float* x, float* gap, int n, int hw, int c, hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0, "tmr_splat_gap: channels %d must be a multiple of 4", c);
  int cols, chunks;
  red_shape(c / 4, cols, chunks);
  hipLaunchKernelGGL(splat_gap_k, dim3(n * chunks), dim3(NT), 0, stream, x, gap, hw, c / 4, cols,
                     chunks);
  TMR_CHECK_LAUNCH("splat_gap");
  return 0;
}

TMR_API int tmr_splat_combine(const float* x, const float* z, float* att, float* out, int n,
                              int hw, int c, hipStream_t stream) {
  hipLaunchKernelGGL(splat_combine_k, dim3(blocks_for((long)n * hw * c)), dim3(NT), 0, stream, x, z,
                     att, out, n, hw, c);
  TMR_CHECK_LAUNCH("splat_combine");
  return 0;
}

TMR_API int tmr_splat_bwd(const float* dout, const float* x, const float* att, float* dz, int n,
                          int hw, int c, hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0, "tmr_splat_bwd: channels %d must be a multiple of 4", c);
  int cols, chunks;
  red_shape(c / 4, cols, chunks);
  hipLaunchKernelGGL(splat_bwd_reduce_k, dim3(n * chunks), dim3(NT), 0, stream, dout, x, att, dz, hw,
                     c / 4, cols, chunks);
  TMR_CHECK_LAUNCH("splat_bwd_reduce");
  return 0;
}

TMR_API int tmr_splat_bwd_apply(const float* dout, const float* att, const float* dgap, float* dx,
                                int n, int hw, int c, hipStream_t stream) {
  hipLaunchKernelGGL(splat_bwd_apply_k, dim3(blocks_for((long)n * hw * 2 * c)), dim3(NT), 0, stream,
                     dout, att, dgap, dx, n, hw, c);
  TMR_CHECK_LAUNCH("splat_bwd_apply");
  return 0;
}

TMR_API int tmr_avgpool2d_fwd(const float* x, float* y, int n, int h, int w, int c, int ho, int wo,
                              int k, int s, int p, int count_include_pad, hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0, "tmr_avgpool2d_fwd: channels %d must be a multiple of 4", c);
  if ((long)n * ho * wo * c / 4 < (1L << 31))
    hipLaunchKernelGGL(avgpool2d_fwd_k<uint32_t>, dim3(blocks_for((long)n * ho * wo * c / 4)), dim3(NT), 0,
                     stream, x, y, n, h, w, c / 4, ho, wo, k, s, p, count_include_pad);
  else
    hipLaunchKernelGGL(avgpool2d_fwd_k<long>, dim3(blocks_for((long)n * ho * wo * c / 4)), dim3(NT), 0,
                     stream, x, y, n, h, w, c / 4, ho, wo, k, s, p, count_include_pad);
  TMR_CHECK_LAUNCH("avgpool2d_fwd");
  return 0;
}

TMR_API int tmr_avgpool2d_bwd(const float* dy, float* dx, int n, int h, int w, int c, int ho,
                              int wo, int k, int s, int p, int count_include_pad,
                              hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0, "tmr_avgpool2d_bwd: channels %d must be a multiple of 4", c);
  if ((long)n * h * w * c / 4 < (1L << 31)) {
    const uint32_t total = (uint32_t)((long)n * h * w * c / 4);
    const dim3 g(blocks_for((long)n * h * w * c / 4));
    const FastDiv dc4 = make_fastdiv((uint32_t)(c / 4)), dw = make_fastdiv((uint32_t)w),
                  dh = make_fastdiv((uint32_t)h);
    if (k == 3 && s == 2 && p == 1)
      hipLaunchKernelGGL((avgpool2d_bwd_fd_k<3, 2, 1>), g, dim3(NT), 0, stream, dy, dx, total, dc4,
                         dw, dh, ho, wo, k, s, p, count_include_pad);
    else if (k == 2 && s == 2 && p == 0)
      hipLaunchKernelGGL((avgpool2d_bwd_fd_k<2, 2, 0>), g, dim3(NT), 0, stream, dy, dx, total, dc4,
                         dw, dh, ho, wo, k, s, p, count_include_pad);
    else
      hipLaunchKernelGGL((avgpool2d_bwd_fd_k<0, 0, 0>), g, dim3(NT), 0, stream, dy, dx, total, dc4,
                         dw, dh, ho, wo, k, s, p, count_include_pad);
  } else
    hipLaunchKernelGGL(avgpool2d_bwd_k<long>, dim3(blocks_for((long)n * h * w * c / 4)), dim3(NT), 0, stream,
                     dy, dx, n, h, w, c / 4, ho, wo, k, s, p, count_include_pad);
  TMR_CHECK_LAUNCH("avgpool2d_bwd");
  return 0;
}

TMR_API int tmr_splat_gap_bn(const void* y, const float* scale, const float* shift, float* gap,
                             int n, int hw, int c, int act16, hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0 && n > 0 && hw > 0, "tmr_splat_gap_bn: bad shape n %d hw %d c %d", n, hw, c);
  int cols, chunks;
  red_shape(c / 4, cols, chunks);
  // bf16: 1024-thread blocks (round 4: one 256-thread block per frame and channel chunk had too
  // few loads in flight)
  if (act16)
    hipLaunchKernelGGL((splat_gap_bn_k<__bf16, 1024>), dim3(n * chunks), dim3(1024), 0, stream,
                       (const __bf16*)y, scale, shift, gap, hw, c / 4, cols, chunks);
  else
    hipLaunchKernelGGL(splat_gap_bn_k<float>, dim3(n * chunks), dim3(NT), 0, stream,
                       (const float*)y, scale, shift, gap, hw, c / 4, cols, chunks);
  TMR_CHECK_LAUNCH("splat_gap_bn");
  return 0;
}

TMR_API int tmr_splat_att(const float* zl, float* att, int n, int c, hipStream_t stream) {
  TMR_CHECK_ARG(n > 0 && c > 0, "tmr_splat_att: bad shape n %d c %d", n, c);
  hipLaunchKernelGGL(splat_att_k, dim3(blocks_for((long)n * c)), dim3(NT), 0, stream, zl, att, n, c);
  TMR_CHECK_LAUNCH("splat_att");
  return 0;
}

TMR_API int tmr_splat_combine_bn(const void* y, const float* scale, const float* shift,
                                 const float* att, void* out, int n, int hw, int c, int act16,
                                 hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0 && n > 0 && hw > 0, "tmr_splat_combine_bn: bad shape n %d hw %d c %d "
                "(channels a multiple of 4)", n, hw, c);
  const long total = (long)n * hw * c / 4;
  TMR_CHECK_ARG(total < (1L << 31), "tmr_splat_combine_bn: %ld element groups exceed 2^31", total);
  const int nb = blocks_for(total);
  const FastDiv dc4 = make_fastdiv((uint32_t)(c / 4)), dhw = make_fastdiv((uint32_t)hw);
  if (act16 && c % 8 == 0 && NT % (c / 8) == 0 &&
      ((((uintptr_t)y) | ((uintptr_t)out)) & 15) == 0) {
    const long npix = (long)n * hw;
    hipLaunchKernelGGL(splat_combine_bn8_k, dim3(blocks_for(npix * (c / 8))), dim3(NT), 0, stream,
                       (const __bf16*)y, scale, shift, att, (__bf16*)out, (uint32_t)npix, c, dhw);
  } else if (act16)
    hipLaunchKernelGGL(splat_combine_bn_k<__bf16>, dim3(nb), dim3(NT), 0, stream, (const __bf16*)y,
                       scale, shift, att, (__bf16*)out, (uint32_t)total, dc4, dhw);
  else
    hipLaunchKernelGGL(splat_combine_bn_k<float>, dim3(nb), dim3(NT), 0, stream, (const float*)y,
                       scale, shift, att, (float*)out, (uint32_t)total, dc4, dhw);
  TMR_CHECK_LAUNCH("splat_combine_bn");
  return 0;
}

TMR_API int tmr_splat_bwd_reduce_bn(const float* dout, const void* y, const float* scale,
                                    const float* shift, const float* mean, const float* att,
                                    float* dzl, float* sums, int n, int hw, int c, int act16,
                                    hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0 && n > 0 && hw > 0, "tmr_splat_bwd_reduce_bn: bad shape n %d hw %d c %d", n, hw, c);
  int cols, chunks;
  red_shape(c / 4, cols, chunks);
  if (act16)
    hipLaunchKernelGGL(splat_bwd_reduce_bn_k<__bf16>, dim3(n * chunks), dim3(NT), 0, stream, dout,
                       (const __bf16*)y, scale, shift, mean, att, dzl, sums, n, hw, c / 4, cols, chunks);
  else
    hipLaunchKernelGGL(splat_bwd_reduce_bn_k<float>, dim3(n * chunks), dim3(NT), 0, stream, dout,
                       (const float*)y, scale, shift, mean, att, dzl, sums, n, hw, c / 4, cols, chunks);
  TMR_CHECK_LAUNCH("splat_bwd_reduce_bn");
  return 0;
}

TMR_API int tmr_splat_bn0_coefs(const float* att, const float* dgap, const float* sums,
                                const float* mean, const float* invstd, const float* gamma,
                                float* coef, float* dgamma, float* dbeta, int n, int hw, int c,
                                hipStream_t stream) {
  TMR_CHECK_ARG(n > 0 && hw > 0 && c > 0, "tmr_splat_bn0_coefs: bad shape n %d hw %d c %d", n, hw, c);
  hipLaunchKernelGGL(splat_bn0_coefs_k, dim3(cdiv(2L * c, CC_COLS)), dim3(CC_COLS * CC_RG), 0, stream,
                     att, dgap, sums, mean, invstd, gamma, coef, dgamma, dbeta, n, hw, c);
  TMR_CHECK_LAUNCH("splat_bn0_coefs");
  return 0;
}

TMR_API int tmr_splat_bwd_apply_bn(const float* dout, const void* y, const float* scale,
                                   const float* shift, const float* mean, const float* att,
                                   const float* dgap, const float* coef, void* dy, int n, int hw,
                                   int c, int act16, hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0 && n > 0 && hw > 0, "tmr_splat_bwd_apply_bn: bad shape n %d hw %d c %d "
                "(channels a multiple of 4)", n, hw, c);
  const long total = (long)n * hw * 2 * c / 4;
  TMR_CHECK_ARG(total < (1L << 31), "tmr_splat_bwd_apply_bn: %ld element groups exceed 2^31", total);
  const int nb = blocks_for(total);
  const FastDiv dj4 = make_fastdiv((uint32_t)(2 * c / 4)), dhw = make_fastdiv((uint32_t)hw);
  if (act16 && c % 8 == 0 && NT % (c / 8) == 0 &&
      ((((uintptr_t)dout) | ((uintptr_t)y) | ((uintptr_t)dy)) & 15) == 0) {
    const long npix = (long)n * hw;
    const int nb8 = blocks_for(npix * (c / 8));   // (a multiple of c/8 threads: NT % (c/8) == 0)
    hipLaunchKernelGGL(splat_bwd_apply_bn8_k, dim3(nb8), dim3(NT), 0, stream, dout,
                       (const __bf16*)y, scale, shift, mean, att, dgap, coef, (__bf16*)dy,
                       (uint32_t)npix, c, dhw);
  } else if (act16)
    hipLaunchKernelGGL(splat_bwd_apply_bn_k<__bf16>, dim3(nb), dim3(NT), 0, stream, dout,
                       (const __bf16*)y, scale, shift, mean, att, dgap, coef, (__bf16*)dy,
                       (uint32_t)total, dj4, dhw);
  else
    hipLaunchKernelGGL(splat_bwd_apply_bn_k<float>, dim3(nb), dim3(NT), 0, stream, dout,
                       (const float*)y, scale, shift, mean, att, dgap, coef, (float*)dy,
                       (uint32_t)total, dj4, dhw);
  TMR_CHECK_LAUNCH("splat_bwd_apply_bn");
  return 0;
}

TMR_API int tmr_avgpool2d_fwd_a16(const void* x, void* y, int n, int h, int w, int c, int ho,
                                  int wo, int k, int s, int p, int count_include_pad,
                                  hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0, "tmr_avgpool2d_fwd_a16: channels %d must be a multiple of 4", c);
  const long groups = (long)n * ho * wo * c / 4;
  if (groups < (1L << 31) && ((k == 3 && s == 2 && p == 1) || (k == 2 && s == 2 && p == 0))) {
    const FastDiv dc4 = make_fastdiv((uint32_t)(c / 4)), dwo = make_fastdiv((uint32_t)wo),
                  dho = make_fastdiv((uint32_t)ho);
    if (k == 3)
      hipLaunchKernelGGL((avgpool2d_fwd_a16_fd_k<3, 2, 1>), dim3(blocks_for(groups)), dim3(NT), 0,
                         stream, (const __bf16*)x, (__bf16*)y, (uint32_t)groups, dc4, dwo, dho, h, w,
                         count_include_pad);
    else
      hipLaunchKernelGGL((avgpool2d_fwd_a16_fd_k<2, 2, 0>), dim3(blocks_for(groups)), dim3(NT), 0,
                         stream, (const __bf16*)x, (__bf16*)y, (uint32_t)groups, dc4, dwo, dho, h, w,
                         count_include_pad);
  } else if (groups < (1L << 31))
    hipLaunchKernelGGL(avgpool2d_fwd_a16_k<uint32_t>, dim3(blocks_for((long)n * ho * wo * c / 4)), dim3(NT), 0,
                     stream, (const __bf16*)x, (__bf16*)y, n, h, w, c / 4, ho, wo, k, s, p,
                     count_include_pad);
  else
    hipLaunchKernelGGL(avgpool2d_fwd_a16_k<long>, dim3(blocks_for((long)n * ho * wo * c / 4)), dim3(NT), 0,
                     stream, (const __bf16*)x, (__bf16*)y, n, h, w, c / 4, ho, wo, k, s, p,
                     count_include_pad);
  TMR_CHECK_LAUNCH("avgpool2d_fwd_a16");
  return 0;
}

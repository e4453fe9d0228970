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
__global__ __launch_bounds__(NT) void avgpool2d_fwd_k(const float* __restrict__ x, float* __restrict__ y,
                                                      int n, int h, int w, int c4, int ho, int wo,
                                                      int k, int s, int p, int incl) {
  const long total = (long)n * ho * wo * c4;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int cq = (int)(i % c4);
    long t = i / c4;
    const int ox = (int)(t % wo);
    t /= wo;
    const int oy = (int)(t % ho);
    const int nn = (int)(t / ho);
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

__global__ __launch_bounds__(NT) void avgpool2d_bwd_k(const float* __restrict__ dy, float* __restrict__ dx,
                                                      int n, int h, int w, int c4, int ho, int wo,
                                                      int k, int s, int p, int incl) {
  const long total = (long)n * h * w * c4;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int cq = (int)(i % c4);
    long t = i / c4;
    const int ix = (int)(t % w);
    t /= w;
    const int iy = (int)(t % h);
    const int nn = (int)(t / h);
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

// one thread per column: rows are few (frames), columns <= 512
__global__ __launch_bounds__(NT) void center_cols_k(const float* __restrict__ x, int rows, int cols,
                                                    float* __restrict__ center, float* __restrict__ xc) {
  const int j = blockIdx.x * NT + threadIdx.x;
  if (j >= cols) return;
  double s = 0.0;
  for (int i = 0; i < rows; ++i) s += x[(long)i * cols + j];
  const float m = (float)(s / (double)rows);
  center[j] = m;
  for (int i = 0; i < rows; ++i) xc[(long)i * cols + j] = x[(long)i * cols + j] - m;
}

__global__ __launch_bounds__(NT) void axpy_k(int n, float alpha, const float* __restrict__ x,
                                             float* __restrict__ y) {
  for (int i = blockIdx.x * NT + threadIdx.x; i < n; i += gridDim.x * NT) y[i] = fmaf(alpha, x[i], y[i]);
}

}  // namespace

TMR_API int tmr_center_cols(const float* x, int rows, int cols, float* center, float* xc,
                            hipStream_t stream) {
  TMR_CHECK_ARG(rows > 0 && cols > 0, "tmr_center_cols: bad shape %dx%d", rows, cols);
  hipLaunchKernelGGL(center_cols_k, dim3((cols + NT - 1) / NT), dim3(NT), 0, stream, x, rows, cols,
                     center, xc);
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
  hipLaunchKernelGGL(avgpool2d_fwd_k, dim3(blocks_for((long)n * ho * wo * c / 4)), dim3(NT), 0,
                     stream, x, y, n, h, w, c / 4, ho, wo, k, s, p, count_include_pad);
  TMR_CHECK_LAUNCH("avgpool2d_fwd");
  return 0;
}

TMR_API int tmr_avgpool2d_bwd(const float* dy, float* dx, int n, int h, int w, int c, int ho,
                              int wo, int k, int s, int p, int count_include_pad,
                              hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0, "tmr_avgpool2d_bwd: channels %d must be a multiple of 4", c);
  hipLaunchKernelGGL(avgpool2d_bwd_k, dim3(blocks_for((long)n * h * w * c / 4)), dim3(NT), 0, stream,
                     dy, dx, n, h, w, c / 4, ho, wo, k, s, p, count_include_pad);
  TMR_CHECK_LAUNCH("avgpool2d_bwd");
  return 0;
}

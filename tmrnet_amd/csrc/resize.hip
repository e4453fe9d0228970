// Frame resize of the input pipeline: transforms.Resize((250, 250)) on the decoded PIL frame
// (code/Training TMRNet/train_only_non-local_pretrained.py:336, :344, :353, :362), i.e. Pillow's
// Image.resize(size, BILINEAR) (libImaging/Resample.c), bit-exact for 8-bit RGB.
//
// Host: the per-axis tables of Pillow's precompute_coeffs (double arithmetic in Pillow's order)
// and normalize_coeffs_8bpc (22-bit fixed point).  Device: the two 8-bit passes, horizontal first
// over the rows the vertical pass reads, each channel clip8((1 << 21) + sum(pixel * k)); a pass
// whose size does not change is skipped (Pillow's need_horizontal / need_vertical).
// Oracle: oracle/resize_ref.py, pinned to Pillow 12.2.0 by tests/golden/resize_pil.json.
#include "common.h"
#include "tmr.h"

#include <math.h>

namespace {

constexpr int kPrecisionBits = 22;   // 32 - 8 - 2, Pillow's PRECISION_BITS for 8 bpc
constexpr int NT = 256;

__device__ __forceinline__ uint8_t clip8(int acc) {
  const int v = acc >> kPrecisionBits;   // arithmetic shift, as Pillow's lookup index
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// horizontal pass: rows [y0, y0 + rows) of in (n, h, w, 3) -> tmp (n, rows, ow, 3)
__global__ __launch_bounds__(NT) void resize_h_k(const uint8_t* __restrict__ in, int h, int w,
                                                 int y0, int rows, int ow,
                                                 const int* __restrict__ bounds,
                                                 const int* __restrict__ kk, int ksize,
                                                 uint8_t* __restrict__ tmp, long total) {
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int xo = (int)(i % ow);
    const long t = i / ow;
    const int yr = (int)(t % rows);
    const long f = t / rows;
    const int xmin = bounds[2 * xo], cnt = bounds[2 * xo + 1];
    const int* k = kk + (long)xo * ksize;
    const uint8_t* src = in + ((f * h + y0 + yr) * (long)w + xmin) * 3;
    int s0 = 1 << (kPrecisionBits - 1), s1 = s0, s2 = s0;
    for (int x = 0; x < cnt; ++x) {
      const int kx = k[x];
      s0 += (int)src[3 * x] * kx;
      s1 += (int)src[3 * x + 1] * kx;
      s2 += (int)src[3 * x + 2] * kx;
    }
    uint8_t* d = tmp + i * 3;
    d[0] = clip8(s0);
    d[1] = clip8(s1);
    d[2] = clip8(s2);
  }
}

// vertical pass: src (n, sh, ow, 3) -> out (n, oh, ow, 3); bounds already relative to src's rows
__global__ __launch_bounds__(NT) void resize_v_k(const uint8_t* __restrict__ src, int sh, int ow,
                                                 int oh, const int* __restrict__ bounds,
                                                 const int* __restrict__ kk, int ksize, int yshift,
                                                 uint8_t* __restrict__ out, long total) {
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int xo = (int)(i % ow);
    const long t = i / ow;
    const int yo = (int)(t % oh);
    const long f = t / oh;
    const int ymin = bounds[2 * yo] - yshift, cnt = bounds[2 * yo + 1];
    const int* k = kk + (long)yo * ksize;
    const uint8_t* s = src + ((f * sh + ymin) * (long)ow + xo) * 3;
    const long rs = (long)ow * 3;
    int s0 = 1 << (kPrecisionBits - 1), s1 = s0, s2 = s0;
    for (int y = 0; y < cnt; ++y) {
      const int ky = k[y];
      s0 += (int)s[y * rs] * ky;
      s1 += (int)s[y * rs + 1] * ky;
      s2 += (int)s[y * rs + 2] * ky;
    }
    uint8_t* d = out + i * 3;
    d[0] = clip8(s0);
    d[1] = clip8(s1);
    d[2] = clip8(s2);
  }
}

int ew_blocks(long n) {
  long b = (n + NT - 1) / NT;
  if (b > 8192) b = 8192;
  return (int)(b > 0 ? b : 1);
}

}  // namespace

TMR_API int tmr_resize_ksize(int in_size, int out_size) {
  if (in_size <= 0 || out_size <= 0) {
    tmr_set_error("tmr_resize_ksize: bad sizes %d -> %d", in_size, out_size);
    return -1;
  }
  double filterscale = (double)in_size / out_size;
  if (filterscale < 1.0) filterscale = 1.0;
  return (int)ceil(1.0 * filterscale) * 2 + 1;
}

TMR_API int tmr_resize_coeffs(int in_size, int out_size, int32_t* bounds, int32_t* k, int ksize) {
  const int need = tmr_resize_ksize(in_size, out_size);
  TMR_CHECK_ARG(need > 0 && ksize == need && bounds && k,
                "tmr_resize_coeffs: ksize %d != %d or null tables", ksize, need);
  // Pillow precompute_coeffs (bilinear: support 1, triangle filter), in its order of operations
  const double scale = (double)in_size / out_size;
  double filterscale = scale;
  if (filterscale < 1.0) filterscale = 1.0;
  const double support = 1.0 * filterscale;
  const double ss = 1.0 / filterscale;
  double w[4096];
  TMR_CHECK_ARG(ksize <= 4096, "tmr_resize_coeffs: downscale %d -> %d too large", in_size, out_size);
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = (xx + 0.5) * scale;
    double ww = 0.0;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    for (int x = 0; x < xmax; ++x) {
      double t = (x + xmin - center + 0.5) * ss;
      if (t < 0.0) t = -t;
      const double v = t < 1.0 ? 1.0 - t : 0.0;
      w[x] = v;
      ww += v;
    }
    for (int x = 0; x < xmax; ++x)
      if (ww != 0.0) w[x] /= ww;
    // normalize_coeffs_8bpc
    int32_t* kr = k + (long)xx * ksize;
    for (int x = 0; x < ksize; ++x) {
      const double v = x < xmax ? w[x] : 0.0;
      kr[x] = v < 0 ? (int32_t)(-0.5 + v * (1 << kPrecisionBits))
                    : (int32_t)(0.5 + v * (1 << kPrecisionBits));
    }
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
  }
  return 0;
}

TMR_API size_t tmr_resize_tmp_bytes(int n, int h, int w, int oh, int ow) {
  if (n <= 0 || h <= 0 || w <= 0 || oh <= 0 || ow <= 0) {
    tmr_set_error("tmr_resize_tmp_bytes: bad shape");
    return 0;
  }
  return (size_t)n * h * ow * 3;
}

TMR_API int tmr_resize_u8(const uint8_t* in, int n, int h, int w, uint8_t* tmp, size_t tmp_bytes,
                          uint8_t* out, int oh, int ow, const int32_t* bounds_h,
                          const int32_t* k_h, int ksize_h, const int32_t* bounds_v,
                          const int32_t* k_v, int ksize_v, int y0, int y1, hipStream_t stream) {
  TMR_CHECK_ARG(in && out && n > 0 && h > 0 && w > 0 && oh > 0 && ow > 0,
                "tmr_resize_u8: bad arguments");
  const bool need_h = ow != w, need_v = oh != h;
  if (!need_h && !need_v) {
    const hipError_t e = hipMemcpyAsync(out, in, (size_t)n * h * w * 3, hipMemcpyDeviceToDevice, stream);
    TMR_CHECK_ARG(e == hipSuccess, "tmr_resize_u8: copy failed (%s)", hipGetErrorString(e));
    return 0;
  }
  if (need_h) {
    TMR_CHECK_ARG(bounds_h && k_h && ksize_h == tmr_resize_ksize(w, ow),
                  "tmr_resize_u8: horizontal tables");
    // rows the vertical pass reads (all of them without a vertical pass)
    if (!need_v) { y0 = 0; y1 = h; }
    TMR_CHECK_ARG(0 <= y0 && y0 < y1 && y1 <= h, "tmr_resize_u8: row box [%d, %d) of %d", y0, y1, h);
    uint8_t* dst = need_v ? tmp : out;
    TMR_CHECK_ARG(dst, "tmr_resize_u8: null tmp");
    TMR_CHECK_ARG(!need_v || tmp_bytes >= (size_t)n * (y1 - y0) * ow * 3, "tmr_resize_u8: tmp too small");
    const long total = (long)n * (y1 - y0) * ow;
    hipLaunchKernelGGL(resize_h_k, dim3(ew_blocks(total)), dim3(NT), 0, stream, in, h, w, y0, y1 - y0,
                       ow, (const int*)bounds_h, (const int*)k_h, ksize_h, dst, total);
    TMR_CHECK_LAUNCH("resize_h");
  }
  if (need_v) {
    TMR_CHECK_ARG(bounds_v && k_v && ksize_v == tmr_resize_ksize(h, oh),
                  "tmr_resize_u8: vertical tables");
    const uint8_t* src = need_h ? tmp : in;
    const int sh = need_h ? y1 - y0 : h;
    const int yshift = need_h ? y0 : 0;
    const long total = (long)n * oh * ow;
    hipLaunchKernelGGL(resize_v_k, dim3(ew_blocks(total)), dim3(NT), 0, stream, src, sh, ow, oh,
                       (const int*)bounds_v, (const int*)k_v, ksize_v, yshift, out, total);
    TMR_CHECK_LAUNCH("resize_v");
  }
  return 0;
}

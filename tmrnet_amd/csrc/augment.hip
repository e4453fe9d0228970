// Per-clip training augmentation of the reference on the device, bit-exact to PIL.
//
// Replaces the PIL transform chain of the reference's default training input
// (use_flip = 1, code/Training TMRNet/train_only_non-local_pretrained.py:342-350):
//   RandomCrop(224) (:101-126) -> ColorJitter(0.1, 0.1, 0.1, 0.05) (:155-177) ->
//   RandomHorizontalFlip (:129-141) -> RandomRotation(5) (:143-153) -> ToTensor -> Normalize
// (use_flip = 0: crop -> flip only, :334-341).  The per-clip parameters come from the
// reference's own seeding rule on the host (tmrnet_amd/augment.py); here every pixel of every
// frame is produced in one pass (plus one per-frame reduction for the contrast mean):
//   * brightness / contrast / saturation = PIL ImageEnhance = Image.blend(degenerate, im, f):
//     uint8 + float(alpha) * diff in fp32, truncated (clipped when alpha > 1);
//   * contrast's degenerate value = int(mean of the "L" image + 0.5), L = (19595 R + 38470 G +
//     7471 B + 0x8000) >> 16, over the brightness-adjusted crop;
//   * hue = torchvision adjust_hue: PIL RGB->HSV, H += uint8 shift (wraps), HSV->RGB, with PIL's
//     mix of float and double arithmetic reproduced operation by operation;
//   * rotation = PIL Image.rotate(angle, NEAREST): the affine_fixed path (16.16 fixed-point
//     coefficients, computed on the host exactly as PIL does), fill 0.
// Validated against PIL over the whole RGB / HSV cubes and every rotation angle
// (tests/test_augment_cpu.py pins the host model, tests/test_augment_gpu.py the kernel).
#include "common.h"
#include "tmr.h"

#pragma clang fp contract(off)   // PIL's C code is compiled without FMA contraction

namespace {

constexpr int NT = 256;

__device__ __forceinline__ int clip8(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

// Image.blend of uint8 values (ImagingBlend): in1 + alpha * (in2 - in1) in fp32
__device__ __forceinline__ int blend_u8(int in1, int in2, float alpha) {
  const float t = (float)in1 + alpha * (float)(in2 - in1);
  if (alpha >= 0.f && alpha <= 1.f) return (int)t;
  if (t <= 0.f) return 0;
  if (t >= 255.f) return 255;
  return (int)t;
}

__device__ __forceinline__ int to_l(int r, int g, int b) {
  return (r * 19595 + g * 38470 + b * 7471 + 0x8000) >> 16;
}

// PIL rgb2hsv_row (Convert.c) then hue shift then hsv2rgb
__device__ void hue_shift(int& r, int& g, int& b, int shift) {
  const int maxc = max(r, max(g, b)), minc = min(r, min(g, b));
  int uh = 0, us = 0;
  const int uv = maxc;
  if (maxc != minc) {
    const float cr = (float)(maxc - minc);
    const float s = cr / (float)maxc;
    const float rc = (float)(maxc - r) / cr;
    const float gc = (float)(maxc - g) / cr;
    const float bc = (float)(maxc - b) / cr;
    float h;
    if (r == maxc) h = bc - gc;
    else if (g == maxc) h = (float)(2.0 + (double)rc - (double)bc);
    else h = (float)(4.0 + (double)gc - (double)rc);
    h = (float)fmod((double)h / 6.0 + 1.0, 1.0);
    uh = clip8((int)((double)h * 255.0));
    us = clip8((int)((double)s * 255.0));
  }
  uh = (uh + shift) & 255;
  if (us == 0) {
    r = g = b = uv;
    return;
  }
  const double x = (double)(float)uh * 6.0 / 255.0;
  const int i = (int)floor(x);
  const float f = (float)(x - (double)(float)i);
  const float fs = (float)((double)(float)us / 255.0);
  const double vv = (double)(float)uv;
  const int up = clip8((int)round(vv * (1.0 - (double)fs)));
  const int uq = clip8((int)round(vv * (1.0 - (double)(fs * f))));
  const int ut = clip8((int)round(vv * (1.0 - (double)fs * (1.0 - (double)f))));
  switch (i % 6) {
    case 0: r = uv; g = ut; b = up; break;
    case 1: r = uq; g = uv; b = up; break;
    case 2: r = up; g = uv; b = ut; break;
    case 3: r = up; g = uq; b = uv; break;
    case 4: r = ut; g = up; b = uv; break;
    default: r = uv; g = up; b = uq; break;
  }
}

// per-frame contrast mean: int(mean(L(brightness(crop))) + 0.5)
__global__ __launch_bounds__(NT) void aug_lmean_k(const uint8_t* __restrict__ fr,
                                                  const tmr_clip_aug* __restrict__ prm,
                                                  int32_t* __restrict__ lmean, int hin, int win,
                                                  int crop) {
  const int fi = blockIdx.x;
  const tmr_clip_aug p = prm[fi];
  if (!p.jitter) {
    if (threadIdx.x == 0) lmean[fi] = 0;
    return;
  }
  const int npx = crop * crop;
  const int x1 = min(max(p.x1, 0), win - crop), y1 = min(max(p.y1, 0), hin - crop);
  int s = 0;
  for (int i = threadIdx.x; i < npx; i += NT) {
    const int y = i / crop, x = i - y * crop;
    const uint8_t* px = fr + (((long)fi * hin + (y + y1)) * win + (x + x1)) * 3;
    const int r = blend_u8(0, px[0], p.brightness);
    const int g = blend_u8(0, px[1], p.brightness);
    const int b = blend_u8(0, px[2], p.brightness);
    s += to_l(r, g, b);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  __shared__ int red[NT / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < NT / 64; ++w) t += red[w];
    lmean[fi] = (int)((double)t / (double)npx + 0.5);
  }
}

__global__ __launch_bounds__(NT) void aug_apply_k(const uint8_t* __restrict__ fr,
                                                  const tmr_clip_aug* __restrict__ prm,
                                                  const int32_t* __restrict__ lmean,
                                                  float4* __restrict__ out, int f, int hin, int win,
                                                  int crop, float m0, float m1, float m2, float s0,
                                                  float s1, float s2) {
  const long total = (long)f * crop * crop;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int x = (int)(i % crop);
    const long t = i / crop;
    const int y = (int)(t % crop);
    const int fi = (int)(t / crop);
    const tmr_clip_aug& p = prm[fi];
    const int x1 = min(max(p.x1, 0), win - crop), y1 = min(max(p.y1, 0), hin - crop);
    // source pixel of the (flipped, jittered) crop: rotation (affine_fixed), then the flip
    int xs = x, ys = y;
    bool inside = true;
    if (p.rotate) {
      xs = (p.a[2] + y * p.a[1] + x * p.a[0]) >> 16;
      ys = (p.a[5] + y * p.a[4] + x * p.a[3]) >> 16;
      inside = xs >= 0 && xs < crop && ys >= 0 && ys < crop;
    }
    int r = 0, g = 0, b = 0;   // RandomRotation fill
    if (inside) {
      if (p.flip) xs = crop - 1 - xs;
      const uint8_t* px = fr + (((long)fi * hin + (ys + y1)) * win + (xs + x1)) * 3;
      r = px[0]; g = px[1]; b = px[2];
      if (p.jitter) {
        r = blend_u8(0, r, p.brightness);
        g = blend_u8(0, g, p.brightness);
        b = blend_u8(0, b, p.brightness);
        const int m = lmean[fi];
        r = blend_u8(m, r, p.contrast);
        g = blend_u8(m, g, p.contrast);
        b = blend_u8(m, b, p.contrast);
        const int l = to_l(r, g, b);
        r = blend_u8(l, r, p.saturation);
        g = blend_u8(l, g, p.saturation);
        b = blend_u8(l, b, p.saturation);
        hue_shift(r, g, b, p.hue_shift);
      }
    }
    const float rf = (float)r / 255.0f, gf = (float)g / 255.0f, bf = (float)b / 255.0f;
    out[i] = make_float4((rf - m0) / s0, (gf - m1) / s1, (bf - m2) / s2, 0.f);
  }
}

int ew_blocks(long n) {
  long b = (n + NT - 1) / NT;
  if (b > 2048 * 8) b = 2048 * 8;
  return (int)(b > 0 ? b : 1);
}

}  // namespace

TMR_API int tmr_clip_augment(const uint8_t* frames, const tmr_clip_aug* params, int32_t* lmean,
                             float* out, int f, int hin, int win, int crop, float m0, float m1,
                             float m2, float s0, float s1, float s2, hipStream_t stream) {
  TMR_CHECK_ARG(f >= 0 && crop > 0 && crop <= hin && crop <= win,
                "tmr_clip_augment: bad geometry f=%d %dx%d crop %d", f, hin, win, crop);
  TMR_CHECK_ARG(params && lmean, "tmr_clip_augment: null params / lmean workspace");
  if (f == 0) return 0;
  hipLaunchKernelGGL(aug_lmean_k, dim3(f), dim3(NT), 0, stream, frames, params, lmean, hin, win,
                     crop);
  TMR_CHECK_LAUNCH("clip_augment (contrast mean)");
  hipLaunchKernelGGL(aug_apply_k, dim3(ew_blocks((long)f * crop * crop)), dim3(NT), 0, stream,
                     frames, params, lmean, (float4*)out, f, hin, win, crop, m0, m1, m2, s0, s1, s2);
  TMR_CHECK_LAUNCH("clip_augment");
  return 0;
}

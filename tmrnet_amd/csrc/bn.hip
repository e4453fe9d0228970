// BatchNorm2d (train-mode batch statistics) + ReLU + residual for NHWC fp32.
//
// Replaces nn.BatchNorm2d / ReLU / the residual add inside torchvision's
// resnet50 Bottleneck (the `share` trunk of
// code/Training TMRNet/train_only_non-local_pretrained.py:204-214).
// Statistics: per-thread fp32 sums of (y - shift_c) (shift = first row, removes
// the mean bias), per-block double partials, fixed-order double reduction ->
// deterministic and accurate for rows up to millions.  HBM-bound kernels:
// float4 loads/stores along channels, grid sized to fill 256 CUs.
#include "common.h"
#include "tmr.h"
#include <type_traits>

namespace {

constexpr int NT = 256;

struct Plan {
  int cthreads;  // threads across channels (each 4 channels)
  int rthreads;  // threads across rows
  int cblocks;   // gridDim.y
  int rpb;       // rows per block
  int nrb;       // row blocks (gridDim.x)
};

Plan make_plan(int rows, int c) {
  Plan p;
  int c4 = c / 4;
  p.cthreads = c4 < 64 ? c4 : 64;
  p.rthreads = NT / p.cthreads;
  p.cblocks = c4 / p.cthreads;
  // ~1024 row blocks for large inputs, >= 8 rows per thread
  int rpb = rows / 1024;
  int minr = p.rthreads * 8;
  if (rpb < minr) rpb = minr;
  rpb = (rpb + p.rthreads - 1) / p.rthreads * p.rthreads;
  p.rpb = rpb;
  p.nrb = (rows + rpb - 1) / rpb;
  return p;
}

// layout of the double workspace: [nrb][c][2] partials, then float coeffs [3][c]
size_t ws_need(int rows, int c) {
  Plan p = make_plan(rows, c);
  return (size_t)p.nrb * c * 2 * sizeof(double) + (size_t)3 * c * sizeof(float) + 64;
}

__global__ __launch_bounds__(NT) void bn_stats_partial(const float* __restrict__ y, int rows, int c,
                                                       int rpb, int cthreads,
                                                       float4* __restrict__ part) {
  const int tc = threadIdx.x % cthreads, tr = threadIdx.x / cthreads;
  const int rthreads = NT / cthreads;
  const int ch = (blockIdx.y * cthreads + tc) * 4;
  const int r0 = blockIdx.x * rpb;
  const int r1 = min(rows, r0 + rpb);
  // shift by the block's first row: removes the mean from the fp32 sums
  const float4 sh = *reinterpret_cast<const float4*>(y + (long)r0 * c + ch);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f), q = s;
  for (int r = r0 + tr; r < r1; r += rthreads) {
    float4 v = *reinterpret_cast<const float4*>(y + (long)r * c + ch);
    float a = v.x - sh.x, b = v.y - sh.y, cc = v.z - sh.z, d = v.w - sh.w;
    s.x += a; s.y += b; s.z += cc; s.w += d;
    q.x += a * a; q.y += b * b; q.z += cc * cc; q.w += d * d;
  }
  __shared__ double red[NT][8];
  red[threadIdx.x][0] = s.x; red[threadIdx.x][1] = s.y; red[threadIdx.x][2] = s.z;
  red[threadIdx.x][3] = s.w; red[threadIdx.x][4] = q.x; red[threadIdx.x][5] = q.y;
  red[threadIdx.x][6] = q.z; red[threadIdx.x][7] = q.w;
  __syncthreads();
  if (tr == 0) {
    double acc[8];
    for (int e = 0; e < 8; ++e) acc[e] = 0.0;
    for (int k = 0; k < rthreads; ++k)
      for (int e = 0; e < 8; ++e) acc[e] += red[k * cthreads + tc][e];
    const double n = (double)(r1 - r0);
    const float shv[4] = {sh.x, sh.y, sh.z, sh.w};
    for (int e = 0; e < 4; ++e) {
      const double ms = acc[e] / n;
      double m2 = acc[4 + e] - acc[e] * ms;
      if (m2 < 0) m2 = 0;
      part[(long)blockIdx.x * c + ch + e] = make_float4((float)n, (float)(shv[e] + ms), (float)m2, 0.f);
    }
  }
}

// Combine of (n, mean, M2) partials in double, fixed order -> deterministic.  One
// workgroup per channel (the conv epilogue emits ~8k partials per channel for layer1-sized
// outputs, so the combine needs the whole chip).  Division-free shifted sums about
// K = the first partial's mean: N = sum n_b, S1 = sum n_b d_b, S2 = sum (M2_b + n_b d_b^2),
// d_b = mean_b - K; then mean = K + S1/N and M2 = S2 - S1^2/N (exact in exact arithmetic;
// the shift keeps the cancellation at the size of the spread of the partial means).
__global__ __launch_bounds__(NT) void bn_finalize_k(const float4* __restrict__ part, int nparts,
                                                    int c, const float* gamma, const float* beta,
                                                    float* rmean, float* rvar, float momentum,
                                                    float eps, float* smean, float* sinv,
                                                    float* scale, float* shift) {
  const int ch = blockIdx.x;
  const double K = part[ch].y;
  double n = 0, s1 = 0, s2 = 0;
  for (int b = threadIdx.x; b < nparts; b += NT) {
    const float4 p = part[(long)b * c + ch];
    const double nb = p.x, d = (double)p.y - K;
    n += nb;
    s1 = fma(nb, d, s1);
    s2 += (double)p.z + nb * d * d;
  }
  __shared__ double red[3][NT];
  red[0][threadIdx.x] = n; red[1][threadIdx.x] = s1; red[2][threadIdx.x] = s2;
  __syncthreads();
  for (int h = NT / 2; h > 0; h >>= 1) {
    if (threadIdx.x < h) {
      red[0][threadIdx.x] += red[0][threadIdx.x + h];
      red[1][threadIdx.x] += red[1][threadIdx.x + h];
      red[2][threadIdx.x] += red[2][threadIdx.x + h];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    n = red[0][0]; s1 = red[1][0]; s2 = red[2][0];
    const double mean = n > 0 ? K + s1 / n : 0.0;
    double m2 = n > 0 ? s2 - s1 * (s1 / n) : 0.0;
    if (m2 < 0) m2 = 0;
    const double var = n > 0 ? m2 / n : 0.0;
    const double inv = 1.0 / sqrt(var + (double)eps);
    smean[ch] = (float)mean;
    sinv[ch] = (float)inv;
    const double gm = gamma ? gamma[ch] : 1.0;
    const double bt = beta ? beta[ch] : 0.0;
    scale[ch] = (float)(gm * inv);
    shift[ch] = (float)(bt - mean * gm * inv);
    if (rmean) {
      const double unb = n > 1 ? m2 / (n - 1.0) : var;
      rmean[ch] = (float)((1.0 - momentum) * rmean[ch] + momentum * mean);
      rvar[ch] = (float)((1.0 - momentum) * rvar[ch] + momentum * unb);
    }
  }
}

__global__ void bn_eval_params_k(const float* gamma, const float* beta, const float* rm,
                                 const float* rv, float eps, int c, float* scale, float* shift) {
  int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  float inv = 1.0f / sqrtf(rv[ch] + eps);
  float g = gamma ? gamma[ch] : 1.f;
  float b = beta ? beta[ch] : 0.f;
  scale[ch] = g * inv;
  shift[ch] = b - rm[ch] * g * inv;
}

// 4 values to 4 consecutive elements of an fp32 or bf16 (RNE, the conv loaders' rounding) tensor
__device__ __forceinline__ void st4(float* p, long i4, float4 v) {
  reinterpret_cast<float4*>(p)[i4] = v;
}
__device__ __forceinline__ void st4(__bf16* p, long i4, float4 v) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  const bf16x2_t a = {(__bf16)v.x, (__bf16)v.y}, b = {(__bf16)v.z, (__bf16)v.w};
  reinterpret_cast<uint2*>(p)[i4] =
      make_uint2(__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b));
}

// channel group of element group i in rows of c groups: a mask when c is a power of two (every
// conv channel count of the trunks), else a 64-bit remainder
__device__ __forceinline__ int chan_of(long i, int c) {
  return (c & (c - 1)) == 0 ? (int)(i & (long)(c - 1)) : (int)(i % c);
}

// DUAL: z (fp32) and a bf16 (RNE) copy z16 -- a block output is both the next block's identity
// residual (fp32) and the operand of its bf16-math convs (bf16, read by the LDS-DMA engine)
// 4 consecutive elements of an fp32 or bf16 tensor as float4 (bf16 -> fp32 is exact)
__device__ __forceinline__ float4 ld4(const float* p, long i4) {
  return reinterpret_cast<const float4*>(p)[i4];
}
__device__ __forceinline__ float4 ld4(const __bf16* p, long i4) {
  const uint2 u = reinterpret_cast<const uint2*>(p)[i4];
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                     __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
}
__device__ __forceinline__ float ld1(const float* p, long i) { return p[i]; }
__device__ __forceinline__ float ld1(const __bf16* p, long i) {
  return __uint_as_float((uint32_t)reinterpret_cast<const unsigned short*>(p)[i] << 16);
}

// TY: element type of y and the residual (bf16 under the bf16-activation contract).  Two elements
// per thread and iteration, both loaded before either is used (as bn_bwd_apply).
template <bool RES, bool RELU, typename TZ = float, bool DUAL = false, typename TY = float>
__global__ __launch_bounds__(NT) void bn_apply_k(const TY* __restrict__ y, const float* __restrict__ scale,
                                                 const float* __restrict__ shift,
                                                 const TY* __restrict__ res, TZ* __restrict__ z,
                                                 long n4, int c4, __bf16* __restrict__ z16 = nullptr) {
  const long stride = (long)gridDim.x * NT;
  auto apply = [&](long i, float4 v, const float4 r) {
    const int cc = chan_of(i, c4) * 4;
    const float4 sc = *reinterpret_cast<const float4*>(scale + cc);
    const float4 sf = *reinterpret_cast<const float4*>(shift + cc);
    v.x = fmaf(v.x, sc.x, sf.x);
    v.y = fmaf(v.y, sc.y, sf.y);
    v.z = fmaf(v.z, sc.z, sf.z);
    v.w = fmaf(v.w, sc.w, sf.w);
    if (RES) {
      v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
    }
    if (RELU) {
      v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
    }
    st4(z, i, v);
    if (DUAL) st4(z16, i, v);
  };
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n4; i += 2 * stride) {
    const long j = i + stride;
    const bool hj = j < n4;
    const float4 v0 = ld4(y, i);
    const float4 r0 = RES ? ld4(res, i) : v0;
    float4 v1 = v0, r1 = r0;
    if (hj) {
      v1 = ld4(y, j);
      if (RES) r1 = ld4(res, j);
    }
    apply(i, v0, r0);
    if (hj) apply(j, v1, r1);
  }
}

// z = act(y*scale + shift + (yr*rscale + rshift)): the Bottleneck's BN3 + residual + ReLU with the
// downsample branch's BatchNorm applied on the fly (its output is never materialised).  Same
// fmaf/add/max sequence as bn_apply of the branch followed by bn_apply with that residual.
template <bool RELU, bool DUAL = false, typename TY = float, typename TZ = float>
__global__ __launch_bounds__(NT) void bn_apply2_k(const TY* __restrict__ y, const float* __restrict__ scale,
                                                  const float* __restrict__ shift,
                                                  const TY* __restrict__ yr,
                                                  const float* __restrict__ rscale,
                                                  const float* __restrict__ rshift,
                                                  TZ* __restrict__ z, long n4, int c4,
                                                  __bf16* __restrict__ z16) {
  const long stride = (long)gridDim.x * NT;
  auto apply = [&](long i, float4 v, const float4 r) {
    const int cc = chan_of(i, c4) * 4;
    const float4 sc = *reinterpret_cast<const float4*>(scale + cc);
    const float4 sf = *reinterpret_cast<const float4*>(shift + cc);
    const float4 rs = *reinterpret_cast<const float4*>(rscale + cc);
    const float4 rf = *reinterpret_cast<const float4*>(rshift + cc);
    v.x = fmaf(v.x, sc.x, sf.x) + fmaf(r.x, rs.x, rf.x);
    v.y = fmaf(v.y, sc.y, sf.y) + fmaf(r.y, rs.y, rf.y);
    v.z = fmaf(v.z, sc.z, sf.z) + fmaf(r.z, rs.z, rf.z);
    v.w = fmaf(v.w, sc.w, sf.w) + fmaf(r.w, rs.w, rf.w);
    if (RELU) {
      v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
    }
    st4(z, i, v);
    if (DUAL) st4(z16, i, v);
  };
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n4; i += 2 * stride) {
    const long j = i + stride;
    const bool hj = j < n4;
    const float4 v0 = ld4(y, i), r0 = ld4(yr, i);
    float4 v1 = v0, r1 = r0;
    if (hj) {
      v1 = ld4(y, j);
      r1 = ld4(yr, j);
    }
    apply(i, v0, r0);
    if (hj) apply(j, v1, r1);
  }
}

// The bf16-activation forms of bn_apply_k / bn_apply2_k (bf16 y, residual or branch input, and z),
// 8 elements per thread: every access a 16-B lane piece (the 4-wide forms move bf16 in 8-B
// pieces), two pieces per thread in flight.  Same fmaf / add / max sequence per element:
// identical outputs.  BR: the residual is the downsample branch's pre-BN y (bn_apply2_k).
__device__ __forceinline__ void unpack8(const uint4 w, float (&v)[8]) {
  const uint32_t u[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[2 * e] = __uint_as_float(u[e] << 16);
    v[2 * e + 1] = __uint_as_float(u[e] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 pack8(const float (&v)[8]) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  uint32_t o[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const bf16x2_t p = {(__bf16)v[2 * e], (__bf16)v[2 * e + 1]};
    o[e] = __builtin_bit_cast(uint32_t, p);
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}
template <bool RES, bool RELU, bool BR>
__global__ __launch_bounds__(NT) void bn_apply8_a16_k(const __bf16* __restrict__ y,
                                                      const float* __restrict__ scale,
                                                      const float* __restrict__ shift,
                                                      const __bf16* __restrict__ res,
                                                      const float* __restrict__ rscale,
                                                      const float* __restrict__ rshift,
                                                      __bf16* __restrict__ z, long n8, int c8) {
  const long stride = (long)gridDim.x * NT;
  auto apply = [&](long i, const uint4 yw, const uint4 rw) {
    const int cc = chan_of(i, c8) * 8;
    float v[8], r[8];
    unpack8(yw, v);
    unpack8(rw, r);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float4 sc = *reinterpret_cast<const float4*>(scale + cc + 4 * h);
      const float4 sf = *reinterpret_cast<const float4*>(shift + cc + 4 * h);
      const float a[4] = {sc.x, sc.y, sc.z, sc.w}, b[4] = {sf.x, sf.y, sf.z, sf.w};
      float ra[4] = {0.f, 0.f, 0.f, 0.f}, rb[4] = {0.f, 0.f, 0.f, 0.f};
      if (BR) {
        const float4 rs = *reinterpret_cast<const float4*>(rscale + cc + 4 * h);
        const float4 rf = *reinterpret_cast<const float4*>(rshift + cc + 4 * h);
        ra[0] = rs.x; ra[1] = rs.y; ra[2] = rs.z; ra[3] = rs.w;
        rb[0] = rf.x; rb[1] = rf.y; rb[2] = rf.z; rb[3] = rf.w;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t;
        if (BR) {
          t = fmaf(v[4 * h + e], a[e], b[e]) + fmaf(r[4 * h + e], ra[e], rb[e]);
        } else {
          t = fmaf(v[4 * h + e], a[e], b[e]);
          if (RES) t += r[4 * h + e];
        }
        if (RELU) t = fmaxf(t, 0.f);
        v[4 * h + e] = t;
      }
    }
    reinterpret_cast<uint4*>(z)[i] = pack8(v);
  };
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n8; i += 2 * stride) {
    const long j = i + stride;
    const bool hj = j < n8;
    const uint4 y0 = reinterpret_cast<const uint4*>(y)[i];
    const uint4 r0 = (RES || BR) ? reinterpret_cast<const uint4*>(res)[i] : y0;
    uint4 y1 = y0, r1 = r0;
    if (hj) {
      y1 = reinterpret_cast<const uint4*>(y)[j];
      if (RES || BR) r1 = reinterpret_cast<const uint4*>(res)[j];
    }
    apply(i, y0, r0);
    if (hj) apply(j, y1, r1);
  }
}

// The ReLU mask of a block output as bits (tmr_bn_apply_bits / tmr_bn_apply2_bits): element e is
// bit e % 32 of word e / 32.  The fp32 residual-gradient dgrads read it (mask 3) instead of
// re-reading the 4-byte z.  Each lane holds 4 consecutive elements (one float4 index i); the 8
// lanes of a word OR their nibbles.  Wave-uniform loop: the waves' lanes stay converged for the
// shuffles.
// T: element type of y, the residual / branch input and z (bf16 under the bf16-activation contract:
// the bit is taken from the stored, rounded value, so it equals the mask-1 test z > 0 exactly)
__device__ __forceinline__ float stored(float v, const float*) { return v; }
__device__ __forceinline__ float stored(float v, const __bf16*) { return (float)(__bf16)v; }
template <bool RES, typename T = float>
__global__ __launch_bounds__(NT) void bn_apply_bits_k(const T* __restrict__ y,
                                                      const float* __restrict__ scale,
                                                      const float* __restrict__ shift,
                                                      const T* __restrict__ res,
                                                      const T* __restrict__ yr,
                                                      const float* __restrict__ rscale,
                                                      const float* __restrict__ rshift,
                                                      T* __restrict__ z,
                                                      uint32_t* __restrict__ bits, long n4, int c4) {
  const int lane = threadIdx.x & 63;
  const long stride = (long)gridDim.x * NT;
  for (long base = blockIdx.x * (long)NT + (threadIdx.x & ~63); base < n4; base += stride) {
    const long i = base + lane;
    uint32_t nib = 0;
    if (i < n4) {
      const int cc = chan_of(i, c4) * 4;
      float4 v = ld4(y, i);
      const float4 sc = *reinterpret_cast<const float4*>(scale + cc);
      const float4 sf = *reinterpret_cast<const float4*>(shift + cc);
      if (yr) {   // bn_apply2: the downsample branch's BatchNorm on the fly
        const float4 r = ld4(yr, i);
        const float4 rs = *reinterpret_cast<const float4*>(rscale + cc);
        const float4 rf = *reinterpret_cast<const float4*>(rshift + cc);
        v.x = fmaf(v.x, sc.x, sf.x) + fmaf(r.x, rs.x, rf.x);
        v.y = fmaf(v.y, sc.y, sf.y) + fmaf(r.y, rs.y, rf.y);
        v.z = fmaf(v.z, sc.z, sf.z) + fmaf(r.z, rs.z, rf.z);
        v.w = fmaf(v.w, sc.w, sf.w) + fmaf(r.w, rs.w, rf.w);
      } else {
        v.x = fmaf(v.x, sc.x, sf.x); v.y = fmaf(v.y, sc.y, sf.y);
        v.z = fmaf(v.z, sc.z, sf.z); v.w = fmaf(v.w, sc.w, sf.w);
        if (RES) {
          const float4 r = ld4(res, i);
          v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
        }
      }
      v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
      st4(z, i, v);
      const T* tag = nullptr;
      nib = (uint32_t)(stored(v.x, tag) > 0.f) | ((uint32_t)(stored(v.y, tag) > 0.f) << 1) |
            ((uint32_t)(stored(v.z, tag) > 0.f) << 2) | ((uint32_t)(stored(v.w, tag) > 0.f) << 3);
    }
    uint32_t w = nib << (4 * (lane & 7));
    w |= (uint32_t)__shfl_xor((int)w, 1, 64);
    w |= (uint32_t)__shfl_xor((int)w, 2, 64);
    w |= (uint32_t)__shfl_xor((int)w, 4, 64);
    if ((lane & 7) == 0 && i < n4) bits[i >> 3] = w;
  }
}

// ReLU mask of the backward: MASK 0 = none, 1 = saved output z > 0, 2 = recomputed
// fmaf(y, scale, shift) > 0 (bit-identical to the forward's z > 0 when there is no residual,
// and saves reading z)
__device__ __forceinline__ float4 relu_mask4(float4 g, float4 m) {
  g.x = m.x > 0.f ? g.x : 0.f; g.y = m.y > 0.f ? g.y : 0.f;
  g.z = m.z > 0.f ? g.z : 0.f; g.w = m.w > 0.f ? g.w : 0.f;
  return g;
}
__device__ __forceinline__ float4 affine4(float4 v, float4 sc, float4 sf) {
  return make_float4(fmaf(v.x, sc.x, sf.x), fmaf(v.y, sc.y, sf.y), fmaf(v.z, sc.z, sf.z),
                     fmaf(v.w, sc.w, sf.w));
}

// WB: write the masked gradient back over dz (dres aliasing dz: the identity branch of a
// residual block takes the masked gradient in place, and the apply pass needs no mask)
// TG: element type of dz (bf16: the bf16 residual-stream gradient of the bf16-activation step,
// tmr_bn_bwd_g16; no write-back)
template <int MASK, bool WB = false, typename TY = float, typename TG = float>
__global__ __launch_bounds__(NT) void bn_bwd_partial(TG* dz, const TY* __restrict__ y,
                                                     const TY* __restrict__ z,
                                                     const float* __restrict__ scale,
                                                     const float* __restrict__ shift,
                                                     const float* __restrict__ mean, int rows, int c,
                                                     int rpb, int cthreads, double* __restrict__ part) {
  const int tc = threadIdx.x % cthreads, tr = threadIdx.x / cthreads;
  const int rthreads = NT / cthreads;
  const int ch = (blockIdx.y * cthreads + tc) * 4;
  const float4 mu = *reinterpret_cast<const float4*>(mean + ch);
  float4 sc = make_float4(0.f, 0.f, 0.f, 0.f), sf = sc;
  if (MASK == 2) {
    sc = *reinterpret_cast<const float4*>(scale + ch);
    sf = *reinterpret_cast<const float4*>(shift + ch);
  }
  const int r0 = blockIdx.x * rpb;
  const int r1 = min(rows, r0 + rpb);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f), q = s;
  for (int r = r0 + tr; r < r1; r += rthreads) {
    const long o = (long)r * c + ch;
    float4 g = ld4(dz, o >> 2);
    const float4 v = ld4(y, o >> 2);
    if (MASK == 1) g = relu_mask4(g, ld4(z, o >> 2));
    if (MASK == 2) g = relu_mask4(g, affine4(v, sc, sf));
    if constexpr (WB) {
      static_assert(std::is_same<TG, float>::value, "bn_bwd_partial: write-back of an fp32 dz only");
      *reinterpret_cast<float4*>(dz + o) = g;
    }
    s.x += g.x; s.y += g.y; s.z += g.z; s.w += g.w;
    q.x = fmaf(g.x, v.x - mu.x, q.x); q.y = fmaf(g.y, v.y - mu.y, q.y);
    q.z = fmaf(g.z, v.z - mu.z, q.z); q.w = fmaf(g.w, v.w - mu.w, q.w);
  }
  __shared__ double red[NT][8];
  red[threadIdx.x][0] = s.x; red[threadIdx.x][1] = s.y; red[threadIdx.x][2] = s.z;
  red[threadIdx.x][3] = s.w; red[threadIdx.x][4] = q.x; red[threadIdx.x][5] = q.y;
  red[threadIdx.x][6] = q.z; red[threadIdx.x][7] = q.w;
  __syncthreads();
  if (tr == 0) {
    double acc[8];
    for (int e = 0; e < 8; ++e) acc[e] = 0.0;
    for (int k = 0; k < rthreads; ++k)
      for (int e = 0; e < 8; ++e) acc[e] += red[k * cthreads + tc][e];
    double* o = part + ((long)blockIdx.x * c + ch) * 2;
    for (int e = 0; e < 4; ++e) {
      o[2 * e] = acc[e];
      o[2 * e + 1] = acc[4 + e];
    }
  }
}

__global__ __launch_bounds__(NT) void bn_bwd_final(const double* __restrict__ part, int nrb, int rows, int c,
                                                   const float* mean, const float* inv,
                                                   const float* gamma, float* dgamma,
                                                   float* dbeta, float* coef) {
  const int ch = blockIdx.x;  // one workgroup per channel, fixed-order tree reduction
  double s = 0.0, q = 0.0;
  for (int b = threadIdx.x; b < nrb; b += NT) {
    s += part[((long)b * c + ch) * 2];
    q += part[((long)b * c + ch) * 2 + 1];
  }
  __shared__ double red[2][NT];
  red[0][threadIdx.x] = s;
  red[1][threadIdx.x] = q;
  __syncthreads();
  for (int h = NT / 2; h > 0; h >>= 1) {
    if (threadIdx.x < h) {
      red[0][threadIdx.x] += red[0][threadIdx.x + h];
      red[1][threadIdx.x] += red[1][threadIdx.x + h];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    s = red[0][0];
    q = red[1][0];
    const double iv = inv[ch];
    const double dbt = s;
    const double dgm = q * iv;  // sum dzh * xhat
    if (dgamma) dgamma[ch] = (float)dgm;
    if (dbeta) dbeta[ch] = (float)dbt;
    const double n = (double)rows;
    const double gm = gamma ? gamma[ch] : 1.0;
    const double A = gm * iv;
    const double mdz = dbt / n, mdx = dgm / n;
    const double B = -gm * iv * iv * mdx;
    const double C = -A * mdz - B * (double)mean[ch];
    coef[ch] = (float)A;
    coef[c + ch] = (float)B;
    coef[2 * c + ch] = (float)C;
  }
}

// Two elements per thread and iteration (i and i + the grid's stride), both elements' loads issued
// before either is consumed: one element at a time kept 32 B in flight per thread and ran at
// 5.2 TB/s (`profiles/r3/rocprof_r4g/`, the fp32 step's largest non-conv kernel).
template <int MASK, bool DRES, typename TD = float, typename TY = float>
__global__ __launch_bounds__(NT) void bn_bwd_apply(const float* __restrict__ dz, const TY* __restrict__ y,
                                                   const TY* __restrict__ z,
                                                   const float* __restrict__ scale,
                                                   const float* __restrict__ shift,
                                                   const float* __restrict__ coef, TD* __restrict__ dy,
                                                   float* __restrict__ dres, long n4, int c4) {
  const int c = c4 * 4;
  const long stride = (long)gridDim.x * NT;
  auto apply = [&](long i, float4 g, const float4 v, const float4 zv) {
    const int cc = chan_of(i, c4) * 4;
    if (MASK == 1) g = relu_mask4(g, zv);
    if (MASK == 2)
      g = relu_mask4(g, affine4(v, *reinterpret_cast<const float4*>(scale + cc),
                                *reinterpret_cast<const float4*>(shift + cc)));
    if (DRES) reinterpret_cast<float4*>(dres)[i] = g;
    const float4 A = *reinterpret_cast<const float4*>(coef + cc);
    const float4 B = *reinterpret_cast<const float4*>(coef + c + cc);
    const float4 C = *reinterpret_cast<const float4*>(coef + 2 * c + cc);
    float4 o;
    o.x = fmaf(A.x, g.x, fmaf(B.x, v.x, C.x));
    o.y = fmaf(A.y, g.y, fmaf(B.y, v.y, C.y));
    o.z = fmaf(A.z, g.z, fmaf(B.z, v.z, C.z));
    o.w = fmaf(A.w, g.w, fmaf(B.w, v.w, C.w));
    st4(dy, i, o);
  };
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n4; i += 2 * stride) {
    const long j = i + stride;
    const bool hj = j < n4;
    const float4 g0 = reinterpret_cast<const float4*>(dz)[i];
    const float4 v0 = ld4(y, i);
    const float4 z0 = MASK == 1 ? ld4(z, i) : g0;
    float4 g1 = g0, v1 = v0, z1 = z0;
    if (hj) {
      g1 = reinterpret_cast<const float4*>(dz)[j];
      v1 = ld4(y, j);
      if (MASK == 1) z1 = ld4(z, j);
    }
    apply(i, g0, v0, z0);
    if (hj) apply(j, g1, v1, z1);
  }
}

// The BatchNorm-backward apply of the bf16-activation step, 8 elements per thread: g (fp32, already
// ReLU-masked by the fused dgrad epilogue) 32 B, y (bf16) 16 B, dy (bf16) 16 B -- every access a
// 16-B lane piece (the 4-wide form moved bf16 in 8-B pieces).  Same fmaf sequence as bn_bwd_apply.
// TG: float, or __bf16 when g was stored bf16 by a TMR_IO_G16 dgrad (16 B of g per thread)
__device__ __forceinline__ void ld_g8(const float* g, long i, float4& a, float4& b) {
  a = reinterpret_cast<const float4*>(g)[2 * i];
  b = reinterpret_cast<const float4*>(g)[2 * i + 1];
}
__device__ __forceinline__ void ld_g8(const __bf16* g, long i, float4& a, float4& b) {
  const uint4 w = reinterpret_cast<const uint4*>(g)[i];
  a = make_float4(__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                  __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u));
  b = make_float4(__uint_as_float(w.z << 16), __uint_as_float(w.z & 0xffff0000u),
                  __uint_as_float(w.w << 16), __uint_as_float(w.w & 0xffff0000u));
}
template <typename TG = float>
__global__ __launch_bounds__(NT) void bn_bwd_apply8_a16(const TG* __restrict__ g,
                                                        const __bf16* __restrict__ y,
                                                        const float* __restrict__ coef,
                                                        __bf16* __restrict__ dy, long n8, int c8) {
  const int c = c8 * 8;
  const long stride = (long)gridDim.x * NT;
  auto apply = [&](long i, const float4 g0, const float4 g1, const uint4 yw) {
    const int cc = chan_of(i, c8) * 8;
    const float gv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    const uint32_t yu[4] = {yw.x, yw.y, yw.z, yw.w};
    float yv[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      yv[2 * e] = __uint_as_float(yu[e] << 16);
      yv[2 * e + 1] = __uint_as_float(yu[e] & 0xffff0000u);
    }
    uint32_t ow[4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float4 A = *reinterpret_cast<const float4*>(coef + cc + 4 * h);
      const float4 B = *reinterpret_cast<const float4*>(coef + c + cc + 4 * h);
      const float4 C = *reinterpret_cast<const float4*>(coef + 2 * c + cc + 4 * h);
      const float o0 = fmaf(A.x, gv[4 * h], fmaf(B.x, yv[4 * h], C.x));
      const float o1 = fmaf(A.y, gv[4 * h + 1], fmaf(B.y, yv[4 * h + 1], C.y));
      const float o2 = fmaf(A.z, gv[4 * h + 2], fmaf(B.z, yv[4 * h + 2], C.z));
      const float o3 = fmaf(A.w, gv[4 * h + 3], fmaf(B.w, yv[4 * h + 3], C.w));
      typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
      const bf16x2_t p = {(__bf16)o0, (__bf16)o1}, q = {(__bf16)o2, (__bf16)o3};
      ow[2 * h] = __builtin_bit_cast(uint32_t, p);
      ow[2 * h + 1] = __builtin_bit_cast(uint32_t, q);
    }
    reinterpret_cast<uint4*>(dy)[i] = make_uint4(ow[0], ow[1], ow[2], ow[3]);
  };
  // two elements in flight per thread (bn_bwd_apply)
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n8; i += 2 * stride) {
    const long j = i + stride;
    const bool hj = j < n8;
    float4 a0, a1;
    ld_g8(g, i, a0, a1);
    const uint4 ya = reinterpret_cast<const uint4*>(y)[i];
    float4 b0 = a0, b1 = a1;
    uint4 yb = ya;
    if (hj) {
      ld_g8(g, j, b0, b1);
      yb = reinterpret_cast<const uint4*>(y)[j];
    }
    apply(i, a0, a1, ya);
    if (hj) apply(j, b0, b1, yb);
  }
}

// ---- per-channel reductions of the GEMM-epilogue partials, two levels ----------------------
// The conv epilogues leave one partial row per m-tile ([nparts][c]; up to ~31k rows for the
// 64x64-tile dgrads of layer1).  Level 1: a (channel-group x row-slab) grid, 64 channels x 4
// row phases per block, coalesced 1-KB rows, double accumulators -> slab sums in ws.  Level 2:
// one block per channel group, 4 slab phases per channel combined in a fixed order
// (deterministic), then the BN math.
constexpr int SLAB_CH = 64;

struct SlabPlan {
  int groups, nslabs, rows;
};

SlabPlan slab_plan(int nparts, int c) {
  SlabPlan p;
  p.groups = cdiv(c, SLAB_CH);
  int target = 512 / p.groups;
  if (target < 1) target = 1;
  int r = cdiv(nparts, 32);
  if (r > target) r = target;
  if (r < 1) r = 1;
  p.rows = cdiv(nparts, r);
  p.nslabs = cdiv(nparts, p.rows);
  return p;
}

size_t slab_ws_bytes(int nparts, int c) {
  const SlabPlan p = slab_plan(nparts, c);
  return (size_t)p.nslabs * 3 * c * sizeof(double);
}

// KIND 0: float4 (count, mean, M2, -) partials -> (N, S1, S2) about K = the first partial's mean
// KIND 1: float2 (sum g, sum g*(y-mean)) partials -> (S, Q, -)
template <int KIND>
__global__ __launch_bounds__(256) void parts_slab_k(const void* __restrict__ part, int nparts, int c,
                                                    int rows, double* __restrict__ ws) {
  const int ch = blockIdx.x * SLAB_CH + (threadIdx.x & (SLAB_CH - 1));
  const int ph = threadIdx.x / SLAB_CH;
  const int b0 = blockIdx.y * rows;
  const int b1 = min(nparts, b0 + rows);
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;
  if (ch < c) {
    if (KIND == 0) {
      const float4* p = (const float4*)part;
      const double K = p[ch].y;
      for (int b = b0 + ph; b < b1; b += 4) {
        const float4 v = p[(long)b * c + ch];
        const double nb = v.x, d = (double)v.y - K;
        a0 += nb;
        a1 = fma(nb, d, a1);
        a2 += (double)v.z + nb * d * d;
      }
    } else {
      const float2* p = (const float2*)part;
      for (int b = b0 + ph; b < b1; b += 4) {
        const float2 v = p[(long)b * c + ch];
        a0 += v.x;
        a1 += v.y;
      }
    }
  }
  __shared__ double red[3][256];
  red[0][threadIdx.x] = a0; red[1][threadIdx.x] = a1; red[2][threadIdx.x] = a2;
  __syncthreads();
  if (ph == 0 && ch < c) {
    double t0 = 0.0, t1 = 0.0, t2 = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      t0 += red[0][q * SLAB_CH + threadIdx.x];
      t1 += red[1][q * SLAB_CH + threadIdx.x];
      t2 += red[2][q * SLAB_CH + threadIdx.x];
    }
    double* w = ws + (long)blockIdx.y * 3 * c;
    w[ch] = t0; w[c + ch] = t1; w[2 * c + ch] = t2;
  }
}

// sum of the slab partials of channel group blockIdx.x: SLAB_PH slab phases per channel (a
// 64 x SLAB_PH block), combined in phase order; true on the one thread per channel holding the totals
constexpr int SLAB_PH = 16;
template <int NV>
__device__ __forceinline__ bool slab_sum(const double* __restrict__ ws, int nslabs, int c, int& ch,
                                         double (&t)[3]) {
  ch = blockIdx.x * SLAB_CH + (threadIdx.x & (SLAB_CH - 1));
  const int ph = threadIdx.x / SLAB_CH;
  double a[3] = {0.0, 0.0, 0.0};
  if (ch < c)
    for (int r = ph; r < nslabs; r += SLAB_PH) {
      const double* w = ws + (long)r * 3 * c;
#pragma unroll
      for (int j = 0; j < NV; ++j) a[j] += w[j * c + ch];
    }
  __shared__ double red[3][SLAB_CH * SLAB_PH];
#pragma unroll
  for (int j = 0; j < 3; ++j) red[j][threadIdx.x] = a[j];
  __syncthreads();
  if (ph != 0 || ch >= c) return false;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    t[j] = 0.0;
#pragma unroll
    for (int q = 0; q < SLAB_PH; ++q) t[j] += red[j][q * SLAB_CH + threadIdx.x];
  }
  return true;
}

__global__ __launch_bounds__(SLAB_CH * SLAB_PH) void finalize_slabs_k(const double* __restrict__ ws, int nslabs,
                                                        const float4* __restrict__ part, int c,
                                                        const float* gamma, const float* beta,
                                                        float* rmean, float* rvar, float momentum,
                                                        float eps, float* smean, float* sinv,
                                                        float* scale, float* shift) {
  int ch;
  double t[3];
  if (!slab_sum<3>(ws, nslabs, c, ch, t)) return;
  const double n = t[0], s1 = t[1], s2 = t[2];
  const double K = part[ch].y;
  const double mean = n > 0 ? K + s1 / n : 0.0;
  double m2 = n > 0 ? s2 - s1 * (s1 / n) : 0.0;
  if (m2 < 0) m2 = 0;
  const double var = n > 0 ? m2 / n : 0.0;
  const double inv = 1.0 / sqrt(var + (double)eps);
  smean[ch] = (float)mean;
  sinv[ch] = (float)inv;
  const double gm = gamma ? gamma[ch] : 1.0;
  const double bt = beta ? beta[ch] : 0.0;
  scale[ch] = (float)(gm * inv);
  shift[ch] = (float)(bt - mean * gm * inv);
  if (rmean) {
    const double unb = n > 1 ? m2 / (n - 1.0) : var;
    rmean[ch] = (float)((1.0 - momentum) * rmean[ch] + momentum * mean);
    rvar[ch] = (float)((1.0 - momentum) * rvar[ch] + momentum * unb);
  }
}

__global__ __launch_bounds__(SLAB_CH * SLAB_PH) void bwd_final_slabs_k(const double* __restrict__ ws, int nslabs,
                                                         int rows, int c, const float* mean,
                                                         const float* inv, const float* gamma,
                                                         float* dgamma, float* dbeta, float* coef) {
  int ch;
  double t[3];
  if (!slab_sum<2>(ws, nslabs, c, ch, t)) return;
  const double s = t[0], q = t[1];
  const double iv = inv[ch];
  const double dbt = s;
  const double dgm = q * iv;  // sum dzh * xhat
  if (dgamma) dgamma[ch] = (float)dgm;
  if (dbeta) dbeta[ch] = (float)dbt;
  const double n = (double)rows;
  const double gm = gamma ? gamma[ch] : 1.0;
  const double A = gm * iv;
  const double mdz = dbt / n, mdx = dgm / n;
  const double B = -gm * iv * iv * mdx;
  const double C = -A * mdz - B * (double)mean[ch];
  coef[ch] = (float)A;
  coef[c + ch] = (float)B;
  coef[2 * c + ch] = (float)C;
}

// share.maxpool -> share.relu -> share.bn1 backward in two passes (the stem: pre-BN output y
// (rows = n*h*w pixels), ReLU mask recomputed from y*scale+shift, dz gathered from the pooled
// gradient -- neither dz nor the maxpool's input gradient is ever written)
struct PoolGeo {
  const float* dyp;
  const uchar4* am;
  FastDiv dHW, dW;
  int ho, wo;
};

__device__ __forceinline__ float4 stem_dz(const PoolGeo& pg, uint32_t r, int cq, int c4) {
  const uint32_t nn = fdiv(r, pg.dHW);
  const uint32_t rem = r - nn * pg.dHW.d;
  const uint32_t iy = fdiv(rem, pg.dW);
  const uint32_t ix = rem - iy * pg.dW.d;
  return maxpool_grad4(pg.dyp, pg.am, (int)nn, (int)iy, (int)ix, cq, c4, pg.ho, pg.wo);
}

// Partial sums from the pooled side: every pooled output passes its gradient to exactly one
// input pixel per channel (its argmax), so sum g and sum g*(y - mean) over the input pixels equal
// the sums over pooled outputs of dyp * mask(y[argmax]) and that times (y[argmax] - mean): one
// read of the pooled gradient and argmax plus one y element per channel, no gather of windows.
template <typename TY = float>
__global__ __launch_bounds__(NT) void stem_bwd_partial_pooled(
    const PoolGeo pg, int h, int w, const TY* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ mean, int prows, int c, int rpb,
    int cthreads, FastDiv dPHW, FastDiv dPW, double* __restrict__ part) {
  const int tc = threadIdx.x % cthreads, tr = threadIdx.x / cthreads;
  const int rthreads = NT / cthreads;
  const int ch = (blockIdx.y * cthreads + tc) * 4;
  const float mu[4] = {mean[ch], mean[ch + 1], mean[ch + 2], mean[ch + 3]};
  const float sc[4] = {scale[ch], scale[ch + 1], scale[ch + 2], scale[ch + 3]};
  const float sf[4] = {shift[ch], shift[ch + 1], shift[ch + 2], shift[ch + 3]};
  const int c4 = c / 4;
  const int r0 = blockIdx.x * rpb;
  const int r1 = min(prows, r0 + rpb);
  float s[4] = {0.f, 0.f, 0.f, 0.f}, q[4] = {0.f, 0.f, 0.f, 0.f};
  for (int r = r0 + tr; r < r1; r += rthreads) {
    const uint32_t nn = fdiv((uint32_t)r, dPHW);
    const uint32_t rem = r - nn * dPHW.d;
    const uint32_t oy = fdiv(rem, dPW);
    const uint32_t ox = rem - oy * dPW.d;
    const long o = (long)r * c4 + ch / 4;
    const uchar4 a = pg.am[o];
    const float4 d = reinterpret_cast<const float4*>(pg.dyp)[o];
    const unsigned char ids[4] = {a.x, a.y, a.z, a.w};
    const float ds[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int iy = (int)oy * 2 - 1 + ids[e] / 3, ix = (int)ox * 2 - 1 + ids[e] % 3;
      const float v = ld1(y, (((long)nn * h + iy) * w + ix) * c + ch + e);
      const float g = fmaf(v, sc[e], sf[e]) > 0.f ? ds[e] : 0.f;
      s[e] += g;
      q[e] = fmaf(g, v - mu[e], q[e]);
    }
  }
  __shared__ double red[NT][8];
  for (int e = 0; e < 4; ++e) {
    red[threadIdx.x][e] = s[e];
    red[threadIdx.x][4 + e] = q[e];
  }
  __syncthreads();
  if (tr == 0) {
    double acc[8];
    for (int e = 0; e < 8; ++e) acc[e] = 0.0;
    for (int k = 0; k < rthreads; ++k)
      for (int e = 0; e < 8; ++e) acc[e] += red[k * cthreads + tc][e];
    double* op = part + ((long)blockIdx.x * c + ch) * 2;
    for (int e = 0; e < 4; ++e) {
      op[2 * e] = acc[e];
      op[2 * e + 1] = acc[4 + e];
    }
  }
}

template <typename TD, typename TY = float>
__global__ __launch_bounds__(NT) void stem_bwd_apply(const PoolGeo pg, const TY* __restrict__ y,
                                                     const float* __restrict__ scale,
                                                     const float* __restrict__ shift,
                                                     const float* __restrict__ coef,
                                                     TD* __restrict__ dy, long n4, int c4) {
  const int c = c4 * 4;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n4; i += (long)gridDim.x * NT) {
    const int cq = chan_of(i, c4);
    const int cc = cq * 4;
    const float4 v = ld4(y, i);
    // (c4 a power of two -- the stem's 64 channels -- divides by a shift, not a 64-bit division)
    const uint32_t row = (c4 & (c4 - 1)) == 0 ? (uint32_t)(i >> __builtin_ctz(c4)) : (uint32_t)(i / c4);
    const float4 g = relu_mask4(stem_dz(pg, row, cq, c4),
                                affine4(v, *reinterpret_cast<const float4*>(scale + cc),
                                        *reinterpret_cast<const float4*>(shift + cc)));
    const float4 A = *reinterpret_cast<const float4*>(coef + cc);
    const float4 B = *reinterpret_cast<const float4*>(coef + c + cc);
    const float4 C = *reinterpret_cast<const float4*>(coef + 2 * c + cc);
    float4 o;
    o.x = fmaf(A.x, g.x, fmaf(B.x, v.x, C.x));
    o.y = fmaf(A.y, g.y, fmaf(B.y, v.y, C.y));
    o.z = fmaf(A.z, g.z, fmaf(B.z, v.z, C.z));
    o.w = fmaf(A.w, g.w, fmaf(B.w, v.w, C.w));
    st4(dy, i, o);
  }
}


// 8 consecutive elements (index i in units of 8) of an fp32 or bf16 tensor, as fp32 values
template <typename T>
__device__ __forceinline__ void ld8(const T* p, long i, float (&v)[8]);
template <>
__device__ __forceinline__ void ld8<float>(const float* p, long i, float (&v)[8]) {
  const float4 a = reinterpret_cast<const float4*>(p)[2 * i], b = reinterpret_cast<const float4*>(p)[2 * i + 1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
template <>
__device__ __forceinline__ void ld8<__bf16>(const __bf16* p, long i, float (&v)[8]) {
  const uint4 w = reinterpret_cast<const uint4*>(p)[i];
  const uint32_t u[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[2 * e] = __uint_as_float(u[e] << 16);
    v[2 * e + 1] = __uint_as_float(u[e] & 0xffff0000u);
  }
}
template <typename T>
__device__ __forceinline__ void st8(T* p, long i, const float (&v)[8]);
template <>
__device__ __forceinline__ void st8<float>(float* p, long i, const float (&v)[8]) {
  reinterpret_cast<float4*>(p)[2 * i] = make_float4(v[0], v[1], v[2], v[3]);
  reinterpret_cast<float4*>(p)[2 * i + 1] = make_float4(v[4], v[5], v[6], v[7]);
}
template <>
__device__ __forceinline__ void st8<__bf16>(__bf16* p, long i, const float (&v)[8]) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  uint32_t w[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const bf16x2_t q = {(__bf16)v[2 * e], (__bf16)v[2 * e + 1]};
    w[e] = __builtin_bit_cast(uint32_t, q);
  }
  reinterpret_cast<uint4*>(p)[i] = make_uint4(w[0], w[1], w[2], w[3]);
}
// The BatchNorm-backward apply with g already masked (MASK 0; tmr_bn_bwd_parts), 8 elements per
// thread, two groups in flight: the fp32 step's form of bn_bwd_apply8_a16 (64 B of g and y per
// group instead of 32; round 6).  Same fmaf sequence per element as bn_bwd_apply: identical dy.
template <typename TG, typename TY, typename TD>
__global__ __launch_bounds__(NT) void bn_bwd_apply8_k(const TG* __restrict__ g,
                                                      const TY* __restrict__ y,
                                                      const float* __restrict__ coef,
                                                      TD* __restrict__ dy, long n8, int c8) {
  const int c = c8 * 8;
  const long stride = (long)gridDim.x * NT;
  auto apply = [&](long i, const float (&gv)[8], const float (&yv)[8]) {
    const int cc = chan_of(i, c8) * 8;
    float o[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float4 A = *reinterpret_cast<const float4*>(coef + cc + 4 * h);
      const float4 B = *reinterpret_cast<const float4*>(coef + c + cc + 4 * h);
      const float4 C = *reinterpret_cast<const float4*>(coef + 2 * c + cc + 4 * h);
      o[4 * h] = fmaf(A.x, gv[4 * h], fmaf(B.x, yv[4 * h], C.x));
      o[4 * h + 1] = fmaf(A.y, gv[4 * h + 1], fmaf(B.y, yv[4 * h + 1], C.y));
      o[4 * h + 2] = fmaf(A.z, gv[4 * h + 2], fmaf(B.z, yv[4 * h + 2], C.z));
      o[4 * h + 3] = fmaf(A.w, gv[4 * h + 3], fmaf(B.w, yv[4 * h + 3], C.w));
    }
    st8(dy, i, o);
  };
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n8; i += 2 * stride) {
    const long j = i + stride;
    const bool hj = j < n8;
    float ga[8], ya[8], gb[8], yb[8];
    ld8(g, i, ga);
    ld8(y, i, ya);
    if (hj) {
      ld8(g, j, gb);
      ld8(y, j, yb);
    }
    apply(i, ga, ya);
    if (hj) apply(j, gb, yb);
  }
}

// The same per 2x2 quad of input pixels (rows 2k, 2k+1, columns 2l, 2l+1): the pooled outputs
// (k .. k+1) x (l .. l+1) are the candidates of all four pixels, so each is loaded once per quad
// -- one pooled load per pixel instead of 2.25 (the launch is bound by those gathered bytes).
// Pixel (py, px) of the quad sums candidate (dy, dx) when (dy <= py, dx <= px, in range) with
// id = (py + 1 - 2dy) * 3 + (px + 1 - 2dx), in the order (0,0), (0,1), (1,0), (1,1): the
// per-pixel kernels' order, so bit-identical.  nq = n * ceil(h/2) * ceil(w/2) * c/8 < 2^31.
// TY / TD: y and dy fp32 or bf16 (round 5: the fp32 step's stem too).
template <typename TY, typename TD>
__global__ __launch_bounds__(NT) void stem_bwd_apply8q(const PoolGeo pg, int h, int w, FastDiv dQHW,
                                                       FastDiv dQW, const TY* __restrict__ y,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift,
                                                       const float* __restrict__ coef,
                                                       TD* __restrict__ dy, int nq, int lc8) {
  const int c8 = 1 << lc8, c = c8 * 8;
  const uint2* am = reinterpret_cast<const uint2*>(pg.am);
  const float4* dp = reinterpret_cast<const float4*>(pg.dyp);
  for (int i = blockIdx.x * NT + threadIdx.x; i < nq; i += gridDim.x * NT) {
    const int cq = i & (c8 - 1);
    const uint32_t q = (uint32_t)i >> lc8;
    const uint32_t nn = fdiv(q, dQHW);
    const uint32_t rem = q - nn * dQHW.d;
    const int k = (int)fdiv(rem, dQW), l = (int)(rem - (uint32_t)k * dQW.d);
    const bool pin[2][2] = {{true, l + 1 < pg.wo}, {k + 1 < pg.ho, k + 1 < pg.ho && l + 1 < pg.wo}};
    uint2 a[2][2];
    float4 d0[2][2], d1[2][2];
#pragma unroll
    for (int ddy = 0; ddy < 2; ++ddy)
#pragma unroll
      for (int ddx = 0; ddx < 2; ++ddx) {
        const int o = (((int)nn * pg.ho + k + ddy) * pg.wo + l + ddx) * c8 + cq;
        if (pin[ddy][ddx]) {
          a[ddy][ddx] = am[o];
          d0[ddy][ddx] = dp[2 * (long)o];       // 64-bit: o < 2^31 is checked, 2 o is not
          d1[ddy][ddx] = dp[2 * (long)o + 1];
        } else {
          a[ddy][ddx] = make_uint2(0xffffffffu, 0xffffffffu);
          d0[ddy][ddx] = d1[ddy][ddx] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    float sc[8], sf[8], A[8], B[8], C[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sc[e] = scale[cq * 8 + e];
      sf[e] = shift[cq * 8 + e];
      A[e] = coef[cq * 8 + e];
      B[e] = coef[c + cq * 8 + e];
      C[e] = coef[2 * c + cq * 8 + e];
    }
#pragma unroll
    for (int py = 0; py < 2; ++py)
#pragma unroll
      for (int px = 0; px < 2; ++px) {
        const int iy = 2 * k + py, ix = 2 * l + px;
        if (iy >= h || ix >= w) continue;
        const long pix = ((long)nn * h + iy) * w + ix;
        float v[8], g[8];
        ld8(y, pix * c8 + cq, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = 0.f;
#pragma unroll
        for (int ddy = 0; ddy < 2; ++ddy)
#pragma unroll
          for (int ddx = 0; ddx < 2; ++ddx) {
            if (ddy > py || ddx > px || !pin[ddy][ddx]) continue;
            const uint32_t id = (uint32_t)((py + 1 - 2 * ddy) * 3 + (px + 1 - 2 * ddx));
            const float dv[8] = {d0[ddy][ddx].x, d0[ddy][ddx].y, d0[ddy][ddx].z, d0[ddy][ddx].w,
                                 d1[ddy][ddx].x, d1[ddy][ddx].y, d1[ddy][ddx].z, d1[ddy][ddx].w};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const uint32_t ab = ((e < 4 ? a[ddy][ddx].x : a[ddy][ddx].y) >> (8 * (e & 3))) & 0xffu;
              if (ab == id) g[e] += dv[e];
            }
          }
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float gm = fmaf(v[e], sc[e], sf[e]) > 0.f ? g[e] : 0.f;
          o[e] = fmaf(A[e], gm, fmaf(B[e], v[e], C[e]));
        }
        st8(dy, pix * c8 + cq, o);
      }
  }
}

// The forward BN + ReLU with the ReLU mask as bits (bn_apply_bits_k's fp32 forms: RES the residual
// add, yr the downsample branch's BN on the fly), 8 elements per thread and two groups in flight
// per thread, each group's 8 mask bits one byte of its word (round 6: the 4-wide form moved its
// 12 B per element at 4.8 TB/s, the 8-wide BN passes at 5.6-5.9).  Same arithmetic per element:
// z and the bits identical to bn_apply_bits_k's.  The loop runs whole waves (the bit words are
// gathered across 4 lanes).
#ifndef TMR_BN_BITS8
#define TMR_BN_BITS8 1   // 0: the 4-wide form only (A/B build)
#endif
template <bool RES>
__global__ __launch_bounds__(NT) void bn_apply_bits8_k(const float* __restrict__ y,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift,
                                                       const float* __restrict__ res,
                                                       const float* __restrict__ yr,
                                                       const float* __restrict__ rscale,
                                                       const float* __restrict__ rshift,
                                                       float* __restrict__ z,
                                                       uint32_t* __restrict__ bits, long n8, int c8) {
  const int lane = threadIdx.x & 63;
  const long stride = (long)gridDim.x * NT;
  // one group: z of elements 8i .. 8i + 7 and their mask byte
  auto apply = [&](long i, const float (&yv)[8], const float (&rv)[8]) -> uint32_t {
    const int cc = chan_of(i, c8) * 8;
    float v[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float4 sc = *reinterpret_cast<const float4*>(scale + cc + 4 * h);
      const float4 sf = *reinterpret_cast<const float4*>(shift + cc + 4 * h);
      const float s4[4] = {sc.x, sc.y, sc.z, sc.w}, f4[4] = {sf.x, sf.y, sf.z, sf.w};
      if (yr) {
        const float4 rs = *reinterpret_cast<const float4*>(rscale + cc + 4 * h);
        const float4 rf = *reinterpret_cast<const float4*>(rshift + cc + 4 * h);
        const float r4[4] = {rs.x, rs.y, rs.z, rs.w}, q4[4] = {rf.x, rf.y, rf.z, rf.w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          v[4 * h + e] = fmaf(yv[4 * h + e], s4[e], f4[e]) + fmaf(rv[4 * h + e], r4[e], q4[e]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[4 * h + e] = fmaf(yv[4 * h + e], s4[e], f4[e]);
          if (RES) v[4 * h + e] += rv[4 * h + e];
        }
      }
    }
    uint32_t b = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] = fmaxf(v[e], 0.f);
      b |= (uint32_t)(v[e] > 0.f) << e;
    }
    st8(z, i, v);
    return b;
  };
  // the word of 4 lanes' bytes (group indices 4k .. 4k + 3: base is a multiple of 64)
  auto put = [&](uint32_t byte, long i, bool ok) {
    uint32_t w = byte << (8 * (lane & 3));
    w |= (uint32_t)__shfl_xor((int)w, 1, 64);
    w |= (uint32_t)__shfl_xor((int)w, 2, 64);
    if ((lane & 3) == 0 && ok) bits[i >> 2] = w;
  };
  const float* rsrc = RES ? res : yr;
  for (long base = blockIdx.x * (long)NT + (threadIdx.x & ~63); base < n8; base += 2 * stride) {
    const long i = base + lane, j = i + stride;
    const bool oi = i < n8, oj = j < n8;
    float ya[8], ra[8], yb[8], rb[8];
    if (oi) {
      ld8(y, i, ya);
      if (rsrc) ld8(rsrc, i, ra);
    }
    if (oj) {
      ld8(y, j, yb);
      if (rsrc) ld8(rsrc, j, rb);
    }
    const uint32_t bi = oi ? apply(i, ya, ra) : 0u;
    const uint32_t bj = oj ? apply(j, yb, rb) : 0u;
    put(bi, i, oi);
    put(bj, j, oj);
  }
}

int ew_blocks(long n4) {
  long b = (n4 + NT - 1) / NT;
  if (b > 2048 * 4) b = 2048 * 4;
  return (int)(b > 0 ? b : 1);
}

}  // namespace

TMR_API size_t tmr_bn_ws_bytes(int rows, int c) {
  if (rows <= 0 || c < 4 || c % 4) {
    tmr_set_error("tmr_bn_ws_bytes: bad size (rows %d, channels %d)", rows, c);
    return 0;
  }
  return ws_need(rows, c);
}

TMR_API int tmr_bn_fwd_stats(const float* y, int rows, int c, const float* gamma,
                             const float* beta, float* running_mean, float* running_var,
                             float momentum, float eps, float* save_mean, float* save_invstd,
                             float* scale, float* shift, void* ws, size_t ws_bytes,
                             hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0 && c >= 4, "tmr_bn_fwd_stats: channels %d must be a multiple of 4", c);
  TMR_CHECK_ARG(rows > 0, "tmr_bn_fwd_stats: empty input");
  TMR_CHECK_ARG(ws && ws_bytes >= ws_need(rows, c), "tmr_bn_fwd_stats: workspace too small");
  Plan p = make_plan(rows, c);
  TMR_CHECK_ARG((c / 4) % p.cthreads == 0, "tmr_bn_fwd_stats: unsupported channel count %d", c);
  float4* part = (float4*)ws;
  hipLaunchKernelGGL(bn_stats_partial, dim3(p.nrb, p.cblocks), dim3(NT), 0, stream, y, rows, c,
                     p.rpb, p.cthreads, part);
  TMR_CHECK_LAUNCH("bn_stats_partial");
  return tmr_bn_finalize(part, p.nrb, c, gamma, beta, running_mean, running_var, momentum, eps,
                         save_mean, save_invstd, scale, shift, stream);
}

TMR_API int tmr_bn_finalize(const void* partials, int nparts, int c, const float* gamma,
                            const float* beta, float* running_mean, float* running_var,
                            float momentum, float eps, float* save_mean, float* save_invstd,
                            float* scale, float* shift, hipStream_t stream) {
  TMR_CHECK_ARG(nparts > 0 && c > 0, "tmr_bn_finalize: empty partials");
  hipLaunchKernelGGL(bn_finalize_k, dim3(c), dim3(NT), 0, stream, (const float4*)partials,
                     nparts, c, gamma, beta, running_mean, running_var, momentum, eps, save_mean,
                     save_invstd, scale, shift);
  TMR_CHECK_LAUNCH("bn_finalize");
  return 0;
}

TMR_API size_t tmr_bn_parts_ws_bytes(int nparts, int c) {
  if (nparts <= 0 || c <= 0) {
    tmr_set_error("tmr_bn_parts_ws_bytes: bad size (parts %d, channels %d)", nparts, c);
    return 0;
  }
  return slab_ws_bytes(nparts, c) + (size_t)3 * c * sizeof(float) + 64;
}

TMR_API int tmr_bn_finalize_ws(const void* partials, int nparts, int c, const float* gamma,
                               const float* beta, float* running_mean, float* running_var,
                               float momentum, float eps, float* save_mean, float* save_invstd,
                               float* scale, float* shift, void* ws, size_t ws_bytes,
                               hipStream_t stream) {
  TMR_CHECK_ARG(nparts > 0 && c > 0, "tmr_bn_finalize_ws: empty partials");
  TMR_CHECK_ARG(ws && ws_bytes >= slab_ws_bytes(nparts, c), "tmr_bn_finalize_ws: workspace too small");
  const SlabPlan p = slab_plan(nparts, c);
  hipLaunchKernelGGL(parts_slab_k<0>, dim3(p.groups, p.nslabs), dim3(256), 0, stream, partials,
                     nparts, c, p.rows, (double*)ws);
  TMR_CHECK_LAUNCH("bn_parts_slab");
  hipLaunchKernelGGL(finalize_slabs_k, dim3(p.groups), dim3(SLAB_CH * SLAB_PH), 0, stream,
                     (const double*)ws, p.nslabs, (const float4*)partials, c, gamma, beta,
                     running_mean, running_var, momentum, eps, save_mean, save_invstd, scale,
                     shift);
  TMR_CHECK_LAUNCH("bn_finalize_slabs");
  return 0;
}

TMR_API int tmr_bn_eval_params(const float* gamma, const float* beta, const float* running_mean,
                               const float* running_var, float eps, int c, float* scale,
                               float* shift, hipStream_t stream) {
  hipLaunchKernelGGL(bn_eval_params_k, dim3(cdiv(c, 256)), dim3(256), 0, stream, gamma, beta,
                     running_mean, running_var, eps, c, scale, shift);
  TMR_CHECK_LAUNCH("bn_eval_params");
  return 0;
}

TMR_API int tmr_bn_apply(const float* y, const float* scale, const float* shift,
                         const float* residual, float* z, int rows, int c, int relu,
                         hipStream_t stream) {
  return tmr_bn_apply_x(y, scale, shift, residual, z, rows, c, relu, 0, stream);
}

TMR_API int tmr_bn_apply_x(const float* y, const float* scale, const float* shift,
                           const float* residual, void* zv, int rows, int c, int relu,
                           int out_bf16, hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0, "tmr_bn_apply: channels %d must be a multiple of 4", c);
  long n4 = (long)rows * c / 4;
  int nb = ew_blocks(n4);
  int c4 = c / 4;
  if (out_bf16) {
    TMR_CHECK_ARG(!residual, "tmr_bn_apply_x: a bf16 output is for conv-operand-only tensors (no residual)");
    if (relu) hipLaunchKernelGGL((bn_apply_k<false, true, __bf16>), dim3(nb), dim3(NT), 0, stream, y, scale, shift, residual, (__bf16*)zv, n4, c4);
    else hipLaunchKernelGGL((bn_apply_k<false, false, __bf16>), dim3(nb), dim3(NT), 0, stream, y, scale, shift, residual, (__bf16*)zv, n4, c4);
    TMR_CHECK_LAUNCH("bn_apply");
    return 0;
  }
  float* z = (float*)zv;
  if (residual) {
    if (relu) hipLaunchKernelGGL((bn_apply_k<true, true>), dim3(nb), dim3(NT), 0, stream, y, scale, shift, residual, z, n4, c4);
    else hipLaunchKernelGGL((bn_apply_k<true, false>), dim3(nb), dim3(NT), 0, stream, y, scale, shift, residual, z, n4, c4);
  } else {
    if (relu) hipLaunchKernelGGL((bn_apply_k<false, true>), dim3(nb), dim3(NT), 0, stream, y, scale, shift, residual, z, n4, c4);
    else hipLaunchKernelGGL((bn_apply_k<false, false>), dim3(nb), dim3(NT), 0, stream, y, scale, shift, residual, z, n4, c4);
  }
  TMR_CHECK_LAUNCH("bn_apply");
  return 0;
}

TMR_API int tmr_bn_apply2(const float* y, const float* scale, const float* shift, const float* yr,
                          const float* rscale, const float* rshift, float* z, int rows, int c,
                          int relu, hipStream_t stream) {
  return tmr_bn_apply2_x(y, scale, shift, yr, rscale, rshift, z, nullptr, rows, c, relu, stream);
}

TMR_API int tmr_bn_apply2_x(const float* y, const float* scale, const float* shift, const float* yr,
                            const float* rscale, const float* rshift, float* z, void* z16,
                            int rows, int c, int relu, hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0, "tmr_bn_apply2: channels %d must be a multiple of 4", c);
  TMR_CHECK_ARG(y && scale && shift && yr && rscale && rshift && z, "tmr_bn_apply2: null operand");
  TMR_CHECK_ARG(yr != z, "tmr_bn_apply2: the branch input must not alias z");
  const long n4 = (long)rows * c / 4;
  __bf16* h = (__bf16*)z16;
  if (relu && h)
    hipLaunchKernelGGL((bn_apply2_k<true, true>), dim3(ew_blocks(n4)), dim3(NT), 0, stream, y, scale,
                       shift, yr, rscale, rshift, z, n4, c / 4, h);
  else if (relu)
    hipLaunchKernelGGL((bn_apply2_k<true>), dim3(ew_blocks(n4)), dim3(NT), 0, stream, y, scale, shift,
                       yr, rscale, rshift, z, n4, c / 4, h);
  else if (h)
    hipLaunchKernelGGL((bn_apply2_k<false, true>), dim3(ew_blocks(n4)), dim3(NT), 0, stream, y, scale,
                       shift, yr, rscale, rshift, z, n4, c / 4, h);
  else
    hipLaunchKernelGGL((bn_apply2_k<false>), dim3(ew_blocks(n4)), dim3(NT), 0, stream, y, scale, shift,
                       yr, rscale, rshift, z, n4, c / 4, h);
  TMR_CHECK_LAUNCH("bn_apply2");
  return 0;
}

TMR_API int tmr_bn_apply_bits(const float* y, const float* scale, const float* shift,
                              const float* residual, float* z, uint32_t* bits, int rows, int c,
                              hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0 && y && scale && shift && z && bits,
                "tmr_bn_apply_bits: null operand or channels %d not a multiple of 4", c);
  const long n4 = (long)rows * c / 4;
  if (n4 == 0) return 0;
  if (TMR_BN_BITS8 && c % 8 == 0 && (((uintptr_t)y | (uintptr_t)residual | (uintptr_t)z) & 15) == 0) {
    if (residual)
      hipLaunchKernelGGL((bn_apply_bits8_k<true>), dim3(ew_blocks(n4 / 2)), dim3(NT), 0, stream, y,
                         scale, shift, residual, nullptr, nullptr, nullptr, z, bits, n4 / 2, c / 8);
    else
      hipLaunchKernelGGL((bn_apply_bits8_k<false>), dim3(ew_blocks(n4 / 2)), dim3(NT), 0, stream, y,
                         scale, shift, nullptr, nullptr, nullptr, nullptr, z, bits, n4 / 2, c / 8);
  } else if (residual)
    hipLaunchKernelGGL((bn_apply_bits_k<true, float>), dim3(ew_blocks(n4)), dim3(NT), 0, stream, y, scale,
                       shift, residual, nullptr, nullptr, nullptr, z, bits, n4, c / 4);
  else
    hipLaunchKernelGGL((bn_apply_bits_k<false, float>), dim3(ew_blocks(n4)), dim3(NT), 0, stream, y, scale,
                       shift, nullptr, nullptr, nullptr, nullptr, z, bits, n4, c / 4);
  TMR_CHECK_LAUNCH("bn_apply_bits");
  return 0;
}

TMR_API int tmr_bn_apply2_bits(const float* y, const float* scale, const float* shift,
                               const float* yr, const float* rscale, const float* rshift, float* z,
                               uint32_t* bits, int rows, int c, hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0 && y && scale && shift && yr && rscale && rshift && z && bits,
                "tmr_bn_apply2_bits: null operand or channels %d not a multiple of 4", c);
  TMR_CHECK_ARG(yr != z, "tmr_bn_apply2_bits: the branch input must not alias z");
  const long n4 = (long)rows * c / 4;
  if (n4 == 0) return 0;
  if (TMR_BN_BITS8 && c % 8 == 0 && (((uintptr_t)y | (uintptr_t)yr | (uintptr_t)z) & 15) == 0)
    hipLaunchKernelGGL((bn_apply_bits8_k<false>), dim3(ew_blocks(n4 / 2)), dim3(NT), 0, stream, y,
                       scale, shift, nullptr, yr, rscale, rshift, z, bits, n4 / 2, c / 8);
  else
    hipLaunchKernelGGL((bn_apply_bits_k<false, float>), dim3(ew_blocks(n4)), dim3(NT), 0, stream, y, scale,
                       shift, nullptr, yr, rscale, rshift, z, bits, n4, c / 4);
  TMR_CHECK_LAUNCH("bn_apply2_bits");
  return 0;
}

TMR_API int tmr_bn_apply_bits_a16(const void* y, const float* scale, const float* shift,
                                  const void* residual, void* z, uint32_t* bits, int rows, int c,
                                  hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0 && y && scale && shift && z && bits,
                "tmr_bn_apply_bits_a16: null operand or channels %d not a multiple of 4", c);
  const long n4 = (long)rows * c / 4;
  if (n4 == 0) return 0;
  const __bf16* yb = (const __bf16*)y;
  if (residual)
    hipLaunchKernelGGL((bn_apply_bits_k<true, __bf16>), dim3(ew_blocks(n4)), dim3(NT), 0, stream, yb,
                       scale, shift, (const __bf16*)residual, nullptr, nullptr, nullptr, (__bf16*)z,
                       bits, n4, c / 4);
  else
    hipLaunchKernelGGL((bn_apply_bits_k<false, __bf16>), dim3(ew_blocks(n4)), dim3(NT), 0, stream, yb,
                       scale, shift, nullptr, nullptr, nullptr, nullptr, (__bf16*)z, bits, n4, c / 4);
  TMR_CHECK_LAUNCH("bn_apply_bits_a16");
  return 0;
}

TMR_API int tmr_bn_apply2_bits_a16(const void* y, const float* scale, const float* shift,
                                   const void* yr, const float* rscale, const float* rshift,
                                   void* z, uint32_t* bits, int rows, int c, hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0 && y && scale && shift && yr && rscale && rshift && z && bits,
                "tmr_bn_apply2_bits_a16: null operand or channels %d not a multiple of 4", c);
  TMR_CHECK_ARG(yr != z, "tmr_bn_apply2_bits_a16: the branch input must not alias z");
  const long n4 = (long)rows * c / 4;
  if (n4 == 0) return 0;
  hipLaunchKernelGGL((bn_apply_bits_k<false, __bf16>), dim3(ew_blocks(n4)), dim3(NT), 0, stream,
                     (const __bf16*)y, scale, shift, nullptr, (const __bf16*)yr, rscale, rshift,
                     (__bf16*)z, bits, n4, c / 4);
  TMR_CHECK_LAUNCH("bn_apply2_bits_a16");
  return 0;
}

TMR_API int tmr_bn_apply_dual(const float* y, const float* scale, const float* shift,
                              const float* residual, float* z, void* z16, int rows, int c, int relu,
                              hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0, "tmr_bn_apply_dual: channels %d must be a multiple of 4", c);
  TMR_CHECK_ARG(y && scale && shift && z && z16, "tmr_bn_apply_dual: null operand");
  const long n4 = (long)rows * c / 4;
  const int nb = ew_blocks(n4), c4 = c / 4;
  __bf16* h = (__bf16*)z16;
  if (residual) {
    if (relu) hipLaunchKernelGGL((bn_apply_k<true, true, float, true>), dim3(nb), dim3(NT), 0, stream, y, scale, shift, residual, z, n4, c4, h);
    else hipLaunchKernelGGL((bn_apply_k<true, false, float, true>), dim3(nb), dim3(NT), 0, stream, y, scale, shift, residual, z, n4, c4, h);
  } else {
    if (relu) hipLaunchKernelGGL((bn_apply_k<false, true, float, true>), dim3(nb), dim3(NT), 0, stream, y, scale, shift, residual, z, n4, c4, h);
    else hipLaunchKernelGGL((bn_apply_k<false, false, float, true>), dim3(nb), dim3(NT), 0, stream, y, scale, shift, residual, z, n4, c4, h);
  }
  TMR_CHECK_LAUNCH("bn_apply_dual");
  return 0;
}

TMR_API int tmr_bn_bwd(const float* dz, const float* y, const float* z, const float* scale,
                       const float* shift, const float* save_mean, const float* save_invstd,
                       const float* gamma, float* dy, float* dres, float* dgamma, float* dbeta,
                       int rows, int c, int relu, void* ws, size_t ws_bytes, hipStream_t stream) {
  return tmr_bn_bwd_x(dz, y, z, scale, shift, save_mean, save_invstd, gamma, dy, dres, dgamma,
                      dbeta, rows, c, relu, ws, ws_bytes, 0, stream);
}

TMR_API int tmr_bn_bwd_x(const float* dz, const float* y, const float* z, const float* scale,
                         const float* shift, const float* save_mean, const float* save_invstd,
                         const float* gamma, void* dyv, float* dres, float* dgamma, float* dbeta,
                         int rows, int c, int relu, void* ws, size_t ws_bytes, int out_bf16,
                         hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0 && c >= 4, "tmr_bn_bwd: channels %d must be a multiple of 4", c);
  TMR_CHECK_ARG(rows > 0, "tmr_bn_bwd: empty input");
  TMR_CHECK_ARG(ws && ws_bytes >= ws_need(rows, c), "tmr_bn_bwd: workspace too small");
  TMR_CHECK_ARG(!relu || z || (scale && shift),
                "tmr_bn_bwd: relu backward needs the saved output z or the forward scale/shift");
  int mask = relu ? (z ? 1 : 2) : 0;
  Plan p = make_plan(rows, c);
  double* part = (double*)ws;
  float* coef = (float*)((char*)ws + (size_t)p.nrb * c * 2 * sizeof(double));
  const dim3 pg(p.nrb, p.cblocks);
  float* dzw = const_cast<float*>(dz);
  if (dres == dz) {
    // in-place identity-branch gradient: pass 1 masks dz itself, pass 2 reads it unmasked
    if (mask == 1)
      hipLaunchKernelGGL((bn_bwd_partial<1, true>), pg, dim3(NT), 0, stream, dzw, y, z, scale, shift, save_mean, rows, c, p.rpb, p.cthreads, part);
    else if (mask == 2)
      hipLaunchKernelGGL((bn_bwd_partial<2, true>), pg, dim3(NT), 0, stream, dzw, y, z, scale, shift, save_mean, rows, c, p.rpb, p.cthreads, part);
    else
      hipLaunchKernelGGL((bn_bwd_partial<0>), pg, dim3(NT), 0, stream, dzw, y, z, scale, shift, save_mean, rows, c, p.rpb, p.cthreads, part);
    mask = 0;
    dres = nullptr;
  } else if (mask == 1)
    hipLaunchKernelGGL((bn_bwd_partial<1>), pg, dim3(NT), 0, stream, dzw, y, z, scale, shift, save_mean, rows, c, p.rpb, p.cthreads, part);
  else if (mask == 2)
    hipLaunchKernelGGL((bn_bwd_partial<2>), pg, dim3(NT), 0, stream, dzw, y, z, scale, shift, save_mean, rows, c, p.rpb, p.cthreads, part);
  else
    hipLaunchKernelGGL((bn_bwd_partial<0>), pg, dim3(NT), 0, stream, dzw, y, z, scale, shift, save_mean, rows, c, p.rpb, p.cthreads, part);
  TMR_CHECK_LAUNCH("bn_bwd_partial");
  hipLaunchKernelGGL(bn_bwd_final, dim3(c), dim3(NT), 0, stream, part, p.nrb, rows, c,
                     save_mean, save_invstd, gamma, dgamma, dbeta, coef);
  TMR_CHECK_LAUNCH("bn_bwd_final");
  long n4 = (long)rows * c / 4;
  int nb = ew_blocks(n4);
  int c4 = c / 4;
#define TMR_BN_APPLY(M, D)                                                                     \
  if (out_bf16)                                                                                  \
    hipLaunchKernelGGL((bn_bwd_apply<M, D, __bf16>), dim3(nb), dim3(NT), 0, stream, dz, y, z,    \
                       scale, shift, coef, (__bf16*)dyv, dres, n4, c4);                          \
  else                                                                                           \
    hipLaunchKernelGGL((bn_bwd_apply<M, D>), dim3(nb), dim3(NT), 0, stream, dz, y, z, scale,     \
                       shift, coef, (float*)dyv, dres, n4, c4)
  if (dres) {
    if (mask == 1) { TMR_BN_APPLY(1, true); } else if (mask == 2) { TMR_BN_APPLY(2, true); } else { TMR_BN_APPLY(0, true); }
  } else {
    if (mask == 1) { TMR_BN_APPLY(1, false); } else if (mask == 2) { TMR_BN_APPLY(2, false); } else { TMR_BN_APPLY(0, false); }
  }
#undef TMR_BN_APPLY
  TMR_CHECK_LAUNCH("bn_bwd_apply");
  return 0;
}

TMR_API int tmr_bn_bwd_maxpool(const float* dyp, const uint8_t* argmax, int n, int h, int w,
                               int ho, int wo, const float* y, const float* scale,
                               const float* shift, const float* save_mean,
                               const float* save_invstd, const float* gamma, float* dy,
                               float* dgamma, float* dbeta, int c, void* ws, size_t ws_bytes,
                               hipStream_t stream) {
  return tmr_bn_bwd_maxpool_x(dyp, argmax, n, h, w, ho, wo, y, scale, shift, save_mean,
                              save_invstd, gamma, dy, dgamma, dbeta, c, ws, ws_bytes, 0, stream);
}

static int bn_bwd_maxpool_impl(const float* dyp, const uint8_t* argmax, int n, int h, int w,
                               int ho, int wo, const float* y, const float* scale,
                               const float* shift, const float* save_mean,
                               const float* save_invstd, const float* gamma, void* dyv,
                               float* dgamma, float* dbeta, int c, void* ws, size_t ws_bytes,
                               int out_bf16, float* coef_out, hipStream_t stream);

TMR_API int tmr_bn_bwd_maxpool_x(const float* dyp, const uint8_t* argmax, int n, int h, int w,
                                 int ho, int wo, const float* y, const float* scale,
                                 const float* shift, const float* save_mean,
                                 const float* save_invstd, const float* gamma, void* dyv,
                                 float* dgamma, float* dbeta, int c, void* ws, size_t ws_bytes,
                                 int out_bf16, hipStream_t stream) {
  TMR_CHECK_ARG(dyv, "tmr_bn_bwd_maxpool: null dy");
  return bn_bwd_maxpool_impl(dyp, argmax, n, h, w, ho, wo, y, scale, shift, save_mean,
                             save_invstd, gamma, dyv, dgamma, dbeta, c, ws, ws_bytes, out_bf16,
                             nullptr, stream);
}

static int bn_bwd_maxpool_impl(const float* dyp, const uint8_t* argmax, int n, int h, int w,
                               int ho, int wo, const float* y, const float* scale,
                               const float* shift, const float* save_mean,
                               const float* save_invstd, const float* gamma, void* dyv,
                               float* dgamma, float* dbeta, int c, void* ws, size_t ws_bytes,
                               int out_bf16, float* coef_out, hipStream_t stream) {
  const long rows_l = (long)n * h * w;
  TMR_CHECK_ARG(c % 4 == 0 && c >= 4 && rows_l > 0 && rows_l < 0x7fffffffL,
                "tmr_bn_bwd_maxpool: bad shape n=%d h=%d w=%d c=%d", n, h, w, c);
  TMR_CHECK_ARG(ho == (h + 2 - 3) / 2 + 1 && wo == (w + 2 - 3) / 2 + 1,
                "tmr_bn_bwd_maxpool: pooled %dx%d is not MaxPool2d(3,2,1) of %dx%d", ho, wo, h, w);
  const int rows = (int)rows_l;
  TMR_CHECK_ARG(ws && ws_bytes >= ws_need(rows, c), "tmr_bn_bwd_maxpool: workspace too small");
  PoolGeo pg;
  pg.dyp = dyp; pg.am = (const uchar4*)argmax;
  pg.dHW = make_fastdiv((uint32_t)(h * w)); pg.dW = make_fastdiv((uint32_t)w);
  pg.ho = ho; pg.wo = wo;
  // partials over the pooled rows (fewer than the input rows: the workspace of `rows` suffices)
  const int prows = n * ho * wo;
  Plan p = make_plan(prows, c);
  double* part = (double*)ws;
  float* coef = coef_out ? coef_out : (float*)((char*)ws + (size_t)p.nrb * c * 2 * sizeof(double));
  hipLaunchKernelGGL(stem_bwd_partial_pooled<float>, dim3(p.nrb, p.cblocks), dim3(NT), 0, stream, pg, h, w,
                     y, scale, shift, save_mean, prows, c, p.rpb, p.cthreads,
                     make_fastdiv((uint32_t)(ho * wo)), make_fastdiv((uint32_t)wo), part);
  TMR_CHECK_LAUNCH("stem_bwd_partial_pooled");
  hipLaunchKernelGGL(bn_bwd_final, dim3(c), dim3(NT), 0, stream, part, p.nrb, rows, c,
                     save_mean, save_invstd, gamma, dgamma, dbeta, coef);
  TMR_CHECK_LAUNCH("bn_bwd_final");
  if (!dyv) return 0;   // coefficients only: the stem's direct wgrad applies them on load
  const long n4 = rows_l * c / 4;
  const int c8 = c / 8;
  // per 2x2 input quad, 8 channels per thread (stem_bwd_apply8q, as the bf16-activation step's
  // stem; round 5 for fp32 y), else one pixel and 4 channels per thread
  if (c % 8 == 0 && (c8 & (c8 - 1)) == 0 && n4 / 2 < 0x7fffffffL &&
      (((uintptr_t)dyp | (uintptr_t)y | (uintptr_t)dyv) & 15) == 0 && ((uintptr_t)argmax & 7) == 0) {
    const int qh = (h + 1) / 2, qw = (w + 1) / 2;
    const int nq = n * qh * qw * c8;
    const FastDiv dqhw = make_fastdiv((uint32_t)(qh * qw)), dqw = make_fastdiv((uint32_t)qw);
    if (out_bf16)
      hipLaunchKernelGGL((stem_bwd_apply8q<float, __bf16>), dim3(ew_blocks(nq)), dim3(NT), 0, stream,
                         pg, h, w, dqhw, dqw, y, scale, shift, coef, (__bf16*)dyv, nq, __builtin_ctz(c8));
    else
      hipLaunchKernelGGL((stem_bwd_apply8q<float, float>), dim3(ew_blocks(nq)), dim3(NT), 0, stream,
                         pg, h, w, dqhw, dqw, y, scale, shift, coef, (float*)dyv, nq, __builtin_ctz(c8));
  } else if (out_bf16)
    hipLaunchKernelGGL(stem_bwd_apply<__bf16>, dim3(ew_blocks(n4)), dim3(NT), 0, stream, pg, y, scale,
                       shift, coef, (__bf16*)dyv, n4, c / 4);
  else
    hipLaunchKernelGGL(stem_bwd_apply<float>, dim3(ew_blocks(n4)), dim3(NT), 0, stream, pg, y, scale,
                       shift, coef, (float*)dyv, n4, c / 4);
  TMR_CHECK_LAUNCH("stem_bwd_apply");
  return 0;
}

TMR_API int tmr_bn_bwd_parts(const float* g, const float* y, const void* parts, int nparts,
                             const float* save_mean, const float* save_invstd, const float* gamma,
                             float* dy, float* dgamma, float* dbeta, int rows, int c, void* ws,
                             size_t ws_bytes, hipStream_t stream) {
  return tmr_bn_bwd_parts_x(g, y, parts, nparts, save_mean, save_invstd, gamma, dy, dgamma, dbeta,
                            rows, c, ws, ws_bytes, 0, stream);
}

TMR_API int tmr_bn_bwd_parts_x(const float* g, const float* y, const void* parts, int nparts,
                               const float* save_mean, const float* save_invstd,
                               const float* gamma, void* dyv, float* dgamma, float* dbeta,
                               int rows, int c, void* ws, size_t ws_bytes, int out_bf16,
                               hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0 && c >= 4 && rows > 0 && nparts > 0,
                "tmr_bn_bwd_parts: bad shape rows=%d c=%d parts=%d", rows, c, nparts);
  TMR_CHECK_ARG(ws && ws_bytes >= tmr_bn_parts_ws_bytes(nparts, c),
                "tmr_bn_bwd_parts: workspace too small (need tmr_bn_parts_ws_bytes)");
  const SlabPlan sp = slab_plan(nparts, c);
  double* slabs = (double*)ws;
  float* coef = (float*)((char*)ws + slab_ws_bytes(nparts, c));
  hipLaunchKernelGGL(parts_slab_k<1>, dim3(sp.groups, sp.nslabs), dim3(256), 0, stream, parts,
                     nparts, c, sp.rows, slabs);
  TMR_CHECK_LAUNCH("bn_parts_slab");
  hipLaunchKernelGGL(bwd_final_slabs_k, dim3(sp.groups), dim3(SLAB_CH * SLAB_PH), 0, stream,
                     (const double*)slabs, sp.nslabs, rows, c, save_mean, save_invstd, gamma,
                     dgamma, dbeta, coef);
  TMR_CHECK_LAUNCH("bn_bwd_final_slabs");
  const long n4 = (long)rows * c / 4;
  if (out_bf16)
    hipLaunchKernelGGL((bn_bwd_apply<0, false, __bf16, float>), dim3(ew_blocks(n4)), dim3(NT), 0, stream, g,
                       y, nullptr, nullptr, nullptr, coef, (__bf16*)dyv, nullptr, n4, c / 4);
  else if (c % 8 == 0 && (((uintptr_t)g | (uintptr_t)y | (uintptr_t)dyv) & 15) == 0)
    hipLaunchKernelGGL((bn_bwd_apply8_k<float, float, float>), dim3(ew_blocks(n4 / 2)), dim3(NT), 0,
                       stream, g, y, coef, (float*)dyv, n4 / 2, c / 8);
  else
    hipLaunchKernelGGL((bn_bwd_apply<0, false, float, float>), dim3(ew_blocks(n4)), dim3(NT), 0, stream, g, y,
                       nullptr, nullptr, nullptr, coef, (float*)dyv, nullptr, n4, c / 4);
  TMR_CHECK_LAUNCH("bn_bwd_apply");
  return 0;
}

#if TMR_PROLOGUES   // include/tmr_prologue.h: the retired operand-prologue A/B build
// ---- BatchNorm backward as per-channel coefficients (the apply folded into the consumer GEMMs) --
// dy = fmaf(A[c], g, fmaf(B[c], y, C[c])) -- the arithmetic of bn_bwd_apply -- is evaluated by
// the dgrad / wgrad operand loaders (tmr_conv_prologue.dy_coef = coef [3][c]), so dy is never
// written.

TMR_API int tmr_bn_bwd_coefs(const void* parts, int nparts, const float* save_mean,
                             const float* save_invstd, const float* gamma, float* coef,
                             float* dgamma, float* dbeta, int rows, int c, void* ws,
                             size_t ws_bytes, hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0 && c >= 4 && rows > 0 && nparts > 0,
                "tmr_bn_bwd_coefs: bad shape rows=%d c=%d parts=%d", rows, c, nparts);
  TMR_CHECK_ARG(parts && save_mean && save_invstd && coef, "tmr_bn_bwd_coefs: null operand");
  TMR_CHECK_ARG(ws && ws_bytes >= tmr_bn_parts_ws_bytes(nparts, c),
                "tmr_bn_bwd_coefs: workspace too small (need tmr_bn_parts_ws_bytes)");
  const SlabPlan sp = slab_plan(nparts, c);
  double* slabs = (double*)ws;
  hipLaunchKernelGGL(parts_slab_k<1>, dim3(sp.groups, sp.nslabs), dim3(256), 0, stream, parts,
                     nparts, c, sp.rows, slabs);
  TMR_CHECK_LAUNCH("bn_parts_slab");
  hipLaunchKernelGGL(bwd_final_slabs_k, dim3(sp.groups), dim3(SLAB_CH * SLAB_PH), 0, stream,
                     (const double*)slabs, sp.nslabs, rows, c, save_mean, save_invstd, gamma,
                     dgamma, dbeta, coef);
  TMR_CHECK_LAUNCH("bn_bwd_final_slabs");
  return 0;
}

TMR_API int tmr_bn_bwd_coefs_dense(float* g, const float* y, const float* z, const float* scale,
                                   const float* shift, const float* save_mean,
                                   const float* save_invstd, const float* gamma, float* coef,
                                   float* dgamma, float* dbeta, int rows, int c, int relu,
                                   void* ws, size_t ws_bytes, hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0 && c >= 4, "tmr_bn_bwd_coefs_dense: channels %d must be a multiple of 4", c);
  TMR_CHECK_ARG(rows > 0, "tmr_bn_bwd_coefs_dense: empty input");
  TMR_CHECK_ARG(g && y && save_mean && save_invstd && coef, "tmr_bn_bwd_coefs_dense: null operand");
  TMR_CHECK_ARG(ws && ws_bytes >= ws_need(rows, c), "tmr_bn_bwd_coefs_dense: workspace too small");
  TMR_CHECK_ARG(!relu || z || (scale && shift),
                "tmr_bn_bwd_coefs_dense: relu backward needs the saved output z or the forward scale/shift");
  Plan p = make_plan(rows, c);
  double* part = (double*)ws;
  const dim3 pg(p.nrb, p.cblocks);
  // the ReLU mask is applied to g in place (the masked gradient is the consumers' dY operand
  // and, for a residual unit, the identity branch's gradient)
  if (relu && z)
    hipLaunchKernelGGL((bn_bwd_partial<1, true>), pg, dim3(NT), 0, stream, g, y, z, scale, shift, save_mean, rows, c, p.rpb, p.cthreads, part);
  else if (relu)
    hipLaunchKernelGGL((bn_bwd_partial<2, true>), pg, dim3(NT), 0, stream, g, y, z, scale, shift, save_mean, rows, c, p.rpb, p.cthreads, part);
  else
    hipLaunchKernelGGL((bn_bwd_partial<0>), pg, dim3(NT), 0, stream, g, y, z, scale, shift, save_mean, rows, c, p.rpb, p.cthreads, part);
  TMR_CHECK_LAUNCH("bn_bwd_partial");
  hipLaunchKernelGGL(bn_bwd_final, dim3(c), dim3(NT), 0, stream, part, p.nrb, rows, c,
                     save_mean, save_invstd, gamma, dgamma, dbeta, coef);
  TMR_CHECK_LAUNCH("bn_bwd_final");
  return 0;
}

// the coefficient half of tmr_bn_bwd_g16 (a unit without ReLU whose output gradient is the bf16
// residual-stream gradient: the downsample BN of the bf16-activation step)
TMR_API int tmr_bn_bwd_coefs_g16(const void* g, const void* y, const float* save_mean,
                                 const float* save_invstd, const float* gamma, float* coef,
                                 float* dgamma, float* dbeta, int rows, int c, void* ws,
                                 size_t ws_bytes, hipStream_t stream) {
  TMR_CHECK_ARG(c % 8 == 0 && c >= 8 && rows > 0, "tmr_bn_bwd_coefs_g16: bad shape rows=%d c=%d", rows, c);
  TMR_CHECK_ARG(g && y && save_mean && save_invstd && coef, "tmr_bn_bwd_coefs_g16: null operand");
  TMR_CHECK_ARG(ws && ws_bytes >= ws_need(rows, c), "tmr_bn_bwd_coefs_g16: workspace too small");
  Plan p = make_plan(rows, c);
  double* part = (double*)ws;
  hipLaunchKernelGGL((bn_bwd_partial<0, false, __bf16, const __bf16>), dim3(p.nrb, p.cblocks), dim3(NT),
                     0, stream, (const __bf16*)g, (const __bf16*)y, nullptr, nullptr, nullptr,
                     save_mean, rows, c, p.rpb, p.cthreads, part);
  TMR_CHECK_LAUNCH("bn_bwd_partial_g16");
  hipLaunchKernelGGL(bn_bwd_final, dim3(c), dim3(NT), 0, stream, part, p.nrb, rows, c,
                     save_mean, save_invstd, gamma, dgamma, dbeta, coef);
  TMR_CHECK_LAUNCH("bn_bwd_final");
  return 0;
}
#endif

// ---- bf16-activation forms (TMR_MATH_BF16 train step, include/tmr.h "_a16"): y, z and the
// residual are bf16 tensors (the conv outputs rounded by their epilogue, the BN outputs rounded
// here), the gradients dz / dres stay fp32, dy (a conv operand) is written bf16.  Same arithmetic
// as the fp32 forms on the bf16 values.

// the 8-wide bf16 applies: channels a multiple of 8, 16-B aligned tensors (else the 4-wide forms)
static bool apply8_ok(int c, const void* y, const void* r, const void* z) {
  return c % 8 == 0 && (((uintptr_t)y | (uintptr_t)r | (uintptr_t)z) & 15) == 0;
}

TMR_API int tmr_bn_apply_a16(const void* y, const float* scale, const float* shift,
                             const void* residual, void* z, int rows, int c, int relu,
                             hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0 && y && scale && shift && z, "tmr_bn_apply_a16: bad arguments (c %d)", c);
  const long n4 = (long)rows * c / 4;
  const int nb = ew_blocks(n4), c4 = c / 4;
  const __bf16 *yb = (const __bf16*)y, *rb = (const __bf16*)residual;
  __bf16* zb = (__bf16*)z;
  if (apply8_ok(c, y, residual, z)) {   // 8 per thread (bn_apply8_a16_k)
    const long n8 = n4 / 2;
    const int nb8 = ew_blocks(n8), c8 = c / 8;
    if (rb) {
      if (relu) hipLaunchKernelGGL((bn_apply8_a16_k<true, true, false>), dim3(nb8), dim3(NT), 0, stream, yb, scale, shift, rb, nullptr, nullptr, zb, n8, c8);
      else hipLaunchKernelGGL((bn_apply8_a16_k<true, false, false>), dim3(nb8), dim3(NT), 0, stream, yb, scale, shift, rb, nullptr, nullptr, zb, n8, c8);
    } else {
      if (relu) hipLaunchKernelGGL((bn_apply8_a16_k<false, true, false>), dim3(nb8), dim3(NT), 0, stream, yb, scale, shift, nullptr, nullptr, nullptr, zb, n8, c8);
      else hipLaunchKernelGGL((bn_apply8_a16_k<false, false, false>), dim3(nb8), dim3(NT), 0, stream, yb, scale, shift, nullptr, nullptr, nullptr, zb, n8, c8);
    }
  } else if (rb) {
    if (relu) hipLaunchKernelGGL((bn_apply_k<true, true, __bf16, false, __bf16>), dim3(nb), dim3(NT), 0, stream, yb, scale, shift, rb, zb, n4, c4, nullptr);
    else hipLaunchKernelGGL((bn_apply_k<true, false, __bf16, false, __bf16>), dim3(nb), dim3(NT), 0, stream, yb, scale, shift, rb, zb, n4, c4, nullptr);
  } else {
    if (relu) hipLaunchKernelGGL((bn_apply_k<false, true, __bf16, false, __bf16>), dim3(nb), dim3(NT), 0, stream, yb, scale, shift, rb, zb, n4, c4, nullptr);
    else hipLaunchKernelGGL((bn_apply_k<false, false, __bf16, false, __bf16>), dim3(nb), dim3(NT), 0, stream, yb, scale, shift, rb, zb, n4, c4, nullptr);
  }
  TMR_CHECK_LAUNCH("bn_apply_a16");
  return 0;
}

TMR_API int tmr_bn_apply2_a16(const void* y, const float* scale, const float* shift, const void* yr,
                              const float* rscale, const float* rshift, void* z, int rows, int c,
                              int relu, hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0, "tmr_bn_apply2_a16: channels %d must be a multiple of 4", c);
  TMR_CHECK_ARG(y && scale && shift && yr && rscale && rshift && z, "tmr_bn_apply2_a16: null operand");
  TMR_CHECK_ARG(yr != z, "tmr_bn_apply2_a16: the branch input must not alias z");
  const long n4 = (long)rows * c / 4;
  const __bf16 *yb = (const __bf16*)y, *rb = (const __bf16*)yr;
  if (apply8_ok(c, y, yr, z)) {   // 8 per thread (bn_apply8_a16_k)
    const long n8 = n4 / 2;
    if (relu)
      hipLaunchKernelGGL((bn_apply8_a16_k<false, true, true>), dim3(ew_blocks(n8)), dim3(NT), 0,
                         stream, yb, scale, shift, rb, rscale, rshift, (__bf16*)z, n8, c / 8);
    else
      hipLaunchKernelGGL((bn_apply8_a16_k<false, false, true>), dim3(ew_blocks(n8)), dim3(NT), 0,
                         stream, yb, scale, shift, rb, rscale, rshift, (__bf16*)z, n8, c / 8);
  } else if (relu)
    hipLaunchKernelGGL((bn_apply2_k<true, false, __bf16, __bf16>), dim3(ew_blocks(n4)), dim3(NT), 0,
                       stream, yb, scale, shift, rb, rscale, rshift, (__bf16*)z, n4, c / 4, nullptr);
  else
    hipLaunchKernelGGL((bn_apply2_k<false, false, __bf16, __bf16>), dim3(ew_blocks(n4)), dim3(NT), 0,
                       stream, yb, scale, shift, rb, rscale, rshift, (__bf16*)z, n4, c / 4, nullptr);
  TMR_CHECK_LAUNCH("bn_apply2_a16");
  return 0;
}

TMR_API int tmr_bn_bwd_a16(const float* dz, const void* y, const void* z, const float* scale,
                           const float* shift, const float* save_mean, const float* save_invstd,
                           const float* gamma, void* dy, float* dres, float* dgamma, float* dbeta,
                           int rows, int c, int relu, void* ws, size_t ws_bytes,
                           hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0 && c >= 4, "tmr_bn_bwd_a16: channels %d must be a multiple of 4", c);
  TMR_CHECK_ARG(rows > 0, "tmr_bn_bwd_a16: empty input");
  TMR_CHECK_ARG(ws && ws_bytes >= ws_need(rows, c), "tmr_bn_bwd_a16: workspace too small");
  TMR_CHECK_ARG(!relu || z || (scale && shift),
                "tmr_bn_bwd_a16: relu backward needs the saved output z or the forward scale/shift");
  int mask = relu ? (z ? 1 : 2) : 0;
  Plan p = make_plan(rows, c);
  double* part = (double*)ws;
  float* coef = (float*)((char*)ws + (size_t)p.nrb * c * 2 * sizeof(double));
  const dim3 pg(p.nrb, p.cblocks);
  float* dzw = const_cast<float*>(dz);
  const __bf16 *yb = (const __bf16*)y, *zb = (const __bf16*)z;
  if (dres == dz) {
    if (mask == 1)
      hipLaunchKernelGGL((bn_bwd_partial<1, true, __bf16>), pg, dim3(NT), 0, stream, dzw, yb, zb, scale, shift, save_mean, rows, c, p.rpb, p.cthreads, part);
    else if (mask == 2)
      hipLaunchKernelGGL((bn_bwd_partial<2, true, __bf16>), pg, dim3(NT), 0, stream, dzw, yb, zb, scale, shift, save_mean, rows, c, p.rpb, p.cthreads, part);
    else
      hipLaunchKernelGGL((bn_bwd_partial<0, false, __bf16>), pg, dim3(NT), 0, stream, dzw, yb, zb, scale, shift, save_mean, rows, c, p.rpb, p.cthreads, part);
    mask = 0;
    dres = nullptr;
  } else if (mask == 1)
    hipLaunchKernelGGL((bn_bwd_partial<1, false, __bf16>), pg, dim3(NT), 0, stream, dzw, yb, zb, scale, shift, save_mean, rows, c, p.rpb, p.cthreads, part);
  else if (mask == 2)
    hipLaunchKernelGGL((bn_bwd_partial<2, false, __bf16>), pg, dim3(NT), 0, stream, dzw, yb, zb, scale, shift, save_mean, rows, c, p.rpb, p.cthreads, part);
  else
    hipLaunchKernelGGL((bn_bwd_partial<0, false, __bf16>), pg, dim3(NT), 0, stream, dzw, yb, zb, scale, shift, save_mean, rows, c, p.rpb, p.cthreads, part);
  TMR_CHECK_LAUNCH("bn_bwd_partial");
  hipLaunchKernelGGL(bn_bwd_final, dim3(c), dim3(NT), 0, stream, part, p.nrb, rows, c,
                     save_mean, save_invstd, gamma, dgamma, dbeta, coef);
  TMR_CHECK_LAUNCH("bn_bwd_final");
  const long n4 = (long)rows * c / 4;
  const int nb = ew_blocks(n4), c4 = c / 4;
  __bf16* db = (__bf16*)dy;
#define TMR_BN_APPLY16(M, D)                                                                    \
  hipLaunchKernelGGL((bn_bwd_apply<M, D, __bf16, __bf16>), dim3(nb), dim3(NT), 0, stream, dz, yb, \
                     zb, scale, shift, coef, db, dres, n4, c4)
  if (dres) {
    if (mask == 1) { TMR_BN_APPLY16(1, true); } else if (mask == 2) { TMR_BN_APPLY16(2, true); } else { TMR_BN_APPLY16(0, true); }
  } else if (mask == 0 && c % 8 == 0 && (((uintptr_t)dz | (uintptr_t)y | (uintptr_t)dy) & 15) == 0) {
    // no mask left to apply (the downsample branch's BN, or a mask already written back): the
    // 8-wide apply of the parts path (same coefficients, same fmaf sequence)
    hipLaunchKernelGGL(bn_bwd_apply8_a16<float>, dim3(ew_blocks(n4 / 2)), dim3(NT), 0, stream, dz,
                       yb, coef, db, n4 / 2, c / 8);
  } else {
    if (mask == 1) { TMR_BN_APPLY16(1, false); } else if (mask == 2) { TMR_BN_APPLY16(2, false); } else { TMR_BN_APPLY16(0, false); }
  }
#undef TMR_BN_APPLY16
  TMR_CHECK_LAUNCH("bn_bwd_apply");
  return 0;
}

// BatchNorm backward of a unit without ReLU (the downsample branch's BN) whose output gradient is
// the bf16 residual-stream gradient of the bf16-activation step (trunk.R16): dz, y, dy bf16
TMR_API int tmr_bn_bwd_g16(const void* dz, const void* y, const float* save_mean,
                           const float* save_invstd, const float* gamma, void* dy, float* dgamma,
                           float* dbeta, int rows, int c, void* ws, size_t ws_bytes,
                           hipStream_t stream) {
  TMR_CHECK_ARG(c % 8 == 0 && c >= 8 && rows > 0, "tmr_bn_bwd_g16: bad shape rows=%d c=%d", rows, c);
  TMR_CHECK_ARG((((uintptr_t)dz | (uintptr_t)y | (uintptr_t)dy) & 15) == 0,
                "tmr_bn_bwd_g16: dz / y / dy must be 16-B aligned");
  TMR_CHECK_ARG(ws && ws_bytes >= ws_need(rows, c), "tmr_bn_bwd_g16: workspace too small");
  Plan p = make_plan(rows, c);
  double* part = (double*)ws;
  float* coef = (float*)((char*)ws + (size_t)p.nrb * c * 2 * sizeof(double));
  const __bf16 *gb = (const __bf16*)dz, *yb = (const __bf16*)y;
  hipLaunchKernelGGL((bn_bwd_partial<0, false, __bf16, const __bf16>), dim3(p.nrb, p.cblocks), dim3(NT),
                     0, stream, gb, yb, nullptr, nullptr, nullptr, save_mean, rows, c, p.rpb,
                     p.cthreads, part);
  TMR_CHECK_LAUNCH("bn_bwd_partial_g16");
  hipLaunchKernelGGL(bn_bwd_final, dim3(c), dim3(NT), 0, stream, part, p.nrb, rows, c,
                     save_mean, save_invstd, gamma, dgamma, dbeta, coef);
  TMR_CHECK_LAUNCH("bn_bwd_final");
  const long n8 = (long)rows * c / 8;
  hipLaunchKernelGGL(bn_bwd_apply8_a16<__bf16>, dim3(ew_blocks(n8)), dim3(NT), 0, stream, gb, yb,
                     coef, (__bf16*)dy, n8, c / 8);
  TMR_CHECK_LAUNCH("bn_bwd_apply_g16");
  return 0;
}

TMR_API int tmr_bn_bwd_parts_a16(const float* g, const void* y, const void* parts, int nparts,
                                 const float* save_mean, const float* save_invstd,
                                 const float* gamma, void* dy, float* dgamma, float* dbeta,
                                 int rows, int c, void* ws, size_t ws_bytes, hipStream_t stream) {
  TMR_CHECK_ARG(c % 4 == 0 && c >= 4 && rows > 0 && nparts > 0,
                "tmr_bn_bwd_parts_a16: bad shape rows=%d c=%d parts=%d", rows, c, nparts);
  TMR_CHECK_ARG(ws && ws_bytes >= tmr_bn_parts_ws_bytes(nparts, c),
                "tmr_bn_bwd_parts_a16: workspace too small (need tmr_bn_parts_ws_bytes)");
  const SlabPlan sp = slab_plan(nparts, c);
  double* slabs = (double*)ws;
  float* coef = (float*)((char*)ws + slab_ws_bytes(nparts, c));
  hipLaunchKernelGGL(parts_slab_k<1>, dim3(sp.groups, sp.nslabs), dim3(256), 0, stream, parts,
                     nparts, c, sp.rows, slabs);
  TMR_CHECK_LAUNCH("bn_parts_slab");
  hipLaunchKernelGGL(bwd_final_slabs_k, dim3(sp.groups), dim3(SLAB_CH * SLAB_PH), 0, stream,
                     (const double*)slabs, sp.nslabs, rows, c, save_mean, save_invstd, gamma,
                     dgamma, dbeta, coef);
  TMR_CHECK_LAUNCH("bn_bwd_final_slabs");
  const long n4 = (long)rows * c / 4;
  // 8 per thread (else the 4-wide form)
  if (c % 8 == 0 && (((uintptr_t)g | (uintptr_t)y | (uintptr_t)dy) & 15) == 0) {
    const long n8 = n4 / 2;
    hipLaunchKernelGGL(bn_bwd_apply8_a16<float>, dim3(ew_blocks(n8)), dim3(NT), 0, stream, g,
                       (const __bf16*)y, coef, (__bf16*)dy, n8, c / 8);
  } else {
    hipLaunchKernelGGL((bn_bwd_apply<0, false, __bf16, __bf16>), dim3(ew_blocks(n4)), dim3(NT), 0,
                       stream, g, (const __bf16*)y, nullptr, nullptr, nullptr, coef, (__bf16*)dy,
                       nullptr, n4, c / 4);
  }
  TMR_CHECK_LAUNCH("bn_bwd_apply");
  return 0;
}

TMR_API int tmr_bn_bwd_parts_g16(const void* g, const void* y, const void* parts, int nparts,
                                 const float* save_mean, const float* save_invstd,
                                 const float* gamma, void* dy, float* dgamma, float* dbeta,
                                 int rows, int c, void* ws, size_t ws_bytes, hipStream_t stream) {
  TMR_CHECK_ARG(c % 8 == 0 && c >= 8 && rows > 0 && nparts > 0,
                "tmr_bn_bwd_parts_g16: bad shape rows=%d c=%d parts=%d", rows, c, nparts);
  TMR_CHECK_ARG((((uintptr_t)g | (uintptr_t)y | (uintptr_t)dy) & 15) == 0,
                "tmr_bn_bwd_parts_g16: g / y / dy must be 16-B aligned");
  TMR_CHECK_ARG(ws && ws_bytes >= tmr_bn_parts_ws_bytes(nparts, c),
                "tmr_bn_bwd_parts_g16: workspace too small (need tmr_bn_parts_ws_bytes)");
  const SlabPlan sp = slab_plan(nparts, c);
  double* slabs = (double*)ws;
  float* coef = (float*)((char*)ws + slab_ws_bytes(nparts, c));
  hipLaunchKernelGGL(parts_slab_k<1>, dim3(sp.groups, sp.nslabs), dim3(256), 0, stream, parts,
                     nparts, c, sp.rows, slabs);
  TMR_CHECK_LAUNCH("bn_parts_slab");
  hipLaunchKernelGGL(bwd_final_slabs_k, dim3(sp.groups), dim3(SLAB_CH * SLAB_PH), 0, stream,
                     (const double*)slabs, sp.nslabs, rows, c, save_mean, save_invstd, gamma,
                     dgamma, dbeta, coef);
  TMR_CHECK_LAUNCH("bn_bwd_final_slabs");
  const long n8 = (long)rows * c / 8;
  hipLaunchKernelGGL(bn_bwd_apply8_a16<__bf16>, dim3(ew_blocks(n8)), dim3(NT), 0, stream,
                     (const __bf16*)g, (const __bf16*)y, coef, (__bf16*)dy, n8, c / 8);
  TMR_CHECK_LAUNCH("bn_bwd_apply_g16");
  return 0;
}

// The BatchNorm backward of a downsample block's two units that share one output gradient g (the
// masked gradient of bn3(y3) + bn_ds(y_ds)): bn3's coefficients from the fused dgrad's partials,
// the downsample BN's from one reduction pass over (g, y_ds), then one apply pass that reads g once
// for both -- dy3 = fmaf(A3, g, fmaf(B3, y3, C3)), dyd = fmaf(Ad, g, fmaf(Bd, yd, Cd)), the fmaf
// sequence of bn_bwd_apply / bn_bwd_apply8_a16 -- instead of two apply passes that each read g.
// T: float (fp32 step: g, y, dy fp32) or __bf16 (bf16-activation step under R16: all bf16, dy
// rounded RNE).  8 elements per thread, 16-B accesses.
template <typename T>
__global__ __launch_bounds__(NT) void bn_bwd_apply_ds8(const T* __restrict__ g, const T* __restrict__ y,
                                                       const T* __restrict__ yd,
                                                       const float* __restrict__ coef,
                                                       const float* __restrict__ coefd,
                                                       T* __restrict__ dy, T* __restrict__ dyd, long n8,
                                                       int c8) {
  const int c = c8 * 8;
  auto apply = [&](long i, const float (&gv)[8], const float (&yv)[8], const float (&dv)[8]) {
    const int cc = chan_of(i, c8) * 8;
    float o[8], od[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = fmaf(coef[cc + e], gv[e], fmaf(coef[c + cc + e], yv[e], coef[2 * c + cc + e]));
      od[e] = fmaf(coefd[cc + e], gv[e], fmaf(coefd[c + cc + e], dv[e], coefd[2 * c + cc + e]));
    }
    st8(dy, i, o);
    st8(dyd, i, od);
  };
  // two groups in flight per thread (round 6: one group moved its 5 tensors at 4.8 TB/s)
  const long stride = (long)gridDim.x * NT;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n8; i += 2 * stride) {
    const long j = i + stride;
    const bool hj = j < n8;
    float ga[8], ya[8], da[8], gb[8], yb[8], db[8];
    ld8(g, i, ga);
    ld8(y, i, ya);
    ld8(yd, i, da);
    if (hj) {
      ld8(g, j, gb);
      ld8(y, j, yb);
      ld8(yd, j, db);
    }
    apply(i, ga, ya, da);
    if (hj) apply(j, gb, yb, db);
  }
}

TMR_API size_t tmr_bn_bwd_parts_ds_ws_bytes(int nparts, int rows, int c) {
  if (nparts <= 0 || rows <= 0 || c < 8 || c % 8) {
    tmr_set_error("tmr_bn_bwd_parts_ds_ws_bytes: bad size (parts %d, rows %d, channels %d)", nparts,
                  rows, c);
    return 0;
  }
  return (tmr_bn_parts_ws_bytes(nparts, c) + 255) / 256 * 256 + ws_need(rows, c);
}

TMR_API int tmr_bn_bwd_parts_ds(const void* g, const void* y, const void* parts, int nparts,
                                const float* mean, const float* invstd, const float* gamma,
                                void* dy, float* dgamma, float* dbeta, const void* yd,
                                const float* mean_d, const float* invstd_d, const float* gamma_d,
                                void* dyd, float* dgamma_d, float* dbeta_d, int rows, int c,
                                int bf16, void* ws, size_t ws_bytes, hipStream_t stream) {
  TMR_CHECK_ARG(c % 8 == 0 && c >= 8 && rows > 0 && nparts > 0,
                "tmr_bn_bwd_parts_ds: bad shape rows=%d c=%d parts=%d", rows, c, nparts);
  TMR_CHECK_ARG(g && y && parts && yd && dy && dyd && mean && invstd && gamma && mean_d && invstd_d &&
                    gamma_d, "tmr_bn_bwd_parts_ds: null operand");
  TMR_CHECK_ARG((((uintptr_t)g | (uintptr_t)y | (uintptr_t)yd | (uintptr_t)dy | (uintptr_t)dyd) & 15) == 0,
                "tmr_bn_bwd_parts_ds: g / y / y_ds / dy / dy_ds must be 16-B aligned");
  const size_t a_bytes = (tmr_bn_parts_ws_bytes(nparts, c) + 255) / 256 * 256;
  TMR_CHECK_ARG(ws && ws_bytes >= a_bytes + ws_need(rows, c),
                "tmr_bn_bwd_parts_ds: workspace too small (need tmr_bn_bwd_parts_ds_ws_bytes)");
  // bn3: the fused dgrad's partials (tmr_bn_bwd_parts_x / _g16's kernels)
  const SlabPlan sp = slab_plan(nparts, c);
  double* slabs = (double*)ws;
  float* coef = (float*)((char*)ws + slab_ws_bytes(nparts, c));
  hipLaunchKernelGGL(parts_slab_k<1>, dim3(sp.groups, sp.nslabs), dim3(256), 0, stream, parts,
                     nparts, c, sp.rows, slabs);
  TMR_CHECK_LAUNCH("bn_parts_slab");
  hipLaunchKernelGGL(bwd_final_slabs_k, dim3(sp.groups), dim3(SLAB_CH * SLAB_PH), 0, stream,
                     (const double*)slabs, sp.nslabs, rows, c, mean, invstd, gamma, dgamma, dbeta, coef);
  TMR_CHECK_LAUNCH("bn_bwd_final_slabs");
  // the downsample BN: one reduction pass over (g, y_ds) (tmr_bn_bwd_x / tmr_bn_bwd_g16's kernels)
  char* wb = (char*)ws + a_bytes;
  Plan p = make_plan(rows, c);
  double* part = (double*)wb;
  float* coefd = (float*)(wb + (size_t)p.nrb * c * 2 * sizeof(double));
  const dim3 pg(p.nrb, p.cblocks);
  if (bf16)
    hipLaunchKernelGGL((bn_bwd_partial<0, false, __bf16, const __bf16>), pg, dim3(NT), 0, stream,
                       (const __bf16*)g, (const __bf16*)yd, (const __bf16*)nullptr,
                       (const float*)nullptr, (const float*)nullptr, mean_d, rows, c, p.rpb,
                       p.cthreads, part);
  else
    hipLaunchKernelGGL((bn_bwd_partial<0>), pg, dim3(NT), 0, stream, (float*)g, (const float*)yd,
                       (const float*)nullptr, (const float*)nullptr, (const float*)nullptr, mean_d,
                       rows, c, p.rpb, p.cthreads, part);
  TMR_CHECK_LAUNCH("bn_bwd_partial");
  hipLaunchKernelGGL(bn_bwd_final, dim3(c), dim3(NT), 0, stream, part, p.nrb, rows, c, mean_d,
                     invstd_d, gamma_d, dgamma_d, dbeta_d, coefd);
  TMR_CHECK_LAUNCH("bn_bwd_final");
  const long n8 = (long)rows * c / 8;
  if (bf16)
    hipLaunchKernelGGL(bn_bwd_apply_ds8<__bf16>, dim3(ew_blocks(n8 / 2)), dim3(NT), 0, stream,
                       (const __bf16*)g, (const __bf16*)y, (const __bf16*)yd, coef, coefd,
                       (__bf16*)dy, (__bf16*)dyd, n8, c / 8);
  else
    hipLaunchKernelGGL(bn_bwd_apply_ds8<float>, dim3(ew_blocks(n8 / 2)), dim3(NT), 0, stream,
                       (const float*)g, (const float*)y, (const float*)yd, coef, coefd, (float*)dy,
                       (float*)dyd, n8, c / 8);
  TMR_CHECK_LAUNCH("bn_bwd_apply_ds");
  return 0;
}

TMR_API int tmr_bn_bwd_maxpool_a16(const float* dyp, const uint8_t* argmax, int n, int h, int w,
                                   int ho, int wo, const void* y, const float* scale,
                                   const float* shift, const float* save_mean,
                                   const float* save_invstd, const float* gamma, void* dy,
                                   float* dgamma, float* dbeta, int c, void* ws, size_t ws_bytes,
                                   hipStream_t stream) {
  const long rows_l = (long)n * h * w;
  TMR_CHECK_ARG(c % 4 == 0 && c >= 4 && rows_l > 0 && rows_l < 0x7fffffffL,
                "tmr_bn_bwd_maxpool_a16: bad shape n=%d h=%d w=%d c=%d", n, h, w, c);
  TMR_CHECK_ARG(ho == (h + 2 - 3) / 2 + 1 && wo == (w + 2 - 3) / 2 + 1,
                "tmr_bn_bwd_maxpool_a16: pooled %dx%d is not MaxPool2d(3,2,1) of %dx%d", ho, wo, h, w);
  const int rows = (int)rows_l;
  TMR_CHECK_ARG(ws && ws_bytes >= ws_need(rows, c), "tmr_bn_bwd_maxpool_a16: workspace too small");
  PoolGeo pg;
  pg.dyp = dyp; pg.am = (const uchar4*)argmax;
  pg.dHW = make_fastdiv((uint32_t)(h * w)); pg.dW = make_fastdiv((uint32_t)w);
  pg.ho = ho; pg.wo = wo;
  const int prows = n * ho * wo;
  Plan p = make_plan(prows, c);
  double* part = (double*)ws;
  float* coef = (float*)((char*)ws + (size_t)p.nrb * c * 2 * sizeof(double));
  const __bf16* yb = (const __bf16*)y;
  hipLaunchKernelGGL(stem_bwd_partial_pooled<__bf16>, dim3(p.nrb, p.cblocks), dim3(NT), 0, stream, pg,
                     h, w, yb, scale, shift, save_mean, prows, c, p.rpb, p.cthreads,
                     make_fastdiv((uint32_t)(ho * wo)), make_fastdiv((uint32_t)wo), part);
  TMR_CHECK_LAUNCH("stem_bwd_partial_pooled");
  hipLaunchKernelGGL(bn_bwd_final, dim3(c), dim3(NT), 0, stream, part, p.nrb, rows, c,
                     save_mean, save_invstd, gamma, dgamma, dbeta, coef);
  TMR_CHECK_LAUNCH("bn_bwd_final");
  const long n4 = rows_l * c / 4;
  const int c8 = c / 8;
  // 8 channels per thread, per 2x2 input quad (its candidate pooled outputs gathered once; the
  // per-pixel form it replaced in round 4 was bound by 2.25 gathers per pixel); else 4-wide
  if (c % 8 == 0 && (c8 & (c8 - 1)) == 0 && n4 / 2 < 0x7fffffffL &&
      (((uintptr_t)dyp | (uintptr_t)y | (uintptr_t)dy) & 15) == 0 && ((uintptr_t)argmax & 7) == 0) {
    const int qh = (h + 1) / 2, qw = (w + 1) / 2;
    const int nq = n * qh * qw * c8;
    hipLaunchKernelGGL((stem_bwd_apply8q<__bf16, __bf16>), dim3(ew_blocks(nq)), dim3(NT), 0, stream,
                       pg, h, w, make_fastdiv((uint32_t)(qh * qw)), make_fastdiv((uint32_t)qw), yb,
                       scale, shift, coef, (__bf16*)dy, nq, __builtin_ctz(c8));
  } else {
    hipLaunchKernelGGL((stem_bwd_apply<__bf16, __bf16>), dim3(ew_blocks(n4)), dim3(NT), 0, stream, pg,
                       yb, scale, shift, coef, (__bf16*)dy, n4, c / 4);
  }
  TMR_CHECK_LAUNCH("stem_bwd_apply");
  return 0;
}

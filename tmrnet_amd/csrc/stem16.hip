// The bf16 7x7/2 stem of the bf16-activation train step (configs C4/C5 with a ResNet-50 trunk):
// share.conv1 of train_only_non-local_pretrained.py:204-214 (torchvision resnet50, 3 -> 64
// channels, 224x224 -> 112x112), bf16 operands, fp32 accumulation, y stored bf16 (RNE) with the
// BatchNorm statistics of the stored values -- the TMR_IO_Y_BF16 contract of the engine's convs.
//
// On the LDS-DMA engine the stem reads an NHWC8 bf16 copy of its input (tmr_nhwc4_to_bf16x8) and
// multiplies 49 taps x 8 channels = 392 reduction rows for 147 real ones.  Here a persistent
// workgroup (two per CU) computes whole output rows (112 pixels x 64 channels) from an LDS patch
// of the 7 input rows, read straight from the NHWC4 fp32 input (rounded to bf16 when published)
// and packed per input row as 3 channels per column: the 7 taps x 3 channels of one kernel row at
// output column ow are the 21 consecutive values starting at element 6 * ow.  The reduction runs
// over kernel rows of 24 (21 real, 3 zero weights) -- 168 + 8 (zero) = 11 k-steps of
// v_mfma_f32_32x32x16_bf16 (147 of 176 multiplies useful, 37.5% on the engine).
//   * A (pixels x k): lane (ow, hh) reads the 8 values of chunk m = 2s + hh (kernel row m / 3,
//     offset 8 (m % 3)) as four ds_read_b32 (the chunk starts 12 ow bytes into the row);
//   * B (k x channels): weights k-major per channel, W[co][k'] (row stride 184: 16-B aligned);
//   * epilogue: the tile rounded to bf16, staged in LDS and stored as 16-B pieces; BatchNorm
//     partials (n, mean, M2) per wave and channel merged over the workgroup's rows (Chan, in
//     double, fixed row order), one partial row per wave of the grid (4 * grid rows, not 4 per
//     output row: ADVICE r3).
#include "common.h"
#include "tmr.h"

namespace {

constexpr int SW = 112;          // output width
constexpr int XROW = 704;        // patch row: 230 padded columns x 3 channels = 690, padded
constexpr int XR = 8;            // 7 kernel rows + a zero row (the 22nd chunk)
constexpr int WLD = 184;         // weight row (k' = kh * 24 + kw * 3 + c, 176 used)
constexpr int KS = 11;           // k-steps of 16
constexpr int GRID16 = 768;      // persistent workgroups (three per CU); the wgrad's slabs

typedef float floatx16_t __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ unsigned short bf16_bits_rne(float v) {
  return __builtin_bit_cast(unsigned short, (__bf16)v);
}

// Input rows of a workgroup's contiguous range of output rows: consecutive rows of a frame share
// 5 of their 7 input rows (kept in an LDS ring by the caller), so output row oh needs the 2 new
// input rows 2 oh + 2, 2 oh + 3 -- fetched two output rows ahead into registers (fetch2 / put2:
// 460 pixels, two float4 per thread) -- or, at the first row of a frame or of the range, all 7
// (load7, synchronous: once per 112 rows).  put(ih, col, value) publishes pixel (ih, col - 3).
struct RowFeed {
  const float* x;
  int h, wd, ho, r0;
  __device__ bool first(int row) const { return row == r0 || row % ho == 0; }
  __device__ void fetch2(int row, float4 (&v)[2]) const {
    const int oh = row % ho, n = row / ho;
    int tt = threadIdx.x;
    asm volatile("" : "+v"(tt));
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int i = tt + 256 * q;
      const int k = i / 230, col = i % 230;
      const int ih = 2 * oh + 2 + k, iw = col - 3;
      v[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k < 2 && ih < h && iw >= 0 && iw < wd)
        v[q] = reinterpret_cast<const float4*>(x)[((long)n * h + ih) * wd + iw];
    }
  }
  template <class Put>
  __device__ void put2(int row, const float4 (&v)[2], Put put) const {
    const int oh = row % ho;
    int tt = threadIdx.x;
    asm volatile("" : "+v"(tt));
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int i = tt + 256 * q;
      const int k = i / 230, col = i % 230;
      if (k < 2) put(2 * oh + 2 + k, col, v[q]);
    }
  }
  template <class Put>
  __device__ void load7(int row, Put put) const {
    const int oh = row % ho, n = row / ho;
    constexpr int PPT = (7 * 230 + 255) / 256;
    float4 v[PPT];
    int tt = threadIdx.x;
    asm volatile("" : "+v"(tt));
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
      const int i = tt + 256 * q;
      const int k = i / 230, col = i % 230;
      const int ih = 2 * oh - 3 + k, iw = col - 3;
      v[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k < 7 && ih >= 0 && ih < h && iw >= 0 && iw < wd)
        v[q] = reinterpret_cast<const float4*>(x)[((long)n * h + ih) * wd + iw];
    }
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
      const int i = tt + 256 * q;
      const int k = i / 230, col = i % 230;
      if (k < 7) put(2 * oh - 3 + k, col, v[q]);
    }
  }
};

__global__ __launch_bounds__(256, 3) void stem16_fwd_k(const float* __restrict__ x,
                                                       const __bf16* __restrict__ w_krsc, int cp,
                                                       __bf16* __restrict__ y,
                                                       float4* __restrict__ stats, int h, int wd,
                                                       int ho, int rows) {
  __shared__ __attribute__((aligned(16))) unsigned short Xr[XR * XROW];   // input-row ring, 11 KB
  __shared__ __attribute__((aligned(16))) unsigned short Ws[64 * WLD];    // 23 KB
  __shared__ __attribute__((aligned(16))) unsigned short Ys[SW * 64];     // 14 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l31 = lane & 31, hh = lane >> 5;

  // zero the weights' padding and the ring once (uninitialised LDS could hold NaN patterns, and
  // NaN x 0 is NaN: the zero weights of k' = 21..23 and 168..175 meet whatever the ring holds)
  for (int i = tid; i < 64 * WLD / 2; i += 256) reinterpret_cast<uint32_t*>(Ws)[i] = 0u;
  for (int i = tid; i < XR * XROW / 2; i += 256) reinterpret_cast<uint32_t*>(Xr)[i] = 0u;
  __syncthreads();
  // weights: KRSC (64, 7, 7, cp) bf16 -> W[co][kh * 24 + kw * 3 + c]
  for (int i = tid; i < 64 * 49 * 3; i += 256) {
    const int c = i % 3, tap = (i / 3) % 49, co = i / 147;
    const int kh = tap / 7, kw = tap % 7;
    Ws[co * WLD + kh * 24 + kw * 3 + c] =
        __builtin_bit_cast(unsigned short, w_krsc[((long)co * 49 + tap) * cp + c]);
  }

  // Each workgroup takes a contiguous range of output rows; the input rows stay in a ring of 8
  // LDS rows (input row ih in slot (ih + 8) & 7) fed by RowFeed.
  const int r0 = (int)((long)blockIdx.x * rows / gridDim.x);
  const int r1 = (int)((long)(blockIdx.x + 1) * rows / gridDim.x);
  RowFeed feed{x, h, wd, ho, r0};
  const int ow = 32 * wave + l31;
  const int owc = ow < SW ? ow : SW - 1;       // clamped read (pixels >= 112 are dropped)
  const int cnt = wave == 3 ? SW - 96 : 32;    // this wave's valid output pixels
  // running BatchNorm statistics of this wave's pixels, channels l31 (acc0) and 32 + l31 (acc1)
  double rn = 0.0, rm0 = 0.0, rq0 = 0.0, rm1 = 0.0, rq1 = 0.0;

  // the new input pixels of the next two rows (two-row loads), in two register sets used
  // alternately (static indices: the loop below is unrolled by two)
  float4 setA[2], setB[2];
  if (r0 + 1 < r1 && !feed.first(r0 + 1)) feed.fetch2(r0 + 1, setB);   // (row r0 fetches r0 + 2)
  auto put_x = [&](int ih, int col, float4 v) {
    unsigned short* d = Xr + ((ih + 8) & 7) * XROW + col * 3;
    d[0] = bf16_bits_rne(v.x); d[1] = bf16_bits_rne(v.y); d[2] = bf16_bits_rne(v.z);
  };
  auto step = [&](int row, float4 (&cur)[2]) {
    if (feed.first(row)) feed.load7(row, put_x);
    else feed.put2(row, cur, put_x);
    __syncthreads();   // the ring rows (and the first time the weights) visible; Ys free
    if (row + 2 < r1 && !feed.first(row + 2)) feed.fetch2(row + 2, cur);   // 2 rows ahead
    // kernel row kh of this output row = input row 2 oh - 3 + kh, in ring slot (2 oh + 5 + kh) & 7
    const int oh = row % ho;

    floatx16_t acc0, acc1;
#pragma unroll
    for (int r = 0; r < 16; ++r) { acc0[r] = 0.f; acc1[r] = 0.f; }
    const unsigned short* wb0 = Ws + l31 * WLD + 8 * hh;
    const unsigned short* wb1 = Ws + (32 + l31) * WLD + 8 * hh;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int m = 2 * s + hh;   // chunk: kernel row m / 3 (7: a zero-weight chunk), offset 8 (m % 3)
      const uint32_t* pa = reinterpret_cast<const uint32_t*>(
          Xr + ((2 * oh + 5 + m / 3) & 7) * XROW + 6 * owc + 8 * (m % 3));
      uint4 av;
      av.x = pa[0]; av.y = pa[1]; av.z = pa[2]; av.w = pa[3];
      const bf16x8_t a = __builtin_bit_cast(bf16x8_t, av);
      const bf16x8_t b0 = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(wb0 + 16 * s));
      const bf16x8_t b1 = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(wb1 + 16 * s));
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b1, acc1, 0, 0, 0);
    }

    // epilogue: rounded values -> LDS tile + this wave's statistics
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int px = 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * hh;
      const unsigned short u0 = bf16_bits_rne(acc0[r]), u1 = bf16_bits_rne(acc1[r]);
      acc0[r] = __uint_as_float((uint32_t)u0 << 16);
      acc1[r] = __uint_as_float((uint32_t)u1 << 16);
      if (px < SW) {
        Ys[px * 64 + l31] = u0;
        Ys[px * 64 + 32 + l31] = u1;
        s0 += acc0[r];
        s1 += acc1[r];
      }
    }
    const float m0 = (s0 + __shfl_xor(s0, 32, 64)) / cnt;
    const float m1 = (s1 + __shfl_xor(s1, 32, 64)) / cnt;
    float q0 = 0.f, q1 = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int px = 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * hh;
      if (px < SW) {
        const float d0 = acc0[r] - m0, d1 = acc1[r] - m1;
        q0 = fmaf(d0, d0, q0);
        q1 = fmaf(d1, d1, q1);
      }
    }
    q0 += __shfl_xor(q0, 32, 64);
    q1 += __shfl_xor(q1, 32, 64);
    {   // Chan: running (n, mean, M2) += this row's (cnt, m, q)
      const double nb = (double)cnt, na = rn, nt = na + nb;
      const double d0 = (double)m0 - rm0, d1 = (double)m1 - rm1;
      rm0 += d0 * nb / nt;
      rm1 += d1 * nb / nt;
      rq0 += (double)q0 + d0 * d0 * na * nb / nt;
      rq1 += (double)q1 + d1 * d1 * na * nb / nt;
      rn = nt;
    }
    __syncthreads();   // the tile staged; this row's ring reads done
    // 16-B pieces of the 112 x 64 bf16 tile (rows of 128 B)
    __bf16* yr = y + (long)row * SW * 64;
    for (int i = tid; i < SW * 8; i += 256)
      reinterpret_cast<uint4*>(yr)[i] = reinterpret_cast<const uint4*>(Ys)[i];
    };
  for (int row = r0; row < r1; row += 2) {
    step(row, setA);
    if (row + 1 < r1) step(row + 1, setB);
  }
  if (r0 < r1) {
    float4* st = stats + ((long)blockIdx.x * 4 + wave) * 64;
    if (hh == 0) st[l31] = make_float4((float)rn, (float)rm0, (float)rq0, 0.f);
    else st[32 + l31] = make_float4((float)rn, (float)rm1, (float)rq1, 0.f);
  }
}

// Weight gradient: dW[co][k'] = sum over output pixels of dy[p][co] * X[p][k'], bf16 operands,
// fp32 accumulation.  Workgroups over contiguous ranges of output rows as in the forward; per row
// the operands are staged in LDS in the MFMA's reduction-contiguous form (the reduction runs over
// the row's 112 pixels, 7 k-steps of 16):
//   * Dt[co][p]: the row's dy transposed (the prefetched 16-B pieces written element-wise);
//   * XI[slot][kw * 3 + c][p]: per input row in a ring of 7 slots (input row ih in slot ih % 7),
//     its im2col columns -- input column col = 2 p + kw feeds the 3-4 kernel columns of its
//     parity -- so output row oh's kernel row kh is slot (2 oh - 3 + kh) % 7 and a row builds only
//     its 2 new input rows (7 at the first row of a frame or of the range);
// so every fragment is one ds_read_b128.  Wave w owns co tile (w & 1) and k' tiles 3 (w >> 1) ..
// + 2 (k' = kh * 24 + kw * 3 + c; three 32x32 accumulators, no cross-wave reduction); at the end
// each wave writes its tiles into the workgroup's partial slab in the engine's wgrad layout
// ((co * 49 + tap) * 4 + c), summed in a fixed order by wgrad_reduce_taps_kernel (deterministic).
constexpr int PLD = 120;   // LDS row of the pixel-contiguous images (112 pixels, 16-B rows)

// DY32: dy stored fp32 (bf16-math step without bf16 operand storage): rounded to bf16 (RNE) as
// it is staged -- the bf16 math rounds it anyway, so both storages give the same weight gradient
template <bool DY32>
__global__ __launch_bounds__(256, 3) void stem16_wgrad_k(const float* __restrict__ x,
                                                         const void* __restrict__ dy,
                                                         float* __restrict__ slabs, int h, int wd,
                                                         int ho, int rows) {
  __shared__ __attribute__((aligned(16))) unsigned short XI[(7 * 21 + 1) * PLD];   // 35 KB
  __shared__ __attribute__((aligned(16))) unsigned short Dt[64 * PLD];             // 15 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l31 = lane & 31, hh = lane >> 5;
  unsigned short* const zrow = XI + 7 * 21 * PLD;   // the columns j = 21..23 and k' >= 168
  if (tid < PLD / 2) reinterpret_cast<uint32_t*>(zrow)[tid] = 0u;

  const int r0 = (int)((long)blockIdx.x * rows / gridDim.x);
  const int r1 = (int)((long)(blockIdx.x + 1) * rows / gridDim.x);
  RowFeed feed{x, h, wd, ho, r0};
  constexpr int NDY = SW * 8, DPT = (NDY + 255) / 256;   // 16-B pieces of a dy row
  auto fetch_dy = [&](int row, uint4 (&dv)[DPT]) {
    int tt = tid;
    asm volatile("" : "+v"(tt));
#pragma unroll
    for (int q = 0; q < DPT; ++q) {
      const int i = tt + 256 * q;
      if constexpr (DY32) {   // 8 fp32 channels -> 8 bf16 (16 B)
        const float4* dr = reinterpret_cast<const float4*>(dy) + (long)row * SW * 16;
        if (i < NDY) {
          const float4 a = dr[2 * i], b = dr[2 * i + 1];
          dv[q] = make_uint4((uint32_t)bf16_bits_rne(a.x) | ((uint32_t)bf16_bits_rne(a.y) << 16),
                             (uint32_t)bf16_bits_rne(a.z) | ((uint32_t)bf16_bits_rne(a.w) << 16),
                             (uint32_t)bf16_bits_rne(b.x) | ((uint32_t)bf16_bits_rne(b.y) << 16),
                             (uint32_t)bf16_bits_rne(b.z) | ((uint32_t)bf16_bits_rne(b.w) << 16));
        } else {
          dv[q] = make_uint4(0u, 0u, 0u, 0u);
        }
      } else {
        const uint4* dr = reinterpret_cast<const uint4*>(dy) + (long)row * SW * 8;
        dv[q] = i < NDY ? dr[i] : make_uint4(0u, 0u, 0u, 0u);
      }
    }
  };
  // input pixel (ih, col) -> its im2col columns in ring slot ih % 7
  auto put_x = [&](int ih, int col, float4 pvq) {
    const unsigned short v[3] = {bf16_bits_rne(pvq.x), bf16_bits_rne(pvq.y), bf16_bits_rne(pvq.z)};
    unsigned short* blk = XI + (((ih + 7) % 7) * 21) * PLD;
#pragma unroll
    for (int kw = 0; kw < 7; ++kw) {
      const int t = col - kw;   // = 2 p
      if ((t & 1) == 0 && t >= 0 && t < 2 * SW) {
        unsigned short* d = blk + (kw * 3) * PLD + (t >> 1);
        d[0] = v[0];
        d[PLD] = v[1];
        d[2 * PLD] = v[2];
      }
    }
  };
  auto put_dy = [&](const uint4 (&dv)[DPT]) {
    int tt = tid;
    asm volatile("" : "+v"(tt));
#pragma unroll
    for (int q = 0; q < DPT; ++q) {
      const int i = tt + 256 * q;
      if (i < NDY) {
        const int p = i >> 3, c0 = (i & 7) * 8;
        const uint32_t w[4] = {dv[q].x, dv[q].y, dv[q].z, dv[q].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          Dt[(c0 + 2 * e) * PLD + p] = (unsigned short)(w[e] & 0xffffu);
          Dt[(c0 + 2 * e + 1) * PLD + p] = (unsigned short)(w[e] >> 16);
        }
      }
    }
  };

  const int mt = wave & 1, nt0 = 3 * (wave >> 1);
  floatx16_t acc[3];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  const unsigned short* pa = Dt + (32 * mt + l31) * PLD + 8 * hh;

  // the new input pixels and the dy of the next two rows, in two register sets used alternately
  // (static indices: the loop below is unrolled by two)
  float4 xA[2], xB[2];
  uint4 dA[DPT], dB[DPT];
  if (r0 < r1) fetch_dy(r0, dA);
  if (r0 + 1 < r1) {
    if (!feed.first(r0 + 1)) feed.fetch2(r0 + 1, xB);
    fetch_dy(r0 + 1, dB);
  }
  auto step = [&](int row, float4 (&xc)[2], uint4 (&dc)[DPT]) {
    __syncthreads();   // the previous row's fragments are read: ring slots / Dt free
    if (feed.first(row)) feed.load7(row, put_x);
    else feed.put2(row, xc, put_x);
    put_dy(dc);
    __syncthreads();   // this row's operands visible
    if (row + 2 < r1) {   // lands under the next two rows' MFMAs
      if (!feed.first(row + 2)) feed.fetch2(row + 2, xc);
      fetch_dy(row + 2, dc);
    }
    const int oh = row % ho;
    const unsigned short* pb[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int kk = 32 * (nt0 + t) + l31;   // this lane's k' column of tile t
      const int kh = kk / 24, j = kk % 24;
      pb[t] = (kh < 7 && j < 21) ? XI + (((2 * oh - 3 + kh + 7) % 7) * 21 + j) * PLD + 8 * hh
                                 : zrow + 8 * hh;
    }
#pragma unroll
    for (int s = 0; s < SW / 16; ++s) {
      const bf16x8_t a = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(pa + 16 * s));
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const bf16x8_t b = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(pb[t] + 16 * s));
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[t], 0, 0, 0);
      }
    }
    };
  for (int row = r0; row < r1; row += 2) {
    step(row, xA, dA);
    if (row + 1 < r1) step(row + 1, xB, dB);
  }
  // this wave's tiles -> the workgroup's slab (channel 3 of each tap not written)
  float* slab = slabs + (long)blockIdx.x * (64 * 49 * 4);
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int kk = 32 * (nt0 + t) + l31;   // k' of this lane's column
    const int kh = kk / 24, j = kk % 24;
    if (kh < 7 && j < 21) {
      const int tap = kh * 7 + j / 3, c = j % 3;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = 32 * mt + (r & 3) + 8 * (r >> 2) + 4 * hh;
        slab[(co * 49 + tap) * 4 + c] = acc[t][r];
      }
    }
  }
}

}  // namespace

int tmr_stem16_wgrad_slabs(int n, int h, int w, int ho, const float* x, const void* dy, int dy32,
                           float* ws, size_t ws_bytes, int* nslabs, hipStream_t stream) {
  TMR_CHECK_ARG(n > 0 && ho > 0 && (w + 6 - 7) / 2 + 1 == SW && w + 6 <= 230 &&
                    (h + 6 - 7) / 2 + 1 == ho,
                "tmr_stem16_wgrad: unsupported geometry %dx%d", h, w);
  TMR_CHECK_ARG((((uintptr_t)x | (uintptr_t)dy) & 15) == 0, "tmr_stem16_wgrad: x / dy must be 16-B aligned");
  const int rows = n * ho;
  const int grid = rows < GRID16 ? rows : GRID16;
  TMR_CHECK_ARG(ws && ws_bytes >= (size_t)grid * 64 * 49 * 4 * sizeof(float),
                "tmr_stem16_wgrad: workspace too small (%zu)", ws_bytes);
  if (dy32)
    hipLaunchKernelGGL(stem16_wgrad_k<true>, dim3(grid), dim3(256), 0, stream, x, dy, ws, h, w, ho,
                       rows);
  else
    hipLaunchKernelGGL(stem16_wgrad_k<false>, dim3(grid), dim3(256), 0, stream, x, dy, ws, h, w, ho,
                       rows);
  TMR_CHECK_LAUNCH("stem16_wgrad");
  *nslabs = grid;
  return 0;
}

// Partial statistics rows of tmr_stem16_fwd_bnstats: 4 per workgroup of its grid
int tmr_stem16_stats_parts(int n, int ho) {
  const int rows = n * ho;
  return 4 * (rows < GRID16 ? rows : GRID16);
}

// x NHWC4 fp32 (n, h, w, 4), the 4th channel ignored; w KRSC (64, 7, 7, cp) bf16 (cp = 4 or 8);
// y (n, ho, 112, 64) bf16; stats: tmr_stem16_stats_parts rows of 64 float4 (n, mean, M2, 0).
int tmr_stem16_fwd_bnstats(int n, int h, int w, int ho, const float* x, const void* w_krsc, int cp,
                           void* y, void* stats, hipStream_t stream) {
  TMR_CHECK_ARG(n > 0 && ho > 0 && (w + 6 - 7) / 2 + 1 == SW && w + 6 <= 230 &&
                    (h + 6 - 7) / 2 + 1 == ho && (cp == 4 || cp == 8),
                "tmr_stem16_fwd_bnstats: unsupported geometry %dx%d (cp %d)", h, w, cp);
  TMR_CHECK_ARG((((uintptr_t)x | (uintptr_t)y) & 15) == 0 && ((uintptr_t)w_krsc & 1) == 0,
                "tmr_stem16_fwd_bnstats: x / y must be 16-B aligned");
  const int rows = n * ho;
  const int grid = rows < GRID16 ? rows : GRID16;
  hipLaunchKernelGGL(stem16_fwd_k, dim3(grid), dim3(256), 0, stream, x, (const __bf16*)w_krsc, cp,
                     (__bf16*)y, (float4*)stats, h, w, ho, rows);
  TMR_CHECK_LAUNCH("stem16_fwd");
  return 0;
}

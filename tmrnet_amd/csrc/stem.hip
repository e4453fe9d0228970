// The fp32 7x7/2 stem convolution of the train step (conv1 + its BatchNorm statistics) as a
// direct convolution: share.conv1 of train_only_non-local_pretrained.py:204-214 (torchvision
// resnet50, 3 -> 64 channels, 224x224 -> 112x112).
//
// On the implicit-GEMM engine the stem's reduction is 49 taps x 4 channels (the NHWC4 input's
// zero 4th channel) padded to 7 k-tiles of 32: 147 useful of 224 multiplied (the engine's
// 16-B pieces cannot pack 3 channels per tap).  Here a persistent workgroup (two per CU) computes
// output rows of one frame (112 pixels x 64 channels) from an LDS copy of the 7 input rows each
// reads -- the next row's patch is fetched into registers under the current row's MFMAs and
// published to the other half of a double buffer -- with the weights staged once and the
// reduction over exactly the 147 real (tap, channel) pairs:
//   * input patch, channel- and column-parity-planar: X[kh][c][col & 1][col >> 1] for the padded
//     columns col = iw + 3 (0 outside the image) -- the 32 lanes of an MFMA operand read
//     consecutive words (column 2*ow + kw: parity kw & 1, half ow + kw / 2);
//   * weights k-major: W[k][co], k = (kh * 7 + kw) * 3 + c (148 rows, the last 0);
//   * v_mfma_f32_32x32x2_f32, each wave 32 output pixels x 64 channels, 74 k-steps;
//   * epilogue: y (NHWC, 64 channels) and each wave's BatchNorm partial (n, mean, M2) per channel
//     over its 32 (last wave: 16) pixels, merged over the workgroup's rows (Chan, in double) --
//     the conv epilogue's statistics format, combined by tmr_bn_finalize -- with no cross-wave
//     exchange, so a row needs a single barrier.
#include "common.h"
#include "tmr.h"

namespace {

constexpr int SW = 112;          // output width
constexpr int XH = 7;            // input rows per output row
constexpr int XHALF = 116;       // padded columns / 2 (230 used)
constexpr int KR = 148;          // 147 real reduction rows + 1 zero row (k-steps of 2)
constexpr int GRID = 512;        // persistent workgroups (two per CU) = the wgrad's partial slabs

typedef float floatx16_t __attribute__((ext_vector_type(16)));

// LDS offset in the patch image of reduction row k = (kh * 7 + kw) * 3 + c at output column 0
__host__ __device__ constexpr int kx_of(int k) {
  return k >= 147 ? 0
                  : ((((k / 3) / 7) * 3 + k % 3) * 2 + ((k / 3) % 7 & 1)) * XHALF + ((k / 3) % 7 >> 1);
}

__global__ __launch_bounds__(256, 2) void stem_fwd_k(const float* __restrict__ x,
                                                     const float* __restrict__ w_krsc,
                                                     float* __restrict__ y,
                                                     float4* __restrict__ stats, int h, int wd,
                                                     int ho, int rows) {
  constexpr int XS = XH * 3 * 2 * XHALF;
  __shared__ float Xs[2 * XS];   // 2 x 19.5 KB: the patch of this row and of the next
  __shared__ float Ws[KR * 64];  // 37.9 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // weights, once per (persistent) workgroup: KRSC (64, 7, 7, 4) -> k-major [k][co] over the 3
  // real channels (consecutive threads: consecutive co, conflict-free LDS writes)
  for (int i = tid; i < 64 * 49; i += 256) {
    const int co = i & 63, tap = i >> 6;
    const float4 v = reinterpret_cast<const float4*>(w_krsc)[co * 49 + tap];
    Ws[(tap * 3 + 0) * 64 + co] = v.x;
    Ws[(tap * 3 + 1) * 64 + co] = v.y;
    Ws[(tap * 3 + 2) * 64 + co] = v.z;
  }
  if (tid < 64) Ws[147 * 64 + tid] = 0.f;
  // input rows ih = 2 * oh - 3 + kh, columns iw = col - 3 (NHWC4: 3 real channels); each thread
  // holds its pieces of the next row's patch in registers while the current row computes
  constexpr int NP = XH * 2 * XHALF, PPT = (NP + 255) / 256;
  float4 pv[PPT];
  auto fetch = [&](int row) {
    const int oh = row % ho, n = row / ho;
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
      const int i = tid + 256 * q;
      const int kh = i / (2 * XHALF), col = i % (2 * XHALF);
      const int ih = 2 * oh - 3 + kh, iw = col - 3;
      pv[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < NP && ih >= 0 && ih < h && iw >= 0 && iw < wd)
        pv[q] = reinterpret_cast<const float4*>(x)[((long)n * h + ih) * wd + iw];
    }
  };
  auto publish = [&](float* X) {
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
      const int i = tid + 256 * q;
      if (i < NP) {
        const int kh = i / (2 * XHALF), col = i % (2 * XHALF);
        const int base = (kh * 3) * 2 * XHALF + (col & 1) * XHALF + (col >> 1);
        X[base] = pv[q].x;
        X[base + 2 * XHALF] = pv[q].y;
        X[base + 4 * XHALF] = pv[q].z;
      }
    }
  };
  const int l31 = lane & 31, hh = lane >> 5;
  const int ow = 32 * wave + l31;
  const int owc = ow < SW ? ow : SW - 1;   // clamped read (rows >= 112 are dropped)
  const int cnt = wave == 3 ? SW - 96 : 32;   // this wave's valid output pixels
  // running BatchNorm statistics of this wave's pixels over the workgroup's rows (Chan, double,
  // fixed row order): one partial row per wave of the grid (not one per output row)
  double rn = 0.0, rm0 = 0.0, rq0 = 0.0, rm1 = 0.0, rq1 = 0.0;
  int row = blockIdx.x, buf = 0;
  if (row < rows) fetch(row);
  for (; row < rows; row += gridDim.x, buf ^= 1) {
    // the other buffer was last read two rows ago, before the previous row's barrier
    float* X = Xs + buf * XS;
    publish(X);
    __syncthreads();   // the patch (and, the first time, the weights) visible
    if (row + (int)gridDim.x < rows) fetch(row + gridDim.x);   // lands under the MFMAs

    // wave: output pixels ow = 32 * wave + (lane & 31) (>= 112: dropped), channels 0..63; lanes
    // 32..63 take the odd reduction row of each k-step
    floatx16_t acc0, acc1;
#pragma unroll
    for (int r = 0; r < 16; ++r) { acc0[r] = 0.f; acc1[r] = 0.f; }
    const float* xa = X + owc;
    const float* wb = Ws + hh * 64 + l31;
#pragma unroll
    for (int s = 0; s < KR / 2; ++s) {
      const float a = xa[hh ? kx_of(2 * s + 1) : kx_of(2 * s)];
      const float b0 = wb[2 * s * 64], b1 = wb[2 * s * 64 + 32];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b1, acc1, 0, 0, 0);
    }

    // epilogue: y rows (pixels) and this wave's BatchNorm partial (no cross-wave exchange)
    const long prow = (long)row * SW;
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int px = 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * hh;
      if (px < SW) {
        y[(prow + px) * 64 + l31] = acc0[r];
        y[(prow + px) * 64 + 32 + l31] = acc1[r];
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
    const double nb = (double)cnt, na = rn, nt = na + nb;
    const double d0 = (double)m0 - rm0, d1 = (double)m1 - rm1;
    rm0 += d0 * nb / nt;
    rm1 += d1 * nb / nt;
    rq0 += (double)q0 + d0 * d0 * na * nb / nt;
    rq1 += (double)q1 + d1 * d1 * na * nb / nt;
    rn = nt;
  }
  if ((int)blockIdx.x < rows) {
    float4* st = stats + ((long)blockIdx.x * 4 + wave) * 64;
    if (hh == 0) st[l31] = make_float4((float)rn, (float)rm0, (float)rq0, 0.f);
    else st[32 + l31] = make_float4((float)rn, (float)rm1, (float)rq1, 0.f);
  }
}

// Weight gradient: dW[co][k] = sum over output pixels p of dy[p][co] * X[p][k] (k the 147 real
// (tap, channel) pairs).  Persistent workgroups over output rows as in the forward (patch double
// buffer, the next row's patch in registers under the MFMAs); wave w takes pixel pairs w, w + 4, ... of a
// row (14 k-steps of 2 pixels): A = dy (32 channels x 2 pixels, straight from HBM, each element
// read once), B = the patch (2 pixels x 32 reduction rows from LDS), 2 x 5 accumulator tiles of
// 32x32 (64 channels x 160 reduction rows).  At the end the four waves add their tiles in LDS and
// the workgroup writes one partial slab in the engine's wgrad layout ((co * 49 + tap) * 4 + c),
// which wgrad_reduce_taps_kernel sums in a fixed order (deterministic).
__global__ __launch_bounds__(256, 2) void stem_wgrad_k(const float* __restrict__ x,
                                                       const float* __restrict__ dy,
                                                       float* __restrict__ slabs, int h, int wd,
                                                       int ho, int rows) {
  constexpr int XS = XH * 3 * 2 * XHALF;
  __shared__ float Xs[2 * XS];   // 2 x 19.5 KB; at the end the 64 x 147 partial
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l31 = lane & 31, hh = lane >> 5;
  constexpr int NP = XH * 2 * XHALF, PPT = (NP + 255) / 256;
  float4 pv[PPT];
  auto fetch = [&](int row) {
    const int oh = row % ho, n = row / ho;
    // the thread index through an empty asm: the per-piece index math is recomputed per row
    // instead of being hoisted out of the row loop into registers the accumulators need
    int tt = tid;
    asm volatile("" : "+v"(tt));
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
      const int i = tt + 256 * q;
      const int kh = i / (2 * XHALF), col = i % (2 * XHALF);
      const int ih = 2 * oh - 3 + kh, iw = col - 3;
      pv[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < NP && ih >= 0 && ih < h && iw >= 0 && iw < wd)
        pv[q] = reinterpret_cast<const float4*>(x)[((long)n * h + ih) * wd + iw];
    }
  };
  int kxl[5];   // this lane's reduction row k = 32 * t + (lane & 31) in the patch image
#pragma unroll
  for (int t = 0; t < 5; ++t) kxl[t] = kx_of(32 * t + l31);
  floatx16_t acc[2][5];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int t = 0; t < 5; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][t][r] = 0.f;

  // the next row's patch is fetched into registers under this row's MFMAs
  if ((int)blockIdx.x < rows) fetch(blockIdx.x);
  for (int row = blockIdx.x, buf = 0; row < rows; row += gridDim.x, buf ^= 1) {
    float* X = Xs + buf * XS;
    int tt = tid;
    asm volatile("" : "+v"(tt));
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
      const int i = tt + 256 * q;
      if (i < NP) {
        const int kh = i / (2 * XHALF), col = i % (2 * XHALF);
        const int base = (kh * 3) * 2 * XHALF + (col & 1) * XHALF + (col >> 1);
        X[base] = pv[q].x;
        X[base + 2 * XHALF] = pv[q].y;
        X[base + 4 * XHALF] = pv[q].z;
      }
    }
    __syncthreads();   // the patch visible (the other buffer was last read two rows ago)
    // this wave's dy: pixels p = 2 * (wave + 4 * j) + (lane >> 5), channels (lane & 31) + 32 m
    const float* dyr = dy + ((long)row * SW + 2 * wave + hh) * 64 + l31;
    const float* xb = X + 2 * wave + hh;
    {
      // A straight from HBM: all of the row's loads issued up front
      float a[14][2];
#pragma unroll
      for (int j = 0; j < 14; ++j) {
        a[j][0] = dyr[8 * j * 64];
        a[j][1] = dyr[8 * j * 64 + 32];
      }
      if (row + (int)gridDim.x < rows) fetch(row + gridDim.x);
#pragma unroll
      for (int j = 0; j < 14; ++j) {
        float b[5];
#pragma unroll
        for (int t = 0; t < 5; ++t) b[t] = xb[kxl[t] + 8 * j];
#pragma unroll
        for (int t = 0; t < 5; ++t) {
          acc[0][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j][0], b[t], acc[0][t], 0, 0, 0);
          acc[1][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j][1], b[t], acc[1][t], 0, 0, 0);
        }
      }
    }
  }

  // the four waves' tiles summed in LDS (fixed order), then one partial slab per workgroup
  float* red = Xs;   // 64 x 147 floats <= 2 * XS
  __syncthreads();
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int t = 0; t < 5; ++t) {
          const int k = 32 * t + l31;
          if (k < 147) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int co = 32 * m + (r & 3) + 8 * (r >> 2) + 4 * hh;
              float& dst = red[co * 147 + k];
              dst = w == 0 ? acc[m][t][r] : dst + acc[m][t][r];
            }
          }
        }
    }
    __syncthreads();
  }
  float* slab = slabs + (long)blockIdx.x * (64 * 49 * 4);
  for (int i = tid; i < 64 * 147; i += 256) {
    const int co = i / 147, k = i - co * 147;
    slab[(co * 49 + k / 3) * 4 + k % 3] = red[i];
  }
}

}  // namespace

// tmr_conv2d_fwd_bnstats for the stem geometry (gemm_conv.hip routes it here): x NHWC4 fp32
// (n, h, w, 4) with the 4th channel ignored, w KRSC (64, 7, 7, 4) fp32, stride 2, pad 3, output
// width 112; one BatchNorm partial row per wave of the grid (tmr_stem_stats_parts rows of 64).
int tmr_stem_stats_parts(int n, int ho) {
  const int rows = n * ho;
  return 4 * (rows < GRID ? rows : GRID);
}

int tmr_stem_fwd_bnstats(int n, int h, int w, int ho, const float* x, const float* w_krsc,
                         float* y, void* stats, hipStream_t stream) {
  TMR_CHECK_ARG(n > 0 && ho > 0 && (w + 6 - 7) / 2 + 1 == SW && 2 * XHALF >= w + 6,
                "tmr_stem_fwd_bnstats: unsupported geometry %dx%d", h, w);
  TMR_CHECK_ARG((((uintptr_t)x | (uintptr_t)w_krsc) & 15) == 0,
                "tmr_stem_fwd_bnstats: x / w must be 16-B aligned");
  // persistent: two workgroups per CU (LDS), each over a strided sequence of output rows (the
  // weights are staged once per workgroup)
  const int rows = n * ho;
  const int grid = rows < GRID ? rows : GRID;
  hipLaunchKernelGGL(stem_fwd_k, dim3(grid), dim3(256), 0, stream, x, w_krsc, y,
                     (float4*)stats, h, w, ho, rows);
  TMR_CHECK_LAUNCH("stem_fwd");
  return 0;
}

// Stem weight gradient (gemm_conv.hip routes the fp32 stem here): partial slabs of the engine's
// wgrad layout (64 x 49 x 4 floats, channel 3 not written) into ws, one per workgroup; *nslabs
// = their number (the caller reduces them).
int tmr_stem_wgrad_slabs(int n, int h, int w, int ho, const float* x, const float* dy, float* ws,
                         size_t ws_bytes, int* nslabs, hipStream_t stream) {
  TMR_CHECK_ARG(n > 0 && ho > 0 && (w + 6 - 7) / 2 + 1 == SW && 2 * XHALF >= w + 6,
                "tmr_stem_wgrad: unsupported geometry %dx%d", h, w);
  TMR_CHECK_ARG(((uintptr_t)x & 15) == 0, "tmr_stem_wgrad: x must be 16-B aligned");
  const int rows = n * ho;
  const int grid = rows < GRID ? rows : GRID;
  TMR_CHECK_ARG(ws && ws_bytes >= (size_t)grid * 64 * 49 * 4 * sizeof(float),
                "tmr_stem_wgrad: workspace too small (%zu)", ws_bytes);
  hipLaunchKernelGGL(stem_wgrad_k, dim3(grid), dim3(256), 0, stream, x, dy, ws, h, w, ho, rows);
  TMR_CHECK_LAUNCH("stem_wgrad");
  *nslabs = grid;
  return 0;
}

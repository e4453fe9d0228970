// Direct 3x3 / stride-1 convolutions of the narrow 112x112 layers of the bf16-activation train step:
// ResNeSt-50's deep stem (the third-party resnest50() called at
// train_non-local_mutiConv_resnest.py:210; conv1 = 3x3/2 3 -> 32, BN, ReLU, 3x3 32 -> 32, BN, ReLU,
// 3x3 32 -> 64) -- its two stride-1 convs, all operands bf16 (TMR_IO_*_BF16), fp32 accumulation.
//
// On the implicit-GEMM engine these run at 140-340 TF: 32-64 output channels leave most of a
// 256x64 tile's columns or k-tiles idle, and every input pixel is gathered 9 times through L2.  Here
// a persistent workgroup computes whole output rows (112 pixels x COUT channels) from a ring of the
// 3 input rows it needs in LDS, each fetched from HBM once (one new row per output row, prefetched
// into registers a row ahead):
//   * forward (d3_k MODE 0): v_mfma_f32_16x16x32_bf16, the 112 pixels as 7 m-tiles of 16, one k-step
//     per (tap, 32 channels); the weights stay in registers (72 VGPRs per wave); y rounded to bf16,
//     staged in LDS and stored as 16-B pieces; BatchNorm partials (n, mean, M2) of the stored values
//     per wave and channel, merged over the workgroup's rows (Chan, double, fixed order);
//   * dgrad (MODE 1): the same kernel over dy with the transposed weights (CRSK) tap-flipped -- the
//     dgrad of a stride-1 pad-1 3x3 conv is that conv -- and the fused BatchNorm backward of the
//     unit that produced the conv input in its epilogue (tmr_conv2d_dgrad_bnbwd's contract: ReLU
//     mask from z (1) or from y * scale + shift (2), beta * old dx, partial sums sum(g) and
//     sum(g * (y - mean)) per channel, one partial row per workgroup);
//   * weight gradient (d3w_k): per output row dW[co][tap][ci] += dy^T x over the row's pixels (K =
//     112 padded to 128), both operands as stored ([pixel][channel]) and read transposed by
//     ds_read_b64_tr_b16; per-workgroup slabs in the engine's wgrad layout, summed in a fixed order
//     by wgrad_reduce_taps_kernel (deterministic).
// LDS pixel rows are padded to 2 C + 32 bytes: conflict-free for the b128 row reads and for the
// transposed reads with the odd 16-lane groups taking their upper 4 rows first
// (scripts/probe/lds_banks.py).
#include "common.h"
#include "tmr.h"

namespace {

constexpr int DW = 112;   // output (= input) width

typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ unsigned short bfb(float v) {
  return __builtin_bit_cast(unsigned short, (__bf16)v);
}
__device__ __forceinline__ float bff(uint32_t u16) { return __uint_as_float(u16 << 16); }

template <int C, int W = DW>
struct Px {
  static constexpr int PS = 2 * C + 32;       // LDS bytes per pixel row
  static constexpr int CPP = C / 8;           // 16-B chunks per pixel
  static constexpr int PIECES = W * CPP;      // 16-B pieces of a W-pixel row
  static constexpr int PPT = (PIECES + 255) / 256;
};

// One W-pixel row of an NHWC bf16 tensor (global row index g) <-> registers <-> an LDS image of
// pixel rows (pixel p at byte (p + off) * PS).
template <int C, int W = DW>
struct RowIO {
  using P = Px<C, W>;
  __device__ static void fetch(const uint4* __restrict__ t, int g, bool valid, uint4 (&v)[P::PPT]) {
    int tt = threadIdx.x;
    asm volatile("" : "+v"(tt));
#pragma unroll
    for (int q = 0; q < P::PPT; ++q) {
      const int i = tt + 256 * q;
      v[q] = (valid && i < P::PIECES) ? t[(long)g * P::PIECES + i] : make_uint4(0u, 0u, 0u, 0u);
    }
  }
  __device__ static void put(unsigned char* img, int off, const uint4 (&v)[P::PPT]) {
    int tt = threadIdx.x;
    asm volatile("" : "+v"(tt));
#pragma unroll
    for (int q = 0; q < P::PPT; ++q) {
      const int i = tt + 256 * q;
      if (i < P::PIECES)
        *reinterpret_cast<uint4*>(img + (i / P::CPP + off) * P::PS + (i % P::CPP) * 16) = v[q];
    }
  }
};

// workgroups per CU (the grid is that many per CU: persistent): three where the registers allow
constexpr int d3_minb(int cin, int cout, int mode) {
  return (mode == 0 && cin == cout) ? 3 : 2;   // the forwards 32 -> 32 and 64 -> 64
}

// MODE 0: forward, y bf16 + BatchNorm partial statistics.  MODE 1: dgrad (x = dy, w = the CRSK copy,
// taps flipped) with the fused BatchNorm backward; out = dx fp32.
// W: row width (112, or 56 with a half-empty last m-tile).  G16 (dgrad): dx -- the masked gradient
// -- stored bf16 and the partial sums those of the rounded values (TMR_IO_G16), no beta.
template <int CIN, int COUT, int MODE, int W = DW, int G16 = 0>
__global__ __launch_bounds__(256, d3_minb(CIN, COUT, MODE))
void d3_k(const uint4* __restrict__ x, const __bf16* __restrict__ wk, void* __restrict__ out,
          float4* __restrict__ stats, const uint4* __restrict__ by, const uint4* __restrict__ bz,
          const float* __restrict__ bsc, const float* __restrict__ bsh,
          const float* __restrict__ bmu, int mask, float beta, float2* __restrict__ part, int h,
          int rows) {
  using PI = Px<CIN, W>;
  constexpr int KPT = CIN / 32, KS = 9 * KPT;
  constexpr int NT = COUT / 16, NPW = 18 / KS, WN = NT / NPW, WM = 4 / WN;
  constexpr int MT = (W + 15) / 16;   // m-tiles of 16 pixels
  constexpr int MPW = (MT + WM - 1) / WM;
  static_assert(NPW * KS == 18 && NT % NPW == 0 && WN * WM == 4, "wave split");
  static_assert(!G16 || MODE == 1, "G16: dgrad only");
  constexpr int SLOT = (16 * MT + 2) * PI::PS;   // pixel columns x = -1 .. 16 MT (zeros past W)
  constexpr int OST = MODE == 0 ? W * COUT * 2 : W * (COUT + 4) * 4;
  __shared__ __attribute__((aligned(16))) unsigned char ring[3 * SLOT];
  __shared__ __attribute__((aligned(16))) unsigned char ost[OST];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int c16 = lane & 15, kg = lane >> 4;

  for (int i = tid; i < 3 * SLOT / 16; i += 256)
    reinterpret_cast<uint4*>(ring)[i] = make_uint4(0u, 0u, 0u, 0u);   // incl. the padding columns

  // this wave's weights for its NPW n-tiles, all k-steps: B[k = (tap, ci)][co], lane (kg, c16)
  bf16x8_t bw[NPW][KS];
#pragma unroll
  for (int j = 0; j < NPW; ++j)
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int co = 16 * (wn * NPW + j) + c16;
      const int tap = s / KPT, tp = MODE == 1 ? 8 - tap : tap;
      const int ci = 32 * (s % KPT) + 8 * kg;
      bw[j][s] = *reinterpret_cast<const bf16x8_t*>(wk + ((long)co * 9 + tp) * CIN + ci);
    }

  const int r0 = (int)((long)blockIdx.x * rows / gridDim.x);
  const int r1 = (int)((long)(blockIdx.x + 1) * rows / gridDim.x);
  const int nvalid = min(MPW, MT - wm * MPW);   // this wave's m-tiles (uniform)
  // this wave's output pixels (the last m-tile of a 56-pixel row holds 8)
  const int npx = min(16 * (wm * MPW + nvalid), W) - 16 * wm * MPW;

  // forward statistics: running (n, mean, M2) of this wave's pixels per channel (lanes kg share)
  double rn = 0.0, rm[NPW], rq[NPW];
#pragma unroll
  for (int j = 0; j < NPW; ++j) { rm[j] = 0.0; rq[j] = 0.0; }
  // dgrad: the thread's 8 channels (fixed: 256 is a multiple of COUT / 8) and its partial sums
  constexpr int CG = COUT / 8, ITEMS = W * CG, IPT = (ITEMS + 255) / 256;
  const int cg = tid % CG;
  float esc[8], esh[8], emu[8];
  double ds[8], dq[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    esc[e] = (MODE == 1 && mask == 2) ? bsc[8 * cg + e] : 0.f;
    esh[e] = (MODE == 1 && mask == 2) ? bsh[8 * cg + e] : (mask == 0 ? 1.f : 0.f);
    emu[e] = MODE == 1 ? bmu[8 * cg + e] : 0.f;
    ds[e] = 0.0;
    dq[e] = 0.0;
  }

  uint4 setA[PI::PPT], setB[PI::PPT];
  auto first = [&](int row) { return row == r0 || row % h == 0; };
  auto slot = [&](int g) { return ring + ((g + 3) % 3) * SLOT; };   // g >= -1

  auto step = [&](int row, uint4 (&cur)[PI::PPT], uint4 (&nxt)[PI::PPT]) {
    const int oh = row % h;
    __syncthreads();   // the previous row's MFMAs / staged output are done
    if (first(row)) {
#pragma unroll 1
      for (int d = -1; d <= 1; ++d) {
        RowIO<CIN, W>::fetch(x, row + d, oh + d >= 0 && oh + d < h, cur);
        RowIO<CIN, W>::put(slot(row + d), 1, cur);
      }
    } else {
      RowIO<CIN, W>::put(slot(row + 1), 1, cur);   // (zeros past the frame's last row)
    }
    __syncthreads();
    // the next row's new input row lands under this row's MFMAs
    if (row + 1 < r1 && !first(row + 1)) RowIO<CIN, W>::fetch(x, row + 2, oh + 2 < h, nxt);
    // dgrad epilogue operands of this row (y, z, old dx), issued before the MFMAs
    uint4 yv[IPT], zv[IPT];
    float4 ov[IPT][2];
    if constexpr (MODE == 1) {
#pragma unroll
      for (int q = 0; q < IPT; ++q) {
        const int it = tid + 256 * q;
        const bool ok = it < ITEMS;
        const long e8 = (long)row * ITEMS + (ok ? it : 0);
        yv[q] = ok ? by[e8] : make_uint4(0u, 0u, 0u, 0u);
        zv[q] = (ok && mask == 1) ? bz[e8] : make_uint4(0u, 0u, 0u, 0u);
        if (!G16 && beta != 0.f && ok) {
          ov[q][0] = reinterpret_cast<const float4*>(out)[2 * e8];
          ov[q][1] = reinterpret_cast<const float4*>(out)[2 * e8 + 1];
        } else {
          ov[q][0] = ov[q][1] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }

    f32x4_t acc[MPW][NPW];
#pragma unroll
    for (int i = 0; i < MPW; ++i)
#pragma unroll
      for (int j = 0; j < NPW; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    const unsigned char* rb[3] = {slot(row - 1), slot(row), slot(row + 1)};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int tap = s / KPT, dy = tap / 3, dx = tap % 3;   // input row row - 1 + dy, column + dx - 1
      const unsigned char* p = rb[dy] + (dx + c16) * PI::PS + (64 * (s % KPT) + 16 * kg);
#pragma unroll
      for (int i = 0; i < MPW; ++i) {
        if (i < nvalid) {
          const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(p + 16 * (wm * MPW + i) * PI::PS);
#pragma unroll
          for (int j = 0; j < NPW; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[j][s], acc[i][j], 0, 0, 0);
        }
      }
    }

    if constexpr (MODE == 0) {
      // rounded values -> the staged tile + this wave's statistics (count 16 * nvalid per channel)
      unsigned short* ys = reinterpret_cast<unsigned short*>(ost);
      float sm[NPW];
#pragma unroll
      for (int j = 0; j < NPW; ++j) sm[j] = 0.f;
#pragma unroll
      for (int i = 0; i < MPW; ++i) {
        if (i < nvalid) {
#pragma unroll
          for (int j = 0; j < NPW; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int px = 16 * (wm * MPW + i) + 4 * kg + r, co = 16 * (wn * NPW + j) + c16;
              const unsigned short u = bfb(acc[i][j][r]);
              acc[i][j][r] = bff(u);   // (pixels past W: exactly 0, not counted)
              if (W % 16 == 0 || px < W) {
                ys[px * COUT + co] = u;
                sm[j] += acc[i][j][r];
              }
            }
        }
      }
      const float cnt = (float)npx;
      float mj[NPW], qj[NPW];
#pragma unroll
      for (int j = 0; j < NPW; ++j) {
        float t = sm[j] + __shfl_xor(sm[j], 16, 64);
        t += __shfl_xor(t, 32, 64);
        mj[j] = t / cnt;
        qj[j] = 0.f;
      }
#pragma unroll
      for (int i = 0; i < MPW; ++i) {
        if (i < nvalid) {
#pragma unroll
          for (int j = 0; j < NPW; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float d = acc[i][j][r] - mj[j];
              if (W % 16 == 0 || 16 * (wm * MPW + i) + 4 * kg + r < W) qj[j] = fmaf(d, d, qj[j]);
            }
        }
      }
      const double nb = (double)cnt, na = rn, nt = na + nb;
#pragma unroll
      for (int j = 0; j < NPW; ++j) {
        float t = qj[j] + __shfl_xor(qj[j], 16, 64);
        t += __shfl_xor(t, 32, 64);
        const double dd = (double)mj[j] - rm[j];
        rm[j] += dd * nb / nt;
        rq[j] += (double)t + dd * dd * na * nb / nt;
      }
      rn = nt;
      __syncthreads();   // the tile staged
      constexpr int YP = W * COUT * 2 / 16;
      uint4* yr = reinterpret_cast<uint4*>(out) + (long)row * YP;
      for (int i = tid; i < YP; i += 256) yr[i] = reinterpret_cast<const uint4*>(ost)[i];
    } else {
      // fp32 dx tile -> LDS (rows of COUT + 4 floats), then 8 channels per thread
      float* gs = reinterpret_cast<float*>(ost);
#pragma unroll
      for (int i = 0; i < MPW; ++i) {
        if (i < nvalid) {
#pragma unroll
          for (int j = 0; j < NPW; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int px = 16 * (wm * MPW + i) + 4 * kg + r, co = 16 * (wn * NPW + j) + c16;
              if (W % 16 == 0 || px < W) gs[px * (COUT + 4) + co] = acc[i][j][r];
            }
        }
      }
      __syncthreads();
      float rs[8], rqq[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) { rs[e] = 0.f; rqq[e] = 0.f; }
#pragma unroll
      for (int q = 0; q < IPT; ++q) {
        const int it = tid + 256 * q;
        if (it < ITEMS) {
          const int px = it / CG;
          const float4 a0 = *reinterpret_cast<const float4*>(gs + px * (COUT + 4) + 8 * cg);
          const float4 a1 = *reinterpret_cast<const float4*>(gs + px * (COUT + 4) + 8 * cg + 4);
          const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
          const float ol[8] = {ov[q][0].x, ov[q][0].y, ov[q][0].z, ov[q][0].w,
                               ov[q][1].x, ov[q][1].y, ov[q][1].z, ov[q][1].w};
          const uint32_t yu[4] = {yv[q].x, yv[q].y, yv[q].z, yv[q].w};
          const uint32_t zu[4] = {zv[q].x, zv[q].y, zv[q].z, zv[q].w};
          float g[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float yy = (e & 1) ? __uint_as_float(yu[e >> 1] & 0xffff0000u) : bff(yu[e >> 1] & 0xffffu);
            const float zz = (e & 1) ? __uint_as_float(zu[e >> 1] & 0xffff0000u) : bff(zu[e >> 1] & 0xffffu);
            float t = fmaf(beta, ol[e], av[e]);
            const bool keep = zz + fmaf(yy, esc[e], esh[e]) > 0.f;   // the engine's mask test
            t = keep ? t : 0.f;
            if (G16) t = bff(bfb(t));   // the stored value, which the partial sums describe
            g[e] = t;
            rs[e] += t;
            rqq[e] = fmaf(t, yy - emu[e], rqq[e]);
          }
          if constexpr (G16) {
            uint32_t pk[4];
#pragma unroll
            for (int e2 = 0; e2 < 4; ++e2)
              pk[e2] = (uint32_t)bfb(g[2 * e2]) | ((uint32_t)bfb(g[2 * e2 + 1]) << 16);
            reinterpret_cast<uint4*>(out)[(long)row * ITEMS + it] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
          } else {
            float4* o = reinterpret_cast<float4*>(out) + 2 * ((long)row * ITEMS + it);
            o[0] = make_float4(g[0], g[1], g[2], g[3]);
            o[1] = make_float4(g[4], g[5], g[6], g[7]);
          }
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        ds[e] += (double)rs[e];
        dq[e] += (double)rqq[e];
      }
    }
  };
  for (int row = r0; row < r1; row += 2) {
    step(row, setA, setB);
    if (row + 1 < r1) step(row + 1, setB, setA);
  }

  if constexpr (MODE == 0) {
    if (kg == 0) {
#pragma unroll
      for (int j = 0; j < NPW; ++j)
        stats[((long)blockIdx.x * WM + wm) * COUT + 16 * (wn * NPW + j) + c16] =
            make_float4((float)rn, (float)rm[j], (float)rq[j], 0.f);
    }
  } else {
    // the workgroup's partial row: per channel, the threads with this channel group (lanes
    // l = cg mod CG of each wave, then the four waves) summed in a fixed order
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      for (int m = CG; m < 64; m <<= 1) {
        ds[e] += __shfl_xor(ds[e], m, 64);
        dq[e] += __shfl_xor(dq[e], m, 64);
      }
    }
    __syncthreads();
    double* red = reinterpret_cast<double*>(ost);   // [4 waves][COUT][2]
    if (lane < CG) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(wave * COUT + 8 * lane + e) * 2] = ds[e];
        red[(wave * COUT + 8 * lane + e) * 2 + 1] = dq[e];
      }
    }
    __syncthreads();
    for (int c = tid; c < COUT; c += 256) {
      double t0 = 0.0, t1 = 0.0;
      for (int w = 0; w < 4; ++w) {
        t0 += red[(w * COUT + c) * 2];
        t1 += red[(w * COUT + c) * 2 + 1];
      }
      part[(long)blockIdx.x * COUT + c] = make_float2((float)t0, (float)t1);
    }
  }
}

// Weight gradient dW[co][tap][ci] = sum over output pixels p of dy[p][co] * x[p + off(tap)][ci]:
// per output row, A = the dy row (co x 128 pixels, pixels >= 112 zero), B = the input row of the
// tap's kernel row shifted by its column offset (128 pixels x ci), both [pixel][channel] images read
// by ds_read_b64_tr_b16.  Wave split: COUT 64 -> wave w owns co tile w (both ci tiles, 9 taps);
// COUT 32 -> (co tile w & 1, ci tile w >> 1).
template <int CIN, int COUT, int W = DW>
__global__ __launch_bounds__(256, 2)
void d3w_k(const uint4* __restrict__ x, const uint4* __restrict__ dy, float* __restrict__ slabs,
           int h, int rows) {
  using PI = Px<CIN, W>;
  using PO = Px<COUT, W>;
  constexpr int KP = 32 * ((W + 31) / 32);   // reduction pixels per row, zero-padded
  constexpr int XR = KP + 2;                 // ring slot rows: pixel columns x = -1 .. KP
  constexpr int XSLOT = XR * PI::PS;
  // tiles per wave: COUT 64 -> co tile w, all CIN / 16 ci tiles; COUT 32 (CIN 32) -> co tile w & 1,
  // ci tile w >> 1
  constexpr int NTW = COUT == 64 ? CIN / 16 : 1;
  static_assert((COUT == 64 && (CIN == 32 || CIN == 64)) || (COUT == 32 && CIN == 32),
                "d3w_k: (32 | 64) -> 64 or 32 -> 32 channels");
  __shared__ __attribute__((aligned(16))) unsigned char ring[3 * XSLOT];
  __shared__ __attribute__((aligned(16))) unsigned char dimg[KP * PO::PS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int tq = li >> 2, tp = li & 3;
  const int mt = COUT == 64 ? wave : (wave & 1);
  const int nt0 = COUT == 64 ? 0 : (wave >> 1);
  for (int i = tid; i < 3 * XSLOT / 16; i += 256)
    reinterpret_cast<uint4*>(ring)[i] = make_uint4(0u, 0u, 0u, 0u);
  for (int i = tid; i < KP * PO::PS / 16; i += 256)
    reinterpret_cast<uint4*>(dimg)[i] = make_uint4(0u, 0u, 0u, 0u);

  f32x4_t acc[9][NTW];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[t][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const int r0 = (int)((long)blockIdx.x * rows / gridDim.x);
  const int r1 = (int)((long)(blockIdx.x + 1) * rows / gridDim.x);
  auto first = [&](int row) { return row == r0 || row % h == 0; };
  auto slot = [&](int gg) { return ring + ((gg + 3) % 3) * XSLOT; };

  // transposed fragment: 8 consecutive pixel rows pr .. pr + 7 (this lane's group's), columns
  // cb .. cb + 15 -> element j = row pr + j of column cb + li; the odd groups read their upper 4
  // rows first (conflict-free pairing), swapped back here
  auto frag = [&](const unsigned char* img, int stride, int pr, int cb) -> bf16x8_t {
    const int hi = g & 1;
    const unsigned char* p = img + (pr + tq) * stride + (cb + 4 * tp) * 2;
    const s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4_t*)(p + 4 * hi * stride));
    const s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4_t*)(p + 4 * (hi ^ 1) * stride));
    const s16x4_t lo = hi ? v1 : v0, up = hi ? v0 : v1;
    const s16x8_t w = __builtin_shufflevector(lo, up, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8_t, w);
  };

  uint4 xA[PI::PPT], xB[PI::PPT], dA[PO::PPT], dB[PO::PPT];
  if (r0 < r1) RowIO<COUT, W>::fetch(dy, r0, true, dA);
  auto step = [&](int row, uint4 (&xc)[PI::PPT], uint4 (&xn)[PI::PPT], uint4 (&dc)[PO::PPT],
                  uint4 (&dn)[PO::PPT]) {
    const int oh = row % h;
    __syncthreads();   // the previous row's fragments are read
    if (first(row)) {
#pragma unroll 1
      for (int d = -1; d <= 1; ++d) {
        RowIO<CIN, W>::fetch(x, row + d, oh + d >= 0 && oh + d < h, xc);
        RowIO<CIN, W>::put(slot(row + d), 1, xc);
      }
    } else {
      RowIO<CIN, W>::put(slot(row + 1), 1, xc);
    }
    RowIO<COUT, W>::put(dimg, 0, dc);
    __syncthreads();
    if (row + 1 < r1) {
      if (!first(row + 1)) RowIO<CIN, W>::fetch(x, row + 2, oh + 2 < h, xn);
      RowIO<COUT, W>::fetch(dy, row + 1, true, dn);
    }
    const unsigned char* rb[3] = {slot(row - 1), slot(row), slot(row + 1)};
    // B fragments read three (tap, ci tile) pairs ahead of their MFMA (7% on the 112-wide
    // 32 -> 64 wgrad; the same LDS reads, fewer exposed latencies)
    constexpr int Q = 9 * NTW, LA = 3;
    auto ldB = [&](int pr, int q) -> bf16x8_t {
      const int t = q / NTW, j = q % NTW, ky = t / 3, kx = t % 3;   // x pixel p + kx - 1 = row p + kx
      return frag(rb[ky], PI::PS, pr + kx, 16 * (nt0 + j));
    };
#pragma unroll
    for (int s = 0; s < KP / 32; ++s) {   // pixels 32 s .. 32 s + 31
      const int pr = 32 * s + 8 * g;
      const bf16x8_t a = frag(dimg, PO::PS, pr, 16 * mt);
      bf16x8_t bq[Q];
#pragma unroll
      for (int q = 0; q < LA; ++q) bq[q] = ldB(pr, q);
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        if (q + LA < Q) bq[q + LA] = ldB(pr, q + LA);
        acc[q / NTW][q % NTW] =
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bq[q], acc[q / NTW][q % NTW], 0, 0, 0);
      }
    }
  };
  for (int row = r0; row < r1; row += 2) {
    step(row, xA, xB, dA, dB);
    if (row + 1 < r1) step(row + 1, xB, xA, dB, dA);
  }
  // this wave's tiles -> the workgroup's slab, layout (co * 9 + tap) * CIN + ci
  float* slab = slabs + (long)blockIdx.x * (COUT * 9 * CIN);
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = 16 * mt + 4 * g + r, ci = 16 * (nt0 + j) + li;
        slab[((long)co * 9 + t) * CIN + ci] = acc[t][j][r];
      }
}

// ---- the deep stem's first conv: 3x3 / stride 2 / pad 1, 3 -> 32 channels, 224 -> 112 ----
// From the NHWC4 fp32 input (rounded to bf16 when published; the 4th channel ignored), packed per
// input row as 3 channels per column (columns x = -1 .. 226): the 3 taps x 3 channels of one
// kernel row at output column ow are the 9 consecutive values from element 6 ow.  The reduction
// runs over 4 kernel rows of 16 (9 real: 27 of 64 multiplies, the 4th row zero weights) -- two
// k-steps of v_mfma_f32_16x16x32_bf16, each lane's 8 values four ds_read_b32 at 12 ow + 16 h bytes.
// Input rows 2 oh - 1 .. 2 oh + 1 in a ring of 3 (slot (r + 3) % 3; consecutive output rows share
// one), the 2 new rows of the next output row prefetched into registers.
constexpr int SXR = 688;   // packed row: 229 columns x 3 channels = 687, padded
constexpr int SW2 = 224;   // input width

struct StemRows {
  const float4* x;
  int hin;
  // rows r, r + 1 of the frame starting at global input row g0 (r + k < hin), two float4 per thread
  __device__ void fetch2(long g0, int r, float4 (&v)[2]) const {
    int tt = threadIdx.x;
    asm volatile("" : "+v"(tt));
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int i = tt + 256 * q, k = i / SW2, col = i % SW2;
      v[q] = (r + k >= 0 && r + k < hin) ? x[(g0 + r + k) * SW2 + col] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
};

__device__ __forceinline__ void put_px3(unsigned short* row, int col, float4 v) {
  unsigned short* d = row + (col + 1) * 3;
  d[0] = bfb(v.x); d[1] = bfb(v.y); d[2] = bfb(v.z);
}

__global__ __launch_bounds__(256, 3)
void d3s_k(const float4* __restrict__ x, const __bf16* __restrict__ wk, __bf16* __restrict__ y,
           float4* __restrict__ stats, int hin, int ho, int rows) {
  constexpr int COUT = 32, MPW = 2;
  __shared__ __attribute__((aligned(16))) unsigned short ring[3 * SXR];
  __shared__ __attribute__((aligned(16))) unsigned short ys[DW * COUT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c16 = lane & 15, kg = lane >> 4;
  for (int i = tid; i < 3 * SXR / 2; i += 256) reinterpret_cast<uint32_t*>(ring)[i] = 0u;
  // weights: B[k = 32 s + 8 kg + e][co]: chunk m = 4 s + kg = (kernel row m / 2, half m % 2),
  // k' = 8 (m % 2) + e = 3 kw + c (< 9), KRSC (32, 3, 3, 4) bf16
  bf16x8_t bw[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int m = 4 * s + kg, kh = m >> 1, co = 16 * j + c16;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int kk = 8 * (m & 1) + e, kw = kk / 3, c = kk % 3;
        bw[j][s][e] = (kh < 3 && kk < 9) ? wk[((co * 3 + kh) * 3 + kw) * 4 + c] : (__bf16)0.f;
      }
    }
  const int r0 = (int)((long)blockIdx.x * rows / gridDim.x);
  const int r1 = (int)((long)(blockIdx.x + 1) * rows / gridDim.x);
  const int nvalid = min(MPW, 7 - wave * MPW);
  double rn = 0.0, rm[2] = {0.0, 0.0}, rq[2] = {0.0, 0.0};
  StemRows feed{x, hin};
  auto first = [&](int row) { return row == r0 || row % ho == 0; };
  auto slot = [&](int r) { return ring + ((r + 3) % 3) * SXR; };
  float4 setA[2], setB[2];
  auto step = [&](int row, float4 (&cur)[2], float4 (&nxt)[2]) {
    const int oh = row % ho;
    const long g0 = (long)(row / ho) * hin;   // the frame's first input row
    __syncthreads();
    // publish rows r .. r + nr - 1 of a two-row register set (nr = 1: row r + 1 would overwrite
    // the slot of row r - 2, which the ring of 3 still holds as 2 oh - 1)
    auto put2 = [&](int r, const float4 (&v)[2], int nr) {
      int tt = threadIdx.x;
      asm volatile("" : "+v"(tt));
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int i = tt + 256 * q, k = i / SW2, col = i % SW2;
        if (k < nr) put_px3(slot(r + k), col, v[q]);
      }
    };
    if (first(row)) {
      feed.fetch2(g0, 2 * oh - 1, cur);
      put2(2 * oh - 1, cur, 2);
      feed.fetch2(g0, 2 * oh + 1, cur);
      put2(2 * oh + 1, cur, 1);
    } else {
      put2(2 * oh, cur, 2);
    }
    __syncthreads();
    if (row + 1 < r1 && !first(row + 1)) feed.fetch2(g0, 2 * oh + 2, nxt);
    f32x4_t acc[MPW][2];
#pragma unroll
    for (int i = 0; i < MPW; ++i) acc[i][0] = acc[i][1] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int m = 4 * s + kg, kh = min(m >> 1, 2);   // (kernel row 3: zero weights)
      const unsigned short* rp = slot(2 * oh - 1 + kh) + 8 * (m & 1);
#pragma unroll
      for (int i = 0; i < MPW; ++i) {
        if (i < nvalid) {
          const int ow = 16 * (wave * MPW + i) + c16;
          const uint32_t* pa = reinterpret_cast<const uint32_t*>(rp + 6 * ow);
          uint4 av;
          av.x = pa[0]; av.y = pa[1]; av.z = pa[2]; av.w = pa[3];
          const bf16x8_t a = __builtin_bit_cast(bf16x8_t, av);
          acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[0][s], acc[i][0], 0, 0, 0);
          acc[i][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[1][s], acc[i][1], 0, 0, 0);
        }
      }
    }
    float sm[2] = {0.f, 0.f};
#pragma unroll
    for (int i = 0; i < MPW; ++i) {
      if (i < nvalid) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int px = 16 * (wave * MPW + i) + 4 * kg + r, co = 16 * j + c16;
            const unsigned short u = bfb(acc[i][j][r]);
            acc[i][j][r] = bff(u);
            ys[px * COUT + co] = u;
            sm[j] += acc[i][j][r];
          }
      }
    }
    const float cnt = 16.f * nvalid;
    float mj[2], qj[2] = {0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float t = sm[j] + __shfl_xor(sm[j], 16, 64);
      t += __shfl_xor(t, 32, 64);
      mj[j] = t / cnt;
    }
#pragma unroll
    for (int i = 0; i < MPW; ++i) {
      if (i < nvalid) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float d = acc[i][j][r] - mj[j];
            qj[j] = fmaf(d, d, qj[j]);
          }
      }
    }
    const double nb = (double)cnt, na = rn, nt = na + nb;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float t = qj[j] + __shfl_xor(qj[j], 16, 64);
      t += __shfl_xor(t, 32, 64);
      const double dd = (double)mj[j] - rm[j];
      rm[j] += dd * nb / nt;
      rq[j] += (double)t + dd * dd * na * nb / nt;
    }
    rn = nt;
    __syncthreads();
    uint4* yr = reinterpret_cast<uint4*>(y) + (long)row * (DW * COUT / 8);
    for (int i = tid; i < DW * COUT / 8; i += 256) yr[i] = reinterpret_cast<const uint4*>(ys)[i];
  };
  for (int row = r0; row < r1; row += 2) {
    step(row, setA, setB);
    if (row + 1 < r1) step(row + 1, setB, setA);
  }
  if (kg == 0) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
      stats[((long)blockIdx.x * 4 + wave) * COUT + 16 * j + c16] =
          make_float4((float)rn, (float)rm[j], (float)rq[j], 0.f);
  }
}

// Its weight gradient: dW[co][kh][kw][c] = sum over output pixels of dy[p][co] * x[2 oh - 1 + kh]
// [2 ow - 1 + kw][c].  Per output row: A = the dy row (co x 128 pixels) by transposed reads as in
// d3w_k; B = per input row its im2col columns transposed, XI[slot][kw * 3 + c][p] (input column
// col = 2 p - 1 + kw; built from each pixel's 3 values into the 1-2 kernel columns of its parity),
// so a B fragment (8 consecutive pixels of one column k' = 9 kh + 3 kw + c) is one ds_read_b128.
// Wave w: co tile w & 1, k' tile w >> 1 (k' 0..31, 27 real).
constexpr int XPL = 136;   // pixels per XI row (128 + 8 pad: 272-B rows)

__global__ __launch_bounds__(256, 2)
void d3sw_k(const float4* __restrict__ x, const uint4* __restrict__ dy, float* __restrict__ slabs,
            int hin, int ho, int rows) {
  using PO = Px<32>;
  __shared__ __attribute__((aligned(16))) unsigned short xi[3 * 9 * XPL + XPL];   // + a zero row
  __shared__ __attribute__((aligned(16))) unsigned char dimg[128 * PO::PS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4, tq = li >> 2, tp = li & 3;
  const int mt = wave & 1, nt = wave >> 1;
  for (int i = tid; i < (3 * 9 * XPL + XPL) / 2; i += 256) reinterpret_cast<uint32_t*>(xi)[i] = 0u;
  for (int i = tid; i < 128 * PO::PS / 16; i += 256)
    reinterpret_cast<uint4*>(dimg)[i] = make_uint4(0u, 0u, 0u, 0u);
  unsigned short* const zrow = xi + 3 * 9 * XPL;
  const int r0 = (int)((long)blockIdx.x * rows / gridDim.x);
  const int r1 = (int)((long)(blockIdx.x + 1) * rows / gridDim.x);
  StemRows feed{x, hin};
  auto first = [&](int row) { return row == r0 || row % ho == 0; };
  auto xslot = [&](int r) { return xi + ((r + 3) % 3) * 9 * XPL; };
  // input pixel (row r, column col) -> its im2col columns: p = (col + 1 - kw) / 2 when even
  auto put2 = [&](int r, const float4 (&v)[2], int nr) {   // (nr: as d3s_k)
    int tt = threadIdx.x;
    asm volatile("" : "+v"(tt));
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int i = tt + 256 * q, k = i / SW2, col = i % SW2;
      if (k >= nr) continue;
      unsigned short* blk = xslot(r + k);
      const unsigned short u[3] = {bfb(v[q].x), bfb(v[q].y), bfb(v[q].z)};
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int t = col + 1 - kw;
        if ((t & 1) == 0 && t >= 0 && t < 2 * DW) {
#pragma unroll
          for (int c = 0; c < 3; ++c) blk[(kw * 3 + c) * XPL + (t >> 1)] = u[c];
        }
      }
    }
  };
  auto frag_a = [&](int pr) -> bf16x8_t {   // as d3w_k's transposed fragment (dy image)
    const int hi = g & 1;
    const unsigned char* p = dimg + (pr + tq) * PO::PS + (16 * mt + 4 * tp) * 2;
    const s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4_t*)(p + 4 * hi * PO::PS));
    const s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4_t*)(p + 4 * (hi ^ 1) * PO::PS));
    const s16x4_t lo = hi ? v1 : v0, up = hi ? v0 : v1;
    return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, up, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  f32x4_t acc = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  float4 xA[2], xB[2];
  uint4 dA[PO::PPT], dB[PO::PPT];
  if (r0 < r1) RowIO<32>::fetch(dy, r0, true, dA);
  auto step = [&](int row, float4 (&xc)[2], float4 (&xn)[2], uint4 (&dc)[PO::PPT],
                  uint4 (&dn)[PO::PPT]) {
    const int oh = row % ho;
    const long g0 = (long)(row / ho) * hin;
    __syncthreads();
    // (rows outside the frame are fetched as zeros and published like any other: every im2col
    // entry a real pixel can write is overwritten, the rest stays zero from the start)
    if (first(row)) {
      feed.fetch2(g0, 2 * oh - 1, xc);
      put2(2 * oh - 1, xc, 2);
      feed.fetch2(g0, 2 * oh + 1, xc);
      put2(2 * oh + 1, xc, 1);
    } else {
      put2(2 * oh, xc, 2);
    }
    RowIO<32>::put(dimg, 0, dc);
    __syncthreads();
    if (row + 1 < r1) {
      if (!first(row + 1)) feed.fetch2(g0, 2 * oh + 2, xn);
      RowIO<32>::fetch(dy, row + 1, true, dn);
    }
    // B column k' = 16 nt + li: kernel row k' / 9, im2col column k' % 9 (k' >= 27: zero row)
    const int kk = 16 * nt + li;
    const unsigned short* pb = kk < 27 ? xslot(2 * oh - 1 + kk / 9) + (kk % 9) * XPL : zrow;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int pr = 32 * s + 8 * g;
      const bf16x8_t a = frag_a(pr);
      const bf16x8_t b = *reinterpret_cast<const bf16x8_t*>(pb + pr);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    }
  };
  for (int row = r0; row < r1; row += 2) {
    step(row, xA, xB, dA, dB);
    if (row + 1 < r1) step(row + 1, xB, xA, dB, dA);
  }
  // slab layout of the engine's 4-channel stem wgrad: (co * 9 + tap) * 4 + c
  float* slab = slabs + (long)blockIdx.x * (32 * 9 * 4);
  const int kk = 16 * nt + li;
  if (kk < 27) {
    const int kh = kk / 9, kw = (kk % 9) / 3, c = kk % 3;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = 16 * mt + 4 * g + r;
      slab[(co * 9 + kh * 3 + kw) * 4 + c] = acc[r];
    }
  }
}

constexpr int kGridW = 2 * 256;

int grid_of(int rows, int cin, int cout, int mode) {
  const int g = d3_minb(cin, cout, mode) * 256;
  return rows < g ? rows : g;
}

}  // namespace

// ---- host entries (gemm_conv.hip routes the deep stem's geometry here) ----

// supported (width, input, output channels) of the forward / wgrad; the dgrad takes the same convs
static bool d3_ok(int w, int cin, int cout) {
  return (w == 112 && cin == 32 && (cout == 32 || cout == 64)) ||
         (w == 56 && cin == 64 && cout == 64);
}

int tmr_d3_stats_parts(int n, int h, int w, int cin, int cout) {
  const int ks = 9 * cin / 32, npw = 18 / ks, wn = (cout / 16) / npw, wm = 4 / wn;   // d3_k's WM
  return grid_of(n * h, cin, cout, 0) * wm;
}

int tmr_d3_dgrad_parts(int n, int h, int w, int cin_conv, int cout_conv) {
  (void)w;
  return grid_of(n * h, cout_conv, cin_conv, 1);   // the dgrad kernel runs over dy
}

size_t tmr_d3_wgrad_ws_bytes(int n, int h, int w, int cin, int cout) {
  (void)w;
  const int rows = n * h;
  return (size_t)(rows < kGridW ? rows : kGridW) * cout * 9 * cin * sizeof(float);
}

int tmr_d3_fwd_bnstats(int n, int h, int w, int cin, int cout, const void* x, const void* w_krsc,
                       void* y, void* stats, hipStream_t stream) {
  TMR_CHECK_ARG(n > 0 && h > 0 && d3_ok(w, cin, cout), "tmr_d3_fwd: unsupported shape (w %d, %d -> %d)",
                w, cin, cout);
  TMR_CHECK_ARG((((uintptr_t)x | (uintptr_t)y | (uintptr_t)w_krsc) & 15) == 0,
                "tmr_d3_fwd: x / y / w must be 16-B aligned");
  const int rows = n * h, grid = grid_of(rows, cin, cout, 0);
#define D3F(CI, CO, W)                                                                            \
  hipLaunchKernelGGL((d3_k<CI, CO, 0, W>), dim3(grid), dim3(256), 0, stream, (const uint4*)x,     \
                     (const __bf16*)w_krsc, y, (float4*)stats, nullptr, nullptr, nullptr, nullptr, \
                     nullptr, 0, 0.f, nullptr, h, rows)
  if (w == 56) D3F(64, 64, 56);
  else if (cout == 64) D3F(32, 64, 112);
  else D3F(32, 32, 112);
#undef D3F
  TMR_CHECK_LAUNCH("d3_fwd");
  return 0;
}

// dgrad of the conv cin_conv -> cout_conv: dy (rows, w, cout_conv) bf16, w_crsk (cin_conv, 3, 3,
// cout_conv) bf16, dx (rows, w, cin_conv) fp32 (read when beta != 0), or bf16 when g16 (the masked
// gradient rounded, no beta); the BatchNorm backward of the unit that produced the conv input:
// y / z bf16 like dx, mask 0 / 1 / 2
int tmr_d3_dgrad_bnbwd(int n, int h, int w, int cin_conv, int cout_conv, const void* dy,
                       const void* w_crsk, void* dx, int g16, float beta, const void* y,
                       const void* z, const float* scale, const float* shift, const float* mean,
                       int mask, void* parts, hipStream_t stream) {
  TMR_CHECK_ARG(n > 0 && h > 0 && d3_ok(w, cin_conv, cout_conv) && (!g16 || w == 56) &&
                    !(g16 && beta != 0.f),
                "tmr_d3_dgrad: unsupported shape (w %d, %d -> %d, g16 %d, beta %g)", w, cin_conv,
                cout_conv, g16, beta);
  TMR_CHECK_ARG((((uintptr_t)dy | (uintptr_t)dx | (uintptr_t)w_crsk | (uintptr_t)y |
                  (uintptr_t)z) & 15) == 0,
                "tmr_d3_dgrad: operands must be 16-B aligned");
  TMR_CHECK_ARG(mask == 0 || (mask == 1 && z) || (mask == 2 && scale && shift),
                "tmr_d3_dgrad: mask %d operands", mask);
  const int rows = n * h, grid = grid_of(rows, cout_conv, cin_conv, 1);
#define D3D(CI, CO, W, G)                                                                         \
  hipLaunchKernelGGL((d3_k<CI, CO, 1, W, G>), dim3(grid), dim3(256), 0, stream, (const uint4*)dy, \
                     (const __bf16*)w_crsk, dx, nullptr, (const uint4*)y, (const uint4*)z, scale,  \
                     shift, mean, mask, beta, (float2*)parts, h, rows)
  if (w == 56 && g16) D3D(64, 64, 56, 1);
  else if (w == 56) D3D(64, 64, 56, 0);
  else if (cout_conv == 64) D3D(64, 32, 112, 0);
  else D3D(32, 32, 112, 0);
#undef D3D
  TMR_CHECK_LAUNCH("d3_dgrad");
  return 0;
}

int tmr_d3_wgrad_slabs(int n, int h, int w, int cin, int cout, const void* x, const void* dy,
                       float* ws, size_t ws_bytes, int* nslabs, hipStream_t stream) {
  TMR_CHECK_ARG(n > 0 && h > 0 && d3_ok(w, cin, cout), "tmr_d3_wgrad: unsupported shape (w %d, %d -> %d)",
                w, cin, cout);
  TMR_CHECK_ARG((((uintptr_t)x | (uintptr_t)dy) & 15) == 0, "tmr_d3_wgrad: x / dy must be 16-B aligned");
  const int rows = n * h, grid = rows < kGridW ? rows : kGridW;
  TMR_CHECK_ARG(ws && ws_bytes >= tmr_d3_wgrad_ws_bytes(n, h, w, cin, cout),
                "tmr_d3_wgrad: workspace too small (%zu)", ws_bytes);
  if (w == 56)
    hipLaunchKernelGGL((d3w_k<64, 64, 56>), dim3(grid), dim3(256), 0, stream, (const uint4*)x,
                       (const uint4*)dy, ws, h, rows);
  else if (cout == 64)
    hipLaunchKernelGGL((d3w_k<32, 64>), dim3(grid), dim3(256), 0, stream, (const uint4*)x,
                       (const uint4*)dy, ws, h, rows);
  else
    hipLaunchKernelGGL((d3w_k<32, 32>), dim3(grid), dim3(256), 0, stream, (const uint4*)x,
                       (const uint4*)dy, ws, h, rows);
  TMR_CHECK_LAUNCH("d3_wgrad");
  *nslabs = grid;
  return 0;
}

// the deep stem's first conv (3x3/2, 3 -> 32 on the NHWC4 fp32 input): stats partial rows
int tmr_d3s_stats_parts(int n, int ho) {
  const int rows = n * ho;
  return 4 * (rows < 3 * 256 ? rows : 3 * 256);
}

int tmr_d3s_fwd_bnstats(int n, int h, const float* x, const void* w_krsc, void* y, void* stats,
                        hipStream_t stream) {
  TMR_CHECK_ARG(n > 0 && h > 0 && h % 2 == 0, "tmr_d3s_fwd: unsupported height %d", h);
  TMR_CHECK_ARG((((uintptr_t)x | (uintptr_t)y) & 15) == 0, "tmr_d3s_fwd: x / y must be 16-B aligned");
  const int ho = h / 2, rows = n * ho, grid = rows < 3 * 256 ? rows : 3 * 256;
  hipLaunchKernelGGL(d3s_k, dim3(grid), dim3(256), 0, stream, (const float4*)x,
                     (const __bf16*)w_krsc, (__bf16*)y, (float4*)stats, h, ho, rows);
  TMR_CHECK_LAUNCH("d3s_fwd");
  return 0;
}

size_t tmr_d3s_wgrad_ws_bytes(int n, int ho) {
  const int rows = n * ho;
  return (size_t)(rows < kGridW ? rows : kGridW) * 32 * 9 * 4 * sizeof(float);
}

int tmr_d3s_wgrad_slabs(int n, int h, const float* x, const void* dy, float* ws, size_t ws_bytes,
                        int* nslabs, hipStream_t stream) {
  TMR_CHECK_ARG(n > 0 && h > 0 && h % 2 == 0, "tmr_d3s_wgrad: unsupported height %d", h);
  TMR_CHECK_ARG((((uintptr_t)x | (uintptr_t)dy) & 15) == 0, "tmr_d3s_wgrad: x / dy must be 16-B aligned");
  const int ho = h / 2, rows = n * ho, grid = rows < kGridW ? rows : kGridW;
  TMR_CHECK_ARG(ws && ws_bytes >= tmr_d3s_wgrad_ws_bytes(n, ho), "tmr_d3s_wgrad: workspace too small");
  hipLaunchKernelGGL(d3sw_k, dim3(grid), dim3(256), 0, stream, (const float4*)x, (const uint4*)dy,
                     ws, h, ho, rows);
  TMR_CHECK_LAUNCH("d3s_wgrad");
  *nslabs = grid;
  return 0;
}

// Implicit-GEMM convolution / GEMM engine, fp32 in / fp32 accumulate on the
// gfx950 f32-input matrix cores (v_mfma_f32_32x32x2_f32, exact fp32 FMA chain).
//
// One templated kernel serves three GEMM views of a 2-D convolution on NHWC
// activations (and plain GEMMs as the 1x1 / 1-pixel special case):
//
//   FWD   : C[m=(n,ho,wo)][j=co]  = sum_{k=(tap,c)}  X[src(m,tap)][c]  * W[co][tap][c]
//   DGRAD : C[m=(n,h,w)][j=ci]    = sum_{k=(tap,co)} dY[src(m,tap)][co] * W[co][tap][ci]
//           (one launch per stride-parity class, so no zero taps are multiplied)
//   WGRAD : C[i=co][j=(tap,c)]    = sum_{m=(n,ho,wo)} dY[m][co] * X[src(m,tap)][c]
//           (reduction split over blockIdx.y into fp32 partial slabs, reduced in
//            a fixed order afterwards -> deterministic)
//
// Replaces the cuDNN Conv2d fwd/dgrad/wgrad and cuBLAS Linear GEMMs the
// reference reaches through torchvision resnet50 / nn.Linear / nn.LSTM
// (code/Training TMRNet/train_only_non-local_pretrained.py:204-240).
//
// Block = 256 threads = 4 waves, tile BM x BN x 16, each wave a
// (BM/WM) x (BN/WN) sub-tile of 32x32 MFMA tiles.  Global->register prefetch of
// tile t+1 overlaps the MFMAs on tile t (double-buffered LDS, one barrier per
// k-tile).  LDS tiles are k-major ([16][BM+pad]) so each MFMA operand read is a
// conflict-free ds_read_b32 of 32 consecutive floats per half-wave.
#include "common.h"
#include "tmr.h"
#include <stdlib.h>

namespace {

enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };
#ifndef TMR_PF
#define TMR_PF 2
#endif
#ifndef TMR_GEMM_WAVES
#define TMR_GEMM_WAVES 3
#endif
#if TMR_GEMM_WAVES > 0
// f32 8-wave workgroups (256x128, 128x256, BK 16) are held to 128 VGPRs: two workgroups per CU, so one
// workgroup's epilogue stores overlap the other's main loop (short-reduction GEMMs)
#define TMR_GEMM_LB __launch_bounds__(64 * WM * WN, (WM * WN == 8 && PREC == 0 && BK == 16 ? 4 : TMR_GEMM_WAVES))
#else
#define TMR_GEMM_LB __launch_bounds__(64 * WM * WN)
#endif

struct GemmArgs {
  const float* A;
  const float* B;
  float* C;
  const float* bias;
  int M, N, K;
  // K-index (FWD/DGRAD) or column-index (WGRAD) decomposition into (tap, channel)
  int log2C, ntaps, tapS, tapSinv;
  int oy0, ox0, dyr, dxs;   // source offset of tap (ri,si) = (oy0 + dyr*ri, ox0 + dxs*si)
  int wr0, ws0, wst, wS;    // DGRAD weight tap index = (wr0 + wst*ri)*wS + (ws0 + wst*si)
  // gather geometry: row -> (n,y,x) on the grid, source pixel (y*sy+oy, x*sx+ox)
  FastDiv dHW, dW;
  int Hs, Ws, sy, sx;
  int lds;   // source pixel stride (elements)
  int ldb;   // FWD: B row stride; DGRAD: stride per co; WGRAD: dY row stride
  // output
  int ldc;
  float beta;
  int oH, oW, osy, osx, oyc, oxc;  // DGRAD output-pixel map of the row grid (n, y, x)
  // WGRAD split-K
  int kchunk;
  long slab;
  // FWD: optional per-(m-tile, column) BatchNorm partials (n, mean, M2, 0)
  float4* stats;
  // FWD inference epilogue: C = [relu](fmaf(acc, scale, bias) + res), res laid out like C
  // (eval-mode BatchNorm, the residual add and ReLU of a Bottleneck fused into the conv)
  const float* scale;
  const float* res;
  int relu;
  // DGRAD epilogue fused with the backward of the BatchNorm(+ReLU) whose output gradient this
  // dgrad produces: C = relu-mask(C) (mask 1: bn_z > 0, 2: fmaf(bn_y, bn_sc, bn_sh) > 0) and
  // per-(m-tile, column) partials (sum g, sum g * (bn_y - bn_mean)) -> bn_part (float2)
  const float* bn_y;
  const float* bn_z;
  const float* bn_sc;
  const float* bn_sh;
  const float* bn_mean;
  float2* bn_part;
  int bn_mask;
  // byte extents of A, B and C (buffer-descriptor range checks; C's also bounds the tensors
  // laid out like C: res, bn_y, bn_z; WGRAD: one split slab)
  uint32_t Abytes, Bbytes, Cbytes;
  int prec;  // TMR_MATH_F32 / TMR_MATH_BF16
};

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  const bf16x2 v = {(__bf16)lo, (__bf16)hi};   // v_cvt_pk_bf16_f32, round to nearest even
  return __builtin_bit_cast(uint32_t, v);
}

// Buffer loads: 32-bit byte offsets against a per-tensor descriptor; an out-of-range
// offset returns zeros, so padding / tails / masked rows need no branches (the compiler
// can then count vmcnt exactly across the software pipeline).
constexpr uint32_t OOB = 0x80000000u;  // tensors are < 2^31 bytes (checked on the host)

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 bld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  // whole-vector bit_cast: extracting v[0..3] one by one makes hipcc (ROCm 7.2) emit a
  // single buffer_load_dword and replicate it (miscompile, checked in the .s)
  const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return __builtin_bit_cast(float4, v);
}
__device__ __forceinline__ float bld1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
// 4 consecutive elements at byte offset `off`; `nvalid` of them in range (AL: all or none)
template <bool AL>
__device__ __forceinline__ float4 ld4v(__amdgpu_buffer_rsrc_t r, uint32_t off, bool ok, int nvalid) {
  if (AL) return bld4(r, ok ? off : OOB);
  float4 v;
  v.x = bld1(r, ok && nvalid > 0 ? off : OOB);
  v.y = bld1(r, ok && nvalid > 1 ? off + 4 : OOB);
  v.z = bld1(r, ok && nvalid > 2 ? off + 8 : OOB);
  v.w = bld1(r, ok && nvalid > 3 ? off + 12 : OOB);
  return v;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const float* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ void tap_split(const GemmArgs& a, int tap, int& ri, int& si) {
  ri = (tap * a.tapSinv) >> 16;
  si = tap - ri * a.tapS;
}

// VAR: 0 = aligned float4 loads, one tap per k-tile (channels per tap >= BK, or a plain GEMM)
//      1 = aligned, tap varies inside a k-tile (the 4-channel stem)
//      2 = unaligned scalar loads (GEMMs with odd leading dimensions), one tap
// PREC: 0 = fp32 operands, LDS k-major, v_mfma_f32_32x32x2_f32
//       1 = operands rounded to bf16 when written to LDS, LDS row-major [row][BK+8] so each
//           lane's 8-element k-fragment is one ds_read_b128, v_mfma_f32_32x32x16_bf16.
//           M/N-contiguous operands are loaded as k-row pairs so the LDS writes are packed
//           bf16x2 dwords (conflict-free); K-contiguous operands write bf16x4.
template <int MODE, int BM, int BN, int WM, int WN, int BK, int VAR, int PREC = 0>
__global__ TMR_GEMM_LB void gemm_kernel(const GemmArgs a) {
  constexpr bool AL = (VAR != 2);
  constexpr int NT = 64 * WM * WN;       // threads per workgroup
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  constexpr int KQ = BK / 4;             // float4 per row of a K-contiguous tile
  constexpr int RA = BM * BK / (4 * NT); // float4 loads per thread per k-tile for A
  constexpr int RB = BN * BK / (4 * NT);
  static_assert(RA >= 1 && RB >= 1, "tile too small for the workgroup");
  // A tile k-major [BK][LDA]; K-contiguous loaders scatter 4 scalars -> pad 2,
  // M/N-contiguous loaders write float4 -> pad 4.
  constexpr bool A_KC = (MODE != MODE_WGRAD);
  constexpr bool B_KC = (MODE == MODE_FWD);
  constexpr int LDA = BM + (A_KC ? 2 : 4);
  constexpr int LDB = BN + (B_KC ? 2 : 4);
  constexpr int LDK = BK + 8;            // bf16 row stride (80 B for BK=32: conflict-free b128)
  static_assert(PREC == 0 || (BK % 16 == 0 && RA % 2 == 0 && RB % 2 == 0), "bf16 tile shape");
  constexpr int SMEM_F = PREC ? (2 * (BM + BN) * LDK + 1) / 2 : 2 * BK * (LDA + LDB);
  __shared__ __attribute__((aligned(16))) float smem[SMEM_F];
  float* As0 = smem;
  float* Bs0 = smem + 2 * BK * LDA;
  __bf16* Ah0 = reinterpret_cast<__bf16*>(smem);
  __bf16* Bh0 = Ah0 + 2 * BM * LDK;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int l31 = lane & 31, hh = lane >> 5;
  // M/N-contiguous operand loads (WGRAD A, DGRAD B, WGRAD B): load q -> (k row, float4 column)
  // fp32: consecutive threads walk the columns of one k row.  bf16: loads q, q^1 are the k-row
  // pair (2kp, 2kp+1) of one column group, so the LDS write packs them into bf16x2 dwords.
  auto mn_krow = [&](int q, int W4) -> int {
    if (PREC) return 2 * ((tid + NT * (q >> 1)) % (BK / 2)) + (q & 1);
    return (tid + NT * q) / W4;
  };
  auto mn_c4 = [&](int q, int W4) -> int {
    if (PREC) return (tid + NT * (q >> 1)) / (BK / 2);
    return (tid + NT * q) % W4;
  };

  // XCD-aware tile order: consecutive logical tiles share an XCD (and its L2);
  // n-tiles of one m-tile are consecutive so the gathered A rows are reused.
  const int nmt = (a.M + BM - 1) / BM;
  const int nnt = (a.N + BN - 1) / BN;
  const int nwg = nmt * nnt;
  int bid = blockIdx.x;
  {
    int xcd = bid & 7, loc = bid >> 3;
    int q = nwg >> 3, r = nwg & 7;
    int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
    bid = (nwg >= 8) ? wg : bid;
  }
  const int m0 = (bid / nnt) * BM;
  const int n0 = (bid % nnt) * BN;

  // reduction range
  int kbeg = 0, kend = a.K;
  if (MODE == MODE_WGRAD) {
    kbeg = blockIdx.y * a.kchunk;
    kend = min(a.K, kbeg + a.kchunk);
  }
  const int ntiles = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  const __amdgpu_buffer_rsrc_t rA = make_rsrc(a.A, a.Abytes);
  const __amdgpu_buffer_rsrc_t rB = make_rsrc(a.B, a.Bbytes);
  const int cmask = (1 << a.log2C) - 1;

  // ---- per-thread loader state (fixed across k-tiles) ----
  // A_KC (FWD/DGRAD): gathered rows -> (pixel byte offset, y, x, in-range)
  uint32_t apix[A_KC ? RA : 1];
  int ay[A_KC ? RA : 1], ax[A_KC ? RA : 1];
  bool aok[A_KC ? RA : 1];
  if (A_KC) {
#pragma unroll
    for (int q = 0; q < RA; ++q) {
      const int m = m0 + (tid + NT * q) / KQ;
      aok[q] = m < a.M;
      const uint32_t mm = aok[q] ? (uint32_t)m : 0u;
      const uint32_t n = fdiv(mm, a.dHW);
      const uint32_t rem = mm - n * a.dHW.d;
      const uint32_t y = fdiv(rem, a.dW);
      const uint32_t x = rem - y * a.dW.d;
      ay[q] = (int)y * a.sy;
      ax[q] = (int)x * a.sx;
      apix[q] = ((uint32_t)(((int)n * a.Hs + ay[q]) * a.Ws + ax[q]) * (uint32_t)a.lds) * 4u;
    }
  }
  // WGRAD B: this thread's columns j -> (tap offset, channel), fixed for the whole kernel
  int bdy[MODE == MODE_WGRAD ? RB : 1], bdx[MODE == MODE_WGRAD ? RB : 1];
  uint32_t bcoff[MODE == MODE_WGRAD ? RB : 1];
  bool bjok[MODE == MODE_WGRAD ? RB : 1];
  if (MODE == MODE_WGRAD) {
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      const int j = n0 + mn_c4(q, BN / 4) * 4;
      int tap, c;
      if (a.ntaps == 1) { tap = 0; c = j; }
      else { tap = j >> a.log2C; c = j & cmask; }
      int ri, si;
      tap_split(a, tap, ri, si);
      bdy[q] = a.oy0 + a.dyr * ri;
      bdx[q] = a.ox0 + a.dxs * si;
      bcoff[q] = (uint32_t)c * 4u;
      bjok[q] = j < a.N && tap < a.ntaps;
    }
  }

  float4 ra0[RA], rb0[RB], ra1[RA], rb1[RB];  // two prefetch register sets

  auto load_tile = [&](int kt, float4 (&ra)[RA], float4 (&rb)[RB]) {
    const int kb = kbeg + kt * BK;
    // ---- A ----
    if (A_KC) {
      // tap of this k-tile (uniform unless VAR==1)
      int tapU = 0, cbU = kb, dyU = a.oy0, dxU = a.ox0;
      if (VAR != 1 && a.ntaps != 1) {
        tapU = kb >> a.log2C;
        cbU = kb & cmask;
        int ri, si;
        tap_split(a, tapU, ri, si);
        dyU = a.oy0 + a.dyr * ri;
        dxU = a.ox0 + a.dxs * si;
      }
#pragma unroll
      for (int q = 0; q < RA; ++q) {
        const int kq4 = ((tid + NT * q) % KQ) * 4;
        const int k = kb + kq4;
        int tap = tapU, c = cbU + kq4, dy = dyU, dx = dxU;
        if (VAR == 1) {
          tap = k >> a.log2C;
          c = k & cmask;
          int ri, si;
          tap_split(a, tap, ri, si);
          dy = a.oy0 + a.dyr * ri;
          dx = a.ox0 + a.dxs * si;
        }
        const int ys = ay[q] + dy, xs = ax[q] + dx;
        const bool ok = aok[q] && k < kend && tap < a.ntaps && (unsigned)ys < (unsigned)a.Hs &&
                        (unsigned)xs < (unsigned)a.Ws;
        const uint32_t off = apix[q] + (uint32_t)(((dy * a.Ws + dx) * a.lds + c) * 4);
        ra[q] = ld4v<AL>(rA, off, ok, kend - k);
      }
    } else {  // WGRAD: A[i][kk] = dY[m][co], co contiguous
#pragma unroll
      for (int q = 0; q < RA; ++q) {
        const int krow = mn_krow(q, BM / 4), c4 = mn_c4(q, BM / 4);
        const int m = kb + krow, i = m0 + c4 * 4;
        const bool ok = (m < kend) && (i < a.M);
        ra[q] = ld4v<AL>(rA, ((uint32_t)m * (uint32_t)a.ldb + (uint32_t)i) * 4u, ok, a.M - i);
      }
    }
    // ---- B ----
    if (MODE == MODE_FWD) {  // B[j][k], k contiguous
#pragma unroll
      for (int q = 0; q < RB; ++q) {
        const int lin = tid + NT * q;
        const int j = n0 + lin / KQ;
        const int k = kb + (lin % KQ) * 4;
        const bool ok = (j < a.N) && (k < kend);
        rb[q] = ld4v<AL>(rB, ((uint32_t)j * (uint32_t)a.ldb + (uint32_t)k) * 4u, ok, kend - k);
      }
    } else if (MODE == MODE_DGRAD) {  // B[k=(tap,co)][j=ci], ci contiguous
      int tapU = 0, cbU = kb;
      if (a.ntaps != 1) {
        tapU = kb >> a.log2C;
        cbU = kb & cmask;
      }
      int ri, si;
      tap_split(a, tapU, ri, si);
      // weight tap of this k-tile (a one-tap parity class still sits at (wr0, ws0))
      const int rsU = (a.wr0 + a.wst * ri) * a.wS + (a.ws0 + a.wst * si);
#pragma unroll
      for (int q = 0; q < RB; ++q) {
        const int krow = mn_krow(q, BN / 4), c4 = mn_c4(q, BN / 4);
        const int k = kb + krow, j = n0 + c4 * 4;
        const bool ok = (k < kend) && (j < a.N);
        const uint32_t co = (uint32_t)(cbU + krow);
        rb[q] = ld4v<AL>(rB, (co * (uint32_t)a.ldb + (uint32_t)rsU * (uint32_t)a.N + (uint32_t)j) * 4u,
                         ok, a.N - j);
      }
    } else {  // WGRAD: B[kk=m][j=(tap,c)] gathered from X
#pragma unroll
      for (int q = 0; q < RB; ++q) {
        const int krow = mn_krow(q, BN / 4);
        const int m = kb + krow;
        const uint32_t mm = m < kend ? (uint32_t)m : 0u;
        const uint32_t n = fdiv(mm, a.dHW);
        const uint32_t rem = mm - n * a.dHW.d;
        const uint32_t y = fdiv(rem, a.dW);
        const uint32_t x = rem - y * a.dW.d;
        const int ys = (int)y * a.sy + bdy[q], xs = (int)x * a.sx + bdx[q];
        const bool ok = m < kend && bjok[q] && (unsigned)ys < (unsigned)a.Hs &&
                        (unsigned)xs < (unsigned)a.Ws;
        const uint32_t off =
            ((uint32_t)(((int)n * a.Hs + ys) * a.Ws + xs) * (uint32_t)a.lds) * 4u + bcoff[q];
        const int j = n0 + mn_c4(q, BN / 4) * 4;
        rb[q] = ld4v<AL>(rB, off, ok, a.N - j);
      }
    }
  };

  auto store_tile_h = [&](int buf, const float4 (&ra)[RA], const float4 (&rb)[RB]) {
    __bf16* Ah = Ah0 + buf * BM * LDK;
    __bf16* Bh = Bh0 + buf * BN * LDK;
    auto kc_store = [&](__bf16* T, int lin, const float4& v) {   // K-contiguous: 4 k of one row
      const int row = lin / KQ, kq = (lin % KQ) * 4;
      const uint2 w = make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w));
      *reinterpret_cast<uint2*>(&T[row * LDK + kq]) = w;
    };
    auto mn_store = [&](__bf16* T, int q, int W4, const float4& v0, const float4& v1) {
      // v0/v1: rows k = 2kp, 2kp+1 of columns 4c4..4c4+3 -> T[col][2kp..2kp+1]
      const int kp = mn_krow(q, W4) >> 1, c4 = mn_c4(q, W4);
      uint32_t* t = reinterpret_cast<uint32_t*>(T);
      t[((4 * c4 + 0) * LDK) / 2 + kp] = pack_bf16x2(v0.x, v1.x);
      t[((4 * c4 + 1) * LDK) / 2 + kp] = pack_bf16x2(v0.y, v1.y);
      t[((4 * c4 + 2) * LDK) / 2 + kp] = pack_bf16x2(v0.z, v1.z);
      t[((4 * c4 + 3) * LDK) / 2 + kp] = pack_bf16x2(v0.w, v1.w);
    };
    if (A_KC) {
#pragma unroll
      for (int q = 0; q < RA; ++q) kc_store(Ah, tid + NT * q, ra[q]);
    } else {
#pragma unroll
      for (int q = 0; q < RA; q += 2) mn_store(Ah, q, BM / 4, ra[q], ra[q + 1]);
    }
    if (B_KC) {
#pragma unroll
      for (int q = 0; q < RB; ++q) kc_store(Bh, tid + NT * q, rb[q]);
    } else {
#pragma unroll
      for (int q = 0; q < RB; q += 2) mn_store(Bh, q, BN / 4, rb[q], rb[q + 1]);
    }
  };

  auto store_tile = [&](int buf, const float4 (&ra)[RA], const float4 (&rb)[RB]) {
    if (PREC) { store_tile_h(buf, ra, rb); return; }
    float* As = As0 + buf * BK * LDA;
    float* Bs = Bs0 + buf * BK * LDB;
    if (A_KC) {
#pragma unroll
      for (int q = 0; q < RA; ++q) {
        const int lin = tid + NT * q;
        const int row = lin / KQ, kq = (lin % KQ) * 4;
        As[(kq + 0) * LDA + row] = ra[q].x;
        As[(kq + 1) * LDA + row] = ra[q].y;
        As[(kq + 2) * LDA + row] = ra[q].z;
        As[(kq + 3) * LDA + row] = ra[q].w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < RA; ++q) {
        const int lin = tid + NT * q;
        const int krow = lin / (BM / 4), c4 = lin % (BM / 4);
        *reinterpret_cast<float4*>(&As[krow * LDA + c4 * 4]) = ra[q];
      }
    }
    if (B_KC) {
#pragma unroll
      for (int q = 0; q < RB; ++q) {
        const int lin = tid + NT * q;
        const int row = lin / KQ, kq = (lin % KQ) * 4;
        Bs[(kq + 0) * LDB + row] = rb[q].x;
        Bs[(kq + 1) * LDB + row] = rb[q].y;
        Bs[(kq + 2) * LDB + row] = rb[q].z;
        Bs[(kq + 3) * LDB + row] = rb[q].w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < RB; ++q) {
        const int lin = tid + NT * q;
        const int krow = lin / (BN / 4), c4 = lin % (BN / 4);
        *reinterpret_cast<float4*>(&Bs[krow * LDB + c4 * 4]) = rb[q];
      }
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int aoff = wm * (BM / WM) + l31;
  const int boff = wn * (BN / WN) + l31;

  auto compute_h = [&](int cur) {
    const __bf16* Ah = Ah0 + cur * BM * LDK;
    const __bf16* Bh = Bh0 + cur * BN * LDK;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8 av[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        av[i] = *reinterpret_cast<const bf16x8*>(&Ah[(aoff + 32 * i) * LDK + 16 * s + 8 * hh]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bv[j] = *reinterpret_cast<const bf16x8*>(&Bh[(boff + 32 * j) * LDK + 16 * s + 8 * hh]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
  };

  auto compute = [&](int cur) {
    if (PREC) { compute_h(cur); return; }
    const float* As = As0 + cur * BK * LDA;
    const float* Bs = Bs0 + cur * BK * LDB;
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) {
      const int kr = 2 * s + hh;
      float av[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) av[i] = As[kr * LDA + aoff + 32 * i];
#pragma unroll
      for (int j = 0; j < TN; ++j) bv[j] = Bs[kr * LDB + boff + 32 * j];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
  };

  // Software pipeline.  Loads past the last k-tile are issued anyway: their offsets are out
  // of range (k >= kend) so they return zeros, and the loop has no load/store branches, which
  // lets the compiler place exact (counted) vmcnt waits.
  // bf16: one register set (BK=32 tiles are twice as many registers per set)
  constexpr int PFD = PREC ? 1 : TMR_PF;
  if constexpr (PFD == 2) {
    // prefetch distance 2: while the MFMAs run on LDS buffer kt&1, one register set holds
    // tile kt+1 (written to the other buffer after the MFMAs) and the other set has tile
    // kt+2's loads in flight.
    if (ntiles > 0) {
      load_tile(0, ra0, rb0);
      load_tile(1, ra1, rb1);
      store_tile(0, ra0, rb0);
      __syncthreads();
      for (int kt = 0; kt < ntiles; kt += 2) {
        load_tile(kt + 2, ra0, rb0);
        compute(0);
        store_tile(1, ra1, rb1);
        __syncthreads();
        if (kt + 1 >= ntiles) break;
        load_tile(kt + 3, ra1, rb1);
        compute(1);
        store_tile(0, ra0, rb0);
        __syncthreads();
      }
    }
  } else {
    if (ntiles > 0) {
      load_tile(0, ra0, rb0);
      store_tile(0, ra0, rb0);
      __syncthreads();
      for (int kt = 0; kt < ntiles; ++kt) {
        load_tile(kt + 1, ra0, rb0);
        compute(kt & 1);
        store_tile((kt & 1) ^ 1, ra0, rb0);
        __syncthreads();
      }
    }
  }

  // ---- epilogue ----
  // Two epilogue forms.  64x64 tiles (one MFMA tile per wave, few live registers): branch-free
  // buffer accesses, loads batched per chunk of rows.  Larger tiles: per-element guarded
  // accesses -- the batched form pushes their main loops past the VGPR budget (spills).
  if constexpr (TM * TN == 1) {
  // The epilogue's thread indices derive from an opaque copy of the thread id: otherwise the
  // compiler computes its row/column offsets before the main loop and keeps them live (or
  // spilled) across it.
  int etid = tid;
  asm volatile("" : "+v"(etid));
  {
  const int wm = (etid >> 6) / WN, wn = (etid >> 6) % WN;
  const int l31 = etid & 31, hh = (etid & 63) >> 5;
  // Branch-free: every access to C (and to the tensors laid out like C) goes through a buffer
  // descriptor over C's extent; rows outside M and columns outside N get an out-of-range offset
  // (loads return 0, stores are dropped).  Rows are handled in chunks of ER accumulator
  // registers so each chunk's loads are issued back to back before any is consumed.
  float* Cb = a.C;
  if (MODE == MODE_WGRAD) Cb += (long)blockIdx.y * a.slab;
  const __amdgpu_buffer_rsrc_t rC = make_rsrc(Cb, a.Cbytes);
  const int col0 = n0 + wn * (BN / WN) + l31;
  constexpr int ER = TN >= 4 ? 4 : 16 / (2 * TN);   // rows per chunk: 16 / 8 / 4 (TN = 1 / 2 / 4)
  uint32_t cob[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j)
    cob[j] = col0 + 32 * j < a.N ? (uint32_t)(col0 + 32 * j) * 4u : OOB;
  // byte offset of accumulator row (i, r) in C; OOB outside M
  auto row_off = [&](int i, int r) -> uint32_t {
    const int row = m0 + wm * (BM / WM) + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hh;
    uint32_t pix = (uint32_t)row;
    if (MODE == MODE_DGRAD) {   // output-pixel map of the parity class (identity when st == 1)
      const uint32_t n = fdiv((uint32_t)row, a.dHW);
      const uint32_t rem = row - n * a.dHW.d;
      const uint32_t y = fdiv(rem, a.dW);
      const uint32_t x = rem - y * a.dW.d;
      pix = ((n * a.oH + y * a.osy + a.oyc) * a.oW + x * a.osx + a.oxc);
    }
    return row < a.M ? pix * (uint32_t)a.ldc * 4u : OOB;
  };
  // rob OOB + a column offset stays >= 2^31 (no wrap): still out of range
  auto eoff = [&](uint32_t rob, int j) -> uint32_t { return cob[j] == OOB ? OOB : rob + cob[j]; };
  auto st1 = [&](float v, uint32_t off) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), rC, off, 0, 0);
  };
  // Every chunk issues all of its loads (old C for beta, y / z of the fused BN backward, the
  // residual of the fused forward) before consuming any; each row offset is computed once, in
  // its chunk (kept out of the other phases so the offsets never stay live across them).
  const bool has_beta = a.beta != 0.f;
  // (1c) fused BatchNorm backward partials (DGRAD): mask, store, per-column tile sums.  Rows /
  // columns outside the output hold acc == 0 (their operand loads returned zeros) and read
  // bn_y == 0, so they add nothing to either sum.
  if (MODE == MODE_DGRAD && a.bn_part != nullptr) {
    const __amdgpu_buffer_rsrc_t rY = make_rsrc(a.bn_y, a.Cbytes);
    const __amdgpu_buffer_rsrc_t rZ = make_rsrc(a.bn_mask == 1 ? a.bn_z : a.bn_y, a.Cbytes);
    const uint32_t zoob = a.bn_mask == 1 ? 0u : OOB;   // z is read only for mask 1
    float cs[TN], cq[TN], mu[TN], bsc[TN], bsh[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = col0 + 32 * j;
      const bool okc = col < a.N;
      mu[j] = okc ? a.bn_mean[col] : 0.f;
      // keep test t = z + fmaf(y, bsc, bsh) > 0, branch-free over the mask modes:
      // 1: z (bsc = bsh = 0); 2: y*scale+shift (z loads are out of range -> 0); 0: 1 > 0
      bsc[j] = (okc && a.bn_mask == 2) ? a.bn_sc[col] : 0.f;
      bsh[j] = (okc && a.bn_mask == 2) ? a.bn_sh[col] : (a.bn_mask == 0 ? 1.f : 0.f);
      cs[j] = 0.f;
      cq[j] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r0 = 0; r0 < 16; r0 += ER) {
        uint32_t off[ER][TN];
        float yv[ER][TN], zv[ER][TN];
#pragma unroll
        for (int r = 0; r < ER; ++r) {
          const uint32_t ro = row_off(i, r0 + r);
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            off[r][j] = eoff(ro, j);
            yv[r][j] = bld1(rY, off[r][j]);
            zv[r][j] = bld1(rZ, zoob | off[r][j]);
          }
        }
        float old[ER][TN];
#pragma unroll
        for (int r = 0; r < ER; ++r)
#pragma unroll
          for (int j = 0; j < TN; ++j) old[r][j] = has_beta ? bld1(rC, off[r][j]) : 0.f;
#pragma unroll
        for (int r = 0; r < ER; ++r)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            float v = fmaf(a.beta, old[r][j], acc[i][j][r0 + r]);
            const bool keep = zv[r][j] + fmaf(yv[r][j], bsc[j], bsh[j]) > 0.f;
            v = keep ? v : 0.f;
            st1(v, off[r][j]);
            cs[j] += v;
            cq[j] = fmaf(v, yv[r][j] - mu[j], cq[j]);
          }
        __builtin_amdgcn_sched_barrier(0);
      }
    float* red = smem;  // [WM][BN][2]; the main loop ended with a barrier
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      cs[j] += __shfl_xor(cs[j], 32, 64);
      cq[j] += __shfl_xor(cq[j], 32, 64);
      if (hh == 0) {
        const int c = wn * (BN / WN) + 32 * j + l31;
        red[(wm * BN + c) * 2] = cs[j];
        red[(wm * BN + c) * 2 + 1] = cq[j];
      }
    }
    __syncthreads();
    if (wm == 0 && hh == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int c = wn * (BN / WN) + 32 * j + l31;
        float t0 = 0.f, t1 = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) {
          t0 += red[(w * BN + c) * 2];
          t1 += red[(w * BN + c) * 2 + 1];
        }
        if (n0 + c < a.N) a.bn_part[(long)(m0 / BM) * a.N + n0 + c] = make_float2(t0, t1);
      }
    }
    return;
  }
  // (2) bias
  float bvals[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = col0 + 32 * j;
    bvals[j] = (MODE == MODE_FWD && a.bias && col < a.N) ? a.bias[col] : 0.f;
  }
  // (1b) fused BatchNorm batch statistics of this output tile (FWD only): exact block mean,
  // then M2 about it; combined across tiles by tmr_bn_finalize (shifted sums in double, fixed order).
  if (MODE == MODE_FWD && a.stats != nullptr) {
    float* red = smem;  // main loop ended with a barrier: LDS is free
    const int nrows = min(BM, a.M - m0);
    const int rbase_w = m0 + wm * (BM / WM) + 4 * hh;
    auto valid = [&](int i, int r) {
      return rbase_w + 32 * i + (r & 3) + 8 * (r >> 2) < a.M;
    };
    float cs[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) t += valid(i, r) ? acc[i][j][r] + bvals[j] : 0.f;
      t += __shfl_xor(t, 32, 64);
      cs[j] = t;
    }
    if (hh == 0)
#pragma unroll
      for (int j = 0; j < TN; ++j) red[wm * BN + wn * (BN / WN) + 32 * j + l31] = cs[j];
    __syncthreads();
    float mj[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) t += red[w * BN + wn * (BN / WN) + 32 * j + l31];
      mj[j] = t / (float)nrows;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float d = acc[i][j][r] + bvals[j] - mj[j];
          t += valid(i, r) ? d * d : 0.f;
        }
      t += __shfl_xor(t, 32, 64);
      cs[j] = t;
    }
    if (hh == 0)
#pragma unroll
      for (int j = 0; j < TN; ++j) red[wm * BN + wn * (BN / WN) + 32 * j + l31] = cs[j];
    __syncthreads();
    if (wm == 0 && hh == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = col0 + 32 * j;
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) t += red[w * BN + wn * (BN / WN) + 32 * j + l31];
        if (col < a.N)
          a.stats[(long)(m0 / BM) * a.N + col] = make_float4((float)nrows, mj[j], t, 0.f);
      }
    }
  }
  // (3) beta, FWD inference epilogue (scale, residual, ReLU), stores
  const bool has_res = MODE == MODE_FWD && a.res != nullptr;
  const __amdgpu_buffer_rsrc_t rR = make_rsrc(has_res ? a.res : Cb, a.Cbytes);
  float scj[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = col0 + 32 * j;
    scj[j] = (MODE == MODE_FWD && a.scale && col < a.N) ? a.scale[col] : 1.f;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int r0 = 0; r0 < 16; r0 += ER) {
      uint32_t off[ER][TN];
      float old[ER][TN], rv[ER][TN];
#pragma unroll
      for (int r = 0; r < ER; ++r) {
        const uint32_t ro = row_off(i, r0 + r);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          off[r][j] = eoff(ro, j);
          old[r][j] = has_beta ? bld1(rC, off[r][j]) : 0.f;
          rv[r][j] = has_res ? bld1(rR, off[r][j]) : 0.f;
        }
      }
#pragma unroll
      for (int r = 0; r < ER; ++r)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          float v = fmaf(acc[i][j][r0 + r], scj[j], bvals[j]);
          v = fmaf(a.beta, old[r][j], v);
          if (MODE == MODE_FWD) {
            v += rv[r][j];
            if (a.relu) v = fmaxf(v, 0.f);
          }
          st1(v, off[r][j]);
        }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  } else {
  float* Cb = a.C;
  if (MODE == MODE_WGRAD) Cb += (long)blockIdx.y * a.slab;
  const int col0 = n0 + wn * (BN / WN) + l31;
  // output row offset for accumulator register r of row-tile i (-1: outside M)
  auto row_off = [&](int i, int r) -> long {
    const int row = m0 + wm * (BM / WM) + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hh;
    if (row >= a.M) return -1;
    if (MODE == MODE_DGRAD && a.osy != 0) {
      uint32_t n = fdiv((uint32_t)row, a.dHW);
      uint32_t rem = row - n * a.dHW.d;
      uint32_t y = fdiv(rem, a.dW);
      uint32_t x = rem - y * a.dW.d;
      long pix = ((long)n * a.oH + (long)y * a.osy + a.oyc) * a.oW + (long)x * a.osx + a.oxc;
      return pix * a.ldc;
    }
    return (long)row * a.ldc;
  };
  // (1) all reads of the old output first (beta), so they are issued back to back
  if (a.beta != 0.f) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long ro = row_off(i, r);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = col0 + 32 * j;
          if (ro >= 0 && col < a.N) acc[i][j][r] += a.beta * Cb[ro + col];
        }
      }
  }
  // (1c) fused BatchNorm backward partials (DGRAD): mask, store, per-column tile sums
  if (MODE == MODE_DGRAD && a.bn_part != nullptr) {
    float cs[TN], cq[TN], mu[TN], bsc[TN], bsh[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = col0 + 32 * j;
      const bool okc = col < a.N;
      mu[j] = okc ? a.bn_mean[col] : 0.f;
      bsc[j] = (okc && a.bn_mask == 2) ? a.bn_sc[col] : 0.f;
      bsh[j] = (okc && a.bn_mask == 2) ? a.bn_sh[col] : 0.f;
      cs[j] = 0.f;
      cq[j] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long ro = row_off(i, r);
        if (ro < 0) continue;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = col0 + 32 * j;
          if (col >= a.N) continue;
          float v = acc[i][j][r];
          const float yv = a.bn_y[ro + col];
          bool keep = true;
          if (a.bn_mask == 1) keep = a.bn_z[ro + col] > 0.f;
          else if (a.bn_mask == 2) keep = fmaf(yv, bsc[j], bsh[j]) > 0.f;
          v = keep ? v : 0.f;
          Cb[ro + col] = v;
          cs[j] += v;
          cq[j] = fmaf(v, yv - mu[j], cq[j]);
        }
      }
    float* red = smem;  // [WM][BN][2]; the main loop ended with a barrier
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      cs[j] += __shfl_xor(cs[j], 32, 64);
      cq[j] += __shfl_xor(cq[j], 32, 64);
      if (hh == 0) {
        const int c = wn * (BN / WN) + 32 * j + l31;
        red[(wm * BN + c) * 2] = cs[j];
        red[(wm * BN + c) * 2 + 1] = cq[j];
      }
    }
    __syncthreads();
    if (wm == 0 && hh == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int c = wn * (BN / WN) + 32 * j + l31;
        float t0 = 0.f, t1 = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) {
          t0 += red[(w * BN + c) * 2];
          t1 += red[(w * BN + c) * 2 + 1];
        }
        if (n0 + c < a.N) a.bn_part[(long)(m0 / BM) * a.N + n0 + c] = make_float2(t0, t1);
      }
    }
    return;
  }
  // (2) bias + stores
  float bvals[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = col0 + 32 * j;
    bvals[j] = (MODE == MODE_FWD && a.bias && col < a.N) ? a.bias[col] : 0.f;
  }
  // (1b) fused BatchNorm batch statistics of this output tile (FWD only): exact block mean,
  // then M2 about it; combined across tiles by tmr_bn_finalize (shifted sums in double, fixed order).
  if (MODE == MODE_FWD && a.stats != nullptr) {
    float* red = smem;  // main loop ended with a barrier: LDS is free
    const int nrows = min(BM, a.M - m0);
    const int rbase_w = m0 + wm * (BM / WM) + 4 * hh;
    auto valid = [&](int i, int r) {
      return rbase_w + 32 * i + (r & 3) + 8 * (r >> 2) < a.M;
    };
    float cs[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) t += valid(i, r) ? acc[i][j][r] + bvals[j] : 0.f;
      t += __shfl_xor(t, 32, 64);
      cs[j] = t;
    }
    if (hh == 0)
#pragma unroll
      for (int j = 0; j < TN; ++j) red[wm * BN + wn * (BN / WN) + 32 * j + l31] = cs[j];
    __syncthreads();
    float mj[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) t += red[w * BN + wn * (BN / WN) + 32 * j + l31];
      mj[j] = t / (float)nrows;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float d = acc[i][j][r] + bvals[j] - mj[j];
          t += valid(i, r) ? d * d : 0.f;
        }
      t += __shfl_xor(t, 32, 64);
      cs[j] = t;
    }
    if (hh == 0)
#pragma unroll
      for (int j = 0; j < TN; ++j) red[wm * BN + wn * (BN / WN) + 32 * j + l31] = cs[j];
    __syncthreads();
    if (wm == 0 && hh == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = col0 + 32 * j;
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) t += red[w * BN + wn * (BN / WN) + 32 * j + l31];
        if (col < a.N)
          a.stats[(long)(m0 / BM) * a.N + col] = make_float4((float)nrows, mj[j], t, 0.f);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const long ro = row_off(i, r);
      if (ro < 0) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = col0 + 32 * j;
        if (col >= a.N) continue;
        float v = acc[i][j][r] + bvals[j];
        if (MODE == MODE_FWD) {
          if (a.scale) v = fmaf(acc[i][j][r], a.scale[col], bvals[j]);
          if (a.res) v += a.res[ro + col];
          if (a.relu) v = fmaxf(v, 0.f);
        }
        Cb[ro + col] = v;
      }
    }
  }
}

// sum over the split slabs in split order, loads issued 8 at a time (the adds stay in order, so
// the result is bit-identical to a plain loop; only the load latency is overlapped)
__device__ __forceinline__ float split_sum(const float* __restrict__ slabs, int nsplit, long slab,
                                           long src) {
  float s = 0.f;
  int p = 0;
  for (; p + 8 <= nsplit; p += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = slabs[(p + u) * slab + src];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; p < nsplit; ++p) s += slabs[p * slab + src];
  return s;
}

// WGRAD split reduction: dW[co][tap][c] (KRSC with c < creal) summed over splits in
// split order, written to OIHW (co, c, r, s) of the real weight.
__global__ void wgrad_reduce_kernel(const float* __restrict__ slabs, int nsplit, long slab,
                                    float* __restrict__ out, int Cout, int ntaps, int Cpad,
                                    int creal, float beta) {
  long total = (long)Cout * ntaps * creal;
  for (long o = blockIdx.x * (long)blockDim.x + threadIdx.x; o < total;
       o += (long)gridDim.x * blockDim.x) {
    // o indexes OIHW: co, c, tap
    int tap = (int)(o % ntaps);
    long t2 = o / ntaps;
    int c = (int)(t2 % creal);
    int co = (int)(t2 / creal);
    long src = ((long)co * ntaps + tap) * Cpad + c;
    const float s = split_sum(slabs, nsplit, slab, src);
    out[o] = beta != 0.f ? s + beta * out[o] : s;
  }
}

// The same reduction for multi-tap weights: one block per (co, 64-channel group) sums the splits
// with reads along c (coalesced), transposes (tap, c) -> (c, tap) through LDS and writes OIHW rows
// contiguously.  Per element the split order is the same as wgrad_reduce_kernel's.
__global__ __launch_bounds__(256) void wgrad_reduce_taps_kernel(const float* __restrict__ slabs,
                                                                int nsplit, long slab,
                                                                float* __restrict__ out, int ntaps,
                                                                int Cpad, int creal, float beta) {
  __shared__ float tile[49 * 64];   // ntaps <= 49 (7x7), checked on the host
  const int co = blockIdx.x;
  const int c0 = blockIdx.y * 64;
  const int nc = min(64, creal - c0);
  for (int idx = threadIdx.x; idx < ntaps * 64; idx += 256) {
    const int tap = idx >> 6, cl = idx & 63;
    float sum = 0.f;
    if (cl < nc) sum = split_sum(slabs, nsplit, slab, ((long)co * ntaps + tap) * Cpad + c0 + cl);
    tile[tap * 64 + cl] = sum;
  }
  __syncthreads();
  float* o = out + ((long)co * creal + c0) * ntaps;
  for (int idx = threadIdx.x; idx < nc * ntaps; idx += 256) {
    const int cl = idx / ntaps, tap = idx - cl * ntaps;
    const float v = tile[tap * 64 + cl];
    o[idx] = beta != 0.f ? v + beta * o[idx] : v;
  }
}

template <int MODE, int BM, int BN, int WM, int WN, int BKT, int PREC = 0>
int launch_cfg(const GemmArgs& a, int var, dim3 grid, hipStream_t st) {
  const dim3 blk(64 * WM * WN);
  if (var == 2)
    hipLaunchKernelGGL((gemm_kernel<MODE, BM, BN, WM, WN, BKT, 2, PREC>), grid, blk, 0, st, a);
  else if (MODE == MODE_FWD && var == 1)
    hipLaunchKernelGGL((gemm_kernel<MODE, BM, BN, WM, WN, BKT, (MODE == MODE_FWD ? 1 : 0), PREC>), grid, blk, 0, st, a);
  else
    hipLaunchKernelGGL((gemm_kernel<MODE, BM, BN, WM, WN, BKT, 0, PREC>), grid, blk, 0, st, a);
  TMR_CHECK_LAUNCH("gemm_kernel");
  return 0;
}

// Tile configurations (BM, BN).  Selection keeps both tile dims useful.
struct TileCfg { int bm, bn; };
constexpr TileCfg kCfgs[] = {{128, 128}, {256, 64}, {64, 256}, {64, 64},
                             {256, 128}, {128, 256}, {256, 256}, {256, 256}, {256, 128}};
constexpr int kNumCfgs = sizeof(kCfgs) / sizeof(kCfgs[0]);

int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
}

// Tile choice per GEMM view, from scripts/convbench.py over the 23 ResNet-50 shapes x 3 views
// (profiles/r1/convbench_cfgs.txt).  Short reductions (K <= 576: the 1x1 dgrads that accumulate
// into the residual gradient, the 3x3 ones at 64 channels) are epilogue/latency bound and run
// best as 64x64 tiles at high occupancy; wgrad prefers 256x128 to 256x256.
int pick_cfg_shape(long M, long N, long K, int mode) {
  if (mode == MODE_DGRAD && K <= 576 && M >= 4096) return 3;
  if (mode == MODE_WGRAD) {
    if (M <= 64 && N >= 512) return 3;
    if (M >= 256 && N >= 128) return 4;
  }
  if (mode == MODE_FWD && N <= 64 && K >= 576 && M >= 4096) return 3;
  if (M >= 256 && N >= 256) return 6;   // 256x256, 16 waves (measured best, convbench)
  if (M >= 256 && N >= 128) return 4;   // 256x128, 8 waves
  if (N <= 64 && M >= 256) return 1;
  if (M <= 64 && N >= 256) return 2;
  if (M <= 64 || N <= 64) return 3;
  return 0;
}

long cfg_tiles(long M, long N, int c) {
  return ((M + kCfgs[c].bm - 1) / kCfgs[c].bm) * ((N + kCfgs[c].bn - 1) / kCfgs[c].bn);
}

int pick_cfg(long M, long N, long K, int mode) {
  static const int forced = env_int("TMR_GEMM_CFG", -1);  // experiments only
  if (forced >= 0 && forced < kNumCfgs) {
    const TileCfg c = kCfgs[forced];
    if (M >= c.bm && N >= c.bn) return forced;
  }
  int cfg = pick_cfg_shape(M, N, K, mode);
  // Plain GEMMs with few output rows (the LSTM input projection and its dgrad: M = B*T = 640,
  // N = K = 2048) leave most of the 256 CUs idle on the big tiles: step down through 256x128,
  // 128x128 and 64x64 until the grid has >= 256 workgroups.  (The conv views have M >= F*49 rows
  // and never get here; WGRAD splits its reduction over blockIdx.y instead.)
  if (mode != MODE_WGRAD && cfg_tiles(M, N, cfg) < 128) {
    const long area = (long)kCfgs[cfg].bm * kCfgs[cfg].bn;
    for (const int c2 : {4, 0, 3}) {
      if ((long)kCfgs[c2].bm * kCfgs[c2].bn >= area || cfg_tiles(M, N, c2) <= cfg_tiles(M, N, cfg))
        continue;
      cfg = c2;
      if (cfg_tiles(M, N, cfg) >= 256) break;
    }
  }
  return cfg;
}

template <int MODE>
int launch_gemm(const GemmArgs& a, bool al, int splits, hipStream_t st) {
  TMR_CHECK_ARG(a.Abytes < 0x80000000u && a.Bbytes < 0x80000000u && a.Cbytes < 0x80000000u,
                "gemm: operand larger than 2 GiB (split the batch)");
  // WGRAD resolves taps per column (fixed per thread); FWD/DGRAD per k-tile when uniform
  // (a k-tile of BK must not straddle two taps: channels per tap >= BK)
  const int bk = a.prec == TMR_MATH_BF16 ? 32 : 16;
  const bool uniform = MODE == MODE_WGRAD || a.ntaps <= 1 || (1 << a.log2C) >= bk;
  int var = al ? (uniform ? 0 : 1) : 2;
  TMR_CHECK_ARG(uniform || (al && MODE == MODE_FWD),
                "gemm: per-element taps need aligned channels and the forward view");
  const int cfg = pick_cfg(a.M, a.N, a.K, MODE);
  const TileCfg c = kCfgs[cfg];
  dim3 grid(cdiv(a.M, c.bm) * cdiv(a.N, c.bn), splits, 1);
  if (grid.x == 0) return 0;
  if (a.prec == TMR_MATH_BF16) {
    switch (cfg) {
      case 0: return launch_cfg<MODE, 128, 128, 2, 2, 32, 1>(a, var, grid, st);
      case 1: return launch_cfg<MODE, 256, 64, 4, 1, 32, 1>(a, var, grid, st);
      case 2: return launch_cfg<MODE, 64, 256, 1, 4, 32, 1>(a, var, grid, st);
      case 3: return launch_cfg<MODE, 64, 64, 2, 2, 32, 1>(a, var, grid, st);
      case 4: case 8: return launch_cfg<MODE, 256, 128, 4, 2, 32, 1>(a, var, grid, st);
      case 5: return launch_cfg<MODE, 128, 256, 2, 4, 32, 1>(a, var, grid, st);
      default: return launch_cfg<MODE, 256, 256, 4, 4, 32, 1>(a, var, grid, st);
    }
  }
  switch (cfg) {
    case 0: return launch_cfg<MODE, 128, 128, 2, 2, 16>(a, var, grid, st);
    case 1: return launch_cfg<MODE, 256, 64, 4, 1, 16>(a, var, grid, st);
    case 2: return launch_cfg<MODE, 64, 256, 1, 4, 16>(a, var, grid, st);
    case 3: return launch_cfg<MODE, 64, 64, 2, 2, 16>(a, var, grid, st);
    case 4: return launch_cfg<MODE, 256, 128, 4, 2, 16>(a, var, grid, st);
    case 5: return launch_cfg<MODE, 128, 256, 2, 4, 16>(a, var, grid, st);
    case 6: return launch_cfg<MODE, 256, 256, 4, 4, 16>(a, var, grid, st);
    case 7: return launch_cfg<MODE, 256, 256, 4, 4, 32>(a, var, grid, st);
    default: return launch_cfg<MODE, 256, 128, 4, 2, 32>(a, var, grid, st);
  }
}

static inline int xld_of(const tmr_conv_desc* d) { return d->x_ld ? d->x_ld : d->c; }
static inline int yld_of(const tmr_conv_desc* d) { return d->y_ld ? d->y_ld : d->k; }
static inline long span(long pixels, int ld, int width) { return pixels > 0 ? (pixels - 1) * ld + width : 0; }

static uint32_t clamp_bytes(long elems) {
  long b = elems * 4;
  return b >= 0x80000000L ? 0x80000000u : (uint32_t)b;
}

int ilog2_exact(int v) {
  if (v <= 0 || (v & (v - 1))) return -1;
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}

bool aligned16(const void* p) { return (((uintptr_t)p) & 15) == 0; }

void set_taps(GemmArgs& a, int nR, int nS) {
  a.ntaps = nR * nS;
  a.tapS = nS > 0 ? nS : 1;
  a.tapSinv = (65536 + a.tapS - 1) / a.tapS;
}

void set_grid(GemmArgs& a, int n, int hg, int wg) {
  (void)n;
  a.dHW = make_fastdiv((uint32_t)(hg * wg));
  a.dW = make_fastdiv((uint32_t)wg);
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
static int conv_fwd_args(const tmr_conv_desc* d, const float* x, const float* w_krsc,
                         const float* bias, float* y, float beta, GemmArgs& a, bool& al) {
  TMR_CHECK_ARG(d, "tmr_conv2d_fwd: null descriptor");
  TMR_CHECK_ARG(d->math == TMR_MATH_F32 || d->math == TMR_MATH_BF16, "tmr_conv2d: bad math mode %d", d->math);
  const int lc = ilog2_exact(d->c);
  TMR_CHECK_ARG(lc >= 2, "tmr_conv2d_fwd: stored input channels %d must be a power of two >= 4", d->c);
  a = GemmArgs{};
  a.A = x; a.B = w_krsc; a.C = y; a.bias = bias;
  a.M = d->n * d->ho * d->wo; a.N = d->k; a.K = d->r * d->s * d->c;
  a.log2C = lc;
  set_taps(a, d->r, d->s);
  a.oy0 = -d->pad; a.ox0 = -d->pad_w; a.dyr = 1; a.dxs = 1;
  set_grid(a, d->n, d->ho, d->wo);
  a.Hs = d->h; a.Ws = d->w; a.sy = d->stride; a.sx = d->stride;
  a.lds = xld_of(d); a.ldb = a.K; a.ldc = yld_of(d); a.beta = beta;
  a.Abytes = clamp_bytes(span((long)d->n * d->h * d->w, a.lds, d->c));
  a.prec = d->math;
  a.Bbytes = clamp_bytes((long)d->k * a.K);
  a.Cbytes = clamp_bytes(span((long)d->n * d->ho * d->wo, a.ldc, d->k));
  al = aligned16(x) && aligned16(w_krsc) && (d->k % 4 == 0) && (a.lds % 4 == 0);
  return 0;
}

// Frames per launch: the buffer descriptors take 32-bit byte offsets, so every operand of one
// launch must stay below 2 GiB; larger batches (e.g. C5's 1920 frames) run as several launches
// over consecutive frame ranges (d->max_frames caps it further, for tests).
static int frames_per_launch(const tmr_conv_desc* d) {
  const long xf = (long)d->h * d->w * xld_of(d) * 4;
  const long yf = (long)d->ho * d->wo * yld_of(d) * 4;
  const long mx = xf > yf ? xf : yf;
  long f = mx > 0 ? 0x7fffffffL / mx : d->n;
  if (d->max_frames > 0 && d->max_frames < f) f = d->max_frames;
  if (f > d->n) f = d->n;
  return (int)(f > 0 ? f : 1);
}

static tmr_conv_desc chunk_desc(const tmr_conv_desc* d, int nc) {
  tmr_conv_desc c = *d;
  c.n = nc;
  return c;
}

static int stats_parts_of(const tmr_conv_desc* d) {
  const long M = (long)d->n * d->ho * d->wo;
  return cdiv(M, kCfgs[pick_cfg(M, d->k, (long)d->r * d->s * d->c, MODE_FWD)].bm);
}

static long x_frame(const tmr_conv_desc* d) { return (long)d->h * d->w * xld_of(d); }
static long y_frame(const tmr_conv_desc* d) { return (long)d->ho * d->wo * yld_of(d); }

TMR_API int tmr_conv2d_fwd(const tmr_conv_desc* d, const float* x, const float* w_krsc,
                           const float* bias, float* y, float beta, hipStream_t stream) {
  TMR_CHECK_ARG(d, "tmr_conv2d_fwd: null descriptor");
  const int fc = frames_per_launch(d);
  for (int f0 = 0; f0 < d->n; f0 += fc) {
    const tmr_conv_desc c = chunk_desc(d, d->n - f0 < fc ? d->n - f0 : fc);
    GemmArgs a;
    bool al;
    int rc = conv_fwd_args(&c, x + f0 * x_frame(d), w_krsc, bias, y + f0 * y_frame(d), beta, a, al);
    if (!rc) rc = launch_gemm<MODE_FWD>(a, al, 1, stream);
    if (rc) return rc;
  }
  return 0;
}

TMR_API int tmr_conv2d_fwd_fused(const tmr_conv_desc* d, const float* x, const float* w_krsc,
                                 const float* scale, const float* shift, const float* residual,
                                 float* y, int relu, hipStream_t stream) {
  TMR_CHECK_ARG(d, "tmr_conv2d_fwd_fused: null descriptor");
  TMR_CHECK_ARG(scale && shift, "tmr_conv2d_fwd_fused: null BatchNorm scale/shift");
  TMR_CHECK_ARG(!residual || residual != y, "tmr_conv2d_fwd_fused: residual must not alias y");
  const int fc = frames_per_launch(d);
  for (int f0 = 0; f0 < d->n; f0 += fc) {
    const tmr_conv_desc c = chunk_desc(d, d->n - f0 < fc ? d->n - f0 : fc);
    GemmArgs a;
    bool al;
    int rc = conv_fwd_args(&c, x + f0 * x_frame(d), w_krsc, shift, y + f0 * y_frame(d), 0.f, a, al);
    if (rc) return rc;
    a.scale = scale;
    a.res = residual ? residual + f0 * y_frame(d) : nullptr;
    a.relu = relu;
    rc = launch_gemm<MODE_FWD>(a, al, 1, stream);
    if (rc) return rc;
  }
  return 0;
}

TMR_API int tmr_conv2d_fwd_stats_parts(const tmr_conv_desc* d) {
  if (!d || d->n <= 0) {
    tmr_set_error("tmr_conv2d_fwd_stats_parts: null or empty descriptor");
    return -1;
  }
  const int fc = frames_per_launch(d);
  int parts = 0;
  for (int f0 = 0; f0 < d->n; f0 += fc) {
    const tmr_conv_desc c = chunk_desc(d, d->n - f0 < fc ? d->n - f0 : fc);
    parts += stats_parts_of(&c);
  }
  return parts;
}

TMR_API int tmr_conv2d_fwd_bnstats(const tmr_conv_desc* d, const float* x, const float* w_krsc,
                                   float* y, void* stats, size_t stats_bytes, hipStream_t stream) {
  TMR_CHECK_ARG(d, "tmr_conv2d_fwd_bnstats: null descriptor");
  TMR_CHECK_ARG(yld_of(d) == d->k, "tmr_conv2d_fwd_bnstats: output must be dense (y_ld == k)");
  const size_t need = (size_t)tmr_conv2d_fwd_stats_parts(d) * d->k * sizeof(float4);
  TMR_CHECK_ARG(stats && stats_bytes >= need, "tmr_conv2d_fwd_bnstats: stats buffer too small (%zu < %zu)",
                stats_bytes, need);
  const int fc = frames_per_launch(d);
  float4* st = (float4*)stats;
  for (int f0 = 0; f0 < d->n; f0 += fc) {
    const tmr_conv_desc c = chunk_desc(d, d->n - f0 < fc ? d->n - f0 : fc);
    GemmArgs a;
    bool al;
    int rc = conv_fwd_args(&c, x + f0 * x_frame(d), w_krsc, nullptr, y + f0 * y_frame(d), 0.f, a, al);
    if (rc) return rc;
    a.stats = st;
    rc = launch_gemm<MODE_FWD>(a, al, 1, stream);
    if (rc) return rc;
    st += (long)stats_parts_of(&c) * d->k;
  }
  return 0;
}

// Fused BatchNorm-backward epilogue state of one dgrad call (nullptr: plain dgrad).  part
// advances over the launches; count_only tallies the partial rows without launching.
struct BnBwdFuse {
  const float *y, *z, *sc, *sh, *mean;
  int mask;
  float2* part;
  long nparts;
  bool count_only;
};

static int conv_dgrad_impl(const tmr_conv_desc* d, const float* dy, const float* w_krsc,
                           float* dx, float beta, hipStream_t stream, BnBwdFuse* fz = nullptr) {
  TMR_CHECK_ARG(d->math == TMR_MATH_F32 || d->math == TMR_MATH_BF16, "tmr_conv2d: bad math mode %d", d->math);
  const int lk = ilog2_exact(d->k);
  TMR_CHECK_ARG(lk >= 2, "tmr_conv2d_dgrad: output channels %d must be a power of two >= 4", d->k);
  TMR_CHECK_ARG(d->c % 4 == 0, "tmr_conv2d_dgrad: input channels %d must be a multiple of 4", d->c);
  const int st = d->stride;
  // one launch per stride-parity class (ph,pw): rows h = st*y + ph
  for (int ph = 0; ph < st; ++ph) {
    for (int pw = 0; pw < st; ++pw) {
      // valid kernel rows r with (ph + pad - r) % st == 0
      int r0 = -1, nR = 0, s0 = -1, nS = 0;
      for (int r = 0; r < d->r; ++r)
        if (((ph + d->pad - r) % st + st) % st == 0) { if (r0 < 0) r0 = r; ++nR; }
      for (int s = 0; s < d->s; ++s)
        if (((pw + d->pad_w - s) % st + st) % st == 0) { if (s0 < 0) s0 = s; ++nS; }
      const int hg = (d->h - ph + st - 1) / st, wg = (d->w - pw + st - 1) / st;
      if (hg <= 0 || wg <= 0) continue;
      GemmArgs a{};
      a.A = dy; a.B = w_krsc; a.C = dx; a.bias = nullptr;
      a.M = d->n * hg * wg; a.N = d->c; a.K = nR * nS * d->k;
      a.log2C = lk;
      set_taps(a, nR, nS);
      if (nR == 0 || nS == 0) { a.K = 0; a.ntaps = 0; }
      // ho = (h + pad - r)/st = y + (ph + pad - r0)/st - ri
      a.oy0 = nR ? (ph + d->pad - r0) / st : 0;
      a.ox0 = nS ? (pw + d->pad_w - s0) / st : 0;
      a.dyr = -1; a.dxs = -1;
      a.wr0 = r0 < 0 ? 0 : r0; a.ws0 = s0 < 0 ? 0 : s0; a.wst = st; a.wS = d->s;
      set_grid(a, d->n, hg, wg);
      a.Hs = d->ho; a.Ws = d->wo; a.sy = 1; a.sx = 1;
      a.lds = yld_of(d); a.ldb = d->r * d->s * d->c; a.ldc = xld_of(d); a.beta = beta;
      a.Abytes = clamp_bytes(span((long)d->n * d->ho * d->wo, a.lds, d->k));
      a.prec = d->math;
      a.Bbytes = clamp_bytes((long)d->k * d->r * d->s * d->c);
      a.Cbytes = clamp_bytes(span((long)d->n * d->h * d->w, a.ldc, d->c));
      a.oH = d->h; a.oW = d->w; a.osy = st; a.osx = st; a.oyc = ph; a.oxc = pw;
      // nothing to add -- unless the fused BN backward must still see (mask, sum) these pixels
      if (a.K == 0 && beta == 1.f && !fz) continue;
      if (fz) {
        const long nmt = cdiv(a.M, kCfgs[pick_cfg(a.M, a.N, a.K, MODE_DGRAD)].bm);
        if (fz->count_only) { fz->nparts += nmt; continue; }
        a.bn_y = fz->y; a.bn_z = fz->z; a.bn_sc = fz->sc; a.bn_sh = fz->sh; a.bn_mean = fz->mean;
        a.bn_mask = fz->mask;
        a.bn_part = fz->part;
        fz->part += nmt * a.N;
        fz->nparts += nmt;
      }
      bool al = aligned16(dy) && aligned16(w_krsc) && aligned16(dx) && a.lds % 4 == 0;
      int rc = launch_gemm<MODE_DGRAD>(a, al, 1, stream);
      if (rc) return rc;
    }
  }
  return 0;
}

static int dgrad_bnbwd_run(const tmr_conv_desc* d, const float* dy, const float* w_krsc, float* dx,
                           float beta, BnBwdFuse* fz, hipStream_t stream) {
  const int fc = frames_per_launch(d);
  const long px_frame = (long)d->h * d->w * d->c;   // dense dx / y / z (checked by the caller)
  float2* part0 = fz->part;
  for (int f0 = 0; f0 < d->n; f0 += fc) {
    const tmr_conv_desc c = chunk_desc(d, d->n - f0 < fc ? d->n - f0 : fc);
    BnBwdFuse fc_ = *fz;
    fc_.y = fz->y ? fz->y + f0 * px_frame : nullptr;
    fc_.z = fz->z ? fz->z + f0 * px_frame : nullptr;
    fc_.nparts = 0;
    int rc = conv_dgrad_impl(&c, dy ? dy + f0 * y_frame(d) : nullptr, w_krsc,
                             dx ? dx + f0 * x_frame(d) : nullptr, beta, stream, &fc_);
    if (rc) return rc;
    fz->part = fc_.part;
    fz->nparts += fc_.nparts;
  }
  fz->part = part0;
  return 0;
}

TMR_API int tmr_conv2d_dgrad_bnbwd_parts(const tmr_conv_desc* d) {
  if (!d || d->n <= 0) {
    tmr_set_error("tmr_conv2d_dgrad_bnbwd_parts: null or empty descriptor");
    return -1;
  }
  BnBwdFuse fz{};
  fz.count_only = true;
  if (dgrad_bnbwd_run(d, nullptr, nullptr, nullptr, 1.f, &fz, nullptr)) return -1;
  return (int)fz.nparts;
}

TMR_API int tmr_conv2d_dgrad_bnbwd(const tmr_conv_desc* d, const float* dy, const float* w_krsc,
                                   float* dx, float beta, const float* y, const float* z,
                                   const float* scale, const float* shift, const float* mean,
                                   int mask, void* parts, size_t parts_bytes, hipStream_t stream) {
  TMR_CHECK_ARG(d, "tmr_conv2d_dgrad_bnbwd: null descriptor");
  TMR_CHECK_ARG(xld_of(d) == d->c, "tmr_conv2d_dgrad_bnbwd: dx must be dense (x_ld == c)");
  TMR_CHECK_ARG(y && mean && parts, "tmr_conv2d_dgrad_bnbwd: null y / mean / parts");
  TMR_CHECK_ARG(mask == 0 || (mask == 1 && z) || (mask == 2 && scale && shift),
                "tmr_conv2d_dgrad_bnbwd: mask %d needs z (1) or scale/shift (2)", mask);
  const int np = tmr_conv2d_dgrad_bnbwd_parts(d);
  TMR_CHECK_ARG(np >= 0 && parts_bytes >= (size_t)np * d->c * sizeof(float2),
                "tmr_conv2d_dgrad_bnbwd: parts buffer too small");
  BnBwdFuse fz{};
  fz.y = y; fz.z = z; fz.sc = scale; fz.sh = shift; fz.mean = mean; fz.mask = mask;
  fz.part = (float2*)parts;
  return dgrad_bnbwd_run(d, dy, w_krsc, dx, beta, &fz, stream);
}

TMR_API int tmr_conv2d_dgrad(const tmr_conv_desc* d, const float* dy, const float* w_krsc,
                             float* dx, float beta, hipStream_t stream) {
  TMR_CHECK_ARG(d, "tmr_conv2d_dgrad: null descriptor");
  const int fc = frames_per_launch(d);
  for (int f0 = 0; f0 < d->n; f0 += fc) {
    const tmr_conv_desc c = chunk_desc(d, d->n - f0 < fc ? d->n - f0 : fc);
    int rc = conv_dgrad_impl(&c, dy + f0 * y_frame(d), w_krsc, dx + f0 * x_frame(d), beta, stream);
    if (rc) return rc;
  }
  return 0;
}

static int wgrad_plan(const tmr_conv_desc* d, int* splits, int* kchunk, long* slab) {
  const long Mred = (long)d->n * d->ho * d->wo;
  const long Mo = d->k, No = (long)d->r * d->s * d->c;
  const TileCfg tc = kCfgs[pick_cfg(Mo, No, Mred, MODE_WGRAD)];
  const long tiles = (long)cdiv(Mo, tc.bm) * cdiv(No, tc.bn);
  // aim for ~target workgroups; at least minrows reduction rows per split
  static const long target = env_int("TMR_WGRAD_TARGET", 512);
  static const long minrows = env_int("TMR_WGRAD_MINROWS", 1024);
  long sp = target / (tiles > 0 ? tiles : 1);
  if (sp < 1) sp = 1;
  long maxsp = Mred / minrows;
  if (maxsp < 1) maxsp = 1;
  if (sp > maxsp) sp = maxsp;
  long kc = (Mred + sp - 1) / sp;
  kc = (kc + 31) / 32 * 32;  // multiple of every BK (16, 32)
  sp = (Mred + kc - 1) / kc;
  *splits = (int)sp;
  *kchunk = (int)kc;
  *slab = Mo * No;
  return 0;
}

TMR_API size_t tmr_conv2d_wgrad_ws_bytes(const tmr_conv_desc* d) {
  if (!d || d->n <= 0 || d->k <= 0 || d->c <= 0 || d->r <= 0 || d->s <= 0) {
    tmr_set_error("tmr_conv2d_wgrad_ws_bytes: null or empty descriptor");
    return 0;
  }
  int sp, kc;
  long slab;
  const tmr_conv_desc c = chunk_desc(d, frames_per_launch(d));   // the largest chunk
  wgrad_plan(&c, &sp, &kc, &slab);
  return (size_t)sp * slab * sizeof(float);
}

static int conv_wgrad_impl(const tmr_conv_desc* d, const float* x, const float* dy,
                           float* dw_oihw, int c_real, float beta, float* ws, size_t ws_bytes,
                           hipStream_t stream);

// frame chunks accumulate into dw in chunk order (beta = 1 after the first): deterministic
TMR_API int tmr_conv2d_wgrad(const tmr_conv_desc* d, const float* x, const float* dy,
                             float* dw_oihw, int c_real, float beta, float* ws, size_t ws_bytes,
                             hipStream_t stream) {
  TMR_CHECK_ARG(d, "tmr_conv2d_wgrad: null descriptor");
  const int fc = frames_per_launch(d);
  for (int f0 = 0; f0 < d->n; f0 += fc) {
    const tmr_conv_desc c = chunk_desc(d, d->n - f0 < fc ? d->n - f0 : fc);
    int rc = conv_wgrad_impl(&c, x + f0 * x_frame(d), dy + f0 * y_frame(d), dw_oihw, c_real,
                             f0 == 0 ? beta : 1.f, ws, ws_bytes, stream);
    if (rc) return rc;
  }
  return 0;
}

static int conv_wgrad_impl(const tmr_conv_desc* d, const float* x, const float* dy,
                           float* dw_oihw, int c_real, float beta, float* ws, size_t ws_bytes,
                           hipStream_t stream) {
  TMR_CHECK_ARG(d->math == TMR_MATH_F32 || d->math == TMR_MATH_BF16, "tmr_conv2d: bad math mode %d", d->math);
  const int lc = ilog2_exact(d->c);
  TMR_CHECK_ARG(lc >= 2, "tmr_conv2d_wgrad: stored input channels %d must be a power of two >= 4", d->c);
  TMR_CHECK_ARG(c_real >= 1 && c_real <= d->c, "tmr_conv2d_wgrad: bad c_real %d", c_real);
  int sp, kc;
  long slab;
  wgrad_plan(d, &sp, &kc, &slab);
  TMR_CHECK_ARG(ws && ws_bytes >= (size_t)sp * slab * sizeof(float),
                "tmr_conv2d_wgrad: workspace too small (%zu < %zu)", ws_bytes,
                (size_t)sp * slab * sizeof(float));
  GemmArgs a{};
  a.A = dy; a.B = x; a.C = ws; a.bias = nullptr;
  a.M = d->k; a.N = d->r * d->s * d->c; a.K = d->n * d->ho * d->wo;
  a.log2C = lc;
  set_taps(a, d->r, d->s);
  a.oy0 = -d->pad; a.ox0 = -d->pad_w; a.dyr = 1; a.dxs = 1;
  set_grid(a, d->n, d->ho, d->wo);
  a.Hs = d->h; a.Ws = d->w; a.sy = d->stride; a.sx = d->stride;
  a.lds = xld_of(d); a.ldb = yld_of(d); a.ldc = a.N; a.beta = 0.f;
  a.kchunk = kc; a.slab = slab;
  a.Abytes = clamp_bytes(span((long)d->n * d->ho * d->wo, a.ldb, d->k));
  a.prec = d->math;
  a.Bbytes = clamp_bytes(span((long)d->n * d->h * d->w, a.lds, d->c));
  a.Cbytes = clamp_bytes(slab);
  bool al = aligned16(x) && aligned16(dy) && (d->k % 4 == 0) && a.lds % 4 == 0 && a.ldb % 4 == 0;
  int rc = launch_gemm<MODE_WGRAD>(a, al, sp, stream);
  if (rc) return rc;
  const int ntaps = d->r * d->s;
  if (ntaps > 1 && ntaps <= 49) {
    hipLaunchKernelGGL(wgrad_reduce_taps_kernel, dim3(d->k, cdiv(c_real, 64)), dim3(256), 0,
                       stream, ws, sp, slab, dw_oihw, ntaps, d->c, c_real, beta);
    TMR_CHECK_LAUNCH("wgrad_reduce_taps_kernel");
    return 0;
  }
  long total = (long)d->k * ntaps * c_real;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, stream, ws, sp, slab,
                     dw_oihw, d->k, ntaps, d->c, c_real, beta);
  TMR_CHECK_LAUNCH("wgrad_reduce_kernel");
  return 0;
}

// Plain GEMMs on the same engine ---------------------------------------------
// C[M][N] (row stride ldc) = beta*C + A[M][K] (row stride lda) * B^T, B = [N][K] (ldb) (+bias[N])
TMR_API int tmr_gemm_nt(int M, int N, int K, const float* A, int lda, const float* B, int ldb,
                        const float* bias, float* C, int ldc, float beta, hipStream_t stream) {
  TMR_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "tmr_gemm_nt: negative size");
  GemmArgs a{};
  a.A = A; a.B = B; a.C = C; a.bias = bias;
  a.M = M; a.N = N; a.K = K; a.log2C = 0;
  set_taps(a, 1, 1);
  a.dyr = 1; a.dxs = 1;
  set_grid(a, M, 1, 1);
  a.Hs = 1; a.Ws = 1; a.sy = 1; a.sx = 1;
  a.lds = lda; a.ldb = ldb; a.ldc = ldc; a.beta = beta;
  a.Abytes = clamp_bytes(M > 0 ? (long)(M - 1) * lda + K : 0);
  a.Bbytes = clamp_bytes(N > 0 ? (long)(N - 1) * ldb + K : 0);
  a.Cbytes = clamp_bytes(M > 0 ? (long)(M - 1) * ldc + N : 0);
  bool al = aligned16(A) && aligned16(B) && lda % 4 == 0 && ldb % 4 == 0 && K % 4 == 0;
  return launch_gemm<MODE_FWD>(a, al, 1, stream);
}

// C[M][N] = beta*C + A[M][K] (lda) * B[K][N] (ldb)
TMR_API int tmr_gemm_nn(int M, int N, int K, const float* A, int lda, const float* B, int ldb,
                        float* C, int ldc, float beta, hipStream_t stream) {
  TMR_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "tmr_gemm_nn: negative size");
  GemmArgs a{};
  a.A = A; a.B = B; a.C = C; a.bias = nullptr;
  a.M = M; a.N = N; a.K = K; a.log2C = 0;
  set_taps(a, 1, 1);
  a.oy0 = 0; a.ox0 = 0; a.dyr = -1; a.dxs = -1;
  a.wr0 = 0; a.ws0 = 0; a.wst = 1; a.wS = 1;
  set_grid(a, M, 1, 1);
  a.Hs = 1; a.Ws = 1; a.sy = 1; a.sx = 1;
  a.lds = lda; a.ldb = ldb; a.ldc = ldc; a.beta = beta;
  a.oH = 1; a.oW = 1; a.osy = 1; a.osx = 1; a.oyc = 0; a.oxc = 0;   // identity row map
  a.Abytes = clamp_bytes(M > 0 ? (long)(M - 1) * lda + K : 0);
  a.Bbytes = clamp_bytes(K > 0 ? (long)(K - 1) * ldb + N : 0);
  a.Cbytes = clamp_bytes(M > 0 ? (long)(M - 1) * ldc + N : 0);
  bool al = aligned16(A) && aligned16(B) && lda % 4 == 0 && ldb % 4 == 0 && K % 4 == 0 &&
            N % 4 == 0;
  return launch_gemm<MODE_DGRAD>(a, al, 1, stream);
}

// C[M][N] = beta*C + A^T B, A = [K][M] (lda), B = [K][N] (ldb)   (no split: small K)
TMR_API int tmr_gemm_tn(int M, int N, int K, const float* A, int lda, const float* B, int ldb,
                        float* C, int ldc, float beta, hipStream_t stream) {
  TMR_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "tmr_gemm_tn: negative size");
  GemmArgs a{};
  a.A = A; a.B = B; a.C = C; a.bias = nullptr;
  a.M = M; a.N = N; a.K = K; a.log2C = 0;
  set_taps(a, 1, 1);
  a.dyr = 1; a.dxs = 1;
  set_grid(a, K, 1, 1);
  a.Hs = 1; a.Ws = 1; a.sy = 1; a.sx = 1;
  a.lds = ldb; a.ldb = lda; a.ldc = ldc; a.beta = beta;
  a.kchunk = K > 0 ? K : 1; a.slab = 0;
  a.Abytes = clamp_bytes(K > 0 ? (long)(K - 1) * lda + M : 0);
  a.Bbytes = clamp_bytes(K > 0 ? (long)(K - 1) * ldb + N : 0);
  a.Cbytes = clamp_bytes(M > 0 ? (long)(M - 1) * ldc + N : 0);
  bool al = aligned16(A) && aligned16(B) && lda % 4 == 0 && ldb % 4 == 0 && M % 4 == 0 &&
            N % 4 == 0;
  return launch_gemm<MODE_WGRAD>(a, al, 1, stream);
}

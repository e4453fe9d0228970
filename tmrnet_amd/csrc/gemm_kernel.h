// Implicit-GEMM engine: the kernel template and its launch selection, shared by the three GEMM
// view translation units (gemm_fwd.hip, gemm_dgrad.hip, gemm_wgrad.hip -- split so the template
// instantiations compile in parallel) and the host side (gemm_conv.hip).
#pragma once
// Implicit-GEMM convolution / GEMM engine (kernel), fp32 in / fp32 accumulate on the
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
#include "tmr_prologue.h"
#include <stdlib.h>

namespace tmrg {

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
  // row stride (columns) of the stats / bn_part partial rows: N, or the total channel count when
  // this launch is one group of a grouped convolution (its columns are a slice of the rows)
  int part_ld;
  // byte extents of A, B and C (buffer-descriptor range checks; C's also bounds the tensors
  // laid out like C: res, bn_y, bn_z; WGRAD: one split slab)
  uint32_t Abytes, Bbytes, Cbytes;
  int prec;  // TMR_MATH_F32 / TMR_MATH_BF16
  // Operand prologue (tmr_conv_prologue): the BatchNorm that produced an operand, applied while
  // it is loaded, so its output is never written to HBM.  pro bit 1, the gathered X operand (FWD
  // A, WGRAD B): x' = relu(fmaf(x, px_scale[c], px_shift[c])) -- the forward BN+ReLU of the unit
  // that produced x (bn_apply_k's arithmetic) -- and 0 wherever the loader is out of range (the
  // zero padding belongs to the post-ReLU tensor).  pro bit 2, the dY operand (DGRAD A, WGRAD A):
  // dy' = fmaf(pd_a[k], g, fmaf(pd_b[k], y, pd_c[k])) with y read from pd_y at g's offset -- the
  // BatchNorm backward of this conv's BN (bn_bwd_apply's arithmetic), 0 out of range.
  const float* px_scale;
  const float* px_shift;
  const float* pd_y;
  const float* pd_a;
  const float* pd_b;
  const float* pd_c;
  int pro;
  // bf16-stored operands (bf16 math only): bit 0 = A, bit 1 = B holds bf16 values (2-byte
  // elements; byte extents and offsets in bf16 units).  Exact w.r.t. the fp32-stored bf16 path:
  // the loaders would round those operands to bf16 (RNE) anyway.
  int sab;
  // DGRAD B operand is the transposed bf16 weight copy Wt[ci][r][s][co] (TMR_IO_WT_BF16; the
  // LDS-DMA engine of gemm16_kernel.h only), row stride ldbt = R*S*Cout elements
  int wt, ldbt;
  // bf16 activations (TMR_MATH_BF16 train step): c16 -- the FWD output C is written as bf16 (RNE),
  // and the BN statistics of the epilogue are those of the rounded values; bn16 -- the y / z read
  // by the fused BN-backward epilogue of DGRAD are bf16
  int c16, bn16;
  // fp32 conv views eligible for the LDS-DMA engine (gemm16_kernel.h use32; set by the conv
  // entry points, never by the plain GEMMs)
  int dma32;
  // DGRAD with the fused BN backward (LDS-DMA engine, LDS-staged epilogue): C -- the masked
  // gradient g -- is stored as bf16 (RNE) and the partials describe the rounded values; no beta
  // (TMR_IO_G16)
  int g16;
  // the fused BN-backward DGRAD's beta operand (the old dx), when it is not C itself: the bf16
  // residual-gradient step (trunk.R16) reads an fp32 gradient and stores the sum as bf16 elsewhere.
  // cold16: the old dx is bf16 (element offsets as C's).  Cold == nullptr: C.
  const void* Cold;
  int cold16;
  // DGRAD: keep the one-tile-per-workgroup launch where the wave-specialised persistent dgrad
  // (gemm16_ws.h) would serve the shape (TMR_IO_TILES; tests)
  int io_tiles;
};

__device__ __forceinline__ float bf16_rne(float v) { return (float)(__bf16)v; }
__device__ __forceinline__ unsigned short bf16_bits(float v) {
  return __builtin_bit_cast(unsigned short, (__bf16)v);
}

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

// 4 bf16 (8 bytes) at byte offset `off` of a bf16 tensor, carried raw in the .x/.y of a float4
// slot (the fp32 loaders' register slot of 4 elements); OOB offsets read zeros
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float4 ld4h(__amdgpu_buffer_rsrc_t r, uint32_t off, bool ok) {
  // whole-vector bit_cast (as bld4): extracting the load's elements one by one makes hipcc
  // (ROCm 7.2) emit one buffer_load_dword (checked in the .s)
  const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(r, ok ? off : OOB, 0, 0);
  const float2 f = __builtin_bit_cast(float2, v);
  return make_float4(f.x, f.y, 0.f, 0.f);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const float* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
}

// Work item of this workgroup in an XCD-aware order.  The grid is (output tiles, reduction
// splits); workgroups are dispatched to the 8 XCDs round-robin in linear order, so a contiguous
// range of a logical sequence per XCD puts neighbouring items on one L2.  Tiles are m-major: the
// n-tiles of one m-tile (which gather the same A rows) are neighbours.  A split-K WGRAD with few
// tiles (<= 32, one XCD's worth) orders (split, tile): all tiles of one reduction split read the
// same dY and X rows (bf16 layer1-3 wgrads 10-45% faster); with more tiles the splits stay the
// outer grid dimension and only the tiles are remapped (measured better for the layer4 shapes).
__device__ __forceinline__ void xcd_work(int& tile, int& split) {
  const int nwg = gridDim.x;
  const bool sm = gridDim.y > 1 && nwg <= 32;
  const int L = sm ? blockIdx.y * nwg + blockIdx.x : blockIdx.x;
  const int total = sm ? nwg * gridDim.y : nwg;
  int w = L;
  if (total >= 8) {
    const int xcd = L & 7, loc = L >> 3;
    const int q = total >> 3, r = total & 7;
    w = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  }
  split = sm ? w / nwg : blockIdx.y;
  tile = sm ? w - split * nwg : w;
}

__device__ __forceinline__ void tap_split(const GemmArgs& a, int tap, int& ri, int& si) {
  ri = (tap * a.tapSinv) >> 16;
  si = tap - ri * a.tapS;
}

// Epilogue, batched form: branch-free buffer accesses over C's extent, each chunk of ER rows
// issuing all of its loads before consuming any (latency-bound short-reduction GEMMs).  Used by
// gemm_kernel's 64x64 tiles and by every tile of the LDS-DMA engine.
template <int MODE, int BM, int BN, int WM, int WN, int TM, int TN>
__device__ __forceinline__ void epilogue_batched(const GemmArgs& a, floatx16 (&acc)[TM][TN],
                                                 float* smem, int m0, int n0, int split) {
  const int tid = threadIdx.x;
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
  if (MODE == MODE_WGRAD) Cb += (long)split * a.slab;
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
  const bool c16 = MODE == MODE_FWD && a.c16;
  auto st1 = [&](float v, uint32_t off) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), rC, off, 0, 0);
  };
  // bf16 tensors laid out like C are accessed a dword (two columns) per lane: lanes 2k, 2k+1 hold
  // columns 2k, 2k+1 of accumulator rows r, r+1 (r even: adjacent output rows); the even lane
  // moves the pair of row r, the odd lane that of row r+1, and the halves are swapped between the
  // two lanes (DPP quad_perm [1,0,3,2]).  Needs an even N (conv channels: multiples of 8).
  const bool odd = (l31 & 1) != 0;
  auto poff = [&](uint32_t off_r, uint32_t off_r1) -> uint32_t {
    const uint32_t o = odd ? off_r1 : off_r;
    return o >= OOB ? OOB : (o >> 1) - (odd ? 2u : 0u);
  };
  auto swap1 = [](uint32_t w) -> uint32_t {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0xB1, 0xF, 0xF, false);
  };
  // the pair dword w loaded at poff -> (value of row r, value of row r+1) in this lane's column
  auto unpair = [&](uint32_t w, float& vr, float& vr1) {
    const uint32_t n = swap1(w);
    vr = odd ? __uint_as_float(n & 0xffff0000u) : __uint_as_float(w << 16);
    vr1 = odd ? __uint_as_float(w & 0xffff0000u) : __uint_as_float(n << 16);
  };
  // store (row r: vr, row r+1: vr1) of this lane's column as bf16 pairs
  auto st_pair = [&](float vr, float vr1, uint32_t off_r, uint32_t off_r1) {
    const uint32_t mine = odd ? (uint32_t)bf16_bits(vr1) : (uint32_t)bf16_bits(vr);
    const uint32_t other = odd ? (uint32_t)bf16_bits(vr) : (uint32_t)bf16_bits(vr1);
    const uint32_t got = swap1(other);   // the neighbour's value of my pair's row
    const uint32_t w = odd ? ((mine << 16) | got) : ((got << 16) | mine);
    __builtin_amdgcn_raw_buffer_store_b32(w, rC, poff(off_r, off_r1), 0, 0);
  };
  if (c16) {   // the stored (rounded) values are the ones the BN statistics describe
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = bf16_rne(acc[i][j][r]);
  }
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
            if (!a.bn16) {
              yv[r][j] = bld1(rY, off[r][j]);
              zv[r][j] = bld1(rZ, zoob | off[r][j]);
            }
          }
        }
        if (a.bn16) {   // bf16 y / z: one dword load per row pair, split between the lane pair
          uint32_t yw[ER / 2][TN], zw[ER / 2][TN];
#pragma unroll
          for (int rp = 0; rp < ER / 2; ++rp)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              const uint32_t po = poff(off[2 * rp][j], off[2 * rp + 1][j]);
              yw[rp][j] = __builtin_amdgcn_raw_buffer_load_b32(rY, po, 0, 0);
              zw[rp][j] = __builtin_amdgcn_raw_buffer_load_b32(rZ, zoob | po, 0, 0);
            }
#pragma unroll
          for (int rp = 0; rp < ER / 2; ++rp)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              unpair(yw[rp][j], yv[2 * rp][j], yv[2 * rp + 1][j]);
              unpair(zw[rp][j], zv[2 * rp][j], zv[2 * rp + 1][j]);
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
        if (n0 + c < a.N) a.bn_part[(long)(m0 / BM) * a.part_ld + n0 + c] = make_float2(t0, t1);
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
  // (the stores go out before the statistics pass, whose barriers then overlap their drain)
  const bool c16w = c16 && TN % 2 == 0 && a.c16 == 2;
  // (1b) fused BatchNorm batch statistics of this output tile (FWD only): exact block mean,
  // then M2 about it; combined across tiles by tmr_bn_finalize (shifted sums in double, fixed order).
  auto stats_pass = [&]() {
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
          a.stats[(long)(m0 / BM) * a.part_ld + col] = make_float4((float)nrows, mj[j], t, 0.f);
      }
    }
  }
  };
  // (3) beta, FWD inference epilogue (scale, residual, ReLU), stores; then the statistics pass
  // (acc is not modified by the stores)
  const bool has_res = MODE == MODE_FWD && a.res != nullptr;
  const __amdgpu_buffer_rsrc_t rR = make_rsrc(has_res ? a.res : Cb, a.Cbytes);
  float scj[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = col0 + 32 * j;
    scj[j] = (MODE == MODE_FWD && a.scale && col < a.N) ? a.scale[col] : 1.f;
  }
  // bf16 output, TN even: whole 128-B lines per row.  The lane pair (2k, 2k+1) stores columns
  // (2k, 2k+1) of accumulator column block 2jp (even lane) and of block 2jp + 1 (odd lane), both of
  // the same row, so the 32 lanes of a half-wave write one row's 64 columns = 128 contiguous bytes
  // (the pair form below, kept for tiles with an odd TN, writes 64-B halves of two rows).  Same
  // values, same bytes.  a.c16 == 2 selects it (every bf16-output forward, gemm_conv.hip).
  if (c16w) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r0 = 0; r0 < 16; r0 += ER) {
#pragma unroll
        for (int r = 0; r < ER; ++r) {
          const uint32_t ro = row_off(i, r0 + r);
#pragma unroll
          for (int jp = 0; jp < TN / 2; ++jp) {
            const float mine = odd ? acc[i][2 * jp + 1][r0 + r] : acc[i][2 * jp][r0 + r];
            const float send = odd ? acc[i][2 * jp][r0 + r] : acc[i][2 * jp + 1][r0 + r];
            const uint32_t got = swap1((uint32_t)bf16_bits(send));
            const uint32_t mb = (uint32_t)bf16_bits(mine);
            const uint32_t w = odd ? ((mb << 16) | got) : ((got << 16) | mb);
            const int scol = odd ? col0 - 1 + 32 * (2 * jp + 1) : col0 + 64 * jp;
            const uint32_t o = (ro >= OOB || scol >= a.N) ? OOB : (ro >> 1) + (uint32_t)scol * 2u;
            __builtin_amdgcn_raw_buffer_store_b32(w, rC, o, 0, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    stats_pass();
    return;
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
      if (c16) {   // bf16 output (no beta / residual / scale: checked on the host)
#pragma unroll
        for (int rp = 0; rp < ER / 2; ++rp)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            st_pair(acc[i][j][r0 + 2 * rp], acc[i][j][r0 + 2 * rp + 1], off[2 * rp][j],
                    off[2 * rp + 1][j]);
        __builtin_amdgcn_sched_barrier(0);
        continue;
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
  stats_pass();
  }
}

// Epilogue of the larger tiles: per-element guarded accesses (the batched branch-free form of the
// 64x64 tiles pushes their main loops past the VGPR budget).  Shared by gemm_kernel and the bf16
// LDS-DMA engine (gemm16_kernel.h).  smem: >= WM * BN * 2 floats, free (the main loop has ended
// with a barrier and no LDS-DMA in flight).
template <int MODE, int BM, int BN, int WM, int WN, int TM, int TN>
__device__ __forceinline__ void epilogue_guarded(const GemmArgs& a, floatx16 (&acc)[TM][TN],
                                                 float* smem, int m0, int n0, int split) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int l31 = lane & 31, hh = lane >> 5;
  float* Cb = a.C;
  if (MODE == MODE_WGRAD) Cb += (long)split * a.slab;
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
  const bool c16 = MODE == MODE_FWD && a.c16;
  if (c16) {   // the stored (rounded) values are the ones the BN statistics describe
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = bf16_rne(acc[i][j][r]);
  }
  auto bnv = [&](const float* p, long o) -> float {
    return a.bn16 ? (float)reinterpret_cast<const __bf16*>(p)[o] : p[o];
  };
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
          const float yv = bnv(a.bn_y, ro + col);
          bool keep = true;
          if (a.bn_mask == 1) keep = bnv(a.bn_z, ro + col) > 0.f;
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
        if (n0 + c < a.N) a.bn_part[(long)(m0 / BM) * a.part_ld + n0 + c] = make_float2(t0, t1);
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
          a.stats[(long)(m0 / BM) * a.part_ld + col] = make_float4((float)nrows, mj[j], t, 0.f);
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
        if (c16) reinterpret_cast<__bf16*>(Cb)[ro + col] = (__bf16)v;
        else Cb[ro + col] = v;
      }
    }
}

// VAR: 0 = aligned float4 loads, one tap per k-tile (channels per tap >= BK, or a plain GEMM)
//      1 = aligned, tap varies inside a k-tile (the 4-channel stem)
//      2 = unaligned scalar loads (GEMMs with odd leading dimensions), one tap
// PREC: 0 = fp32 operands, LDS k-major, v_mfma_f32_32x32x2_f32
//       1 = operands rounded to bf16 when written to LDS, LDS row-major [row][BK+8] so each
//           lane's 8-element k-fragment is one ds_read_b128, v_mfma_f32_32x32x16_bf16.
//           M/N-contiguous operands are loaded as k-row pairs so the LDS writes are packed
//           bf16x2 dwords (conflict-free); K-contiguous operands write bf16x4.
template <int MODE, int BM, int BN, int WM, int WN, int BK, int VAR, int PREC = 0, int PRO = 0,
          int SAB = 0>
__global__ TMR_GEMM_LB void gemm_kernel(const GemmArgs a) {
  constexpr bool AL = (VAR != 2);
  // bf16-stored operands: 8-byte loads of 4 bf16 per slot (the fp32 slot of 4 elements, half the
  // bytes, no conversion), written to LDS as they are
  constexpr bool SA = (SAB & 1) != 0, SB = (SAB & 2) != 0;
  constexpr uint32_t ESA = SA ? 2u : 4u, ESB = SB ? 2u : 4u;   // element bytes of A / B
  static_assert(SAB == 0 || (PREC == 1 && PRO == 0 && AL), "bf16 storage: bf16 math, aligned");
  // operand prologues (GemmArgs::pro): X operand BN+ReLU on A (FWD) or B (WGRAD); dY operand BN
  // backward on A (DGRAD, WGRAD)
  constexpr bool PX_A = (PRO & 1) && MODE == MODE_FWD;
  constexpr bool PX_B = (PRO & 1) && MODE == MODE_WGRAD;
  constexpr bool PD_A = (PRO & 2) && MODE != MODE_FWD;
  static_assert(PRO == 0 || VAR == 0, "operand prologues need aligned, tap-uniform k-tiles");
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
  const int nnt = (a.N + BN - 1) / BN;
  int bid, split;
  xcd_work(bid, split);
  const int m0 = (bid / nnt) * BM;
  const int n0 = (bid % nnt) * BN;

  // reduction range
  int kbeg = 0, kend = a.K;
  if (MODE == MODE_WGRAD) {
    kbeg = split * a.kchunk;
    kend = min(a.K, kbeg + a.kchunk);
  }
  const int ntiles = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  const __amdgpu_buffer_rsrc_t rA = make_rsrc(a.A, a.Abytes);
  const __amdgpu_buffer_rsrc_t rB = make_rsrc(a.B, a.Bbytes);
  // dY prologue: the pre-BN conv output y, laid out exactly like dY (same offsets and extent)
  const __amdgpu_buffer_rsrc_t rY = make_rsrc(PD_A ? a.pd_y : a.A, a.Abytes);
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
      apix[q] = ((uint32_t)(((int)n * a.Hs + ay[q]) * a.Ws + ax[q]) * (uint32_t)a.lds) * ESA;
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
      bcoff[q] = (uint32_t)c * ESB;
      bjok[q] = j < a.N && tap < a.ntaps;
    }
  }

  // prologue constants fixed per thread (the WGRAD operands' columns never change): dY columns
  // i (output channels) of A, X channels of B
  // fp32: a thread's M/N-contiguous column is the same for every q (NT is a multiple of the row
  // width); bf16: one column per k-row pair q / 2
  constexpr int QA = PREC ? RA / 2 : 1, QB = PREC ? RB / 2 : 1;
  auto qa = [](int q) { return PREC ? q >> 1 : 0; };
  float4 wpa[(PD_A && MODE == MODE_WGRAD) ? QA : 1], wpb[(PD_A && MODE == MODE_WGRAD) ? QA : 1],
      wpc[(PD_A && MODE == MODE_WGRAD) ? QA : 1];
  float4 xsb[PX_B ? QB : 1], xhb[PX_B ? QB : 1];
  if constexpr (PD_A && MODE == MODE_WGRAD) {
#pragma unroll
    for (int p = 0; p < QA; ++p) {
      const int i = m0 + mn_c4(PREC ? 2 * p : 0, BM / 4) * 4;
      const int ii = i < a.M ? i : 0;
      wpa[p] = *reinterpret_cast<const float4*>(a.pd_a + ii);
      wpb[p] = *reinterpret_cast<const float4*>(a.pd_b + ii);
      wpc[p] = *reinterpret_cast<const float4*>(a.pd_c + ii);
    }
  }
  if constexpr (PX_B) {
#pragma unroll
    for (int p = 0; p < QB; ++p) {
      const int q = PREC ? 2 * p : 0;
      const int c = bjok[q] ? (int)(bcoff[q] / ESB) : 0;
      xsb[p] = *reinterpret_cast<const float4*>(a.px_scale + c);
      xhb[p] = *reinterpret_cast<const float4*>(a.px_shift + c);
    }
  }
  // per prefetch set: in-range bits of the prologue operands, the y values of the dY prologue and
  // the per-k-tile channel coefficients (FWD: scale, shift; DGRAD: A, B, C)
  struct Aux {
    uint32_t oka, okb;
    float4 ya[PD_A ? RA : 1];
    float4 c0, c1, c2;
  };
  Aux aux0{}, aux1{};

  float4 ra0[RA], rb0[RB], ra1[RA], rb1[RB];  // two prefetch register sets

  auto load_tile = [&](int kt, float4 (&ra)[RA], float4 (&rb)[RB], Aux& aux) {
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
        const uint32_t off = apix[q] + (uint32_t)(((dy * a.Ws + dx) * a.lds + c) * (int)ESA);
        if constexpr (SA) ra[q] = ld4h(rA, off, ok);
        else ra[q] = ld4v<AL>(rA, off, ok, kend - k);
        if constexpr (PD_A) aux.ya[q] = ld4v<AL>(rY, off, ok, kend - k);
        if constexpr (PX_A || PD_A) {
          if (q == 0) aux.oka = 0;
          aux.oka |= (uint32_t)ok << q;
        }
      }
      if constexpr (PX_A || PD_A) {
        // channel quad of this thread's k-column (KQ divides NT: the same for every q)
        const int cq = (cbU + (tid % KQ) * 4) & cmask;
        if constexpr (PX_A) {
          aux.c0 = *reinterpret_cast<const float4*>(a.px_scale + cq);
          aux.c1 = *reinterpret_cast<const float4*>(a.px_shift + cq);
        } else {
          aux.c0 = *reinterpret_cast<const float4*>(a.pd_a + cq);
          aux.c1 = *reinterpret_cast<const float4*>(a.pd_b + cq);
          aux.c2 = *reinterpret_cast<const float4*>(a.pd_c + cq);
        }
      }
    } else {  // WGRAD: A[i][kk] = dY[m][co], co contiguous
#pragma unroll
      for (int q = 0; q < RA; ++q) {
        const int krow = mn_krow(q, BM / 4), c4 = mn_c4(q, BM / 4);
        const int m = kb + krow, i = m0 + c4 * 4;
        const bool ok = (m < kend) && (i < a.M);
        const uint32_t off = ((uint32_t)m * (uint32_t)a.ldb + (uint32_t)i) * ESA;
        if constexpr (SA) ra[q] = ld4h(rA, off, ok);
        else ra[q] = ld4v<AL>(rA, off, ok, a.M - i);
        if constexpr (PD_A) {
          aux.ya[q] = ld4v<AL>(rY, off, ok, a.M - i);
          if (q == 0) aux.oka = 0;
          aux.oka |= (uint32_t)ok << q;
        }
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
        const uint32_t off = ((uint32_t)j * (uint32_t)a.ldb + (uint32_t)k) * ESB;
        if constexpr (SB) rb[q] = ld4h(rB, off, ok);
        else rb[q] = ld4v<AL>(rB, off, ok, kend - k);
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
        const uint32_t off = (co * (uint32_t)a.ldb + (uint32_t)rsU * (uint32_t)a.N + (uint32_t)j) * ESB;
        if constexpr (SB) rb[q] = ld4h(rB, off, ok);
        else rb[q] = ld4v<AL>(rB, off, ok, a.N - j);
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
            ((uint32_t)(((int)n * a.Hs + ys) * a.Ws + xs) * (uint32_t)a.lds) * ESB + bcoff[q];
        const int j = n0 + mn_c4(q, BN / 4) * 4;
        if constexpr (SB) rb[q] = ld4h(rB, off, ok);
        else rb[q] = ld4v<AL>(rB, off, ok, a.N - j);
        if constexpr (PX_B) {
          if (q == 0) aux.okb = 0;
          aux.okb |= (uint32_t)ok << q;
        }
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
    // bf16-stored slots: 4 raw bf16 in .x/.y
    auto kc_store16 = [&](__bf16* T, int lin, const float4& v) {
      const int row = lin / KQ, kq = (lin % KQ) * 4;
      *reinterpret_cast<uint2*>(&T[row * LDK + kq]) =
          make_uint2(__builtin_bit_cast(uint32_t, v.x), __builtin_bit_cast(uint32_t, v.y));
    };
    auto mn_store16 = [&](__bf16* T, int q, int W4, const float4& v0, const float4& v1) {
      const int kp = mn_krow(q, W4) >> 1, c4 = mn_c4(q, W4);
      const uint32_t a0 = __builtin_bit_cast(uint32_t, v0.x), a1 = __builtin_bit_cast(uint32_t, v0.y);
      const uint32_t b0 = __builtin_bit_cast(uint32_t, v1.x), b1 = __builtin_bit_cast(uint32_t, v1.y);
      uint32_t* t = reinterpret_cast<uint32_t*>(T);
      t[((4 * c4 + 0) * LDK) / 2 + kp] = (a0 & 0xffffu) | (b0 << 16);
      t[((4 * c4 + 1) * LDK) / 2 + kp] = (a0 >> 16) | (b0 & 0xffff0000u);
      t[((4 * c4 + 2) * LDK) / 2 + kp] = (a1 & 0xffffu) | (b1 << 16);
      t[((4 * c4 + 3) * LDK) / 2 + kp] = (a1 >> 16) | (b1 & 0xffff0000u);
    };
    if (A_KC) {
#pragma unroll
      for (int q = 0; q < RA; ++q) {
        if constexpr (SA) kc_store16(Ah, tid + NT * q, ra[q]);
        else kc_store(Ah, tid + NT * q, ra[q]);
      }
    } else {
#pragma unroll
      for (int q = 0; q < RA; q += 2) {
        if constexpr (SA) mn_store16(Ah, q, BM / 4, ra[q], ra[q + 1]);
        else mn_store(Ah, q, BM / 4, ra[q], ra[q + 1]);
      }
    }
    if (B_KC) {
#pragma unroll
      for (int q = 0; q < RB; ++q) {
        if constexpr (SB) kc_store16(Bh, tid + NT * q, rb[q]);
        else kc_store(Bh, tid + NT * q, rb[q]);
      }
    } else {
#pragma unroll
      for (int q = 0; q < RB; q += 2) {
        if constexpr (SB) mn_store16(Bh, q, BN / 4, rb[q], rb[q + 1]);
        else mn_store(Bh, q, BN / 4, rb[q], rb[q + 1]);
      }
    }
  };

  // the prologue transforms, applied when a prefetch set is written to LDS
  auto relu_aff = [](float4 v, float4 sc, float4 sf, bool ok) -> float4 {
    float4 o;
    o.x = fmaxf(fmaf(v.x, sc.x, sf.x), 0.f); o.y = fmaxf(fmaf(v.y, sc.y, sf.y), 0.f);
    o.z = fmaxf(fmaf(v.z, sc.z, sf.z), 0.f); o.w = fmaxf(fmaf(v.w, sc.w, sf.w), 0.f);
    return ok ? o : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  auto bn_bwd4 = [](float4 g, float4 y, float4 A, float4 B, float4 C, bool ok) -> float4 {
    float4 o;
    o.x = fmaf(A.x, g.x, fmaf(B.x, y.x, C.x)); o.y = fmaf(A.y, g.y, fmaf(B.y, y.y, C.y));
    o.z = fmaf(A.z, g.z, fmaf(B.z, y.z, C.z)); o.w = fmaf(A.w, g.w, fmaf(B.w, y.w, C.w));
    return ok ? o : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  auto store_tile = [&](int buf, const float4 (&ra_in)[RA], const float4 (&rb_in)[RB],
                        const Aux& aux) {
    float4 ra[RA], rb[RB];
#pragma unroll
    for (int q = 0; q < RA; ++q) {
      const bool ok = (aux.oka >> q) & 1u;
      if constexpr (PX_A) ra[q] = relu_aff(ra_in[q], aux.c0, aux.c1, ok);
      else if constexpr (PD_A && MODE == MODE_DGRAD)
        ra[q] = bn_bwd4(ra_in[q], aux.ya[q], aux.c0, aux.c1, aux.c2, ok);
      else if constexpr (PD_A && MODE == MODE_WGRAD)
        ra[q] = bn_bwd4(ra_in[q], aux.ya[q], wpa[qa(q)], wpb[qa(q)], wpc[qa(q)], ok);
      else ra[q] = ra_in[q];
    }
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      if constexpr (PX_B) rb[q] = relu_aff(rb_in[q], xsb[qa(q)], xhb[qa(q)], (aux.okb >> q) & 1u);
      else rb[q] = rb_in[q];
    }
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
  constexpr int PFD = (PREC || PRO) ? 1 : TMR_PF;   // prologue variants: one register set
  if constexpr (PFD == 2) {
    // prefetch distance 2: while the MFMAs run on LDS buffer kt&1, one register set holds
    // tile kt+1 (written to the other buffer after the MFMAs) and the other set has tile
    // kt+2's loads in flight.
    if (ntiles > 0) {
      load_tile(0, ra0, rb0, aux0);
      load_tile(1, ra1, rb1, aux1);
      store_tile(0, ra0, rb0, aux0);
      __syncthreads();
      for (int kt = 0; kt < ntiles; kt += 2) {
        load_tile(kt + 2, ra0, rb0, aux0);
        compute(0);
        store_tile(1, ra1, rb1, aux1);
        __syncthreads();
        if (kt + 1 >= ntiles) break;
        load_tile(kt + 3, ra1, rb1, aux1);
        compute(1);
        store_tile(0, ra0, rb0, aux0);
        __syncthreads();
      }
    }
  } else {
    if (ntiles > 0) {
      load_tile(0, ra0, rb0, aux0);
      store_tile(0, ra0, rb0, aux0);
      __syncthreads();
      for (int kt = 0; kt < ntiles; ++kt) {
        load_tile(kt + 1, ra0, rb0, aux0);
        compute(kt & 1);
        store_tile((kt & 1) ^ 1, ra0, rb0, aux0);
        __syncthreads();
      }
    }
  }

  // ---- epilogue ----
  // Two epilogue forms.  64x64 tiles (one MFMA tile per wave, few live registers): branch-free
  // buffer accesses, loads batched per chunk of rows.  Larger tiles: per-element guarded
  // accesses -- the batched form pushes their main loops past the VGPR budget (spills).
  if constexpr (TM * TN == 1) {
    epilogue_batched<MODE, BM, BN, WM, WN, TM, TN>(a, acc, smem, m0, n0, split);
  } else {
    epilogue_guarded<MODE, BM, BN, WM, WN, TM, TN>(a, acc, smem, m0, n0, split);
  }
}

template <int MODE, int BM, int BN, int WM, int WN, int BKT, int PREC = 0>
int launch_cfg(const GemmArgs& a, int var, dim3 grid, hipStream_t st) {
  const dim3 blk(64 * WM * WN);
  if constexpr (PREC == 1) {
    if (a.sab) {   // bf16-stored operands (combinations checked by launch_gemm_t)
      if constexpr (MODE == MODE_FWD) {
        if (a.sab == 2 && var == 1)
          hipLaunchKernelGGL((gemm_kernel<MODE, BM, BN, WM, WN, BKT, 1, 1, 0, 2>), grid, blk, 0, st, a);
        else if (a.sab == 2)
          hipLaunchKernelGGL((gemm_kernel<MODE, BM, BN, WM, WN, BKT, 0, 1, 0, 2>), grid, blk, 0, st, a);
        else
          hipLaunchKernelGGL((gemm_kernel<MODE, BM, BN, WM, WN, BKT, 0, 1, 0, 3>), grid, blk, 0, st, a);
      } else if constexpr (MODE == MODE_DGRAD) {
        hipLaunchKernelGGL((gemm_kernel<MODE, BM, BN, WM, WN, BKT, 0, 1, 0, 3>), grid, blk, 0, st, a);
      } else {
        if (a.sab == 1)
          hipLaunchKernelGGL((gemm_kernel<MODE, BM, BN, WM, WN, BKT, 0, 1, 0, 1>), grid, blk, 0, st, a);
        else
          hipLaunchKernelGGL((gemm_kernel<MODE, BM, BN, WM, WN, BKT, 0, 1, 0, 3>), grid, blk, 0, st, a);
      }
      TMR_CHECK_LAUNCH("gemm_kernel");
      return 0;
    }
  }
#if TMR_PROLOGUES
  if (a.pro) {   // operand prologues (var == 0, checked by launch_gemm_t; A/B build only)
    if constexpr (MODE == MODE_FWD) {
      hipLaunchKernelGGL((gemm_kernel<MODE, BM, BN, WM, WN, BKT, 0, PREC, 1>), grid, blk, 0, st, a);
    } else if constexpr (MODE == MODE_DGRAD) {
      hipLaunchKernelGGL((gemm_kernel<MODE, BM, BN, WM, WN, BKT, 0, PREC, 2>), grid, blk, 0, st, a);
    } else {
      if (a.pro == 1)
        hipLaunchKernelGGL((gemm_kernel<MODE, BM, BN, WM, WN, BKT, 0, PREC, 1>), grid, blk, 0, st, a);
      else if (a.pro == 2)
        hipLaunchKernelGGL((gemm_kernel<MODE, BM, BN, WM, WN, BKT, 0, PREC, 2>), grid, blk, 0, st, a);
      else
        hipLaunchKernelGGL((gemm_kernel<MODE, BM, BN, WM, WN, BKT, 0, PREC, 3>), grid, blk, 0, st, a);
    }
    TMR_CHECK_LAUNCH("gemm_kernel");
    return 0;
  }
#endif
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

inline int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
}

// Tile choice per GEMM view, from scripts/convbench.py over the 23 ResNet-50 shapes x 3 views
// (profiles/r1/convbench_cfgs.txt).  Short reductions (K <= 576: the 1x1 dgrads that accumulate
// into the residual gradient, the 3x3 ones at 64 channels) are epilogue/latency bound and run
// best as 64x64 tiles at high occupancy; wgrad prefers 256x128 to 256x256.
inline int pick_cfg_shape(long M, long N, long K, int mode) {
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

inline long cfg_tiles(long M, long N, int c) {
  return ((M + kCfgs[c].bm - 1) / kCfgs[c].bm) * ((N + kCfgs[c].bn - 1) / kCfgs[c].bn);
}

inline int pick_cfg(long M, long N, long K, int mode) {
  static const int forced = env_int("TMR_GEMM_CFG", -1);  // experiments only
  if (forced >= 0 && forced < kNumCfgs) {
    const TileCfg c = kCfgs[forced];
    if (M >= c.bm && N >= c.bn) return forced;
  }
  int cfg = pick_cfg_shape(M, N, K, mode);
  // Plain GEMMs with few output rows (the LSTM input projection and its dgrad: M = B*T = 640,
  // N = K = 2048) leave most of the 256 CUs idle on the big tiles: step down through 256x128,
  // 128x128 and 64x64 until the grid has >= 256 workgroups.  (The conv views have M >= F*49 rows
  // and never get here; the conv WGRAD splits its reduction over blockIdx.y instead.  A plain
  // A^T B GEMM (tmr_gemm_tn, WGRAD view without splits) with a short reduction -- the split
  // attention's fc weight gradients over the frames, K = F -- steps down the same way.)
  if ((mode != MODE_WGRAD || K <= 8192) && cfg_tiles(M, N, cfg) < 128) {
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
int launch_gemm_t(const GemmArgs& a, bool al, int splits, hipStream_t st) {
  TMR_CHECK_ARG(a.Abytes < 0x80000000u && a.Bbytes < 0x80000000u && a.Cbytes < 0x80000000u,
                "gemm: operand larger than 2 GiB (split the batch)");
  // WGRAD resolves taps per column (fixed per thread); FWD/DGRAD per k-tile when uniform
  // (a k-tile of BK must not straddle two taps: channels per tap >= BK)
  const int bk = a.prec == TMR_MATH_BF16 ? 32 : 16;
  const bool uniform = MODE == MODE_WGRAD || a.ntaps <= 1 || (1 << a.log2C) >= bk;
  int var = al ? (uniform ? 0 : 1) : 2;
  TMR_CHECK_ARG(!a.pro || var == 0,
                "gemm: operand prologues need aligned operands with one tap per k-tile");
  TMR_CHECK_ARG(!a.sab || (a.prec == TMR_MATH_BF16 && !a.pro &&
                           (MODE == MODE_FWD ? ((a.sab == 2 && var <= 1) || (a.sab == 3 && var == 0))
                            : MODE == MODE_DGRAD ? (a.sab == 3 && var == 0)
                                                 : ((a.sab == 1 || a.sab == 3) && var == 0))),
                "gemm: unsupported bf16-stored operand combination (sab %d, view %d, var %d)",
                a.sab, MODE, var);
  TMR_CHECK_ARG(!a.pro || ((a.pro & 1) ? (MODE != MODE_DGRAD && a.px_scale && a.px_shift) : true),
                "gemm: X-operand prologue needs scale/shift (forward or wgrad view)");
  TMR_CHECK_ARG(!a.pro || ((a.pro & 2) ? (MODE != MODE_FWD && a.pd_y && a.pd_a && a.pd_b && a.pd_c)
                                       : true),
                "gemm: dY-operand prologue needs y and coefficients (dgrad or wgrad view)");
  TMR_CHECK_ARG(uniform || (al && MODE == MODE_FWD),
                "gemm: per-element taps need aligned channels and the forward view");
  TMR_CHECK_ARG(!a.wt, "gemm: transposed weights (TMR_IO_WT_BF16 / TMR_IO_WT_F32) need the LDS-DMA "
                "path: bf16 dy with 8-channel multiples, or fp32 dy, 16-B aligned operands");
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

// per-view launchers (gemm_fwd.hip / gemm_dgrad.hip / gemm_wgrad.hip)
int launch_gemm_fwd(const GemmArgs& a, bool al, int splits, hipStream_t st);
int launch_gemm_dgrad(const GemmArgs& a, bool al, int splits, hipStream_t st);
int launch_gemm_dgrad_par(const GemmArgs* as, int n, hipStream_t st);
int launch_gemm_wgrad(const GemmArgs& a, bool al, int splits, hipStream_t st);

}  // namespace tmrg

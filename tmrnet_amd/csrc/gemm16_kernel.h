// bf16 implicit-GEMM engine on LDS-DMA staging (gfx950).  The bf16-math conv views whose operands
// are all stored as bf16 in HBM (tmr_conv_desc.io: x, dy and the weights -- the dgrad view reads a
// transposed [Cin][R][S][Cout] weight copy, TMR_IO_WT_BF16) run here instead of gemm_kernel's
// register-staged path:
//
//   * operands go global -> LDS with `buffer_load_dwordx4 ... lds` (LDS-DMA): no VGPR staging, no
//     conversion, no ds_write; each lane's source address is its own, so the implicit-GEMM gather
//     (pixel + tap offset, zero padding by out-of-range offsets -- an out-of-range LDS-DMA writes
//     zeros) costs a few VALU ops per 16-B piece;
//   * BK = 64 (four v_mfma_f32_32x32x16_bf16 k-steps per k-tile), two LDS stages: the k-tile t+1
//     pieces are issued right after the barrier that publishes tile t and land under its MFMAs;
//   * K-contiguous operands (FWD A/B, DGRAD A/B) use a [rows][64] image (128-B rows) with the
//     16-B chunk index XOR-swizzled by (row >> 1) & 7: every ds_read_b128 lane group of the MFMA
//     operand read hits 16 distinct bank quads.  The swizzle is applied to the SOURCE address of
//     the LDS-DMA (the LDS image itself is lane-linear) and to the read;
//   * the WGRAD operands are reduction-major in HBM (dY[m][co], X[pixel][c]): their image is
//     [64 k-rows][R columns] and the MFMA fragments come from ds_read_b64_tr_b16 (a 4x16 block
//     per 16 lanes, delivered column-major), two per 8-k fragment; chunks XOR-swizzled by k so
//     each 32-lane half covers all 64 banks.
//
// Accumulator layout, XCD-aware tile order and the epilogue (BN statistics, fused BN backward,
// beta, split-K slabs, dgrad parity scatter) are gemm_kernel's (epilogue_batched: branch-free
// buffer accesses, each chunk of rows issuing all its loads first -- the fused BN-backward dgrads
// are bound by that traffic), and the k order of the accumulation is the register-staged bf16
// path's, so FWD / DGRAD results are bit-identical to it.
#pragma once
#include "gemm16_select.h"
#include <cstring>
#include <type_traits>

namespace tmrg {

typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
#define TMR_LDS_AS __attribute__((address_space(3)))

// one 16-B LDS-DMA piece per lane: LDS dst = (wave-uniform) dst + 16 * lane
__device__ __forceinline__ void glds16(__amdgpu_buffer_rsrc_t r, unsigned char* dst, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (TMR_LDS_AS void*)dst, 16, voff, 0, 0, 0);
}

// reduction-major image with R columns: chunk swizzle of k-row k
template <int R>
__device__ __forceinline__ int mn_swz(int k) {
  return R >= 128 ? ((k & 3) << 2) : (((k >> 1) & 1) << 2);
}

// Fused BatchNorm-backward epilogue of the DGRAD view through LDS (the tile is written to LDS in
// row chunks, then each thread owns 8 consecutive columns of a row: 16-B / 32-B vector accesses of
// y, z (bf16 or fp32), the old dx (beta) and the new dx, instead of one scalar access per
// accumulator register).  Per row: beta, ReLU mask (z > 0, or y*scale+shift > 0, or bits, or
// none), store, and per-column sums of g and g*(y - mean); the tile's column sums -> bn_part (one
// partial row per m-tile, as epilogue_batched).
//
// The epilogue is HBM-bound (12-16 B per output element) and its rows are independent, so its
// global operands are software-pipelined: the first D rows of each thread are loaded before the
// main loop (they land under the MFMAs), and row t + D is issued right after row t is consumed.
// Every (row, 8-column group) belongs to one thread, so reading the old dx of a later row before
// this row's store cannot alias.  With loads issued one row at a time a thread keeps ~64 B in
// flight and the launch is latency-bound (3.6 TB/s on the 56x56 residual dgrads).
// 8 consecutive elements of the fused BN-backward dgrad's output at element offset `off`: fp32, or
// bf16 (already rounded values, GemmArgs::g16) as one 16-B store
__device__ __forceinline__ void store_g8(const GemmArgs& a, long off, const float (&v)[8]) {
  if (a.g16) {
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      w[e] = (__float_as_uint(v[2 * e]) >> 16) | (__float_as_uint(v[2 * e + 1]) & 0xffff0000u);
    *reinterpret_cast<uint4*>(reinterpret_cast<__bf16*>(a.C) + off) = make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    *reinterpret_cast<float4*>(a.C + off) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(a.C + off + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

// the 8 old-dx values of the fused BN-backward epilogue's beta at element offset `off` (fp32, or
// bf16 when GemmArgs::cold16), raw: (c0, c1) = 32 B of fp32, or c0 = 16 B of bf16
__device__ __forceinline__ void load_old8(const GemmArgs& a, long off, uint4& c0, uint4& c1,
                                          bool c16) {
  const void* base = a.Cold ? a.Cold : (const void*)a.C;
  if (c16) {
    c0 = *reinterpret_cast<const uint4*>(reinterpret_cast<const __bf16*>(base) + off);
  } else {
    c0 = *reinterpret_cast<const uint4*>(reinterpret_cast<const float*>(base) + off);
    c1 = *reinterpret_cast<const uint4*>(reinterpret_cast<const float*>(base) + off + 4);
  }
}
__device__ __forceinline__ void load_old8(const GemmArgs& a, long off, uint4& c0, uint4& c1) {
  load_old8(a, off, c0, c1, a.cold16);
}
__device__ __forceinline__ void unpack_old8(const uint4& c0, const uint4& c1, float (&old)[8],
                                            bool c16) {
  if (c16) {
    const uint32_t u[4] = {c0.x, c0.y, c0.z, c0.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      old[2 * e] = __uint_as_float(u[e] << 16);
      old[2 * e + 1] = __uint_as_float(u[e] & 0xffff0000u);
    }
  } else {
    const uint32_t u[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) old[e] = __uint_as_float(u[e]);
  }
}
__device__ __forceinline__ void unpack_old8(const GemmArgs& a, const uint4& c0, const uint4& c1,
                                            float (&old)[8]) {
  unpack_old8(c0, c1, old, a.cold16);
}

// Epilogue forms of the fused BN-backward dgrads (round 6): the flags a form fixes at compile time,
// so its row slots hold only the fields it loads.  EPF 1: the bf16-activation step -- y, z
// (mask 1) and the old gradient (beta) bf16, no ReLU bits; EPF 2: the fp32 step -- y and the old
// gradient fp32, no stored z (mask 0 / 2 / 3); EPF 0: every flag read at run time.
template <int EPF>
struct EpiForm {
  __device__ __forceinline__ static bool bn16(const GemmArgs& a) {
    return EPF == 1 ? true : (EPF == 2 ? false : a.bn16 != 0);
  }
  __device__ __forceinline__ static bool mask1(const GemmArgs& a) { return EPF == 2 ? false : a.bn_mask == 1; }
  __device__ __forceinline__ static bool mask3(const GemmArgs& a) { return EPF == 1 ? false : a.bn_mask == 3; }
  __device__ __forceinline__ static bool cold16(const GemmArgs& a) {
    return EPF == 1 ? true : (EPF == 2 ? false : a.cold16 != 0);
  }
};
// the form a launch qualifies for (host)
inline int epi_form(const GemmArgs& a) {
  if (a.bn16 && a.bn_mask != 3 && (a.beta == 0.f || a.cold16)) return 1;
  if (!a.bn16 && a.bn_mask != 1 && !a.cold16) return 2;
  return 0;
}

#ifndef TMR_EPI_DEPTH
#define TMR_EPI_DEPTH 3
#endif
// rows in flight of the 8-wave tiles' epilogue, loads issued after the main loop (0: their
// one-row-at-a-time epilogue_lds_bnbwd; 1-2 spill at the 128-VGPR budget of those tiles)
#ifndef TMR_EPI_LATE
#define TMR_EPI_LATE 0
#endif
// rows whose loads the 4-wave tiles add once the accumulators are staged (round 6): the
// accumulators are dead then, so the registers of TOP more rows are free; issued before the
// first row is consumed, so the whole tile's epilogue operands are in flight at once
#ifndef TMR_EPI_TOPUP
#define TMR_EPI_TOPUP 0
#endif
#ifndef TMR_EPI_TOPUP_F16
#define TMR_EPI_TOPUP_F16 5
#endif
#ifndef TMR_EPI_TOPUP_F32
#define TMR_EPI_TOPUP_F32 2
#endif
// the compile-time epilogue forms (EpiForm) for the 4-wave dgrads; 0 = the run-time form only.
// Round 6 (profiles/r6/epi_forms/): with the forms the bf16 tiles take every row of the tile in
// flight once the accumulators are staged (3 before the main loop + 5), the fp32 ones 3 + 2 (more
// spills): C5 dgrad view 50.1 -> 46.5 ms/step (304 -> 328 TF), C2 50.6 -> 49.9 ms; bit-identical.
// Tried: 5 bf16 rows before the main loop (no gain), the fp32 N >= 512 dgrads on the 4-wave tile
// (slower), 2 / 4 late rows in the 8-wave tiles (spill: C2 dgrad +2.4 ms).
#ifndef TMR_EPI_FORMS
#define TMR_EPI_FORMS 1
#endif
// rows in flight before the main loop in the bf16 form (4-wave tiles)
#ifndef TMR_EPI_DEPTH_F16
#define TMR_EPI_DEPTH_F16 TMR_EPI_DEPTH
#endif
// rows in flight after the main loop in the forms of the 8-wave tiles (0: one row at a time)
#ifndef TMR_EPI_LATE_F
#define TMR_EPI_LATE_F 0
#endif
template <int BM, int BN, int WM, int WN, int SMEMB, int DEPTH = TMR_EPI_DEPTH, int TOP = 0,
          int EPF = 0>
struct LdsBnbwd {
  using Form = EpiForm<EPF>;
  static constexpr int NT = 64 * WM * WN;
  static constexpr int LDC = BN + 4;                   // padded fp32 row of the staged tile
  static constexpr int CG = BN / 8;                    // column groups of 8
  static constexpr int RPP = NT / CG;                  // rows per pass over a chunk
  static constexpr int WR = BM / WM;                   // rows of one wave row-block
  static constexpr int RC0 = (SMEMB / 4 / LDC) / WR * WR;
  // rows staged per chunk (whole row-blocks; configs where one row-block does not fit never run
  // this epilogue)
  static constexpr int RCH = RC0 < WR ? WR : (RC0 < BM ? RC0 : BM);
  static constexpr int NCH = (BM + RCH - 1) / RCH;
  static constexpr int PC = (RCH + RPP - 1) / RPP;     // row slots of a thread per chunk
  static constexpr int NR = NCH * PC;                  // row slots of a thread
  static constexpr int D = NR < DEPTH ? NR : DEPTH;   // rows in flight during the main loop
  static constexpr int DT = NR < D + TOP ? NR : D + TOP;   // ... once the tile is staged
  static_assert(NT % CG == 0, "epilogue row partition");

  struct In {         // one row's global operands as loaded
    uint4 y0, y1, z0, z1, c0, c1;
    uint32_t bits;
    long off;
    bool ok;
  };

  // issue the loads of row slot t (tile-relative row r)
  __device__ __forceinline__ static void issue(const GemmArgs& a, int t, int m0, int n0, In& x) {
    const int etid = threadIdx.x;
    const int cg = etid % CG, rsub = etid / CG;
    const int ci = t / PC, j = t % PC;
    const int rr = rsub + j * RPP;                     // row within chunk ci
    const int nrow = (BM - ci * RCH) < RCH ? (BM - ci * RCH) : RCH;
    const int col = n0 + 8 * cg;
    const int row = m0 + ci * RCH + rr;
    x.ok = rr < nrow && col < a.N && row < a.M;
    long pix = row;
    if (x.ok && a.osy != 0) {   // the parity class's output pixel
      const uint32_t n = fdiv((uint32_t)row, a.dHW);
      const uint32_t rem = row - n * a.dHW.d;
      const uint32_t y = fdiv(rem, a.dW);
      const uint32_t xx = rem - y * a.dW.d;
      pix = ((long)n * a.oH + (long)y * a.osy + a.oyc) * a.oW + (long)xx * a.osx + a.oxc;
    }
    x.off = pix * a.ldc + col;
    if (!x.ok) return;
    const long off = x.off;
    if (Form::bn16(a)) {
      x.y0 = *reinterpret_cast<const uint4*>(reinterpret_cast<const __bf16*>(a.bn_y) + off);
      if (Form::mask1(a))
        x.z0 = *reinterpret_cast<const uint4*>(reinterpret_cast<const __bf16*>(a.bn_z) + off);
    } else {
      x.y0 = *reinterpret_cast<const uint4*>(a.bn_y + off);
      x.y1 = *reinterpret_cast<const uint4*>(a.bn_y + off + 4);
      if (Form::mask1(a)) {
        x.z0 = *reinterpret_cast<const uint4*>(a.bn_z + off);
        x.z1 = *reinterpret_cast<const uint4*>(a.bn_z + off + 4);
      }
    }
    if (Form::mask3(a)) x.bits = reinterpret_cast<const uint32_t*>(a.bn_z)[off >> 5];
    if (a.beta != 0.f) load_old8(a, off, x.c0, x.c1, Form::cold16(a));
  }

  __device__ __forceinline__ static void prefetch(const GemmArgs& a, int m0, int n0, In (&pf)[DT]) {
#pragma unroll
    for (int t = 0; t < D; ++t) issue(a, t, m0, n0, pf[t]);
  }

  template <int TM, int TN>
  __device__ __forceinline__ static void run(const GemmArgs& a, floatx16 (&acc)[TM][TN], float* lds,
                                             int m0, int n0, In (&pf)[DT]) {
    int etid = threadIdx.x;
    asm volatile("" : "+v"(etid));   // keep the epilogue's index math out of the main loop
    const int lane = etid & 63, wave = etid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int l31 = lane & 31, hh = lane >> 5;
    const int cg = etid % CG, rsub = etid / CG;
    const int col = n0 + 8 * cg;
    const bool okc = col < a.N;                   // N is a multiple of 8 (LDS-DMA engine)
    // per-column coefficients of this thread's 8 columns
    float mu[8], bsc[8], bsh[8], cs[8], cq[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = okc ? col + e : 0;
      mu[e] = okc ? a.bn_mean[c] : 0.f;
      bsc[e] = (okc && a.bn_mask == 2) ? a.bn_sc[c] : 0.f;
      bsh[e] = (okc && a.bn_mask == 2) ? a.bn_sh[c] : (a.bn_mask == 0 ? 1.f : 0.f);
      cs[e] = 0.f;
      cq[e] = 0.f;
    }
    const bool has_beta = a.beta != 0.f;
#pragma unroll
    for (int ci = 0; ci < NCH; ++ci) {
      // (1) the waves whose rows lie in chunk ci stage their accumulators
      __syncthreads();
      const int wr0 = wm * WR;
      if (wr0 >= ci * RCH && wr0 < ci * RCH + RCH) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int row = wr0 - ci * RCH + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hh;
              lds[row * LDC + wn * (BN / WN) + 32 * j + l31] = acc[i][j][r];
            }
      }
      __syncthreads();
      if (ci == 0) {   // the accumulators are staged: top the rows in flight up to DT
#pragma unroll
        for (int t = D; t < DT; ++t) issue(a, t, m0, n0, pf[t]);
      }
      // (2) this thread's rows of the chunk, 8 columns each
#pragma unroll
      for (int j = 0; j < PC; ++j) {
        const int t = ci * PC + j;
        In& x = pf[t % DT];
        if (x.ok) {
          const long off = x.off;
          float yv[8], zv[8], old[8];
          if (Form::bn16(a)) {
            const uint32_t yu[4] = {x.y0.x, x.y0.y, x.y0.z, x.y0.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              yv[2 * e] = __uint_as_float(yu[e] << 16);
              yv[2 * e + 1] = __uint_as_float(yu[e] & 0xffff0000u);
            }
            if (Form::mask1(a)) {
              const uint32_t zu[4] = {x.z0.x, x.z0.y, x.z0.z, x.z0.w};
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                zv[2 * e] = __uint_as_float(zu[e] << 16);
                zv[2 * e + 1] = __uint_as_float(zu[e] & 0xffff0000u);
              }
            }
          } else {
            const uint32_t yu[8] = {x.y0.x, x.y0.y, x.y0.z, x.y0.w, x.y1.x, x.y1.y, x.y1.z, x.y1.w};
#pragma unroll
            for (int e = 0; e < 8; ++e) yv[e] = __uint_as_float(yu[e]);
            if (Form::mask1(a)) {
              const uint32_t zu[8] = {x.z0.x, x.z0.y, x.z0.z, x.z0.w, x.z1.x, x.z1.y, x.z1.z, x.z1.w};
#pragma unroll
              for (int e = 0; e < 8; ++e) zv[e] = __uint_as_float(zu[e]);
            }
          }
          if (Form::mask3(a)) {   // ReLU mask bits: this thread's 8 elements share one word
            const uint32_t b8 = x.bits >> (off & 31);
#pragma unroll
            for (int e = 0; e < 8; ++e) zv[e] = ((b8 >> e) & 1u) ? 1.f : 0.f;
          } else if (!Form::mask1(a)) {
#pragma unroll
            for (int e = 0; e < 8; ++e) zv[e] = 0.f;
          }
          if (has_beta) {
            unpack_old8(x.c0, x.c1, old, Form::cold16(a));
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) old[e] = 0.f;
          }
          const int rr = rsub + j * RPP;
          const float4 a0 = *reinterpret_cast<const float4*>(lds + rr * LDC + 8 * cg);
          const float4 a1 = *reinterpret_cast<const float4*>(lds + rr * LDC + 8 * cg + 4);
          const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
          float v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float tv = fmaf(a.beta, old[e], av[e]);
            const bool keep = zv[e] + fmaf(yv[e], bsc[e], bsh[e]) > 0.f;
            tv = keep ? tv : 0.f;
            if (a.g16) tv = bf16_rne(tv);   // stored bf16: the partials describe the stored g
            v[e] = tv;
            cs[e] += tv;
            cq[e] = fmaf(tv, yv[e] - mu[e], cq[e]);
          }
          store_g8(a, off, v);
        }
        if (t + DT < NR) issue(a, t + DT, m0, n0, x);   // the slot's next row
      }
    }
    // (3) column sums over the RPP row slots -> bn_part
    __syncthreads();
    float* red = lds;   // [RPP][BN][2]
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(rsub * BN + 8 * cg + e) * 2] = cs[e];
      red[(rsub * BN + 8 * cg + e) * 2 + 1] = cq[e];
    }
    __syncthreads();
    for (int c = etid; c < BN; c += NT) {
      float t0 = 0.f, t1 = 0.f;
      for (int q = 0; q < RPP; ++q) {
        t0 += red[(q * BN + c) * 2];
        t1 += red[(q * BN + c) * 2 + 1];
      }
      if (n0 + c < a.N) a.bn_part[(long)(m0 / BM) * a.part_ld + n0 + c] = make_float2(t0, t1);
    }
  }
};

// The same epilogue with one row's loads at a time (no lookahead): the 8/16-wave tiles, which run
// at a 128-VGPR budget that LdsBnbwd's extra row set would spill.
template <int BM, int BN, int WM, int WN, int TM, int TN>
__device__ __forceinline__ void epilogue_lds_bnbwd(const GemmArgs& a, floatx16 (&acc)[TM][TN],
                                                   float* lds, int lds_floats, int m0, int n0) {
  constexpr int NT = 64 * WM * WN;
  constexpr int LDC = BN + 4;                   // padded fp32 row of the staged tile
  constexpr int CG = BN / 8;                    // column groups of 8
  constexpr int RPP = NT / CG;                  // rows processed per pass over the chunk
  static_assert(NT % CG == 0, "threads per column group");
  int etid = threadIdx.x;
  asm volatile("" : "+v"(etid));   // keep the epilogue's index math out of the main loop
  const int lane = etid & 63, wave = etid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int l31 = lane & 31, hh = lane >> 5;
  const int cg = etid % CG, rsub = etid / CG;
  const int col = n0 + 8 * cg;
  const bool okc = col < a.N;                   // N is a multiple of 8 (LDS-DMA engine)
  // per-column coefficients of this thread's 8 columns
  float mu[8], bsc[8], bsh[8], cs[8], cq[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = okc ? col + e : 0;
    mu[e] = okc ? a.bn_mean[c] : 0.f;
    bsc[e] = (okc && a.bn_mask == 2) ? a.bn_sc[c] : 0.f;
    bsh[e] = (okc && a.bn_mask == 2) ? a.bn_sh[c] : (a.bn_mask == 0 ? 1.f : 0.f);
    cs[e] = 0.f;
    cq[e] = 0.f;
  }
  const bool has_beta = a.beta != 0.f;
  const int rchunk = min(BM, (lds_floats / LDC) / (BM / WM) * (BM / WM));   // whole wave rows
  for (int r0 = 0; r0 < BM; r0 += rchunk) {
    // (1) the waves whose rows lie in [r0, r0 + rchunk) stage their accumulators
    __syncthreads();
    const int wr0 = wm * (BM / WM);
    if (wr0 >= r0 && wr0 < r0 + rchunk) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = wr0 - r0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hh;
            lds[row * LDC + wn * (BN / WN) + 32 * j + l31] = acc[i][j][r];
          }
    }
    __syncthreads();
    // (2) rows of the chunk, 8 columns per thread
    const int nrow = min(rchunk, BM - r0);
    for (int rr = rsub; rr < nrow; rr += RPP) {
      const int row = m0 + r0 + rr;
      const bool ok = okc && row < a.M;
      long pix = row;
      if (ok && a.osy != 0) {   // the parity class's output pixel
        const uint32_t n = fdiv((uint32_t)row, a.dHW);
        const uint32_t rem = row - n * a.dHW.d;
        const uint32_t y = fdiv(rem, a.dW);
        const uint32_t x = rem - y * a.dW.d;
        pix = ((long)n * a.oH + (long)y * a.osy + a.oyc) * a.oW + (long)x * a.osx + a.oxc;
      }
      const long off = pix * a.ldc + col;   // element offset in dx / y / z
      float yv[8], zv[8], old[8];
      if (ok) {
        if (a.bn16) {
          const uint4 yw = *reinterpret_cast<const uint4*>(reinterpret_cast<const __bf16*>(a.bn_y) + off);
          const uint32_t yu[4] = {yw.x, yw.y, yw.z, yw.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            yv[2 * e] = __uint_as_float(yu[e] << 16);
            yv[2 * e + 1] = __uint_as_float(yu[e] & 0xffff0000u);
          }
          if (a.bn_mask == 1) {
            const uint4 zw = *reinterpret_cast<const uint4*>(reinterpret_cast<const __bf16*>(a.bn_z) + off);
            const uint32_t zu[4] = {zw.x, zw.y, zw.z, zw.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              zv[2 * e] = __uint_as_float(zu[e] << 16);
              zv[2 * e + 1] = __uint_as_float(zu[e] & 0xffff0000u);
            }
          }
        } else {
          const float4 y0 = *reinterpret_cast<const float4*>(a.bn_y + off);
          const float4 y1 = *reinterpret_cast<const float4*>(a.bn_y + off + 4);
          yv[0] = y0.x; yv[1] = y0.y; yv[2] = y0.z; yv[3] = y0.w;
          yv[4] = y1.x; yv[5] = y1.y; yv[6] = y1.z; yv[7] = y1.w;
          if (a.bn_mask == 1) {
            const float4 z0 = *reinterpret_cast<const float4*>(a.bn_z + off);
            const float4 z1 = *reinterpret_cast<const float4*>(a.bn_z + off + 4);
            zv[0] = z0.x; zv[1] = z0.y; zv[2] = z0.z; zv[3] = z0.w;
            zv[4] = z1.x; zv[5] = z1.y; zv[6] = z1.z; zv[7] = z1.w;
          }
        }
        if (a.bn_mask == 3) {   // ReLU mask bits: this thread's 8 elements share one word
          const uint32_t wrd = reinterpret_cast<const uint32_t*>(a.bn_z)[off >> 5];
          const uint32_t b8 = wrd >> (off & 31);
#pragma unroll
          for (int e = 0; e < 8; ++e) zv[e] = ((b8 >> e) & 1u) ? 1.f : 0.f;
        } else if (a.bn_mask != 1) {
#pragma unroll
          for (int e = 0; e < 8; ++e) zv[e] = 0.f;
        }
        if (has_beta) {
          uint4 c0, c1;
          load_old8(a, off, c0, c1);
          unpack_old8(a, c0, c1, old);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) old[e] = 0.f;
        }
        const float4 a0 = *reinterpret_cast<const float4*>(lds + rr * LDC + 8 * cg);
        const float4 a1 = *reinterpret_cast<const float4*>(lds + rr * LDC + 8 * cg + 4);
        const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float t = fmaf(a.beta, old[e], av[e]);
          const bool keep = zv[e] + fmaf(yv[e], bsc[e], bsh[e]) > 0.f;
          t = keep ? t : 0.f;
          if (a.g16) t = bf16_rne(t);
          v[e] = t;
          cs[e] += t;
          cq[e] = fmaf(t, yv[e] - mu[e], cq[e]);
        }
        store_g8(a, off, v);
      }
    }
  }
  // (3) column sums over the RPP row slots -> bn_part
  __syncthreads();
  float* red = lds;   // [RPP][BN][2]
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[(rsub * BN + 8 * cg + e) * 2] = cs[e];
    red[(rsub * BN + 8 * cg + e) * 2 + 1] = cq[e];
  }
  __syncthreads();
  for (int c = etid; c < BN; c += NT) {
    float t0 = 0.f, t1 = 0.f;
    for (int q = 0; q < RPP; ++q) {
      t0 += red[(q * BN + c) * 2];
      t1 += red[(q * BN + c) * 2 + 1];
    }
    if (n0 + c < a.N) a.bn_part[(long)(m0 / BM) * a.part_ld + n0 + c] = make_float2(t0, t1);
  }
}

typedef float f32x4_t __attribute__((ext_vector_type(4)));

// F32: the fp32 form of the engine (every operand fp32 in HBM, GemmArgs::dma32).  The K-contiguous
// images are byte-identical -- [rows][128 B], 16-B chunks of 4 floats instead of 8 bf16, the same
// swizzle and LDS-DMA pieces -- so BK = 32 elements; each ds_read_b128 fragment holds 4
// consecutive k of one row, lane half hh the chunk 2s + hh, and feeds 4 v_mfma_f32_32x32x2_f32
// (MFMA t reduces k = 8s + t from half 0 and 8s + 4 + t from half 1: the same k for A and B).
// WGRAD (reduction-major images [32 k-rows][R floats]): fragment element t of k-step s is
// k = 8s + 2t + hh, one ds_read_b32 each; odd k-rows have their chunks XOR 8 (columns ^ 32), so
// the two lane halves (rows k, k + 1) read disjoint bank halves.
//
// PRO (fp32 form only; GemmArgs::pro): operand prologues -- the BatchNorm that produced an
// operand applied in LDS, so its output is never written to HBM.  Bit 1, the X operand (FWD A,
// WGRAD B): x' = relu(fmaf(x, scale[c], shift[c])) (bn_apply_k's arithmetic), 0 where the
// gather is out of range (the zero padding belongs to the post-ReLU tensor).  Bit 2, the dY
// operand (DGRAD A, WGRAD A): dy' = fmaf(A[c], g, fmaf(B[c], y, C[c])) (bn_bwd_apply's), with y
// brought into an LDS scratch image by a second LDS-DMA at g's offsets, 0 out of range.  Each
// lane transforms the 16-B pieces it issued, after its own LDS-DMA has landed (vmcnt) and
// before the barrier that publishes the k-tile, so no extra barrier; the coefficient tables
// are staged in LDS once per workgroup.
//
// NST = 1 (FWD launches of one k-tile, K <= BK: the second stage would never be used): one LDS
// stage -- 32-40 KB instead of 64-80 KB, so three 4-wave workgroups fit a CU instead of one or
// two: the short-reduction launches are bound by their epilogue's stores, and more workgroups
// keep more of them in flight.  Same k order and epilogue: bit-identical to NST = 2.
// waves per SIMD the launch bounds promise (the register budget of a config)
template <int BM, int BN, int WM, int WN, int NST>
constexpr int occ16() {
  return (WM * WN >= 16 || (WM * WN == 8 && (BM * BN <= 128 * 128 || NST == 1))) ? 4 : 2;
}

// the body of one workgroup: output tile `bid` (m-major over the n-tiles), reduction split `split`
template <int MODE, int BM, int BN, int WM, int WN, int TAPV, int PIPE, int F32, int PRO, int NST,
          int EPF = 0>
__device__ __forceinline__ void gemm16_body(const GemmArgs& a, const int bid, const int split) {
  constexpr uint32_t ES = F32 ? 4u : 2u;   // element bytes
  constexpr int EPC = 16 / ES;             // elements per 16-B chunk
  constexpr int BK = 128 / ES;             // elements per k-tile (128-B image rows)
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr bool MN = (MODE == MODE_WGRAD);   // both operands reduction-major
  constexpr int ABYTES = BM * 128, BBYTES = BN * 128, STAGE = ABYTES + BBYTES;   // 128-B rows
  constexpr int NIA = ABYTES / (1024 * NW), NIB = BBYTES / (1024 * NW);   // pieces / wave / tile
  static_assert(NIA >= 1 && NIB >= 1 && NIA * 1024 * NW == ABYTES && NIB * 1024 * NW == BBYTES,
                "LDS-DMA pieces per wave");
  static_assert(TM >= 1 && TN >= 1, "wave tile");
  static_assert(!MN || (BM >= 64 && BN >= 64), "reduction-major images need >= 64 columns");
  // reduction-major images: 16-B chunks per k-row
  constexpr int CPRA = BM * (int)ES / 16, CPRB = BN * (int)ES / 16;
  using Frag = typename std::conditional<F32 != 0, f32x4_t, bf16x8>::type;
  constexpr int EPI = WM * BN * 2 * 4;
  static_assert(NST == 2 || (NST == 1 && MODE != MODE_WGRAD && (PRO & 2) == 0),
                "one-stage form: FWD / DGRAD, no dY prologue");
  // the DGRAD view's LDS-staged BN-backward epilogue stages the whole tile at once where it fits
  // 70 KB (every dgrad tile but 256x256: a few KB over the two k-tile stages), so the
  // accumulators are dead before its global loads start; else whole wave row-blocks per chunk
  constexpr int LDSROWB = (BN + 4) * (BM / WM) * 4, LDSFULL = (BN + 4) * BM * 4;
  constexpr int LDSNEED = MODE != MODE_DGRAD ? 0 : (LDSFULL <= 70 * 1024 ? LDSFULL : LDSROWB);
  constexpr int SMEM1 = STAGE > EPI ? (STAGE > LDSNEED ? STAGE : LDSNEED) : (EPI > LDSNEED ? EPI : LDSNEED);
  constexpr int SMEM2 = 2 * STAGE > EPI ? 2 * STAGE : EPI;
  constexpr int SMEM = NST == 1 ? SMEM1 : (SMEM2 > LDSNEED ? SMEM2 : LDSNEED);
  static_assert(!(PRO & 1) || MODE != MODE_DGRAD, "X prologue: FWD / WGRAD views");
  static_assert(!(PRO & 2) || MODE != MODE_FWD, "dY prologue: DGRAD / WGRAD views");
  // prologue regions after the stages / epilogue buffer: dY's y image (one stage: each lane reads
  // back only the pieces it issued), dY coefficients A|B|C, X scale|shift
  constexpr int YIMG = (PRO & 2) ? ABYTES : 0;
  constexpr int DCOEF = (PRO & 2) ? 3 * PRO_DMAX * 4 : 0;
  constexpr int XCOEF = (PRO & 1) ? 2 * PRO_XMAX * 4 : 0;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM + YIMG + DCOEF + XCOEF];
  unsigned char* const ysm = smem + SMEM;
  float* const dcoef = reinterpret_cast<float*>(smem + SMEM + YIMG);
  float* const xcoef = reinterpret_cast<float*>(smem + SMEM + YIMG + DCOEF);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int l31 = lane & 31, hh = lane >> 5;

  const int nnt = (a.N + BN - 1) / BN;
  const int m0 = (bid / nnt) * BM;
  const int n0 = (bid % nnt) * BN;

  int kbeg = 0, kend = a.K;
  if (MODE == MODE_WGRAD) {
    kbeg = split * a.kchunk;
    kend = min(a.K, kbeg + a.kchunk);
  }
  const int ntiles = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  const __amdgpu_buffer_rsrc_t rA = make_rsrc(a.A, a.Abytes);
  const __amdgpu_buffer_rsrc_t rB = make_rsrc(a.B, a.Bbytes);
  const int cmask = (1 << a.log2C) - 1;

  // ---------------- per-lane piece state (fixed across k-tiles) ----------------
  // K-contiguous pieces: piece q of this wave = image rows 8 * (wave + NW * q) .. + 7, lane -> row
  // + lane / 8, chunk (lane & 7) ^ swizzle
  auto kc_row = [&](int q) { return 8 * (wave + NW * q) + (lane >> 3); };
  auto kc_chunk = [&](int q) { return (lane & 7) ^ ((kc_row(q) >> 1) & 7); };
  // reduction-major pieces (R columns): piece q = 64 chunks = 512 / R k-rows of the image

  // A: FWD / DGRAD gathered rows (pixel byte offset, y, x, in range)
  uint32_t apix[MN ? 1 : NIA];
  int ay[MN ? 1 : NIA], ax[MN ? 1 : NIA], ach[MN ? 1 : NIA];
  bool aok[MN ? 1 : NIA];
  // A: WGRAD dY columns (co byte offset), k-row of the piece
  uint32_t aco[MN ? NIA : 1];
  int akr[MN ? NIA : 1];
  bool acok[MN ? NIA : 1];
  if constexpr (!MN) {
#pragma unroll
    for (int q = 0; q < NIA; ++q) {
      const int m = m0 + kc_row(q);
      aok[q] = m < a.M;
      const uint32_t mm = aok[q] ? (uint32_t)m : 0u;
      const uint32_t n = fdiv(mm, a.dHW);
      const uint32_t rem = mm - n * a.dHW.d;
      const uint32_t y = fdiv(rem, a.dW);
      const uint32_t x = rem - y * a.dW.d;
      ay[q] = (int)y * a.sy;
      ax[q] = (int)x * a.sx;
      apix[q] = (uint32_t)(((int)n * a.Hs + ay[q]) * a.Ws + ax[q]) * (uint32_t)a.lds * ES;
      ach[q] = EPC * kc_chunk(q);
    }
  } else {
#pragma unroll
    for (int q = 0; q < NIA; ++q) {
      const int s = 64 * (wave + NW * q) + lane;
      const int k = s / CPRA;
      const int ch = (s % CPRA) ^ (F32 ? (k & 1) << 3 : mn_swz<BM>(k));
      const int i = m0 + EPC * ch;
      akr[q] = k;
      acok[q] = i < a.M;
      aco[q] = (uint32_t)i * ES;
    }
  }
  // B: FWD weight rows / DGRAD transposed-weight rows (row byte offset, chunk), WGRAD X columns
  uint32_t brow[MN ? 1 : NIB];
  int bch[MN ? 1 : NIB];
  bool bok[NIB];
  int bdy[MN ? NIB : 1], bdx[MN ? NIB : 1], bkr[MN ? NIB : 1];
  uint32_t bco[MN ? NIB : 1];
  if constexpr (!MN) {
#pragma unroll
    for (int q = 0; q < NIB; ++q) {
      const int j = n0 + kc_row(q);
      bok[q] = j < a.N;
      const uint32_t jj = bok[q] ? (uint32_t)j : 0u;
      brow[q] = jj * (uint32_t)(MODE == MODE_DGRAD ? a.ldbt : a.ldb) * ES;
      bch[q] = EPC * kc_chunk(q);
    }
  } else {
#pragma unroll
    for (int q = 0; q < NIB; ++q) {
      const int s = 64 * (wave + NW * q) + lane;
      const int k = s / CPRB;
      const int ch = (s % CPRB) ^ (F32 ? (k & 1) << 3 : mn_swz<BN>(k));
      const int j = n0 + EPC * ch;
      const int tap = a.ntaps == 1 ? 0 : (j >> a.log2C);
      const int c = a.ntaps == 1 ? j : (j & cmask);
      int ri, si;
      tap_split(a, tap, ri, si);
      bdy[q] = a.oy0 + a.dyr * ri;
      bdx[q] = a.ox0 + a.dxs * si;
      bco[q] = (uint32_t)c * ES;
      bok[q] = j < a.N && tap < a.ntaps;
      bkr[q] = k;
    }
  }

  // prologue pieces of the k-tile in flight: in range, first channel of the 4 (A: X or dY,
  // B: WGRAD's X); set by stage(), consumed by transform() of the same tile
  bool pokA[PRO ? NIA : 1], pokB[PRO ? NIB : 1];
  int pcA[PRO ? NIA : 1];
  const __amdgpu_buffer_rsrc_t rY = make_rsrc((PRO & 2) ? a.pd_y : a.A, a.Abytes);

  // ---------------- stage one k-tile into LDS buffer `buf` ----------------
  auto stage = [&](int kt, int buf) {
    const int kb = kbeg + kt * BK;
    unsigned char* As = smem + buf * STAGE;
    unsigned char* Bs = As + ABYTES;
    if constexpr (!MN) {
      // tap of this k-tile (uniform unless TAPV)
      int tapU = 0, cbU = kb, dyU = a.oy0, dxU = a.ox0;
      if (!TAPV && a.ntaps != 1) {
        tapU = kb >> a.log2C;
        cbU = kb & cmask;
        int ri, si;
        tap_split(a, tapU, ri, si);
        dyU = a.oy0 + a.dyr * ri;
        dxU = a.ox0 + a.dxs * si;
      }
#pragma unroll
      for (int q = 0; q < NIA; ++q) {
        const int k = kb + ach[q];
        int tap = tapU, c = cbU + ach[q], dy = dyU, dx = dxU;
        if (TAPV) {
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
        const uint32_t off = apix[q] + (uint32_t)((dy * a.Ws + dx) * a.lds + c) * ES;
        glds16(rA, As + 1024 * (wave + NW * q), ok ? off : OOB);
        if constexpr (PRO != 0) {
          pokA[q] = ok;
          pcA[q] = c;
          if constexpr ((PRO & 2) != 0) glds16(rY, ysm + 1024 * (wave + NW * q), ok ? off : OOB);
        }
      }
      if constexpr (MODE == MODE_FWD) {
        // B[j][k] = W[co][tap][c]: k-contiguous rows of the KRSC weights
#pragma unroll
        for (int q = 0; q < NIB; ++q) {
          const int k = kb + bch[q];
          const bool ok = bok[q] && k < kend;
          glds16(rB, Bs + 1024 * (wave + NW * q), ok ? brow[q] + (uint32_t)k * ES : OOB);
        }
      } else {
        // B[j=ci][k=(tap,co)] = Wt[ci][rs(tap)][co]
        int tapB = 0, coB = kb, rsB = 0;
        if (!TAPV) {
          if (a.ntaps != 1) {
            tapB = kb >> a.log2C;
            coB = kb & cmask;
          }
          int ri, si;
          tap_split(a, tapB, ri, si);
          rsB = (a.wr0 + a.wst * ri) * a.wS + (a.ws0 + a.wst * si);
        }
#pragma unroll
        for (int q = 0; q < NIB; ++q) {
          const int k = kb + bch[q];
          int tap = tapB, co = coB + bch[q], rs = rsB;
          if (TAPV) {
            tap = k >> a.log2C;
            co = k & cmask;
            int ri, si;
            tap_split(a, tap, ri, si);
            rs = (a.wr0 + a.wst * ri) * a.wS + (a.ws0 + a.wst * si);
          }
          const bool ok = bok[q] && k < kend && tap < a.ntaps;
          const uint32_t off = brow[q] + (uint32_t)((rs << a.log2C) + co) * ES;
          glds16(rB, Bs + 1024 * (wave + NW * q), ok ? off : OOB);
        }
      }
    } else {
      // WGRAD A[k=m][i=co] = dY[m][co]
#pragma unroll
      for (int q = 0; q < NIA; ++q) {
        const int m = kb + akr[q];
        const bool ok = acok[q] && m < kend;
        const uint32_t off = (uint32_t)m * (uint32_t)a.ldb * ES + aco[q];
        glds16(rA, As + 1024 * (wave + NW * q), ok ? off : OOB);
        if constexpr ((PRO & 2) != 0) {
          pokA[q] = ok;
          pcA[q] = (int)(aco[q] / ES);
          glds16(rY, ysm + 1024 * (wave + NW * q), ok ? off : OOB);
        }
      }
      // WGRAD B[k=m][j=(tap,c)] = X[src(m, tap)][c]
#pragma unroll
      for (int q = 0; q < NIB; ++q) {
        const int m = kb + bkr[q];
        const uint32_t mm = m < kend ? (uint32_t)m : 0u;
        const uint32_t n = fdiv(mm, a.dHW);
        const uint32_t rem = mm - n * a.dHW.d;
        const uint32_t y = fdiv(rem, a.dW);
        const uint32_t x = rem - y * a.dW.d;
        const int ys = (int)y * a.sy + bdy[q], xs = (int)x * a.sx + bdx[q];
        const bool ok = m < kend && bok[q] && (unsigned)ys < (unsigned)a.Hs &&
                        (unsigned)xs < (unsigned)a.Ws;
        const uint32_t off = (uint32_t)(((int)n * a.Hs + ys) * a.Ws + xs) * (uint32_t)a.lds * ES + bco[q];
        glds16(rB, Bs + 1024 * (wave + NW * q), ok ? off : OOB);
        if constexpr ((PRO & 1) != 0) pokB[q] = ok;
      }
    }
  };

  // ---------------- operand prologues on this lane's landed pieces of buffer `buf` ----------------
  auto transform = [&](int buf) {
    unsigned char* As = smem + buf * STAGE;
    unsigned char* Bs = As + ABYTES;
    if constexpr ((PRO & 2) != 0 && F32 == 0) {   // dY = A operand (DGRAD, WGRAD), bf16 pieces
      // 8 channels c .. c + 7 of the masked gradient g and of y, both stored bf16:
      // fmaf(A, g, fmaf(B, y, C)) rounded RNE -- bn_bwd_apply8_a16's arithmetic, so the operand
      // equals the dy that pass would have stored
#pragma unroll
      for (int q = 0; q < NIA; ++q) {
        uint4* p = reinterpret_cast<uint4*>(As + 1024 * (wave + NW * q) + 16 * lane);
        const uint4 gw = *p;
        const uint4 yw = *reinterpret_cast<const uint4*>(ysm + 1024 * (wave + NW * q) + 16 * lane);
        const uint32_t gu[4] = {gw.x, gw.y, gw.z, gw.w}, yu[4] = {yw.x, yw.y, yw.z, yw.w};
        const int c = pcA[q];
        uint32_t w[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float4 A4 = *reinterpret_cast<const float4*>(dcoef + c + 4 * h);
          const float4 B4 = *reinterpret_cast<const float4*>(dcoef + PRO_DMAX + c + 4 * h);
          const float4 C4 = *reinterpret_cast<const float4*>(dcoef + 2 * PRO_DMAX + c + 4 * h);
          const float o0 = fmaf(A4.x, __uint_as_float(gu[2 * h] << 16),
                                fmaf(B4.x, __uint_as_float(yu[2 * h] << 16), C4.x));
          const float o1 = fmaf(A4.y, __uint_as_float(gu[2 * h] & 0xffff0000u),
                                fmaf(B4.y, __uint_as_float(yu[2 * h] & 0xffff0000u), C4.y));
          const float o2 = fmaf(A4.z, __uint_as_float(gu[2 * h + 1] << 16),
                                fmaf(B4.z, __uint_as_float(yu[2 * h + 1] << 16), C4.z));
          const float o3 = fmaf(A4.w, __uint_as_float(gu[2 * h + 1] & 0xffff0000u),
                                fmaf(B4.w, __uint_as_float(yu[2 * h + 1] & 0xffff0000u), C4.w));
          typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
          const bf16x2_t lo = {(__bf16)o0, (__bf16)o1}, hi = {(__bf16)o2, (__bf16)o3};
          w[2 * h] = __builtin_bit_cast(uint32_t, lo);
          w[2 * h + 1] = __builtin_bit_cast(uint32_t, hi);
        }
        *p = pokA[q] ? make_uint4(w[0], w[1], w[2], w[3]) : make_uint4(0u, 0u, 0u, 0u);
      }
    } else if constexpr ((PRO & 2) != 0) {   // dY = A operand (DGRAD, WGRAD), fp32
#pragma unroll
      for (int q = 0; q < NIA; ++q) {
        float4* p = reinterpret_cast<float4*>(As + 1024 * (wave + NW * q) + 16 * lane);
        const float4 g = *p;
        const float4 yv = *reinterpret_cast<const float4*>(ysm + 1024 * (wave + NW * q) + 16 * lane);
        const int c = pcA[q];
        const float4 A4 = *reinterpret_cast<const float4*>(dcoef + c);
        const float4 B4 = *reinterpret_cast<const float4*>(dcoef + PRO_DMAX + c);
        const float4 C4 = *reinterpret_cast<const float4*>(dcoef + 2 * PRO_DMAX + c);
        float4 o;
        o.x = fmaf(A4.x, g.x, fmaf(B4.x, yv.x, C4.x));
        o.y = fmaf(A4.y, g.y, fmaf(B4.y, yv.y, C4.y));
        o.z = fmaf(A4.z, g.z, fmaf(B4.z, yv.z, C4.z));
        o.w = fmaf(A4.w, g.w, fmaf(B4.w, yv.w, C4.w));
        *p = pokA[q] ? o : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    if constexpr ((PRO & 1) != 0) {   // X = A operand (FWD) or B operand (WGRAD)
      constexpr int NX = MODE == MODE_FWD ? NIA : NIB;
#pragma unroll
      for (int q = 0; q < NX; ++q) {
        unsigned char* img = MODE == MODE_FWD ? As : Bs;
        int c;
        bool ok;
        if constexpr (MODE == MODE_FWD) {
          c = pcA[q];
          ok = pokA[q];
        } else {
          c = (int)(bco[q] / ES);
          ok = pokB[q];
        }
        if constexpr (F32) {
          float4* p = reinterpret_cast<float4*>(img + 1024 * (wave + NW * q) + 16 * lane);
          const float4 v = *p;
          const float4 sc = *reinterpret_cast<const float4*>(xcoef + c);
          const float4 sh = *reinterpret_cast<const float4*>(xcoef + PRO_XMAX + c);
          float4 o;
          o.x = fmaxf(fmaf(v.x, sc.x, sh.x), 0.f);
          o.y = fmaxf(fmaf(v.y, sc.y, sh.y), 0.f);
          o.z = fmaxf(fmaf(v.z, sc.z, sh.z), 0.f);
          o.w = fmaxf(fmaf(v.w, sc.w, sh.w), 0.f);
          *p = ok ? o : make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
          // bf16 piece: 8 channels c .. c + 7 of the stored pre-BN y; relu(fmaf(y, sc, sh))
          // rounded RNE -- bn_apply8_a16_k's arithmetic, so the operand equals the z it would
          // have stored
          uint4* p = reinterpret_cast<uint4*>(img + 1024 * (wave + NW * q) + 16 * lane);
          const uint4 v = *p;
          const uint32_t u[4] = {v.x, v.y, v.z, v.w};
          uint32_t w[4];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const float4 sc = *reinterpret_cast<const float4*>(xcoef + c + 4 * h);
            const float4 sh = *reinterpret_cast<const float4*>(xcoef + PRO_XMAX + c + 4 * h);
            const float o0 = fmaxf(fmaf(__uint_as_float(u[2 * h] << 16), sc.x, sh.x), 0.f);
            const float o1 = fmaxf(fmaf(__uint_as_float(u[2 * h] & 0xffff0000u), sc.y, sh.y), 0.f);
            const float o2 = fmaxf(fmaf(__uint_as_float(u[2 * h + 1] << 16), sc.z, sh.z), 0.f);
            const float o3 = fmaxf(fmaf(__uint_as_float(u[2 * h + 1] & 0xffff0000u), sc.w, sh.w), 0.f);
            typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
            const bf16x2_t lo = {(__bf16)o0, (__bf16)o1}, hi = {(__bf16)o2, (__bf16)o3};
            w[2 * h] = __builtin_bit_cast(uint32_t, lo);
            w[2 * h + 1] = __builtin_bit_cast(uint32_t, hi);
          }
          *p = ok ? make_uint4(w[0], w[1], w[2], w[3]) : make_uint4(0u, 0u, 0u, 0u);
        }
      }
    }
  };

  // ---------------- MFMA operand reads ----------------
  // K-contiguous: row `row`, k-step s -> 8 k at chunk 2s + hh; the swizzle depends on row bits
  // 1..3 only, which are l31's (the tile bases are multiples of 32)
  const int kx = (l31 >> 1) & 7;
  // reduction-major (tr reads): lane (g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3) supplies
  // k-row 16s + 8(g >> 1) + 4t + q, columns cb + 16(g & 1) + 4p .. + 3
  const int tg = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;
  auto tr_frag = [&](const unsigned char* img, int R, int swz, int cb, int s) -> bf16x8 {
    const int col = cb + 16 * (tg & 1) + 4 * tp;
    const int k0 = 16 * s + 8 * (tg >> 1) + tq;
    const uint32_t cbyte = (uint32_t)((((col >> 3) ^ swz) << 4) + (col & 7) * 2);
    const s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (TMR_LDS_AS s16x4_t*)(img + k0 * R * 2 + cbyte));
    const s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (TMR_LDS_AS s16x4_t*)(img + (k0 + 4) * R * 2 + cbyte));
    const s16x8_t w = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, w);
  };
  const int swzA = mn_swz<BM>(tq), swzB = mn_swz<BN>(tq);
  // fp32 reduction-major fragment: element t = k-row 8s + 2t + hh of column cb + l31 (chunk
  // swizzle of that row: hh << 3)
  auto mn_frag32 = [&](const unsigned char* img, int R, int cb, int s) -> f32x4_t {
    const int col = cb + l31;
    const uint32_t cbyte = (uint32_t)((((col >> 2) ^ (hh << 3)) << 4) + (col & 3) * 4);
    f32x4_t v;
#pragma unroll
    for (int t = 0; t < 4; ++t)
      v[t] = *reinterpret_cast<const float*>(img + (8 * s + 2 * t + hh) * R * 4 + cbyte);
    return v;
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // the LDS-staged BN-backward epilogue (whole wave row-blocks of (BM / WM) padded rows must fit:
  // all configs but 256x256, which the dgrad tile rules never pick): its first rows' global
  // operands are loaded now and land under the main loop
  constexpr bool LDSEPI = MODE == MODE_DGRAD && LDSROWB <= SMEM;
  // prefetching form (LdsBnbwd): the 4-wave tiles issue their first rows' loads before the main
  // loop; the 8-wave ones (128-VGPR budget) right after it, two rows deep, once the whole tile is
  // staged (their accumulators are dead by then); the 16-wave ones keep epilogue_lds_bnbwd
  constexpr bool PRE = LDSEPI && NW < 8;
  constexpr int LATED = EPF != 0 ? TMR_EPI_LATE_F : TMR_EPI_LATE;
  constexpr bool LATE = LDSEPI && NW == 8 && LDSNEED == LDSFULL && LATED > 0;
  // a compile-time form (EPF 1 / 2) drops the fields its rows never load: then more rows of the
  // tile go in flight -- before the main loop (DEPTH) and once the accumulators are staged (TOP)
  // (the late rows of the 8-wave tiles are issued once the accumulators are staged: DEPTH 0)
  using Epi = LdsBnbwd<BM, BN, WM, WN, SMEM,
                      PRE ? (EPF == 1 ? TMR_EPI_DEPTH_F16 : TMR_EPI_DEPTH) : (LATE ? 0 : 1),
                      PRE ? (EPF == 1 ? TMR_EPI_TOPUP_F16 : (EPF == 2 ? TMR_EPI_TOPUP_F32 : TMR_EPI_TOPUP))
                          : (LATE ? LATED : 0),
                      EPF>;
  typename Epi::In pf[(PRE || LATE) ? Epi::DT : 1];
  if constexpr (PRE) {
    if (a.bn_part != nullptr) Epi::prefetch(a, m0, n0, pf);
  }

  const int arow0 = wm * (BM / WM) + l31;
  const int brow0 = wn * (BN / WN) + l31;
  // the operand fragments of k-step s of LDS buffer buf
  auto frags = [&](int buf, int s, Frag (&av)[TM], Frag (&bv)[TN]) {
    const unsigned char* As = smem + buf * STAGE;
    const unsigned char* Bs = As + ABYTES;
    const int ch = (2 * s + hh) ^ kx;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if constexpr (!MN)
        av[i] = *reinterpret_cast<const Frag*>(As + (arow0 + 32 * i) * 128 + (ch << 4));
      else if constexpr (!F32)
        av[i] = tr_frag(As, BM, swzA, wm * (BM / WM) + 32 * i, s);
      else
        av[i] = mn_frag32(As, BM, wm * (BM / WM) + 32 * i, s);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if constexpr (!MN)
        bv[j] = *reinterpret_cast<const Frag*>(Bs + (brow0 + 32 * j) * 128 + (ch << 4));
      else if constexpr (!F32)
        bv[j] = tr_frag(Bs, BN, swzB, wn * (BN / WN) + 32 * j, s);
      else
        bv[j] = mn_frag32(Bs, BN, wn * (BN / WN) + 32 * j, s);
    }
  };
  auto mfmas = [&](const Frag (&av)[TM], const Frag (&bv)[TN]) {
    if (PIPE) __builtin_amdgcn_s_setprio(1);
    if constexpr (F32) {
      // t outermost: TM * TN independent accumulator chains between dependent MFMAs
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i][t], bv[j][t], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (PIPE) __builtin_amdgcn_s_setprio(0);
  };
  // k-steps per k-tile: two 16-B chunks (lane halves) per step -> 16 bf16 or 8 floats
  constexpr int KSTEPS = BK / (2 * EPC);
  static_assert(KSTEPS == 4, "four k-steps per k-tile (the PIPE 1 schedule)");
  auto compute = [&](int buf) {
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
      Frag av[TM], bv[TN];
      frags(buf, s, av, bv);
      mfmas(av, bv);
    }
  };

  if constexpr (PRO != 0) {
    // coefficient tables -> LDS (published by the barrier below, before any transform)
    if constexpr ((PRO & 2) != 0) {
      const int cd = MODE == MODE_WGRAD ? a.ldb : a.lds;
      for (int i = tid; i < cd; i += 64 * NW) {
        dcoef[i] = a.pd_a[i];
        dcoef[PRO_DMAX + i] = a.pd_b[i];
        dcoef[2 * PRO_DMAX + i] = a.pd_c[i];
      }
    }
    if constexpr ((PRO & 1) != 0) {
      for (int i = tid; i < a.lds; i += 64 * NW) {
        xcoef[i] = a.px_scale[i];
        xcoef[PRO_XMAX + i] = a.px_shift[i];
      }
    }
    __syncthreads();
  }

  // ---------------- main loop: two LDS stages ----------------
  // Iteration kt: wait for this wave's pieces of tile kt, barrier (every wave's pieces landed;
  // every wave finished reading the other buffer in iteration kt-1), issue tile kt+1 into the
  // other buffer, MFMAs on tile kt while it lands.
  if (ntiles > 0 && PIPE == 0) {
    stage(0, 0);
    for (int kt = 0; kt < ntiles; ++kt) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if constexpr (PRO != 0) transform(kt & 1);
      __syncthreads();
      if (kt + 1 < ntiles) stage(kt + 1, (kt + 1) & 1);
      compute(kt & 1);
    }
  } else if (NST == 1 && ntiles > 0) {
    // one stage (the host launches this form for one k-tile; a longer reduction is still
    // correct, serialised: barrier, issue, wait)
    for (int kt = 0; kt < ntiles; ++kt) {
      if (kt > 0) __syncthreads();   // every wave's reads of tile kt - 1 done
      stage(kt, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if constexpr (PRO != 0) transform(0);
      __syncthreads();
      compute(0);
    }
  } else if (ntiles > 0) {
    // PIPE 1: the first k-step's fragment reads go out before the LDS-DMA issue of the next
    // tile (its address arithmetic then overlaps their latency), each later k-step's reads
    // before the previous k-step's MFMAs; MFMA clusters at raised priority
    stage(0, 0);
    for (int kt = 0; kt < ntiles; ++kt) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if constexpr (PRO != 0) transform(kt & 1);
      __syncthreads();
      const int buf = kt & 1;
      Frag a0[TM], b0[TN], a1[TM], b1[TN];
      frags(buf, 0, a0, b0);
      if (kt + 1 < ntiles) stage(kt + 1, buf ^ 1);
      frags(buf, 1, a1, b1);
      mfmas(a0, b0);
      frags(buf, 2, a0, b0);
      mfmas(a1, b1);
      frags(buf, 3, a1, b1);
      mfmas(a0, b0);
      mfmas(a1, b1);
    }
  }
  __syncthreads();   // LDS reads done (no LDS-DMA in flight) before the epilogue reuses smem

  if constexpr (LDSEPI) {
    if (a.bn_part != nullptr) {   // (the only form that reads mask-3 bits: launch_gemm16_t)
      if constexpr (PRE) {
        Epi::run(a, acc, reinterpret_cast<float*>(smem), m0, n0, pf);
      } else if constexpr (LATE) {
        Epi::prefetch(a, m0, n0, pf);
        Epi::run(a, acc, reinterpret_cast<float*>(smem), m0, n0, pf);
      } else
        epilogue_lds_bnbwd<BM, BN, WM, WN, TM, TN>(a, acc, reinterpret_cast<float*>(smem), SMEM / 4,
                                                    m0, n0);
      return;
    }
  }
  epilogue_batched<MODE, BM, BN, WM, WN, TM, TN>(a, acc, reinterpret_cast<float*>(smem), m0, n0,
                                                 split);
}

template <int MODE, int BM, int BN, int WM, int WN, int TAPV, int PIPE = 1, int F32 = 0, int PRO = 0,
          int NST = 2, int EPF = 0>
__global__ __launch_bounds__(64 * WM * WN, (occ16<BM, BN, WM, WN, NST>()))
void gemm16_kernel(const GemmArgs a) {
  int bid, split;
  xcd_work(bid, split);   // XCD-aware tile order (gemm_kernel.h)
  gemm16_body<MODE, BM, BN, WM, WN, TAPV, PIPE, F32, PRO, NST, EPF>(a, bid, split);
}

// Tile w of a GemmPar launch -> (class, tile of that class).  The classes' tiles go out in
// chunks of PAR_G consecutive tiles, round-robin over the classes (sorted by tile count, largest
// first; chunk round r holds chunk r of every class with more than r chunks), so each XCD's
// contiguous range of w holds every class in proportion while the workgroups resident on one XCD
// at a time mostly belong to one class.  Measured (profiles/r5/dgrad_par/): per-tile round-robin,
// which puts the classes side by side on every CU, and class-major order (two XCDs per class)
// both ran the strided dgrads ~1.3-2x slower than four launches; chunks of 32-128 tiles ran them
// 5-7% faster (launch ramps and tails gone).  The grid is padded to whole chunks: t past the
// class's tiles is a workgroup with nothing to do.
__device__ __forceinline__ void par_tile(const GemmPar& p, int w, int& cls, int& t) {
  const int ch = w / PAR_G, off = w - ch * PAR_G;
  int base = 0, prev = 0;
  cls = 0;
  t = 1 << 30;
  for (int n = p.n; n > 0; --n) {
    const int tn = (p.c[n - 1].tiles + PAR_G - 1) / PAR_G;
    const int span = n * (tn - prev);
    if (ch < base + span) {
      const int q = ch - base;
      cls = q % n;
      t = (prev + q / n) * PAR_G + off;
      return;
    }
    base += span;
    prev = tn;
  }
}

template <int BM, int BN, int WM, int WN, int F32, int EPF = 0>
__global__ __launch_bounds__(64 * WM * WN, (occ16<BM, BN, WM, WN, 2>()))
void gemm16_par_kernel(const GemmPar p) {
  int w, split;
  xcd_work(w, split);
  int cls, t;
  par_tile(p, w, cls, t);
  cls = __builtin_amdgcn_readfirstlane(cls);
  t = __builtin_amdgcn_readfirstlane(t);
  if (t >= p.c[cls].tiles) return;   // the padding of a class's last chunk
  // the class's own values, each made opaque in an SGPR: loaded from the kernel arguments at a
  // class-dependent offset, the compiler would otherwise re-load them inside the main loop (its
  // waits on those scalar loads also drain the LDS reads, lgkmcnt)
  GemmArgs a = p.a;
  const ParClass& c = p.c[cls];
  auto own = [](auto v) {
    asm volatile("" : "+s"(v));
    return v;
  };
  a.M = own(c.M);
  a.K = own(c.K);
  a.ntaps = own(c.ntaps);
  a.tapS = own(c.tapS);
  a.tapSinv = own(c.tapSinv);
  a.oy0 = own(c.oy0);
  a.ox0 = own(c.ox0);
  a.wr0 = own(c.wr0);
  a.ws0 = own(c.ws0);
  a.oyc = own(c.oyc);
  a.oxc = own(c.oxc);
  a.dHW = FastDiv{own(c.dHW.d), own(c.dHW.m), own(c.dHW.s)};
  a.dW = FastDiv{own(c.dW.d), own(c.dW.m), own(c.dW.s)};
  a.bn_part = own(c.bn_part);
  gemm16_body<MODE_DGRAD, BM, BN, WM, WN, 0, 1, F32, 0, 2, EPF>(a, t, 0);
}

}  // namespace tmrg
#include "gemm16_ws.h"
namespace tmrg {

template <int MODE, int BM, int BN, int WM, int WN, int F32, int PRO = 0>
int launch16_cfg(const GemmArgs& a, bool tapv, dim3 grid, hipStream_t st) {
  const dim3 blk(64 * WM * WN);
  // one-k-tile bf16 FWD launches on the 4-wave 128x128 / 256x64 tiles: the one-stage form
  // (bit-identical to the two-stage form, which it replaced in round 4).  56x56 64->64: 0.427 ->
  // 0.378 ms; the DGRAD view measured slower in it (its 233-VGPR LDS-staged epilogue caps the
  // occupancy at two workgroups anyway; profiles/r4/nst1/)
  // (fp32, round 5: the same forms for K <= 64 / 128 / 256, two to eight k-tiles serialised
  // through the one stage, measured no faster: C2 forward family 47.1 -> 46.9 / 47.2 / 47.7 ms,
  // profiles/r5/nst1_f32/; not taken)
  constexpr int kmax = 64;
  if constexpr (MODE == MODE_FWD && (PRO & 2) == 0 && F32 == 0 && WM * WN == 4 &&
                ((BM == 128 && BN == 128) || (BM == 256 && BN == 64))) {
    if (!tapv && a.K > 0 && a.K <= kmax) {
      hipLaunchKernelGGL((gemm16_kernel<MODE, BM, BN, WM, WN, 0, 1, F32, PRO, 1>), grid, blk, 0, st, a);
      TMR_CHECK_LAUNCH("gemm16_kernel (one stage)");
      return 0;
    }
  }
  // ... and the one-k-tile bf16 forwards the tile rules give 256x256 (N >= 256: the 64 -> 256
  // expansions): 256x128 as 8 waves in the one-stage form at 128 VGPRs -- two workgroups per CU
  // (one 16-wave 256x256 workgroup fills the register file), so one's epilogue stores overlap
  // the other's loads.  Same BM (the statistics' part rows), same per-wave tiles: bit-identical to
  // the 256x256 launch it replaced.
  if constexpr (MODE == MODE_FWD && (PRO & 2) == 0 && F32 == 0 && BM == 256 && BN == 256) {
    if (!tapv && a.K > 0 && a.K <= kmax) {
      const dim3 g2((unsigned)(cdiv(a.M, 256) * cdiv(a.N, 128)), grid.y, 1);
      hipLaunchKernelGGL((gemm16_kernel<MODE, 256, 128, 4, 2, 0, 1, F32, PRO, 1>), g2, dim3(512), 0, st, a);
      TMR_CHECK_LAUNCH("gemm16_kernel (one stage, 256x128)");
      return 0;
    }
  }
  // the fused BN-backward dgrads of the 4-wave tiles in their compile-time epilogue form
  // (EpiForm: bf16 step EPF 1, fp32 step EPF 2)
  constexpr bool FORMS = MODE == MODE_DGRAD && PRO == 0 && TMR_EPI_FORMS &&
                         (WM * WN == 4 || (WM * WN == 8 && TMR_EPI_LATE_F > 0));
  if constexpr (FORMS) {
    const int f = a.bn_part != nullptr ? epi_form(a) : 0;
    if (f == (F32 ? 2 : 1)) {
      if (tapv)
        hipLaunchKernelGGL((gemm16_kernel<MODE, BM, BN, WM, WN, 1, 1, F32, 0, 2, F32 ? 2 : 1>), grid, blk, 0, st, a);
      else
        hipLaunchKernelGGL((gemm16_kernel<MODE, BM, BN, WM, WN, 0, 1, F32, 0, 2, F32 ? 2 : 1>), grid, blk, 0, st, a);
      TMR_CHECK_LAUNCH("gemm16_kernel (dgrad epilogue form)");
      return 0;
    }
  }
  if constexpr (PRO != 0) {   // one tap per k-tile (pro32_ok)
    hipLaunchKernelGGL((gemm16_kernel<MODE, BM, BN, WM, WN, 0, 1, F32, PRO>), grid, blk, 0, st, a);
  } else if (tapv) {
    hipLaunchKernelGGL((gemm16_kernel<MODE, BM, BN, WM, WN, 1, 1, F32>), grid, blk, 0, st, a);
  } else {
    hipLaunchKernelGGL((gemm16_kernel<MODE, BM, BN, WM, WN, 0, 1, F32>), grid, blk, 0, st, a);
  }
  TMR_CHECK_LAUNCH(F32 ? "gemm16_kernel (fp32)" : "gemm16_kernel");
  return 0;
}

template <int MODE, int F32, int PRO>
int launch16_switch(const GemmArgs& a, int cfg, bool tapv, dim3 grid, hipStream_t st) {
  switch (cfg) {
    case 1: return launch16_cfg<MODE, 256, 128, 4, 2, F32, PRO>(a, tapv, grid, st);
    case 2: return launch16_cfg<MODE, 128, 128, 2, 2, F32, PRO>(a, tapv, grid, st);
    case 3: return launch16_cfg<MODE, 256, 64, 4, 1, F32, PRO>(a, tapv, grid, st);
    case 4: return launch16_cfg<MODE, 64, 256, 1, 4, F32, PRO>(a, tapv, grid, st);
    case 7: return launch16_cfg<MODE, 128, 128, 4, 2, F32, PRO>(a, tapv, grid, st);
    case 5: return launch16_cfg<MODE, 64, 64, 2, 2, F32, PRO>(a, tapv, grid, st);
    default: break;
  }
  if constexpr ((PRO & 2) == 0) {   // 256x256: no room for the dY prologue's LDS (pick_cfg16)
    if (cfg == 0) return launch16_cfg<MODE, 256, 256, 2, 4, F32, PRO>(a, tapv, grid, st);
    if (cfg == 6) return launch16_cfg<MODE, 256, 256, 4, 4, F32, PRO>(a, tapv, grid, st);
  }
  TMR_CHECK_ARG(false, "gemm16: no tile config %d for prologue %d", cfg, PRO);
  return 1;
}

// the launch's arguments against what the engine and tile config `cfg` support
template <int MODE, int F32>
int check16(const GemmArgs& a, int cfg) {
  TMR_CHECK_ARG(((uintptr_t)a.A & 15) == 0 && ((uintptr_t)a.B & 15) == 0,
                "gemm (LDS-DMA path): operands must be 16-B aligned");
  constexpr bool f32 = F32 != 0;
  TMR_CHECK_ARG((a.prec == TMR_MATH_F32) == f32, "gemm (LDS-DMA path): precision dispatch");
  TMR_CHECK_ARG(!f32 || (a.lds % 4 == 0 && a.log2C >= 2 &&
                         (MODE == MODE_DGRAD ? (a.ldbt % 4 == 0 && a.N % 8 == 0 && a.ldc % 4 == 0 &&
                                                ((uintptr_t)a.C & 15) == 0)
                                             : a.ldb % 4 == 0)),
                "gemm (fp32 LDS-DMA path): 4-channel pieces, 16-B row strides (view %d)", MODE);
  const Cfg16 c = kCfgs16[cfg];
  // the BN-partial rows of a fused dgrad were counted with the prologue-free tile rows
  TMR_CHECK_ARG(MODE != MODE_DGRAD || !a.bn_part || c.bm == kCfgs16[pick_cfg16(a.M, a.N, a.K, MODE, f32)].bm,
                "gemm (LDS-DMA path): the dY prologue changed a fused dgrad's tile rows");
  TMR_CHECK_ARG(!a.pro || (f32 ? pro32_ok(a, MODE) : pro16_ok(a, MODE)),
                "gemm (LDS-DMA path): operand prologue %d not supported here (view %d)", a.pro, MODE);
  // ReLU-mask bits are read by the LDS-staged BN-backward epilogue only (every dgrad tile but
  // 256x256, whose wave row-blocks do not fit the staging buffer)
  TMR_CHECK_ARG(a.bn_part == nullptr || a.bn_mask != 3 ||
                    (MODE == MODE_DGRAD && !(c.bm == 256 && c.bn == 256)),
                "gemm: ReLU-mask bits (mask 3) need the LDS-DMA dgrad's LDS-staged epilogue (tile %dx%d)",
                c.bm, c.bn);
  TMR_CHECK_ARG(!a.g16 || (MODE == MODE_DGRAD && a.bn_part != nullptr &&
                           !(c.bm == 256 && c.bn == 256) && ((uintptr_t)a.C & 15) == 0 &&
                           a.ldc % 8 == 0),
                "gemm: a bf16 BN-backward gradient (TMR_IO_G16) needs the fused LDS-staged dgrad "
                "epilogue, 16-B aligned rows (tile %dx%d)", c.bm, c.bn);
  TMR_CHECK_ARG((!a.Cold && !a.cold16) ||
                    (MODE == MODE_DGRAD && a.bn_part != nullptr && !(c.bm == 256 && c.bn == 256) &&
                     ((uintptr_t)(a.Cold ? a.Cold : a.C) & 15) == 0),
                "gemm: a separate / bf16 old dx needs the fused LDS-staged dgrad epilogue (tile %dx%d)",
                c.bm, c.bn);
  return 0;
}

template <int MODE, int F32>
int launch_gemm16_t(const GemmArgs& a, int splits, hipStream_t st) {
  constexpr bool f32 = F32 != 0;
  const int cfg = pick_cfg16(a.M, a.N, a.K, MODE, f32, a.pro);
  const Cfg16 c = kCfgs16[cfg];
  if (const int rc = check16<MODE, F32>(a, cfg)) return rc;
  dim3 grid(cdiv(a.M, c.bm) * cdiv(a.N, c.bn), splits, 1);
  if (grid.x == 0) return 0;
  // a k-tile (64 bf16 / 32 fp32) spans several taps when the channels per tap are fewer (or not
  // a multiple)
  const int bk = f32 ? 32 : 64;
  const bool tapv = MODE != MODE_WGRAD && a.ntaps > 1 && ((1 << a.log2C) % bk) != 0;
  if (MODE == MODE_WGRAD && (c.bm < 64 || c.bn < 64)) return -1;
  if constexpr (MODE == MODE_DGRAD) {   // the wave-specialised persistent form (gemm16_ws.h)
    const int rc = launch_dgrad_ws<F32>(a, cfg, st);
    if (rc >= 0) return rc;
  }
#if TMR_PROLOGUES
  // prologue variants (A/B build; fp32 and bf16): FWD X, DGRAD dY, WGRAD dY / dY + X / X
  if (a.pro) {
    if constexpr (MODE == MODE_FWD) return launch16_switch<MODE, F32, 1>(a, cfg, tapv, grid, st);
    if constexpr (MODE == MODE_DGRAD) return launch16_switch<MODE, F32, 2>(a, cfg, tapv, grid, st);
    if constexpr (MODE == MODE_WGRAD) {
      if (a.pro == 2) return launch16_switch<MODE, F32, 2>(a, cfg, tapv, grid, st);
      if (a.pro == 3) return launch16_switch<MODE, F32, 3>(a, cfg, tapv, grid, st);
      return launch16_switch<MODE, F32, 1>(a, cfg, tapv, grid, st);
    }
  }
#endif
  return launch16_switch<MODE, F32, 0>(a, cfg, tapv, grid, st);
}

template <int MODE, int F32>
int launch_gemm16(const GemmArgs& a, int splits, hipStream_t st) {
  return launch_gemm16_t<MODE, F32>(a, splits, st);
}

// The stride-parity classes of one strided dgrad in one launch (gemm16_par_kernel): every class
// on the tile config its own launch would use, one tap per k-tile (no TAPV form), no operand
// prologue.  Returns -1 (nothing launched) when the classes do not qualify: the caller launches
// them one by one.  Each tile computes exactly what its class's own launch computes.
template <int F32>
int launch_gemm16_par(const GemmArgs* as, int n, hipStream_t st) {
  constexpr bool f32 = F32 != 0;
  static_assert(sizeof(GemmPar) <= 4096, "kernel argument size");
  if (n < 2 || n > PAR_MAX) return -1;
  const int cfg = pick_cfg16(as[0].M, as[0].N, as[0].K, MODE_DGRAD, f32, as[0].pro);
  const int bk = f32 ? 32 : 64;
  for (int i = 0; i < n; ++i) {
    const GemmArgs& a = as[i];
    if (a.pro || (a.prec == TMR_MATH_F32) != f32 || !use16(a, MODE_DGRAD)) return -1;
    if (pick_cfg16(a.M, a.N, a.K, MODE_DGRAD, f32, 0) != cfg) return -1;
    if (a.ntaps > 1 && ((1 << a.log2C) % bk) != 0) return -1;   // the TAPV form
  }
  switch (cfg) {
    case 1: case 2: case 3: case 5: case 7: break;
    default: return -1;
  }
  GemmPar p{};
  p.n = n;

  const Cfg16 c = kCfgs16[cfg];
  // the class's own fields (ParClass); every other argument must be the first class's
  auto own = [](const GemmArgs& a, int tiles) {
    return ParClass{a.M, a.K, a.ntaps, a.tapS, a.tapSinv, a.oy0, a.ox0, a.wr0, a.ws0, a.oyc, a.oxc,
                    tiles, a.dHW, a.dW, a.bn_part};
  };
  auto put = [](GemmArgs& a, const ParClass& q) {
    a.M = q.M; a.K = q.K; a.ntaps = q.ntaps; a.tapS = q.tapS; a.tapSinv = q.tapSinv;
    a.oy0 = q.oy0; a.ox0 = q.ox0; a.wr0 = q.wr0; a.ws0 = q.ws0; a.oyc = q.oyc; a.oxc = q.oxc;
    a.dHW = q.dHW; a.dW = q.dW; a.bn_part = q.bn_part;
  };
  // classes by tile count, largest first (par_tile's round-robin)
  int ord[PAR_MAX];
  for (int i = 0; i < n; ++i) ord[i] = i;
  auto tiles = [&](const GemmArgs& a) { return (int)(cdiv(a.M, c.bm) * cdiv(a.N, c.bn)); };
  for (int i = 1; i < n; ++i)
    for (int j = i; j > 0 && tiles(as[ord[j]]) > tiles(as[ord[j - 1]]); --j) std::swap(ord[j], ord[j - 1]);
  p.a = as[ord[0]];
  long total = 0;
  for (int i = 0; i < n; ++i) {
    const GemmArgs& a = as[ord[i]];
    if (const int rc = check16<MODE_DGRAD, F32>(a, cfg)) return rc;
    p.c[i] = own(a, tiles(a));
    GemmArgs b = p.a;
    put(b, p.c[i]);
    if (std::memcmp(&b, &a, sizeof(GemmArgs)) != 0) return -1;   // differs elsewhere: not a class
    total += (long)(p.c[i].tiles + PAR_G - 1) / PAR_G * PAR_G;   // whole chunks (par_tile)
  }
  if (total == 0) return 0;
  TMR_CHECK_ARG(total < (1L << 31), "gemm (parity classes): %ld tiles", total);
  const dim3 grid((unsigned)total, 1, 1);
  // the 4-wave tiles' fused BN-backward dgrads in their compile-time epilogue form (EpiForm)
  constexpr int EF = F32 ? 2 : 1;
  const bool form = TMR_EPI_FORMS && p.a.bn_part != nullptr && epi_form(p.a) == EF;
  switch (cfg) {
    case 1: hipLaunchKernelGGL((gemm16_par_kernel<256, 128, 4, 2, F32>), grid, dim3(512), 0, st, p); break;
    case 2:
      if (form) hipLaunchKernelGGL((gemm16_par_kernel<128, 128, 2, 2, F32, EF>), grid, dim3(256), 0, st, p);
      else hipLaunchKernelGGL((gemm16_par_kernel<128, 128, 2, 2, F32>), grid, dim3(256), 0, st, p);
      break;
    case 3:
      if (form) hipLaunchKernelGGL((gemm16_par_kernel<256, 64, 4, 1, F32, EF>), grid, dim3(256), 0, st, p);
      else hipLaunchKernelGGL((gemm16_par_kernel<256, 64, 4, 1, F32>), grid, dim3(256), 0, st, p);
      break;
    case 5:
      if (form) hipLaunchKernelGGL((gemm16_par_kernel<64, 64, 2, 2, F32, EF>), grid, dim3(256), 0, st, p);
      else hipLaunchKernelGGL((gemm16_par_kernel<64, 64, 2, 2, F32>), grid, dim3(256), 0, st, p);
      break;
    case 7: hipLaunchKernelGGL((gemm16_par_kernel<128, 128, 4, 2, F32>), grid, dim3(512), 0, st, p); break;
  }
  TMR_CHECK_LAUNCH("gemm16_par_kernel");
  return 0;
}

}  // namespace tmrg

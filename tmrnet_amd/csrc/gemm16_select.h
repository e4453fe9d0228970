// Host-side launch selection of the LDS-DMA implicit-GEMM engine (gemm16_kernel.h): eligibility
// per view, tile rules, and the per-(view, precision) launchers instantiated in
// gemm16_<view>_<prec>.hip.  The register-staged translation units include only this header, so
// an edit of the engine rebuilds the six small engine units and nothing else.
#pragma once
#include "gemm_kernel.h"

namespace tmrg {

// ---------------------------------------------------------------- launch selection
struct Cfg16 { int bm, bn; };
constexpr Cfg16 kCfgs16[] = {{256, 256}, {256, 128}, {128, 128}, {256, 64}, {64, 256}, {64, 64},
                              {256, 256},    // 6: 256x256 as 16 waves (4x4, 64x64 per wave)
                              {128, 128}};   // 7: 128x128 as 8 waves (4x2, 32x64 per wave)

// Eligibility: bf16 math, every operand bf16 in HBM (sab 3; DGRAD with the transposed weights),
// no operand prologue, 16-B pieces of 8 channels (channels per tap, row strides multiples of 8).
// fp32 form (GemmArgs::dma32, set by the conv entry points): FWD with every operand fp32 and
// 16-B aligned, 4-channel pieces; DGRAD whenever the weights come transposed (wt: the engine is
// the only reader of that layout, so eligibility is checked again by launch_gemm16_t).
// Operand prologues on the fp32 engine (GemmArgs::pro; gemm16_kernel PRO): the per-channel
// coefficient tables are staged in LDS, so their channel counts are bounded
constexpr int PRO_XMAX = 512;    // X-operand channels (the inputs of conv2 / conv3: planes <= 512)
constexpr int PRO_DMAX = 2048;   // dY-operand channels (conv outputs <= 2048)
inline bool pro32_ok(const GemmArgs& a, int mode) {
  if (!a.pro) return true;
  // one tap per 32-float k-tile (the transform takes the piece's channel from the tile's tap)
  if (mode != MODE_WGRAD && a.ntaps != 1 && a.log2C < 5) return false;
  if ((a.pro & 1) && (mode == MODE_DGRAD || a.lds > PRO_XMAX || a.lds % 4)) return false;
  if (a.pro & 2) {
    if (mode == MODE_FWD || ((uintptr_t)a.pd_y & 15)) return false;
    const int cd = mode == MODE_WGRAD ? a.ldb : a.lds;
    if (cd > PRO_DMAX || cd % 4) return false;
  }
  return true;
}

inline bool use32(const GemmArgs& a, int mode) {
#if TMR_PROLOGUES
  // the A/B build only (make PROLOGUES=1): TMR_GEMM32=0 keeps the fp32 forward / wgrad views on the
  // register-staged engine, whose prologue form the fold test compares with this engine's
  const bool on = env_int("TMR_GEMM32", 1) != 0;
#else
  const bool on = true;
#endif
  if (a.prec != TMR_MATH_F32 || a.sab) return false;
  if (!pro32_ok(a, mode)) return false;
  if (mode == MODE_DGRAD) return a.wt != 0;
  if (!on || !a.dma32) return false;
  if ((((uintptr_t)a.A | (uintptr_t)a.B) & 15) != 0) return false;
  if (mode == MODE_WGRAD)
    return a.M % 4 == 0 && a.log2C >= 2 && a.ldb % 4 == 0 && a.lds % 4 == 0 && a.N % 4 == 0;
  return a.lds % 4 == 0 && a.ldb % 4 == 0 && a.log2C >= 2 && (a.ntaps != 1 || a.K % 4 == 0);
}

// bf16 form (A/B build, round 5): the X prologue (relu(bn) of the operand, rounded to bf16 as the
// BN pass would store it) and the dY prologue (the BN backward of bf16 g and y, rounded as
// bn_bwd_apply8_a16 stores dy), one tap per 64-element k-tile, 8-channel pieces
inline bool pro16_ok(const GemmArgs& a, int mode) {
  if (!a.pro) return true;
  if (mode != MODE_WGRAD && a.ntaps != 1 && a.log2C < 6) return false;
  if ((a.pro & 1) && (mode == MODE_DGRAD || a.lds > PRO_XMAX || a.lds % 8)) return false;
  if (a.pro & 2) {
    if (mode == MODE_FWD || ((uintptr_t)a.pd_y & 15)) return false;
    const int cd = mode == MODE_WGRAD ? a.ldb : a.lds;
    if (cd > PRO_DMAX || cd % 8) return false;
  }
  return true;
}

inline bool use16(const GemmArgs& a, int mode) {
  if (a.prec == TMR_MATH_F32) return use32(a, mode);
  if (a.prec != TMR_MATH_BF16 || a.sab != 3 || !pro16_ok(a, mode)) return false;
  if (mode == MODE_DGRAD && !a.wt) return false;
  if (a.lds % 8) return false;
  if (mode == MODE_WGRAD) return a.M % 8 == 0 && a.log2C >= 3 && a.ldb % 8 == 0 && a.N % 8 == 0;
  if (mode == MODE_FWD && a.ldb % 8) return false;
  if (mode == MODE_DGRAD && a.ldbt % 8) return false;
  return a.ntaps == 1 ? (a.K % 8 == 0 && (mode == MODE_FWD || a.log2C >= 3)) : a.log2C >= 3;
}

inline long cfg16_tiles(long M, long N, int c) {
  return ((M + kCfgs16[c].bm - 1) / kCfgs16[c].bm) * ((N + kCfgs16[c].bn - 1) / kCfgs16[c].bn);
}

// Tile choice per view, from scripts/convbench.py --io16 --stats --bnbwd with each config forced
// over the 23 ResNet-50 conv shapes x 3 views (profiles/r2/convbench16_cfgs/, cb16c/): 256x256
// pays for the forwards and the wgrads with 256-512 output channels, as 16 waves (four per SIMD:
// 5-20% over 8 waves, whose two waves per SIMD stall on the same barrier); the dgrads, whose
// fused BatchNorm-backward epilogue moves 12-16 B per output element, want the occupancy of
// 128x128 / 256x64 tiles.
// fp32 (f32): measured separately (profiles/r2/convbench32_dma_cfgs/, wgrad32_cfgs/): the
// wgrads with 64 output channels want 64-wide tiles, the big-FLOP wgrads (>= 100 GFLOP: 3x3,
// strided downsample) 256x256 as 16 waves, the rest 128x128 as 8 waves; the N = 128 forwards and
// the >= 512-column dgrads 128x128 as 8 waves.
inline int pick_cfg16_base(long M, long N, long K, int mode, bool f32);
// pro: the launch's operand prologues -- a dY prologue (bit 2) stages y and 24 KB of coefficients
// in LDS besides the two k-tile stages, which a 256x256 tile (128 KB of stages) cannot fit: its
// 8-wave 128x128 form instead
inline int pick_cfg16(long M, long N, long K, int mode, bool f32 = false, int pro = 0) {
  const int cfg = pick_cfg16_base(M, N, K, mode, f32);
  if ((pro & 2) && kCfgs16[cfg].bm == 256 && kCfgs16[cfg].bn == 256) return 7;
  return cfg;
}
inline int pick_cfg16_base(long M, long N, long K, int mode, bool f32) {
  static const int forced = env_int("TMR_GEMM16_CFG", -1);   // experiments only
  if (forced >= 0 && forced < (int)(sizeof(kCfgs16) / sizeof(kCfgs16[0]))) return forced;
  int cfg;
  if (f32 && mode == MODE_WGRAD) {
    if (M <= 64) return (N <= 64 || N >= 512) ? 5 : 4;
    if (N <= 64) return 5;
    if (M >= 256 && N >= 256 && 2.0 * M * N * K >= 100e9) return 6;
    return 7;
  }
  if (f32 && M >= 256 && mode == MODE_DGRAD && N >= 512) {
    static const int wide = env_int("TMR_DGRAD32_WIDE_CFG", 7);   // A/B of this rule
    return cfg16_tiles(M, N, wide) >= 256 ? wide : 2;
  }
  if (f32 && M >= 256 && mode == MODE_FWD && N == 128)
    return cfg16_tiles(M, N, 7) >= 256 ? 7 : 2;
  if (mode == MODE_WGRAD) {
    if (M <= 64) cfg = N <= 64 ? 5 : (N >= 512 ? 4 : 2);
    else if (N <= 64) cfg = 3;
    // round 5 (profiles/r5/tile_rules/): 128x128 as 8 waves, or 256x256 as 16 waves for the wide
    // wgrads (N >= 1024: 3x3, 1024-channel inputs) while each of the ~512 / tiles split-K slices
    // still reduces >= 4096 rows; shorter slices (layer3/4 spatial at 640 frames, the grouped
    // split-attention convs one group at a time) spend the 256x256 tile's time on its prologue and
    // its 256 KB slab.  Replaced the round-2 rule (128x128 4-wave / 256x256 by M and K): C5 wgrads
    // -1.1 ms, C4 -0.4 ms per step.
    else cfg = (M >= 256 && N >= 1024 && K * cfg16_tiles(M, N, 6) >= (1L << 21)) ? 6 : 7;
  } else if (N <= 64) {
    cfg = M >= 256 ? 3 : 5;
  } else if (mode == MODE_FWD && N >= 256 && M >= 256) {
    cfg = 6;   // 256x256 as 16 waves: four waves per SIMD hide the barrier / load waits
  } else {
    cfg = 2;
  }
  // too few tiles to fill the 256 CUs: smaller tiles -- except the fp32 256x256 forwards at >= 224
  // tiles (layer4 at 640 frames: 246), which measured 4-6% faster than 492 256x128 tiles (round 5)
  if (mode != MODE_WGRAD && cfg16_tiles(M, N, cfg) < (f32 && cfg == 6 ? 224 : 256)) {
    for (const int c2 : {1, 2, 5}) {
      if ((long)kCfgs16[c2].bm * kCfgs16[c2].bn >= (long)kCfgs16[cfg].bm * kCfgs16[cfg].bn ||
          cfg16_tiles(M, N, c2) <= cfg16_tiles(M, N, cfg))
        continue;
      cfg = c2;
      if (cfg16_tiles(M, N, cfg) >= 256) break;
    }
  }
  return cfg;
}

// rows / columns of the output tile the launch for `a` will use (host planning: BN-partial rows,
// wgrad split counts)
inline int gemm_tile_bm(const GemmArgs& a, int mode) {
  return use16(a, mode) ? kCfgs16[pick_cfg16(a.M, a.N, a.K, mode, a.prec == TMR_MATH_F32, a.pro)].bm
                        : kCfgs[pick_cfg(a.M, a.N, a.K, mode)].bm;
}
inline long gemm_tiles(const GemmArgs& a, int mode) {
  return use16(a, mode) ? cfg16_tiles(a.M, a.N, pick_cfg16(a.M, a.N, a.K, mode, a.prec == TMR_MATH_F32, a.pro))
                        : cfg_tiles(a.M, a.N, pick_cfg(a.M, a.N, a.K, mode));
}

// the stride-parity classes of one strided dgrad as one launch (launch_gemm16_par): the
// arguments every class shares once, the few that differ per class in a table
constexpr int PAR_MAX = 4;
struct ParClass {
  int M, K, ntaps, tapS, tapSinv, oy0, ox0, wr0, ws0, oyc, oxc, tiles;
  FastDiv dHW, dW;
  float2* bn_part;
};
struct GemmPar {
  GemmArgs a;               // the first class's arguments
  ParClass c[PAR_MAX];      // by tile count, largest first
  int n;
};
// tiles of one class in a row (par_tile): a round of one XCD's workgroup slots (32 CUs x 2)
constexpr int PAR_G = 64;

// wave-specialised dgrad launches so far (gemm16_ws.h; tmr_dgrad_ws_launches)
extern long g_dgrad_ws_launches;

// one view x precision per translation unit (gemm16_<view>_<prec>.hip, explicit instantiations:
// they compile in parallel)
template <int F32>
int launch_gemm16_par(const GemmArgs* as, int n, hipStream_t st);
extern template int launch_gemm16_par<0>(const GemmArgs*, int, hipStream_t);
extern template int launch_gemm16_par<1>(const GemmArgs*, int, hipStream_t);
template <int MODE, int F32>
int launch_gemm16(const GemmArgs& a, int splits, hipStream_t st);
extern template int launch_gemm16<MODE_FWD, 0>(const GemmArgs&, int, hipStream_t);
extern template int launch_gemm16<MODE_FWD, 1>(const GemmArgs&, int, hipStream_t);
extern template int launch_gemm16<MODE_DGRAD, 0>(const GemmArgs&, int, hipStream_t);
extern template int launch_gemm16<MODE_DGRAD, 1>(const GemmArgs&, int, hipStream_t);
extern template int launch_gemm16<MODE_WGRAD, 0>(const GemmArgs&, int, hipStream_t);
extern template int launch_gemm16<MODE_WGRAD, 1>(const GemmArgs&, int, hipStream_t);

}  // namespace tmrg

// Implicit-GEMM convolution / GEMM engine: host side and C ABI (kernel template: gemm_kernel.h).
#include "gemm16_select.h"

#include <type_traits>

using namespace tmrg;

// the prologue forms behind the plain entry points (pro = nullptr); exported as the
// include/tmr_prologue.h entry points in the A/B build only (TMR_PROLOGUES, end of file)
static int conv_fwd_bnstats_pro(const tmr_conv_desc* d, const float* x, const float* w_krsc,
                                float* y, void* stats, size_t stats_bytes,
                                const tmr_conv_prologue* pro, hipStream_t stream);
static int conv_dgrad_pro(const tmr_conv_desc* d, const float* dy, const float* w_krsc, float* dx,
                          float beta, const tmr_conv_prologue* pro, hipStream_t stream);
static int conv_dgrad_bnbwd_pro(const tmr_conv_desc* d, const float* dy, const float* w_krsc,
                                float* dx, float beta, const float* y, const float* z,
                                const float* scale, const float* shift, const float* mean,
                                int mask, void* parts, size_t parts_bytes,
                                const tmr_conv_prologue* pro, hipStream_t stream);
static int conv_wgrad_pro(const tmr_conv_desc* d, const float* x, const float* dy,
                          float* dw_oihw, int c_real, float beta, float* ws, size_t ws_bytes,
                          const tmr_conv_prologue* pro, hipStream_t stream);

namespace {

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

template <int MODE>
int launch_gemm(const GemmArgs& a, bool al, int splits, hipStream_t st) {
  if (MODE == MODE_FWD) return launch_gemm_fwd(a, al, splits, st);
  if (MODE == MODE_DGRAD) return launch_gemm_dgrad(a, al, splits, st);
  return launch_gemm_wgrad(a, al, splits, st);
}

static inline int xld_of(const tmr_conv_desc* d) { return d->x_ld ? d->x_ld : d->c; }
static inline int yld_of(const tmr_conv_desc* d) { return d->y_ld ? d->y_ld : d->k; }
static inline long span(long pixels, int ld, int width) { return pixels > 0 ? (pixels - 1) * ld + width : 0; }

// element bytes of the conv operands (tmr_conv_desc.io: bf16-stored x / w / dy)
static inline int esz_x(const tmr_conv_desc* d) { return (d->io & TMR_IO_X_BF16) ? 2 : 4; }
static inline int esz_w(const tmr_conv_desc* d) { return (d->io & (TMR_IO_W_BF16 | TMR_IO_WT_BF16)) ? 2 : 4; }
static inline int esz_dy(const tmr_conv_desc* d) { return (d->io & TMR_IO_DY_BF16) ? 2 : 4; }
static inline int esz_y(const tmr_conv_desc* d) { return (d->io & TMR_IO_Y_BF16) ? 2 : 4; }
static inline int esz_bn(const tmr_conv_desc* d) { return (d->io & TMR_IO_BN_BF16) ? 2 : 4; }
static inline int esz_dx(const tmr_conv_desc* d) { return (d->io & TMR_IO_G16) ? 2 : 4; }
template <typename T>
static inline T* adv(T* p, long elems, int esz) {   // p + elems elements of esz bytes
  return p ? (T*)((typename std::conditional<std::is_const<T>::value, const char*, char*>::type)p +
                  elems * esz)
           : p;
}
static uint32_t clamp_bytes_e(long elems, int esz) {
  long b = elems * esz;
  return b >= 0x80000000L ? 0x80000000u : (uint32_t)b;
}

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

// Operand prologues of one launch (tmr_conv_prologue; GemmArgs::pro).  X: the gathered input
// operand of FWD / WGRAD; dY: the output-gradient operand of DGRAD / WGRAD, with its y at the
// launch's frame offset y_off.  Dense layouts only (the offsets of y are dY's).
int set_prologue(GemmArgs& a, const tmr_conv_prologue* pro, const tmr_conv_desc* d, bool x_ok,
                 bool dy_ok, long y_off) {
  if (!pro) return 0;
#if !TMR_PROLOGUES
  TMR_CHECK_ARG(false, "tmr_conv2d: operand prologues exist in the A/B build only (TMR_PROLOGUES)");
#endif
  if (pro->x_scale || pro->x_shift) {
    TMR_CHECK_ARG(x_ok, "tmr_conv2d: an X-operand prologue applies to the forward and wgrad views");
    TMR_CHECK_ARG(pro->x_scale && pro->x_shift, "tmr_conv2d: X prologue needs scale and shift");
    TMR_CHECK_ARG(!d->x_ld || d->x_ld == d->c, "tmr_conv2d: X prologue needs a dense x (x_ld == c)");
    a.px_scale = pro->x_scale;
    a.px_shift = pro->x_shift;
    a.pro |= 1;
  }
  if (pro->dy_y || pro->dy_coef) {
    TMR_CHECK_ARG(dy_ok, "tmr_conv2d: a dY-operand prologue applies to the dgrad and wgrad views");
    TMR_CHECK_ARG(pro->dy_y && pro->dy_coef, "tmr_conv2d: dY prologue needs y and coefficients");
    TMR_CHECK_ARG(!d->y_ld || d->y_ld == d->k, "tmr_conv2d: dY prologue needs a dense dy (y_ld == k)");
    a.pd_y = adv(pro->dy_y, y_off, esz_dy(d));   // y has dY's element type
    a.pd_a = pro->dy_coef;
    a.pd_b = pro->dy_coef + d->k;
    a.pd_c = pro->dy_coef + 2 * d->k;
    a.pro |= 2;
  }
  return 0;
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
static int conv_fwd_args(const tmr_conv_desc* d, const float* x, const float* w_krsc,
                         const float* bias, float* y, float beta, GemmArgs& a, bool& al) {
  TMR_CHECK_ARG(d, "tmr_conv2d_fwd: null descriptor");
  TMR_CHECK_ARG(d->math == TMR_MATH_F32 || d->math == TMR_MATH_BF16, "tmr_conv2d: bad math mode %d", d->math);
  TMR_CHECK_ARG((d->io & ~(TMR_IO_ENGINE | TMR_IO_CLASSES | TMR_IO_TILES)) == 0 || d->math == TMR_MATH_BF16, "tmr_conv2d: bf16-stored operands (io %d) need TMR_MATH_BF16", d->io);
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
  a.Abytes = clamp_bytes_e(span((long)d->n * d->h * d->w, a.lds, d->c), esz_x(d));
  a.prec = d->math;
  a.Bbytes = clamp_bytes_e((long)d->k * a.K, esz_w(d));
  a.sab = ((d->io & TMR_IO_X_BF16) ? 1 : 0) | ((d->io & TMR_IO_W_BF16) ? 2 : 0);
  a.Cbytes = clamp_bytes(span((long)d->n * d->ho * d->wo, a.ldc, d->k));
  // (2: the whole-line store form of epilogue_batched, where the tile allows it)
  a.c16 = (d->io & TMR_IO_Y_BF16) ? 2 : 0;
  a.dma32 = d->math == TMR_MATH_F32;
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
  GemmArgs a;
  bool al;
  if (conv_fwd_args(d, nullptr, nullptr, nullptr, nullptr, 0.f, a, al)) return 0;
  return cdiv(a.M, gemm_tile_bm(a, MODE_FWD));
}

static long x_frame(const tmr_conv_desc* d) { return (long)d->h * d->w * xld_of(d); }
static long y_frame(const tmr_conv_desc* d) { return (long)d->ho * d->wo * yld_of(d); }

// Grouped convolutions (tmr_conv_desc.groups = G > 1): group g reads input channels
// [g*c/G, (g+1)*c/G) and writes output channels [g*k/G, (g+1)*k/G); each group is one launch on
// channel slices (pixel strides = the whole tensors').  Weights per group are consecutive blocks
// of (k/G)*(c/G)*r*s elements: KRSC (k, r, s, c/G), the transposed copy (G, c/G, r, s, k/G), and
// OIHW gradients (k, c/G, r, s), i.e. torch's grouped Conv2d weight layout.
static int ngroups(const tmr_conv_desc* d) { return d->groups > 1 ? d->groups : 1; }
static int group_split(const tmr_conv_desc* d, tmr_conv_desc& g) {
  const int G = ngroups(d);
  TMR_CHECK_ARG(d->c % G == 0 && d->k % G == 0, "tmr_conv2d: channels %d / %d not divisible by %d groups",
                d->c, d->k, G);
  g = *d;
  g.x_ld = xld_of(d);
  g.y_ld = yld_of(d);
  g.c = d->c / G;
  g.k = d->k / G;
  g.groups = 0;
  return 0;
}
static long group_wsize(const tmr_conv_desc* g) { return (long)g->k * g->r * g->s * g->c; }

TMR_API int tmr_conv2d_fwd(const tmr_conv_desc* d, const float* x, const float* w_krsc,
                           const float* bias, float* y, float beta, hipStream_t stream) {
  TMR_CHECK_ARG(d, "tmr_conv2d_fwd: null descriptor");
  if (ngroups(d) > 1) {
    tmr_conv_desc g;
    if (group_split(d, g)) return 1;
    for (int i = 0; i < d->groups; ++i) {
      const int rc = tmr_conv2d_fwd(&g, adv(x, (long)i * g.c, esz_x(d)), adv(w_krsc, i * group_wsize(&g), esz_w(d)),
                                    bias ? bias + (long)i * g.k : nullptr,
                                    adv(y, (long)i * g.k, esz_y(d)), beta, stream);
      if (rc) return rc;
    }
    return 0;
  }
  const int fc = frames_per_launch(d);
  for (int f0 = 0; f0 < d->n; f0 += fc) {
    const tmr_conv_desc c = chunk_desc(d, d->n - f0 < fc ? d->n - f0 : fc);
    GemmArgs a;
    bool al;
    int rc = conv_fwd_args(&c, adv(x, f0 * x_frame(d), esz_x(d)), w_krsc, bias, adv(y, f0 * y_frame(d), esz_y(d)), beta, a, al);
    if (!rc && a.c16 && (beta != 0.f || bias)) {
      tmr_set_error("tmr_conv2d_fwd: a bf16 output (TMR_IO_Y_BF16) takes no beta / bias");
      rc = 1;
    }
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
  if (ngroups(d) > 1) {
    tmr_conv_desc g;
    if (group_split(d, g)) return 1;
    for (int i = 0; i < d->groups; ++i) {
      const long o = (long)i * g.k;
      const int rc = tmr_conv2d_fwd_fused(&g, adv(x, (long)i * g.c, esz_x(d)),
                                          adv(w_krsc, i * group_wsize(&g), esz_w(d)), scale + o,
                                          shift + o, residual ? residual + o : nullptr, y + o, relu,
                                          stream);
      if (rc) return rc;
    }
    return 0;
  }
  const int fc = frames_per_launch(d);
  for (int f0 = 0; f0 < d->n; f0 += fc) {
    const tmr_conv_desc c = chunk_desc(d, d->n - f0 < fc ? d->n - f0 : fc);
    GemmArgs a;
    bool al;
    int rc = conv_fwd_args(&c, adv(x, f0 * x_frame(d), esz_x(d)), w_krsc, shift, y + f0 * y_frame(d), 0.f, a, al);
    if (rc) return rc;
    TMR_CHECK_ARG(!a.c16, "tmr_conv2d_fwd_fused: the inference epilogue writes fp32 (no TMR_IO_Y_BF16)");
    a.scale = scale;
    a.res = residual ? residual + f0 * y_frame(d) : nullptr;
    a.relu = relu;
    rc = launch_gemm<MODE_FWD>(a, al, 1, stream);
    if (rc) return rc;
  }
  return 0;
}

// The fp32 7x7/2 stem with BatchNorm statistics runs as a direct convolution over its 147 real
// (tap, channel) pairs (stem.hip): a partial row per output row and wave; its weight gradient too
// (partial slabs per workgroup, reduced by wgrad_reduce_taps_kernel).  TMR_IO_ENGINE: the
// implicit-GEMM engine (tests).
int tmr_stem_stats_parts(int n, int ho);
int tmr_stem_fwd_bnstats(int n, int h, int w, int ho, const float* x, const float* w_krsc,
                         float* y, void* stats, hipStream_t stream);
int tmr_stem_wgrad_slabs(int n, int h, int w, int ho, const float* x, const float* dy, float* ws,
                         size_t ws_bytes, int* nslabs, hipStream_t stream);
constexpr long kStemSlabs = 512, kStemSlab = 64 * 49 * 4;   // stem.hip's grid and slab
constexpr long kStem16Slabs = 768;                            // stem16.hip's grid
static bool stem_geometry(const tmr_conv_desc* d) {
  return d->math == TMR_MATH_F32 && d->io == 0 &&
         ngroups(d) == 1 && d->c == 4 && d->k == 64 && d->r == 7 && d->s == 7 && d->stride == 2 &&
         d->pad == 3 && d->pad_w == 3 && d->wo == 112 && d->w <= 226 && xld_of(d) == 4 &&
         yld_of(d) == 64;
}
static bool stem_direct(const tmr_conv_desc* d) {
  return !(d->io & TMR_IO_ENGINE) && stem_geometry(d);
}
// the bf16-activation step's stem (stem16.hip): bf16 math on the NHWC4 fp32 input, bf16 KRSC
// weights (4 or 8 channels per tap), y bf16 with the statistics of the rounded values
int tmr_stem16_stats_parts(int n, int ho);
int tmr_stem16_fwd_bnstats(int n, int h, int w, int ho, const float* x, const void* w_krsc, int cp,
                           void* y, void* stats, hipStream_t stream);
static bool stem16_geometry(const tmr_conv_desc* d) {
  return d->math == TMR_MATH_BF16 && d->io == (TMR_IO_W_BF16 | TMR_IO_Y_BF16) &&
         ngroups(d) == 1 && d->c == 4 && d->k == 64 && d->r == 7 && d->s == 7 && d->stride == 2 &&
         d->pad == 3 && d->pad_w == 3 && d->wo == 112 && d->w <= 224 && xld_of(d) == 4 &&
         yld_of(d) == 64 && (d->h + 6 - 7) / 2 + 1 == d->ho;
}
static bool stem16_direct(const tmr_conv_desc* d) {
  return !(d->io & TMR_IO_ENGINE) && stem16_geometry(d);
}
// its weight gradient (bf16 dy, the NHWC4 fp32 input)
int tmr_stem16_wgrad_slabs(int n, int h, int w, int ho, const float* x, const void* dy, int dy32,
                           float* ws, size_t ws_bytes, int* nslabs, hipStream_t stream);
// (dy bf16 or fp32: both storages of the bf16-math step take this kernel, so they stay
// bit-identical)
static bool stem16_wgrad_geometry(const tmr_conv_desc* d) {
  return d->math == TMR_MATH_BF16 && (d->io == TMR_IO_DY_BF16 || d->io == 0) && ngroups(d) == 1 &&
         d->c == 4 &&
         d->k == 64 && d->r == 7 && d->s == 7 && d->stride == 2 && d->pad == 3 && d->pad_w == 3 &&
         d->wo == 112 && d->w <= 224 && xld_of(d) == 4 && yld_of(d) == 64 &&
         (d->h + 6 - 7) / 2 + 1 == d->ho;
}

// the narrow stride-1 3x3 convs of the bf16-activation step (ResNeSt-50's deep stem: 32 -> 32,
// 32 -> 64 at 112x112) as direct convolutions over an LDS ring of input rows (direct3.hip); every
// operand bf16 in HBM, dense NHWC.  TMR_IO_ENGINE: the implicit-GEMM engine (tests).
int tmr_d3_stats_parts(int n, int h, int w, int cin, int cout);
int tmr_d3_dgrad_parts(int n, int h, int w, int cin_conv, int cout_conv);
size_t tmr_d3_wgrad_ws_bytes(int n, int h, int w, int cin, int cout);
int tmr_d3_fwd_bnstats(int n, int h, int w, int cin, int cout, const void* x, const void* w_krsc,
                       void* y, void* stats, hipStream_t stream);
int tmr_d3_dgrad_bnbwd(int n, int h, int w, int cin_conv, int cout_conv, const void* dy,
                       const void* w_crsk, void* dx, int g16, float beta, const void* y,
                       const void* z, const float* scale, const float* shift, const float* mean,
                       int mask, void* parts, hipStream_t stream);
int tmr_d3_wgrad_slabs(int n, int h, int w, int cin, int cout, const void* x, const void* dy,
                       float* ws, size_t ws_bytes, int* nslabs, hipStream_t stream);
// (round 4, C5: ResNet-50 layer1's 64 -> 64 3x3 convs at 56x56 too)
static bool d3_shape(const tmr_conv_desc* d) {
  const bool wc = (d->w == 112 && d->c == 32 && (d->k == 32 || d->k == 64)) ||
                  (d->w == 56 && d->c == 64 && d->k == 64);
  return !(d->io & TMR_IO_ENGINE) && d->math == TMR_MATH_BF16 && ngroups(d) == 1 &&
         d->r == 3 && d->s == 3 && d->stride == 1 && d->pad == 1 && d->pad_w == 1 && wc &&
         d->wo == d->w && d->ho == d->h && xld_of(d) == d->c && yld_of(d) == d->k &&
         d->max_frames == 0;
}
// ... and the deep stem's first conv, 3x3/2 3 -> 32, on the NHWC4 fp32 input (bf16 math)
int tmr_d3s_stats_parts(int n, int ho);
int tmr_d3s_fwd_bnstats(int n, int h, const float* x, const void* w_krsc, void* y, void* stats,
                        hipStream_t stream);
size_t tmr_d3s_wgrad_ws_bytes(int n, int ho);
int tmr_d3s_wgrad_slabs(int n, int h, const float* x, const void* dy, float* ws, size_t ws_bytes,
                        int* nslabs, hipStream_t stream);
static bool d3s_shape(const tmr_conv_desc* d) {
  return !(d->io & TMR_IO_ENGINE) && d->math == TMR_MATH_BF16 && ngroups(d) == 1 &&
         d->c == 4 && d->k == 32 && d->r == 3 && d->s == 3 && d->stride == 2 && d->pad == 1 &&
         d->pad_w == 1 && d->w == 224 && d->wo == 112 && d->h % 2 == 0 && d->ho == d->h / 2 &&
         xld_of(d) == 4 && yld_of(d) == 32 && d->max_frames == 0;
}
static bool d3s_fwd(const tmr_conv_desc* d) {
  return d3s_shape(d) && d->io == (TMR_IO_W_BF16 | TMR_IO_Y_BF16);
}
static bool d3s_wgrad(const tmr_conv_desc* d) { return d3s_shape(d) && d->io == TMR_IO_DY_BF16; }
static bool d3_fwd(const tmr_conv_desc* d) {
  return d3_shape(d) && d->io == (TMR_IO_X_BF16 | TMR_IO_W_BF16 | TMR_IO_Y_BF16);
}
static bool d3_dgrad(const tmr_conv_desc* d) {
  const int io = d->io & ~TMR_IO_G16;   // (a bf16 masked gradient: the 56-wide convs)
  return d3_shape(d) && io == (TMR_IO_DY_BF16 | TMR_IO_WT_BF16 | TMR_IO_BN_BF16) &&
         (!(d->io & TMR_IO_G16) || d->w == 56);
}
static bool d3_wgrad(const tmr_conv_desc* d) {
  return d3_shape(d) && d->io == (TMR_IO_X_BF16 | TMR_IO_DY_BF16);
}

TMR_API int tmr_conv2d_fwd_stats_parts(const tmr_conv_desc* d) {
  if (!d || d->n <= 0) {
    tmr_set_error("tmr_conv2d_fwd_stats_parts: null or empty descriptor");
    return -1;
  }
  if (stem_direct(d)) return tmr_stem_stats_parts(d->n, d->ho);
  if (stem16_direct(d)) return tmr_stem16_stats_parts(d->n, d->ho);
  if (d3_fwd(d)) return tmr_d3_stats_parts(d->n, d->h, d->w, d->c, d->k);
  if (d3s_fwd(d)) return tmr_d3s_stats_parts(d->n, d->ho);
  tmr_conv_desc g = *d;
  if (ngroups(d) > 1 && group_split(d, g)) return -1;   // every group has the same row tiling
  const int fc = frames_per_launch(&g);
  int parts = 0;
  for (int f0 = 0; f0 < g.n; f0 += fc) {
    const tmr_conv_desc c = chunk_desc(&g, g.n - f0 < fc ? g.n - f0 : fc);
    parts += stats_parts_of(&c);
  }
  return parts;
}

TMR_API int tmr_conv2d_fwd_bnstats(const tmr_conv_desc* d, const float* x, const float* w_krsc,
                                   float* y, void* stats, size_t stats_bytes, hipStream_t stream) {
  return conv_fwd_bnstats_pro(d, x, w_krsc, y, stats, stats_bytes, nullptr, stream);
}

// stats: partial rows of part_ld columns (this launch's k columns at the pointer)
static int fwd_bnstats_impl(const tmr_conv_desc* d, const float* x, const float* w_krsc, float* y,
                            float4* st, int part_ld, const tmr_conv_prologue* pro,
                            hipStream_t stream) {
  const int fc = frames_per_launch(d);
  for (int f0 = 0; f0 < d->n; f0 += fc) {
    const tmr_conv_desc c = chunk_desc(d, d->n - f0 < fc ? d->n - f0 : fc);
    GemmArgs a;
    bool al;
    int rc = conv_fwd_args(&c, adv(x, f0 * x_frame(d), esz_x(d)), w_krsc, nullptr, adv(y, f0 * y_frame(d), esz_y(d)), 0.f, a, al);
    if (!rc) rc = set_prologue(a, pro, d, true, false, 0);
    if (rc) return rc;
    a.stats = st;
    a.part_ld = part_ld;
    rc = launch_gemm<MODE_FWD>(a, al, 1, stream);
    if (rc) return rc;
    st += (long)stats_parts_of(&c) * part_ld;
  }
  return 0;
}

static int conv_fwd_bnstats_pro(const tmr_conv_desc* d, const float* x,
                                const float* w_krsc, float* y, void* stats,
                                size_t stats_bytes, const tmr_conv_prologue* pro,
                                hipStream_t stream) {
  TMR_CHECK_ARG(d, "tmr_conv2d_fwd_bnstats: null descriptor");
  TMR_CHECK_ARG(yld_of(d) == d->k, "tmr_conv2d_fwd_bnstats: output must be dense (y_ld == k)");
  const int np = tmr_conv2d_fwd_stats_parts(d);
  TMR_CHECK_ARG(np >= 0, "tmr_conv2d_fwd_bnstats: bad descriptor");
  const size_t need = (size_t)np * d->k * sizeof(float4);
  TMR_CHECK_ARG(stats && stats_bytes >= need, "tmr_conv2d_fwd_bnstats: stats buffer too small (%zu < %zu)",
                stats_bytes, need);
  // the parts query (above) sized `stats` for the direct stem's row layout: an operand prologue
  // would route the stem to the engine, which writes a different number of partial rows
  TMR_CHECK_ARG(!(pro && (stem_direct(d) || stem16_direct(d) || d3_fwd(d) || d3s_fwd(d))),
                "tmr_conv2d_fwd_bnstats: the 7x7 stem takes no operand prologue");
  if (stem_direct(d))
    return tmr_stem_fwd_bnstats(d->n, d->h, d->w, d->ho, x, w_krsc, y, stats, stream);
  if (stem16_direct(d))
    return tmr_stem16_fwd_bnstats(d->n, d->h, d->w, d->ho, x, w_krsc, 4, y, stats, stream);
  if (!pro && d3_fwd(d))
    return tmr_d3_fwd_bnstats(d->n, d->h, d->w, d->c, d->k, x, w_krsc, y, stats, stream);
  if (!pro && d3s_fwd(d)) return tmr_d3s_fwd_bnstats(d->n, d->h, x, w_krsc, y, stats, stream);
  if (ngroups(d) == 1) return fwd_bnstats_impl(d, x, w_krsc, y, (float4*)stats, d->k, pro, stream);
  TMR_CHECK_ARG(!pro, "tmr_conv2d_fwd_bnstats: operand prologues take no groups");
  tmr_conv_desc g;
  if (group_split(d, g)) return 1;
  for (int i = 0; i < d->groups; ++i) {
    const int rc = fwd_bnstats_impl(&g, adv(x, (long)i * g.c, esz_x(d)), adv(w_krsc, i * group_wsize(&g), esz_w(d)),
                                    adv(y, (long)i * g.k, esz_y(d)), (float4*)stats + (long)i * g.k,
                                    d->k, nullptr, stream);
    if (rc) return rc;
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
  int part_ld;   // columns per partial row (the total channels of a grouped dgrad)
  const void* old;   // the beta operand when it is not dx itself (nullptr: dx)
  int old16;         // the beta operand is bf16
};

static int conv_dgrad_impl(const tmr_conv_desc* d, const float* dy, const float* w_krsc,
                           float* dx, float beta, hipStream_t stream, BnBwdFuse* fz = nullptr,
                           const tmr_conv_prologue* pro = nullptr) {
  TMR_CHECK_ARG(d->math == TMR_MATH_F32 || d->math == TMR_MATH_BF16, "tmr_conv2d: bad math mode %d", d->math);
  const int lk = ilog2_exact(d->k);
  TMR_CHECK_ARG(lk >= 2, "tmr_conv2d_dgrad: output channels %d must be a power of two >= 4", d->k);
  TMR_CHECK_ARG(d->c % 4 == 0, "tmr_conv2d_dgrad: input channels %d must be a multiple of 4", d->c);
  TMR_CHECK_ARG(!(d->io & TMR_IO_WT_BF16) || !(d->io & TMR_IO_W_BF16),
                "tmr_conv2d_dgrad: TMR_IO_WT_BF16 and TMR_IO_W_BF16 are exclusive weight layouts");
  TMR_CHECK_ARG(!(d->io & TMR_IO_WT_F32) ||
                    (d->math == TMR_MATH_F32 && (d->io & ~(TMR_IO_ENGINE | TMR_IO_CLASSES | TMR_IO_TILES)) == TMR_IO_WT_F32),
                "tmr_conv2d_dgrad: TMR_IO_WT_F32 (fp32 transposed weights) needs TMR_MATH_F32 and "
                "no bf16-stored operand");
  TMR_CHECK_ARG((d->io & ~(TMR_IO_WT_F32 | TMR_IO_ENGINE | TMR_IO_CLASSES | TMR_IO_TILES)) == 0 ||
                    d->math == TMR_MATH_BF16,
                "tmr_conv2d: bf16-stored operands (io %d) need TMR_MATH_BF16", d->io);
  const int st = d->stride;
  // one GEMM per stride-parity class (ph,pw): rows h = st*y + ph.  Stride 2 on the LDS-DMA
  // engine: the classes go out as one launch (launch_gemm_dgrad_par; TMR_IO_CLASSES: one each)
  const bool par = st == 2 && !pro && !(d->io & TMR_IO_CLASSES);
  GemmArgs pend[PAR_MAX];
  bool pend_al[PAR_MAX];
  int npend = 0;
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
      a.Abytes = clamp_bytes_e(span((long)d->n * d->ho * d->wo, a.lds, d->k), esz_dy(d));
      a.prec = d->math;
      a.Bbytes = clamp_bytes_e((long)d->k * d->r * d->s * d->c, esz_w(d));
      a.sab = ((d->io & TMR_IO_DY_BF16) ? 1 : 0) | ((d->io & (TMR_IO_W_BF16 | TMR_IO_WT_BF16)) ? 2 : 0);
      if (d->io & (TMR_IO_WT_BF16 | TMR_IO_WT_F32)) {   // w = Wt[ci][r][s][co] (bf16 / fp32)
        a.wt = 1;
        a.ldbt = d->r * d->s * d->k;
      }
      a.Cbytes = clamp_bytes(span((long)d->n * d->h * d->w, a.ldc, d->c));
      a.oH = d->h; a.oW = d->w; a.osy = st; a.osx = st; a.oyc = ph; a.oxc = pw;
      // nothing to add -- unless the fused BN backward must still see (mask, sum) these pixels
      if (a.K == 0 && beta == 1.f && !fz) continue;
      if (fz) {
        const long nmt = cdiv(a.M, gemm_tile_bm(a, MODE_DGRAD));
        if (fz->count_only) { fz->nparts += nmt; continue; }
        a.bn_y = fz->y; a.bn_z = fz->z; a.bn_sc = fz->sc; a.bn_sh = fz->sh; a.bn_mean = fz->mean;
        a.bn_mask = fz->mask;
        a.bn16 = (d->io & TMR_IO_BN_BF16) ? 1 : 0;
        if (d->io & TMR_IO_G16) {   // dx (g) stored bf16: C's extent in bytes of bf16
          a.g16 = 1;
          a.Cbytes = clamp_bytes_e(span((long)d->n * d->h * d->w, a.ldc, d->c), 2);
        }
        a.bn_part = fz->part;
        a.part_ld = fz->part_ld;
        a.Cold = fz->old;
        a.cold16 = fz->old16;
        a.io_tiles = (d->io & TMR_IO_TILES) ? 1 : 0;
        fz->part += nmt * fz->part_ld;
        fz->nparts += nmt;
      }
      bool al = aligned16(dy) && aligned16(w_krsc) && aligned16(dx) && a.lds % 4 == 0;
      int rc = set_prologue(a, pro, d, false, true, 0);
      if (!rc && par) {
        pend[npend] = a;
        pend_al[npend++] = al;
        continue;
      }
      if (!rc) rc = launch_gemm<MODE_DGRAD>(a, al, 1, stream);
      if (rc) return rc;
    }
  }
  if (npend > 0) {
    int rc = launch_gemm_dgrad_par(pend, npend, stream);
    if (rc < 0) {   // not eligible: one launch per class
      rc = 0;
      for (int i = 0; i < npend && rc == 0; ++i)
        rc = launch_gemm<MODE_DGRAD>(pend[i], pend_al[i], 1, stream);
    }
    if (rc) return rc;
  }
  return 0;
}

// the prologue of the frame chunk starting at frame f0 (dY's y moves with dY)
static tmr_conv_prologue chunk_pro(const tmr_conv_prologue* pro, const tmr_conv_desc* d, int f0) {
  tmr_conv_prologue p = *pro;
  if (p.dy_y) p.dy_y = adv(p.dy_y, f0 * y_frame(d), esz_dy(d));
  return p;
}

static int dgrad_bnbwd_run(const tmr_conv_desc* d, const float* dy, const float* w_krsc, float* dx,
                           float beta, BnBwdFuse* fz, hipStream_t stream,
                           const tmr_conv_prologue* pro = nullptr) {
  const int fc = frames_per_launch(d);
  const long px_frame = (long)d->h * d->w * xld_of(d);   // y / z laid out like dx
  float2* part0 = fz->part;
  for (int f0 = 0; f0 < d->n; f0 += fc) {
    const tmr_conv_desc c = chunk_desc(d, d->n - f0 < fc ? d->n - f0 : fc);
    BnBwdFuse fc_ = *fz;
    fc_.y = adv(fz->y, f0 * px_frame, esz_bn(d));
    // mask 3: z is bits, 32 elements per word (px_frame % 32 == 0, checked by the caller)
    fc_.z = fz->mask == 3 ? (const float*)((const uint32_t*)fz->z + f0 * px_frame / 32)
                          : adv(fz->z, f0 * px_frame, esz_bn(d));
    fc_.nparts = 0;
    if (fz->old) fc_.old = adv(fz->old, f0 * x_frame(d), fz->old16 ? 2 : 4);
    tmr_conv_prologue pc{};
    if (pro) pc = chunk_pro(pro, d, f0);
    int rc = conv_dgrad_impl(&c, adv(dy, f0 * y_frame(d), esz_dy(d)), w_krsc,
                             dx ? adv(dx, f0 * x_frame(d), esz_dx(d)) : nullptr, beta, stream, &fc_,
                             pro ? &pc : nullptr);
    if (rc) return rc;
    fz->part = fc_.part;
    fz->nparts += fc_.nparts;
  }
  fz->part = part0;
  return 0;
}

long tmrg::g_dgrad_ws_launches = 0;
TMR_API long tmr_dgrad_ws_launches(void) { return __atomic_load_n(&g_dgrad_ws_launches, __ATOMIC_RELAXED); }

TMR_API int tmr_conv2d_dgrad_bnbwd_parts(const tmr_conv_desc* d) {
  if (!d || d->n <= 0) {
    tmr_set_error("tmr_conv2d_dgrad_bnbwd_parts: null or empty descriptor");
    return -1;
  }
  if (d3_dgrad(d)) return tmr_d3_dgrad_parts(d->n, d->h, d->w, d->c, d->k);
  tmr_conv_desc g = *d;
  if (ngroups(d) > 1 && group_split(d, g)) return -1;   // every group has the same row tiling
  BnBwdFuse fz{};
  fz.count_only = true;
  fz.part_ld = g.c;
  if (dgrad_bnbwd_run(&g, nullptr, nullptr, nullptr, 1.f, &fz, nullptr)) return -1;
  return (int)fz.nparts;
}

TMR_API int tmr_conv2d_dgrad_bnbwd(const tmr_conv_desc* d, const float* dy, const float* w_krsc,
                                   float* dx, float beta, const float* y, const float* z,
                                   const float* scale, const float* shift, const float* mean,
                                   int mask, void* parts, size_t parts_bytes, hipStream_t stream) {
  return conv_dgrad_bnbwd_pro(d, dy, w_krsc, dx, beta, y, z, scale, shift, mean, mask, parts,
                                    parts_bytes, nullptr, stream);
}

static int dgrad_bnbwd_entry(const tmr_conv_desc* d, const float* dy, const float* w_krsc,
                             float* dx, float beta, const void* dx_old, int old_bf16,
                             const float* y, const float* z, const float* scale,
                             const float* shift, const float* mean, int mask, void* parts,
                             size_t parts_bytes, const tmr_conv_prologue* pro, hipStream_t stream);

static int conv_dgrad_bnbwd_pro(const tmr_conv_desc* d, const float* dy,
                                const float* w_krsc, float* dx, float beta, const float* y,
                                const float* z, const float* scale, const float* shift,
                                const float* mean, int mask, void* parts,
                                size_t parts_bytes, const tmr_conv_prologue* pro,
                                hipStream_t stream) {
  TMR_CHECK_ARG(d, "tmr_conv2d_dgrad_bnbwd: null descriptor");
  // in place: a bf16 gradient (TMR_IO_G16) accumulates into its own bf16 values
  return dgrad_bnbwd_entry(d, dy, w_krsc, dx, beta, nullptr, (d->io & TMR_IO_G16) ? 1 : 0, y, z,
                           scale, shift, mean, mask, parts, parts_bytes, pro, stream);
}

TMR_API int tmr_conv2d_dgrad_bnbwd_acc(const tmr_conv_desc* d, const float* dy,
                                       const float* w_krsc, void* dx, float beta,
                                       const void* dx_old, int old_bf16, const float* y,
                                       const float* z, const float* scale, const float* shift,
                                       const float* mean, int mask, void* parts,
                                       size_t parts_bytes, hipStream_t stream) {
  TMR_CHECK_ARG(d, "tmr_conv2d_dgrad_bnbwd_acc: null descriptor");
  TMR_CHECK_ARG(beta != 0.f && dx_old && ((uintptr_t)dx_old & 15) == 0 &&
                    (d->io & TMR_IO_G16) && (d->io & TMR_IO_WT_BF16),
                "tmr_conv2d_dgrad_bnbwd_acc: needs beta != 0, a 16-B aligned old dx and a bf16 "
                "output (TMR_IO_G16) on the bf16 LDS-DMA engine (TMR_IO_WT_BF16)");
  return dgrad_bnbwd_entry(d, dy, w_krsc, (float*)dx, beta, dx_old, old_bf16 ? 1 : 0, y, z, scale,
                           shift, mean, mask, parts, parts_bytes, nullptr, stream);
}

static int dgrad_bnbwd_entry(const tmr_conv_desc* d, const float* dy, const float* w_krsc,
                             float* dx, float beta, const void* dx_old, int old_bf16,
                             const float* y, const float* z, const float* scale,
                             const float* shift, const float* mean, int mask, void* parts,
                             size_t parts_bytes, const tmr_conv_prologue* pro, hipStream_t stream) {
  TMR_CHECK_ARG(xld_of(d) == d->c, "tmr_conv2d_dgrad_bnbwd: dx must be dense (x_ld == c)");
  TMR_CHECK_ARG(ngroups(d) == 1 || (mask != 3 && !pro),
                "tmr_conv2d_dgrad_bnbwd: a grouped dgrad takes no ReLU-mask bits / prologue");
  TMR_CHECK_ARG(y && mean && parts, "tmr_conv2d_dgrad_bnbwd: null y / mean / parts");
  TMR_CHECK_ARG(!(d->io & TMR_IO_G16) ||
                    (d->math == TMR_MATH_BF16 && (d->io & TMR_IO_WT_BF16) &&
                     (d->c / ngroups(d)) % 8 == 0),
                "tmr_conv2d_dgrad_bnbwd: a bf16 gradient (TMR_IO_G16) needs bf16 math on the LDS-DMA "
                "engine (TMR_IO_WT_BF16), channels per group a multiple of 8");
  TMR_CHECK_ARG(!dx_old || ngroups(d) == 1, "tmr_conv2d_dgrad_bnbwd: a separate old dx takes no groups");
  // a grouped dgrad writes each group's channel slice of a bf16 gradient with beta == 0 only (the
  // trunk's G16 on ResNeSt's radix-2 conv); accumulating into a bf16 dx runs ungrouped
  TMR_CHECK_ARG(ngroups(d) == 1 || beta == 0.f || !(d->io & TMR_IO_G16),
                "tmr_conv2d_dgrad_bnbwd: a grouped dgrad accumulates (beta != 0) into fp32 dx only");
  TMR_CHECK_ARG(mask == 0 || (mask == 1 && z) || (mask == 2 && scale && shift) || (mask == 3 && z),
                "tmr_conv2d_dgrad_bnbwd: mask %d needs z (1, 3: bits) or scale/shift (2)", mask);
  TMR_CHECK_ARG(mask != 3 || ((d->io & (TMR_IO_WT_F32 | TMR_IO_WT_BF16)) &&
                              ((long)d->h * d->w * d->c) % 32 == 0),
                "tmr_conv2d_dgrad_bnbwd: ReLU-mask bits (mask 3) need the LDS-DMA dgrad "
                "(TMR_IO_WT_F32 / TMR_IO_WT_BF16) and h*w*c a multiple of 32");
  const int np = tmr_conv2d_dgrad_bnbwd_parts(d);
  TMR_CHECK_ARG(np >= 0 && parts_bytes >= (size_t)np * d->c * sizeof(float2),
                "tmr_conv2d_dgrad_bnbwd: parts buffer too small");
  if (d3_dgrad(d)) {   // (the parts query above counted the direct kernel's rows)
    TMR_CHECK_ARG(!pro && !dx_old && !((d->io & TMR_IO_G16) && beta != 0.f),
                  "tmr_conv2d_dgrad_bnbwd: the direct 3x3 dgrad takes no prologue / old dx / "
                  "accumulating bf16 gradient");
    return tmr_d3_dgrad_bnbwd(d->n, d->h, d->w, d->c, d->k, dy, w_krsc, dx,
                              (d->io & TMR_IO_G16) ? 1 : 0, beta, y, z, scale, shift, mean, mask,
                              parts, stream);
  }
  if (ngroups(d) > 1) {
    tmr_conv_desc g;
    if (group_split(d, g)) return 1;
    for (int i = 0; i < d->groups; ++i) {
      const long o = (long)i * g.c;
      BnBwdFuse fz{};
      fz.y = adv(y, o, esz_bn(d)); fz.z = adv(z, o, esz_bn(d));
      fz.sc = scale ? scale + o : nullptr; fz.sh = shift ? shift + o : nullptr; fz.mean = mean + o;
      fz.mask = mask;
      fz.part = (float2*)parts + o;
      fz.part_ld = d->c;
      fz.old16 = 0;   // (beta != 0 with a bf16 dx is rejected above)
      const int rc = dgrad_bnbwd_run(&g, adv(dy, (long)i * g.k, esz_dy(d)), adv(w_krsc, i * group_wsize(&g), esz_w(d)),
                                     adv(dx, o, esz_dx(d)), beta, &fz, stream);
      if (rc) return rc;
    }
    return 0;
  }
  BnBwdFuse fz{};
  fz.y = y; fz.z = z; fz.sc = scale; fz.sh = shift; fz.mean = mean; fz.mask = mask;
  fz.part = (float2*)parts;
  fz.part_ld = d->c;
  fz.old = dx_old;
  fz.old16 = beta != 0.f ? old_bf16 : 0;
  return dgrad_bnbwd_run(d, dy, w_krsc, dx, beta, &fz, stream, pro);
}

TMR_API int tmr_conv2d_dgrad(const tmr_conv_desc* d, const float* dy, const float* w_krsc,
                             float* dx, float beta, hipStream_t stream) {
  return conv_dgrad_pro(d, dy, w_krsc, dx, beta, nullptr, stream);
}

static int conv_dgrad_pro(const tmr_conv_desc* d, const float* dy, const float* w_krsc,
                          float* dx, float beta, const tmr_conv_prologue* pro,
                          hipStream_t stream) {
  TMR_CHECK_ARG(d, "tmr_conv2d_dgrad: null descriptor");
  if (ngroups(d) > 1) {
    TMR_CHECK_ARG(!pro, "tmr_conv2d_dgrad: operand prologues take no groups");
    tmr_conv_desc g;
    if (group_split(d, g)) return 1;
    for (int i = 0; i < d->groups; ++i) {
      const int rc = conv_dgrad_pro(&g, adv(dy, (long)i * g.k, esz_dy(d)), adv(w_krsc, i * group_wsize(&g), esz_w(d)),
                                          dx + (long)i * g.c, beta, nullptr, stream);
      if (rc) return rc;
    }
    return 0;
  }
  const int fc = frames_per_launch(d);
  for (int f0 = 0; f0 < d->n; f0 += fc) {
    const tmr_conv_desc c = chunk_desc(d, d->n - f0 < fc ? d->n - f0 : fc);
    tmr_conv_prologue pc{};
    if (pro) pc = chunk_pro(pro, d, f0);
    int rc = conv_dgrad_impl(&c, adv(dy, f0 * y_frame(d), esz_dy(d)), w_krsc, dx + f0 * x_frame(d), beta, stream,
                             nullptr, pro ? &pc : nullptr);
    if (rc) return rc;
  }
  return 0;
}

// the WGRAD view of a conv (no pointers, no split plan)
static void wgrad_fill(const tmr_conv_desc* d, GemmArgs& a) {
  a = GemmArgs{};
  a.M = d->k; a.N = d->r * d->s * d->c; a.K = d->n * d->ho * d->wo;
  a.log2C = ilog2_exact(d->c);
  set_taps(a, d->r, d->s);
  a.oy0 = -d->pad; a.ox0 = -d->pad_w; a.dyr = 1; a.dxs = 1;
  set_grid(a, d->n, d->ho, d->wo);
  a.Hs = d->h; a.Ws = d->w; a.sy = d->stride; a.sx = d->stride;
  a.lds = xld_of(d); a.ldb = yld_of(d); a.ldc = a.N; a.beta = 0.f;
  a.Abytes = clamp_bytes_e(span((long)d->n * d->ho * d->wo, a.ldb, d->k), esz_dy(d));
  a.prec = d->math;
  a.Bbytes = clamp_bytes_e(span((long)d->n * d->h * d->w, a.lds, d->c), esz_x(d));
  a.sab = ((d->io & TMR_IO_DY_BF16) ? 1 : 0) | ((d->io & TMR_IO_X_BF16) ? 2 : 0);
  a.dma32 = d->math == TMR_MATH_F32;
}

static int wgrad_plan(const tmr_conv_desc* d, int* splits, int* kchunk, long* slab) {
  const long Mred = (long)d->n * d->ho * d->wo;
  const long Mo = d->k, No = (long)d->r * d->s * d->c;
  GemmArgs a;
  wgrad_fill(d, a);
  const long tiles = gemm_tiles(a, MODE_WGRAD);
  // aim for ~target workgroups; at least minrows reduction rows per split
  static const long target = env_int("TMR_WGRAD_TARGET", 512);
  static const long minrows = env_int("TMR_WGRAD_MINROWS", 1024);
  long sp = target / (tiles > 0 ? tiles : 1);
  if (sp < 1) sp = 1;
  long maxsp = Mred / minrows;
  if (maxsp < 1) maxsp = 1;
  if (sp > maxsp) sp = maxsp;
  long kc = (Mred + sp - 1) / sp;
  kc = (kc + 63) / 64 * 64;  // multiple of every BK (16, 32, 64)
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
  tmr_conv_desc g = *d;
  if (ngroups(d) > 1 && group_split(d, g)) return 0;   // one group's workspace, reused in turn
  int sp, kc;
  long slab;
  // the plans of the two chunk sizes a launch runs (the largest, and the remainder): a smaller
  // chunk can keep more splits (its chunk length rounds up less)
  const int fc = frames_per_launch(&g);
  const tmr_conv_desc c = chunk_desc(&g, fc < g.n ? fc : g.n);
  wgrad_plan(&c, &sp, &kc, &slab);
  size_t bytes = (size_t)sp * slab * sizeof(float);
  if (g.n > fc && g.n % fc != 0) {
    const tmr_conv_desc cr = chunk_desc(&g, g.n % fc);
    wgrad_plan(&cr, &sp, &kc, &slab);
    if ((size_t)sp * slab * sizeof(float) > bytes) bytes = (size_t)sp * slab * sizeof(float);
  }
  if (stem_geometry(d) && bytes < (size_t)kStemSlabs * kStemSlab * sizeof(float))
    bytes = (size_t)kStemSlabs * kStemSlab * sizeof(float);
  if (stem16_wgrad_geometry(d) && bytes < (size_t)kStem16Slabs * kStemSlab * sizeof(float))
    bytes = (size_t)kStem16Slabs * kStemSlab * sizeof(float);
  if (d3_wgrad(d) && bytes < tmr_d3_wgrad_ws_bytes(d->n, d->h, d->w, d->c, d->k))
    bytes = tmr_d3_wgrad_ws_bytes(d->n, d->h, d->w, d->c, d->k);
  if (d3s_wgrad(d) && bytes < tmr_d3s_wgrad_ws_bytes(d->n, d->ho))
    bytes = tmr_d3s_wgrad_ws_bytes(d->n, d->ho);
  return bytes;
}

static int conv_wgrad_impl(const tmr_conv_desc* d, const float* x, const float* dy,
                           float* dw_oihw, int c_real, float beta, float* ws, size_t ws_bytes,
                           hipStream_t stream, const tmr_conv_prologue* pro);

// frame chunks accumulate into dw in chunk order (beta = 1 after the first): deterministic
TMR_API int tmr_conv2d_wgrad(const tmr_conv_desc* d, const float* x, const float* dy,
                             float* dw_oihw, int c_real, float beta, float* ws, size_t ws_bytes,
                             hipStream_t stream) {
  return conv_wgrad_pro(d, x, dy, dw_oihw, c_real, beta, ws, ws_bytes, nullptr, stream);
}

static int conv_wgrad_pro(const tmr_conv_desc* d, const float* x, const float* dy,
                          float* dw_oihw, int c_real, float beta, float* ws,
                          size_t ws_bytes, const tmr_conv_prologue* pro,
                          hipStream_t stream) {
  TMR_CHECK_ARG(d, "tmr_conv2d_wgrad: null descriptor");
  if (ngroups(d) > 1) {   // c_real = real input channels per group; dw (k, c_real, r, s)
    TMR_CHECK_ARG(!pro, "tmr_conv2d_wgrad: operand prologues take no groups");
    tmr_conv_desc g;
    if (group_split(d, g)) return 1;
    for (int i = 0; i < d->groups; ++i) {
      const int rc = conv_wgrad_pro(&g, adv(x, (long)i * g.c, esz_x(d)), adv(dy, (long)i * g.k, esz_dy(d)),
                                          dw_oihw + (long)i * g.k * c_real * g.r * g.s, c_real,
                                          beta, ws, ws_bytes, nullptr, stream);
      if (rc) return rc;
    }
    return 0;
  }
  const int fc = frames_per_launch(d);
  for (int f0 = 0; f0 < d->n; f0 += fc) {
    const tmr_conv_desc c = chunk_desc(d, d->n - f0 < fc ? d->n - f0 : fc);
    tmr_conv_prologue pc{};
    if (pro) pc = chunk_pro(pro, d, f0);
    int rc = conv_wgrad_impl(&c, adv(x, f0 * x_frame(d), esz_x(d)), adv(dy, f0 * y_frame(d), esz_dy(d)), dw_oihw, c_real,
                             f0 == 0 ? beta : 1.f, ws, ws_bytes, stream, pro ? &pc : nullptr);
    if (rc) return rc;
  }
  return 0;
}

static int conv_wgrad_impl(const tmr_conv_desc* d, const float* x, const float* dy,
                           float* dw_oihw, int c_real, float beta, float* ws, size_t ws_bytes,
                           hipStream_t stream, const tmr_conv_prologue* pro) {
  TMR_CHECK_ARG(d->math == TMR_MATH_F32 || d->math == TMR_MATH_BF16, "tmr_conv2d: bad math mode %d", d->math);
  const int lc = ilog2_exact(d->c);
  TMR_CHECK_ARG(lc >= 2, "tmr_conv2d_wgrad: stored input channels %d must be a power of two >= 4", d->c);
  TMR_CHECK_ARG(c_real >= 1 && c_real <= d->c, "tmr_conv2d_wgrad: bad c_real %d", c_real);
  const bool s16 = !pro && c_real == 3 && !(d->io & TMR_IO_ENGINE) &&
                   stem16_wgrad_geometry(d);
  if (s16 || (!pro && c_real == 3 && stem_direct(d))) {
    int ns = 0;
    const int rc = s16 ? tmr_stem16_wgrad_slabs(d->n, d->h, d->w, d->ho, x, dy,
                                                (d->io & TMR_IO_DY_BF16) ? 0 : 1, ws, ws_bytes,
                                                &ns, stream)
                       : tmr_stem_wgrad_slabs(d->n, d->h, d->w, d->ho, x, dy, ws, ws_bytes, &ns, stream);
    if (rc) return rc;
    hipLaunchKernelGGL(wgrad_reduce_taps_kernel, dim3(d->k, 1), dim3(256), 0, stream, ws, ns,
                       kStemSlab, dw_oihw, 49, 4, 3, beta);
    TMR_CHECK_LAUNCH("wgrad_reduce_taps_kernel");
    return 0;
  }
  if (!pro && c_real == 3 && d3s_wgrad(d)) {
    int ns = 0;
    const int rc = tmr_d3s_wgrad_slabs(d->n, d->h, x, dy, ws, ws_bytes, &ns, stream);
    if (rc) return rc;
    hipLaunchKernelGGL(wgrad_reduce_taps_kernel, dim3(d->k, 1), dim3(256), 0, stream, ws, ns,
                       (long)32 * 9 * 4, dw_oihw, 9, 4, 3, beta);
    TMR_CHECK_LAUNCH("wgrad_reduce_taps_kernel");
    return 0;
  }
  if (!pro && d3_wgrad(d)) {
    int ns = 0;
    const int rc = tmr_d3_wgrad_slabs(d->n, d->h, d->w, d->c, d->k, x, dy, ws, ws_bytes, &ns, stream);
    if (rc) return rc;
    hipLaunchKernelGGL(wgrad_reduce_taps_kernel, dim3(d->k, cdiv(c_real, 64)), dim3(256), 0, stream,
                       ws, ns, (long)d->k * 9 * d->c, dw_oihw, 9, d->c, c_real, beta);
    TMR_CHECK_LAUNCH("wgrad_reduce_taps_kernel");
    return 0;
  }
  int sp, kc;
  long slab;
  wgrad_plan(d, &sp, &kc, &slab);
  TMR_CHECK_ARG(ws && ws_bytes >= (size_t)sp * slab * sizeof(float),
                "tmr_conv2d_wgrad: workspace too small (%zu < %zu)", ws_bytes,
                (size_t)sp * slab * sizeof(float));
  GemmArgs a;
  wgrad_fill(d, a);
  (void)lc;
  a.A = dy; a.B = x; a.C = ws; a.bias = nullptr;
  a.kchunk = kc; a.slab = slab;
  a.Cbytes = clamp_bytes(slab);
  bool al = aligned16(x) && aligned16(dy) && (d->k % 4 == 0) && a.lds % 4 == 0 && a.ldb % 4 == 0;
  int rc = set_prologue(a, pro, d, true, true, 0);
  if (!rc) rc = launch_gemm<MODE_WGRAD>(a, al, sp, stream);
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

#if TMR_PROLOGUES
TMR_API int tmr_conv2d_fwd_bnstats_pro(const tmr_conv_desc* d, const float* x,
                                       const float* w_krsc, float* y, void* stats,
                                       size_t stats_bytes, const tmr_conv_prologue* pro,
                                       hipStream_t stream) {
  return conv_fwd_bnstats_pro(d, x, w_krsc, y, stats, stats_bytes, pro, stream);
}

TMR_API int tmr_conv2d_dgrad_pro(const tmr_conv_desc* d, const float* dy, const float* w_krsc,
                                 float* dx, float beta, const tmr_conv_prologue* pro,
                                 hipStream_t stream) {
  return conv_dgrad_pro(d, dy, w_krsc, dx, beta, pro, stream);
}

TMR_API int tmr_conv2d_dgrad_bnbwd_pro(const tmr_conv_desc* d, const float* dy,
                                       const float* w_krsc, float* dx, float beta, const float* y,
                                       const float* z, const float* scale, const float* shift,
                                       const float* mean, int mask, void* parts,
                                       size_t parts_bytes, const tmr_conv_prologue* pro,
                                       hipStream_t stream) {
  return conv_dgrad_bnbwd_pro(d, dy, w_krsc, dx, beta, y, z, scale, shift, mean, mask, parts,
                              parts_bytes, pro, stream);
}

TMR_API int tmr_conv2d_dgrad_bnbwd_acc_pro(const tmr_conv_desc* d, const float* dy,
                                           const float* w_krsc, void* dx, float beta,
                                           const void* dx_old, int old_bf16, const float* y,
                                           const float* z, const float* scale, const float* shift,
                                           const float* mean, int mask, void* parts,
                                           size_t parts_bytes, const tmr_conv_prologue* pro,
                                           hipStream_t stream) {
  TMR_CHECK_ARG(d, "tmr_conv2d_dgrad_bnbwd_acc_pro: null descriptor");
  TMR_CHECK_ARG(beta != 0.f && dx_old && ((uintptr_t)dx_old & 15) == 0 &&
                    (d->io & TMR_IO_G16) && (d->io & TMR_IO_WT_BF16),
                "tmr_conv2d_dgrad_bnbwd_acc_pro: needs beta != 0, a 16-B aligned old dx and a bf16 "
                "output (TMR_IO_G16) on the bf16 LDS-DMA engine (TMR_IO_WT_BF16)");
  return dgrad_bnbwd_entry(d, dy, w_krsc, (float*)dx, beta, dx_old, old_bf16 ? 1 : 0, y, z, scale,
                           shift, mean, mask, parts, parts_bytes, pro, stream);
}

TMR_API int tmr_conv2d_wgrad_pro(const tmr_conv_desc* d, const float* x, const float* dy,
                                 float* dw_oihw, int c_real, float beta, float* ws,
                                 size_t ws_bytes, const tmr_conv_prologue* pro,
                                 hipStream_t stream) {
  return conv_wgrad_pro(d, x, dy, dw_oihw, c_real, beta, ws, ws_bytes, pro, stream);
}
#endif

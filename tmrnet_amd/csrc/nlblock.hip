// The clip branch after the LSTM as C entry points: NLBlock forward/backward, TimeConv
// forward/weight-gradient and nn.Linear forward/backward (code/Training TMRNet/
// NLBlock_MutiConv6_3.py:10-79, train_only_non-local_pretrained.py:235-239).
//
// NLBlock attention core in re-associated GEMV form (include/tmr.h, tmr_nl_attn_fwd): the only
// HBM-heavy operand is Lt -- (B, L, 512) rows, dense or gathered from the resident LFB bank by the
// row table -- so the kernels split every clip's L rows over 32-row workgroups (grid L/32 x B:
// 640 workgroups at C5's B = 64, L = 300) and read each row once per pass:
//   forward : per chunk, scores s_l = scale * Lt_l.u, chunk max m, e_l = exp(s_l - m), the chunk's
//             sum S and context sum_l e_l Lt_l; a combine kernel rescales the chunks to the clip
//             max (the online-softmax identity), writes p and ctx.
//   backward: pass A dp_l = dctx.Lt_l and per-chunk sum_l p_l dp_l; pass B
//             ds_l = scale p_l (dp_l - sum p dp) and per-chunk sum_l ds_l Lt_l (+ dLt for a dense
//             Lt); a combine kernel adds the chunks in order (deterministic).
#include "common.h"
#include "tmr.h"

namespace {

constexpr int NT = 256;
constexpr int RW = 8;              // rows per wave
constexpr int RC = RW * (NT / 64); // rows per workgroup (chunk)

__device__ __forceinline__ float dot4(const float4 a, const float4 b, float s) {
  s = fmaf(a.x, b.x, s); s = fmaf(a.y, b.y, s); s = fmaf(a.z, b.z, s); s = fmaf(a.w, b.w, s);
  return s;
}
__device__ __forceinline__ float4 axpy4(float a, const float4 x, float4 y) {
  y.x = fmaf(a, x.x, y.x); y.y = fmaf(a, x.y, y.y); y.z = fmaf(a, x.z, y.z); y.w = fmaf(a, x.w, y.w);
  return y;
}

// Lt row index of (clip b, row l)
__device__ __forceinline__ long lt_row(const int32_t* rows, int b, int L, int l) {
  return rows ? (long)rows[(long)b * L + l] : (long)b * L + l;
}

// DV = D / 256 float4 per lane
template <int DV>
__global__ __launch_bounds__(NT) void nl_fwd_part_k(const float* __restrict__ lt,
                                                    const int32_t* __restrict__ rows,
                                                    const float* __restrict__ u,
                                                    float* __restrict__ p, float* __restrict__ pm,
                                                    float* __restrict__ ps, float* __restrict__ pv,
                                                    int L, float scale) {
  constexpr int D = 256 * DV;
  __shared__ float sm_m[NT / 64], sm_s[NT / 64];
  __shared__ __attribute__((aligned(16))) float sm_v[NT / 64][D];
  const int b = blockIdx.y, ch = blockIdx.x, nch = gridDim.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float4 uu[DV];
#pragma unroll
  for (int q = 0; q < DV; ++q)
    uu[q] = *reinterpret_cast<const float4*>(&u[(long)b * D + 256 * q + 4 * lane]);
  float4 row[RW][DV];
  float s[RW];
  const int l0 = ch * RC + wave * RW;
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    const int l = l0 + r;
    const bool ok = l < L;
    const long rr = ok ? lt_row(rows, b, L, l) : 0;
#pragma unroll
    for (int q = 0; q < DV; ++q)
      row[r][q] = ok ? *reinterpret_cast<const float4*>(&lt[rr * D + 256 * q + 4 * lane])
                     : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float m = -INFINITY;
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < DV; ++q) t = dot4(row[r][q], uu[q], t);
    t = warp_sum(t) * scale;
    s[r] = l0 + r < L ? t : -INFINITY;
    m = fmaxf(m, s[r]);
  }
  float sum = 0.f;
  float4 v[DV];
#pragma unroll
  for (int q = 0; q < DV; ++q) v[q] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    if (l0 + r < L) {
      const float e = expf(s[r] - m);
      sum += e;
#pragma unroll
      for (int q = 0; q < DV; ++q) v[q] = axpy4(e, row[r][q], v[q]);
      if (lane == 0) p[(long)b * L + l0 + r] = s[r];   // raw score; normalised by the combine
    }
  }
#pragma unroll
  for (int q = 0; q < DV; ++q) *reinterpret_cast<float4*>(&sm_v[wave][256 * q + 4 * lane]) = v[q];
  if (lane == 0) { sm_m[wave] = m; sm_s[wave] = sum; }
  __syncthreads();
  float M = -INFINITY;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) M = fmaxf(M, sm_m[w]);
  float f[NT / 64];
  float S = 0.f;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    f[w] = sm_m[w] == -INFINITY ? 0.f : expf(sm_m[w] - M);
    S = fmaf(sm_s[w], f[w], S);
  }
  const long o = (long)b * nch + ch;
  for (int c = threadIdx.x; c < D; c += NT) {
    float a = 0.f;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) a = fmaf(sm_v[w][c], f[w], a);
    pv[o * D + c] = a;
  }
  if (threadIdx.x == 0) { pm[o] = M; ps[o] = S; }
}

__global__ __launch_bounds__(NT) void nl_fwd_comb_k(const float* __restrict__ pm,
                                                    const float* __restrict__ ps,
                                                    const float* __restrict__ pv,
                                                    float* __restrict__ p, float* __restrict__ ctx,
                                                    int L, int D, int nch) {
  extern __shared__ float fs[];   // [nch] chunk scale factors
  __shared__ float sh[2];
  const int b = blockIdx.x;
  if (threadIdx.x == 0) {
    float M = -INFINITY;
    for (int j = 0; j < nch; ++j) M = fmaxf(M, pm[(long)b * nch + j]);
    float S = 0.f;
    for (int j = 0; j < nch; ++j) {
      const float f = expf(pm[(long)b * nch + j] - M);
      fs[j] = f;
      S = fmaf(ps[(long)b * nch + j], f, S);
    }
    sh[0] = M;
    sh[1] = 1.0f / S;
  }
  __syncthreads();
  const float M = sh[0], inv = sh[1];
  for (int c = threadIdx.x; c < D; c += NT) {
    float a = 0.f;
    for (int j = 0; j < nch; ++j) a = fmaf(pv[((long)b * nch + j) * D + c], fs[j], a);
    ctx[(long)b * D + c] = a * inv;
  }
  for (int l = threadIdx.x; l < L; l += NT) {
    const long i = (long)b * L + l;
    p[i] = expf(p[i] - M) * inv;
  }
}

// pass A: dp_l = dctx . Lt_l, chunk partial sum_l p_l dp_l
template <int DV>
__global__ __launch_bounds__(NT) void nl_bwd_a_k(const float* __restrict__ lt,
                                                 const int32_t* __restrict__ rows,
                                                 const float* __restrict__ p,
                                                 const float* __restrict__ dctx,
                                                 float* __restrict__ dp, float* __restrict__ tp,
                                                 int L) {
  constexpr int D = 256 * DV;
  __shared__ float sm_t[NT / 64];
  const int b = blockIdx.y, ch = blockIdx.x, nch = gridDim.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float4 gg[DV];
#pragma unroll
  for (int q = 0; q < DV; ++q)
    gg[q] = *reinterpret_cast<const float4*>(&dctx[(long)b * D + 256 * q + 4 * lane]);
  const int l0 = ch * RC + wave * RW;
  float4 row[RW][DV];
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    const int l = l0 + r;
    const bool ok = l < L;
    const long rr = ok ? lt_row(rows, b, L, l) : 0;
#pragma unroll
    for (int q = 0; q < DV; ++q)
      row[r][q] = ok ? *reinterpret_cast<const float4*>(&lt[rr * D + 256 * q + 4 * lane])
                     : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float t = 0.f;
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    float d = 0.f;
#pragma unroll
    for (int q = 0; q < DV; ++q) d = dot4(row[r][q], gg[q], d);
    d = warp_sum(d);
    const int l = l0 + r;
    if (l < L) {
      if (lane == 0) dp[(long)b * L + l] = d;
      t = fmaf(p[(long)b * L + l], d, t);
    }
  }
  if (lane == 0) sm_t[wave] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) a += sm_t[w];
    tp[(long)b * nch + ch] = a;
  }
}

// pass B: ds_l = scale p_l (dp_l - t), chunk partial sum_l ds_l Lt_l; dLt (dense Lt only)
template <int DV>
__global__ __launch_bounds__(NT) void nl_bwd_b_k(const float* __restrict__ lt,
                                                 const int32_t* __restrict__ rows,
                                                 const float* __restrict__ u,
                                                 const float* __restrict__ p,
                                                 const float* __restrict__ dctx,
                                                 const float* __restrict__ dp,
                                                 const float* __restrict__ tp,
                                                 float* __restrict__ wpart, float* __restrict__ dlt,
                                                 int L, float scale) {
  constexpr int D = 256 * DV;
  __shared__ __attribute__((aligned(16))) float sm_w[NT / 64][D];
  __shared__ float sh_t;
  const int b = blockIdx.y, ch = blockIdx.x, nch = gridDim.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) {
    float a = 0.f;
    for (int j = 0; j < nch; ++j) a += tp[(long)b * nch + j];
    sh_t = a;
  }
  __syncthreads();
  const float t = sh_t;
  const int l0 = ch * RC + wave * RW;
  float4 acc[DV];
#pragma unroll
  for (int q = 0; q < DV; ++q) acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    const int l = l0 + r;
    if (l < L) {
      const long rr = lt_row(rows, b, L, l);
      const float pl = p[(long)b * L + l];
      const float ds = scale * pl * (dp[(long)b * L + l] - t);
#pragma unroll
      for (int q = 0; q < DV; ++q) {
        const int c = 256 * q + 4 * lane;
        const float4 x = *reinterpret_cast<const float4*>(&lt[rr * D + c]);
        acc[q] = axpy4(ds, x, acc[q]);
        if (dlt) {
          const float4 g = *reinterpret_cast<const float4*>(&dctx[(long)b * D + c]);
          const float4 uv = *reinterpret_cast<const float4*>(&u[(long)b * D + c]);
          float4 o;
          o.x = fmaf(pl, g.x, ds * uv.x); o.y = fmaf(pl, g.y, ds * uv.y);
          o.z = fmaf(pl, g.z, ds * uv.z); o.w = fmaf(pl, g.w, ds * uv.w);
          *reinterpret_cast<float4*>(&dlt[((long)b * L + l) * D + c]) = o;
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < DV; ++q) *reinterpret_cast<float4*>(&sm_w[wave][256 * q + 4 * lane]) = acc[q];
  __syncthreads();
  const long o = (long)b * nch + ch;
  for (int c = threadIdx.x; c < D; c += NT) {
    float a = 0.f;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) a += sm_w[w][c];
    wpart[o * D + c] = a;
  }
}

__global__ void nl_bwd_comb_k(const float* __restrict__ wpart, float* __restrict__ ut, int D,
                              int nch, long n) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long b = i / D;
  const int c = (int)(i % D);
  float a = 0.f;
  for (int j = 0; j < nch; ++j) a += wpart[(b * nch + j) * D + c];
  ut[i] = a;
}

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
int nchunks(int l) { return (l + RC - 1) / RC; }

struct AttnWs {
  size_t pm, ps, pv, tp, dp, wp, total;
};
AttnWs attn_ws(int b, int l, int d) {
  AttnWs w;
  const size_t nc = (size_t)b * nchunks(l);
  size_t o = 0;
  w.pm = o; o += al256(nc * 4);
  w.ps = o; o += al256(nc * 4);
  w.pv = o; o += al256(nc * d * 4);
  const size_t fwd = o;
  o = 0;
  w.tp = o; o += al256(nc * 4);
  w.dp = o; o += al256((size_t)b * l * 4);
  w.wp = o; o += al256(nc * d * 4);
  w.total = fwd > o ? fwd : o;
  return w;
}

bool attn_dims_ok(int d) { return d == 256 || d == 512 || d == 1024; }

}  // namespace

TMR_API size_t tmr_nl_attn_ws_bytes(int b, int l, int d) {
  if (b < 0 || l < 1 || !attn_dims_ok(d)) {
    tmr_set_error("tmr_nl_attn_ws_bytes: bad sizes b=%d l=%d d=%d", b, l, d);
    return 0;
  }
  return attn_ws(b, l, d).total;
}

TMR_API int tmr_nl_attn_fwd(const float* lt, const int32_t* rows, const float* u, float* p,
                            float* ctx, int b, int l, int d, float scale, void* ws, size_t ws_bytes,
                            hipStream_t stream) {
  TMR_CHECK_ARG(attn_dims_ok(d), "tmr_nl_attn_fwd: feature dim %d must be 256, 512 or 1024", d);
  TMR_CHECK_ARG(l >= 1 && l <= (1 << 20), "tmr_nl_attn_fwd: bad L %d", l);
  TMR_CHECK_ARG(b >= 0, "tmr_nl_attn_fwd: bad B %d", b);
  if (b == 0) return 0;
  const AttnWs w = attn_ws(b, l, d);
  TMR_CHECK_ARG(ws && ws_bytes >= w.total, "tmr_nl_attn_fwd: workspace %zu < %zu bytes", ws_bytes,
                w.total);
  char* c = (char*)ws;
  float *pm = (float*)(c + w.pm), *ps = (float*)(c + w.ps), *pv = (float*)(c + w.pv);
  const int nch = nchunks(l);
  const dim3 grid(nch, b);
  if (d == 256)
    hipLaunchKernelGGL(nl_fwd_part_k<1>, grid, dim3(NT), 0, stream, lt, rows, u, p, pm, ps, pv, l, scale);
  else if (d == 512)
    hipLaunchKernelGGL(nl_fwd_part_k<2>, grid, dim3(NT), 0, stream, lt, rows, u, p, pm, ps, pv, l, scale);
  else
    hipLaunchKernelGGL(nl_fwd_part_k<4>, grid, dim3(NT), 0, stream, lt, rows, u, p, pm, ps, pv, l, scale);
  TMR_CHECK_LAUNCH("nl_attn_fwd part");
  hipLaunchKernelGGL(nl_fwd_comb_k, dim3(b), dim3(NT), nch * sizeof(float), stream, pm, ps, pv, p,
                     ctx, l, d, nch);
  TMR_CHECK_LAUNCH("nl_attn_fwd combine");
  return 0;
}

TMR_API int tmr_nl_attn_bwd(const float* lt, const int32_t* rows, const float* u, const float* p,
                            const float* dctx, float* ut, float* dlt, int b, int l, int d,
                            float scale, void* ws, size_t ws_bytes, hipStream_t stream) {
  TMR_CHECK_ARG(attn_dims_ok(d), "tmr_nl_attn_bwd: feature dim %d must be 256, 512 or 1024", d);
  TMR_CHECK_ARG(l >= 1 && l <= (1 << 20), "tmr_nl_attn_bwd: bad L %d", l);
  TMR_CHECK_ARG(!(dlt && rows), "tmr_nl_attn_bwd: dLt only for a dense Lt");
  TMR_CHECK_ARG(b >= 0, "tmr_nl_attn_bwd: bad B %d", b);
  if (b == 0) return 0;
  const AttnWs w = attn_ws(b, l, d);
  TMR_CHECK_ARG(ws && ws_bytes >= w.total, "tmr_nl_attn_bwd: workspace %zu < %zu bytes", ws_bytes,
                w.total);
  char* c = (char*)ws;
  float *tp = (float*)(c + w.tp), *dp = (float*)(c + w.dp), *wp = (float*)(c + w.wp);
  const int nch = nchunks(l);
  const dim3 grid(nch, b);
#define NL_BWD(DV)                                                                              \
  hipLaunchKernelGGL(nl_bwd_a_k<DV>, grid, dim3(NT), 0, stream, lt, rows, p, dctx, dp, tp, l);  \
  TMR_CHECK_LAUNCH("nl_attn_bwd a");                                                            \
  hipLaunchKernelGGL(nl_bwd_b_k<DV>, grid, dim3(NT), 0, stream, lt, rows, u, p, dctx, dp, tp,   \
                     wp, dlt, l, scale);                                                        \
  TMR_CHECK_LAUNCH("nl_attn_bwd b");
  if (d == 256) { NL_BWD(1) } else if (d == 512) { NL_BWD(2) } else { NL_BWD(4) }
#undef NL_BWD
  const long n = (long)b * d;
  hipLaunchKernelGGL(nl_bwd_comb_k, dim3(cdiv(n, 256)), dim3(256), 0, stream, wp, ut, d, nch, n);
  TMR_CHECK_LAUNCH("nl_attn_bwd combine");
  return 0;
}

// ---------------------------------------------------------------- nn.Linear
TMR_API int tmr_linear_fwd(const float* x, int rows, int in, int out, const float* w,
                           const float* bias, float* y, hipStream_t stream) {
  TMR_CHECK_ARG(rows >= 0 && in > 0 && out > 0, "tmr_linear_fwd: bad sizes %d x %d -> %d", rows,
                in, out);
  TMR_CHECK_ARG(x && w && y, "tmr_linear_fwd: null operand");
  return tmr_gemm_nt(rows, out, in, x, in, w, in, bias, y, out, 0.f, stream);
}

TMR_API int tmr_linear_bwd(const float* dy, const float* x, int rows, int in, int out,
                           const float* w, float* dx, float* dw, float* db, float beta,
                           hipStream_t stream) {
  TMR_CHECK_ARG(rows >= 0 && in > 0 && out > 0, "tmr_linear_bwd: bad sizes %d x %d -> %d", rows,
                in, out);
  TMR_CHECK_ARG(dy && (!dx || w) && (!dw || x), "tmr_linear_bwd: null operand");
  int rc;
  if (dw && (rc = tmr_gemm_tn(out, in, rows, dy, out, x, in, dw, in, beta, stream))) return rc;
  if (db && (rc = tmr_col_sum(dy, rows, out, out, db, beta, stream))) return rc;
  if (dx && (rc = tmr_gemm_nn(rows, in, out, dy, out, w, in, dx, in, 0.f, stream))) return rc;
  return 0;
}

// ---------------------------------------------------------------- NLBlock
namespace {
constexpr int ND = 512;   // LayerNorm([1, 512]) fixes the feature size (NLBlock_MutiConv6_3.py:17)

struct NlSaved {
  size_t q, u, p, c, sll, a, mu, rs, total;
};
NlSaved nl_saved(int b, int l) {
  NlSaved s;
  const size_t v = al256((size_t)b * ND * 4);
  size_t o = 0;
  s.q = o; o += v;
  s.u = o; o += v;
  s.p = o; o += al256((size_t)b * l * 4);
  s.c = o; o += v;
  s.sll = o; o += v;
  s.a = o; o += v;
  s.mu = o; o += al256((size_t)b * 4);
  s.rs = o; o += al256((size_t)b * 4);
  s.total = o;
  return s;
}
struct NlWs {
  size_t attn, dz, da, dsll, dc, ut, dq, total;
};
NlWs nl_ws(int b, int l) {
  NlWs w;
  const size_t v = al256((size_t)b * ND * 4);
  size_t o = 0;
  w.dz = o; o += v;
  w.da = o; o += v;
  w.dsll = o; o += v;
  w.dc = o; o += v;
  w.ut = o; o += v;
  w.dq = o; o += v;
  w.attn = o; o += al256(attn_ws(b, l, ND).total);
  w.total = o;
  return w;
}
}  // namespace

TMR_API size_t tmr_nlblock_saved_bytes(int b, int l) {
  if (b < 0 || l < 1) {
    tmr_set_error("tmr_nlblock_saved_bytes: bad sizes b=%d l=%d", b, l);
    return 0;
  }
  return nl_saved(b, l).total;
}
TMR_API size_t tmr_nlblock_ws_bytes(int b, int l) {
  if (b < 0 || l < 1) {
    tmr_set_error("tmr_nlblock_ws_bytes: bad sizes b=%d l=%d", b, l);
    return 0;
  }
  return nl_ws(b, l).total;
}

TMR_API int tmr_nlblock_fwd(const tmr_nlblock_weights* w, const float* st, const float* lt,
                            const int32_t* rows, int b, int l, const float* mask, float* out,
                            void* saved, size_t saved_bytes, void* ws, size_t ws_bytes,
                            hipStream_t stream) {
  TMR_CHECK_ARG(w && st && lt && out && saved && ws, "tmr_nlblock_fwd: null operand");
  TMR_CHECK_ARG(b >= 0 && l >= 1, "tmr_nlblock_fwd: bad sizes b=%d l=%d", b, l);
  const NlSaved S = nl_saved(b, l);
  const NlWs W = nl_ws(b, l);
  TMR_CHECK_ARG(saved_bytes >= S.total, "tmr_nlblock_fwd: saved buffer %zu < %zu bytes",
                saved_bytes, S.total);
  TMR_CHECK_ARG(ws_bytes >= W.total, "tmr_nlblock_fwd: workspace %zu < %zu bytes", ws_bytes,
                W.total);
  if (b == 0) return 0;
  char* sv = (char*)saved;
  float *q = (float*)(sv + S.q), *u = (float*)(sv + S.u), *p = (float*)(sv + S.p);
  float *c = (float*)(sv + S.c), *sll = (float*)(sv + S.sll), *a = (float*)(sv + S.a);
  float *mu = (float*)(sv + S.mu), *rs = (float*)(sv + S.rs);
  float* z = (float*)((char*)ws + W.dz);   // linear4 output (scratch)
  const float scale = 1.0f / sqrtf((float)ND);
  int rc;
  // q = linear1(St) (:27); u = W2^T q so that Lt_l.u = q.(W2 Lt_l) (:28-30 in GEMV form)
  if ((rc = tmr_gemm_nt(b, ND, ND, st, ND, w->w1, ND, w->b1, q, ND, 0.f, stream))) return rc;
  if ((rc = tmr_gemm_nn(b, ND, ND, q, ND, w->w2, ND, u, ND, 0.f, stream))) return rc;
  // softmax(scale * scores) over the L rows and ctx = sum_l p_l Lt_l (:31-34)
  if ((rc = tmr_nl_attn_fwd(lt, rows, u, p, c, b, l, ND, scale, (char*)ws + W.attn,
                            ws_bytes - W.attn, stream)))
    return rc;
  // SLL = linear3(ctx) (sum_l p_l = 1 carries the bias through) (:33-34)
  if ((rc = tmr_gemm_nt(b, ND, ND, c, ND, w->w3, ND, w->b3, sll, ND, 0.f, stream))) return rc;
  // LayerNorm([1,512]) + ReLU (:35-36), linear4 (:37), dropout mask + residual (:38-40)
  if ((rc = tmr_layernorm_relu_fwd(sll, w->ln_w, w->ln_b, a, mu, rs, b, ND, 1e-5f, stream)))
    return rc;
  if ((rc = tmr_gemm_nt(b, ND, ND, a, ND, w->w4, ND, w->b4, z, ND, 0.f, stream))) return rc;
  return tmr_residual_mask(st, z, mask, out, (long)b * ND, stream);
}

TMR_API int tmr_nlblock_bwd(const tmr_nlblock_weights* w, const float* dout, const float* st,
                            const float* lt, const int32_t* rows, int b, int l, const float* mask,
                            const void* saved, size_t saved_bytes, float* dst, float* dlt,
                            const tmr_nlblock_grads* g, void* ws, size_t ws_bytes,
                            hipStream_t stream) {
  TMR_CHECK_ARG(w && g && dout && st && lt && saved && ws && dst, "tmr_nlblock_bwd: null operand");
  TMR_CHECK_ARG(g->w1 && g->b1 && g->w2 && g->b2 && g->w3 && g->b3 && g->ln_w && g->ln_b && g->w4 &&
                    g->b4,
                "tmr_nlblock_bwd: null gradient");
  TMR_CHECK_ARG(b >= 0 && l >= 1, "tmr_nlblock_bwd: bad sizes b=%d l=%d", b, l);
  TMR_CHECK_ARG(!(dlt && rows), "tmr_nlblock_bwd: dLt only for a dense Lt");
  const NlSaved S = nl_saved(b, l);
  const NlWs W = nl_ws(b, l);
  TMR_CHECK_ARG(saved_bytes >= S.total, "tmr_nlblock_bwd: saved buffer %zu < %zu bytes",
                saved_bytes, S.total);
  TMR_CHECK_ARG(ws_bytes >= W.total, "tmr_nlblock_bwd: workspace %zu < %zu bytes", ws_bytes,
                W.total);
  const char* sv = (const char*)saved;
  const float *q = (const float*)(sv + S.q), *u = (const float*)(sv + S.u);
  const float *p = (const float*)(sv + S.p), *c = (const float*)(sv + S.c);
  const float *sll = (const float*)(sv + S.sll), *a = (const float*)(sv + S.a);
  const float *mu = (const float*)(sv + S.mu), *rs = (const float*)(sv + S.rs);
  char* wc = (char*)ws;
  float *dz = (float*)(wc + W.dz), *da = (float*)(wc + W.da), *dsll = (float*)(wc + W.dsll);
  float *dc = (float*)(wc + W.dc), *ut = (float*)(wc + W.ut), *dq = (float*)(wc + W.dq);
  const float scale = 1.0f / sqrtf((float)ND);
  const long n = (long)b * ND;
  int rc;
  // dropout + residual: dz = dout * mask
  if ((rc = tmr_mul(dout, mask, nullptr, dz, n, stream))) return rc;
  // linear4
  if ((rc = tmr_linear_bwd(dz, a, b, ND, ND, w->w4, da, g->w4, g->b4, 0.f, stream))) return rc;
  // LayerNorm + ReLU
  if ((rc = tmr_layernorm_relu_bwd(da, sll, a, w->ln_w, mu, rs, dsll, g->ln_w, g->ln_b, b, ND,
                                   stream)))
    return rc;
  // linear3
  if ((rc = tmr_linear_bwd(dsll, c, b, ND, ND, w->w3, dc, g->w3, g->b3, 0.f, stream))) return rc;
  // attention core: ut = dL/du (+ dLt for a dense Lt)
  if ((rc = tmr_nl_attn_bwd(lt, rows, u, p, dc, ut, dlt, b, l, ND, scale, wc + W.attn,
                            ws_bytes - W.attn, stream)))
    return rc;
  // u = W2^T q: dq = W2 ut, dW2 = q ut^T; the q.b2 score term is constant over l and cancels
  // in the softmax, so dL/db2 = 0 exactly
  if ((rc = tmr_gemm_nt(b, ND, ND, ut, ND, w->w2, ND, nullptr, dq, ND, 0.f, stream))) return rc;
  if ((rc = tmr_gemm_tn(ND, ND, b, q, ND, ut, ND, g->w2, ND, 0.f, stream))) return rc;
  if (hipMemsetAsync(g->b2, 0, ND * sizeof(float), stream) != hipSuccess) {
    tmr_set_error("tmr_nlblock_bwd: memset failed");
    return 2;
  }
  // linear1, and dSt = dout (residual) + W1^T dq
  if ((rc = tmr_mul(dout, nullptr, nullptr, dst, n, stream))) return rc;
  if ((rc = tmr_gemm_tn(ND, ND, b, dq, ND, st, ND, g->w1, ND, 0.f, stream))) return rc;
  if ((rc = tmr_col_sum(dq, b, ND, ND, g->b1, 0.f, stream))) return rc;
  return tmr_gemm_nn(b, ND, ND, dq, ND, w->w1, ND, dst, ND, 1.f, stream);
}

// ---------------------------------------------------------------- TimeConv
namespace {
constexpr int TC = 512;   // Conv1d(512, 512, k) (NLBlock_MutiConv6_3.py:46-48)
const int kTK[3] = {3, 5, 7};

tmr_conv_desc tc_desc(int b, int l, int k) {
  tmr_conv_desc d{};
  d.n = b; d.h = l; d.w = 1; d.c = TC; d.k = TC;
  d.r = k; d.s = 1; d.stride = 1; d.pad = (k - 1) / 2;
  d.ho = l; d.wo = 1; d.pad_w = 0;
  d.math = TMR_MATH_F32;
  return d;
}
struct TcWs {
  size_t y[3], wk[3], wg, total;
};
TcWs tc_ws(int b, int l) {
  TcWs w;
  size_t o = 0;
  const size_t act = al256((size_t)b * l * TC * 4);
  for (int i = 0; i < 3; ++i) { w.y[i] = o; o += act; }
  for (int i = 0; i < 3; ++i) { w.wk[i] = o; o += al256((size_t)TC * TC * kTK[i] * 4); }
  size_t g = 0;
  for (int i = 0; i < 3; ++i) {
    const tmr_conv_desc d = tc_desc(b, l, kTK[i]);
    const size_t s = tmr_conv2d_wgrad_ws_bytes(&d);
    g = s > g ? s : g;
  }
  w.wg = o; o += al256(g);
  w.total = o;
  return w;
}
}  // namespace

TMR_API size_t tmr_timeconv_saved_bytes(int b, int l) {
  if (b < 0 || l < 1) {
    tmr_set_error("tmr_timeconv_saved_bytes: bad sizes b=%d l=%d", b, l);
    return 0;
  }
  return al256((size_t)b * l * TC);
}
TMR_API size_t tmr_timeconv_ws_bytes(int b, int l) {
  if (b < 0 || l < 1) {
    tmr_set_error("tmr_timeconv_ws_bytes: bad sizes b=%d l=%d", b, l);
    return 0;
  }
  return tc_ws(b, l).total;
}

TMR_API int tmr_timeconv_fwd(const float* x, int b, int l, const float* w3, const float* b3,
                             const float* w5, const float* b5, const float* w7, const float* b7,
                             float* out, void* saved, size_t saved_bytes, void* ws,
                             size_t ws_bytes, hipStream_t stream) {
  TMR_CHECK_ARG(x && w3 && b3 && w5 && b5 && w7 && b7 && out && saved && ws,
                "tmr_timeconv_fwd: null operand");
  TMR_CHECK_ARG(b >= 0 && l >= 1, "tmr_timeconv_fwd: bad sizes b=%d l=%d", b, l);
  const TcWs W = tc_ws(b, l);
  TMR_CHECK_ARG(ws_bytes >= W.total, "tmr_timeconv_fwd: workspace %zu < %zu bytes", ws_bytes,
                W.total);
  TMR_CHECK_ARG(saved_bytes >= tmr_timeconv_saved_bytes(b, l),
                "tmr_timeconv_fwd: saved buffer %zu < %zu bytes", saved_bytes,
                tmr_timeconv_saved_bytes(b, l));
  if (b == 0) return 0;
  char* wc = (char*)ws;
  const float* ws_w[3] = {w3, w5, w7};
  const float* ws_b[3] = {b3, b5, b7};
  float* y[3];
  int rc;
  for (int i = 0; i < 3; ++i) {
    const int k = kTK[i];
    float* wk = (float*)(wc + W.wk[i]);
    y[i] = (float*)(wc + W.y[i]);
    // Conv1d weight (Cout, Cin, k) = OIHW with W = 1 -> KRSC
    if ((rc = tmr_weight_oihw_to_krsc(ws_w[i], wk, TC, TC, k, 1, TC, stream))) return rc;
    const tmr_conv_desc d = tc_desc(b, l, k);
    if ((rc = tmr_conv2d_fwd(&d, x, wk, ws_b[i], y[i], 0.f, stream))) return rc;
  }
  return tmr_timeconv_max5_fwd(x, y[0], y[1], y[2], out, (uint8_t*)saved, b, l, TC, stream);
}

TMR_API int tmr_timeconv_wgrad(const float* dy, const float* x, int b, int l, const float* w3,
                               const float* w5, const float* w7, const void* saved,
                               size_t saved_bytes, float* dx, float* dw3, float* db3, float* dw5,
                               float* db5, float* dw7, float* db7, void* ws, size_t ws_bytes,
                               hipStream_t stream) {
  TMR_CHECK_ARG(dy && x && saved && ws && dw3 && db3 && dw5 && db5 && dw7 && db7,
                "tmr_timeconv_wgrad: null operand");
  TMR_CHECK_ARG(!dx || (w3 && w5 && w7), "tmr_timeconv_wgrad: dx needs the weights");
  TMR_CHECK_ARG(b >= 0 && l >= 1, "tmr_timeconv_wgrad: bad sizes b=%d l=%d", b, l);
  const TcWs W = tc_ws(b, l);
  TMR_CHECK_ARG(ws_bytes >= W.total, "tmr_timeconv_wgrad: workspace %zu < %zu bytes", ws_bytes,
                W.total);
  TMR_CHECK_ARG(saved_bytes >= tmr_timeconv_saved_bytes(b, l),
                "tmr_timeconv_wgrad: saved buffer %zu < %zu bytes", saved_bytes,
                tmr_timeconv_saved_bytes(b, l));
  char* wc = (char*)ws;
  float* d[3];
  for (int i = 0; i < 3; ++i) d[i] = (float*)(wc + W.y[i]);
  int rc;
  // route dy through the max-of-5 (first maximum wins), identity branch into dx
  if ((rc = tmr_timeconv_max5_bwd(dy, (const uint8_t*)saved, d[0], d[1], d[2], dx, b, l, TC,
                                  stream)))
    return rc;
  const float* ws_w[3] = {w3, w5, w7};
  float* dws[3] = {dw3, dw5, dw7};
  float* dbs[3] = {db3, db5, db7};
  for (int i = 0; i < 3; ++i) {
    const int k = kTK[i];
    const tmr_conv_desc dd = tc_desc(b, l, k);
    if ((rc = tmr_conv2d_wgrad(&dd, x, d[i], dws[i], TC, 0.f, (float*)(wc + W.wg),
                               ws_bytes - W.wg, stream)))
      return rc;
    if ((rc = tmr_col_sum(d[i], b * l, TC, TC, dbs[i], 0.f, stream))) return rc;
    if (dx) {
      float* wk = (float*)(wc + W.wk[i]);
      if ((rc = tmr_weight_oihw_to_krsc(ws_w[i], wk, TC, TC, k, 1, TC, stream))) return rc;
      if ((rc = tmr_conv2d_dgrad(&dd, d[i], wk, dx, 1.f, stream))) return rc;
    }
  }
  return 0;
}

// Clip-level kernels after the frame encoder: LSTM cell (per-step path), LayerNorm+ReLU,
// LFB index/gather, dropout, cross-entropy, bias grads, SGD.  (NLBlock attention: nlblock.hip.)
//
// Reference (paths under code/):
//   LSTM            nn.LSTM(2048,512) -- Training TMRNet/train_only_non-local_pretrained.py:215,:230-233
//   NLBlock         Training TMRNet/NLBlock_MutiConv6_3.py:25-40
//   LFB gather      train_only_non-local_pretrained.py:293-311 (dict :507-511), call :707-713
//   head + loss     train_only_non-local_pretrained.py:236-239, :631, :720-721
//   SGD             torch.optim.SGD, :646-655, :725
#include "common.h"
#include "tmr.h"

namespace {
constexpr int NT = 256;

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// ---------------------------------------------------------------- LSTM cell
__global__ void lstm_cell_fwd_k(const float* __restrict__ gx, int ldgx,
                                const float* __restrict__ ghh, const float* __restrict__ cp,
                                float* __restrict__ h, int ldh, float* __restrict__ c,
                                float* __restrict__ act, int b, int hd) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= b * hd) return;
  const int bb = i / hd, j = i % hd;
  const float* g = gx + (long)bb * ldgx;
  float ai = g[j], af = g[hd + j], ag = g[2 * hd + j], ao = g[3 * hd + j];
  if (ghh) {
    const float* q = ghh + (long)bb * 4 * hd;
    ai += q[j]; af += q[hd + j]; ag += q[2 * hd + j]; ao += q[3 * hd + j];
  }
  const float ig = sigm(ai), fg = sigm(af), gg = tanhf(ag), og = sigm(ao);
  const float cprev = cp ? cp[i] : 0.f;
  const float cn = fg * cprev + ig * gg;
  c[i] = cn;
  h[(long)bb * ldh + j] = og * tanhf(cn);
  if (act) {
    float* a = act + (long)bb * 4 * hd;
    a[j] = ig; a[hd + j] = fg; a[2 * hd + j] = gg; a[3 * hd + j] = og;
  }
}

__global__ void lstm_cell_bwd_k(const float* __restrict__ dho, int lddh,
                                const float* __restrict__ dhr, const float* __restrict__ dcn,
                                const float* __restrict__ act, const float* __restrict__ c,
                                const float* __restrict__ cp, float* __restrict__ dg, int lddg,
                                float* __restrict__ dcp, int b, int hd) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= b * hd) return;
  const int bb = i / hd, j = i % hd;
  float dh = dho ? dho[(long)bb * lddh + j] : 0.f;
  if (dhr) dh += dhr[i];
  const float* a = act + (long)bb * 4 * hd;
  const float ig = a[j], fg = a[hd + j], gg = a[2 * hd + j], og = a[3 * hd + j];
  const float tc = tanhf(c[i]);
  float dc = dh * og * (1.f - tc * tc);
  if (dcn) dc += dcn[i];
  const float dor = dh * tc;
  const float cprev = cp ? cp[i] : 0.f;
  float* d = dg + (long)bb * lddg;
  d[j] = dc * gg * ig * (1.f - ig);
  d[hd + j] = dc * cprev * fg * (1.f - fg);
  d[2 * hd + j] = dc * ig * (1.f - gg * gg);
  d[3 * hd + j] = dor * og * (1.f - og);
  dcp[i] = dc * fg;
}

// ------------------------------------------------------------ LayerNorm+ReLU
// one wave per row
__global__ __launch_bounds__(NT) void ln_relu_fwd_k(const float* __restrict__ x,
                                                    const float* __restrict__ g,
                                                    const float* __restrict__ bt,
                                                    float* __restrict__ y, float* __restrict__ mean,
                                                    float* __restrict__ rstd, int rows, int D,
                                                    float eps) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* xr = x + (long)r * D;
  float s = 0.f;
  for (int c = lane; c < D; c += 64) s += xr[c];
  s = warp_sum(s);
  const float mu = s / (float)D;
  float q = 0.f;
  for (int c = lane; c < D; c += 64) {
    const float d = xr[c] - mu;
    q = fmaf(d, d, q);
  }
  q = warp_sum(q);
  const float rs = 1.0f / sqrtf(q / (float)D + eps);
  for (int c = lane; c < D; c += 64) {
    const float v = (xr[c] - mu) * rs * g[c] + bt[c];
    y[(long)r * D + c] = fmaxf(v, 0.f);
  }
  if (lane == 0) { mean[r] = mu; rstd[r] = rs; }
}

__global__ __launch_bounds__(NT) void ln_relu_bwd_k(const float* __restrict__ dy,
                                                    const float* __restrict__ x,
                                                    const float* __restrict__ y,
                                                    const float* __restrict__ g,
                                                    const float* __restrict__ mean,
                                                    const float* __restrict__ rstd,
                                                    float* __restrict__ dx, int rows, int D) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float mu = mean[r], rs = rstd[r];
  const long o = (long)r * D;
  float s1 = 0.f, s2 = 0.f;
  for (int c = lane; c < D; c += 64) {
    const float gy = y[o + c] > 0.f ? dy[o + c] : 0.f;
    const float dxh = gy * g[c];
    const float xh = (x[o + c] - mu) * rs;
    s1 += dxh;
    s2 = fmaf(dxh, xh, s2);
  }
  s1 = warp_sum(s1) / (float)D;
  s2 = warp_sum(s2) / (float)D;
  for (int c = lane; c < D; c += 64) {
    const float gy = y[o + c] > 0.f ? dy[o + c] : 0.f;
    const float dxh = gy * g[c];
    const float xh = (x[o + c] - mu) * rs;
    dx[o + c] = rs * (dxh - s1 - xh * s2);
  }
}

// per-column parameter grads (fixed row order -> deterministic)
__global__ void ln_relu_param_k(const float* __restrict__ dy, const float* __restrict__ x,
                                const float* __restrict__ y, const float* __restrict__ mean,
                                const float* __restrict__ rstd, float* __restrict__ dg,
                                float* __restrict__ db, int rows, int D) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= D) return;
  float sg = 0.f, sb = 0.f;
  for (int r = 0; r < rows; ++r) {
    const long o = (long)r * D + c;
    const float gy = y[o] > 0.f ? dy[o] : 0.f;
    sb += gy;
    sg = fmaf(gy, (x[o] - mean[r]) * rstd[r], sg);
  }
  if (dg) dg[c] = sg;
  if (db) db[c] = sb;
}

// ---------------------------------------------------------------- LFB table
__global__ void lfb_index_k(const int64_t* __restrict__ vs, int ns, const int64_t* __restrict__ st,
                            int b, int L, int32_t* __restrict__ rows) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= b * L) return;
  const int bb = i / L, k = i % L;
  long q = st[bb] - k - 1;
  if (q < 0) q = 0;
  // lower_bound(vs, q)
  int lo = 0, hi = ns;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (vs[mid] < q) lo = mid + 1;
    else hi = mid;
  }
  rows[i] = lo < ns ? lo : ns - 1;
}

__global__ void lfb_gather_k(const float* __restrict__ bank, const int32_t* __restrict__ rows,
                             float* __restrict__ out, long n, int d4) {
  const long total = n * d4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long r = i / d4;
    const int c = (int)(i % d4);
    reinterpret_cast<float4*>(out)[i] = reinterpret_cast<const float4*>(bank)[(long)rows[r] * d4 + c];
  }
}

// ------------------------------------------------------------------ dropout
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__global__ void dropout_mask_k(float* __restrict__ m, long n, float p, float keep_scale,
                               uint64_t seed, uint64_t off) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    const uint64_t h = mix64(seed * 0x9e3779b97f4a7c15ull + off + (uint64_t)i);
    const float u = (float)(h >> 40) * (1.0f / 16777216.0f);  // [0,1)
    m[i] = u >= p ? keep_scale : 0.f;
  }
}

// --------------------------------------------------------------------- loss
__global__ void ce_sum_k(const float* __restrict__ x, const int64_t* __restrict__ y,
                         const float* __restrict__ w, int b, int k, float gscale,
                         float* __restrict__ loss, float* __restrict__ dx,
                         int64_t* __restrict__ preds) {
  extern __shared__ float ls[];  // [b]
  for (int i = threadIdx.x; i < b; i += blockDim.x) {
    const float* xr = x + (long)i * k;
    float mx = xr[0];
    int am = 0;
    for (int j = 1; j < k; ++j)
      if (xr[j] > mx) { mx = xr[j]; am = j; }
    float s = 0.f;
    for (int j = 0; j < k; ++j) s += expf(xr[j] - mx);
    const float lse = mx + logf(s);
    const int lab = (int)y[i];
    const float wi = w ? w[lab] : 1.f;
    ls[i] = wi * (lse - xr[lab]);
    if (preds) preds[i] = am;
    if (dx) {
      const float inv = 1.0f / s;
      for (int j = 0; j < k; ++j) {
        const float sm = expf(xr[j] - mx) * inv;
        dx[(long)i * k + j] = gscale * wi * (sm - (j == lab ? 1.f : 0.f));
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < b; ++i) t += ls[i];
    loss[0] = t;
  }
}

// nn.Softmax over classes + torch.max(probs, 1) (eval scripts, e.g.
// eval/python/test_singlenet_phase_non-local_pretrained_2fc_copy_mutiConv6_3.py:470-473):
// one thread per clip row; argmax = first maximal logit (softmax is monotone, so the max
// probability is at the max logit; the same tie rule as ce_sum_k).
__global__ void softmax_max_k(const float* __restrict__ x, int b, int k, float* __restrict__ probs,
                              float* __restrict__ pmax, int64_t* __restrict__ preds) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= b) return;
  const float* xr = x + (long)i * k;
  float mx = xr[0];
  int am = 0;
  for (int j = 1; j < k; ++j)
    if (xr[j] > mx) { mx = xr[j]; am = j; }
  float s = 0.f;
  for (int j = 0; j < k; ++j) s += expf(xr[j] - mx);
  const float inv = 1.0f / s;
  if (probs)
    for (int j = 0; j < k; ++j) probs[(long)i * k + j] = expf(xr[j] - mx) * inv;
  if (pmax) pmax[i] = inv;   // exp(0) / s
  if (preds) preds[i] = am;
}

// ------------------------------------------------------------ column sums
// 16 columns x 16 row lanes per block: lane q sums rows q, q+16, ... (8 loads in flight), the 16
// lane sums are added in lane order (deterministic)
__global__ __launch_bounds__(256) void col_sum_k(const float* __restrict__ x, int rows, int cols,
                                                 int ld, float* __restrict__ out, float beta) {
  __shared__ float part[16][17];
  const int cl = threadIdx.x & 15, q = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  float s = 0.f;
  if (c < cols) {
    int r = q;
    for (; r + 16 * 7 < rows; r += 16 * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = x[(long)(r + 16 * u) * ld + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; r < rows; r += 16) s += x[(long)r * ld + c];
  }
  part[q][cl] = s;
  __syncthreads();
  if (q == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += part[i][cl];
    out[c] = beta != 0.f ? t + beta * out[c] : t;
  }
}

// --------------------------------------------------------------------- SGD
__global__ void sgd_k(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ buf,
                      long n, float lr, float mom, float damp, float wd, int nesterov, int first) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    const float pv = p[i];
    float d = g[i];
    if (wd != 0.f) d = d + wd * pv;
    if (mom != 0.f) {
      float bv = first ? d : mom * buf[i] + (1.f - damp) * d;
      buf[i] = bv;
      d = nesterov ? d + mom * bv : bv;
    }
    p[i] = pv - lr * d;
  }
}

// Multi-tensor SGD: one launch for every parameter of every group.  Workgroup b handles
// SGD_CHUNK elements of the tensor whose [block_begin, next block_begin) range holds b (binary
// search over the small table, read through the scalar cache).
constexpr int SGD_CHUNK = 8192;
__global__ __launch_bounds__(256) void sgd_multi_k(const tmr_sgd_tensor* __restrict__ tab, int nt,
                                                   const int32_t* __restrict__ status) {
  // a device-side failure of this step (health word) leaves the weights untouched
  if (status && *status) return;
  const long b = blockIdx.x;
  int lo = 0, hi = nt - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tab[mid].block_begin <= b) lo = mid; else hi = mid - 1;
  }
  const tmr_sgd_tensor t = tab[lo];
  const long base = (b - t.block_begin) * SGD_CHUNK;
  const long end = base + SGD_CHUNK < t.n ? base + SGD_CHUNK : t.n;
  for (long i = base + threadIdx.x; i < end; i += 256) {
    const float pv = t.p[i];
    float d = t.g[i];
    if (t.weight_decay != 0.f) d = d + t.weight_decay * pv;
    if (t.momentum != 0.f) {
      const float bv = t.first_step ? d : t.momentum * t.buf[i] + (1.f - t.dampening) * d;
      t.buf[i] = bv;
      d = t.nesterov ? d + t.momentum * bv : bv;
    }
    t.p[i] = pv - t.lr * d;
  }
}

// Multi-tensor Adam (torch.optim.Adam, amsgrad off): the table layout of SGD, moments m / v.
// Per element the arithmetic of torch's _multi_tensor_adam: lerp of m toward the gradient
// (weight 1 - beta1 < 0.5 branch), v = v * beta2 + (1 - beta2) * d * d, denom = sqrt(v) /
// sqrt(bc2) + eps, p -= step_size * m / denom (step_size = lr / bc1 from the host, in double).
__global__ __launch_bounds__(256) void adam_multi_k(const tmr_adam_tensor* __restrict__ tab, int nt,
                                                    const int32_t* __restrict__ status) {
  if (status && *status) return;
  const long b = blockIdx.x;
  int lo = 0, hi = nt - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tab[mid].block_begin <= b) lo = mid; else hi = mid - 1;
  }
  const tmr_adam_tensor t = tab[lo];
  const long base = (b - t.block_begin) * SGD_CHUNK;
  const long end = base + SGD_CHUNK < t.n ? base + SGD_CHUNK : t.n;
  const float w1 = 1.f - t.beta1, w2 = 1.f - t.beta2;
  for (long i = base + threadIdx.x; i < end; i += 256) {
    const float pv = t.p[i];
    float d = t.maximize ? -t.g[i] : t.g[i];
    if (t.weight_decay != 0.f) d = d + t.weight_decay * pv;
    const float mo = t.m[i];
    const float m = w1 < 0.5f ? mo + w1 * (d - mo) : d - (d - mo) * (1.f - w1);
    const float v = t.v[i] * t.beta2 + w2 * (d * d);
    t.m[i] = m;
    t.v[i] = v;
    const float denom = sqrtf(v) / t.bc2_sqrt + t.eps;
    t.p[i] = pv - t.step_size * (m / denom);
  }
}

int blocks_for(long n, int bs) {
  long b = (n + bs - 1) / bs;
  if (b > 8192) b = 8192;
  return (int)(b > 0 ? b : 1);
}

}  // namespace

TMR_API int tmr_lstm_cell_fwd(const float* gx, int ldgx, const float* ghh, const float* c_prev,
                              float* h_out, int ldh, float* c_out, float* act, int b, int hdim,
                              hipStream_t stream) {
  hipLaunchKernelGGL(lstm_cell_fwd_k, dim3(cdiv((long)b * hdim, NT)), dim3(NT), 0, stream, gx,
                     ldgx, ghh, c_prev, h_out, ldh, c_out, act, b, hdim);
  TMR_CHECK_LAUNCH("lstm_cell_fwd");
  return 0;
}

TMR_API int tmr_lstm_cell_bwd(const float* dh_out, int lddh, const float* dh_rec,
                              const float* dc_next, const float* act, const float* c,
                              const float* c_prev, float* dgates, int lddg, float* dc_prev, int b,
                              int hdim, hipStream_t stream) {
  hipLaunchKernelGGL(lstm_cell_bwd_k, dim3(cdiv((long)b * hdim, NT)), dim3(NT), 0, stream, dh_out,
                     lddh, dh_rec, dc_next, act, c, c_prev, dgates, lddg, dc_prev, b, hdim);
  TMR_CHECK_LAUNCH("lstm_cell_bwd");
  return 0;
}

TMR_API int tmr_layernorm_relu_fwd(const float* x, const float* gamma, const float* beta,
                                   float* y, float* mean, float* rstd, int rows, int d, float eps,
                                   hipStream_t stream) {
  hipLaunchKernelGGL(ln_relu_fwd_k, dim3(cdiv(rows, NT / 64)), dim3(NT), 0, stream, x, gamma, beta,
                     y, mean, rstd, rows, d, eps);
  TMR_CHECK_LAUNCH("layernorm_relu_fwd");
  return 0;
}

TMR_API int tmr_layernorm_relu_bwd(const float* dy, const float* x, const float* y,
                                   const float* gamma, const float* mean, const float* rstd,
                                   float* dx, float* dgamma, float* dbeta, int rows, int d,
                                   hipStream_t stream) {
  hipLaunchKernelGGL(ln_relu_bwd_k, dim3(cdiv(rows, NT / 64)), dim3(NT), 0, stream, dy, x, y, gamma,
                     mean, rstd, dx, rows, d);
  TMR_CHECK_LAUNCH("layernorm_relu_bwd");
  if (dgamma || dbeta) {
    hipLaunchKernelGGL(ln_relu_param_k, dim3(cdiv(d, 256)), dim3(256), 0, stream, dy, x, y, mean,
                       rstd, dgamma, dbeta, rows, d);
    TMR_CHECK_LAUNCH("layernorm_relu_param");
  }
  return 0;
}

TMR_API int tmr_lfb_index(const int64_t* valid_starts, int nstarts, const int64_t* clip_starts,
                          int b, int l, int32_t* rows, hipStream_t stream) {
  TMR_CHECK_ARG(nstarts > 0, "tmr_lfb_index: empty valid-start list");
  if (b * l == 0) return 0;
  hipLaunchKernelGGL(lfb_index_k, dim3(cdiv((long)b * l, NT)), dim3(NT), 0, stream, valid_starts,
                     nstarts, clip_starts, b, l, rows);
  TMR_CHECK_LAUNCH("lfb_index");
  return 0;
}

TMR_API int tmr_lfb_gather(const float* bank, const int32_t* rows, float* out, long nrows, int d,
                           hipStream_t stream) {
  TMR_CHECK_ARG(d % 4 == 0, "tmr_lfb_gather: feature dim must be a multiple of 4");
  if (nrows == 0) return 0;
  hipLaunchKernelGGL(lfb_gather_k, dim3(blocks_for(nrows * (d / 4), NT)), dim3(NT), 0, stream, bank,
                     rows, out, nrows, d / 4);
  TMR_CHECK_LAUNCH("lfb_gather");
  return 0;
}

TMR_API int tmr_dropout_mask(float* mask, long n, float p, uint64_t seed, uint64_t offset,
                             hipStream_t stream) {
  TMR_CHECK_ARG(p >= 0.f && p < 1.f, "tmr_dropout_mask: p must be in [0,1)");
  if (n == 0) return 0;
  hipLaunchKernelGGL(dropout_mask_k, dim3(blocks_for(n, NT)), dim3(NT), 0, stream, mask, n, p,
                     1.0f / (1.0f - p), seed, offset);
  TMR_CHECK_LAUNCH("dropout_mask");
  return 0;
}

TMR_API int tmr_ce_sum(const float* logits, const int64_t* labels, const float* weight, int b,
                       int k, float gscale, float* loss, float* dlogits, int64_t* preds,
                       hipStream_t stream) {
  TMR_CHECK_ARG(b >= 1 && b <= 65536 && k >= 1, "tmr_ce_sum: bad shape b=%d k=%d", b, k);
  hipLaunchKernelGGL(ce_sum_k, dim3(1), dim3(256), b * sizeof(float), stream, logits, labels,
                     weight, b, k, gscale, loss, dlogits, preds);
  TMR_CHECK_LAUNCH("ce_sum");
  return 0;
}

TMR_API int tmr_softmax_max(const float* logits, int b, int k, float* probs, float* pmax,
                            int64_t* preds, hipStream_t stream) {
  TMR_CHECK_ARG(b >= 0 && k >= 1, "tmr_softmax_max: bad shape b=%d k=%d", b, k);
  if (b == 0) return 0;
  hipLaunchKernelGGL(softmax_max_k, dim3(cdiv(b, 256)), dim3(256), 0, stream, logits, b, k, probs,
                     pmax, preds);
  TMR_CHECK_LAUNCH("softmax_max");
  return 0;
}

TMR_API int tmr_col_sum(const float* x, int rows, int cols, int ld, float* out, float beta,
                        hipStream_t stream) {
  if (cols == 0) return 0;
  hipLaunchKernelGGL(col_sum_k, dim3(cdiv(cols, 16)), dim3(256), 0, stream, x, rows, cols, ld, out,
                     beta);
  TMR_CHECK_LAUNCH("col_sum");
  return 0;
}

TMR_API int tmr_sgd_step(float* p, const float* g, float* buf, long n, float lr, float momentum,
                         float dampening, float weight_decay, int nesterov, int first_step,
                         hipStream_t stream) {
  if (n == 0) return 0;
  TMR_CHECK_ARG(momentum == 0.f || buf, "tmr_sgd_step: momentum needs a buffer");
  hipLaunchKernelGGL(sgd_k, dim3(blocks_for(n, NT)), dim3(NT), 0, stream, p, g, buf, n, lr,
                     momentum, dampening, weight_decay, nesterov, first_step);
  TMR_CHECK_LAUNCH("sgd_step");
  return 0;
}

TMR_API int64_t tmr_sgd_chunk(void) { return SGD_CHUNK; }

TMR_API int tmr_adam_step_multi(const tmr_adam_tensor* table, int ntensors, int64_t nblocks,
                                const int32_t* status, hipStream_t stream) {
  if (ntensors == 0 || nblocks == 0) return 0;
  TMR_CHECK_ARG(table && ntensors > 0 && nblocks > 0 && nblocks < (1L << 31),
                "tmr_adam_step_multi: bad table (%d tensors, %ld blocks)", ntensors, (long)nblocks);
  hipLaunchKernelGGL(adam_multi_k, dim3((unsigned)nblocks), dim3(256), 0, stream, table, ntensors,
                     status);
  TMR_CHECK_LAUNCH("adam_step_multi");
  return 0;
}

TMR_API int tmr_sgd_step_multi(const tmr_sgd_tensor* table, int ntensors, int64_t nblocks,
                               const int32_t* status, hipStream_t stream) {
  if (ntensors == 0 || nblocks == 0) return 0;
  TMR_CHECK_ARG(table && ntensors > 0 && nblocks > 0 && nblocks < (1L << 31),
                "tmr_sgd_step_multi: bad table (%d tensors, %ld blocks)", ntensors, (long)nblocks);
  hipLaunchKernelGGL(sgd_multi_k, dim3((unsigned)nblocks), dim3(256), 0, stream, table, ntensors,
                     status);
  TMR_CHECK_LAUNCH("sgd_step_multi");
  return 0;
}

// --------------------------------------------------- small elementwise glue
namespace {
__global__ void residual_mask_k(const float* __restrict__ base, const float* __restrict__ z,
                                const float* __restrict__ m, float* __restrict__ out, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    out[i] = base[i] + (m ? z[i] * m[i] : z[i]);
}
__global__ void mask_relu_fwd_k(const float* __restrict__ h, const float* __restrict__ m,
                                float* __restrict__ a, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    a[i] = fmaxf(m ? h[i] * m[i] : h[i], 0.f);
}
__global__ void mask_relu_bwd_k(const float* __restrict__ da, const float* __restrict__ a,
                                const float* __restrict__ m, float* __restrict__ dh, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    const float g = a[i] > 0.f ? da[i] : 0.f;
    dh[i] = m ? g * m[i] : g;
  }
}
__global__ void mul_k(const float* __restrict__ a, const float* __restrict__ b,
                      const float* __restrict__ s, float* __restrict__ out, long n) {
  const float sc = s ? s[0] : 1.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    out[i] = (b ? a[i] * b[i] : a[i]) * sc;
}
}  // namespace

TMR_API int tmr_residual_mask(const float* base, const float* z, const float* mask, float* out,
                              long n, hipStream_t stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(residual_mask_k, dim3(blocks_for(n, NT)), dim3(NT), 0, stream, base, z, mask,
                     out, n);
  TMR_CHECK_LAUNCH("residual_mask");
  return 0;
}
TMR_API int tmr_mask_relu_fwd(const float* h, const float* mask, float* a, long n,
                              hipStream_t stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(mask_relu_fwd_k, dim3(blocks_for(n, NT)), dim3(NT), 0, stream, h, mask, a, n);
  TMR_CHECK_LAUNCH("mask_relu_fwd");
  return 0;
}
TMR_API int tmr_mask_relu_bwd(const float* da, const float* a, const float* mask, float* dh,
                              long n, hipStream_t stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(mask_relu_bwd_k, dim3(blocks_for(n, NT)), dim3(NT), 0, stream, da, a, mask,
                     dh, n);
  TMR_CHECK_LAUNCH("mask_relu_bwd");
  return 0;
}
TMR_API int tmr_mul(const float* a, const float* b, const float* scalar, float* out, long n,
                    hipStream_t stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(mul_k, dim3(blocks_for(n, NT)), dim3(NT), 0, stream, a, b, scalar, out, n);
  TMR_CHECK_LAUNCH("mul");
  return 0;
}

// ------------------------------------------------------------ small bookkeeping kernels
namespace {
__global__ void fill_k(float* __restrict__ x, long n, float v) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    x[i] = v;
}
__global__ void counters_add_k(int64_t* const* __restrict__ ptrs, int n, int64_t v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) *ptrs[i] += v;
}
}  // namespace

// the LSTM output at the last step of each clip (y.view(-1, 512)[T-1::T]) and its gradient
namespace {
__global__ void seq_last_k(const float* __restrict__ y, float* __restrict__ out, int b, int t, int h) {
  const long n = (long)b * h;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long bb = i / h;
    out[i] = y[(bb * t + (t - 1)) * h + (i - bb * h)];
  }
}
__global__ void seq_last_bwd_k(const float* __restrict__ d1, const float* __restrict__ d2,
                               float* __restrict__ dy, int b, int t, int h) {
  const long n = (long)b * t * h;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long j = i % h, bt = i / h;
    const long bb = bt / t;
    float v = 0.f;
    if (bt - bb * t == t - 1) {
      v = d1[bb * h + j];
      if (d2) v += d2[bb * h + j];
    }
    dy[i] = v;
  }
}
}  // namespace

TMR_API int tmr_seq_last(const float* y, float* out, int b, int t, int h, hipStream_t stream) {
  TMR_CHECK_ARG(b >= 0 && t > 0 && h > 0, "tmr_seq_last: bad shape b %d t %d h %d", b, t, h);
  if (b == 0) return 0;
  hipLaunchKernelGGL(seq_last_k, dim3(blocks_for((long)b * h, NT)), dim3(NT), 0, stream, y, out, b, t, h);
  TMR_CHECK_LAUNCH("seq_last");
  return 0;
}

TMR_API int tmr_seq_last_bwd(const float* d1, const float* d2, float* dy, int b, int t, int h,
                             hipStream_t stream) {
  TMR_CHECK_ARG(b >= 0 && t > 0 && h > 0 && d1, "tmr_seq_last_bwd: bad arguments");
  if (b == 0) return 0;
  hipLaunchKernelGGL(seq_last_bwd_k, dim3(blocks_for((long)b * t * h, NT)), dim3(NT), 0, stream, d1,
                     d2, dy, b, t, h);
  TMR_CHECK_LAUNCH("seq_last_bwd");
  return 0;
}

TMR_API int tmr_fill_f32(float* x, long n, float v, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(fill_k, dim3(blocks_for(n, NT)), dim3(NT), 0, stream, x, n, v);
  TMR_CHECK_LAUNCH("fill_f32");
  return 0;
}

TMR_API int tmr_counters_add(int64_t* const* ptrs, int n, int64_t v, hipStream_t stream) {
  if (n <= 0) return 0;
  TMR_CHECK_ARG(ptrs, "tmr_counters_add: null pointer table");
  hipLaunchKernelGGL(counters_add_k, dim3(cdiv(n, NT)), dim3(NT), 0, stream, ptrs, n, v);
  TMR_CHECK_LAUNCH("counters_add");
  return 0;
}

// ------------------------------------------------------------ TimeConv max-of-5
// NLBlock_MutiConv6_3.py:52-79: y = max over (x, conv3(x), conv5(x), conv7(x),
// maxpool2(pad_left0(x))) with the first maximum winning (AdaptiveMaxPool2d / MaxPool1d
// tie rule).  code: 0 identity, 1..3 conv branches, 4 maxpool -> x[t-1] (or the zero pad).
namespace {
__global__ void max5_fwd_k(const float* __restrict__ x, const float* __restrict__ y1,
                           const float* __restrict__ y2, const float* __restrict__ y3,
                           float* __restrict__ out, uint8_t* __restrict__ code, int L, int C,
                           long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    const int t = (int)((i / C) % L);
    const float xv = x[i];
    const float prev = t > 0 ? x[i - C] : 0.f;
    // MaxPool1d(2,1) over (prev, x): first max wins -> prev on ties
    const bool mp_prev = !(xv > prev);
    const float mp = mp_prev ? prev : xv;
    float best = xv;
    uint8_t c = 0;
    const float v1 = y1[i], v2 = y2[i], v3 = y3[i];
    if (v1 > best) { best = v1; c = 1; }
    if (v2 > best) { best = v2; c = 2; }
    if (v3 > best) { best = v3; c = 3; }
    if (mp > best) { best = mp; c = mp_prev ? 4 : 0; }
    out[i] = best;
    code[i] = c;
  }
}
__global__ void max5_bwd_k(const float* __restrict__ dy, const uint8_t* __restrict__ code,
                           float* __restrict__ d1, float* __restrict__ d2, float* __restrict__ d3,
                           float* __restrict__ dx, int L, int C, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    const uint8_t c = code[i];
    const float g = dy[i];
    d1[i] = c == 1 ? g : 0.f;
    d2[i] = c == 2 ? g : 0.f;
    d3[i] = c == 3 ? g : 0.f;
    if (dx) {
      const int t = (int)((i / C) % L);
      float v = c == 0 ? g : 0.f;
      if (t + 1 < L && code[i + C] == 4) v += dy[i + C];  // maxpool of step t+1 chose x[t]
      dx[i] = v;
    }
  }
}
}  // namespace

TMR_API int tmr_timeconv_max5_fwd(const float* x, const float* y1, const float* y2,
                                  const float* y3, float* out, uint8_t* code, int b, int l, int c,
                                  hipStream_t stream) {
  const long n = (long)b * l * c;
  if (n == 0) return 0;
  hipLaunchKernelGGL(max5_fwd_k, dim3(blocks_for(n, NT)), dim3(NT), 0, stream, x, y1, y2, y3, out,
                     code, l, c, n);
  TMR_CHECK_LAUNCH("timeconv_max5_fwd");
  return 0;
}

TMR_API int tmr_timeconv_max5_bwd(const float* dy, const uint8_t* code, float* d1, float* d2,
                                  float* d3, float* dx, int b, int l, int c, hipStream_t stream) {
  const long n = (long)b * l * c;
  if (n == 0) return 0;
  hipLaunchKernelGGL(max5_bwd_k, dim3(blocks_for(n, NT)), dim3(NT), 0, stream, dy, code, d1, d2,
                     d3, dx, l, c, n);
  TMR_CHECK_LAUNCH("timeconv_max5_bwd");
  return 0;
}

// nn.LSTM(2048, 512, batch_first=True) forward and backward as C entry points
// (code/Training TMRNet/train_only_non-local_pretrained.py:215, :230-233; gate order i, f, g, o).
//
//   forward : gx = x W_ih^T + (b_ih + b_hh) for all b*t frames (one MFMA GEMM), then the t-step
//             recurrence in ONE persistent launch: every step computes the gate GEMM
//             h_{t-1} W_hh^T, sigma/tanh and the cell update without leaving the kernel.
//   backward: BPTT in one persistent launch (dh = dy_t + dg_{t+1} W_hh, gate backward, dc), then
//             one GEMM each for dW_ih, dW_hh, dx and a column sum for the biases.
//
// Persistent geometry (hidden size 512): workgroup (jx, by) owns hidden units 8*jx..8*jx+7 -- the
// 32 rows of W_hh (forward) / 32 columns of W_hh^T (backward) that feed them stay in LDS for all
// steps -- and clips 16*by..16*by+15; 64 x ceil(b/16) workgroups, one per CU.  Consecutive steps
// hand h_t (forward) / dgates_t (backward) between workgroups through HBM behind a grid barrier:
// one monotonic counter, agent-scope release before the arrival and agent-scope acquire after
// the wait (every spin bounded; a give-up sets the timeout word).  The launch is cooperative, so
// a grid that is not fully resident is refused at launch instead of deadlocking; it then falls
// back to the per-step path (one gate GEMM + one cell kernel per step).
#include "common.h"
#include "tmr.h"

namespace {

constexpr int LH = 512;        // hidden size served by the persistent kernels
constexpr int HU = 8;          // hidden units per workgroup
constexpr int NGC = 4 * HU;    // gate columns per workgroup
constexpr int BBC = 16;        // clips per workgroup
constexpr int WLD = LH + 4;    // LDS row stride of the forward W_hh slice
constexpr int CH = 512;        // backward: gate-gradient columns staged per chunk
constexpr int TLD = 4 * LH + 4;  // LDS row stride of the backward W_hh^T slice
constexpr int DLD = CH + 4;
constexpr unsigned SPIN_LIMIT = 1u << 23;   // x s_sleep(2): ~0.5 s, then give up

typedef __attribute__((address_space(1))) unsigned gu32;

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// Grid barrier number `target` / nwg.  sync[0] = arrival counter, sync[1] = timeout word; both
// zeroed by the host before every launch.  Returns false after a give-up (then every workgroup
// leaves its loop: the results are garbage and the timeout word says so).
__device__ bool grid_barrier(unsigned* sync, unsigned target) {
  gu32* cnt = (gu32*)sync;
  gu32* tmo = (gu32*)(sync + 1);
  __shared__ int ok_s;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave drains its own stores
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int ok = 1;
    unsigned spins = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > SPIN_LIMIT ||
          __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
        __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ok_s = ok;
  }
  __syncthreads();
  return ok_s != 0;
}

// ---------------------------------------------------------------- forward recurrence
// gx (b,t,4H): x W_ih^T + b_ih + b_hh.  Writes y (b,t,H) = h_t, and when given: cs (t,b,H) cell
// states, acts (t,b,4H) gate activations (i,f,g,o) for the backward, cn (b,H).
__global__ __launch_bounds__(256) void lstm_rec_fwd_k(const float* __restrict__ gx,
                                                      const float* __restrict__ whh,
                                                      float* __restrict__ y, float* __restrict__ cs,
                                                      float* __restrict__ acts,
                                                      float* __restrict__ cn, int B, int T,
                                                      unsigned* sync) {
  __shared__ __attribute__((aligned(16))) float wsl[NGC * WLD];   // W_hh rows of this slice
  __shared__ __attribute__((aligned(16))) float hs[BBC * WLD];    // h_{t-1} of this clip group
  __shared__ float gs[BBC][NGC + 1];                               // gate pre-activations
  const int tid = threadIdx.x;
  const int j0 = blockIdx.x * HU;
  const int b0 = blockIdx.y * BBC;
  const int nwg = gridDim.x * gridDim.y;
  // gate column c of this slice: gate q = c / HU, unit u = c % HU -> W_hh row q*H + j0 + u
  for (int idx = tid; idx < NGC * (LH / 4); idx += 256) {
    const int c = idx / (LH / 4), k4 = idx % (LH / 4);
    const int row = (c / HU) * LH + j0 + (c % HU);
    *reinterpret_cast<float4*>(&wsl[c * WLD + 4 * k4]) =
        *reinterpret_cast<const float4*>(&whh[(long)row * LH + 4 * k4]);
  }
  // dot-product role: clip tb, gate columns 2*tc, 2*tc+1
  const int tb = tid >> 4, tc = tid & 15;
  const int gb = b0 + tb;
  const int c0 = 2 * tc, c1 = 2 * tc + 1;
  const int gcol0 = (c0 / HU) * LH + j0 + (c0 % HU);
  const int gcol1 = (c1 / HU) * LH + j0 + (c1 % HU);
  // cell role (tid < 128): clip cb, unit cu; the cell state lives in a register for all steps
  const int cb = tid / HU, cu = tid % HU;
  const int cgb = b0 + cb, cj = j0 + cu;
  const bool cell = tid < BBC * HU && cgb < B;
  float creg = 0.f;
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    if (t > 0) {
      for (int idx = tid; idx < BBC * (LH / 4); idx += 256) {
        const int bl = idx / (LH / 4), k4 = idx % (LH / 4);
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (b0 + bl < B)
          v = *reinterpret_cast<const float4*>(&y[((long)(b0 + bl) * T + (t - 1)) * LH + 4 * k4]);
        *reinterpret_cast<float4*>(&hs[bl * WLD + 4 * k4]) = v;
      }
      __syncthreads();
    }
    float a0 = 0.f, a1 = 0.f;
    if (t > 0) {
      const float* hrow = &hs[tb * WLD];
      const float* w0 = &wsl[c0 * WLD];
      const float* w1 = &wsl[c1 * WLD];
#pragma unroll 8
      for (int k = 0; k < LH; k += 4) {
        const float4 h4 = *reinterpret_cast<const float4*>(hrow + k);
        const float4 x0 = *reinterpret_cast<const float4*>(w0 + k);
        const float4 x1 = *reinterpret_cast<const float4*>(w1 + k);
        a0 = fmaf(h4.x, x0.x, a0); a0 = fmaf(h4.y, x0.y, a0);
        a0 = fmaf(h4.z, x0.z, a0); a0 = fmaf(h4.w, x0.w, a0);
        a1 = fmaf(h4.x, x1.x, a1); a1 = fmaf(h4.y, x1.y, a1);
        a1 = fmaf(h4.z, x1.z, a1); a1 = fmaf(h4.w, x1.w, a1);
      }
    }
    if (gb < B) {
      const float* g = gx + ((long)gb * T + t) * (4 * LH);
      gs[tb][c0] = g[gcol0] + a0;
      gs[tb][c1] = g[gcol1] + a1;
    }
    __syncthreads();
    if (cell) {
      const float ig = sigm(gs[cb][cu]), fg = sigm(gs[cb][HU + cu]);
      const float gg = tanhf(gs[cb][2 * HU + cu]), og = sigm(gs[cb][3 * HU + cu]);
      creg = fg * creg + ig * gg;
      y[((long)cgb * T + t) * LH + cj] = og * tanhf(creg);
      if (cs) cs[((long)t * B + cgb) * LH + cj] = creg;
      if (acts) {
        float* a = acts + ((long)t * B + cgb) * (4 * LH);
        a[cj] = ig; a[LH + cj] = fg; a[2 * LH + cj] = gg; a[3 * LH + cj] = og;
      }
    }
    if (t + 1 < T && !grid_barrier(sync, (unsigned)((t + 1) * nwg))) return;
  }
  if (cell && cn) cn[(long)cgb * LH + cj] = creg;
}

// ---------------------------------------------------------------- backward recurrence
// dy (b,t,H): dL/dh_t from the output sequence.  Writes dg (b,t,4H) = dL/d(gate pre-activations)
// and hprev (b,t,H) = h_{t-1} (0 at t = 0), the operand of dW_hh.
__global__ __launch_bounds__(256) void lstm_rec_bwd_k(const float* __restrict__ dy,
                                                      const float* __restrict__ whh,
                                                      const float* __restrict__ y,
                                                      const float* __restrict__ cs,
                                                      const float* __restrict__ acts,
                                                      float* __restrict__ dg,
                                                      float* __restrict__ hprev, int B, int T,
                                                      unsigned* sync) {
  __shared__ __attribute__((aligned(16))) float wt[HU * TLD];     // W_hh[:, j0 + u] as rows u
  __shared__ __attribute__((aligned(16))) float ds[BBC * DLD];    // one chunk of dg_{t+1}
  __shared__ float part[BBC * HU][2];
  const int tid = threadIdx.x;
  const int j0 = blockIdx.x * HU;
  const int b0 = blockIdx.y * BBC;
  const int nwg = gridDim.x * gridDim.y;
  for (int idx = tid; idx < 4 * LH * HU; idx += 256) {
    const int c = idx / HU, u = idx % HU;
    wt[u * TLD + c] = whh[(long)c * LH + j0 + u];
  }
  // dot role: clip db, unit du, half dh of each staged chunk
  const int dhalf = tid & 1, du = (tid >> 1) & (HU - 1), db = tid >> 4;
  // cell role (tid < 128)
  const int cb = tid / HU, cu = tid % HU;
  const int cgb = b0 + cb, cj = j0 + cu;
  const bool cell = tid < BBC * HU && cgb < B;
  float dc = 0.f;
  __syncthreads();
  for (int t = T - 1; t >= 0; --t) {
    float acc = 0.f;
    if (t + 1 < T) {
      for (int cc0 = 0; cc0 < 4 * LH; cc0 += CH) {
        for (int idx = tid; idx < BBC * (CH / 4); idx += 256) {
          const int bl = idx / (CH / 4), k4 = idx % (CH / 4);
          float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
          if (b0 + bl < B)
            v = *reinterpret_cast<const float4*>(
                &dg[((long)(b0 + bl) * T + (t + 1)) * (4 * LH) + cc0 + 4 * k4]);
          *reinterpret_cast<float4*>(&ds[bl * DLD + 4 * k4]) = v;
        }
        __syncthreads();
        const float* drow = &ds[db * DLD + dhalf * (CH / 2)];
        const float* wrow = &wt[du * TLD + cc0 + dhalf * (CH / 2)];
#pragma unroll 8
        for (int k = 0; k < CH / 2; k += 4) {
          const float4 d4 = *reinterpret_cast<const float4*>(drow + k);
          const float4 w4 = *reinterpret_cast<const float4*>(wrow + k);
          acc = fmaf(d4.x, w4.x, acc); acc = fmaf(d4.y, w4.y, acc);
          acc = fmaf(d4.z, w4.z, acc); acc = fmaf(d4.w, w4.w, acc);
        }
        __syncthreads();
      }
    }
    part[db * HU + du][dhalf] = acc;
    __syncthreads();
    if (cell) {
      float dh = dy[((long)cgb * T + t) * LH + cj] + (part[tid][0] + part[tid][1]);
      const float* a = acts + ((long)t * B + cgb) * (4 * LH);
      const float ig = a[cj], fg = a[LH + cj], gg = a[2 * LH + cj], og = a[3 * LH + cj];
      const float c = cs[((long)t * B + cgb) * LH + cj];
      const float cp = t > 0 ? cs[((long)(t - 1) * B + cgb) * LH + cj] : 0.f;
      const float tc = tanhf(c);
      const float dct = dh * og * (1.f - tc * tc) + dc;
      float* d = dg + ((long)cgb * T + t) * (4 * LH);
      d[cj] = dct * gg * ig * (1.f - ig);
      d[LH + cj] = dct * cp * fg * (1.f - fg);
      d[2 * LH + cj] = dct * ig * (1.f - gg * gg);
      d[3 * LH + cj] = dh * tc * og * (1.f - og);
      dc = dct * fg;
      hprev[((long)cgb * T + t) * LH + cj] = t > 0 ? y[((long)cgb * T + (t - 1)) * LH + cj] : 0.f;
    }
    if (t > 0 && !grid_barrier(sync, (unsigned)((T - t) * nwg))) return;
  }
}

// ---------------------------------------------------------------- per-step fallback pieces
__global__ void add2_k(const float* __restrict__ a, const float* __restrict__ b,
                       float* __restrict__ o, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = a[i] + b[i];
}

__global__ void copy_hprev_k(const float* __restrict__ y, float* __restrict__ hp, int B, int T,
                             int H) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= (long)B * T * H) return;
  const int j = (int)(i % H);
  const long bt = i / H;
  const int t = (int)(bt % T);
  hp[i] = t > 0 ? y[(bt - 1) * H + j] : 0.f;
}

__global__ void copy_k(const float* __restrict__ a, float* __restrict__ o, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = a[i];
}

// TMR_LSTM_PERSIST=0 forces the per-step path (tests exercise both; read per call, no state)
bool persist_allowed() {
  const char* v = getenv("TMR_LSTM_PERSIST");
  return !(v && v[0] == '0');
}

// workspace layout (bytes, 256-aligned pieces)
struct LstmWs {
  size_t sync, bias, gx, ghh, dg, hprev, dcp, dhb, total;
};
size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
LstmWs lstm_ws(int b, int t, int i, int h) {
  (void)i;
  LstmWs w;
  size_t o = 0;
  w.sync = o; o += 256;
  w.bias = o; o += al256((size_t)4 * h * 4);
  w.gx = o; o += al256((size_t)b * t * 4 * h * 4);   // forward gx; backward dg (same size)
  w.dg = w.gx;
  w.ghh = o; o += al256((size_t)b * 4 * h * 4);       // per-step path: h W_hh^T
  w.hprev = o; o += al256((size_t)b * t * h * 4);
  w.dcp = o; o += al256((size_t)2 * b * h * 4);
  w.dhb = o; o += al256((size_t)b * h * 4);
  w.total = o;
  return w;
}

}  // namespace

TMR_API size_t tmr_lstm_saved_bytes(int b, int t, int h) {
  if (b < 0 || t < 0 || h <= 0) {
    tmr_set_error("tmr_lstm_saved_bytes: bad sizes b=%d t=%d h=%d", b, t, h);
    return 0;
  }
  return al256((size_t)t * b * h * 4) + al256((size_t)t * b * 4 * h * 4);
}

TMR_API size_t tmr_lstm_ws_bytes(int b, int t, int i, int h) {
  if (b < 0 || t < 0 || i <= 0 || h <= 0) {
    tmr_set_error("tmr_lstm_ws_bytes: bad sizes b=%d t=%d i=%d h=%d", b, t, i, h);
    return 0;
  }
  return lstm_ws(b, t, i, h).total;
}

static bool lstm_persistent_shape(int b, int h) { return h == LH && b > 0; }

TMR_API int tmr_lstm_fwd(const float* x, int b, int t, int i, int h, const float* w_ih,
                         const float* w_hh, const float* b_ih, const float* b_hh, float* y,
                         float* hn, float* cn, void* saved, size_t saved_bytes, void* ws,
                         size_t ws_bytes, hipStream_t stream) {
  TMR_CHECK_ARG(b >= 0 && t >= 0 && i > 0 && h > 0, "tmr_lstm_fwd: bad sizes b=%d t=%d i=%d h=%d",
                b, t, i, h);
  TMR_CHECK_ARG(x && w_ih && w_hh && b_ih && b_hh && y, "tmr_lstm_fwd: null operand");
  const LstmWs L = lstm_ws(b, t, i, h);
  TMR_CHECK_ARG(ws && ws_bytes >= L.total, "tmr_lstm_fwd: workspace %zu < %zu bytes", ws_bytes,
                L.total);
  float* cs = nullptr;
  float* acts = nullptr;
  if (saved) {
    TMR_CHECK_ARG(saved_bytes >= tmr_lstm_saved_bytes(b, t, h),
                  "tmr_lstm_fwd: saved buffer %zu < %zu bytes", saved_bytes,
                  tmr_lstm_saved_bytes(b, t, h));
    cs = (float*)saved;
    acts = (float*)((char*)saved + al256((size_t)t * b * h * 4));
  }
  if (b == 0 || t == 0) return 0;
  char* w = (char*)ws;
  float* bias = (float*)(w + L.bias);
  float* gx = (float*)(w + L.gx);
  hipLaunchKernelGGL(add2_k, dim3(cdiv(4 * h, 256)), dim3(256), 0, stream, b_ih, b_hh, bias, 4 * h);
  TMR_CHECK_LAUNCH("lstm bias");
  int rc = tmr_gemm_nt(b * t, 4 * h, i, x, i, w_ih, i, bias, gx, 4 * h, 0.f, stream);
  if (rc) return rc;
  if (persist_allowed() && lstm_persistent_shape(b, h)) {
    unsigned* sync = (unsigned*)(w + L.sync);
    if (hipMemsetAsync(sync, 0, 16, stream) != hipSuccess) {
      tmr_set_error("tmr_lstm_fwd: memset failed");
      return 2;
    }
    dim3 grid(LH / HU, cdiv(b, BBC));
    const float* gxc = gx;
    void* args[] = {(void*)&gxc, (void*)&w_hh, (void*)&y, (void*)&cs, (void*)&acts, (void*)&cn,
                    (void*)&b, (void*)&t, (void*)&sync};
    hipError_t e = hipLaunchCooperativeKernel((const void*)lstm_rec_fwd_k, grid, dim3(256), args,
                                              0, stream);
    if (e == hipSuccess) {
      if (hn) {
        // h_n = y[:, t-1, :]
        TMR_CHECK_ARG(hipMemcpy2DAsync(hn, (size_t)h * 4, y + (size_t)(t - 1) * h,
                                       (size_t)t * h * 4, (size_t)h * 4, b,
                                       hipMemcpyDeviceToDevice, stream) == hipSuccess,
                      "tmr_lstm_fwd: h_n copy failed");
      }
      return 0;
    }
    (void)hipGetLastError();   // not resident (cooperative check): per-step path below
  }
  // per-step path: gate GEMM + fused cell kernel per step
  float* ghh = (float*)(w + L.ghh);
  float* cbuf[2] = {(float*)(w + L.dcp), (float*)(w + L.dcp) + (size_t)b * h};
  for (int s = 0; s < t; ++s) {
    if (s > 0) {
      rc = tmr_gemm_nt(b, 4 * h, h, y + (size_t)(s - 1) * h, t * h, w_hh, h, nullptr, ghh, 4 * h,
                       0.f, stream);
      if (rc) return rc;
    }
    float* c_out = cs ? cs + (size_t)s * b * h : cbuf[s & 1];
    const float* c_prev = s == 0 ? nullptr : (cs ? cs + (size_t)(s - 1) * b * h : cbuf[(s - 1) & 1]);
    rc = tmr_lstm_cell_fwd(gx + (size_t)s * 4 * h, t * 4 * h, s > 0 ? ghh : nullptr, c_prev,
                           y + (size_t)s * h, t * h, c_out, acts ? acts + (size_t)s * b * 4 * h : nullptr,
                           b, h, stream);
    if (rc) return rc;
    if (s == t - 1 && cn) {
      hipLaunchKernelGGL(copy_k, dim3(cdiv((long)b * h, 256)), dim3(256), 0, stream, c_out, cn, b * h);
      TMR_CHECK_LAUNCH("lstm c_n");
    }
  }
  if (hn) {
    TMR_CHECK_ARG(hipMemcpy2DAsync(hn, (size_t)h * 4, y + (size_t)(t - 1) * h, (size_t)t * h * 4,
                                   (size_t)h * 4, b, hipMemcpyDeviceToDevice, stream) == hipSuccess,
                  "tmr_lstm_fwd: h_n copy failed");
  }
  return 0;
}

TMR_API int tmr_lstm_bwd(const float* dy, const float* x, int b, int t, int i, int h,
                         const float* w_ih, const float* w_hh, const float* y, const void* saved,
                         size_t saved_bytes, float* dx, float* dw_ih, float* dw_hh, float* db_ih,
                         float* db_hh, void* ws, size_t ws_bytes, hipStream_t stream) {
  TMR_CHECK_ARG(b >= 0 && t >= 0 && i > 0 && h > 0, "tmr_lstm_bwd: bad sizes b=%d t=%d i=%d h=%d",
                b, t, i, h);
  TMR_CHECK_ARG(dy && x && w_ih && w_hh && y && saved && dw_ih && dw_hh && db_ih && db_hh,
                "tmr_lstm_bwd: null operand");
  const LstmWs L = lstm_ws(b, t, i, h);
  TMR_CHECK_ARG(ws && ws_bytes >= L.total, "tmr_lstm_bwd: workspace %zu < %zu bytes", ws_bytes,
                L.total);
  TMR_CHECK_ARG(saved_bytes >= tmr_lstm_saved_bytes(b, t, h),
                "tmr_lstm_bwd: saved buffer %zu < %zu bytes", saved_bytes,
                tmr_lstm_saved_bytes(b, t, h));
  const float* cs = (const float*)saved;
  const float* acts = (const float*)((const char*)saved + al256((size_t)t * b * h * 4));
  char* w = (char*)ws;
  float* dg = (float*)(w + L.dg);
  float* hprev = (float*)(w + L.hprev);
  int rc;
  if (b == 0 || t == 0) {
    (void)hipMemsetAsync(dw_ih, 0, (size_t)4 * h * i * 4, stream);
    (void)hipMemsetAsync(dw_hh, 0, (size_t)4 * h * h * 4, stream);
    (void)hipMemsetAsync(db_ih, 0, (size_t)4 * h * 4, stream);
    (void)hipMemsetAsync(db_hh, 0, (size_t)4 * h * 4, stream);
    return 0;
  }
  bool done = false;
  if (persist_allowed() && lstm_persistent_shape(b, h)) {
    unsigned* sync = (unsigned*)(w + L.sync);
    if (hipMemsetAsync(sync, 0, 16, stream) != hipSuccess) {
      tmr_set_error("tmr_lstm_bwd: memset failed");
      return 2;
    }
    dim3 grid(LH / HU, cdiv(b, BBC));
    void* args[] = {(void*)&dy, (void*)&w_hh, (void*)&y, (void*)&cs, (void*)&acts, (void*)&dg,
                    (void*)&hprev, (void*)&b, (void*)&t, (void*)&sync};
    hipError_t e = hipLaunchCooperativeKernel((const void*)lstm_rec_bwd_k, grid, dim3(256), args,
                                              0, stream);
    if (e == hipSuccess) done = true;
    else (void)hipGetLastError();
  }
  if (!done) {
    float* dcp[2] = {(float*)(w + L.dcp), (float*)(w + L.dcp) + (size_t)b * h};
    float* dhb = (float*)(w + L.dhb);
    const float* dh_rec = nullptr;
    const float* dc_next = nullptr;
    for (int s = t - 1; s >= 0; --s) {
      rc = tmr_lstm_cell_bwd(dy + (size_t)s * h, t * h, dh_rec, dc_next, acts + (size_t)s * b * 4 * h,
                             cs + (size_t)s * b * h, s > 0 ? cs + (size_t)(s - 1) * b * h : nullptr,
                             dg + (size_t)s * 4 * h, t * 4 * h, dcp[s & 1], b, h, stream);
      if (rc) return rc;
      dc_next = dcp[s & 1];
      if (s > 0) {
        rc = tmr_gemm_nn(b, h, 4 * h, dg + (size_t)s * 4 * h, t * 4 * h, w_hh, h, dhb, h, 0.f, stream);
        if (rc) return rc;
        dh_rec = dhb;
      }
    }
    hipLaunchKernelGGL(copy_hprev_k, dim3(cdiv((long)b * t * h, 256)), dim3(256), 0, stream, y,
                       hprev, b, t, h);
    TMR_CHECK_LAUNCH("lstm hprev");
  }
  const int rows = b * t;
  rc = tmr_gemm_tn(4 * h, i, rows, dg, 4 * h, x, i, dw_ih, i, 0.f, stream);
  if (rc) return rc;
  rc = tmr_gemm_tn(4 * h, h, rows, dg, 4 * h, hprev, h, dw_hh, h, 0.f, stream);
  if (rc) return rc;
  rc = tmr_col_sum(dg, rows, 4 * h, 4 * h, db_ih, 0.f, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(copy_k, dim3(cdiv(4 * h, 256)), dim3(256), 0, stream, db_ih, db_hh, 4 * h);
  TMR_CHECK_LAUNCH("lstm db_hh");
  if (dx) {
    rc = tmr_gemm_nn(rows, i, 4 * h, dg, 4 * h, w_ih, i, dx, i, 0.f, stream);
    if (rc) return rc;
  }
  return 0;
}

// Timeout word of the last persistent launch on this workspace (0 = every grid barrier
// completed).  Read it after the stream has drained; for tests and diagnostics.
TMR_API int tmr_lstm_sync_status(const void* ws, unsigned* timeout_out, hipStream_t stream) {
  TMR_CHECK_ARG(ws && timeout_out, "tmr_lstm_sync_status: null pointer");
  unsigned v[2] = {0, 0};
  if (hipMemcpyAsync(v, ws, 8, hipMemcpyDeviceToHost, stream) != hipSuccess ||
      hipStreamSynchronize(stream) != hipSuccess) {
    tmr_set_error("tmr_lstm_sync_status: copy failed");
    return 2;
  }
  *timeout_out = v[1];
  return 0;
}

/*
 * libtmr -- MI355X (gfx950) HIP kernels for TMRNet's per-clip train-step hot path.
 *
 * Plain C ABI: raw device pointers, sizes and a hipStream_t.  The caller (the
 * Python layer in tmrnet_amd/, or any FFI) owns every buffer; the library never
 * allocates.  Every entry point returns 0 on success and non-zero on error;
 * tmr_last_error() returns a thread-local message for the last failure.
 * Entry points keep no global mutable state and enqueue only on the passed
 * stream, so they are re-entrant across threads/devices.
 *
 * Activations are NHWC fp32 ("rows x C" for per-channel ops, rows = N*H*W).
 * Conv weights are consumed in KRSC ([Cout][R][S][Cin]); gradients are written
 * in the reference's OIHW layout so they drop into torch parameters directly.
 *
 * Each entry point names the reference operation it replaces (paths relative to
 * the reference checkout's code/ directory).  The reference itself has no
 * native code: these replace the cuDNN/cuBLAS kernels that its PyTorch modules
 * reach.
 */
#ifndef TMR_H_
#define TMR_H_

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TMR_ABI_VERSION 8

int tmr_abi_version(void);
const char* tmr_last_error(void);
/* Empty the calling thread's error message (size queries report failure through it). */
void tmr_clear_error(void);

/* ---------------- convolution / GEMM (gemm_conv.hip) ----------------------
 * Replaces torchvision resnet50's nn.Conv2d fwd/bwd (cuDNN), reached from
 * `share.forward` at Training TMRNet/train_only_non-local_pretrained.py:228,
 * and the nn.Linear / nn.LSTM GEMMs of :215-239 and NLBlock_MutiConv6_3.py:27-37.
 */
typedef struct tmr_conv_desc {
  int n, h, w, c; /* input NHWC; c = stored channels (power of two >= 4) */
  int k;          /* output channels */
  int r, s, stride, pad; /* pad = padding along h */
  int ho, wo;             /* output spatial size */
  int pad_w;              /* padding along w */
  int x_ld, y_ld;         /* pixel strides (elements) of x/dx and y/dy; 0 = dense (c, k).
                             A channel slice of a wider tensor = grouped convolution. */
  int math;               /* TMR_MATH_F32: fp32 operands on v_mfma_f32_32x32x2_f32;
                             TMR_MATH_BF16: operands rounded to bf16 (RNE) when staged to LDS,
                             v_mfma_f32_32x32x16_bf16, fp32 accumulation and fp32 tensors in HBM
                             (the bf16 configs C4/C5 of BASELINE.json) */
  int max_frames;         /* frames per kernel launch, 0 = automatic.  Operands of one launch
                             must stay < 2 GiB (32-bit buffer offsets): larger batches run as
                             consecutive frame chunks (wgrad accumulates them in order) */
  int io;                 /* TMR_MATH_BF16 only: operands stored as bf16 (2-byte elements) --
                             TMR_IO_X_BF16 the input x (fwd A, wgrad B), TMR_IO_W_BF16 the KRSC
                             weights (fwd / dgrad B), TMR_IO_DY_BF16 the output gradient dy (dgrad
                             / wgrad A).  Exact: the bf16 math rounds those operands to bf16 (RNE)
                             anyway, so a tensor consumed only as a conv operand may be stored
                             rounded.  Outputs (y, dx, dw) stay fp32. */
  int groups;             /* nn.Conv2d groups (0 or 1: none).  c and k are the totals; group g reads
                             input channels [g*c/G, (g+1)*c/G) and writes [g*k/G, (g+1)*k/G), i.e.
                             the grouped 3x3 conv of ResNeSt's SplAtConv2d (radix 2,
                             train_non-local_mutiConv_resnest.py:210-220).  Weights are torch's grouped
                             layout per group block: KRSC (k, r, s, c/G), the transposed copy
                             (G, c/G, r, s, k/G), OIHW gradients (k, c_real, r, s) with c_real the real
                             input channels per group.  BatchNorm partials (stats / parts) keep rows
                             over all channels.  No operand prologues, no ReLU-mask bits. */
} tmr_conv_desc;
#define TMR_MATH_F32 0
#define TMR_MATH_BF16 1
#define TMR_IO_X_BF16 1
#define TMR_IO_W_BF16 2
#define TMR_IO_DY_BF16 4
#define TMR_IO_Y_BF16 16   /* forward: y written as bf16 (RNE); the BatchNorm partials of
                              tmr_conv2d_fwd_bnstats describe the rounded values (no beta/bias) */
#define TMR_IO_BN_BF16 32  /* tmr_conv2d_dgrad_bnbwd: the y / z of the fused BN backward are bf16 */
#define TMR_IO_G16 128     /* tmr_conv2d_dgrad_bnbwd, bf16 math on the LDS-DMA engine: dx -- the
                              ReLU-masked BN-output gradient g -- is written as bf16 (RNE) and the
                              partials describe the rounded values; c a multiple of 8 (the
                              non-residual units of the bf16 train step; tmr_bn_bwd_parts_g16
                              reads it).  With beta: the old dx is bf16 in place, or any fp32 /
                              bf16 tensor given to tmr_conv2d_dgrad_bnbwd_acc (the residual
                              stream's gradient of the bf16 train step) */
#define TMR_IO_WT_BF16 8   /* dgrad only: w is the transposed bf16 weight copy Wt[Cin][R][S][Cout]
                              (tmr_weight_oihw_to_crsk_x), read K-contiguous by the LDS-DMA engine */
#define TMR_IO_ENGINE 256  /* any math: run the implicit-GEMM engine even where a direct kernel
                              serves the geometry (the 7x7 stems, stem.hip / stem16.hip; the narrow
                              3x3 convs, direct3.hip) -- the independent second implementation the
                              tests compare those kernels with.  Changes the fp32 summation order
                              only. */
#define TMR_IO_CLASSES 512 /* dgrad, any math: a strided dgrad as one launch per stride-parity
                              class, as before round 5 -- the form the one-launch path
                              (every class's tiles in one grid) is compared with; same values */
#define TMR_IO_TILES 1024 /* fused BN-backward dgrad, any math: one output tile per workgroup (the
                              LDS-DMA engine's launch) also where the wave-specialised persistent
                              dgrad serves the shape (1x1 stride-1, round 6) -- the form that one is
                              compared with; same dx bits, partials bit-identical on 4-wave tiles */
#define TMR_IO_WT_F32 64   /* dgrad only, TMR_MATH_F32 (the io bits fp32 math takes: this one and
                              TMR_IO_ENGINE): w is the
                              transposed fp32 copy Wt[Cin][R][S][Cout] (tmr_weight_oihw_to_crsk_x,
                              out_bf16 0); the fp32 LDS-DMA engine reads it K-contiguous.  dy, dx
                              16-B aligned, Cin a multiple of 4 */

/* y[n,ho,wo,k] = beta*y + sum x * w_krsc (+ bias[k]) */
int tmr_conv2d_fwd(const tmr_conv_desc* d, const float* x, const float* w_krsc,
                   const float* bias, float* y, float beta, hipStream_t stream);
/* Inference conv + BatchNorm(running stats) [+ residual] [+ ReLU] in one launch (eval-mode
 * Bottleneck units: LFB construction, Training TMRNet/train_only_non-local_pretrained.py:570-590,
 * and the eval scripts): y = [relu](fmaf(conv(x, w_krsc), scale[k], shift[k]) + residual),
 * the same arithmetic as tmr_conv2d_fwd followed by tmr_bn_apply, without the y round trip.
 * scale/shift from tmr_bn_eval_params; residual (NHWC like y) may be NULL, must not alias y. */
int tmr_conv2d_fwd_fused(const tmr_conv_desc* d, const float* x, const float* w_krsc,
                         const float* scale, const float* shift, const float* residual, float* y,
                         int relu, hipStream_t stream);
/* Forward conv whose epilogue also emits BatchNorm batch-statistic partials of y:
 * stats = float4 [tmr_conv2d_fwd_stats_parts(d)][k] of (count, mean, M2, 0) per output-row
 * tile, consumed by tmr_bn_finalize (fuses the separate statistics pass of nn.BatchNorm2d). */
int tmr_conv2d_fwd_stats_parts(const tmr_conv_desc* d);
int tmr_conv2d_fwd_bnstats(const tmr_conv_desc* d, const float* x, const float* w_krsc, float* y,
                           void* stats, size_t stats_bytes, hipStream_t stream);
/* dx[n,h,w,c] = beta*dx + conv_transpose(dy, w_krsc) */
int tmr_conv2d_dgrad(const tmr_conv_desc* d, const float* dy, const float* w_krsc, float* dx,
                     float beta, hipStream_t stream);
/* dgrad whose epilogue also runs the first pass of the backward of the BatchNorm(+ReLU) that
 * produced this conv's input (the previous unit of the Bottleneck chain): dx receives the
 * ReLU-masked gradient (mask 1: z > 0, 2: y*scale+shift > 0, 0: none) -- i.e. the BN output
 * gradient, and for a residual unit the identity branch's gradient -- and parts the per-tile
 * column sums (sum g, sum g*(y - mean)) as float2 [tmr_conv2d_dgrad_bnbwd_parts(d)][c], finished
 * by tmr_bn_bwd_parts.  Removes the separate statistics pass over (dz, y[, z]) of tmr_bn_bwd.
 * dx, y, z dense NHWC (x_ld == c).  mask 3: z is the ReLU mask as bits (tmr_bn_apply_bits /
 * tmr_bn_apply2_bits; the LDS-DMA dgrad with transposed weights, TMR_IO_WT_F32 or TMR_IO_WT_BF16, and
 * h*w*c a multiple of 32). */
int tmr_conv2d_dgrad_bnbwd_parts(const tmr_conv_desc* d);
int tmr_conv2d_dgrad_bnbwd(const tmr_conv_desc* d, const float* dy, const float* w_krsc, float* dx,
                           float beta, const float* y, const float* z, const float* scale,
                           const float* shift, const float* mean, int mask, void* parts,
                           size_t parts_bytes, hipStream_t stream);
size_t tmr_conv2d_wgrad_ws_bytes(const tmr_conv_desc* d);
/* dw_oihw[k, c_real, r, s] = beta*dw + sum_m dy[m,k] * im2col(x)[m,(r,s,c)] */
int tmr_conv2d_wgrad(const tmr_conv_desc* d, const float* x, const float* dy, float* dw_oihw,
                     int c_real, float beta, float* ws, size_t ws_bytes, hipStream_t stream);
/* tmr_conv2d_dgrad_bnbwd with the beta operand read from dx_old (fp32, or bf16 when old_bf16)
 * instead of dx, and dx written as bf16 (TMR_IO_G16, bf16 math on the LDS-DMA engine): the
 * Bottleneck's conv1 dgrad adding into the residual stream's gradient -- the sum of the identity
 * branch and conv1 branch gradients of the block input (train_only_non-local_pretrained.py:210-213,
 * torchvision Bottleneck `out += identity`), masked by the previous block's ReLU and rounded to
 * bf16 once.  beta != 0, dx_old 16-B aligned; dx_old may equal dx (bf16 in place). */
int tmr_conv2d_dgrad_bnbwd_acc(const tmr_conv_desc* d, const float* dy, const float* w_krsc,
                               void* dx, float beta, const void* dx_old, int old_bf16,
                               const float* y, const float* z, const float* scale,
                               const float* shift, const float* mean, int mask, void* parts,
                               size_t parts_bytes, hipStream_t stream);
/* C[M][N] = beta*C + A[M][K] * B[N][K]^T (+bias) */
int tmr_gemm_nt(int M, int N, int K, const float* A, int lda, const float* B, int ldb,
                const float* bias, float* C, int ldc, float beta, hipStream_t stream);
/* C[M][N] = beta*C + A[M][K] * B[K][N] */
int tmr_gemm_nn(int M, int N, int K, const float* A, int lda, const float* B, int ldb, float* C,
                int ldc, float beta, hipStream_t stream);
/* C[M][N] = beta*C + A[K][M]^T * B[K][N] */
int tmr_gemm_tn(int M, int N, int K, const float* A, int lda, const float* B, int ldb, float* C,
                int ldc, float beta, hipStream_t stream);

/* ---------------- layout / input (pool_layout.hip) ------------------------------ */
/* OIHW -> KRSC with input channels zero-padded to cpad (torch Conv2d weight layout in) */
int tmr_weight_oihw_to_krsc(const float* w, float* wk, int k, int c, int r, int s, int cpad,
                            hipStream_t stream);
/* NCHW fp32 -> NHWC fp32 with channels zero-padded to cpad (module-boundary input, :227) */
int tmr_nchw_to_nhwc(const float* x, float* y, int n, int c, int h, int w, int cpad,
                     hipStream_t stream);
/* NHWC (c channels of cstore stored) -> NCHW */
int tmr_nhwc_to_nchw(const float* x, float* y, int n, int c, int cstore, int h, int w,
                     hipStream_t stream);
/* Per-clip RandomCrop + ToTensor + Normalize (train_only_non-local_pretrained.py:101-126,
 * :335-341): frames uint8 [F][hin][win][3], offsets int32 [F/seq][2] = (x1,y1),
 * out fp32 NHWC [F][crop][crop][4] (4th channel 0). */
int tmr_crop_normalize(const uint8_t* frames, const int32_t* offsets, float* out, int f, int hin,
                       int win, int seq_len, int crop, float m0, float m1, float m2, float s0,
                       float s1, float s2, hipStream_t stream);

/* ---------------- training augmentation (augment.hip) ----------------------
 * The reference's default per-clip training transform (use_flip = 1,
 * Training TMRNet/train_only_non-local_pretrained.py:342-350; classes :101-177):
 * RandomCrop -> ColorJitter -> RandomHorizontalFlip -> RandomRotation -> ToTensor -> Normalize,
 * bit-exact to PIL (ImageEnhance blends, L conversion, RGB<->HSV, Image.rotate NEAREST).
 * One tmr_clip_aug per FRAME (device memory), filled on the host by the reference's seeding
 * rule (tmrnet_amd/augment.py). */
typedef struct tmr_clip_aug {
  int32_t x1, y1;       /* crop offset in the input frame */
  int32_t flip;         /* horizontal flip (after the jitter) */
  int32_t rotate;       /* 1: PIL affine_fixed nearest rotation with a[] (16.16 fixed point) */
  int32_t a[6];         /* a0, a1, a2 (x origin), a3, a4, a5 (y origin) */
  int32_t jitter;       /* 1: brightness, contrast, saturation, hue */
  int32_t hue_shift;    /* uint8 shift added to the PIL HSV hue (mod 256) */
  float brightness, contrast, saturation;
  int32_t reserved;
} tmr_clip_aug;
/* frames uint8 [f][hin][win][3]; lmean int32 [f] workspace; out fp32 NHWC [f][crop][crop][4] */
int tmr_clip_augment(const uint8_t* frames, const tmr_clip_aug* params, int32_t* lmean, float* out,
                     int f, int hin, int win, int crop, float m0, float m1, float m2, float s0,
                     float s1, float s2, hipStream_t stream);

/* ---------------- batch norm + ReLU + residual (bn.hip) ---------------------
 * Replaces nn.BatchNorm2d (train mode, batch statistics, eps, momentum) + ReLU +
 * the bottleneck residual add of torchvision resnet50.  ws: double workspace of
 * tmr_bn_ws_bytes(rows, c) bytes. */
size_t tmr_bn_ws_bytes(int rows, int c);
/* batch stats of y -> save_mean, save_invstd, scale=gamma*invstd, shift=beta-mean*scale;
 * running stats updated in place (unbiased var), PyTorch semantics */
int tmr_bn_fwd_stats(const float* y, int rows, int c, const float* gamma, const float* beta,
                     float* running_mean, float* running_var, float momentum, float eps,
                     float* save_mean, float* save_invstd, float* scale, float* shift, void* ws,
                     size_t ws_bytes, hipStream_t stream);
/* combine (count, mean, M2) partials (float4 [nparts][c]) -> the outputs of tmr_bn_fwd_stats */
int tmr_bn_finalize(const void* partials, int nparts, int c, const float* gamma, const float* beta,
                    float* running_mean, float* running_var, float momentum, float eps,
                    float* save_mean, float* save_invstd, float* scale, float* shift,
                    hipStream_t stream);
/* tmr_bn_finalize with a two-level reduction (channel-group x row-slab blocks, then one thread
 * per channel adding the slabs in order; deterministic): ws >= tmr_bn_parts_ws_bytes(nparts, c) */
size_t tmr_bn_parts_ws_bytes(int nparts, int c);
int tmr_bn_finalize_ws(const void* partials, int nparts, int c, const float* gamma,
                       const float* beta, float* running_mean, float* running_var, float momentum,
                       float eps, float* save_mean, float* save_invstd, float* scale, float* shift,
                       void* ws, size_t ws_bytes, hipStream_t stream);
/* eval mode: scale/shift from running stats */
int tmr_bn_eval_params(const float* gamma, const float* beta, const float* running_mean,
                       const float* running_var, float eps, int c, float* scale, float* shift,
                       hipStream_t stream);
/* z = act(y*scale + shift (+ residual)), act = ReLU if relu */
int tmr_bn_apply(const float* y, const float* scale, const float* shift, const float* residual,
                 float* z, int rows, int c, int relu, hipStream_t stream);
/* z = act(y*scale + shift + (yr*rscale + rshift)): Bottleneck bn3 + downsample-branch BN
 * (torchvision Bottleneck.forward: out = bn3(conv3) + downsample(x); relu) with the branch's BN
 * applied on the fly -- identical to tmr_bn_apply(yr, rscale, rshift, NULL, r, 0) followed by
 * tmr_bn_apply(y, scale, shift, r, z, relu), without materialising r. */
int tmr_bn_apply2(const float* y, const float* scale, const float* shift, const float* yr,
                  const float* rscale, const float* rshift, float* z, int rows, int c, int relu,
                  hipStream_t stream);
/* backward of z = act(bn(y) (+res)): dy, optional dres (= grad at the pre-activation),
 * dgamma, dbeta.  ReLU mask: z > 0 from the saved output z when z != NULL, otherwise
 * y*scale+shift > 0 recomputed from the forward's scale/shift (valid without a residual;
 * saves one full read of z).  z/scale/shift unused when relu == 0.  dres may alias dz: the
 * first pass then overwrites dz with the masked gradient (the residual branch's gradient, in
 * place) and the second pass reads it back without re-reading the mask source. */
/* share.bn1 -> relu -> maxpool backward (:205-207) without materialising the maxpool's input
 * gradient: dz is gathered from the pooled gradient dyp (n,ho,wo,c) and argmax, masked by
 * y*scale+shift > 0 (y = the stem conv's pre-BN output (n,h,w,c)); then the BatchNorm backward
 * of tmr_bn_bwd.  ws >= tmr_bn_ws_bytes(n*h*w, c).  Same result as tmr_maxpool2d_bwd followed by
 * tmr_bn_bwd(relu=1, z=NULL). */
int tmr_bn_bwd_maxpool(const float* dyp, const uint8_t* argmax, int n, int h, int w, int ho, int wo,
                       const float* y, const float* scale, const float* shift,
                       const float* save_mean, const float* save_invstd, const float* gamma,
                       float* dy, float* dgamma, float* dbeta, int c, void* ws, size_t ws_bytes,
                       hipStream_t stream);
/* BatchNorm backward from the fused-dgrad partials: g = the already masked output gradient;
 * dy = gamma*invstd*(g - mean(g) - xhat*mean(g*xhat)); ws >= tmr_bn_parts_ws_bytes(nparts, c). */
int tmr_bn_bwd_parts(const float* g, const float* y, const void* parts, int nparts,
                     const float* save_mean, const float* save_invstd, const float* gamma,
                     float* dy, float* dgamma, float* dbeta, int rows, int c, void* ws,
                     size_t ws_bytes, hipStream_t stream);
int tmr_bn_bwd(const float* dz, const float* y, const float* z, const float* scale,
               const float* shift, const float* save_mean, const float* save_invstd,
               const float* gamma, float* dy, float* dres, float* dgamma, float* dbeta, int rows,
               int c, int relu, void* ws, size_t ws_bytes, hipStream_t stream);

/* bf16-output forms (out_bf16 = 1: the output tensor holds bf16, RNE -- the rounding the bf16
 * conv loaders apply; for tensors consumed only as bf16-math conv operands, TMR_IO_*_BF16):
 * z of a non-residual BN+ReLU (tmr_bn_apply), dy of the BatchNorm backward (tmr_bn_bwd_parts,
 * tmr_bn_bwd, tmr_bn_bwd_maxpool; dres, dgamma, dbeta stay fp32), KRSC weights. */
int tmr_bn_apply_x(const float* y, const float* scale, const float* shift, const float* residual,
                   void* z, int rows, int c, int relu, int out_bf16, hipStream_t stream);
int tmr_bn_bwd_parts_x(const float* g, const float* y, const void* parts, int nparts,
                       const float* save_mean, const float* save_invstd, const float* gamma,
                       void* dy, float* dgamma, float* dbeta, int rows, int c, void* ws,
                       size_t ws_bytes, int out_bf16, hipStream_t stream);
int tmr_bn_bwd_x(const float* dz, const float* y, const float* z, const float* scale,
                 const float* shift, const float* save_mean, const float* save_invstd,
                 const float* gamma, void* dy, float* dres, float* dgamma, float* dbeta, int rows,
                 int c, int relu, void* ws, size_t ws_bytes, int out_bf16, hipStream_t stream);
int tmr_bn_bwd_maxpool_x(const float* dyp, const uint8_t* argmax, int n, int h, int w, int ho,
                         int wo, const float* y, const float* scale, const float* shift,
                         const float* save_mean, const float* save_invstd, const float* gamma,
                         void* dy, float* dgamma, float* dbeta, int c, void* ws, size_t ws_bytes,
                         int out_bf16, hipStream_t stream);
int tmr_weight_oihw_to_krsc_x(const float* w, void* wk, int k, int c, int r, int s, int cpad,
                              int out_bf16, hipStream_t stream);
/* bf16 operands of the LDS-DMA conv engine (every operand of a bf16-math conv stored bf16):
 * the transposed weights of the dgrad view Wt[Cin][R][S][Cout] (TMR_IO_WT_BF16); a block output
 * written fp32 (identity residual, ReLU mask) AND as a bf16 copy (next convs' operand) in one pass
 * (tmr_bn_apply_dual; tmr_bn_apply2_x with z16 != NULL); the stem maxpool output as bf16 (it is
 * only a conv operand). */
int tmr_weight_oihw_to_crsk_x(const float* w, void* wt, int k, int c, int r, int s, int out_bf16,
                              hipStream_t stream);
/* Every weight layout of a train step in one launch: the table (device memory, n entries, block0
 * ascending from 0, each entry ceil(n_out / tmr_weight_layouts_epb()) blocks; total_blocks their
 * sum) lists OIHW fp32 sources and their KRSC (kind 0, channels zero-padded to cpad) or CRSK
 * (kind 1) destinations, fp32 or bf16 (RNE) -- the values of tmr_weight_oihw_to_krsc_x /
 * tmr_weight_oihw_to_crsk_x per entry (the per-conv launches of the trunk's forward, ~70 a step). */
typedef struct tmr_wlayout {
  const float* w;
  void* out;
  long long n;       /* destination elements */
  long long block0;  /* first block of this entry */
  int k, c, rs, cpad;
  int kind, bf16;
} tmr_wlayout;
int tmr_weight_layouts_epb(void);
int tmr_weight_layouts_multi(const tmr_wlayout* table, int n, int total_blocks, hipStream_t stream);
int tmr_bn_apply_dual(const float* y, const float* scale, const float* shift, const float* residual,
                      float* z, void* z16, int rows, int c, int relu, hipStream_t stream);
/* Block outputs of the fp32 train step: tmr_bn_apply (residual optional) / tmr_bn_apply2 with
 * ReLU, plus the ReLU mask as bits (element e = bit e % 32 of bits[e / 32]; ceil(rows*c/32)
 * words) for the residual-gradient dgrads (tmr_conv2d_dgrad_bnbwd mask 3): 1/32 of z's bytes. */
int tmr_bn_apply_bits(const float* y, const float* scale, const float* shift,
                      const float* residual, float* z, uint32_t* bits, int rows, int c,
                      hipStream_t stream);
int tmr_bn_apply2_bits(const float* y, const float* scale, const float* shift, const float* yr,
                       const float* rscale, const float* rshift, float* z, uint32_t* bits,
                       int rows, int c, hipStream_t stream);
int tmr_bn_apply2_x(const float* y, const float* scale, const float* shift, const float* yr,
                    const float* rscale, const float* rshift, float* z, void* z16, int rows, int c,
                    int relu, hipStream_t stream);
int tmr_maxpool2d_fwd_bn_x(const float* x, const float* scale, const float* shift, void* y,
                           uint8_t* argmax, int n, int h, int w, int c, int ho, int wo, int out_bf16,
                           hipStream_t stream);

/* bf16-activation contract of the bf16 train step (TMR_MATH_BF16; tests/test_bf16_gpu.py,
 * oracle.emulate_bf16_convs(activations=True)): every conv output y is stored rounded to bf16
 * (TMR_IO_Y_BF16; BN statistics of the rounded values), every BatchNorm(+residual)(+ReLU) output
 * z is computed in fp32 from the bf16 y / residual and stored rounded to bf16; gradients dz / dres
 * stay fp32, dy (a conv operand) bf16.  "_a16" = y, z, residual (and the stem / avgpool inputs)
 * are bf16 tensors; otherwise the arithmetic of the fp32 forms. */
int tmr_bn_apply_a16(const void* y, const float* scale, const float* shift, const void* residual,
                     void* z, int rows, int c, int relu, hipStream_t stream);
int tmr_bn_apply2_a16(const void* y, const float* scale, const float* shift, const void* yr,
                      const float* rscale, const float* rshift, void* z, int rows, int c, int relu,
                      hipStream_t stream);
/* tmr_bn_apply_bits / tmr_bn_apply2_bits for bf16 activations: z bf16 and its ReLU mask as bits
 * (taken from the rounded z, so mask 3 equals the mask-1 test z > 0) for the residual-gradient
 * dgrads of the bf16 LDS-DMA engine (TMR_IO_WT_BF16, mask 3) */
int tmr_bn_apply_bits_a16(const void* y, const float* scale, const float* shift,
                          const void* residual, void* z, uint32_t* bits, int rows, int c,
                          hipStream_t stream);
int tmr_bn_apply2_bits_a16(const void* y, const float* scale, const float* shift, const void* yr,
                           const float* rscale, const float* rshift, void* z, uint32_t* bits,
                           int rows, int c, hipStream_t stream);
int tmr_bn_bwd_a16(const float* dz, const void* y, const void* z, const float* scale,
                   const float* shift, const float* save_mean, const float* save_invstd,
                   const float* gamma, void* dy, float* dres, float* dgamma, float* dbeta, int rows,
                   int c, int relu, void* ws, size_t ws_bytes, hipStream_t stream);
int tmr_bn_bwd_parts_a16(const float* g, const void* y, const void* parts, int nparts,
                         const float* save_mean, const float* save_invstd, const float* gamma,
                         void* dy, float* dgamma, float* dbeta, int rows, int c, void* ws,
                         size_t ws_bytes, hipStream_t stream);
/* tmr_bn_bwd_parts_a16 with g stored bf16 (written by a TMR_IO_G16 dgrad); c a multiple of 8,
 * g / y / dy 16-B aligned.  Replaces the same BatchNorm2d backward as tmr_bn_bwd_parts. */
int tmr_bn_bwd_parts_g16(const void* g, const void* y, const void* parts, int nparts,
                         const float* save_mean, const float* save_invstd, const float* gamma,
                         void* dy, float* dgamma, float* dbeta, int rows, int c, void* ws,
                         size_t ws_bytes, hipStream_t stream);
/* BatchNorm2d backward (no ReLU) of the downsample branch's BN when its output gradient is the
 * bf16 residual-stream gradient (train_only_non-local_pretrained.py:210-213, the Bottleneck
 * `downsample` Sequential): dz, y, dy bf16, c a multiple of 8, 16-B aligned; ws as tmr_bn_ws_bytes */
int tmr_bn_bwd_g16(const void* dz, const void* y, const float* save_mean,
                   const float* save_invstd, const float* gamma, void* dy, float* dgamma,
                   float* dbeta, int rows, int c, void* ws, size_t ws_bytes, hipStream_t stream);
/* The BatchNorm2d backward of a downsample Bottleneck's bn3 and downsample BN together (both take
 * the gradient g of the block's pre-ReLU sum; train_only_non-local_pretrained.py:210-213 /
 * torchvision Bottleneck `out += identity`): bn3 from the fused dgrad's partials (as
 * tmr_bn_bwd_parts_x / _g16), the downsample BN from one pass over (g, y_ds) (as tmr_bn_bwd_x /
 * tmr_bn_bwd_g16), then one apply pass reading g once and writing dy (bn3) and dy_ds -- the same
 * values as the two separate calls.  bf16 = 0: g, y, y_ds, dy, dy_ds fp32; 1: all bf16 (the
 * bf16-activation step's residual gradient).  c a multiple of 8, operands 16-B aligned;
 * ws >= tmr_bn_bwd_parts_ds_ws_bytes(nparts, rows, c). */
size_t tmr_bn_bwd_parts_ds_ws_bytes(int nparts, int rows, int c);
int tmr_bn_bwd_parts_ds(const void* g, const void* y, const void* parts, int nparts,
                        const float* save_mean, const float* save_invstd, const float* gamma,
                        void* dy, float* dgamma, float* dbeta, const void* y_ds,
                        const float* save_mean_ds, const float* save_invstd_ds,
                        const float* gamma_ds, void* dy_ds, float* dgamma_ds, float* dbeta_ds,
                        int rows, int c, int bf16, void* ws, size_t ws_bytes, hipStream_t stream);
int tmr_bn_bwd_maxpool_a16(const float* dyp, const uint8_t* argmax, int n, int h, int w, int ho,
                           int wo, const void* y, const float* scale, const float* shift,
                           const float* save_mean, const float* save_invstd, const float* gamma,
                           void* dy, float* dgamma, float* dbeta, int c, void* ws, size_t ws_bytes,
                           hipStream_t stream);
int tmr_maxpool2d_fwd_bn_a16(const void* x, const float* scale, const float* shift, void* y,
                             uint8_t* argmax, int n, int h, int w, int c, int ho, int wo,
                             hipStream_t stream);
int tmr_avgpool_fwd_a16(const void* x, float* y, int n, int hw, int c, hipStream_t stream);
/* fp32 -> bf16 (RNE) copy of a tensor consumed as a bf16 conv operand (n % 8 == 0) */
int tmr_cast_f32_bf16(const float* x, void* y, long n, hipStream_t stream);
/* The stem input of the bf16 train step: NHWC4 fp32 pixels (tmr_crop_normalize / the augment
 * output, 3 colours + 0) -> NHWC8 bf16 (RNE, channels 3-7 zero), so the 7x7 stem's 16-B pieces
 * are one tap's 8 channels and the stem runs on the bf16 LDS-DMA engine.  Exact w.r.t. the
 * bf16 math, which rounds x to bf16 anyway. */
int tmr_nhwc4_to_bf16x8(const float* x4, void* y8, long npix, hipStream_t stream);

/* ---------------- input pipeline: frame resize (resize.hip) ----------------------- */
/* transforms.Resize((250,250)) of the decoded PIL frame (Training TMRNet/
 * train_only_non-local_pretrained.py:336, pil_loader :96-99) = Pillow's Image.resize(size,
 * BILINEAR), bit-exact for 8-bit RGB.  Host (no GPU): the per-axis tables of Pillow's
 * precompute_coeffs + normalize_coeffs_8bpc -- bounds [out][2] = (first input index, count),
 * k [out][ksize] 22-bit fixed point, ksize = tmr_resize_ksize(in, out).  Device: in (n, h, w, 3)
 * uint8 -> out (n, oh, ow, 3) uint8 through tmp (horizontal pass over input rows [y0, y1) -- the
 * rows the vertical pass reads: y0 = bounds_v[0], y1 = bounds_v[2*(oh-1)] + bounds_v[2*oh-1]);
 * a pass whose size does not change is skipped, as in Pillow.  Tables live in device memory. */
int tmr_resize_ksize(int in_size, int out_size);
int tmr_resize_coeffs(int in_size, int out_size, int32_t* bounds, int32_t* k, int ksize);
size_t tmr_resize_tmp_bytes(int n, int h, int w, int oh, int ow);
int tmr_resize_u8(const uint8_t* in, int n, int h, int w, uint8_t* tmp, size_t tmp_bytes,
                  uint8_t* out, int oh, int ow, const int32_t* bounds_h, const int32_t* k_h,
                  int ksize_h, const int32_t* bounds_v, const int32_t* k_v, int ksize_v, int y0,
                  int y1, hipStream_t stream);

/* ---------------- pooling (pool_layout.hip) --------------------------------------- */
/* MaxPool2d(3,2,1) of share.maxpool (train_only_non-local_pretrained.py:207), NHWC */
int tmr_maxpool2d_fwd(const float* x, float* y, uint8_t* argmax, int n, int h, int w, int c,
                      int ho, int wo, hipStream_t stream);
int tmr_maxpool2d_bwd(const float* dy, const uint8_t* argmax, float* dx, int n, int h, int w,
                      int c, int ho, int wo, hipStream_t stream);
/* share.bn1 -> share.relu -> share.maxpool (:205-207) in one pass: x is the stem conv's pre-BN
 * output, relu(x*scale + shift) is applied per loaded element (same result and argmax as
 * tmr_bn_apply + tmr_maxpool2d_fwd; the stem's 112x112x64 BN output is never written). */
int tmr_maxpool2d_fwd_bn(const float* x, const float* scale, const float* shift, float* y,
                         uint8_t* argmax, int n, int h, int w, int c, int ho, int wo,
                         hipStream_t stream);
/* AdaptiveAvgPool2d(1) of share.avgpool (:214): x [n][hw][c] -> y [n][c] */
int tmr_avgpool_fwd(const float* x, float* y, int n, int hw, int c, hipStream_t stream);
int tmr_avgpool_bwd(const float* dy, float* dx, int n, int hw, int c, hipStream_t stream);

/* ---------------- ResNeSt-50 blocks (resnest.hip) --------------------------
 * SplAtConv2d (radix 2, cardinality 1) of the resnest50() trunk used at
 * Training TMRNet/train_non-local_mutiConv_resnest.py:210-220.  x: [n][hw][2c] (after the
 * grouped conv + bn0 + ReLU), z: fc2 logits [n][2c], att: r-softmax [n][2c]. */
/* gap[n][c] = mean_hw(x[:, :, c] + x[:, :, c+C]) */
int tmr_splat_gap(const float* x, float* gap, int n, int hw, int c, hipStream_t stream);
/* att = softmax over the radix pair of z; out[n,hw,c] = att0*x0 + att1*x1 (att may be NULL) */
int tmr_splat_combine(const float* x, const float* z, float* att, float* out, int n, int hw, int c,
                      hipStream_t stream);
/* dz = softmax-backward of (sum_hw dout * x_r) */
int tmr_splat_bwd(const float* dout, const float* x, const float* att, float* dz, int n, int hw,
                  int c, hipStream_t stream);
/* dx[n,hw,r*C+c] = att_r*dout[n,hw,c] + dgap[n][c]/hw */
int tmr_splat_bwd_apply(const float* dout, const float* att, const float* dgap, float* dx, int n,
                        int hw, int c, hipStream_t stream);
/* center[j] = mean_i x[i][j] (double accumulation); xc[i][j] = x[i][j] - center[j].
 * The fc1 -> BatchNorm of SplAtConv2d runs on centered GAP rows: BN removes any per-channel
 * constant exactly, and the GAP rows of a batch agree to ~1%, so centering first keeps fp32
 * rounding relative to the batch spread instead of the magnitude. */
int tmr_center_cols(const float* x, int rows, int cols, float* center, float* xc,
                    hipStream_t stream);
/* y[i] += alpha * x[i] */
int tmr_axpy(int n, float alpha, const float* x, float* y, hipStream_t stream);
/* AvgPool2d(k, s, p) NHWC; divisor k*k (count_include_pad) or the number of valid cells */
int tmr_avgpool2d_fwd(const float* x, float* y, int n, int h, int w, int c, int ho, int wo, int k,
                      int s, int p, int count_include_pad, hipStream_t stream);
int tmr_avgpool2d_bwd(const float* dy, float* dx, int n, int h, int w, int c, int ho, int wo, int k,
                      int s, int p, int count_include_pad, hipStream_t stream);

/* Split attention with bn0 + ReLU applied on load (the whole-trunk ResNeSt train step): y is the
 * grouped conv's pre-BN output [n][hw][2c] (bf16 when act16, else fp32) and
 * x_r = relu(y_r*scale + shift) -- rounded to bf16 under act16, the value a stored bf16 activation
 * would hold -- is recomputed wherever it is read, so the post-BN tensor is never written.
 *   gap_bn:   gap[n][c] = mean_hw(x_0 + x_1)
 *   att:      att[n][r*c+j] = softmax over the radix pair of the fc2 logits zl [n][2c]
 *   combine_bn: out[n,hw,j] = att_0*x_0 + att_1*x_1 (out bf16 when act16)
 *   bwd_reduce_bn: per (frame, channel) over hw -- dzl (softmax backward of sum_hw dout*x_r) and
 *             sums float [4][n][2c] = (sum m*dout, sum m, sum m*dout*(y-mean), sum m*(y-mean)),
 *             m the ReLU mask; the bn0 input gradient g = m*(att*dout + dgap/hw) is known only after
 *             the fc backward, and its BatchNorm sums are linear in these.
 *   bn0_coefs: the BatchNorm sums of g from sums/att/dgap (frames in order) -> dgamma, dbeta and
 *             coef [3][2c] with dy = coef0*(g - coef1 - (y - mean)*coef2)
 *   bwd_apply_bn: dy[n,hw,j] (bf16 when act16: a conv operand) from dout, y, att, dgap, coef. */
int tmr_splat_gap_bn(const void* y, const float* scale, const float* shift, float* gap, int n,
                     int hw, int c, int act16, hipStream_t stream);
int tmr_splat_att(const float* zl, float* att, int n, int c, hipStream_t stream);
int tmr_splat_combine_bn(const void* y, const float* scale, const float* shift, const float* att,
                         void* out, int n, int hw, int c, int act16, hipStream_t stream);
int tmr_splat_bwd_reduce_bn(const float* dout, const void* y, const float* scale,
                            const float* shift, const float* mean, const float* att, float* dzl,
                            float* sums, int n, int hw, int c, int act16, hipStream_t stream);
int tmr_splat_bn0_coefs(const float* att, const float* dgap, const float* sums, const float* mean,
                        const float* invstd, const float* gamma, float* coef, float* dgamma,
                        float* dbeta, int n, int hw, int c, hipStream_t stream);
int tmr_splat_bwd_apply_bn(const float* dout, const void* y, const float* scale,
                           const float* shift, const float* mean, const float* att,
                           const float* dgap, const float* coef, void* dy, int n, int hw, int c,
                           int act16, hipStream_t stream);
/* tmr_avgpool2d_fwd on bf16 activations: fp32 sums of the bf16 inputs, the output rounded */
int tmr_avgpool2d_fwd_a16(const void* x, void* y, int n, int h, int w, int c, int ho, int wo,
                          int k, int s, int p, int count_include_pad, hipStream_t stream);

/* ---------------- misc (head.hip) ------------------------------------------ */
/* out[j] = beta*out[j] + sum_i x[i*ld + j]   (Linear bias grads) */
int tmr_col_sum(const float* x, int rows, int cols, int ld, float* out, float beta,
                hipStream_t stream);
/* y = x * mask (mask already scaled by 1/(1-p)); mask from counter-based RNG */
int tmr_dropout_mask(float* mask, long n, float p, uint64_t seed, uint64_t offset,
                     hipStream_t stream);
/* CrossEntropyLoss(reduction='sum', weight) fwd+bwd, train_only_non-local_pretrained.py:631,
 * :720-721: loss[0] = sum_b w[y_b]*(lse_b - x_b[y_b]); dlogits = gscale*w[y_b]*(softmax-onehot);
 * preds = argmax (torch.max tie rule: first). weight may be NULL. */
int tmr_ce_sum(const float* logits, const int64_t* labels, const float* weight, int b, int k,
               float gscale, float* loss, float* dlogits, int64_t* preds, hipStream_t stream);
/* Eval head: probs = nn.Softmax(dim=1)(logits), (pmax, preds) = torch.max(probs, 1)
 * (eval/python/test_singlenet_phase_non-local_pretrained_2fc_copy_mutiConv6_3.py:470-473).
 * Any output pointer may be NULL. */
int tmr_softmax_max(const float* logits, int b, int k, float* probs, float* pmax, int64_t* preds,
                    hipStream_t stream);
/* torch.optim.SGD step (momentum, dampening, weight_decay, nesterov), :725 */
int tmr_sgd_step(float* p, const float* g, float* buf, long n, float lr, float momentum,
                 float dampening, float weight_decay, int nesterov, int first_step,
                 hipStream_t stream);
/* Multi-tensor SGD: every (param, grad, momentum buffer) of every param group in ONE launch
 * (optimizer.step() of :725 over the groups of :646-655).  table: DEVICE array of ntensors
 * entries; entry t covers workgroups [block_begin_t, block_begin_{t+1}), i.e. block_begin is the
 * prefix sum of ceil(n / tmr_sgd_chunk()) and nblocks the total.  status: the device health
 * word (tmrnet_amd/health.py) or NULL; when it is non-zero at launch time (a device-side failure
 * earlier in this step, e.g. a persistent LSTM that gave up a grid barrier) no weight changes. */
typedef struct tmr_sgd_tensor {
  float* p;
  const float* g;
  float* buf;           /* NULL when momentum == 0 */
  int64_t n;
  int64_t block_begin;
  float lr, momentum, dampening, weight_decay;
  int32_t nesterov, first_step;
} tmr_sgd_tensor;
int64_t tmr_sgd_chunk(void);
int tmr_sgd_step_multi(const tmr_sgd_tensor* table, int ntensors, int64_t nblocks,
                       const int32_t* status, hipStream_t stream);
/* Multi-tensor torch.optim.Adam step (the -o 1 optimizer, train_only_non-local_pretrained.py:644-645,
 * code/models.py:63-68; amsgrad off): same table scheme as tmr_sgd_step_multi (chunks of
 * tmr_sgd_chunk()), per tensor the moments m / v and the host-computed step_size = lr / (1 -
 * beta1^step), bc2_sqrt = sqrt(1 - beta2^step); status as for tmr_sgd_step_multi. */
typedef struct tmr_adam_tensor {
  float* p;
  const float* g;
  float* m;
  float* v;
  int64_t n;
  int64_t block_begin;
  float beta1, beta2, eps, weight_decay, step_size, bc2_sqrt;
  int32_t maximize, reserved;
} tmr_adam_tensor;
int tmr_adam_step_multi(const tmr_adam_tensor* table, int ntensors, int64_t nblocks,
                        const int32_t* status, hipStream_t stream);
/* LFB row table of get_long_feature (train_only_non-local_pretrained.py:293-311):
 * rows[b][k] = index of the first valid start >= max(start_b - k - 1, 0) in the sorted
 * valid-start list (== the reference's dict walk, incl. own-row fallback and
 * cross-video reuse). */
int tmr_lfb_index(const int64_t* valid_starts, int nstarts, const int64_t* clip_starts, int b,
                  int l, int32_t* rows, hipStream_t stream);
/* out[i][:] = bank[rows[i]][:]  (the (B,L,512) long_feature tensor of :713) */
int tmr_lfb_gather(const float* bank, const int32_t* rows, float* out, long nrows, int d,
                   hipStream_t stream);
/* LayerNorm over the last dim (NLBlock layer_norm, NLBlock_MutiConv6_3.py:17,:35) + ReLU */
int tmr_layernorm_relu_fwd(const float* x, const float* gamma, const float* beta, float* y,
                           float* mean, float* rstd, int rows, int d, float eps,
                           hipStream_t stream);
int tmr_layernorm_relu_bwd(const float* dy, const float* x, const float* y, const float* gamma,
                           const float* mean, const float* rstd, float* dx, float* dgamma,
                           float* dbeta, int rows, int d, hipStream_t stream);

/* elementwise glue of the clip head (train_only_non-local_pretrained.py:236-239,
 * NLBlock_MutiConv6_3.py:38-40) */
/* out = base + z*mask (mask NULL: base + z) -- NLBlock dropout + residual */
int tmr_residual_mask(const float* base, const float* z, const float* mask, float* out, long n,
                      hipStream_t stream);
/* a = relu(h*mask) -- head dropout(0.5) then F.relu */
int tmr_mask_relu_fwd(const float* h, const float* mask, float* a, long n, hipStream_t stream);
int tmr_mask_relu_bwd(const float* da, const float* a, const float* mask, float* dh, long n,
                      hipStream_t stream);
/* The LSTM output of each clip's last step, y.contiguous().view(-1, 512)[T-1::T]
 * (train_only_non-local_pretrained.py:232): out (b, h) from y (b, t, h); and its backward for a
 * tensor read by two consumers (the NLBlock query and the head, :235-236): dy (b, t, h) = d1 + d2
 * at step t-1 (d2 may be NULL), 0 elsewhere -- one pass, no separate zero fill or add. */
int tmr_seq_last(const float* y, float* out, int b, int t, int h, hipStream_t stream);
int tmr_seq_last_bwd(const float* d1, const float* d2, float* dy, int b, int t, int h,
                     hipStream_t stream);
/* x[i] = v (the exactly-zero fc1 bias gradient of the split attention) */
int tmr_fill_f32(float* x, long n, float v, hipStream_t stream);
/* *ptrs[i] += v for i < n: every BatchNorm num_batches_tracked counter of a train step
 * (nn.BatchNorm2d's `num_batches_tracked += 1`) in one launch; ptrs is a DEVICE array */
int tmr_counters_add(int64_t* const* ptrs, int n, int64_t v, hipStream_t stream);
/* out = a*b*scalar[0] (b, scalar may be NULL) */
int tmr_mul(const float* a, const float* b, const float* scalar, float* out, long n,
            hipStream_t stream);

/* ---------------- NLBlock attention core (nlblock.hip) ----------------------
 * NLBlock_MutiConv6_3.py:28-34 in GEMV form.  With q = linear1(St) and
 * u = W2^T q, the reference scores q.(W2 Lt_l + b2) equal Lt_l.u + q.b2; the
 * q.b2 term is constant over l and cancels in the softmax, so
 *   p_l = softmax_l(scale * Lt_l . u),  ctx = sum_l p_l Lt_l,
 * and SLL = linear3 applied to ctx (sum_l p_l = 1).  Lt rows come either from a
 * dense (B,L,D) tensor (rows == NULL) or straight from the resident LFB bank via
 * the row table (lt = bank, rows = tmr_lfb_index output).  Each clip's L rows are
 * split over 32-row workgroups (one read of Lt per pass) and combined in a fixed
 * order.  d = 256, 512 or 1024; ws >= tmr_nl_attn_ws_bytes(b, l, d). */
size_t tmr_nl_attn_ws_bytes(int b, int l, int d);
int tmr_nl_attn_fwd(const float* lt, const int32_t* rows, const float* u, float* p, float* ctx,
                    int b, int l, int d, float scale, void* ws, size_t ws_bytes,
                    hipStream_t stream);
/* given dctx: dp_l = dctx.Lt_l; ds_l = scale*p_l*(dp_l - sum_k p_k dp_k);
 * ut = sum_l ds_l Lt_l (= dL/du); dlt (optional, dense Lt only) = p_l*dctx + ds_l*u */
int tmr_nl_attn_bwd(const float* lt, const int32_t* rows, const float* u, const float* p,
                    const float* dctx, float* ut, float* dlt, int b, int l, int d, float scale,
                    void* ws, size_t ws_bytes, hipStream_t stream);

/* ---------------- module-level entry points (nlblock.hip, lstm.hip) ---------
 * The reference's module ops as single C calls, for callers without Python.
 * "saved" buffers carry what the forward keeps for the backward (caller-owned, opaque, sized by
 * the *_saved_bytes query); "ws" is scratch (*_ws_bytes).  Weights/grads in the reference's
 * torch layouts (nn.Linear (out, in), nn.Conv1d (out, in, k), nn.LSTM (4H, I) / (4H, H)). */

/* nn.Linear (train_only_non-local_pretrained.py:216-217, NLBlock_MutiConv6_3.py:13-16):
 * y = x W^T + b (bias may be NULL); backward dx = dy W, dw = beta*dw + dy^T x,
 * db = beta*db + colsum(dy); dx / dw / db may each be NULL. */
int tmr_linear_fwd(const float* x, int rows, int in, int out, const float* w, const float* bias,
                   float* y, hipStream_t stream);
int tmr_linear_bwd(const float* dy, const float* x, int rows, int in, int out, const float* w,
                   float* dx, float* dw, float* db, float beta, hipStream_t stream);

/* NLBlock(512) forward/backward (NLBlock_MutiConv6_3.py:10-40; called at
 * train_only_non-local_pretrained.py:235).  St (b,512), Lt dense (b,l,512) or bank rows
 * (lt = bank, rows = (b,l) int32), mask = the Dropout(0.2) mask already scaled by 1/0.8 (NULL in
 * eval).  out = St + dropout(linear4(relu(LN(linear3(attn(St, Lt)))))).  The backward writes
 * dSt, every parameter gradient (dL/db2 = 0 exactly: q.b2 cancels in the softmax) and, for a
 * dense Lt only, dLt (may be NULL). */
typedef struct tmr_nlblock_weights {
  const float *w1, *b1, *w2, *b2, *w3, *b3, *ln_w, *ln_b, *w4, *b4;
} tmr_nlblock_weights;
typedef struct tmr_nlblock_grads {
  float *w1, *b1, *w2, *b2, *w3, *b3, *ln_w, *ln_b, *w4, *b4;
} tmr_nlblock_grads;
size_t tmr_nlblock_saved_bytes(int b, int l);
size_t tmr_nlblock_ws_bytes(int b, int l);
int tmr_nlblock_fwd(const tmr_nlblock_weights* w, const float* st, const float* lt,
                    const int32_t* rows, int b, int l, const float* mask, float* out, void* saved,
                    size_t saved_bytes, void* ws, size_t ws_bytes, hipStream_t stream);
int tmr_nlblock_bwd(const tmr_nlblock_weights* w, const float* dout, const float* st,
                    const float* lt, const int32_t* rows, int b, int l, const float* mask,
                    const void* saved, size_t saved_bytes, float* dst, float* dlt,
                    const tmr_nlblock_grads* g, void* ws, size_t ws_bytes, hipStream_t stream);

/* TimeConv forward / weight gradient (NLBlock_MutiConv6_3.py:43-79, any L; called at
 * train_non-local_mutiConv_resnet.py:246): x (b,l,512) -> max(x, conv3, conv5, conv7,
 * maxpool2(pad_left0 x)); weights Conv1d (512,512,k) + bias for k = 3, 5, 7.  The backward writes
 * the six parameter gradients and, when dx != NULL, dL/dx (the reference never needs it: the LFB
 * is constant). */
size_t tmr_timeconv_saved_bytes(int b, int l);
size_t tmr_timeconv_ws_bytes(int b, int l);
int tmr_timeconv_fwd(const float* x, int b, int l, const float* w3, const float* b3,
                     const float* w5, const float* b5, const float* w7, const float* b7,
                     float* out, void* saved, size_t saved_bytes, void* ws, size_t ws_bytes,
                     hipStream_t stream);
int tmr_timeconv_wgrad(const float* dy, const float* x, int b, int l, const float* w3,
                       const float* w5, const float* w7, const void* saved, size_t saved_bytes,
                       float* dx, float* dw3, float* db3, float* dw5, float* db5, float* dw7,
                       float* db7, void* ws, size_t ws_bytes, hipStream_t stream);

/* nn.LSTM(i, h, batch_first=True) forward / BPTT (train_only_non-local_pretrained.py:215,
 * :230-231; gates i,f,g,o).  x (b,t,i) -> y (b,t,h); hn, cn (b,h) may be NULL; saved NULL =
 * inference.  Forward: x W_ih^T + b_ih + b_hh for all b*t frames in one GEMM, then the t-step
 * recurrence (gate GEMM h W_hh^T + sigma/tanh + cell update) in ONE persistent launch with grid
 * barriers (h = 512; per-step launches otherwise, or when the grid could not be resident at
 * once).  The backward likewise runs BPTT in one launch, then dW_ih, dW_hh, dx (may be NULL) as
 * GEMMs and db_ih = db_hh = colsum(dgates).  dy = dL/dy for every step (zeros where unused).
 * Shared device: if a barrier gives up (another stream or process held CUs, so the grid was not
 * resident in time), the next launch on the stream recomputes the recurrence in barrier-free
 * workgroups with the same arithmetic (same bits) and marks the word "recovered" (2); in a
 * normal step that launch exits at once.  TMR_LSTM_RECOVER=0 (env, test hook) skips it. */
size_t tmr_lstm_saved_bytes(int b, int t, int h);
size_t tmr_lstm_ws_bytes(int b, int t, int i, int h);
int tmr_lstm_fwd(const float* x, int b, int t, int i, int h, const float* w_ih,
                 const float* w_hh, const float* b_ih, const float* b_hh, float* y, float* hn,
                 float* cn, void* saved, size_t saved_bytes, void* ws, size_t ws_bytes,
                 hipStream_t stream);
int tmr_lstm_bwd(const float* dy, const float* x, int b, int t, int i, int h, const float* w_ih,
                 const float* w_hh, const float* y, const void* saved, size_t saved_bytes,
                 float* dx, float* dw_ih, float* dw_hh, float* db_ih, float* db_hh, void* ws,
                 size_t ws_bytes, hipStream_t stream);
/* timeout word of the last persistent LSTM launch on ws (0 = every grid barrier completed,
 * 1 = a barrier gave up and the results are invalid, 2 = gave up and recomputed);
 * synchronises the stream */
int tmr_lstm_sync_status(const void* ws, unsigned* timeout_out, hipStream_t stream);
/* *status |= 1 when the last persistent LSTM launch on ws gave up a grid barrier and was not
 * recomputed (its results are then invalid); enqueued on the stream, no synchronisation -- the
 * caller reads the status word once per train step (tmrnet_amd/health.py) and raises.
 * TMR_LSTM_SPIN_LIMIT (env) overrides the barrier's spin limit (tests force a give-up with it). */
int tmr_lstm_status_or(const void* ws, int32_t* status, hipStream_t stream);
/* Test instrumentation: `wgs` workgroups of 1024 threads that sleep about `ms` milliseconds on
 * `stream` (every wave leaves after a bounded sleep count), to hold wave slots while another
 * stream launches work -- the persistent LSTM next to a resident kernel (no reference
 * counterpart). */
int tmr_test_hold_cus(int wgs, float ms, hipStream_t stream);
/* Test instrumentation: the wave-specialised fused BN-backward dgrads this process has launched
 * (gemm16_ws.h: the 1x1 stride-1 dgrads of the train step, round 6), so a test can tell which
 * kernel served a call (its results equal the one-tile-per-workgroup launch's; no reference
 * counterpart). */
long tmr_dgrad_ws_launches(void);

/* TimeConv (NLBlock_MutiConv6_3.py:43-79, generalised in L): the three Conv1d branches run
 * on tmr_conv2d_* (L as H, W=1); these kernels take the elementwise max of
 * (x, conv3, conv5, conv7, maxpool2(pad_left0(x))) with the reference's first-max tie rule,
 * and route the gradient back.  code: uint8 [b][l][c]. */
int tmr_timeconv_max5_fwd(const float* x, const float* y1, const float* y2, const float* y3,
                          float* out, uint8_t* code, int b, int l, int c, hipStream_t stream);
int tmr_timeconv_max5_bwd(const float* dy, const uint8_t* code, float* d1, float* d2, float* d3,
                          float* dx, int b, int l, int c, hipStream_t stream);

/* ---------------- LSTM cell (head.hip; the per-step path of tmr_lstm_fwd/bwd) --
 * nn.LSTM(2048,512) gates in PyTorch order i,f,g,o (train_only_non-local_pretrained.py:215,
 * :230-231).  gx: x W_ih^T + b_ih + b_hh for step t (row stride ldgx); ghh: h_{t-1} W_hh^T
 * (NULL at t=0); c_prev NULL at t=0.  act saves (i,f,g,o) activations [b][4h] for the
 * backward (NULL: inference, nothing saved). */
int tmr_lstm_cell_fwd(const float* gx, int ldgx, const float* ghh, const float* c_prev,
                      float* h_out, int ldh, float* c_out, float* act, int b, int hdim,
                      hipStream_t stream);
/* dh = dh_out (row stride lddh) + dh_rec (NULL ok); dc_next (NULL at t=T-1);
 * writes dgates (pre-activation, row stride lddg) and dc_prev. */
int tmr_lstm_cell_bwd(const float* dh_out, int lddh, const float* dh_rec, const float* dc_next,
                      const float* act, const float* c, const float* c_prev, float* dgates,
                      int lddg, float* dc_prev, int b, int hdim, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* TMR_H_ */

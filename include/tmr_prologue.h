/*
 * libtmr operand prologues -- a retired A/B experiment, exported only by an A/B build
 * (`make PROLOGUES=1` -> tmrnet_amd/libtmr_pro.so; the default libtmr.so has none of these
 * symbols).  The trunk reaches it with TMR_FOLD_BN=1 TMR_LIB_PATH=tmrnet_amd/libtmr_pro.so.
 *
 * Bit-identical to the explicit BatchNorm passes but measured slower on both conv engines: the
 * register-staged engine C2 210 vs 181 ms/step (round 2, profiles/r2/convbench_fold/) and the fp32
 * LDS-DMA engine 3312 vs 3680 frames/s (round 4, profiles/r4/fold_ab/) -- the per-element
 * transform costs the MFMA-bound fp32 GEMMs more than the HBM-bound passes it removes.
 */
#ifndef TMR_PROLOGUE_H_
#define TMR_PROLOGUE_H_

#include "tmr.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Operand prologues: the BatchNorm around a conv applied while its operands are loaded, so the
 * tensors it would produce are never written to HBM.
 *   x_scale/x_shift: the X operand (forward input, wgrad input) is read as
 *     relu(x * x_scale[c] + x_shift[c]), and as 0 at the zero padding -- the train-mode
 *     BatchNorm + ReLU of the Bottleneck unit that produced x (torchvision Bottleneck bn1/bn2 +
 *     relu, train_only_non-local_pretrained.py:210-213), whose output z = relu(bn(y)) then never
 *     exists: the consumer conv reads y.  Identical values to tmr_bn_apply(y, ..., relu = 1).
 *   dy_y/dy_coef: the dY operand (dgrad and wgrad output gradient) is read as
 *     A[k]*g + B[k]*y + C[k] (fmaf(A, g, fmaf(B, y, C))) -- with bf16 math on the LDS-DMA engine
 *     g and y are bf16 (dY's element type) and the result is rounded RNE, as
 *     tmr_bn_bwd_parts_g16 stores dy --, g = the ReLU-masked gradient at this
 *     conv's BatchNorm output, y = this conv's pre-BN output, coef = [3][k] from
 *     tmr_bn_bwd_coefs(_dense) -- the BatchNorm backward, whose dy then never exists.  Identical
 *     values to the apply pass of tmr_bn_bwd_parts.
 * Either half may be NULL; dense NHWC operands only (x_ld == c, y_ld == k). */
typedef struct tmr_conv_prologue {
  const float* x_scale;
  const float* x_shift;
  const float* dy_y;
  const float* dy_coef;
} tmr_conv_prologue;
int tmr_conv2d_fwd_bnstats_pro(const tmr_conv_desc* d, const float* x, const float* w_krsc,
                               float* y, void* stats, size_t stats_bytes,
                               const tmr_conv_prologue* pro, hipStream_t stream);
int tmr_conv2d_dgrad_pro(const tmr_conv_desc* d, const float* dy, const float* w_krsc, float* dx,
                         float beta, const tmr_conv_prologue* pro, hipStream_t stream);
int tmr_conv2d_dgrad_bnbwd_pro(const tmr_conv_desc* d, const float* dy, const float* w_krsc,
                               float* dx, float beta, const float* y, const float* z,
                               const float* scale, const float* shift, const float* mean,
                               int mask, void* parts, size_t parts_bytes,
                               const tmr_conv_prologue* pro, hipStream_t stream);
/* tmr_conv2d_dgrad_bnbwd_acc with a dY-operand prologue (bf16 LDS-DMA engine: the conv1 dgrad of
 * a Bottleneck under the bf16 residual gradient, reading bn1's g and y1) */
int tmr_conv2d_dgrad_bnbwd_acc_pro(const tmr_conv_desc* d, const float* dy, const float* w_krsc,
                                   void* dx, float beta, const void* dx_old, int old_bf16,
                                   const float* y, const float* z, const float* scale,
                                   const float* shift, const float* mean, int mask, void* parts,
                                   size_t parts_bytes, const tmr_conv_prologue* pro,
                                   hipStream_t stream);
int tmr_conv2d_wgrad_pro(const tmr_conv_desc* d, const float* x, const float* dy, float* dw_oihw,
                         int c_real, float beta, float* ws, size_t ws_bytes,
                         const tmr_conv_prologue* pro, hipStream_t stream);
/* BatchNorm backward as per-channel coefficients, for a dY-operand prologue (the apply pass is
 * folded into the consumer convs): coef = [3][c] with dy = fmaf(A, g, fmaf(B, y, C));
 * dgamma / dbeta as tmr_bn_bwd.  From the fused-dgrad partials (g already masked; ws >=
 * tmr_bn_parts_ws_bytes(nparts, c)), or from g itself (one reduction pass over g and y, the ReLU
 * mask -- z > 0 or y*scale+shift > 0 -- applied to g IN PLACE when relu; ws >=
 * tmr_bn_ws_bytes(rows, c)). */
int tmr_bn_bwd_coefs(const void* parts, int nparts, const float* save_mean,
                     const float* save_invstd, const float* gamma, float* coef, float* dgamma,
                     float* dbeta, int rows, int c, void* ws, size_t ws_bytes,
                     hipStream_t stream);
int tmr_bn_bwd_coefs_dense(float* g, const float* y, const float* z, const float* scale,
                           const float* shift, const float* save_mean, const float* save_invstd,
                           const float* gamma, float* coef, float* dgamma, float* dbeta, int rows,
                           int c, int relu, void* ws, size_t ws_bytes, hipStream_t stream);
/* The bf16-activation step's downsample BN (no ReLU, output gradient g the bf16 residual-stream
 * gradient, y bf16): tmr_bn_bwd_g16 without its apply pass (ws >= tmr_bn_ws_bytes(rows, c)). */
int tmr_bn_bwd_coefs_g16(const void* g, const void* y, const float* save_mean,
                         const float* save_invstd, const float* gamma, float* coef, float* dgamma,
                         float* dbeta, int rows, int c, void* ws, size_t ws_bytes,
                         hipStream_t stream);

#ifdef __cplusplus
}
#endif

#endif  /* TMR_PROLOGUE_H_ */

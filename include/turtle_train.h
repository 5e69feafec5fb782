/* libturtle_hip training-path kernels (turtlevsr_amd/csrc/train_ops.hip).
 *
 * The training step (config 5, video_restoration_model.py:78-108) runs the Turtle_t1 graph under
 * torch autograd on the GPU with channels-last (NHWC) activations; these entry points are the
 * hand-written forward / backward kernels of its ops, bound by turtlevsr_amd/train_ops.py as
 * torch.autograd.Functions. Activations are pixel rows: element (p, c) at base[p * ld + c], base
 * 16-byte aligned, ld * element size a multiple of 16 B. `dtype` 0 = fp32, 1 = bf16, 2 = fp16
 * (the GEMM entry points take 0 / 1); weights and weight gradients fp32 unless stated. `stream` is
 * a hipStream_t. Gradient buffers documented as "accumulated" are added into (atomics): zero them
 * first. Return 0 or an error (negative: bad argument; positive: hipError_t).
 */
#ifndef TURTLE_TRAIN_H
#define TURTLE_TRAIN_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* LayerNorm over channels per pixel (turtle_t1_arch.py:67-112, WithBias_LayerNorm / BiasFree_LayerNorm):
 * x [P][ldx] -> y [P][ldy] (C channels, C % 8 == 0, C <= 2048); w, b [C]; saves mu, rstd [P].
 * dtype: bits 0-3 = x's type (0 fp32, 1 bf16, 2 fp16); bits 4-7 = 1 + y's type when y differs (only fp32 x
 * with bf16 / fp16 y: autocast's cast of the fp32 residual stream folded into the LayerNorm). */
int turtle_train_ln_fwd(const void* x, int64_t ldx, const float* w, const float* b, void* y, int64_t ldy, float* mu, float* rstd,
                        int64_t P, int C, int biasfree, int dtype, void* stream);
/* dx [P][lddx] in x's type, dy in y's type (dtype as ln_fwd); dw, db [C] accumulated (db unused for BiasFree).
 * dres [P][lddres] (x's type) or NULL: the gradient of the block's residual use of x (x + branch(LN(x)),
 * turtle_t1_arch.py:808-809), added into dx in the same pass (no separate gradient-accumulation add) */
int turtle_train_ln_bwd(const void* x, int64_t ldx, const float* w, const float* mu, const float* rstd, const void* dy,
                        int64_t lddy, void* dx, int64_t lddx, const void* dres, int64_t lddres, float* dw, float* db, int64_t P,
                        int C, int biasfree, int dtype, void* stream);

/* depthwise 3x3, stride 1, pad 1, groups = C (nn.Conv2d(C, C, 3, padding=1, groups=C), e.g.
 * turtle_t1_arch.py:167-169, 237, 716-722): x [N][H][W][ldx] -> y [N][H][W][ldy]; w9 tap-major
 * [9][C] (tap = 3 dy + dx), b [C] or NULL. flip = 1 uses the taps rotated by 180 degrees (the input
 * gradient: dx = dw3x3_flip(dy), b = NULL). */
int turtle_train_dw3x3_fwd(const void* x, int64_t ldx, const float* w9, const float* b, void* y, int64_t ldy, int64_t N, int C,
                           int H, int W, int flip, int dtype, void* stream);
/* dw9 [9][C], db [C] (or NULL) accumulated from x and dy */
int turtle_train_dw3x3_wgrad(const void* x, int64_t ldx, const void* dy, int64_t lddy, float* dw9, float* db, int64_t N, int C,
                             int H, int W, int dtype, void* stream);

/* GatedFeedForward gate (turtle_t1_arch.py:176): x [P][ldx] (x1 = channels [0, h), x2 = [h, 2h))
 * -> y [P][ldy] = gelu(x1) * x2 (exact erf GELU); backward dx [P][lddx] (2h channels) from x, dy. */
int turtle_train_gate_fwd(const void* x, int64_t ldx, void* y, int64_t ldy, int64_t P, int h, int dtype, void* stream);
int turtle_train_gate_bwd(const void* x, int64_t ldx, const void* dy, int64_t lddy, void* dx, int64_t lddx, int64_t P, int h,
                          int dtype, void* stream);

/* plain GELU (exact erf form; FeedForward's conv4 activation turtle_t1_arch.py:181-210, ReducedAttn's
 * after conv2 704-742): y [P][ldy] = gelu(x) over C channels; backward dx = dy * gelu'(x). Replaces
 * torch.nn.functional.gelu in the training graph. */
int turtle_train_gelu_fwd(const void* x, int64_t ldx, void* y, int64_t ldy, int64_t P, int C, int dtype, void* stream);
int turtle_train_gelu_bwd(const void* x, int64_t ldx, const void* dy, int64_t lddy, void* dx, int64_t lddx, int64_t P, int C,
                          int dtype, void* stream);

/* SAB window convolution nn.Conv2d(C, C, ws, stride=ws, padding=1, groups=C) (k2_dwconv / q2_dwconv,
 * turtle_t1_arch.py:306-308 and their use in StateAlignBlock.forward 560-571) on NHWC rows:
 * x [N][H][W][ldx] -> y [N][th][tw][ldy], th = (H + 2 - ws) / ws + 1 (tw likewise); wt fp32 [ws*ws][C] (the
 * weight [C][1][ws][ws] transposed tap-major), b [C] or NULL. dgrad: dx [N][H][W][lddx] from dy (input
 * pixels no token covers get 0). wgrad: dwt [ws*ws][C] fp32 += (caller zeroes it); the bias gradient is
 * turtle_train_colsum over dy. Replaces MIOpen's grouped convolution (forward and both backward passes). */
int turtle_train_window_fwd(const void* x, int64_t ldx, const float* wt, const float* b, void* y, int64_t ldy, int64_t N, int C,
                            int H, int W, int ws, int th, int tw, int dtype, void* stream);
int turtle_train_window_dgrad(const void* dy, int64_t lddy, const float* wt, void* dx, int64_t lddx, int64_t N, int C, int H, int W,
                              int ws, int th, int tw, int dtype, void* stream);
int turtle_train_window_wgrad(const void* x, int64_t ldx, const void* dy, int64_t lddy, float* dwt, int64_t N, int C, int H, int W,
                              int ws, int th, int tw, int dtype, void* stream);

/* column sums db[n] += sum_p dy[p][n] (a 1x1 convolution's bias gradient), N % 8 == 0 */
int turtle_train_colsum(const void* dy, int64_t ld, float* db, int64_t P, int N, int dtype, void* stream);
/* per-image column sums of squares (the channel-attention L2 norms over HW, turtle_t1_arch.py:690-691):
 * out[img][n] += sum over the img_px pixels of image img of x[p][n]^2; out fp32 [P / img_px][N], zeroed by the caller */
int turtle_train_colsumsq(const void* x, int64_t ld, float* out, int64_t P, int N, int64_t img_px, int dtype, void* stream);

/* per-image column dot products out[img][n] += sum over the img_px pixels of image img of a[p][n] b[p][n]
 * (the L2-normalisation backward's sum dy . y); out fp32 [P / img_px][N], zeroed by the caller */
int turtle_train_coldot(const void* a, int64_t lda, const void* b, int64_t ldb, float* out, int64_t P, int N, int64_t img_px,
                        int dtype, void* stream);
/* per-image column scaling y[p][c] = x[p][c] s[img][c] (s fp32 [P / img_px][C]): the forward of the per-channel
 * L2 normalisation over HW (turtle_t1_arch.py:236-237, 649-651: F.normalize(dim=-1) of the [b, heads, ch, HW]
 * view) with s = 1 / max(|x_col|, 1e-12) from turtle_train_colsumsq */
int turtle_train_colscale(const void* x, int64_t ldx, const float* s, void* y, int64_t ldy, int64_t P, int C, int64_t img_px,
                          int dtype, void* stream);
/* its backward dx = (dy - y d) s, d fp32 [P / img_px][C] = sum_p dy y (0 where the norm was clamped) */
int turtle_train_l2n_bwd(const void* dy, int64_t lddy, const void* y, int64_t ldy, const float* d, const float* s, void* dx,
                         int64_t lddx, int64_t P, int C, int64_t img_px, int dtype, void* stream);

/* StateAlignBlock attention row (turtle_t1_arch.py:394-416 top-5, 448-464 L1 ball, 115-132 clipped_softmax,
 * combined as in 585-599): s fp32 [R][n] (rows ordered (image, frame, query i), n keys on a (n / tw) x tw token
 * grid); m_j = [j in the row's top-5] + [L1 distance of tokens i, j <= radius] (0 / 1 / 2: the reference's
 * s * (top + ball)); entries with s_j m_j == 0 masked; a = softmax of s m over the rest, renormalised, in the
 * activation dtype (dtype), plus a fp32 and m (uint8 [R][n]) for the backward. n <= 1024. */
int turtle_train_sab_softmax_fwd(const float* s, int64_t R, int n, int tw, int radius, void* a, float* a_save, void* m_save,
                                 int dtype, void* stream);
/* its backward: ds fp32 [R][n] = m_j a_j (da_j - sum_k da_k a_k), da in dtype */
int turtle_train_sab_softmax_bwd(const void* da, const float* a_save, const void* m_save, int64_t R, int n, float* ds, int dtype,
                                 void* stream);

/* the per-image weight of the normalised channel-attention Gram backward (turtle_t1_arch.py:690-697
 * differentiated): wd[b] [2c][2c] = [[diag(aq[b]), D[b]], [D[b]^T, diag(ak[b])]], D [B][heads][ch][ch] fp32
 * block-diagonal per head (ch = c / heads), aq / ak fp32 [B][c]; wd in the activation dtype, dense */
int turtle_train_gram_wd(const float* D, const float* aq, const float* ak, void* wd, int64_t B, int c, int heads, int dtype,
                         void* stream);

/* pointwise GEMM (a 1x1 convolution, nn.Conv2d(K, N, 1) on NHWC rows; also its input gradient with
 * W transposed, and the channel-attention A.v with per-image weights):
 *   y[p][n] = sum_k x[p][k] w[img(p)][n][k] + bias[n]
 * w [N][K] in the activation dtype; wstride = 0: one weight set, else set i at w + i * wstride
 * elements for the i-th run of img_px pixels. bias fp32 [N] or NULL. K % 8 == N % 8 == 0. Runs on
 * the inference GEMM family (gemm*.hip). res [P][ldr] in the activation dtype or NULL: added in the
 * epilogue (the block's residual x + branch, turtle_t1_arch.py:808-809: one rounding, no separate add). */
int turtle_train_gemm(const void* x, int64_t ldx, const void* w, int64_t wstride, int64_t img_px, const float* bias,
                      const void* res, int64_t ldr, void* y, int64_t ldy, int64_t P, int K, int N, int dtype, void* stream);

/* reduction GEMM over pixels (a 1x1 convolution's weight gradient dW = dY^T X; the channel
 * attention Gram q^T k over HW, turtle_t1_arch.py:694-697, and its backward):
 *   c[img][n][k] (+)= sum_{p in img} a[p][n] b[p][k]
 * img_px = 0: one product over all P pixels; else one per run of img_px pixels (P % img_px == 0).
 * c fp32 [nimg][N][K]; accumulate = 1 adds into c. Needs a workspace of
 * turtle_train_rgemm_workspace(P, N, K, img_px) bytes. Deterministic (fixed reduction order). */
size_t turtle_train_rgemm_workspace(int64_t P, int N, int K, int64_t img_px);
int turtle_train_rgemm(const void* a, int64_t lda, const void* b, int64_t ldb, float* c, int64_t P, int N, int K, int64_t img_px,
                       int accumulate, int dtype, void* ws, size_t ws_bytes, void* stream);

/* dense 3x3 convolution, stride 1, padding 1, on NHWC rows (Down / Upsample body[0] 3x3 convolutions,
 * turtle_t1_arch.py:136-154): y [P][ldy] = conv3x3(x) (+ bias), w [N][9][Cin] in the activation dtype
 * (tap = 3 ky + kx), bias fp32 [N] or NULL; Cin % 8 == N % 8 == 0. The inference implicit-GEMM family.
 * The input gradient is the same call on dy with w'[ci][tap][n] = w[n][8 - tap][ci]. */
int turtle_train_conv3x3(const void* x, int64_t ldx, const void* w, const float* bias, void* y, int64_t ldy, int64_t B, int H,
                         int W, int Cin, int N, int dtype, void* stream);
/* its weight gradient: dw fp32 [9][N][Cin] = sum_p dy[p][n] x[p + off(tap)][ci] (zero padding), deterministic;
 * needs turtle_train_conv3x3_wgrad_workspace(B * H * W, N, Cin) bytes of workspace */
size_t turtle_train_conv3x3_wgrad_workspace(int64_t P, int N, int Cin);
int turtle_train_conv3x3_wgrad(const void* dy, int64_t lddy, const void* x, int64_t ldx, float* dw, int64_t B, int H, int W, int N,
                               int Cin, int dtype, void* ws, size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif

/* libturtle_hip training-path kernels (turtlevsr_amd/csrc/train_ops.hip).
 *
 * The training step (config 5, video_restoration_model.py:78-108) runs the Turtle_t1 graph under
 * torch autograd on the GPU; these entry points are the hand-written forward / backward kernels of
 * the ops whose aten lowering is the slow part of that graph, bound by turtlevsr_amd/train_ops.py
 * as torch.autograd.Functions. Tensors are NCHW, contiguous, device pointers; `dtype` 0 = fp32,
 * 1 = bf16 activations (weights and weight gradients fp32); `stream` is a hipStream_t. Weight /
 * bias gradient buffers are accumulated into (atomics): zero them first. Return 0 or an error
 * (negative: bad argument; positive: hipError_t).
 */
#ifndef TURTLE_TRAIN_H
#define TURTLE_TRAIN_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* LayerNorm over channels per pixel (turtle_t1_arch.py:67-112, WithBias_LayerNorm / BiasFree_LayerNorm):
 * x, y [N][C][HW]; w, b [C]; saves mu, rstd [N*HW] for the backward. */
int turtle_train_ln_fwd(const void* x, const float* w, const float* b, void* y, float* mu, float* rstd, int64_t N, int C,
                        int64_t HW, int biasfree, int dtype, void* stream);
/* dx [N][C][HW]; dw, db [C] accumulated (db unused for BiasFree) */
int turtle_train_ln_bwd(const void* x, const float* w, const float* mu, const float* rstd, const void* dy, void* dx,
                        float* dw, float* db, int64_t N, int C, int64_t HW, int biasfree, int dtype, void* stream);

/* depthwise 3x3, stride 1, pad 1, groups = C (nn.Conv2d(C, C, 3, padding=1, groups=C), e.g.
 * turtle_t1_arch.py:167-169, 237, 716-722): w [C][9], b [C] or NULL. flip = 1 convolves with the
 * taps rotated by 180 degrees (the input gradient: dx = dw3x3_flip(dy), b = NULL). N*C <= 65535. */
int turtle_train_dw3x3_fwd(const void* x, const float* w, const float* b, void* y, int64_t N, int C, int H, int W, int flip,
                           int dtype, void* stream);
/* dw [C][9], db [C] (or NULL) accumulated from x and dy */
int turtle_train_dw3x3_wgrad(const void* x, const void* dy, float* dw, float* db, int64_t N, int C, int H, int W, int dtype,
                             void* stream);

/* GatedFeedForward gate (turtle_t1_arch.py:176): x [N][2h][HW] -> y [N][h][HW] = gelu(x[:h]) * x[h:]
 * (exact erf GELU); backward dx [N][2h][HW] from x and dy. */
int turtle_train_gate_fwd(const void* x, void* y, int64_t N, int h, int64_t HW, int dtype, void* stream);
int turtle_train_gate_bwd(const void* x, const void* dy, void* dx, int64_t N, int h, int64_t HW, int dtype, void* stream);

#ifdef __cplusplus
}
#endif
#endif

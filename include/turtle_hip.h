/* turtle_hip.h - C ABI of libturtle_hip.so, the MI355X (gfx950) Turtle per-frame restoration path.
 *
 * This is the drop-in boundary for the reference's arch plug-in
 *   basicsr/models/archs/turtle_t1_arch.py  (make_model 10-53, Turtle_t1.forward 1045-1132)
 *   basicsr/models/archs/turtlesuper_t1_arch.py (TurtleSuper_t1.forward 1049-1147)
 * The reference has no native FFI; these entry points are what its Python module binds (via
 * ctypes): plain pointers and sizes, device pointers are hipMalloc'd memory
 * (e.g. torch.Tensor.data_ptr() on a ROCm device), all work is stream-ordered on `stream`.
 *
 * Every function returns 0 on success, a negative TURTLE_E* code on failure; the message is
 * available from turtle_last_error() (thread-local), mirroring the reference's Python exceptions.
 */
#ifndef TURTLE_HIP_H
#define TURTLE_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TURTLE_OK 0
#define TURTLE_EINVAL -1   /* bad argument / shape (the reference raises RuntimeError / einops errors) */
#define TURTLE_ENOWEIGHT -2 /* missing or mis-shaped weight (load_state_dict strict=True)        */
#define TURTLE_EHIP -3     /* HIP runtime error                                                   */
#define TURTLE_ESTATE -4   /* call order (e.g. forward before turtle_load_weights)                */

#define TURTLE_DTYPE_F32 0
#define TURTLE_DTYPE_BF16 1

/* attention / FFN type codes (TurtleAttnBlock, turtle_t1_arch.py:780-802) */
#define TURTLE_ATTN_REDUCED 0
#define TURTLE_ATTN_CHANNEL 1
#define TURTLE_ATTN_FHR 2
#define TURTLE_ATTN_CHM 3
#define TURTLE_ATTN_NONE 4
#define TURTLE_FFN_FFW 0
#define TURTLE_FFN_GFFW 1

/* Arch keys read by make_model (turtle_t1_arch.py:12-52), already defaulted by the caller. */
typedef struct TurtleConfig {
  int n_colors;
  int dim;
  int enc_blocks[3];
  int middle_blocks;
  int dec_blocks[3];
  int num_refinement_blocks;
  float ffn_expansion_factor;
  int bias;
  int layernorm_biasfree;   /* LayerNorm_type == 'BiasFree' */
  int use_both_input;
  int num_frames_tocache;
  int num_heads[4];
  /* [encoder1..3, decoder1..3, refinement][type1, type2] */
  int level_attn[7][2];
  int level_ffn[7];         /* encoder1..3, decoder1..3, refinement */
  int latent_attn[3];
  int latent_ffn;
  int super_resolution;     /* 1: TurtleSuper_t1 (4x bilinear front-end) */
  int dtype;                /* TURTLE_DTYPE_* storage / MFMA type; accumulation is fp32 */
  int variant;              /* 0: Turtle_t1 (turtle_t1_arch.py); 1: the t0 network "Turtle"
                               (turtle_arch.py: StateAlignBlock 459-533, option `model: Turtle_arch`) */
} TurtleConfig;

typedef struct TurtleHandle TurtleHandle;

/* make_model(opt): validate the config and create a handle (no device memory yet). */
int turtle_create(const TurtleConfig* cfg, TurtleHandle** out);
void turtle_destroy(TurtleHandle* h);

/* Number of state-dict entries and their names / shapes, in the reference's state_dict() order. */
int turtle_num_weights(const TurtleHandle* h);
int turtle_weight_info(const TurtleHandle* h, int idx, const char** name, int* ndim, int64_t shape[4]);

/* Stage one state-dict tensor (host fp32, C-contiguous, `numel` elements). */
int turtle_set_weight(TurtleHandle* h, const char* name, const float* host_data, int64_t numel);
/* Validate that every entry is staged (strict load), pack and upload to the device. */
int turtle_load_weights(TurtleHandle* h);

/* History-state layout. For cache slot i (0..7, order of Turtle_t1.forward's k_to_cache list):
 *   kind[i] = 0 none, 1 FHR rows, 2 SAB frames.
 *   FHR:  shape [B, heads, rows, P]      with strides (P*heads*rows, rows, 1, heads*rows)
 *   SAB:  k [B, frames, 1, N, 2c] (t0: ws*ws*c), v [B, frames, 1, N, ws*ws*c], contiguous.
 * `t_in[i]` = rows (FHR) / frames (SAB) of the incoming cache (0 when the caller passes None).
 * Writes kind[8], and for each slot the 5-d shapes (unused trailing dims = 1) of the k and v
 * tensors forward() will return: k_shape[i*5 + d], v_shape[i*5 + d]. */
int turtle_cache_layout(const TurtleHandle* h, int B, int H, int W, const int t_in[8],
                        int kind[8], int64_t k_shape[40], int64_t v_shape[40]);

/* Device workspace bytes needed by turtle_forward for frames of B x H x W. */
int turtle_workspace_size(const TurtleHandle* h, int B, int H, int W, size_t* bytes);

/* One causal step (Turtle_t1.forward): inp [B, 2, n_colors, H, W] fp32 contiguous (device),
 * out [B, n_colors, Hout, Wout] fp32 (Hout = H, or 4H for super-resolution).
 * k_in/v_in[i]: incoming caches (NULL when t_in[i] == 0), k_out/v_out[i]: caller-allocated
 * tensors of the shapes given by turtle_cache_layout (NULL for kind 0). Storage dtype of caches
 * = the handle's dtype. */
int turtle_forward(TurtleHandle* h, const float* inp, int B, int H, int W, float* out,
                   const void* const k_in[8], const void* const v_in[8], const int t_in[8],
                   void* const k_out[8], void* const v_out[8],
                   void* workspace, size_t workspace_bytes, void* stream);

/* Per-kernel-class timing with HIP events on the forward's stream (measurement only).
 * turtle_profile_begin(h, cls): from now on every launch of class `cls` (TURTLE_K_*, or
 * TURTLE_K_ALL) issued by turtle_forward is bracketed by two events, and its algorithmic HBM
 * bytes and FLOPs (each distinct input read once, each output written once) are accumulated.
 * turtle_profile_end(h, out): waits for the events, stops profiling and writes, for each class
 * c < TURTLE_K_COUNT: out[4c] = summed kernel ms, out[4c+1] = launches, out[4c+2] = bytes,
 * out[4c+3] = FLOPs. */
#define TURTLE_K_GEMM 0       /* pointwise 1x1 and implicit 3x3 convolutions (MFMA)        */
#define TURTLE_K_DW 1         /* depthwise 3x3 (+GELU / gate)                              */
#define TURTLE_K_ATTN 2       /* channel-attention Gram + finalize + W_eff                 */
#define TURTLE_K_SAB_SCORE 3  /* SAB q.k^T + top-5                                         */
#define TURTLE_K_SAB_AV 4     /* SAB clipped softmax + sparse A.v gather                   */
#define TURTLE_K_WINDOW 5     /* SAB window conv + L2 norm                                 */
#define TURTLE_K_OTHER 6      /* stem, ending, cache roll / copies                          */
#define TURTLE_K_FUSED 7      /* fused pointwise -> depthwise -> pointwise blocks (fused.hip) */
#define TURTLE_K_COUNT 8
#define TURTLE_K_ALL 99
int turtle_profile_begin(TurtleHandle* h, int kernel_class);
int turtle_profile_end(TurtleHandle* h, double out[4 * TURTLE_K_COUNT]);
/* Restrict profiling to launches whose shape tag (the TURTLE_PROF_DUMP tag column) equals `tag`
 * (NULL or "" profiles every launch of the class again): keeps the event overhead of a timed
 * region to the one launch shape being measured. */
int turtle_profile_filter(TurtleHandle* h, const char* tag);

/* Kernel-selection switches (performance A/B only; every setting computes the same function;
 * defaults in brackets). Names and semantics are those turtle_set_option (turtle.cpp) accepts:
 *   "fuse"         [1] block-level fused kernels (fused2.hip row walk / fused.hip) for input widths <= 128
 *   "fuse_fp32"    [0] ... also in the fp32 build (the round-1 fused.hip kernel; 0: GEMM + depthwise + GEMM, faster)
 *   "fused2"       [1] the bf16 row-walk fused kernel (fused2.hip); 0: the round-1 fused.hip kernel
 *   "ffn"          [1] FeedForward in one kernel (ffn.hip) at widths 64 / 128 (bf16)
 *   "gffn"         [1] GatedFeedForward in one kernel at width 256 (gffn.hip: LN -> project_in -> dwconv -> gelu gate ->
 *                  project_out + residual, the hidden map never in HBM; bf16); 0: pn GEMM + dwgemm
 *   "gffn_min_blocks" [256] minimum tile count for a gffn launch (one block per CU)
 *   "gemm_pn"      [1] persistent resident-panel GEMM for LN-folded 1x1 convolutions, K <= 512
 *   "gemm_ar"      [1] A-resident per-panel GEMM for the K = 256 residual projections
 *   "gemm_kt"      [1] 2-D tiled deep-ring GEMM (3x3 up/down convolutions, K >= 640, small maps)
 *   "gemm_lds"     [1] LDS-pipelined GEMM (fallback where the kernels above do not apply)
 *   "panel_gemm"   [1] register-panel GEMM fallback; 0: K-loop GEMM
 *   "gemm_f32"     [1] fp32 GEMM on an LDS-DMA ring (gemm_f32.hip) for the LN / GELU / multi-source fp32 GEMMs
 *   "gemm_sk"      [1] split-K GEMM (gemm_sk.hip): single-source projections of GEMMs over <= sk_max_px pixels
 *   "sk_max_px"    [4096] ... its pixel limit (set before the workspace is sized)
 *   "gemm9"        [1] 256-pixel-row GEMM (gemm9.hip): 1 the 'wide' projection class (latent LN projections, project_out
 *                  K = 1280, latent / level-3 W_eff),
 *                  2 every eligible projection, 0 never
 *   "gemm8"        [3] 256 x 256 four-phase GEMM (gemm8.hip): 1 the 'wide' class, 2 every eligible projection,
 *                  3 the multi-source projections with K >= 1024 (where it measures fastest), 0 never
 *   "gemm8_ps"     [0] ... in its persistent form (one block per CU walks its tiles as one K-tile stream)
 *   "kt_max_px"    [32768] (integer) below this many pixels every eligible GEMM goes to the 2-D tiled kernel
 *   "attn_fin"     [0] channel-attention row softmax inside the W_eff launch (attn.hip)
 *   "sab_waves"    [0] waves per SAB score block: 4 (64 queries) or 8 (128 queries per staged key tile); 0 = 8 at
 *                  token widths d >= 256, 4 below
 *   "tilepd"       [1] level-3 LN -> pointwise -> depthwise with the hidden map on chip (tilepd.hip:
 *                  channel-attention qkv + qkv_dwconv)
 *   "tilepd_gate"  [0] ... also the GatedFeedForward's project_in + dwconv + gelu gate (slower than pn + dwgemm)
 *   "tilepd_cb"    [1] its GatedFeedForward output channel-blocked for the project_out GEMM
 *   "tilepd_min_blocks" [256] minimum tile count for a tilepd launch (one block per CU)
 *   "dwgemm"       [1] depthwise as the operand prologue of the following GEMM (dwgemm.hip)
 *   "dwgemm_attn"  [1] ... for the level-3 channel attention's v path (W_eff GEMM)
 *   "dwgemm_cb"    [1] ... for the level-3 GatedFeedForward, hidden map stored channel-blocked
 *   "dwgemm_min_blocks" [384] minimum block count for a dwgemm launch
 *   "dw_rows"      [1] row-sweeping depthwise kernel; 0: per-pixel 9-tap gather kernel
 *   "down_tile"    [1] LDS-tiled level-1 Downsample (spatial.hip)
 *   "stem_mfma"    [1] input_projection / ending 3x3 on the matrix cores (bf16, dim 64)
 *   "sab_mfma"     [1] SAB sparse A.v on the matrix cores (bf16)
 *   "sab_db"       [0] SAB A.v: 0 two blocks per CU; 1 double-buffered at one block per CU; 2 two blocks per CU
 *                  with the top-5 tail rows fetched a chunk ahead (slower)
 *   "split_out"    [1] output-adjacent weights (ending, reduce_chan_level1) as split bf16 pairs
 * Unknown names return TURTLE_EINVAL. */
int turtle_set_option(TurtleHandle* h, const char* name, int value);

const char* turtle_last_error(void);

/* Hash of the kernel sources (turtlevsr_amd/csrc + build.py, turtlevsr_amd/build.py source_hash) the
 * library was built from: the Python binding refuses a library whose hash is not the tree's. */
const char* turtle_source_hash(void);

#ifdef __cplusplus
}
#endif
#endif

// Kernel argument blocks and launchers (host + device visible).
#pragma once
#include "common.h"

#include <vector>

namespace turtle {

// length of the constant zero / one vectors (GemmArgs.zeros / ones) that stand in for absent per-channel
// bias / scale / LayerNorm vectors: the GEMM kernels read them at the output channel, so N <= this
constexpr int TURTLE_CONST_VEC = 65536;

// STORE_CB16: channel-blocked [C / 16][pixels][16] (cb_px pixels per block): the hidden map of a
// GatedFeedForward whose depthwise + gate runs in dwgemm.hip reads one K step as contiguous rows
enum StoreMode { STORE_NHWC = 0, STORE_SHUFFLE = 1, STORE_UNSHUFFLE = 2, STORE_CB16 = 3 };

struct GemmArgs {
  SrcList a;                       // A sources, K-concatenated
  int64_t M;                       // output pixels (all images)
  int N;                           // output channels
  int HW, Wimg;                    // pixels per image, image width (GEMM pixel grid)
  const void* w;                   // [N][ldw] (storage type), per-image set if wstride != 0
  int64_t ldw, wstride;
  int wdiv;                        // weight set index = image / wdiv
  int conv3, cin;                  // implicit 3x3 (K = 9 * cin, tap-major)
  int ln;                          // LayerNorm prologue over a.s[0]
  const float* ln_s;               // rowsum(W*g) (null: BiasFree)
  const float* ln_t;               // W.b         (null: BiasFree)
  const float* bias;
  const float* scale;
  int gelu;
  const void* res;                 // residual (pixel-major, same pixel index as out)
  int64_t ldr;
  int offr;
  void* out;
  int64_t ldo;
  int offo;
  int store_mode;
  const float* zeros;              // >= 16384 zero floats / 8192 ones (absent vectors, residual)
  const float* ones;
  int allow_panel;                 // panel kernel permitted (turtle_set_option "panel_gemm")
  int allow_lds;                   // LDS-pipelined kernel permitted (turtle_set_option "gemm_lds")
  int allow_pn;                    // resident-panel kernel permitted (turtle_set_option "gemm_pn")
  int allow_ar;                    // A-resident per-panel kernel permitted (turtle_set_option "gemm_ar")
  int allow_kt;                    // 2-D tiled deep-ring kernel permitted (turtle_set_option "gemm_kt")
  int dbg;                         // tools/kbench ablations of the pn kernel (0 in the product path)
  unsigned long long* stamps;      // tools/kbench s_memtime stamps of the pn kernel (null in the product path)
  int64_t cb_px;                   // STORE_CB16: pixels per 16-channel block (= M)
  int allow_g8;                    // 256 x 256 four-phase kernel permitted (turtle_set_option "gemm8")
  int kt_max_px;                   // GEMMs over fewer pixels go to the 2-D tiled kernel (0: 32768)
  int allow_g9;                    // 256 x 256 four-wave kernel permitted (turtle_set_option "gemm9")
  int allow_f32;                   // fp32 occupancy-tiled kernel permitted (turtle_set_option "gemm_f32")
};
template <typename T> void launch_gemm(const GemmArgs& g, hipStream_t st);
bool gemm_f32_ok(const GemmArgs& g);                              // gemm_f32.hip (fp32)
bool gemm_sk_ok(const GemmArgs& g);                               // gemm_sk.hip (bf16 split-K, small frames)
int gemm_sk_splits(int64_t M, int N, int K);
size_t gemm_sk_workspace_bytes(int64_t M, int N, int K);
void launch_gemm_sk(const GemmArgs& g, void* ws, hipStream_t st);
void launch_ln_stats(const GemmArgs& g, float2* stats, hipStream_t st);   // gemm9.hip
bool gemm_f32_preferred(const GemmArgs& g);
void launch_gemm_f32(const GemmArgs& g, hipStream_t st);
bool gemm_lds_ok(const GemmArgs& g);                              // gemm2.hip (bf16)
void launch_gemm_lds(const GemmArgs& g, hipStream_t st);
bool gemm_pn_ok(const GemmArgs& g);                               // gemm3.hip (bf16)
void launch_gemm_pn(const GemmArgs& g, hipStream_t st);
bool gemm_ar_ok(const GemmArgs& g);                               // gemm3.hip (bf16)
void launch_gemm_ar(const GemmArgs& g, hipStream_t st);
bool gemm_kt_ok(const GemmArgs& g);                               // gemm5.hip (bf16)
void launch_gemm_kt(const GemmArgs& g, hipStream_t st);
bool gemm8_ok(const GemmArgs& g);                                 // gemm8.hip (bf16)
void launch_gemm8(const GemmArgs& g, hipStream_t st);
bool gemm9_ok(const GemmArgs& g);                                 // gemm9.hip (bf16)
size_t gemm9_stats_bytes(const GemmArgs& g);                      // LN statistics workspace
void launch_gemm9(const GemmArgs& g, void* stats, hipStream_t st);

enum DwMode { DW_PLAIN = 0, DW_GELU = 1, DW_GATE = 2 };
struct DwArgs {
  const void* in; int64_t ldi; int offi;
  void* out; int64_t ldo; int offo;
  const float* w;                  // [9][Cw] tap-major fp32 (Cw = C, or 2C for DW_GATE)
  const float* bias;               // [Cw] or null
  int nimg, H, W, C;               // C = output channels
  int mode;
  int tok_ws;                      // > 0: SAB dilated token-major output [img][n][(p1*ws+p2)*C + c]
  int64_t tok_img_stride;          // element stride between images of the token-major output
  int rows;                        // row-sweeping kernel (default) vs per-pixel gather
};
template <typename T> void launch_dw(const DwArgs& a, hipStream_t st);

// spatial.hip: level-1 Downsample as an LDS-tiled 3x3 conv (Cin -> Cin / 2, bf16) with the
// PixelUnshuffle(2) store; weights as pre-packed MFMA A fragments [Cout / 16][9 Cin / 32][64 lanes][8]
struct DownTileArgs {
  const void* x; int64_t ldx; int Cin;        // input NHWC [nimg][H][W][ldx]
  const void* wfrag;
  void* out; int64_t ldo;                     // output NHWC [nimg][H/2][W/2][ldo], channels 0 .. 2 Cin - 1
  int nimg, H, W;
};
bool down_tile_ok(const DownTileArgs& a);
void launch_down_tile(const DownTileArgs& a, hipStream_t st);

struct WinArgs {                   // SAB q2/k2 window conv (ws x ws, stride ws, pad 1) + L2 norm
  const void* in; int64_t ldi; int offi;
  const float* w;                  // [ws*ws][C] fp32
  const float* bias;               // [C] or null
  void* out; int64_t out_img_stride;   // token rows of C elements; image stride in elements
  int nimg, H, W, C, ws;
};
template <typename T> void launch_window(const WinArgs& a, hipStream_t st);

#define TURTLE_MAX_T 8
struct SabScoreArgs {
  const void* q;                   // [B][N][d] normalised query tokens
  int64_t q_bstride;
  const void* k[TURTLE_MAX_T];     // frame t: [N][d] for batch 0
  int64_t k_bstride[TURTLE_MAX_T];
  int B, T, N, d, th, tw;
  int nsplit;                      // key range split across blocks (partial top-5 lists)
  const float* tau;                // temperature (device scalar)
  float* topv;                     // [B*T][nsplit][N][5]
  int* topi;
  float* ballv;                    // [B*T][N][41] scores of the L1-ball keys (|di|+|dj| <= 4)
  int dbg;                         // tools/sabbench ablations (0 in the product path)
  int waves;                       // 4 or 8 waves (64 / 128 queries) per block; 0 = 4
};
template <typename T> void launch_sab_score(const SabScoreArgs& a, hipStream_t st);
int sab_score_nsplit(int B, int T, int N, int d, int waves = 4);

constexpr int SAB_MAXC = 48;       // candidate slots per query (41 ball + 5 top-k, padded)
struct SabPrepArgs {               // candidates + clipped softmax per (b, t, query)
  const float* topv; const int* topi; const float* ballv;
  int BT, N, th, tw, nsplit;
  int* cnt;                        // [BT][N] surviving candidates | (ball candidates, listed first) << 16
  int* ci;                         // [BT][N][SAB_MAXC] key index (padding: the query's own index)
  float* cw;                       //                   softmax weight (padding: 0)
  float* ballw;                    // [BT][N][41] dense ball weights (may alias ballv)
};
void launch_sab_prep(const SabPrepArgs& a, hipStream_t st);

struct SabGatherArgs {             // out = sum_c w_c v[key_c], dilated token -> pixel regroup
  const void* v[TURTLE_MAX_T]; int64_t v_bstride[TURTLE_MAX_T];   // [N][ws*ws*C]
  int B, T, N, th, tw, ws, C;
  const int* cnt; const int* ci; const float* cw;
  const float* ballw;              // [B*T][N][41] dense ball weights (matrix-core A.v)
  void* out;                       // [B*T][Hl][Wl][C] pixel-major
  int db;                          // sab_av_mfma: 0 two blocks / CU; 1 double-buffered (1 block / CU); 2 two
                                   // blocks / CU with the tail rows fetched one chunk ahead
};
bool sab_av_mfma_ok(const SabGatherArgs& a);
void launch_sab_av_mfma(const SabGatherArgs& a, hipStream_t st);   // bf16
template <typename T> void launch_sab_gather(const SabGatherArgs& a, hipStream_t st);

#define TURTLE_MAX_SEG 6
struct GramSeg {                   // ch key columns per head from a pixel-major source
  const void* base; int64_t ld; int off; int hstride; int img_mul, img_add; int norm;
};
struct GramArgs {
  const void* q; int64_t ldq; int qoff;   // q channel h*ch+i at qoff
  GramSeg seg[TURTLE_MAX_SEG]; int nseg;
  int B, heads, ch, HW, nchunk, chunk;
  float* part;                     // [B*heads][nchunk][ch*ncol + ch + ncol]
};
template <typename T> void launch_gram(const GramArgs& a, hipStream_t st);

struct AttnFinArgs {               // per-row Gram reduction + softmax
  const float* part; int nchunk;
  int B, heads, ch, nseg;
  unsigned norm_mask;              // bit s: segment s is L2-normalised over HW
  const float* tau;                // [heads]
  float* kinv;                     // [B][heads*ch] 1/max(|k_cur|,eps) of segment `cur_seg`, or null
  int cur_seg;
  float* red;                      // scratch [B*heads][ch*ncol + ch + ncol] summed partials
  float* attn;                     // [B*heads][ch][ncol]
  int sum_only;                    // 1: only the reduction (the softmax runs inside attn_weff_fin)
};
void launch_attn_finalize(const AttnFinArgs& a, hipStream_t st);
int attn_nsplit(int nchunk);

struct WeffArgs {                  // W_eff[b][o][col] = sum_i Wp[o][h*ch+i] * A[b][h][i][seg*ch+j]
  const float* attn;               // softmaxed attention [B*heads][ch][ncol]
  const float* wp;                 // wp fp32 [C][C]
  int B, heads, ch, nseg, C;
  int64_t seg_col[TURTLE_MAX_SEG]; // column of (seg, h=0, j=0) in W_eff
  int seg_hstride[TURTLE_MAX_SEG]; // column step per head
  int Keff;
  void* weff;                      // [B][C][Keff] storage type
};
template <typename T> void launch_weff(const WeffArgs& a, hipStream_t st);
// row softmax + W_eff in one launch (reads f.red, ignores a.attn): needs ch % 4 == 0, C % 4 == 0,
// ch <= 128, ncol <= 128, ch * ncol <= 8192
bool weff_fin_ok(const WeffArgs& a);
template <typename T> void launch_weff_fin(const WeffArgs& a, const AttnFinArgs& f, hipStream_t st);

struct FhrCacheArgs {              // latent FHR cache roll: keep last Rnew rows of [old R ; cur ch]
  const void* old; int R;          // [B][P][heads][R] (R may be 0)
  const void* cur; int64_t ldc; int coff;   // current k or v, pixel-major
  const float* kinv;               // [B][heads*ch] scale for current rows (k) or null (v)
  void* out; int Rnew;             // [B][P][heads][Rnew]
  int B, P, heads, ch;
};
template <typename T> void launch_fhr_cache(const FhrCacheArgs& a, hipStream_t st);

struct StemArgs {                  // input_projection 3x3 on the padded (or 4x bilinear) frame
  const float* inp;                // [B][2][Cin][H][W] fp32 (caller layout)
  int64_t in_bstride, in_fstride;  // element strides of batch / frame
  int B, Cimg, Hin, Win;           // source frame size
  int Hp, Wp;                      // padded working size
  int use_both;                    // channels = [prev, cur]
  int sr;                          // 4x bilinear upsample of the current frame before padding
  const float* w;                  // [Cout][Cin_tot][3][3]
  const float* bias;
  int Cout;
  void* out;                       // [B][Hp][Wp][Cout]
};
template <typename T> void launch_stem(const StemArgs& a, hipStream_t st);

struct EndArgs {                   // ending 3x3 Cin->Cimg + bias + current frame, cropped, NCHW fp32
  const void* x; int Cin;          // [B][Hp][Wp][Cin]
  const float* w; const float* bias;
  const float* inp; int64_t in_bstride, in_fstride;
  int B, Cimg, Hin, Win, Hp, Wp, Hout, Wout, sr;
  float* out;                      // [B][Cimg][Hout][Wout]
  const void* wfrag;               // bf16 MFMA A fragments of w (turtle.cpp pack_all), matrix-core kernel
};
template <typename T> void launch_ending(const EndArgs& a, hipStream_t st);
bool stem_end_mfma_ok(int cin_end, int cin_stem, int cout_stem);   // bf16 matrix-core stem / ending
// false (nothing launched) unless the packed 64-channel fragments and <= 4 image channels are given
bool launch_ending_mfma(const EndArgs& a, hipStream_t st);
// a launcher reached with arguments its dispatcher should have excluded: raises the library error
// (turtle.cpp; the C ABI returns TURTLE_EINVAL) instead of ending the host process
[[noreturn]] void kernel_arg_error(const char* what);
void launch_stem_mfma(const StemArgs& a, hipStream_t st);

enum FusedMode { F_DWONLY = 0, F_GELU = 1, F_GATE = 2 };
struct FusedDst {                  // F_DWONLY output for channels [cbeg, cend)
  void* p; int64_t ld; int off; int cbeg, cend, ccount; int tok_ws; int64_t tok_stride;
};
struct FusedArgs {                 // fused.hip: [LN ->] pw -> dw3x3 -> [act -> pw (+res)]
  const void* x; int64_t ldx; int offx; int C;
  int nimg, H, W;
  const void* w1; int N1;          // [N1][C]
  int ln; const float* ln_s; const float* ln_t; const float* b1;
  const float* dww; const float* dwb;   // [9][N1], [N1]
  const uint32_t* dww2;            // bf16 tap pairs [5][N1] (bf16 path: v_dot2_f32_bf16)
  int hidden;                      // F_GATE: N1/2, else N1
  int mode;
  const void* w2; int N2;          // [N2][hidden], N2 <= 128
  const float* b2; const float* scale2;
  const void* res; int64_t ldr; int offr;
  void* out; int64_t ldo; int offo;
  FusedDst dst[3]; int ndst;
  int dbg;                         // tools/fbench ablations (0 in the product path)
  unsigned long long* stamps;      // tools/fbench s_memtime stamps (null in the product path)
  int up;                          // fused2.hip: 16-channel hidden units per GEMM2 pass (set by its launcher)
};
template <typename T> void launch_fused(const FusedArgs& a, hipStream_t st);
bool fused2_ok(const FusedArgs& a);                               // fused2.hip (bf16 row walk)
void launch_fused2(const FusedArgs& a, hipStream_t st);

struct DwGemmArgs {                // dwgemm.hip: out = res + b + W [gelu(dw(x1)) * dw(x2) | dw(x)], bf16
  const void* in; int64_t ldi; int offi;   // hidden map, pixel-major [nimg][H][W][ldi]; x1 at offi, x2 at offi + K
  const void* dww16; const float* dwb;     // [9][NH*K] bf16 tap-major, [NH*K] fp32 or null
  int gate;                        // 1: GatedFeedForward gate (NH = 2), 0: plain depthwise
  int nimg, H, W, K;               // K = GEMM depth = depthwise output channels
  const void* w; int64_t ldw; int64_t wstride; int wdiv;   // [N][ldw] bf16; per-image sets if wstride
  int N;
  const float* bias;               // [N] or null
  const void* res; int64_t ldr; int offr;
  void* out; int64_t ldo; int offo;
  const float* zeros;              // >= 16 zero floats
  int64_t cb_px;                   // > 0: `in` is channel-blocked [C / 16][cb_px][16] (STORE_CB16), ldi / offi unused
  int dbg;                         // tools/dgbench ablations (0 in the product path)
};
bool dwgemm_ok(const DwGemmArgs& g);
int64_t dwgemm_blocks(const DwGemmArgs& g);
void launch_dwgemm(const DwGemmArgs& g, hipStream_t st);

// tilepd.hip: LN -> pointwise (C = 256) -> depthwise 3x3 (-> gelu gate) with the hidden map kept on
// chip (bf16 in / out, fp32 accumulation)
enum TilePdMode { TP_DW = 0, TP_GATE = 2 };
struct TilePdArgs {
  const void* x; int64_t ldx; int offx; int C;   // input [nimg][H][W][ldx], C channels at offx
  int nimg, H, W;
  const void* w1; int N1;                        // [N1][C] bf16 (LayerNorm-folded when ln)
  int ln, centred;                               // LayerNorm prologue; centred: WithBias (BiasFree: x * rstd)
  const float* tb;                               // [N1] GEMM1 epilogue W1 b_ln + b1 (null: 0)
  const void* dww16; const float* dwb;           // [9][N1] bf16 taps, [N1] fp32 bias or null
  int mode;                                      // TP_GATE: hid = N1 / 2 outputs gelu(dw h1) * dw h2; TP_DW: N1 outputs
  void* out; int64_t ldo; int offo;              // [nimg][H][W][ldo] bf16 (cb_px == 0)
  int64_t cb_px;                                 // > 0: channel-blocked output [channels / 16][cb_px][16] (ldo / offo unused)
  int dbg;                                       // tools/tpbench ablations (0 in the product path)
};
bool tilepd_ok(const TilePdArgs& a);
int64_t tilepd_blocks(const TilePdArgs& a);
void launch_tilepd(const TilePdArgs& a, hipStream_t st);

// gffn.hip: the whole GatedFeedForward block at input width 256, out = x + W2 (gelu(dw H1) * dw H2) + b2
// with [H1 ; H2] = W1' LN(x) + tb; bf16 in / out, f16 operands on chip, fp32 accumulation
struct GffnArgs {
  const void* x; void* out;        // [nimg][H][W][C] bf16, out != x (neighbouring tiles read x's halo)
  int nimg, H, W, hd;              // hd = hidden width (multiple of 64)
  int C;                           // input / output width: 256 (level 3) or 128 (level 2)
  int centred;                     // WithBias LayerNorm (BiasFree: x * rstd)
  const void* w1f;                 // W1' as f16 MFMA A fragments (gffn_pack)
  const float* tbp;                // [2 hd] W1 b_ln + b1 in the fragments' row order
  const uint32_t* dwp;             // depthwise taps + bias as f16 pairs in P2 lane order
  const void* w2f;                 // W2 as f16 MFMA A fragments
  const float* b2;                 // [C] project_out bias or null
  int dbg;                         // tools/gfbench ablations (0 in the product path)
};
struct GffnHost {                  // gffn_pack output (host), uploaded as four segments
  std::vector<uint16_t> w1f, w2f;
  std::vector<float> tbp;
  std::vector<uint32_t> dwp;
};
bool gffn_ok(const GffnArgs& a);
int64_t gffn_blocks(const GffnArgs& a);
void launch_gffn(const GffnArgs& a, hipStream_t st);
// w1 [2 hd][256] (LayerNorm weight folded), tb [2 hd] (or empty), dw9 [9][2 hd] tap-major, dwb [2 hd] (or
// empty), w2 [256][hd]
void gffn_pack(int C, int hd, const std::vector<double>& w1, const std::vector<double>& tb, const std::vector<double>& dw9,
               const std::vector<double>& dwb, const std::vector<double>& w2, GffnHost& o);

struct FfnArgs {                   // ffn.hip: out = x + g2 * (W2 gelu(LN-folded W1 x) + b2), bf16, C in {64, 128}
  const void* x; void* out;        // [M][C] pixel-major; out may alias x
  int64_t M; int C;
  const void* w1f; const void* w2f;   // W1' [2C][C] / W2 [C][2C] in MFMA A-fragment order (turtle.cpp pack_ffn_frags)
  const float* s1; const float* t1;   // [2C] rowsum(W1'), W1 b_ln + b1 (null: 0)
  const float* b2; const float* g2;   // [C] conv5 bias, gamma (null: 0 / 1)
};
bool ffn_ok(const FfnArgs& a);
void launch_ffn(const FfnArgs& a, hipStream_t st);

void launch_cast_f32(const float* src, void* dst, int64_t n, int to_bf16, hipStream_t st);

// t0 StateAlignBlock (turtle_arch.py:459-533), t0.hip
struct T0PeArgs {                  // 2-D sinusoidal encoding (turtle_arch.py:412-439), [H*W][C]
  void* out; int H, W, C;
};
template <typename T> void launch_t0_pe(const T0PeArgs& a, hipStream_t st);
struct T0KnormArgs {               // k[b][n][:] = normalize(k[b][n][:] + kpos[n][:]) over D features
  void* k; int64_t k_bstride; const void* kpos; int B, N, D;
};
template <typename T> void launch_t0_knorm(const T0KnormArgs& a, hipStream_t st);
struct T0UntokArgs {               // out[b*T + t] = inverse dilated regroup of v token frame t
  const void* v[TURTLE_MAX_T]; int64_t v_bstride[TURTLE_MAX_T];   // [N][ws*ws*C]
  void* out; int B, T, H, W, C, ws;
};
template <typename T> void launch_t0_untok(const T0UntokArgs& a, hipStream_t st);

}  // namespace turtle

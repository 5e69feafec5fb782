// libturtle_hip: weight packing, frame driver and the C ABI (include/turtle_hip.h).
//
// The frame driver issues the per-frame kernel sequence of Turtle_t1.forward
// (turtle_t1_arch.py:1045-1132) on the caller's stream. Every block is restructured around the
// HBM roofline: LayerNorm is folded into the following pointwise GEMM, attention outputs are
// folded into the projection weights (W_eff), GELU / gate / bias / scale / residual live in
// epilogues, skip concats are multi-source GEMM operands and the SAB never materialises N x N.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/turtle_hip.h"
#include "kernels.h"

using namespace turtle;

static thread_local std::string g_err;

struct TurtleError : std::runtime_error {
  int code;
  TurtleError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};
#define TFAIL(code, msg) throw TurtleError(code, msg)
namespace turtle {
[[noreturn]] void kernel_arg_error(const char* what) { TFAIL(TURTLE_EINVAL, what); }
}
#define HIPCHK(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) TFAIL(TURTLE_EHIP, std::string(#x ": ") + hipGetErrorString(e_)); \
  } while (0)

static const size_t NONE = (size_t)-1;

// ------------------------------------------------------------------------------------------
// architecture (mirror of turtlevsr_amd/arch.py, itself make_model + Turtle_t1.__init__)
// ------------------------------------------------------------------------------------------
struct Blk {
  std::string prefix;
  int dim, attn, ffn, heads, ntc, ws, hidden;
  int level;          // 0..7 index into Arch::levels
  int cache_slot;     // -1 or 0..7 (only the cache-carrying block of a level)
};

struct Level {
  std::string name;
  int dim;
  int scale;          // pixels per side relative to the padded frame (1, 2, 4, 8)
  std::vector<Blk> blocks;
};

struct Arch {
  TurtleConfig cfg;
  int dim, in_ch, out_ch;
  std::vector<Level> levels;   // encoder_level1..3, latent, decoder_level3..1, refinement
  std::vector<std::pair<std::string, std::vector<int64_t>>> params;   // state_dict order
};

static const char* attn_name(int a) {
  switch (a) {
    case TURTLE_ATTN_REDUCED: return "ReducedAttn";
    case TURTLE_ATTN_CHANNEL: return "Channel";
    case TURTLE_ATTN_FHR: return "FHR";
    case TURTLE_ATTN_CHM: return "CHM";
    case TURTLE_ATTN_NONE: return "NoAttn";
  }
  return "?";
}

static void build_arch(Arch& A) {
  const TurtleConfig& c = A.cfg;
  if (c.dim <= 0 || c.dim % 8) TFAIL(TURTLE_EINVAL, "dim must be a positive multiple of 8");
  if (c.n_colors < 1 || c.n_colors > 4) TFAIL(TURTLE_EINVAL, "n_colors must be 1..4");
  if (c.middle_blocks < 2) TFAIL(TURTLE_EINVAL, "LatentCacheBlock should have more than 2 layers (turtle_t1_arch.py:899-901)");
  if (c.super_resolution && c.use_both_input) TFAIL(TURTLE_EINVAL, "TurtleSuper_t1 with use_both_input is not runnable in the reference");
  if (c.variant != 0 && c.variant != 1) TFAIL(TURTLE_EINVAL, "variant must be 0 (Turtle_t1) or 1 (t0 Turtle)");
  if (c.variant == 1 && c.super_resolution) TFAIL(TURTLE_EINVAL, "the super-resolution network is t1 only (turtlesuper_t1_arch.py)");
  A.dim = c.dim;
  A.in_ch = c.n_colors * (c.use_both_input ? 2 : 1);
  A.out_ch = c.n_colors;
  const int d = c.dim, ntc = c.num_frames_tocache;
  auto chk = [](int at, int ft) {
    if (at < 0 || at > 4) TFAIL(TURTLE_EINVAL, "attention type not defined (turtle_t1_arch.py:790-792)");
    if (ft < 0 || ft > 1) TFAIL(TURTLE_EINVAL, "FFW type not defined (turtle_t1_arch.py:800-802)");
  };
  auto level = [&](const char* name, int dd, int scale, int n, int t1, int t2, int ffn, int heads, int nt, int sp, int slot) {
    Level L{name, dd, scale, {}};
    for (int i = 0; i < n; ++i) {
      int at = i == n - 1 ? t2 : t1;
      chk(at, ffn);
      Blk b{std::string(name) + ".transformer_blocks." + std::to_string(i), dd, at, ffn, heads, nt, 2 * sp,
            (int)(dd * c.ffn_expansion_factor), (int)A.levels.size(), i == n - 1 ? slot : -1};
      L.blocks.push_back(b);
    }
    A.levels.push_back(L);
  };
  level("encoder_level1", d, 1, c.enc_blocks[0], c.level_attn[0][0], c.level_attn[0][1], c.level_ffn[0], c.num_heads[0], ntc, 1, 0);
  level("encoder_level2", 2 * d, 2, c.enc_blocks[1], c.level_attn[1][0], c.level_attn[1][1], c.level_ffn[1], c.num_heads[1], ntc, 1, 1);
  level("encoder_level3", 4 * d, 4, c.enc_blocks[2], c.level_attn[2][0], c.level_attn[2][1], c.level_ffn[2], c.num_heads[2], ntc, 1, 2);
  {
    Level L{"latent", 8 * d, 8, {}};
    const int n = c.middle_blocks;
    for (int i = 0; i < n; ++i) {
      int at = i == 0 ? c.latent_attn[0] : (i == n - 1 ? c.latent_attn[2] : c.latent_attn[1]);
      chk(at, c.latent_ffn);
      Blk b{"latent.transformer_blocks." + std::to_string(i), 8 * d, at, c.latent_ffn, c.num_heads[3], ntc, 2,
            (int)(8 * d * c.ffn_expansion_factor), 3, i == 0 ? 3 : (i == n - 1 ? 4 : -1)};
      L.blocks.push_back(b);
    }
    A.levels.push_back(L);
  }
  level("decoder_level3", 4 * d, 4, c.dec_blocks[0], c.level_attn[3][0], c.level_attn[3][1], c.level_ffn[3], c.num_heads[2], ntc, 2, 5);
  level("decoder_level2", 2 * d, 2, c.dec_blocks[1], c.level_attn[4][0], c.level_attn[4][1], c.level_ffn[4], c.num_heads[1], ntc, 4, 6);
  level("decoder_level1", d, 1, c.dec_blocks[2], c.level_attn[5][0], c.level_attn[5][1], c.level_ffn[5], c.num_heads[0], 2, 8, 7);
  level("refinement", d, 1, c.num_refinement_blocks, c.level_attn[6][0], c.level_attn[6][1], c.level_ffn[6], c.num_heads[0], ntc, 1, -1);
  for (auto& L : A.levels) {
    if (L.blocks.empty()) TFAIL(TURTLE_EINVAL, "every level needs >= 1 block");
    for (auto& b : L.blocks) {
      if (b.hidden % 8) TFAIL(TURTLE_EINVAL, "GatedFeedForward hidden width must be a multiple of 8");
      if (b.attn != TURTLE_ATTN_REDUCED && b.attn != TURTLE_ATTN_NONE) {
        if (b.heads <= 0 || b.dim % b.heads || (b.dim / b.heads) % 16)
          TFAIL(TURTLE_EINVAL, "channels per head must be a multiple of 16");
      }
    }
  }

  // state_dict entries in registration order (see turtlevsr_amd/params.py)
  auto P = [&](const std::string& n, std::vector<int64_t> s) { A.params.push_back({n, s}); };
  auto conv = [&](const std::string& n, int cin, int cout, int k, int groups, bool bias) {
    P(n + ".weight", {cout, cin / groups, k, k});
    if (bias) P(n + ".bias", {cout});
  };
  const bool bias = c.bias != 0;
  auto ln = [&](const std::string& n, int ch) {
    P(n + ".body.weight", {ch});
    if (!c.layernorm_biasfree) P(n + ".body.bias", {ch});
  };
  auto chan = [&](const std::string& n, int ch, int heads) {
    P(n + ".temperature", {heads, 1, 1});
    conv(n + ".qkv", ch, 3 * ch, 1, 1, bias);
    conv(n + ".qkv_dwconv", 3 * ch, 3 * ch, 3, 3 * ch, bias);
    conv(n + ".project_out", ch, ch, 1, 1, bias);
  };
  auto block = [&](const Blk& b) {
    const int ch = b.dim;
    ln(b.prefix + ".norm1", ch);
    const std::string a = b.prefix + ".attn";
    if (b.attn == TURTLE_ATTN_REDUCED) {
      P(a + ".beta", {1, ch, 1, 1});
      conv(a + ".conv1", ch, 2 * ch, 1, 1, true);
      conv(a + ".conv2", 2 * ch, 2 * ch, 3, 2 * ch, true);
      conv(a + ".conv3", 2 * ch, ch, 1, 1, true);
    } else if (b.attn == TURTLE_ATTN_CHANNEL || b.attn == TURTLE_ATTN_FHR) {
      chan(a, ch, b.heads);
    } else if (b.attn == TURTLE_ATTN_CHM) {
      const std::string s = a + ".spatial_aligner";
      P(s + ".temperature", {1, 1, 1});
      conv(s + ".qk", ch, 2 * ch, 1, 1, bias);
      conv(s + ".qk_dwconv", 2 * ch, 2 * ch, 3, 2 * ch, bias);
      conv(s + ".v", ch, ch, 1, 1, bias);
      conv(s + ".v_dwconv", ch, ch, 3, ch, bias);
      conv(s + ".k2", ch, 2 * ch, 1, 1, bias);
      conv(s + ".k2_dwconv", 2 * ch, 2 * ch, b.ws, 2 * ch, bias);
      conv(s + ".q2", ch, 2 * ch, 1, 1, bias);
      conv(s + ".q2_dwconv", 2 * ch, 2 * ch, b.ws, 2 * ch, bias);
      conv(s + ".project_out", ch, ch, 1, 1, bias);
      chan(a + ".ChanAttn", ch, b.heads);
      conv(a + ".kv", ch, 2 * ch, 1, 1, bias);
      conv(a + ".kv_dwconv", 2 * ch, 2 * ch, 3, 2 * ch, bias);
    }
    ln(b.prefix + ".norm2", ch);
    const std::string f = b.prefix + ".ffn";
    if (b.ffn == TURTLE_FFN_GFFW) {
      conv(f + ".project_in", ch, 2 * b.hidden, 1, 1, bias);
      conv(f + ".dwconv", 2 * b.hidden, 2 * b.hidden, 3, 2 * b.hidden, bias);
      conv(f + ".project_out", b.hidden, ch, 1, 1, bias);
    } else {
      P(f + ".gamma", {1, ch, 1, 1});
      conv(f + ".conv4", ch, 2 * ch, 1, 1, true);
      conv(f + ".conv5", 2 * ch, ch, 1, 1, true);
    }
  };
  auto lvl = [&](int i) { for (auto& b : A.levels[i].blocks) block(b); };
  conv("input_projection", A.in_ch, d, 3, 1, bias);
  lvl(0); conv("down1_2.body.0", d, d / 2, 3, 1, false);
  lvl(1); conv("down2_3.body.0", 2 * d, d, 3, 1, false);
  lvl(2); conv("down3_4.body.0", 4 * d, 2 * d, 3, 1, false);
  lvl(3);
  conv("up4_3.body.0", 8 * d, 16 * d, 3, 1, false); conv("reduce_chan_level3", 8 * d, 4 * d, 1, 1, bias); lvl(4);
  conv("up3_2.body.0", 4 * d, 8 * d, 3, 1, false); conv("reduce_chan_level2", 4 * d, 2 * d, 1, 1, bias); lvl(5);
  conv("up2_1.body.0", 2 * d, 4 * d, 3, 1, false); conv("reduce_chan_level1", 2 * d, d, 1, 1, bias); lvl(6);
  lvl(7);
  conv("ending", d, A.out_ch, 3, 1, true);
}

// ------------------------------------------------------------------------------------------
// packed weights
// ------------------------------------------------------------------------------------------
struct GemmW {
  size_t w = NONE, s = NONE, t = NONE, bias = NONE, scale = NONE;
  size_t tb = NONE;   // LN GEMMs: W b_ln + bias (the vendor path's bias after an explicit LN prologue)
  int N = 0, K = 0; bool ln = false;
};
struct DwW { size_t w = NONE, bias = NONE, w2 = NONE, w16 = NONE; int C = 0; };   // w2: bf16 tap pairs [5][C] (u32); w16: bf16 [9][C]
struct BlockW {
  GemmW a_in, a_out, q2, k2, kv, f_in, f_out, t0_kpw;   // t0_kpw: W_k of the t0 aligner (pos term)
  DwW t0_kdw;                                           // t0 k-half depthwise taps without bias
  DwW a_dw, sab_qk_dw, sab_v_dw, fhr_dw, kv_dw, f_dw, chm_dw6;
  DwW a_dw_qk, a_dw_v;
  size_t ffn_w1f = NONE, ffn_w2f = NONE;                // FeedForward conv4' / conv5 in MFMA fragment order (ffn.hip)
  size_t gf_w1f = NONE, gf_tbp = NONE, gf_dwp = NONE, gf_w2f = NONE;
  int gf_hd = 0;                                  // gffn's hidden width (level 1: 160 padded to 192 with zero weights)   // GatedFeedForward at width 256 as one kernel (gffn.hip)                                  // channel attention: qkv_dwconv split (q,k | v) for the dwgemm v path
  size_t q2_win = NONE, q2_winb = NONE, k2_win = NONE, k2_winb = NONE, sab_tau = NONE;
  size_t wp = NONE, po_bias = NONE, tau = NONE;   // channel-attention projection (fp32) + temperature
};
struct ModelW {
  size_t stem_w = NONE, stem_b = NONE, end_w = NONE, end_b = NONE;
  size_t end_wf = NONE;                      // ending 3x3 as bf16 MFMA A fragments [9 Cin / 32][64 lanes][8] (spatial.hip)
  size_t down_wf = NONE;                     // level-1 Downsample 3x3 as bf16 A fragments [Cout / 16][9 Cin / 32][64][8] (down_tile_kernel)
  size_t zeros = NONE, ones = NONE;          // constant vectors for branch-free kernel operands
  GemmW down[3], up[3], reduce[3];
  bool reduce_split = false;                 // reduce[2] packed as split-bf16 [W_hi | W_lo] (K doubled)
  std::vector<std::vector<BlockW>> blocks;   // [level][block]
};

struct Packer {
  std::vector<char> host;
  bool bf16;
  size_t align(size_t a = 256) { size_t o = (host.size() + a - 1) / a * a; host.resize(o); return o; }
  size_t f32(const std::vector<double>& v) {
    size_t o = align();
    host.resize(o + v.size() * 4);
    float* p = reinterpret_cast<float*>(host.data() + o);
    for (size_t i = 0; i < v.size(); ++i) p[i] = (float)v[i];
    return o;
  }
  template <typename E>
  size_t raw(const std::vector<E>& v) {
    size_t o = align();
    host.resize(o + v.size() * sizeof(E));
    std::memcpy(host.data() + o, v.data(), v.size() * sizeof(E));
    return o;
  }
  size_t u32(const std::vector<uint32_t>& v) {
    size_t o = align();
    host.resize(o + v.size() * 4);
    std::memcpy(host.data() + o, v.data(), v.size() * 4);
    return o;
  }
  static uint16_t bf16_bits(double x) {
    float f = (float)x;
    uint32_t u; std::memcpy(&u, &f, 4);
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
  }
  static double bf16_value(double x) {
    const uint32_t u = (uint32_t)bf16_bits(x) << 16;
    float f; std::memcpy(&f, &u, 4);
    return f;
  }
  // depthwise 3x3 table [9][C] -> bf16 tap pairs [5][C]: lo = tap 2i, hi = tap 2i+1 (0 for tap 9),
  // the operand layout of v_dot2_f32_bf16 in the fused kernel's depthwise stage
  size_t dw_pairs(const std::vector<double>& w9, int C) {
    std::vector<uint32_t> o((size_t)5 * C);
    for (int i = 0; i < 5; ++i)
      for (int c = 0; c < C; ++c) {
        const uint32_t lo = bf16_bits(w9[(size_t)(2 * i) * C + c]);
        const uint32_t hi = 2 * i + 1 < 9 ? bf16_bits(w9[(size_t)(2 * i + 1) * C + c]) : 0u;
        o[(size_t)i * C + c] = lo | (hi << 16);
      }
    return u32(o);
  }
  // storage-typed matrix; returns offset and writes back the rounded values (for LN rowsums)
  // depthwise 3x3 table [9][C] as bf16 (the dwgemm kernel's block-diagonal MFMA operand)
  size_t bf16tab(const std::vector<double>& w9) {
    size_t o = align();
    host.resize(o + w9.size() * 2);
    uint16_t* p = reinterpret_cast<uint16_t*>(host.data() + o);
    for (size_t i = 0; i < w9.size(); ++i) p[i] = bf16_bits(w9[i]);
    return o;
  }
  size_t stor(std::vector<double>& v) {
    size_t o = align();
    if (bf16) {
      host.resize(o + v.size() * 2);
      uint16_t* p = reinterpret_cast<uint16_t*>(host.data() + o);
      for (size_t i = 0; i < v.size(); ++i) {
        float f = (float)v[i];
        uint32_t u; std::memcpy(&u, &f, 4);
        uint32_t r = (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
        p[i] = (uint16_t)r;
        uint32_t back = r << 16; float fb; std::memcpy(&fb, &back, 4);
        v[i] = fb;
      }
    } else {
      host.resize(o + v.size() * 4);
      float* p = reinterpret_cast<float*>(host.data() + o);
      for (size_t i = 0; i < v.size(); ++i) { p[i] = (float)v[i]; v[i] = p[i]; }
    }
    return o;
  }
};

struct ProfRec { int cls; hipEvent_t a, b; double bytes, flops; std::string tag; };

struct TurtleHandle {
  Arch arch;
  int prof_cls = -1;
  std::vector<ProfRec> prof;
  std::string prof_tag;                               // shape note of the next launch (per-launch dump)
  std::string prof_filter;                            // non-empty: profile only launches with this tag
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  std::map<std::string, std::vector<float>> staged;
  ModelW mw;
  char* dev = nullptr;
  size_t dev_bytes = 0;
  bool loaded = false;
  bool fuse = getenv("TURTLE_NO_FUSE") == nullptr;   // block-level fused kernels (fused.hip)
  bool fuse_fp32 = false;                             // fp32 build: the round-1 fused block kernel (fused.hip) instead of GEMM + dw +
                                                      // GEMM (540p fp32 16.6 -> 20.5 frames/s without it: profiles/r04o_*)
  bool fused2 = true;                                 // bf16 row-walk fused kernels (fused2.hip) where eligible
  bool panel = getenv("TURTLE_NO_PANEL") == nullptr; // panel GEMM (gemm.hip)
  bool dw_rows = true;                                // row-sweeping depthwise kernel (spatial.hip)
  bool gemm_lds = true;                               // LDS-pipelined bf16 GEMM (gemm2.hip)
  bool gemm_pn = true;                                // resident-panel bf16 GEMM, K <= 512 (gemm3.hip)
  bool gemm_ar = true;                                // A-resident per-panel bf16 GEMM, K 256..1280 (gemm3.hip)
  bool gemm_kt = true;                                // 2-D tiled deep-ring bf16 GEMM (gemm5.hip)
  bool gemm_f32 = true;                               // fp32 occupancy-tiled GEMM (gemm_f32.hip)
  bool gemm_sk = true;                                // split-K bf16 GEMM for the small-frame wide projections (gemm_sk.hip)
  int64_t sk_max_px = 4096;                           // ... for GEMMs over at most this many pixels (set before sizing the workspace)
  int kt_max_px = 32768;                              // below this many pixels the 2-D tiled GEMM takes every shape it can
  int sab_waves = 0;                                  // waves per SAB score block: 4 (64 queries), 8 (128), 0 = 8 at
                                                      // d >= 256, else 4 (tools/sabbench, profiles/r04_sabbench_waves.log)
  bool attn_fin = false;                              // channel-attention softmax rows inside the W_eff kernel (attn.hip)
  bool gemm8_ps = false;                              // ... in its persistent form (one block per CU walks its tiles)
  int gemm8 = 3;                                      // 256 x 256 four-phase bf16 GEMM (gemm8.hip): 1 for the
                                                      // 'wide' projection class (below), 2 every eligible projection
  int gemm9 = 1;                                      // 256-pixel-row bf16 GEMM (gemm9.hip): 1 for the 'wide'
                                                      // projection class (below), 2 every eligible projection, 0 off
  bool stem_mfma = true;                              // bf16 matrix-core stem / ending (spatial.hip)
  int sab_db = 0;                                     // SAB A.v: 0 two blocks / CU; 1 double-buffered, one block / CU;
                                                      // 2 two blocks / CU with the tail rows fetched a chunk ahead
  bool sab_mfma = true;                               // matrix-core SAB A.v over query tiles (sab.hip)
  bool dwgemm = true;                                 // depthwise (+ gate) folded into the next GEMM's operand, c >= 256 (dwgemm.hip)
  int gram_blocks = getenv("TURTLE_GRAM_BLOCKS") ? atoi(getenv("TURTLE_GRAM_BLOCKS")) : 512;   // Gram pixel splits: blocks over all (b, head)
  bool tilepd = true;                                 // level-3 LN -> qkv -> qkv_dwconv in one kernel (tilepd.hip)
  bool tilepd_gate = false;                           // ... and the GatedFeedForward's project_in -> dwconv -> gate (slower
                                                      // than the pn GEMM + dwgemm pair it replaces: profiles/r04h_*)
  bool tilepd_cb = true;                              // tilepd GATE output channel-blocked (read by the 2-D tiled GEMM)
  int tilepd_min_blocks = 256;                        // one block per CU: below one full round the GEMM + dw path stays
  bool ffn = true;                                    // FeedForward as one kernel at widths 64 / 128 (ffn.hip)
  bool gffn = true;                                   // GatedFeedForward at width 256 as one kernel (gffn.hip): the hidden
                                                      // map never in HBM (instead of the pn GEMM + dwgemm pair)
  int gffn_min_blocks = 256;                          // one block per CU: below one full round the GEMM path stays
  bool gffn_c128 = true;                              // ... also at width 128 (level 2) instead of the fused2 row walk
                                                      // (1080p: 364 vs 421 us per launch)
  bool gffn_c64 = false;                              // ... and at width 64 (level 1, hidden padded to a multiple of 64):
                                                      // measured slower than the fused2 walk (812 vs 607 us), off
  bool dwgemm_cb = true;                              // GatedFeedForward hidden map channel-blocked for dwgemm (STORE_CB16)
  bool down_tile = true;                              // level-1 Downsample as the LDS-tiled conv kernel (spatial.hip down_tile_kernel)
  bool split_out = true;                              // split-bf16 weights for reduce_chan_level1 (bf16 builds)
  bool dwgemm_attn = true;                            // channel attention: v's depthwise inside the W_eff GEMM (dwgemm.hip)
  int dwgemm_min_blocks = 384;                        // one 160 KB block per CU: below ~1.5 rounds (latent level) dw + GEMM is faster
  bool bf16() const { return arch.cfg.dtype == TURTLE_DTYPE_BF16; }
  const void* ptr(size_t off) const { return off == NONE ? nullptr : dev + off; }
  const float* fptr(size_t off) const { return reinterpret_cast<const float*>(ptr(off)); }
};

static const std::vector<float>& W(TurtleHandle* h, const std::string& n) {
  auto it = h->staged.find(n);
  if (it == h->staged.end()) TFAIL(TURTLE_ENOWEIGHT, "missing weight " + n);
  return it->second;
}
static bool has(TurtleHandle* h, const std::string& n) { return h->staged.count(n) != 0; }
static std::vector<double> dvec(const std::vector<float>& v) { return std::vector<double>(v.begin(), v.end()); }

// 1x1 conv [N][K] (+bias), optionally LayerNorm-folded with norm `lnname`; rows [r0, r1) of W
static void pack_rows(const std::vector<float>& w, int K, int r0, int r1, std::vector<double>& out) {
  for (int r = r0; r < r1; ++r)
    for (int k = 0; k < K; ++k) out.push_back(w[(size_t)r * K + k]);
}

static GemmW pack_gemm(TurtleHandle* h, Packer& pk, std::vector<double> Wm, int N, int K,
                       const std::string& lnname, std::vector<double> bias) {
  GemmW g; g.N = N; g.K = K;
  std::vector<double> s, t;
  if (!lnname.empty()) {
    g.ln = true;
    const auto& gw = W(h, lnname + ".body.weight");
    const bool bf = h->arch.cfg.layernorm_biasfree != 0;
    std::vector<double> orig = Wm;
    for (int n = 0; n < N; ++n)
      for (int k = 0; k < K; ++k) Wm[(size_t)n * K + k] *= gw[k];
    g.w = pk.stor(Wm);   // rounds Wm in place
    if (!bf) {
      const auto& gb = W(h, lnname + ".body.bias");
      s.assign(N, 0.0); t.assign(N, 0.0);
      for (int n = 0; n < N; ++n)
        for (int k = 0; k < K; ++k) { s[n] += Wm[(size_t)n * K + k]; t[n] += orig[(size_t)n * K + k] * gb[k]; }
      g.s = pk.f32(s); g.t = pk.f32(t);
    }
  } else {
    g.w = pk.stor(Wm);
  }
  if (!bias.empty()) g.bias = pk.f32(bias);
  if (g.ln) {
    std::vector<double> tb(N, 0.0);
    for (int n = 0; n < N; ++n) tb[n] = (t.empty() ? 0.0 : t[n]) + (bias.empty() ? 0.0 : bias[n]);
    g.tb = pk.f32(tb);
  }
  return g;
}

static std::vector<double> opt_bias(TurtleHandle* h, const std::string& n) {
  return has(h, n) ? dvec(W(h, n)) : std::vector<double>();
}

static DwW pack_dw(TurtleHandle* h, Packer& pk, const std::string& n, int c0, int C, int taps = 9, bool with_bias = true) {
  // conv weight [Ctot][1][k][k] -> [taps][C] for channels [c0, c0 + C)
  const auto& w = W(h, n + ".weight");
  std::vector<double> o((size_t)taps * C);
  for (int c = 0; c < C; ++c)
    for (int t = 0; t < taps; ++t) o[(size_t)t * C + c] = w[(size_t)(c0 + c) * taps + t];
  DwW d; d.C = C; d.w = pk.f32(o);
  if (taps == 9) { d.w2 = pk.dw_pairs(o, C); d.w16 = pk.bf16tab(o); }
  if (with_bias && has(h, n + ".bias")) {
    const auto& b = W(h, n + ".bias");
    d.bias = pk.f32(std::vector<double>(b.begin() + c0, b.begin() + c0 + C));
  }
  return d;
}

// several depthwise 3x3 convs side by side -> one [9][sum C] table (fused multi-output dw)
static DwW pack_dw_cat(TurtleHandle* h, Packer& pk, const std::vector<std::string>& names, const std::vector<int>& cs,
                       std::vector<int> c0s = {}) {
  c0s.resize(names.size(), 0);
  int Ct = 0;
  for (int c : cs) Ct += c;
  std::vector<double> o((size_t)9 * Ct), bias;
  bool any_bias = false;
  for (auto& n : names) any_bias |= has(h, n + ".bias");
  int c0 = 0;
  for (size_t i = 0; i < names.size(); ++i) {
    const auto& w = W(h, names[i] + ".weight");
    for (int c = 0; c < cs[i]; ++c)
      for (int t = 0; t < 9; ++t) o[(size_t)t * Ct + c0 + c] = w[(size_t)(c0s[i] + c) * 9 + t];
    if (any_bias)
      for (int c = 0; c < cs[i]; ++c) bias.push_back(has(h, names[i] + ".bias") ? W(h, names[i] + ".bias")[c0s[i] + c] : 0.0);
    c0 += cs[i];
  }
  DwW d; d.C = Ct; d.w = pk.f32(o);
  d.w2 = pk.dw_pairs(o, Ct);
  d.w16 = pk.bf16tab(o);
  if (any_bias) d.bias = pk.f32(bias);
  return d;
}

// dense 3x3 [Cout][Cin][3][3] -> [Cout'][9][Cin], with an optional output-channel permutation
static GemmW pack_conv3(TurtleHandle* h, Packer& pk, const std::string& n, int Cin, int Cout, bool shuffle_perm) {
  const auto& w = W(h, n + ".weight");
  std::vector<double> o((size_t)Cout * 9 * Cin);
  const int Cq = Cout / 4;
  for (int np = 0; np < Cout; ++np) {
    // PixelShuffle(2): input channel c*4 + s -> output channel c at sub-pixel s; store row s*Cq + c
    const int src = shuffle_perm ? (np % Cq) * 4 + np / Cq : np;
    for (int ci = 0; ci < Cin; ++ci)
      for (int t = 0; t < 9; ++t) o[((size_t)np * 9 + t) * Cin + ci] = w[((size_t)src * Cin + ci) * 9 + t];
  }
  GemmW g; g.N = Cout; g.K = 9 * Cin; g.w = pk.stor(o);
  return g;
}

// FeedForward weights for ffn.hip: the bf16 matrices already packed at host offsets w1 ([2C][C],
// LN-folded) and w2 ([C][2C]) re-laid as 16x16x32 MFMA A fragments (1 KB: lane l, 8 bf16 at l * 16).
// W1 fragment (hc, s, ks): row l & 15 = 4 g' + e' -> hidden 32 hc + 8 g' + 4 s + e', k = 32 ks + 8 (l >> 4) + j;
// W2 fragment (hc, t): row -> output 32 (t >> 1) + 8 g' + 4 (t & 1) + e', k = 32 hc + 8 (l >> 4) + j
static void pack_ffn_frags(Packer& pk, size_t w1, size_t w2, int C, size_t& o1, size_t& o2) {
  const int H = 2 * C, KS1 = C / 32, HC = H / 32, T2 = C / 16;
  std::vector<uint16_t> a((size_t)H * C), b((size_t)C * H), fa(a.size()), fb(b.size());
  std::memcpy(a.data(), pk.host.data() + w1, a.size() * 2);
  std::memcpy(b.data(), pk.host.data() + w2, b.size() * 2);
  for (int hc = 0; hc < HC; ++hc)
    for (int s = 0; s < 2; ++s)
      for (int ks = 0; ks < KS1; ++ks)
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 8; ++j) {
            const int m = l & 15, hrow = 32 * hc + 8 * (m >> 2) + 4 * s + (m & 3), k = 32 * ks + 8 * (l >> 4) + j;
            fa[((((size_t)(hc * 2 + s) * KS1 + ks) * 64 + l) * 8) + j] = a[(size_t)hrow * C + k];
          }
  for (int hc = 0; hc < HC; ++hc)
    for (int t = 0; t < T2; ++t)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 8; ++j) {
          const int m = l & 15, orow = 32 * (t >> 1) + 8 * (m >> 2) + 4 * (t & 1) + (m & 3), k = 32 * hc + 8 * (l >> 4) + j;
          fb[(((size_t)(hc * T2 + t) * 64 + l) * 8) + j] = b[(size_t)orow * H + k];
        }
  o1 = pk.align();
  pk.host.resize(o1 + fa.size() * 2);
  std::memcpy(pk.host.data() + o1, fa.data(), fa.size() * 2);
  o2 = pk.align();
  pk.host.resize(o2 + fb.size() * 2);
  std::memcpy(pk.host.data() + o2, fb.data(), fb.size() * 2);
}

static void pack_all(TurtleHandle* h) {
  Arch& A = h->arch;
  Packer pk; pk.bf16 = h->bf16();
  ModelW& M = h->mw;
  M.reduce_split = false;
  M.down_wf = NONE;
  const int d = A.dim;
  M.stem_w = pk.f32(dvec(W(h, "input_projection.weight")));
  if (has(h, "input_projection.bias")) M.stem_b = pk.f32(dvec(W(h, "input_projection.bias")));
  M.end_w = pk.f32(dvec(W(h, "ending.weight")));
  {
    // A fragment s, lane l: output channel l & 15 (< Cimg, else 0), k = 32 s + 8 (l >> 4) + j -> (tap, ci)
    const auto& ew = W(h, "ending.weight");
    const int cin = d, cimg = (int)(ew.size() / ((size_t)cin * 9));
    // split-bf16 weights: A rows 0..3 hold bf16(w), rows 4..7 the bf16 rounding of the remainder
    // w - bf16(w), summed in the kernel epilogue (~16-bit weight mantissa at no MFMA cost: the ending
    // is the layer whose weight rounding moves the output PSNR most, tools/psnr_probe.py --by-module)
    if (cin % 32 == 0 && cimg <= 4) {
      const int ks = 9 * cin / 32;
      std::vector<double> f((size_t)ks * 64 * 8, 0.0);
      for (int s = 0; s < ks; ++s)
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 8; ++j) {
            const int k = s * 32 + (l >> 4) * 8 + j, tap = k / cin, ci = k - tap * cin, row = l & 15, co = row & 3;
            if (co >= cimg || row >= (h->split_out ? 8 : 4)) continue;
            const double w = ew[((size_t)co * cin + ci) * 9 + tap];
            f[((size_t)s * 64 + l) * 8 + j] = row < 4 ? w : w - Packer::bf16_value(w);
          }
      M.end_wf = pk.bf16tab(f);
    }
  }
  M.end_b = pk.f32(dvec(W(h, "ending.bias")));
  const char* downs[3] = {"down1_2.body.0", "down2_3.body.0", "down3_4.body.0"};
  const char* ups[3] = {"up4_3.body.0", "up3_2.body.0", "up2_1.body.0"};
  const char* reds[3] = {"reduce_chan_level3", "reduce_chan_level2", "reduce_chan_level1"};
  for (int i = 0; i < 3; ++i) {
    const int c = d << i;                 // down i: level i channels -> c/2 (then unshuffle x4)
    M.down[i] = pack_conv3(h, pk, downs[i], c, c / 2, false);
    if (i == 0 && pk.bf16 && c == 64) {
      // A fragments of the tiled kernel: fragment (ct, s), lane l: output channel 16 ct + (l & 15),
      // k = 32 s + 8 (l >> 4) + j -> (tap = k / c, ci = k % c); weight [c/2][c][3][3]
      const auto& dwt = W(h, std::string(downs[i]) + ".weight");
      const int co_n = c / 2, ks = 9 * c / 32;
      std::vector<double> f((size_t)(co_n / 16) * ks * 64 * 8, 0.0);
      for (int ct = 0; ct < co_n / 16; ++ct)
        for (int s2 = 0; s2 < ks; ++s2)
          for (int l = 0; l < 64; ++l)
            for (int j = 0; j < 8; ++j) {
              const int k = s2 * 32 + (l >> 4) * 8 + j, tap = k / c, ci = k - tap * c, co = ct * 16 + (l & 15);
              f[(((size_t)ct * ks + s2) * 64 + l) * 8 + j] = dwt[((size_t)co * c + ci) * 9 + tap];
            }
      M.down_wf = pk.bf16tab(f);
    }
    const int cu = d << (3 - i);          // up i: level (3-i) channels -> 2c, shuffled to c/2
    M.up[i] = pack_conv3(h, pk, ups[i], cu, 2 * cu, true);
    const int cr = cu;                    // reduce: cat(up c/2, skip c/2) = cu -> cu/2
    std::vector<double> rw = dvec(W(h, std::string(reds[i]) + ".weight"));
    if (i == 2 && pk.bf16 && h->split_out) {
      // reduce_chan_level1 (the last 1x1 before the full-resolution decoder, second in output-PSNR
      // sensitivity to weight rounding): split-bf16 weights [W_hi | W_lo], K doubled over the
      // sources [up, skip, up, skip] (turtle.cpp upcat)
      std::vector<double> w2;
      for (int n = 0; n < cr / 2; ++n) {
        for (int k = 0; k < cr; ++k) w2.push_back(Packer::bf16_value(rw[(size_t)n * cr + k]));
        for (int k = 0; k < cr; ++k) w2.push_back(rw[(size_t)n * cr + k] - Packer::bf16_value(rw[(size_t)n * cr + k]));
      }
      M.reduce[i] = pack_gemm(h, pk, w2, cr / 2, 2 * cr, "", opt_bias(h, std::string(reds[i]) + ".bias"));
      M.reduce_split = true;
    } else {
      M.reduce[i] = pack_gemm(h, pk, rw, cr / 2, cr, "", opt_bias(h, std::string(reds[i]) + ".bias"));
    }
  }
  M.blocks.clear();
  for (auto& L : A.levels) {
    std::vector<BlockW> bws;
    for (auto& b : L.blocks) {
      BlockW bw;
      const int c = b.dim;
      const std::string n1 = b.prefix + ".norm1", n2 = b.prefix + ".norm2", a = b.prefix + ".attn", f = b.prefix + ".ffn";
      if (b.attn == TURTLE_ATTN_REDUCED) {
        bw.a_in = pack_gemm(h, pk, dvec(W(h, a + ".conv1.weight")), 2 * c, c, n1, dvec(W(h, a + ".conv1.bias")));
        bw.a_dw = pack_dw(h, pk, a + ".conv2", 0, 2 * c);
        bw.a_out = pack_gemm(h, pk, dvec(W(h, a + ".conv3.weight")), c, 2 * c, "", dvec(W(h, a + ".conv3.bias")));
        bw.a_out.scale = pk.f32(dvec(W(h, a + ".beta")));
      } else if (b.attn == TURTLE_ATTN_CHANNEL || b.attn == TURTLE_ATTN_FHR) {
        bw.a_in = pack_gemm(h, pk, dvec(W(h, a + ".qkv.weight")), 3 * c, c, n1, opt_bias(h, a + ".qkv.bias"));
        bw.a_dw = pack_dw(h, pk, a + ".qkv_dwconv", 0, 3 * c);
        bw.a_dw_qk = pack_dw(h, pk, a + ".qkv_dwconv", 0, 2 * c);
        bw.a_dw_v = pack_dw(h, pk, a + ".qkv_dwconv", 2 * c, c);
        bw.wp = pk.f32(dvec(W(h, a + ".project_out.weight")));
        if (has(h, a + ".project_out.bias")) bw.po_bias = pk.f32(dvec(W(h, a + ".project_out.bias")));
        bw.tau = pk.f32(dvec(W(h, a + ".temperature")));
      } else if (b.attn == TURTLE_ATTN_CHM) {
        const std::string s = a + ".spatial_aligner", ca = a + ".ChanAttn";
        // one LN-folded GEMM for everything that reads norm1(x): [SAB qk | SAB v | FHR qkv]
        // (t0: the query half of qk is dead, only k = rows [c, 2c) is packed: [k | SAB v | FHR qkv])
        const bool t0 = A.cfg.variant == 1;
        const int q0 = t0 ? c : 0;
        std::vector<double> w6, b6;
        pack_rows(W(h, s + ".qk.weight"), c, q0, 2 * c, w6);
        pack_rows(W(h, s + ".v.weight"), c, 0, c, w6);
        pack_rows(W(h, ca + ".qkv.weight"), c, 0, 3 * c, w6);
        if (A.cfg.bias) {
          const auto& qb = W(h, s + ".qk.bias");
          for (int i = q0; i < 2 * c; ++i) b6.push_back(qb[i]);
          for (auto x : W(h, s + ".v.bias")) b6.push_back(x);
          for (auto x : W(h, ca + ".qkv.bias")) b6.push_back(x);
        }
        bw.a_in = pack_gemm(h, pk, w6, 6 * c - q0, c, n1, b6);
        bw.sab_qk_dw = pack_dw(h, pk, s + ".qk_dwconv", q0, 2 * c - q0);
        bw.sab_v_dw = pack_dw(h, pk, s + ".v_dwconv", 0, c);
        bw.fhr_dw = pack_dw(h, pk, ca + ".qkv_dwconv", 0, 3 * c);
        bw.chm_dw6 = pack_dw_cat(h, pk, {s + ".qk_dwconv", s + ".v_dwconv", ca + ".qkv_dwconv"}, {2 * c - q0, c, 3 * c},
                                 {q0, 0, 0});
        if (t0) {
          // W_k (x + pos) = W_k x + W_k pos: the encoding's term is W_k pos through the bias-free taps
          std::vector<double> wk;
          pack_rows(W(h, s + ".qk.weight"), c, c, 2 * c, wk);
          bw.t0_kpw = pack_gemm(h, pk, wk, c, c, "", {});
          bw.t0_kdw = pack_dw(h, pk, s + ".qk_dwconv", c, c, 9, false);
        }
        if (!t0) bw.q2 = pack_gemm(h, pk, dvec(W(h, s + ".q2.weight")), 2 * c, c, "", opt_bias(h, s + ".q2.bias"));
        if (!t0) {
          bw.k2 = pack_gemm(h, pk, dvec(W(h, s + ".k2.weight")), 2 * c, c, "", opt_bias(h, s + ".k2.bias"));
          const int taps = b.ws * b.ws;
          DwW qw = pack_dw(h, pk, s + ".q2_dwconv", 0, 2 * c, taps), kw = pack_dw(h, pk, s + ".k2_dwconv", 0, 2 * c, taps);
          bw.q2_win = qw.w; bw.q2_winb = qw.bias; bw.k2_win = kw.w; bw.k2_winb = kw.bias;
          bw.sab_tau = pk.f32(dvec(W(h, s + ".temperature")));
        }
        // kv(project_out_sab(o)) = (W_kv W_po) o + (W_kv b_po + b_kv): one GEMM over the T frames
        const auto& wkv = W(h, a + ".kv.weight");
        const auto& wpo = W(h, s + ".project_out.weight");
        std::vector<double> wm((size_t)2 * c * c, 0.0), bm;
        for (int o = 0; o < 2 * c; ++o)
          for (int j = 0; j < c; ++j) {
            double acc = 0;
            for (int i = 0; i < c; ++i) acc += (double)wkv[(size_t)o * c + i] * wpo[(size_t)i * c + j];
            wm[(size_t)o * c + j] = acc;
          }
        if (has(h, a + ".kv.bias") || has(h, s + ".project_out.bias")) {
          bm.assign(2 * c, 0.0);
          for (int o = 0; o < 2 * c; ++o) {
            double acc = has(h, a + ".kv.bias") ? W(h, a + ".kv.bias")[o] : 0.0;
            if (has(h, s + ".project_out.bias"))
              for (int i = 0; i < c; ++i) acc += (double)wkv[(size_t)o * c + i] * W(h, s + ".project_out.bias")[i];
            bm[o] = acc;
          }
        }
        bw.kv = pack_gemm(h, pk, wm, 2 * c, c, "", bm);
        bw.kv_dw = pack_dw(h, pk, a + ".kv_dwconv", 0, 2 * c);
        bw.wp = pk.f32(dvec(W(h, ca + ".project_out.weight")));
        if (has(h, ca + ".project_out.bias")) bw.po_bias = pk.f32(dvec(W(h, ca + ".project_out.bias")));
        bw.tau = pk.f32(dvec(W(h, ca + ".temperature")));
      }
      if (b.ffn == TURTLE_FFN_GFFW) {
        bw.f_in = pack_gemm(h, pk, dvec(W(h, f + ".project_in.weight")), 2 * b.hidden, c, n2, opt_bias(h, f + ".project_in.bias"));
        bw.f_dw = pack_dw(h, pk, f + ".dwconv", 0, 2 * b.hidden);
        bw.f_out = pack_gemm(h, pk, dvec(W(h, f + ".project_out.weight")), c, b.hidden, "", opt_bias(h, f + ".project_out.bias"));
        const int hp = (b.hidden + 63) / 64 * 64;     // gffn hidden width: padded with zero channels (exact)
        if (pk.bf16 && (c == 256 || c == 128 || c == 64) && (b.hidden % 64 == 0 || c == 64) && hp <= 768) {
          // the whole block as one kernel (gffn.hip): f16 fragments of W1 diag(g) and W2, tb = W1 b_ln + b1;
          // hidden channel j of each gate half maps to kernel channel j (j < hd), the rest are zero
          const int hd = b.hidden;
          const auto& w1 = W(h, f + ".project_in.weight");
          const auto& gw = W(h, n2 + ".body.weight");
          const auto& w2r = W(h, f + ".project_out.weight");
          std::vector<double> w1f((size_t)2 * hp * c, 0.0), tb((size_t)2 * hp, 0.0), dw9((size_t)9 * 2 * hp, 0.0), dwb,
              w2p((size_t)c * hp, 0.0);
          const bool lnb = !A.cfg.layernorm_biasfree;
          const bool hasdb = has(h, f + ".dwconv.bias");
          if (hasdb) dwb.assign((size_t)2 * hp, 0.0);
          const auto& dww = W(h, f + ".dwconv.weight");
          for (int half = 0; half < 2; ++half)
            for (int j = 0; j < hd; ++j) {
              const int n = half * hd + j, np = half * hp + j;   // reference channel, kernel channel
              double t = has(h, f + ".project_in.bias") ? W(h, f + ".project_in.bias")[n] : 0.0;
              for (int k = 0; k < c; ++k) {
                w1f[(size_t)np * c + k] = (double)w1[(size_t)n * c + k] * gw[k];
                if (lnb) t += (double)w1[(size_t)n * c + k] * W(h, n2 + ".body.bias")[k];
              }
              tb[np] = t;
              for (int t9 = 0; t9 < 9; ++t9) dw9[(size_t)t9 * 2 * hp + np] = dww[(size_t)n * 9 + t9];
              if (hasdb) dwb[np] = W(h, f + ".dwconv.bias")[n];
            }
          for (int o = 0; o < c; ++o)
            for (int j = 0; j < hd; ++j) w2p[(size_t)o * hp + j] = w2r[(size_t)o * hd + j];
          GffnHost gh;
          gffn_pack(c, hp, w1f, tb, dw9, dwb, w2p, gh);
          bw.gf_w1f = pk.raw(gh.w1f); bw.gf_tbp = pk.raw(gh.tbp); bw.gf_dwp = pk.raw(gh.dwp); bw.gf_w2f = pk.raw(gh.w2f);
          bw.gf_hd = hp;
        }
      } else {
        bw.f_in = pack_gemm(h, pk, dvec(W(h, f + ".conv4.weight")), 2 * c, c, n2, dvec(W(h, f + ".conv4.bias")));
        bw.f_out = pack_gemm(h, pk, dvec(W(h, f + ".conv5.weight")), c, 2 * c, "", dvec(W(h, f + ".conv5.bias")));
        bw.f_out.scale = pk.f32(dvec(W(h, f + ".gamma")));
        if (pk.bf16 && (c == 64 || c == 128)) pack_ffn_frags(pk, bw.f_in.w, bw.f_out.w, c, bw.ffn_w1f, bw.ffn_w2f);
      }
      bws.push_back(bw);
    }
    M.blocks.push_back(bws);
  }
  M.zeros = pk.f32(std::vector<double>(TURTLE_CONST_VEC, 0.0));
  M.ones = pk.f32(std::vector<double>(TURTLE_CONST_VEC, 1.0));
  pk.align();
  // same arch and dtype -> same packed size: repack in place, so device addresses (and launches
  // captured against them) stay valid across a weight update
  if (h->dev && h->dev_bytes != pk.host.size()) { (void)hipFree(h->dev); h->dev = nullptr; }
  if (!h->dev) HIPCHK(hipMalloc(&h->dev, pk.host.size()));
  else HIPCHK(hipDeviceSynchronize());   // no in-flight forward still reads the old weights
  HIPCHK(hipMemcpy(h->dev, pk.host.data(), pk.host.size(), hipMemcpyHostToDevice));
  h->dev_bytes = pk.host.size();
}

// ------------------------------------------------------------------------------------------
// frame driver
// ------------------------------------------------------------------------------------------
struct Arena {
  char* base;
  size_t cap, off = 0, peak = 0;
  bool dry;
  void* alloc(size_t bytes) {
    size_t o = (off + 255) / 256 * 256;
    off = o + bytes;
    peak = std::max(peak, off);
    if (!dry && off > cap) TFAIL(TURTLE_EINVAL, "workspace too small");
    return dry ? nullptr : base + o;
  }
};

struct CacheIO {
  const void* k_in[8]; const void* v_in[8]; int t_in[8];
  void* k_out[8]; void* v_out[8];
};

template <typename T>
struct Runner {
  TurtleHandle* h;
  hipStream_t st;
  Arena ar;
  int B, Hp, Wp;
  const CacheIO* io;
  static constexpr size_t ES = sizeof(T);

  T* buf(int64_t elems) { return reinterpret_cast<T*>(ar.alloc((size_t)elems * ES)); }

  hipEvent_t event() {
    if (h->ev_used == h->ev_pool.size()) {
      hipEvent_t e;
      HIPCHK(hipEventCreate(&e));
      h->ev_pool.push_back(e);
    }
    return h->ev_pool[h->ev_used++];
  }
  // launch `f` as kernel class `cls`, bracketed by events when that class is being profiled
  template <typename F>
  void launch(int cls, double bytes, double flops, F&& f) {
    if (dry()) return;
    const bool p = (h->prof_cls == TURTLE_K_ALL || h->prof_cls == cls) &&
                   (h->prof_filter.empty() || h->prof_filter == h->prof_tag);
    if (!p) { f(); h->prof_tag.clear(); return; }
    ProfRec r{cls, event(), event(), bytes, flops, std::move(h->prof_tag)};
    h->prof_tag.clear();
    HIPCHK(hipEventRecord(r.a, st));
    f();
    HIPCHK(hipEventRecord(r.b, st));
    h->prof.push_back(r);
  }
  // describe the next launch for the per-launch profile dump (TURTLE_PROF_DUMP)
  template <typename... A>
  void tag(const char* fmt, A... args) {
    if (h->prof_cls < 0) return;
    char buf[160];
    snprintf(buf, sizeof buf, fmt, args...);
    h->prof_tag = buf;
  }
  float* fbuf(int64_t elems) { return reinterpret_cast<float*>(ar.alloc((size_t)elems * 4)); }
  bool dry() const { return ar.dry; }

  static SrcList src1(const void* p, int64_t ld, int off, int K, int mul = 1, int add = 0) {
    SrcList s{}; s.n = 1; s.Ktot = K; s.s[0] = SrcDesc{p, ld, off, K, mul, add};
    return s;
  }
  void gemm(const GemmW& w, const SrcList& a, int64_t M, int HW, int Wimg, void* out, int64_t ldo, int offo,
            const void* res = nullptr, int64_t ldr = 0, int offr = 0, int gelu = 0,
            int store = STORE_NHWC, const void* wptr = nullptr, int64_t wstride = 0, int wdiv = 1,
            int N = -1, const float* bias = nullptr, int conv3 = 0, int cin = 0) {
    // per-pixel LayerNorm statistics of the gemm9 kernel (gemm9.hip): workspace reserved by shape only,
    // so sizing - which runs without packed weights - and every switch setting reserve the same bytes
    const bool g9_ws = ES == 2 && w.ln && a.n == 1 && !conv3 && (a.Ktot == 256 || a.Ktot == 512 || a.Ktot == 1024);
    const size_t mark = ar.off;                     // this GEMM's workspace: released after its launch (one stream)
    float* st9 = g9_ws ? fbuf(2 * M) : nullptr;
    // split-K partials of the small-frame wide projections (gemm_sk.hip), reserved by shape only too
    const int Nn = N >= 0 ? N : w.N;
    const bool sk_ws = ES == 2 && M <= h->sk_max_px && a.n == 1 && !conv3 && a.Ktot % 64 == 0 && Nn % 8 == 0 && Nn > 0;
    void* wsk = sk_ws ? ar.alloc(gemm_sk_workspace_bytes(M, Nn, a.Ktot)) : nullptr;
    struct Release { Arena& a; size_t m; ~Release() { a.off = m; } } release{ar, mark};
    if (dry()) return;
    GemmArgs g{};
    g.a = a; g.M = M; g.N = N >= 0 ? N : w.N; g.HW = HW; g.Wimg = Wimg;
    g.w = wptr ? wptr : h->ptr(w.w); g.ldw = a.Ktot; g.wstride = wstride; g.wdiv = wdiv;
    g.conv3 = conv3; g.cin = cin;
    g.ln = w.ln; g.ln_s = h->fptr(w.s); g.ln_t = h->fptr(w.t);
    g.bias = bias ? bias : h->fptr(w.bias); g.scale = h->fptr(w.scale); g.gelu = gelu;
    g.res = res; g.ldr = ldr; g.offr = offr;
    g.out = out; g.ldo = ldo; g.offo = offo; g.store_mode = store; g.cb_px = store == STORE_CB16 ? M : 0;
    g.zeros = h->fptr(h->mw.zeros); g.ones = h->fptr(h->mw.ones); g.allow_panel = h->panel; g.allow_lds = h->gemm_lds; g.allow_pn = h->gemm_pn;
    g.allow_ar = h->gemm_ar; g.allow_kt = h->gemm_kt; g.allow_f32 = h->gemm_f32; g.kt_max_px = h->kt_max_px;
    // channel-blocked stores: the pn GEMM, or gemm8 when every projection may take it (eligibility
    // tested on a copy; g.allow_g8 is set in one place, below)
    GemmArgs g8t = g;
    g8t.allow_g8 = 1;
    const bool cb_g8 = ES == 2 && h->gemm8 == 2 && gemm8_ok(g8t);
    if (store == STORE_CB16 && (ES != 2 || !gemm_pn_ok(g)) && !cb_g8)
      TFAIL(TURTLE_EINVAL, "channel-blocked store needs the pn GEMM (M " + std::to_string(M) + " N " + std::to_string(g.N) +
                               " K " + std::to_string(a.Ktot) + " HW " + std::to_string(HW) + ")");
    if (g.ln && a.n != 1) TFAIL(TURTLE_EINVAL, "LN GEMM needs a single source");
    if (g.N > TURTLE_CONST_VEC || a.Ktot > TURTLE_CONST_VEC) TFAIL(TURTLE_EINVAL, "GEMM wider than the constant vectors");
    // algorithmic traffic: A once (a 3x3 reads each input pixel once), W per weight set, out
    // (+ residual) once
    const double Ka = conv3 ? cin : a.Ktot;
    const double nset = wstride ? (double)(M / HW) / wdiv : 1.0;
    const double bytes = ES * ((double)M * Ka + nset * g.N * a.Ktot + (double)M * g.N * (res ? 2 : 1));
    bool lt = wide_class(g);
    if (ES == 2 && h->gemm8) {
      // 1: the wide class, 2: every eligible projection, 3: the K-concatenated multi-source
      // projections with K >= 1024 (the FHR / CHM W_eff GEMMs, where it measures ~7-10 % faster than
      // the 2-D tiled kernel: profiles/r04_g8bench.log; elsewhere hipBLASLt / pn / kt stay faster)
      g.allow_g8 = h->gemm8_ps ? 2 : 1;           // 2: the persistent form (gemm8.hip)
      // (mode 3 only where the 256 x 256 tiles still give every CU one: small frames go to kt)
      const int64_t g8_tiles = ((M + 255) / 256) * ((g.N + 255) / 256);
      const bool pick = h->gemm8 == 2 || (h->gemm8 == 1 && lt) ||
                        (h->gemm8 == 3 && a.n >= 2 && a.Ktot >= 1024 && !conv3 && g8_tiles >= 256);
      if (gemm8_ok(g) && pick) lt = false;
      else g.allow_g8 = 0;
    }
    // 256-pixel-row GEMM (gemm9.hip): 1 the wide class over <= 65536 pixels (the latent level; above
    // it the ar / kt kernels measure faster in the frame: level-3 W_eff 57 vs 64 us,
    // profiles/r05d_1080p_launch_report.txt), 2 every eligible projection
    bool use9 = false;
    if (ES == 2 && h->gemm9 && (h->gemm9 == 2 || (lt && M <= 65536))) {
      GemmArgs t9 = g;
      t9.allow_g9 = 1;
      if (gemm9_ok(t9) && (!g.ln || st9)) {
        use9 = true;
        g.allow_g8 = 0;
        g.allow_g9 = 1;
      }
    }
    // small frames (<= sk_max_px pixels): single-source projections on the split-K kernel (gemm_sk.hip),
    // whose 64 x 64 tiles (x K splits) fill the chip where 256-row or panel tiles give a handful of
    // blocks - unsplit (epilogue in the kernel) wherever that gives >= 256 tiles, split only for the
    // K >= 1024 wide projections (the latent project_out of a 256x256 frame: 36 -> 18 us); split at
    // K <= 640 its partial round trip costs more than it gains (M = 1024, N = 2560 split in two: 26 ->
    // 43 us, unsplit 20.6 us; profiles/r05sk2_*, r05sk4_*)
    bool use_sk = false;
    const bool sk_one = wsk && gemm_sk_splits(M, g.N, a.Ktot) == 1;
    if (ES == 2 && h->gemm_sk && wsk && !g.allow_g8 && ((lt && a.Ktot >= 1024) || sk_one) && gemm_sk_ok(g)) {
      use_sk = true;
      use9 = false;
    }
    tag("gemm M=%lld N=%d K=%d conv3=%d ln=%d res=%d store=%d nsrc=%d%s%s%s%s%s", (long long)M, g.N, a.Ktot, conv3, g.ln,
        res != nullptr, store, a.n, a.cb_px ? " cb" : "", lt ? " wide" : "", g.allow_g8 ? " g8" : "", use9 ? " g9" : "",
        use_sk ? " sk" : "");
    launch(TURTLE_K_GEMM, bytes, 2.0 * M * g.N * a.Ktot, [&] {
      if (use_sk) launch_gemm_sk(g, wsk, st);
      else if (use9) launch_gemm9(g, st9, st);
      else launch_gemm<T>(g, st);
    });
  }
  // The 'wide' projection class: single-source bf16 projections, NHWC stores, no activation or
  // scale, K >= 512 or (<= 140k pixels per weight set and >= 256 output channels) - the latent-level
  // LN projections (qkv, GatedFFN project_in), project_out (K = 1280), the latent / level-3 W_eff
  // GEMMs. Until round 4 these ran on hipBLASLt (measured faster than the ar / pn / kt kernels,
  // DESIGN.md §3.4); gemm9 takes them in-tree. Multi-image per-image weight sets stay on the 2-D
  // tiled kernel (one launch over all images, profiles/r04_256_b8_launch_report*.txt).
  bool wide_class(const GemmArgs& g) const {
    if (ES != 2 || g.a.cb_px || g.conv3 || g.gelu || g.scale || g.store_mode != STORE_NHWC || g.a.n != 1) return false;
    const SrcDesc& s = g.a.s[0];
    if (s.img_mul != 1 || s.img_add != 0 || s.K != g.a.Ktot) return false;
    if (g.wstride && (g.HW <= 0 || g.M % g.HW || g.M / g.HW > 1)) return false;
    if (g.ln && g.a.Ktot < 512) return false;     // the pn kernel's LN projections (levels 1-3)
    const int64_t Mi = g.wstride ? g.HW : g.M;
    return g.a.Ktot >= 512 || (Mi <= 140000 && g.N >= 256);
  }
  void dw(const DwW& w, const void* in, int64_t ldi, int offi, void* out, int64_t ldo, int offo,
          int nimg, int H, int Wd, int mode, int tok_ws = 0, int64_t tok_stride = 0) {
    if (dry()) return;
    DwArgs a{};
    a.in = in; a.ldi = ldi; a.offi = offi; a.out = out; a.ldo = ldo; a.offo = offo;
    a.w = h->fptr(w.w); a.bias = h->fptr(w.bias);
    a.nimg = nimg; a.H = H; a.W = Wd; a.C = mode == DW_GATE ? w.C / 2 : w.C; a.mode = mode;
    a.tok_ws = tok_ws; a.tok_img_stride = tok_stride; a.rows = h->dw_rows;
    const double px = (double)nimg * H * Wd, cin = mode == DW_GATE ? 2.0 * a.C : a.C;
    tag("dw nimg=%d H=%d W=%d C=%d mode=%d tok=%d", nimg, H, Wd, a.C, mode, tok_ws);
    launch(TURTLE_K_DW, ES * px * (cin + a.C), 18.0 * px * cin, [&] { launch_dw<T>(a, st); });
  }

  // [LN ->] pw -> dw3x3 -> [act -> pw (+res)] in one kernel (fused.hip)
  void fused(int mode, const GemmW& w1, const DwW& dwp, const T* x, int64_t ldx, int offx, int C, int nimg, int H, int Wd,
             int hidden, const GemmW* w2, const T* res, T* out, const std::vector<FusedDst>& dsts) {
    if (dry()) return;
    FusedArgs f{};
    f.x = x; f.ldx = ldx; f.offx = offx; f.C = C; f.nimg = nimg; f.H = H; f.W = Wd;
    f.w1 = h->ptr(w1.w); f.N1 = w1.N; f.ln = w1.ln; f.ln_s = h->fptr(w1.s); f.ln_t = h->fptr(w1.t); f.b1 = h->fptr(w1.bias);
    f.dww = h->fptr(dwp.w); f.dwb = h->fptr(dwp.bias); f.hidden = hidden; f.mode = mode;
    f.dww2 = reinterpret_cast<const uint32_t*>(h->ptr(dwp.w2));
    if (!f.dww2) TFAIL(TURTLE_EINVAL, "fused: depthwise weights without the tap-pair table");
    double px = (double)nimg * H * Wd;
    double bytes = ES * px * C, flops = 2.0 * px * C * w1.N + 18.0 * px * w1.N;
    if (w2) {
      if (w2->N > 128 || w2->N % 16) TFAIL(TURTLE_EINVAL, "fused GEMM2 needs N2 <= 128, N2 % 16 == 0");
      f.w2 = h->ptr(w2->w); f.N2 = w2->N; f.b2 = h->fptr(w2->bias); f.scale2 = h->fptr(w2->scale);
      f.res = res; f.ldr = w2->N; f.offr = 0; f.out = out; f.ldo = w2->N; f.offo = 0;
      // algorithmic bytes count each distinct tensor once: the residual of a fused block is its own
      // input x (already counted), re-read from L2 by the epilogue
      bytes += ES * px * w2->N * ((res && res != x) ? 2 : 1);
      flops += 2.0 * px * hidden * w2->N;
    } else {
      if (dsts.empty() || dsts.size() > 3) TFAIL(TURTLE_EINVAL, "fused dw-only needs 1..3 destinations");
      for (size_t i = 0; i < dsts.size(); ++i) f.dst[i] = dsts[i];
      f.ndst = (int)dsts.size();
      bytes += ES * px * w1.N;
    }
    if (dwp.C != w1.N) TFAIL(TURTLE_EINVAL, "fused: dw width != pointwise width");
    if (C > 128) TFAIL(TURTLE_EINVAL, "fused: input width > 128");
    tag("fused mode=%d nimg=%d H=%d W=%d C=%d N1=%d N2=%d ln=%d ndst=%d", mode, nimg, H, Wd, C, w1.N, f.N2, f.ln, f.ndst);
    const bool rw = ES == 2 && h->fused2 && fused2_ok(f);
    if (rw) tag("fused2 mode=%d nimg=%d H=%d W=%d C=%d N1=%d N2=%d ln=%d ndst=%d", mode, nimg, H, Wd, C, w1.N, f.N2, f.ln, f.ndst);
    launch(TURTLE_K_FUSED, bytes, flops, [&] {
      if (rw) launch_fused2(f, st);
      else launch_fused<T>(f, st);
    });
  }
  // fused.hip handles input widths <= 128 in 16-channel slices and 32-deep GEMM2 K steps
  bool can_fuse(int c, int mode, int n1, int hidden) const {
    if (!h->fuse || (ES == 4 && !h->fuse_fp32) || c > 128 || c % 16) return false;
    if (mode == F_DWONLY) return n1 % 16 == 0;
    return hidden % 32 == 0;
  }
  // out (+)= W [gelu(dw(x1)) * dw(x2) | dw(x)] + bias (+ res) with the depthwise computed in the
  // GEMM's operand prologue (dwgemm.hip); returns false (nothing launched) where not eligible
  bool dwgemm(const DwW& dwp, int gate, const T* in, int64_t ldi, int offi, int nimg, int H, int Wd, int K,
              const void* wptr, int64_t ldw, int64_t wstride, int N, const float* bias, const T* res, int64_t ldr,
              T* out, int64_t ldo, int64_t cb_px = 0) {
    if (ES != 2 || !h->dwgemm || dwp.C != (gate ? 2 * K : K)) return false;
    DwGemmArgs a{};
    a.in = in; a.ldi = ldi; a.offi = offi; a.dww16 = h->ptr(dwp.w16); a.dwb = h->fptr(dwp.bias); a.gate = gate;
    a.nimg = nimg; a.H = H; a.W = Wd; a.K = K;
    a.w = wptr; a.ldw = ldw; a.wstride = wstride; a.wdiv = 1; a.N = N; a.bias = bias;
    a.res = res; a.ldr = ldr; a.offr = 0; a.out = out; a.ldo = ldo; a.offo = 0;
    a.zeros = h->fptr(h->mw.zeros); a.cb_px = cb_px;
    if (dwgemm_blocks(a) < h->dwgemm_min_blocks) return false;
    if (dry()) return true;
    if (!dwgemm_ok(a)) return false;
    return dwgemm_launch(a);
  }
  // shape-only eligibility of the channel-attention v path (decided before qkv is produced, and the
  // same in the sizing dry run): alignment is guaranteed by the arena (256 B) and widths % 32
  bool can_dwgemm_v(int c, int nimg, int H, int Wd) const {
    if (ES != 2 || !h->dwgemm || !h->dwgemm_attn || c % 32 || c > 512) return false;
    if ((int64_t)H * Wd * 3 * c >= ((int64_t)1 << 31)) return false;   // dwgemm_ok: 32-bit input offsets
    DwGemmArgs a{};
    a.nimg = nimg; a.H = H; a.W = Wd; a.N = c;
    return dwgemm_blocks(a) >= h->dwgemm_min_blocks;
  }
  // shape-only: the GatedFeedForward hidden map channel-blocked between the pn GEMM and dwgemm
  bool can_dwgemm_cb(int c, int hd, int nimg, int H, int Wd) const {
    if (ES != 2 || !h->dwgemm || !h->dwgemm_cb || !h->gemm_pn || hd % 32 || hd > 2048) return false;
    if (c != 64 && c != 128 && c != 256 && c != 384 && c != 512) return false;
    const int64_t P = (int64_t)nimg * H * Wd;
    if ((2 * hd) % 64 || (int64_t)H * Wd < 128 || (int64_t)(hd / 16 + 3) * P * 32 >= ((int64_t)1 << 31)) return false;
    DwGemmArgs a{};
    a.nimg = nimg; a.H = H; a.W = Wd; a.N = c;
    if (dwgemm_blocks(a) < h->dwgemm_min_blocks) return false;
    GemmArgs g{};                                  // the project_in GEMM as gemm() will build it
    g.a = src1(nullptr, c, 0, c); g.M = P; g.N = 2 * hd; g.HW = H * Wd; g.Wimg = Wd; g.ldw = c; g.ln = 1;
    g.ldo = 2 * hd; g.store_mode = STORE_CB16; g.cb_px = P; g.allow_pn = h->gemm_pn;
    return gemm_pn_ok(g);
  }
  bool dwgemm_launch(DwGemmArgs& a) {
    const int gate = a.gate, K = a.K, N = a.N, nimg = a.nimg, H = a.H, Wd = a.W;
    const bool res = a.res != nullptr;
    const int64_t wstride = a.wstride;
    const double px = (double)nimg * H * Wd, cin = gate ? 2.0 * K : K;
    const double nset = wstride ? nimg : 1.0;
    tag("dwgemm gate=%d nimg=%d H=%d W=%d K=%d N=%d", gate, nimg, H, Wd, K, N);
    launch(TURTLE_K_GEMM, ES * (px * cin + nset * (double)N * K + px * N * (res ? 2 : 1)),
           2.0 * px * N * K + 18.0 * px * cin, [&] { launch_dwgemm(a, st); });
    return true;
  }
  // LN -> pointwise -> depthwise (-> gate) with the hidden map on chip (tilepd.hip), input width 256
  // (shape-only, same in the dry run)
  bool can_tilepd(int c, int n1, int nimg, int H, int Wd) const {
    if (ES != 2 || !h->tilepd || c != 256 || n1 % 32 || n1 > 1536) return false;
    TilePdArgs a{};
    a.nimg = nimg; a.H = H; a.W = Wd;
    return tilepd_blocks(a) >= h->tilepd_min_blocks;
  }
  void tilepd(int mode, const GemmW& w1, const DwW& dwp, const T* x, int c, T* out, int64_t ldo, int nimg, int H, int Wd,
              int64_t cb_px = 0) {
    if (dry()) return;
    TilePdArgs a{};
    a.x = x; a.ldx = c; a.offx = 0; a.C = c; a.nimg = nimg; a.H = H; a.W = Wd;
    a.w1 = h->ptr(w1.w); a.N1 = w1.N; a.ln = w1.ln ? 1 : 0; a.centred = h->arch.cfg.layernorm_biasfree ? 0 : 1;
    a.tb = w1.ln ? h->fptr(w1.tb) : h->fptr(w1.bias);
    a.dww16 = h->ptr(dwp.w16); a.dwb = h->fptr(dwp.bias); a.mode = mode;
    a.out = out; a.ldo = ldo; a.offo = 0; a.cb_px = cb_px;
    if (dwp.C != w1.N || w1.K != c) TFAIL(TURTLE_EINVAL, "tilepd: depthwise / pointwise widths disagree");
    if (!tilepd_ok(a)) TFAIL(TURTLE_EINVAL, "tilepd: arguments outside the kernel's contract");
    const double px = (double)nimg * H * Wd, nout = mode == TP_GATE ? w1.N / 2 : w1.N;
    tag("tilepd mode=%d nimg=%d H=%d W=%d C=%d N1=%d", mode, nimg, H, Wd, c, w1.N);
    launch(TURTLE_K_FUSED, ES * px * (c + nout), 2.0 * px * c * w1.N + 18.0 * px * w1.N, [&] { launch_tilepd(a, st); });
  }
  // FeedForward in one kernel (ffn.hip): bf16, widths 64 / 128 (shape-only, same in the dry run)
  bool can_ffn(int c) const { return ES == 2 && h->ffn && (c == 64 || c == 128); }
  // the whole GatedFeedForward at width 256 (128) in one kernel (gffn.hip); out = xin + ffn(norm2(xin))
  GffnArgs gffn_args(const BlockW& bw, const T* xin, T* out, int c, int hd, int H, int Wd) const {
    GffnArgs g{};
    g.x = xin; g.out = out; g.nimg = B; g.H = H; g.W = Wd; g.hd = (hd + 63) / 64 * 64; g.C = c;   // (= bw.gf_hd)
    g.centred = h->arch.cfg.layernorm_biasfree ? 0 : 1;
    g.w1f = h->ptr(bw.gf_w1f); g.tbp = h->fptr(bw.gf_tbp);
    g.dwp = reinterpret_cast<const uint32_t*>(h->ptr(bw.gf_dwp)); g.w2f = h->ptr(bw.gf_w2f);
    g.b2 = h->fptr(bw.f_out.bias);
    return g;
  }
  bool can_gffn(const BlockW& bw, int c, int hd, int H, int Wd) const {
    if (ES != 2 || !h->gffn || !(c == 256 || (c == 128 && h->gffn_c128) || (c == 64 && h->gffn_c64))) return false;
    if ((hd % 64 && c != 64) || (hd + 63) / 64 * 64 > 768) return false;
    if (!dry() && bw.gf_w1f == NONE) return false;
    GffnArgs g{};
    g.nimg = B; g.H = H; g.W = Wd; g.hd = hd;
    return gffn_blocks(g) >= h->gffn_min_blocks;
  }
  void gffn(const BlockW& bw, const T* xin, T* out, int c, int hd, int H, int Wd) {
    if (dry()) return;
    GffnArgs g = gffn_args(bw, xin, out, c, hd, H, Wd);
    if (!gffn_ok(g)) TFAIL(TURTLE_EINVAL, "gffn: arguments outside the kernel's contract");
    const double px = (double)B * H * Wd;
    if (c == 256) tag("gffn nimg=%d H=%d W=%d hd=%d", B, H, Wd, hd);
    else tag("gffn nimg=%d H=%d W=%d C=%d hd=%d", B, H, Wd, c, hd);
    launch(TURTLE_K_FUSED, ES * px * 2.0 * c, px * (2.0 * c * 2 * hd + 2.0 * hd * c + 18.0 * 2 * hd), [&] { launch_gffn(g, st); });
  }
  void ffn(const BlockW& bw, T* x, int64_t P, int c) {
    if (dry()) return;
    FfnArgs f{};
    f.x = x; f.out = x; f.M = P; f.C = c;
    f.w1f = h->ptr(bw.ffn_w1f); f.w2f = h->ptr(bw.ffn_w2f);
    f.s1 = h->fptr(bw.f_in.s); f.t1 = h->fptr(bw.f_in.tb); f.b2 = h->fptr(bw.f_out.bias); f.g2 = h->fptr(bw.f_out.scale);
    if (!bw.f_in.ln || !ffn_ok(f)) TFAIL(TURTLE_EINVAL, "ffn: FeedForward weights not packed for the fused kernel");
    tag("ffn M=%lld C=%d", (long long)P, c);
    launch(TURTLE_K_FUSED, ES * 2.0 * P * c, 2.0 * P * (2.0 * c * c * 2), [&] { launch_ffn(f, st); });
  }
  static FusedDst dst_map(void* p, int64_t ld, int off, int cbeg, int cend) {
    return FusedDst{p, ld, off, cbeg, cend, cend - cbeg, 0, 0};
  }

  struct Seg { const void* base; int64_t ld; int off; int hstride; int mul, add; int norm; int64_t col; int colh; };

  // channel attention core: Gram over (q, key segments), softmax, W_eff, then out = x + W_eff [v srcs]
  void chan_attn(const BlockW& bw, const Blk& b, const T* q, int64_t ldq, int qoff, const std::vector<Seg>& segs,
                 const SrcList& vsrc, int HW, int Wimg, T* x, float* kinv, int cur_seg,
                 const DwW* vdw = nullptr, const T* vraw = nullptr, int64_t ldv = 0, int offv = 0) {
    const int c = b.dim, ch = c / b.heads, nseg = (int)segs.size(), ncol = nseg * ch;
    if (ncol > 512 || nseg > TURTLE_MAX_SEG) TFAIL(TURTLE_EINVAL, "channel attention: more than 512 key columns");
    // pixel splits: ~1024 blocks over all (b, head) at large maps, >= 256 pixels each, whole
    // 128-pixel steps of the bf16 Gram
    int nchunk = std::max(1, std::min((HW + 255) / 256, std::max(1, h->gram_blocks / (B * b.heads))));
    int chunk = (HW + nchunk - 1) / nchunk;
    chunk = (chunk + 127) / 128 * 128;
    nchunk = (HW + chunk - 1) / chunk;
    const int stride = ch * ncol + ch + ncol;
    float* part = fbuf((int64_t)B * b.heads * nchunk * stride);
    float* red = fbuf((int64_t)B * b.heads * stride);
    float* attn = fbuf((int64_t)B * b.heads * ch * ncol);
    T* weff = buf((int64_t)B * c * vsrc.Ktot);
    if (dry()) return;
    if (ch > 128) TFAIL(TURTLE_EINVAL, "channel attention: more than 128 channels per head");
    GramArgs g{};
    g.q = q; g.ldq = ldq; g.qoff = qoff; g.nseg = nseg;
    unsigned mask = 0;
    for (int s = 0; s < nseg; ++s) {
      g.seg[s] = GramSeg{segs[s].base, segs[s].ld, segs[s].off, segs[s].hstride, segs[s].mul, segs[s].add, segs[s].norm};
      if (segs[s].norm) mask |= 1u << s;
    }
    g.B = B; g.heads = b.heads; g.ch = ch; g.HW = HW; g.nchunk = nchunk; g.chunk = chunk; g.part = part;
    tag("gram B=%d HW=%d c=%d heads=%d nseg=%d nchunk=%d", B, HW, c, b.heads, nseg, nchunk);
    launch(TURTLE_K_ATTN, ES * (double)B * HW * c * (1 + nseg), 2.0 * B * b.heads * ch * ncol * (double)HW,
           [&] { launch_gram<T>(g, st); });
    AttnFinArgs f{};
    f.part = part; f.nchunk = nchunk; f.B = B; f.heads = b.heads; f.ch = ch; f.nseg = nseg;
    f.norm_mask = mask; f.tau = h->fptr(bw.tau); f.kinv = kinv; f.cur_seg = cur_seg; f.red = red; f.attn = attn;
    WeffArgs we{};
    we.attn = attn; we.wp = h->fptr(bw.wp); we.B = B; we.heads = b.heads; we.ch = ch; we.nseg = nseg; we.C = c;
    for (int s = 0; s < nseg; ++s) { we.seg_col[s] = segs[s].col; we.seg_hstride[s] = segs[s].colh; }
    we.Keff = vsrc.Ktot; we.weff = weff;
    const bool fin = h->attn_fin && weff_fin_ok(we);   // softmax rows inside the W_eff launch
    f.sum_only = fin;
    tag("attn_rows nbh=%d ch=%d ncol=%d nchunk=%d%s", B * b.heads, ch, ncol, nchunk, fin ? " sum" : "");
    launch(TURTLE_K_ATTN, 4.0 * B * b.heads * (double)nchunk * stride, 0, [&] { launch_attn_finalize(f, st); });
    tag("weff B=%d C=%d heads=%d ncol=%d%s", B, c, b.heads, ncol, fin ? " fin" : "");
    launch(TURTLE_K_ATTN, ES * (double)B * c * vsrc.Ktot + 4.0 * B * b.heads * ch * ncol, 2.0 * B * c * (double)b.heads * ncol * ch,
           [&] { if (fin) launch_weff_fin<T>(we, f, st); else launch_weff<T>(we, st); });
    if (vdw) {
      // v's depthwise folded into the W_eff GEMM's operand prologue (dwgemm.hip): out = x + W_eff dw(v) + b
      if (!dwgemm(*vdw, 0, vraw, ldv, offv, B, HW / Wimg, Wimg, c, weff, c, (int64_t)c * c, c, h->fptr(bw.po_bias), x, c,
                  x, c))
        TFAIL(TURTLE_EINVAL, "channel attention: dwgemm v path not eligible");
      return;
    }
    GemmW pw; pw.N = c; pw.K = vsrc.Ktot;
    gemm(pw, vsrc, (int64_t)B * HW, HW, Wimg, x, c, 0, x, c, 0, 0, STORE_NHWC, weff, (int64_t)c * vsrc.Ktot, 1, c,
         h->fptr(bw.po_bias));
  }

  // one TurtleAttnBlock (turtle_t1_arch.py:804-811). x / xalt ping-pong: a fused kernel reads its
  // input with a halo, so it cannot update the residual stream in place.
  void block(const Blk& b, const BlockW& bw, T*& x, T*& xalt, int H, int Wd) {
    const int c = b.dim, HW = H * Wd;
    const int64_t P = (int64_t)B * HW;
    const size_t mark = ar.off;
    if (b.attn == TURTLE_ATTN_REDUCED) {
      if (can_fuse(c, F_GELU, 2 * c, 2 * c)) {
        fused(F_GELU, bw.a_in, bw.a_dw, x, c, 0, c, B, H, Wd, 2 * c, &bw.a_out, x, xalt, {});
        std::swap(x, xalt);
      } else {
        T* t1 = buf(P * 2 * c);
        T* t2 = buf(P * 2 * c);
        gemm(bw.a_in, src1(x, c, 0, c), P, HW, Wd, t1, 2 * c, 0);
        dw(bw.a_dw, t1, 2 * c, 0, t2, 2 * c, 0, B, H, Wd, DW_GELU);
        gemm(bw.a_out, src1(t2, 2 * c, 0, 2 * c), P, HW, Wd, x, c, 0, x, c, 0);
      }
    } else if (b.attn == TURTLE_ATTN_CHANNEL || (b.attn == TURTLE_ATTN_FHR && b.cache_slot < 0)) {
      T* t2 = buf(P * 3 * c);
      const int ch = c / b.heads;
      std::vector<Seg> segs{{t2, 3 * c, c, ch, 1, 0, 1, 0, ch}};
      if (!can_fuse(c, F_DWONLY, 3 * c, 0) && can_tilepd(c, 3 * c, B, H, Wd)) {
        // LN -> qkv -> qkv_dwconv in one kernel (the 3c-channel qkv map never reaches HBM), then the
        // Gram and the W_eff GEMM over the depthwised q, k, v
        tilepd(TP_DW, bw.a_in, bw.a_dw, x, c, t2, 3 * c, B, H, Wd);
        chan_attn(bw, b, t2, 3 * c, 0, segs, src1(t2, 3 * c, 2 * c, c), HW, Wd, x, nullptr, -1);
      } else if (!can_fuse(c, F_DWONLY, 3 * c, 0) && can_dwgemm_v(c, B, H, Wd)) {
        // qkv GEMM, depthwise of q,k only; v's depthwise runs inside the W_eff GEMM (dwgemm.hip)
        T* t1 = buf(P * 3 * c);
        gemm(bw.a_in, src1(x, c, 0, c), P, HW, Wd, t1, 3 * c, 0);
        dw(bw.a_dw_qk, t1, 3 * c, 0, t2, 3 * c, 0, B, H, Wd, DW_PLAIN);
        chan_attn(bw, b, t2, 3 * c, 0, segs, src1(t1, 3 * c, 2 * c, c), HW, Wd, x, nullptr, -1, &bw.a_dw_v, t1, 3 * c,
                  2 * c);
      } else {
        qkv_dw(bw, x, c, t2, B, H, Wd);
        chan_attn(bw, b, t2, 3 * c, 0, segs, src1(t2, 3 * c, 2 * c, c), HW, Wd, x, nullptr, -1);
      }
    } else if (b.attn == TURTLE_ATTN_FHR) {
      fhr(b, bw, x, H, Wd);
    } else if (b.attn == TURTLE_ATTN_CHM) {
      chm(b, bw, x, H, Wd);
    }
    ar.off = mark;
    // feed-forward
    if (b.ffn == TURTLE_FFN_GFFW) {
      const int hd = b.hidden;
      if (can_gffn(bw, c, hd, H, Wd)) {                // width 256 / 128: the block as one kernel
        gffn(bw, x, xalt, c, hd, H, Wd);
        std::swap(x, xalt);
      } else if (can_fuse(c, F_GATE, 2 * hd, hd)) {
        fused(F_GATE, bw.f_in, bw.f_dw, x, c, 0, c, B, H, Wd, hd, &bw.f_out, x, xalt, {});
        std::swap(x, xalt);
      } else if (h->tilepd_gate && can_tilepd(c, 2 * hd, B, H, Wd)) {
        // LN -> project_in -> dwconv -> gelu gate in one kernel (the 2h-channel hidden map stays on
        // chip), G [P][h] -> project_out GEMM with the residual
        // (G channel-blocked [h / 16][P][16]: a unit's output row is one 448-byte run; the 2-D tiled
        // GEMM reads it as its A operand)
        T* t2 = buf(P * hd);
        const bool cb = h->tilepd_cb && h->gemm_kt;      // the channel-blocked operand needs the 2-D tiled GEMM
        tilepd(TP_GATE, bw.f_in, bw.f_dw, x, c, t2, hd, B, H, Wd, cb ? P : 0);
        SrcList gs = src1(t2, hd, 0, hd);
        gs.cb_px = cb ? P : 0;
        gemm(bw.f_out, gs, P, HW, Wd, x, c, 0, x, c, 0);
      } else if (can_dwgemm_cb(c, hd, B, H, Wd)) {
        // project_in stores the hidden map channel-blocked ([2 hd / 16][P][16]): each dwgemm K step
        // then reads contiguous 32-byte pixel rows
        T* t1 = buf(P * 2 * hd);
        gemm(bw.f_in, src1(x, c, 0, c), P, HW, Wd, t1, 2 * hd, 0, nullptr, 0, 0, 0, STORE_CB16);
        // (the sizing dry run may hold no packed weights: nothing to check or launch there)
        if (!dry() && !dwgemm(bw.f_dw, 1, t1, 0, 0, B, H, Wd, hd, h->ptr(bw.f_out.w), hd, 0, c, h->fptr(bw.f_out.bias), x, c,
                              x, c, P))
          TFAIL(TURTLE_EINVAL, "GatedFeedForward: channel-blocked dwgemm not eligible");
      } else {
        T* t1 = buf(P * 2 * hd);
        T* t2 = buf(P * hd);   // dw + gate output of the unfolded path
        gemm(bw.f_in, src1(x, c, 0, c), P, HW, Wd, t1, 2 * hd, 0);
        if (!dwgemm(bw.f_dw, 1, t1, 2 * hd, 0, B, H, Wd, hd, h->ptr(bw.f_out.w), hd, 0, c, h->fptr(bw.f_out.bias),
                    x, c, x, c)) {
          dw(bw.f_dw, t1, 2 * hd, 0, t2, hd, 0, B, H, Wd, DW_GATE);
          gemm(bw.f_out, src1(t2, hd, 0, hd), P, HW, Wd, x, c, 0, x, c, 0);
        }
      }
    } else if (can_ffn(c)) {
      ffn(bw, x, P, c);
    } else {
      T* t1 = buf(P * 2 * c);
      gemm(bw.f_in, src1(x, c, 0, c), P, HW, Wd, t1, 2 * c, 0, nullptr, 0, 0, /*gelu*/ 1);
      gemm(bw.f_out, src1(t1, 2 * c, 0, 2 * c), P, HW, Wd, x, c, 0, x, c, 0);
    }
    ar.off = mark;
  }

  // LN(x) -> qkv 1x1 -> qkv_dwconv into `out` [P][3c] (fused, or GEMM + dw)
  void qkv_dw(const BlockW& bw, const T* x, int c, T* out, int nimg, int H, int Wd) {
    if (can_fuse(c, F_DWONLY, 3 * c, 0)) {
      fused(F_DWONLY, bw.a_in, bw.a_dw, x, c, 0, c, nimg, H, Wd, 3 * c, nullptr, nullptr, nullptr,
            {dst_map(out, 3 * c, 0, 0, 3 * c)});
    } else {
      const int64_t P = (int64_t)nimg * H * Wd;
      T* t1 = buf(P * 3 * c);
      gemm(bw.a_in, src1(x, c, 0, c), P, H * Wd, Wd, t1, 3 * c, 0);
      dw(bw.a_dw, t1, 3 * c, 0, out, 3 * c, 0, nimg, H, Wd, DW_PLAIN);
    }
  }

  // latent FrameHistoryRouter with cache slot (turtle_t1_arch.py:218-286)
  void fhr(const Blk& b, const BlockW& bw, T* x, int H, int Wd) {
    const int c = b.dim, HW = H * Wd, ch = c / b.heads, slot = b.cache_slot;
    const int64_t P = (int64_t)B * HW;
    const int R = io->t_in[slot];
    const int Rnew = std::min(R + ch, b.ntc * ch);
    T* t2 = buf(P * 3 * c);
    float* kinv = fbuf((int64_t)B * c);
    qkv_dw(bw, x, c, t2, B, H, Wd);
    std::vector<Seg> segs;
    const int Tc = R / ch;
    for (int t = 0; t < Tc; ++t)
      segs.push_back(Seg{io->k_in[slot], (int64_t)b.heads * R, t * ch, R, 1, 0, 0, (int64_t)t * ch, R});
    segs.push_back(Seg{t2, 3 * c, c, ch, 1, 0, 1, (int64_t)b.heads * R, ch});
    SrcList vs{};
    if (R) { vs.s[vs.n++] = SrcDesc{io->v_in[slot], (int64_t)b.heads * R, 0, b.heads * R, 1, 0}; }
    vs.s[vs.n++] = SrcDesc{t2, 3 * c, 2 * c, c, 1, 0};
    vs.Ktot = b.heads * R + c;
    // the new cache reads the pre-attention current k/v, so roll it before x is updated in place
    chan_attn(bw, b, t2, 3 * c, 0, segs, vs, HW, Wd, x, kinv, Tc);
    if (dry()) return;
    FhrCacheArgs fk{};
    fk.old = io->k_in[slot]; fk.R = R; fk.cur = t2; fk.ldc = 3 * c; fk.coff = c; fk.kinv = kinv;
    fk.out = io->k_out[slot]; fk.Rnew = Rnew; fk.B = B; fk.P = HW; fk.heads = b.heads; fk.ch = ch;
    tag("fhr_cache k B=%d P=%d heads=%d R=%d Rnew=%d", B, HW, b.heads, R, Rnew);
    launch(TURTLE_K_OTHER, ES * (double)B * HW * b.heads * (R + ch + Rnew), 0, [&] { launch_fhr_cache<T>(fk, st); });
    FhrCacheArgs fv = fk;
    fv.old = io->v_in[slot]; fv.coff = 2 * c; fv.kinv = nullptr; fv.out = io->v_out[slot];
    tag("fhr_cache v B=%d P=%d heads=%d R=%d Rnew=%d", B, HW, b.heads, R, Rnew);
    launch(TURTLE_K_OTHER, ES * (double)B * HW * b.heads * (R + ch + Rnew), 0, [&] { launch_fhr_cache<T>(fv, st); });
  }

  // t0 CausalHistoryModel (turtle_arch.py:535-590): the aligner's attention is discarded
  // (`out = v`, turtle_arch.py:521-523), so the aligned frames are the v token frames themselves
  // and only k (for the cache) and v are computed: k = normalize(dilated(dw(qk(x + pos))[k]))
  void chm_t0(const Blk& b, const BlockW& bw, T* x, int H, int Wd) {
    const int c = b.dim, HW = H * Wd, ch = c / b.heads, ws = b.ws, slot = b.cache_slot;
    const int64_t P = (int64_t)B * HW;
    const int th = H / ws, tw = Wd / ws, N = th * tw;
    const int64_t D = (int64_t)ws * ws * c;
    // the discarded attention still runs topk(5) over the keys (turtle_arch.py:509-510)
    if (N < 5) TFAIL(TURTLE_EINVAL, "selected index k out of range: SAB needs >= 5 tokens (input too small)");
    const int Tin = slot >= 0 ? io->t_in[slot] : 0;
    const int NT = Tin + 1;
    const int Tnew = std::min(NT, b.ntc);
    if (NT > TURTLE_MAX_T) TFAIL(TURTLE_EINVAL, "too many cached frames");
    T* kout = slot >= 0 ? reinterpret_cast<T*>(io->k_out[slot]) : buf((int64_t)B * Tnew * N * D);
    T* vout = slot >= 0 ? reinterpret_cast<T*>(io->v_out[slot]) : buf((int64_t)B * Tnew * N * D);
    const T* kin = slot >= 0 ? reinterpret_cast<const T*>(io->k_in[slot]) : nullptr;
    const T* vin = slot >= 0 ? reinterpret_cast<const T*>(io->v_in[slot]) : nullptr;
    const int64_t cstride = (int64_t)Tnew * N * D;
    T* kcur = kout + (int64_t)(Tnew - 1) * N * D;
    T* vcur = vout + (int64_t)(Tnew - 1) * N * D;
    T* fq = buf(P * 3 * c);
    T* pe = buf((int64_t)HW * c);
    T* kp = buf((int64_t)HW * c);
    T* kpos = buf((int64_t)N * D);
    T* xs = buf(P * NT * c);
    T* kvd = buf(P * NT * 2 * c);
    // LN(x) -> [SAB k | SAB v | FHR qkv] -> depthwise; k and v go straight into the new caches'
    // current frame in the dilated token layout
    if (can_fuse(c, F_DWONLY, 5 * c, 0)) {
      FusedDst dk{kcur, 0, 0, 0, c, c, ws, cstride}, dv{vcur, 0, 0, c, 2 * c, c, ws, cstride};
      fused(F_DWONLY, bw.a_in, bw.chm_dw6, x, c, 0, c, B, H, Wd, 5 * c, nullptr, nullptr, nullptr,
            {dk, dv, dst_map(fq, 3 * c, 0, 2 * c, 5 * c)});
    } else {
      T* t5 = buf(P * 5 * c);
      gemm(bw.a_in, src1(x, c, 0, c), P, HW, Wd, t5, 5 * c, 0);
      dw(bw.sab_qk_dw, t5, 5 * c, 0, kcur, 0, 0, B, H, Wd, DW_PLAIN, ws, cstride);
      dw(bw.sab_v_dw, t5, 5 * c, c, vcur, 0, 0, B, H, Wd, DW_PLAIN, ws, cstride);
      dw(bw.fhr_dw, t5, 5 * c, 2 * c, fq, 3 * c, 0, B, H, Wd, DW_PLAIN);
    }
    // positional term dw(W_k pos) in token layout (one image, shared by the batch), then
    // k += it and L2-normalise each token (F.normalize over ws*ws*c, turtle_arch.py:494-495)
    if (!dry()) {
      T0PeArgs pa{pe, H, Wd, c};
      tag("t0_pe H=%d W=%d C=%d", H, Wd, c);
      launch(TURTLE_K_OTHER, ES * (double)HW * c, 0, [&] { launch_t0_pe<T>(pa, st); });
    }
    gemm(bw.t0_kpw, src1(pe, c, 0, c), HW, HW, Wd, kp, c, 0);
    dw(bw.t0_kdw, kp, c, 0, kpos, 0, 0, 1, H, Wd, DW_PLAIN, ws, (int64_t)N * D);
    if (!dry()) {
      T0KnormArgs ka{kcur, cstride, kpos, B, N, (int)D};
      tag("t0_knorm B=%d N=%d D=%d", B, N, (int)D);
      launch(TURTLE_K_OTHER, ES * ((double)B * N * D * 3 + (double)N * D), 0, [&] { launch_t0_knorm<T>(ka, st); });
      if (Tnew > 1) {   // keep the last Tnew-1 cached frames (reference: cat then [-ntc:]); in place: no copy
        const int keep = Tnew - 1, first = Tin - keep;
        const bool kin_place = B == 1 && kout == kin + (int64_t)first * N * D;
        const bool vin_place = B == 1 && vout == vin + (int64_t)first * N * D;
        if (!kin_place || !vin_place) {
          tag("sab_cache_shift keep=%d N=%d", keep, N);
          launch(TURTLE_K_OTHER, 2.0 * ES * B * keep * (double)N * D * ((kin_place ? 0 : 1) + (vin_place ? 0 : 1)), 0, [&] {
            if (!kin_place)
              HIPCHK(hipMemcpy2DAsync(kout, (size_t)cstride * ES, kin + (int64_t)first * N * D, (size_t)Tin * N * D * ES,
                                      (size_t)keep * N * D * ES, B, hipMemcpyDeviceToDevice, st));
            if (!vin_place)
              HIPCHK(hipMemcpy2DAsync(vout, (size_t)cstride * ES, vin + (int64_t)first * N * D, (size_t)Tin * N * D * ES,
                                      (size_t)keep * N * D * ES, B, hipMemcpyDeviceToDevice, st));
          });
        }
      }
      // out = v of every frame, back to pixel-major frames (b, t) -> image b*NT + t
      T0UntokArgs ua{};
      for (int t = 0; t < NT; ++t) {
        ua.v[t] = t < Tin ? vin + (int64_t)t * N * D : vcur;
        ua.v_bstride[t] = t < Tin ? (int64_t)Tin * N * D : cstride;
      }
      ua.out = xs; ua.B = B; ua.T = NT; ua.H = H; ua.W = Wd; ua.C = c; ua.ws = ws;
      tag("t0_untok BT=%d H=%d W=%d C=%d", B * NT, H, Wd, c);
      launch(TURTLE_K_OTHER, 2.0 * ES * P * NT * c, 0, [&] { launch_t0_untok<T>(ua, st); });
    }
    chm_tail(b, bw, x, xs, kvd, fq, NT, H, Wd);
  }

  // Causal History Model: SAB + kv conv on the aligned frames + FHR (turtle_t1_arch.py:612-662)
  void chm(const Blk& b, const BlockW& bw, T* x, int H, int Wd) {
    if (h->arch.cfg.variant == 1) { chm_t0(b, bw, x, H, Wd); return; }
    const int c = b.dim, HW = H * Wd, ch = c / b.heads, ws = b.ws, slot = b.cache_slot;
    const int64_t P = (int64_t)B * HW;
    const int th = H / ws, tw = Wd / ws, N = th * tw, d2 = 2 * c, D = ws * ws * c;
    // q/k tokens come from a ws x ws stride-ws conv with padding 1: (H + 2 - ws) / ws + 1 per side,
    // which equals the v token grid H / ws only for ws >= 3. A CHM on an encoder / latent /
    // refinement level (Scale_patchsize 1 -> ws 2) makes the reference's attn @ v raise
    // (turtle_t1_arch.py:573-599): refuse it the same way instead of computing something else
    if ((H + 2 - ws) / ws + 1 != th || (Wd + 2 - ws) / ws + 1 != tw)
      TFAIL(TURTLE_EINVAL, "SAB q/k token grid " + std::to_string((H + 2 - ws) / ws + 1) + "x" +
                               std::to_string((Wd + 2 - ws) / ws + 1) + " != v token grid " + std::to_string(th) + "x" +
                               std::to_string(tw) + " (CHM with window " + std::to_string(ws) +
                               " cannot run: turtle_t1_arch.py:599 raises)");
    if (N < 5) TFAIL(TURTLE_EINVAL, "selected index k out of range: SAB needs >= 5 tokens (input too small)");
    const int Tin = slot >= 0 ? io->t_in[slot] : 0;
    const int NT = Tin + 1;
    const int Tnew = std::min(NT, b.ntc);
    // SAB caches: fresh outputs (slot) or scratch (a CHM outside a cache slot discards them)
    T* kout = slot >= 0 ? reinterpret_cast<T*>(io->k_out[slot]) : buf((int64_t)B * Tnew * N * d2);
    T* vout = slot >= 0 ? reinterpret_cast<T*>(io->v_out[slot]) : buf((int64_t)B * Tnew * N * D);
    const T* kin = slot >= 0 ? reinterpret_cast<const T*>(io->k_in[slot]) : nullptr;
    const T* vin = slot >= 0 ? reinterpret_cast<const T*>(io->v_in[slot]) : nullptr;
    T* qkd = buf(P * 2 * c);
    T* fq = buf(P * 3 * c);
    T* q2f = buf(P * d2);
    T* k2f = buf(P * d2);
    T* qtok = buf((int64_t)B * N * d2);
    // score blocks stage KT keys x d2 channels as 16-byte vectors split evenly over the block's
    // threads (sab.hip load_tile): 8 waves only where that split is whole (d2 = 320 / 448 at bf16
    // are not), else 4; a width neither divides is refused instead of reading stale LDS
    const int sab_kt = d2 <= 256 ? 64 : 32, sab_vec = 16 / (int)ES;
    auto sab_fits = [&](int w) { return d2 <= 512 && d2 % sab_vec == 0 && (sab_kt * (d2 / sab_vec)) % (w * 64) == 0; };
    int sab_waves = h->sab_waves ? h->sab_waves : (d2 >= 256 ? 8 : 4);
    if (!sab_fits(sab_waves)) sab_waves = 4;
    if (!sab_fits(sab_waves))
      TFAIL(TURTLE_EINVAL, "SAB token width " + std::to_string(d2) + " is not supported by the score kernel (d <= 512, whole 16-byte staging split)");
    const int nsplit = sab_score_nsplit(B, NT, N, d2, sab_waves);
    // partial lists sized for either block size, so the sab_waves switch never changes the workspace
    const int nsplit_ws = std::max(sab_score_nsplit(B, NT, N, d2, 4), sab_score_nsplit(B, NT, N, d2, 8));
    float* topv = fbuf((int64_t)B * NT * nsplit_ws * N * 5);
    int* topi = reinterpret_cast<int*>(fbuf((int64_t)B * NT * nsplit_ws * N * 5));
    float* ballv = fbuf((int64_t)B * NT * N * 41);
    int* ccnt = reinterpret_cast<int*>(fbuf((int64_t)B * NT * N));
    int* cidx = reinterpret_cast<int*>(fbuf((int64_t)B * NT * N * SAB_MAXC));
    float* cwt = fbuf((int64_t)B * NT * N * SAB_MAXC);
    T* xs = buf(P * NT * c);
    T* kvd = buf(P * NT * 2 * c);
    // LN(x) -> [SAB qk | SAB v | FHR qkv] -> their depthwise convs; SAB v goes straight into the new
    // cache's current frame in the dilated token-major layout
    T* vcur = vout + (int64_t)(Tnew - 1) * N * D;
    if (can_fuse(c, F_DWONLY, 6 * c, 0)) {
      FusedDst dv{vcur, 0, 0, 2 * c, 3 * c, c, ws, (int64_t)Tnew * N * D};
      fused(F_DWONLY, bw.a_in, bw.chm_dw6, x, c, 0, c, B, H, Wd, 6 * c, nullptr, nullptr, nullptr,
            {dst_map(qkd, 2 * c, 0, 0, 2 * c), dv, dst_map(fq, 3 * c, 0, 3 * c, 6 * c)});
    } else {
      T* t6 = buf(P * 6 * c);
      gemm(bw.a_in, src1(x, c, 0, c), P, HW, Wd, t6, 6 * c, 0);
      dw(bw.sab_qk_dw, t6, 6 * c, 0, qkd, 2 * c, 0, B, H, Wd, DW_PLAIN);
      dw(bw.sab_v_dw, t6, 6 * c, 2 * c, vcur, 0, 0, B, H, Wd, DW_PLAIN, ws, (int64_t)Tnew * N * D);
      dw(bw.fhr_dw, t6, 6 * c, 3 * c, fq, 3 * c, 0, B, H, Wd, DW_PLAIN);
    }
    gemm(bw.q2, src1(qkd, 2 * c, 0, c), P, HW, Wd, q2f, d2, 0);
    gemm(bw.k2, src1(qkd, 2 * c, c, c), P, HW, Wd, k2f, d2, 0);
    if (!dry()) {
      WinArgs wa{};
      wa.in = q2f; wa.ldi = d2; wa.offi = 0; wa.w = h->fptr(bw.q2_win); wa.bias = h->fptr(bw.q2_winb);
      wa.out = qtok; wa.out_img_stride = (int64_t)N * d2; wa.nimg = B; wa.H = H; wa.W = Wd; wa.C = d2; wa.ws = ws;
      const double wbytes = ES * ((double)P * d2 + (double)B * N * d2), wflops = 2.0 * P * d2;
      launch(TURTLE_K_WINDOW, wbytes, wflops, [&] { launch_window<T>(wa, st); });
      wa.in = k2f; wa.w = h->fptr(bw.k2_win); wa.bias = h->fptr(bw.k2_winb);
      wa.out = kout + (int64_t)(Tnew - 1) * N * d2; wa.out_img_stride = (int64_t)Tnew * N * d2;
      launch(TURTLE_K_WINDOW, wbytes, wflops, [&] { launch_window<T>(wa, st); });
      // keep the last Tnew-1 cached frames in the new cache (reference: cat then [-ntc:])
      // (a kept frame already in place - the caller's frame arena, model.py _sab_out - is not copied)
      if (Tnew > 1) {
        const int keep = Tnew - 1, first = Tin - keep;
        const bool kin_place = B == 1 && kout == kin + (int64_t)first * N * d2;
        const bool vin_place = B == 1 && vout == vin + (int64_t)first * N * D;
        if (!kin_place || !vin_place) {
          tag("sab_cache_shift keep=%d N=%d", keep, N);
          launch(TURTLE_K_OTHER, 2.0 * ES * B * keep * (double)N * ((kin_place ? 0 : d2) + (vin_place ? 0 : D)), 0, [&] {
            if (!kin_place)
              HIPCHK(hipMemcpy2DAsync(kout, (size_t)Tnew * N * d2 * ES, kin + (int64_t)first * N * d2, (size_t)Tin * N * d2 * ES,
                                      (size_t)keep * N * d2 * ES, B, hipMemcpyDeviceToDevice, st));
            if (!vin_place)
              HIPCHK(hipMemcpy2DAsync(vout, (size_t)Tnew * N * D * ES, vin + (int64_t)first * N * D, (size_t)Tin * N * D * ES,
                                      (size_t)keep * N * D * ES, B, hipMemcpyDeviceToDevice, st));
          });
        }
      }
      if (NT > TURTLE_MAX_T) TFAIL(TURTLE_EINVAL, "too many cached frames");
      SabScoreArgs sa{};
      sa.q = qtok; sa.q_bstride = (int64_t)N * d2; sa.B = B; sa.T = NT; sa.N = N; sa.d = d2;
      sa.th = th; sa.tw = tw; sa.nsplit = nsplit; sa.waves = sab_waves;
      sa.tau = h->fptr(bw.sab_tau); sa.topv = topv; sa.topi = topi; sa.ballv = ballv;
      SabGatherArgs ga{};
      ga.B = B; ga.T = NT; ga.N = N; ga.th = th; ga.tw = tw; ga.ws = ws; ga.C = c;
      ga.cnt = ccnt; ga.ci = cidx; ga.cw = cwt; ga.ballw = ballv; ga.out = xs; ga.db = h->sab_db;
      for (int t = 0; t < NT; ++t) {
        if (t < Tin) {
          sa.k[t] = kin + (int64_t)t * N * d2; sa.k_bstride[t] = (int64_t)Tin * N * d2;
          ga.v[t] = vin + (int64_t)t * N * D; ga.v_bstride[t] = (int64_t)Tin * N * D;
        } else {
          sa.k[t] = kout + (int64_t)(Tnew - 1) * N * d2; sa.k_bstride[t] = (int64_t)Tnew * N * d2;
          ga.v[t] = vout + (int64_t)(Tnew - 1) * N * D; ga.v_bstride[t] = (int64_t)Tnew * N * D;
        }
      }
      tag("sab_score B=%d T=%d N=%d d=%d nsplit=%d", B, NT, N, d2, nsplit);
      launch(TURTLE_K_SAB_SCORE, ES * (double)B * N * d2 * (1 + NT) + 8.0 * B * NT * N * (5 * nsplit + 41),
             2.0 * B * NT * (double)N * N * d2, [&] { launch_sab_score<T>(sa, st); });
      SabPrepArgs pa{};
      pa.topv = topv; pa.topi = topi; pa.ballv = ballv; pa.BT = B * NT; pa.N = N; pa.th = th; pa.tw = tw;
      pa.nsplit = nsplit; pa.cnt = ccnt; pa.ci = cidx; pa.cw = cwt; pa.ballw = ballv;
      tag("sab_prep BT=%d N=%d", B * NT, N);
      launch(TURTLE_K_SAB_AV, 4.0 * B * NT * (double)N * (10 * nsplit + 41 + 2 * SAB_MAXC), 0, [&] { launch_sab_prep(pa, st); });
      // <= 46 surviving keys per row (5 top + 41 ball): SURVEY.md §8(a) sparse A.v
      tag("sab_gather BT=%d N=%d D=%d", B * NT, N, D);
      launch(TURTLE_K_SAB_AV, ES * ((double)B * NT * N * D + (double)B * NT * HW * c),
             2.0 * B * NT * (double)N * 46 * D, [&] {
               if (h->sab_mfma && ES == 2 && sab_av_mfma_ok(ga)) launch_sab_av_mfma(ga, st);
               else launch_sab_gather<T>(ga, st);
             });
    }
    chm_tail(b, bw, x, xs, kvd, fq, NT, H, Wd);
  }

  // kv conv on the aligned frames + FHR(x, k_hist, v_hist) (turtle_t1_arch.py:640-662)
  void chm_tail(const Blk& b, const BlockW& bw, T* x, T* xs, T* kvd, T* fq, int NT, int H, int Wd) {
    const int c = b.dim, HW = H * Wd, ch = c / b.heads;
    const int64_t P = (int64_t)B * HW;
    // kv = (W_kv W_po) xs over the B*T aligned frames, then dw3x3 per frame
    if (can_fuse(c, F_DWONLY, 2 * c, 0)) {
      fused(F_DWONLY, bw.kv, bw.kv_dw, xs, c, 0, c, B * NT, H, Wd, 2 * c, nullptr, nullptr, nullptr,
            {dst_map(kvd, 2 * c, 0, 0, 2 * c)});
    } else {
      T* kv = buf(P * NT * 2 * c);
      gemm(bw.kv, src1(xs, c, 0, c), P * NT, HW, Wd, kv, 2 * c, 0);
      dw(bw.kv_dw, kv, 2 * c, 0, kvd, 2 * c, 0, B * NT, H, Wd, DW_PLAIN);
    }
    // FHR(x, k_hist, v_hist): keys = [hist frames..., current]
    std::vector<Seg> segs;
    SrcList vs{};
    for (int t = 0; t < NT; ++t) {
      segs.push_back(Seg{kvd, 2 * c, 0, ch, NT, t, 1, (int64_t)t * c, ch});
      vs.s[vs.n++] = SrcDesc{kvd, 2 * c, c, c, NT, t};
    }
    segs.push_back(Seg{fq, 3 * c, c, ch, 1, 0, 1, (int64_t)NT * c, ch});
    vs.s[vs.n++] = SrcDesc{fq, 3 * c, 2 * c, c, 1, 0};
    vs.Ktot = (NT + 1) * c;
    if ((int)segs.size() > TURTLE_MAX_SEG || vs.n > TURTLE_MAX_SRC) TFAIL(TURTLE_EINVAL, "too many history frames");
    chan_attn(bw, b, fq, 3 * c, 0, segs, vs, HW, Wd, x, nullptr, -1);
  }

  // runs a level on the pair (x, alt); returns the buffer holding the level's output
  T* level(int li, T* x, T* alt, int H, int Wd) {
    const auto& L = h->arch.levels[li];
    static const BlockW none{};   // workspace sizing runs before (or without) packed weights
    for (size_t i = 0; i < L.blocks.size(); ++i)
      block(L.blocks[i], dry() && h->mw.blocks.empty() ? none : h->mw.blocks[li][i], x, alt, H, Wd);
    return x;
  }

  void run(const float* inp, int Hin, int Win, float* out, int Hout, int Wout) {
    const Arch& A = h->arch;
    const int d = A.dim;
    const int64_t P1 = (int64_t)B * Hp * Wp;
    T* e1 = buf(P1 * d);
    T* e2 = buf(P1 / 4 * 2 * d);
    T* e3 = buf(P1 / 16 * 4 * d);
    T* lat = buf(P1 / 64 * 8 * d);
    T* d3 = buf(P1 / 16 * 4 * d);
    T* d2 = buf(P1 / 4 * 2 * d);
    T* d1 = buf(P1 * d);
    T* up = buf(P1 * d);      // Upsample output, largest at level 1: P1 * d/2... sized generously
    // ping-pong partners of the residual streams (fused blocks write out of place)
    T* a1 = buf(P1 * d);
    T* a2 = buf(P1 / 4 * 2 * d);
    T* a3 = buf(P1 / 16 * 4 * d);
    T* a4 = buf(P1 / 64 * 8 * d);
    T* a5 = buf(P1 / 16 * 4 * d);
    T* a6 = buf(P1 / 4 * 2 * d);
    if (!dry()) {
      StemArgs s{};
      s.inp = inp; s.in_bstride = (int64_t)2 * A.cfg.n_colors * Hin * Win; s.in_fstride = (int64_t)A.cfg.n_colors * Hin * Win;
      s.B = B; s.Cimg = A.cfg.n_colors; s.Hin = Hin; s.Win = Win; s.Hp = Hp; s.Wp = Wp;
      s.use_both = A.cfg.use_both_input; s.sr = A.cfg.super_resolution;
      s.w = h->fptr(h->mw.stem_w); s.bias = h->fptr(h->mw.stem_b); s.Cout = d; s.out = e1;
      tag("stem %dx%d", Hp, Wp);
      launch(TURTLE_K_OTHER, 4.0 * B * A.in_ch * Hin * Win + ES * (double)P1 * d, 18.0 * P1 * d * A.in_ch,
             [&] {
               if (h->stem_mfma && ES == 2 && stem_end_mfma_ok(d, A.in_ch, d)) launch_stem_mfma(s, st);
               else launch_stem<T>(s, st);
             });
    }
    int H = Hp, Wd = Wp;
    e1 = level(0, e1, a1, H, Wd);
    auto down = [&](int i, const T* x, int c, T* y, int H0, int W0) {
      if (i == 0 && ES == 2 && h->down_tile && h->mw.down_wf != NONE) {
        if (dry()) return;
        DownTileArgs dt{};
        dt.x = x; dt.ldx = c; dt.Cin = c; dt.wfrag = h->ptr(h->mw.down_wf); dt.out = y; dt.ldo = 2 * c;
        dt.nimg = B; dt.H = H0; dt.W = W0;
        if (down_tile_ok(dt)) {
          tag("down_tile nimg=%d H=%d W=%d C=%d", B, H0, W0, c);
          launch(TURTLE_K_GEMM, ES * (double)B * H0 * W0 * (c + c / 2), 2.0 * B * H0 * W0 * (c / 2) * 9.0 * c,
                 [&] { launch_down_tile(dt, st); });
          return;
        }
      }
      gemm(h->mw.down[i], src1(x, c, 0, 9 * c), (int64_t)B * H0 * W0, H0 * W0, W0, y, 2 * c, 0, nullptr, 0, 0, 0,
           STORE_UNSHUFFLE, nullptr, 0, 1, -1, nullptr, 1, c);
    };
    down(0, e1, d, e2, Hp, Wp);
    e2 = level(1, e2, a2, Hp / 2, Wp / 2);
    down(1, e2, 2 * d, e3, Hp / 2, Wp / 2);
    e3 = level(2, e3, a3, Hp / 4, Wp / 4);
    down(2, e3, 4 * d, lat, Hp / 4, Wp / 4);
    lat = level(3, lat, a4, Hp / 8, Wp / 8);
    auto upcat = [&](int i, const T* x, int c, int H0, int W0, const T* skip, T* y) {
      // Upsample (3x3 c->2c + PixelShuffle) into `up`, then reduce_chan over [up | skip]
      gemm(h->mw.up[i], src1(x, c, 0, 9 * c), (int64_t)B * H0 * W0, H0 * W0, W0, up, c / 2, 0, nullptr, 0, 0, 0,
           STORE_SHUFFLE, nullptr, 0, 1, -1, nullptr, 1, c);
      SrcList s{}; s.n = 2; s.Ktot = c;
      s.s[0] = SrcDesc{up, c / 2, 0, c / 2, 1, 0};
      s.s[1] = SrcDesc{skip, c / 2, 0, c / 2, 1, 0};
      if (i == 2 && h->mw.reduce_split) {          // split-bf16 weights: the same two sources twice
        s.n = 4; s.Ktot = 2 * c; s.s[2] = s.s[0]; s.s[3] = s.s[1];
      }
      const int H1 = 2 * H0, W1 = 2 * W0;
      gemm(h->mw.reduce[i], s, (int64_t)B * H1 * W1, H1 * W1, W1, y, c / 2, 0);
    };
    upcat(0, lat, 8 * d, Hp / 8, Wp / 8, e3, d3);
    d3 = level(4, d3, a5, Hp / 4, Wp / 4);
    upcat(1, d3, 4 * d, Hp / 4, Wp / 4, e2, d2);
    d2 = level(5, d2, a6, Hp / 2, Wp / 2);
    upcat(2, d2, 2 * d, Hp / 2, Wp / 2, e1, d1);
    // decoder_level1 + refinement ping-pong with a1 (the encoder-1 partner; e1 itself is consumed)
    T* d1alt = e1 == a1 ? up : a1;
    d1 = level(6, d1, d1alt, Hp, Wp);
    d1 = level(7, d1, d1 == d1alt ? (d1alt == up ? a1 : up) : d1alt, Hp, Wp);
    if (!dry()) {
      EndArgs e{};
      e.x = d1; e.Cin = d; e.w = h->fptr(h->mw.end_w); e.bias = h->fptr(h->mw.end_b);
      e.wfrag = h->ptr(h->mw.end_wf);
      e.inp = inp; e.in_bstride = (int64_t)2 * A.cfg.n_colors * Hin * Win; e.in_fstride = (int64_t)A.cfg.n_colors * Hin * Win;
      e.B = B; e.Cimg = A.cfg.n_colors; e.Hin = Hin; e.Win = Win; e.Hp = Hp; e.Wp = Wp; e.Hout = Hout; e.Wout = Wout;
      e.sr = A.cfg.super_resolution; e.out = out;
      tag("ending %dx%d", Hout, Wout);
      launch(TURTLE_K_OTHER, ES * (double)P1 * d + 8.0 * B * A.out_ch * Hout * Wout, 18.0 * P1 * d * A.out_ch,
             [&] {
               if (!(h->stem_mfma && ES == 2 && stem_end_mfma_ok(d, A.in_ch, d) && e.wfrag && launch_ending_mfma(e, st)))
                 launch_ending<T>(e, st);
             });
    }
  }
};

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------
template <typename F>
static int guard(F&& f) {
  try {
    f();
    return TURTLE_OK;
  } catch (const TurtleError& e) {
    g_err = e.what();
    return e.code;
  } catch (const std::exception& e) {
    g_err = e.what();
    return TURTLE_EINVAL;
  }
}

static void padded(const TurtleHandle* h, int H, int W, int& Hp, int& Wp, int& Hout, int& Wout) {
  const int s = h->arch.cfg.super_resolution ? 4 : 1;
  Hout = H * s; Wout = W * s;
  Hp = (Hout + 31) / 32 * 32;
  Wp = (Wout + 31) / 32 * 32;
}

template <typename T>
static size_t ws_size(TurtleHandle* h, int B, int H, int W) {
  int Hp, Wp, Ho, Wo;
  padded(h, H, W, Hp, Wp, Ho, Wo);
  CacheIO io{};
  for (const auto& L : h->arch.levels)
    for (const auto& b : L.blocks)
      if (b.cache_slot >= 0) io.t_in[b.cache_slot] = b.attn == TURTLE_ATTN_FHR ? b.ntc * (b.dim / b.heads) : b.ntc;
  Runner<T> r{h, nullptr, Arena{nullptr, 0, 0, 0, true}, B, Hp, Wp, &io};
  r.run(nullptr, H, W, nullptr, Ho, Wo);
  return r.ar.peak + 4096;
}

extern "C" {

const char* turtle_last_error(void) { return g_err.c_str(); }

int turtle_profile_begin(TurtleHandle* h, int kernel_class) {
  return guard([&] {
    if (!h) TFAIL(TURTLE_EINVAL, "null handle");
    h->prof.clear();
    h->ev_used = 0;
    h->prof_cls = kernel_class;
  });
}

int turtle_profile_end(TurtleHandle* h, double out[4 * TURTLE_K_COUNT]) {
  return guard([&] {
    if (!h || !out) TFAIL(TURTLE_EINVAL, "null argument");
    for (int i = 0; i < 4 * TURTLE_K_COUNT; ++i) out[i] = 0;
    const char* dump = getenv("TURTLE_PROF_DUMP");   // per-launch lines: class ms bytes flops tag
    FILE* df = dump ? fopen(dump, "a") : nullptr;
    for (auto& r : h->prof) {
      HIPCHK(hipEventSynchronize(r.b));
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, r.a, r.b));
      if (df) fprintf(df, "%d\t%.4f\t%.0f\t%.0f\t%s\n", r.cls, ms, r.bytes, r.flops, r.tag.c_str());
      if (r.cls < 0 || r.cls >= TURTLE_K_COUNT) continue;
      out[4 * r.cls] += ms;
      out[4 * r.cls + 1] += 1;
      out[4 * r.cls + 2] += r.bytes;
      out[4 * r.cls + 3] += r.flops;
    }
    if (df) fclose(df);
    h->prof.clear();
    h->ev_used = 0;
    h->prof_cls = -1;
  });
}

int turtle_profile_filter(TurtleHandle* h, const char* tag) {
  return guard([&] {
    if (!h) TFAIL(TURTLE_EINVAL, "null handle");
    h->prof_filter = tag ? tag : "";
  });
}

int turtle_set_option(TurtleHandle* h, const char* name, int value) {
  return guard([&] {
    if (!h || !name) TFAIL(TURTLE_EINVAL, "null argument");
    const std::string n = name;
    if (n == "fuse") h->fuse = value != 0;
    else if (n == "fuse_fp32") h->fuse_fp32 = value != 0;
    else if (n == "panel_gemm") h->panel = value != 0;
    else if (n == "dw_rows") h->dw_rows = value != 0;
    else if (n == "dwgemm") h->dwgemm = value != 0;
    else if (n == "dwgemm_attn") h->dwgemm_attn = value != 0;
    else if (n == "dwgemm_cb") h->dwgemm_cb = value != 0;
    else if (n == "split_out") {                 // changes the packed weights: re-pack when loaded
      h->split_out = value != 0;
      if (h->loaded) pack_all(h);
    }
    else if (n == "ffn") h->ffn = value != 0;
    else if (n == "tilepd") h->tilepd = value != 0;
    else if (n == "tilepd_cb") h->tilepd_cb = value != 0;
    else if (n == "tilepd_gate") h->tilepd_gate = value != 0;
    else if (n == "gffn") h->gffn = value != 0;
    else if (n == "gffn_min_blocks") h->gffn_min_blocks = (int)value;
    else if (n == "gffn_c128") h->gffn_c128 = value != 0;
    else if (n == "gffn_c64") h->gffn_c64 = value != 0;
    else if (n == "tilepd_min_blocks") h->tilepd_min_blocks = (int)value;
    else if (n == "down_tile") h->down_tile = value != 0;
    else if (n == "sab_db") h->sab_db = (int)value;
    else if (n == "dwgemm_min_blocks") h->dwgemm_min_blocks = (int)value;
    else if (n == "gemm_lds") h->gemm_lds = value != 0;
    else if (n == "gemm_pn") h->gemm_pn = value != 0;
    else if (n == "gemm_ar") h->gemm_ar = value != 0;
    else if (n == "gemm_kt") h->gemm_kt = value != 0;
    else if (n == "gemm_f32") h->gemm_f32 = value != 0;
    else if (n == "gemm_sk") h->gemm_sk = value != 0;
    else if (n == "sk_max_px") h->sk_max_px = value;
    else if (n == "gemm8") h->gemm8 = (int)value;
    else if (n == "gemm8_ps") h->gemm8_ps = value != 0;
    else if (n == "gemm9") h->gemm9 = (int)value;
    else if (n == "attn_fin") h->attn_fin = value != 0;
    else if (n == "sab_waves") h->sab_waves = (int)value;
    else if (n == "kt_max_px") h->kt_max_px = (int)value;
    else if (n == "sab_mfma") h->sab_mfma = value != 0;
    else if (n == "stem_mfma") h->stem_mfma = value != 0;
    else if (n == "fused2") h->fused2 = value != 0;
    else TFAIL(TURTLE_EINVAL, "unknown option '" + n + "'");
  });
}

int turtle_create(const TurtleConfig* cfg, TurtleHandle** out) {
  return guard([&] {
    if (!cfg || !out) TFAIL(TURTLE_EINVAL, "null argument");
    auto* h = new TurtleHandle();
    h->arch.cfg = *cfg;
    try {
      build_arch(h->arch);
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

void turtle_destroy(TurtleHandle* h) {
  if (!h) return;
  for (auto e : h->ev_pool) (void)hipEventDestroy(e);
  if (h->dev) (void)hipFree(h->dev);
  delete h;
}

int turtle_num_weights(const TurtleHandle* h) { return h ? (int)h->arch.params.size() : 0; }

int turtle_weight_info(const TurtleHandle* h, int idx, const char** name, int* ndim, int64_t shape[4]) {
  return guard([&] {
    if (!h || idx < 0 || idx >= (int)h->arch.params.size()) TFAIL(TURTLE_EINVAL, "weight index out of range");
    const auto& p = h->arch.params[idx];
    *name = p.first.c_str();
    *ndim = (int)p.second.size();
    for (int i = 0; i < 4; ++i) shape[i] = i < *ndim ? p.second[i] : 1;
  });
}

int turtle_set_weight(TurtleHandle* h, const char* name, const float* data, int64_t numel) {
  return guard([&] {
    if (!h || !name || !data) TFAIL(TURTLE_EINVAL, "null argument");
    for (const auto& p : h->arch.params) {
      if (p.first != name) continue;
      int64_t n = 1;
      for (auto s : p.second) n *= s;
      if (n != numel) TFAIL(TURTLE_ENOWEIGHT, std::string("size mismatch for ") + name);
      h->staged[name] = std::vector<float>(data, data + numel);
      h->loaded = false;
      return;
    }
    TFAIL(TURTLE_ENOWEIGHT, std::string("unexpected key ") + name + " in state_dict");
  });
}

int turtle_load_weights(TurtleHandle* h) {
  return guard([&] {
    if (!h) TFAIL(TURTLE_EINVAL, "null handle");
    for (const auto& p : h->arch.params)
      if (!h->staged.count(p.first)) TFAIL(TURTLE_ENOWEIGHT, "missing key " + p.first + " in state_dict");
    pack_all(h);
    h->loaded = true;
  });
}

int turtle_cache_layout(const TurtleHandle* h, int B, int H, int W, const int t_in[8], int kind[8],
                        int64_t k_shape[40], int64_t v_shape[40]) {
  return guard([&] {
    if (!h || B <= 0 || H <= 0 || W <= 0) TFAIL(TURTLE_EINVAL, "bad shape");
    int Hp, Wp, Ho, Wo;
    padded(h, H, W, Hp, Wp, Ho, Wo);
    for (int i = 0; i < 40; ++i) k_shape[i] = v_shape[i] = 1;
    for (int i = 0; i < 8; ++i) kind[i] = 0;
    for (const auto& L : h->arch.levels)
      for (const auto& b : L.blocks) {
        if (b.cache_slot < 0) continue;
        const int s = b.cache_slot, Hl = Hp / L.scale, Wl = Wp / L.scale, c = b.dim;
        int64_t* ks = k_shape + 5 * s;
        int64_t* vs = v_shape + 5 * s;
        if (b.attn == TURTLE_ATTN_FHR) {
          const int ch = c / b.heads;
          const int rows = std::min(t_in[s] + ch, b.ntc * ch);
          kind[s] = 1;
          ks[0] = vs[0] = B; ks[1] = vs[1] = b.heads; ks[2] = vs[2] = rows; ks[3] = vs[3] = (int64_t)Hl * Wl;
        } else if (b.attn == TURTLE_ATTN_CHM) {
          const int N = (Hl / b.ws) * (Wl / b.ws);
          const int frames = std::min(t_in[s] + 1, b.ntc);
          kind[s] = 2;
          ks[0] = vs[0] = B; ks[1] = vs[1] = frames; ks[2] = vs[2] = 1; ks[3] = vs[3] = N;
          vs[4] = (int64_t)b.ws * b.ws * c;
          ks[4] = h->arch.cfg.variant == 1 ? vs[4] : 2 * c;   // t0 caches dilated k tokens (turtle_arch.py:480-491)
        }
      }
  });
}

int turtle_workspace_size(const TurtleHandle* h, int B, int H, int W, size_t* bytes) {
  return guard([&] {
    if (!h || !bytes || B <= 0 || H <= 0 || W <= 0) TFAIL(TURTLE_EINVAL, "bad argument");
    auto* hh = const_cast<TurtleHandle*>(h);
    *bytes = h->bf16() ? ws_size<bf16>(hh, B, H, W) : ws_size<float>(hh, B, H, W);
  });
}

int turtle_forward(TurtleHandle* h, const float* inp, int B, int H, int W, float* out,
                   const void* const k_in[8], const void* const v_in[8], const int t_in[8],
                   void* const k_out[8], void* const v_out[8], void* workspace, size_t workspace_bytes,
                   void* stream) {
  return guard([&] {
    if (!h) TFAIL(TURTLE_EINVAL, "null handle");
    if (!h->loaded) TFAIL(TURTLE_ESTATE, "turtle_load_weights has not been called");
    if (!inp || !out || B <= 0 || H <= 0 || W <= 0) TFAIL(TURTLE_EINVAL, "bad input");
    int Hp, Wp, Ho, Wo;
    padded(h, H, W, Hp, Wp, Ho, Wo);
    CacheIO io{};
    int kind[8];
    int64_t ks[40], vs[40];
    turtle_cache_layout(h, B, H, W, t_in, kind, ks, vs);
    for (int i = 0; i < 8; ++i) {
      io.k_in[i] = k_in ? k_in[i] : nullptr;
      io.v_in[i] = v_in ? v_in[i] : nullptr;
      io.t_in[i] = t_in ? t_in[i] : 0;
      io.k_out[i] = k_out ? k_out[i] : nullptr;
      io.v_out[i] = v_out ? v_out[i] : nullptr;
      if (kind[i] && (!io.k_out[i] || !io.v_out[i])) TFAIL(TURTLE_EINVAL, "missing cache output buffer for slot " + std::to_string(i));
      if (kind[i] && io.t_in[i] && (!io.k_in[i] || !io.v_in[i])) TFAIL(TURTLE_EINVAL, "missing cache input for slot " + std::to_string(i));
      if (!kind[i]) io.t_in[i] = 0;
    }
    // validate incoming cache extents
    for (const auto& L : h->arch.levels)
      for (const auto& b : L.blocks) {
        if (b.cache_slot < 0) continue;
        const int s = b.cache_slot;
        if (b.attn == TURTLE_ATTN_FHR) {
          const int ch = b.dim / b.heads;
          if (io.t_in[s] % ch || io.t_in[s] > b.ntc * ch) TFAIL(TURTLE_EINVAL, "bad FHR cache rows");
          if (io.t_in[s] / ch + 1 > TURTLE_MAX_SEG) TFAIL(TURTLE_EINVAL, "FHR cache too long");
        } else if (b.attn == TURTLE_ATTN_CHM) {
          if (io.t_in[s] > b.ntc) TFAIL(TURTLE_EINVAL, "bad SAB cache frames");
          if (io.t_in[s] + 2 > TURTLE_MAX_SEG) TFAIL(TURTLE_EINVAL, "SAB cache too long");
        }
      }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    auto go = [&](auto tag) {
      using T = decltype(tag);
      Runner<T> r{h, st, Arena{reinterpret_cast<char*>(workspace), workspace_bytes, 0, 0, false}, B, Hp, Wp, &io};
      r.run(inp, H / 1, W / 1, out, Ho, Wo);
    };
    if (h->bf16()) go(bf16{}); else go(float{});
    HIPCHK(hipGetLastError());
  });
}

}  // extern "C"

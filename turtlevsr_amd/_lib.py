"""ctypes binding of libturtle_hip.so (include/turtle_hip.h).

The product path has no fallback: if the library is missing or fails to load, importing the
HIP model raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TURTLE_HIP_LIB", os.path.join(_HERE, "lib", "libturtle_hip.so"))

DTYPE_F32, DTYPE_BF16 = 0, 1
ATTN = {"ReducedAttn": 0, "Channel": 1, "FHR": 2, "CHM": 3, "NoAttn": 4}
FFN = {"FFW": 0, "GFFW": 1}


class TurtleConfig(C.Structure):
    _fields_ = [
        ("n_colors", C.c_int), ("dim", C.c_int), ("enc_blocks", C.c_int * 3), ("middle_blocks", C.c_int),
        ("dec_blocks", C.c_int * 3), ("num_refinement_blocks", C.c_int), ("ffn_expansion_factor", C.c_float),
        ("bias", C.c_int), ("layernorm_biasfree", C.c_int), ("use_both_input", C.c_int),
        ("num_frames_tocache", C.c_int), ("num_heads", C.c_int * 4), ("level_attn", (C.c_int * 2) * 7),
        ("level_ffn", C.c_int * 7), ("latent_attn", C.c_int * 3), ("latent_ffn", C.c_int),
        ("super_resolution", C.c_int), ("dtype", C.c_int), ("variant", C.c_int),
    ]


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    # torch's bundled HIP runtime must be the one our library binds to (same soname
    # libamdhip64.so.7): load torch first, or two HIP runtimes would coexist in the process.
    import torch  # noqa: F401
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libturtle_hip.so not found at {LIB_PATH}: run `python -m turtlevsr_amd.build`")
    L = C.CDLL(LIB_PATH)
    vp, ip, i64p = C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int64)
    L.turtle_create.argtypes = [C.POINTER(TurtleConfig), C.POINTER(vp)]
    L.turtle_destroy.argtypes = [vp]
    L.turtle_destroy.restype = None
    L.turtle_num_weights.argtypes = [vp]
    L.turtle_weight_info.argtypes = [vp, C.c_int, C.POINTER(C.c_char_p), ip, i64p]
    L.turtle_set_weight.argtypes = [vp, C.c_char_p, vp, C.c_int64]
    L.turtle_load_weights.argtypes = [vp]
    L.turtle_cache_layout.argtypes = [vp, C.c_int, C.c_int, C.c_int, ip, ip, i64p, i64p]
    L.turtle_workspace_size.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_size_t)]
    L.turtle_forward.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, vp, C.POINTER(vp), C.POINTER(vp), ip,
                                 C.POINTER(vp), C.POINTER(vp), vp, C.c_size_t, vp]
    L.turtle_profile_begin.argtypes = [vp, C.c_int]
    L.turtle_profile_end.argtypes = [vp, C.POINTER(C.c_double)]
    L.turtle_profile_filter.argtypes = [vp, C.c_char_p]
    L.turtle_set_option.argtypes = [vp, C.c_char_p, C.c_int]
    L.turtle_last_error.restype = C.c_char_p
    L.turtle_source_hash.restype = C.c_char_p
    check_source_hash(L)
    _lib = L
    return L


def check_source_hash(L, expected: str | None = None):
    """The loaded library must be built from this tree's kernel sources (the .so is git-ignored and
    travels prebuilt): a stale library raises unless TURTLE_ALLOW_STALE_LIB=1."""
    got = L.turtle_source_hash().decode()
    if expected is None:
        from .build import source_hash
        expected = source_hash()
    if got != expected and os.environ.get("TURTLE_ALLOW_STALE_LIB") != "1":
        raise RuntimeError(f"{LIB_PATH} was built from kernel sources {got}, this tree's are {expected}: "
                           "rebuild with `python -m turtlevsr_amd.build` (or set TURTLE_ALLOW_STALE_LIB=1)")
    return got


def source_hash() -> str:
    """The kernel-source hash the loaded library reports (turtle_source_hash)."""
    return lib().turtle_source_hash().decode()


EXPORTED = ["turtle_create", "turtle_destroy", "turtle_num_weights", "turtle_weight_info", "turtle_set_weight",
            "turtle_load_weights", "turtle_cache_layout", "turtle_workspace_size", "turtle_forward",
            "turtle_profile_begin", "turtle_profile_end", "turtle_profile_filter", "turtle_set_option",
            "turtle_last_error", "turtle_source_hash"]
K_CLASSES = ["gemm", "dwconv", "chan_attn", "sab_score", "sab_av", "sab_window", "other", "fused"]
K_ALL = 99


def check(rc: int):
    if rc != 0:
        msg = lib().turtle_last_error().decode(errors="replace")
        raise RuntimeError(f"libturtle_hip error {rc}: {msg}")


def config_from_arch(arch, sr: bool, dtype: int) -> TurtleConfig:
    """Fill the C config from a resolved ``turtlevsr_amd.arch.TurtleArch``."""
    cfg = TurtleConfig()
    lv = arch.levels
    cfg.n_colors = arch.out_ch
    cfg.dim = arch.dim
    for i, n in enumerate(("encoder_level1", "encoder_level2", "encoder_level3")):
        cfg.enc_blocks[i] = len(lv[n].blocks)
    cfg.middle_blocks = len(lv["latent"].blocks)
    for i, n in enumerate(("decoder_level3", "decoder_level2", "decoder_level1")):
        cfg.dec_blocks[i] = len(lv[n].blocks)
    cfg.num_refinement_blocks = len(lv["refinement"].blocks)
    cfg.ffn_expansion_factor = float(arch.ffe)
    cfg.bias = int(arch.bias)
    cfg.layernorm_biasfree = int(arch.ln_type == "BiasFree")
    cfg.use_both_input = int(arch.use_both)
    cfg.num_frames_tocache = arch.ntc
    cfg.num_heads[:] = list(arch.heads)
    order = ("encoder_level1", "encoder_level2", "encoder_level3", "decoder_level3", "decoder_level2",
             "decoder_level1", "refinement")
    for i, n in enumerate(order):
        blocks = lv[n].blocks
        cfg.level_attn[i][0] = ATTN[blocks[0].attn] if len(blocks) > 1 else ATTN.get(arch.type1[n], 0)
        cfg.level_attn[i][1] = ATTN[blocks[-1].attn]
        cfg.level_ffn[i] = FFN[blocks[0].ffn]
    lb = lv["latent"].blocks
    cfg.latent_attn[0] = ATTN[lb[0].attn]
    cfg.latent_attn[1] = ATTN[lb[1].attn] if len(lb) > 2 else ATTN.get(arch.type1["latent_mid"], 0)
    cfg.latent_attn[2] = ATTN[lb[-1].attn]
    cfg.latent_ffn = FFN[lb[0].ffn]
    cfg.super_resolution = int(sr)
    cfg.dtype = dtype
    cfg.variant = int(getattr(arch, "t0", False))
    return cfg

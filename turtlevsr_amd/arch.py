"""Architecture resolution: option dict -> levels / blocks (make_model, turtle_t1_arch.py:10-53).

Pure host logic shared by the parameter holder (``model.py``) and the HIP frame driver
(``model.py`` / ``csrc/turtle.cpp``). It reads the same keys with the same defaults as the reference's
``make_model`` and mirrors the level wiring of ``Turtle_t1.__init__`` (turtle_t1_arch.py:932-1043):

* ``LevelBlock`` (813-865): ``num_blocks - 1`` blocks of ``attn_type1`` then one ``attn_type2``;
  only the last block sees the history cache.
* ``LatentCacheBlock`` (867-928): first block ``attn_type1``, middle ``attn_type2``, last
  ``attn_type3``; first and last see caches [3] and [4].
* decoder_level3/2/1 read the ``decoder1/2/3`` keys, use Scale_patchsize 2/4/8 (SAB window 4/8/16)
  and decoder_level1 forces ``num_frames_tocache = 2`` (1009-1027).

Unknown attention / FFN types raise ``ValueError`` (the reference prints and calls ``exit()``,
790-792, 800-802).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List

ATTN_TYPES = ("ReducedAttn", "Channel", "FHR", "CHM", "NoAttn")
FFN_TYPES = ("FFW", "GFFW")

# cache slot of each level's cache-carrying block (Turtle_t1.forward 1065-1124)
CACHE_SLOTS = ["encoder_level1", "encoder_level2", "encoder_level3", "latent.first",
               "latent.last", "decoder_level3", "decoder_level2", "decoder_level1"]


@dataclass
class BlockSpec:
    prefix: str
    dim: int
    attn: str
    ffn: str
    heads: int
    ntc: int
    ws: int
    hidden: int          # GatedFeedForward hidden width int(dim * ffn_expansion_factor)


@dataclass
class LevelSpec:
    name: str
    dim: int
    blocks: List[BlockSpec] = field(default_factory=list)


@dataclass
class TurtleArch:
    dim: int
    in_ch: int           # channels entering input_projection (x2 with use_both_input)
    out_ch: int
    bias: bool
    ln_type: str
    use_both: bool
    ntc: int
    levels: Dict[str, LevelSpec]
    ffe: float = 1.0
    heads: tuple = (1, 1, 1, 1)
    type1: Dict[str, str] = field(default_factory=dict)   # raw attn_type1 per level (+ latent_mid)
    t0: bool = False     # option `model: Turtle_arch` -> the t0 network (turtle_arch.py)

    @property
    def order(self):
        return ["encoder_level1", "encoder_level2", "encoder_level3", "latent",
                "decoder_level3", "decoder_level2", "decoder_level1", "refinement"]


def _check(attn: str, ffn: str):
    if attn not in ATTN_TYPES:
        raise ValueError(f"{attn} Not defined (turtle_t1_arch.py:790-792)")
    if ffn not in FFN_TYPES:
        raise ValueError(f"{ffn} Not defined (turtle_t1_arch.py:800-802)")


def resolve(opt: dict) -> TurtleArch:
    dim = int(opt["dim"])
    heads = list(opt.get("num_heads", [1, 1, 1, 1]))
    ntc = int(opt.get("num_frames_tocache", 1))
    ffe = opt.get("ffn_expansion_factor", 1)
    bias = bool(opt.get("bias", False))
    o = opt

    def level(name, d, n, t1, t2, ffw, h, nt, scale):
        lv = LevelSpec(name, d)
        for i in range(n):
            a = t2 if i == n - 1 else t1
            _check(a, ffw)
            lv.blocks.append(BlockSpec(f"{name}.transformer_blocks.{i}", d, a, ffw, h, nt, 2 * scale, int(d * ffe)))
        return lv

    def latent(name, d, n, t1, t2, t3, ffw, h, nt):
        if n < 2:
            raise ValueError("LatentCacheBlock should have more than 2 layers (turtle_t1_arch.py:899-901)")
        lv = LevelSpec(name, d)
        for i in range(n):
            a = t1 if i == 0 else (t3 if i == n - 1 else t2)
            _check(a, ffw)
            lv.blocks.append(BlockSpec(f"{name}.transformer_blocks.{i}", d, a, ffw, h, nt, 2, int(d * ffe)))
        return lv

    eb, db = o["Enc_blocks"], o["Dec_blocks"]
    levels = {
        "encoder_level1": level("encoder_level1", dim, eb[0], o["encoder1_attn_type1"], o["encoder1_attn_type2"], o["encoder1_ffw_type"], heads[0], ntc, 1),
        "encoder_level2": level("encoder_level2", dim * 2, eb[1], o["encoder2_attn_type1"], o["encoder2_attn_type2"], o["encoder2_ffw_type"], heads[1], ntc, 1),
        "encoder_level3": level("encoder_level3", dim * 4, eb[2], o["encoder3_attn_type1"], o["encoder3_attn_type2"], o["encoder3_ffw_type"], heads[2], ntc, 1),
        "latent": latent("latent", dim * 8, o["Middle_blocks"], o["latent_attn_type1"], o["latent_attn_type2"], o["latent_attn_type3"], o["latent_ffw_type"], heads[3], ntc),
        "decoder_level3": level("decoder_level3", dim * 4, db[0], o["decoder1_attn_type1"], o["decoder1_attn_type2"], o["decoder1_ffw_type"], heads[2], ntc, 2),
        "decoder_level2": level("decoder_level2", dim * 2, db[1], o["decoder2_attn_type1"], o["decoder2_attn_type2"], o["decoder2_ffw_type"], heads[1], ntc, 4),
        "decoder_level1": level("decoder_level1", dim, db[2], o["decoder3_attn_type1"], o["decoder3_attn_type2"], o["decoder3_ffw_type"], heads[0], 2, 8),
        "refinement": level("refinement", dim, o.get("num_refinement_blocks", 1), o["refinement_attn_type1"], o["refinement_attn_type2"], o["refinement_ffw_type"], heads[0], ntc, 1),
    }
    use_both = bool(o["use_both_input"])
    n_col = int(o["n_colors"])
    type1 = {"encoder_level1": o["encoder1_attn_type1"], "encoder_level2": o["encoder2_attn_type1"],
             "encoder_level3": o["encoder3_attn_type1"], "decoder_level3": o["decoder1_attn_type1"],
             "decoder_level2": o["decoder2_attn_type1"], "decoder_level1": o["decoder3_attn_type1"],
             "refinement": o["refinement_attn_type1"], "latent_mid": o["latent_attn_type2"]}
    return TurtleArch(dim=dim, in_ch=n_col * (2 if use_both else 1), out_ch=n_col, bias=bias,
                      ln_type=o.get("LayerNorm_type", "WithBias"), use_both=use_both, ntc=ntc,
                      levels=levels, ffe=ffe, heads=tuple(heads), type1=type1, t0=is_t0(o))


def is_t0(opt: dict) -> bool:
    """`model` selects the arch module (video_restoration_model.py:18-21): Turtle_arch is the t0
    network (turtle_arch.py, StateAlignBlock 459-533), anything else Turtle_t1 / TurtleSuper_t1."""
    return str(opt.get("model", "")).lower() in ("turtle_arch", "turtle")

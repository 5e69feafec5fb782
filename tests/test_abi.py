"""CPU-side checks of the C ABI: the library loads, exports every symbol of include/turtle_hip.h,
reproduces the reference state_dict surface, sizes workspaces and reports errors. No kernels run."""
import ctypes as C
import json
import os
import re

import pytest
import yaml

from golden_io import key_shapes
from turtlevsr_amd import _lib
from turtlevsr_amd.arch import resolve

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOPRO = os.path.join(REPO, "options", "Turtle_Deblur_Gopro.yml")


def gopro():
    with open(GOPRO) as f:
        return yaml.safe_load(f)


def handle(opt, sr=False, dtype=0):
    L = _lib.lib()
    h = C.c_void_p()
    _lib.check(L.turtle_create(C.byref(_lib.config_from_arch(resolve(opt), sr, dtype)), C.byref(h)))
    return L, h


def test_exports_match_header():
    hdr = open(os.path.join(REPO, "include", "turtle_hip.h")).read()
    declared = set(re.findall(r"\b(turtle_[a-z_]+)\s*\(", hdr))
    assert declared == set(_lib.EXPORTED)
    L = _lib.lib()
    for s in declared:
        assert hasattr(L, s)


def test_library_is_built_from_this_tree(monkeypatch):
    """the library reports the kernel-source hash it was built from; the binding accepts
    the tree's hash and refuses any other (a stale prebuilt .so) unless explicitly overridden."""
    from turtlevsr_amd.build import source_hash
    L = _lib.lib()
    assert L.turtle_source_hash().decode() == source_hash()
    assert _lib.check_source_hash(L) == source_hash()
    monkeypatch.delenv("TURTLE_ALLOW_STALE_LIB", raising=False)
    with pytest.raises(RuntimeError, match="built from kernel sources"):
        _lib.check_source_hash(L, expected="0123456789abcdef")
    monkeypatch.setenv("TURTLE_ALLOW_STALE_LIB", "1")
    assert _lib.check_source_hash(L, expected="0123456789abcdef") == source_hash()


def test_training_exports_match_header():
    """Every entry point include/turtle_train.h declares is exported by libturtle_hip.so."""
    hdr = open(os.path.join(REPO, "include", "turtle_train.h")).read()
    declared = set(re.findall(r"\b(turtle_train_[a-z0-9_]+)\s*\(", hdr))
    assert len(declared) >= 10
    L = _lib.lib()
    for s in declared:
        assert hasattr(L, s), s


@pytest.mark.parametrize("model,sr", [("Turtle_t1", False), ("TurtleSuper_t1", True)])
def test_state_dict_surface(model, sr):
    L, h = handle(gopro(), sr)
    n = L.turtle_num_weights(h)
    got = []
    for i in range(n):
        nm, nd, sh = C.c_char_p(), C.c_int(), (C.c_int64 * 4)()
        _lib.check(L.turtle_weight_info(h, i, C.byref(nm), C.byref(nd), sh))
        got.append((nm.value.decode(), tuple(sh[:nd.value])))
    assert got == list(key_shapes(model).items())
    L.turtle_destroy(h)


def test_workspace_and_cache_layout():
    L, h = handle(gopro(), False, 1)
    ws = C.c_size_t()
    _lib.check(L.turtle_workspace_size(h, 1, 1080, 1920, C.byref(ws)))
    assert 1e9 < ws.value < 64e9
    kind, ks, vs = (C.c_int * 8)(), (C.c_int64 * 40)(), (C.c_int64 * 40)()
    _lib.check(L.turtle_cache_layout(h, 1, 256, 256, (C.c_int * 8)(*([0] * 8)), kind, ks, vs))
    assert list(kind) == [0, 0, 0, 1, 1, 2, 2, 2]
    assert tuple(ks[15:19]) == (1, 8, 64, 1024)             # latent FHR after frame 0
    assert tuple(ks[25:30]) == (1, 1, 1, 256, 512)          # dec3 SAB k, N = 256 tokens
    assert tuple(vs[35:40]) == (1, 1, 1, 256, 16 * 16 * 64)  # dec1 SAB v
    t_in = (C.c_int * 8)(0, 0, 0, 192, 192, 3, 3, 2)
    _lib.check(L.turtle_cache_layout(h, 2, 256, 256, t_in, kind, ks, vs))
    assert ks[17] == 192 and ks[26] == 3 and ks[36] == 2


def test_errors_are_reported():
    o = gopro()
    o["decoder1_attn_type2"] = "MEST"   # Turtle_Denoise_Davis.yml: undefined in every arch
    with pytest.raises(ValueError):
        resolve(o)
    L, h = handle(gopro())
    rc = L.turtle_load_weights(h)
    assert rc == -2 and b"missing key" in L.turtle_last_error()
    rc = L.turtle_set_weight(h, b"nope.weight", C.c_void_p(1), 1)
    assert rc == -2


def test_t0_variant_layout_and_plugin():
    """The t0 network (option `model: Turtle_arch`, turtle_arch.py): same state_dict as Turtle_t1,
    SAB k caches hold dilated ws*ws*c tokens (turtle_arch.py:480-495); SR is t1 only."""
    o = dict(gopro(), model="Turtle_arch")
    arch = resolve(o)
    assert arch.t0 and not resolve(gopro()).t0
    L, h = handle(o, False, 1)
    kind, ks, vs = (C.c_int * 8)(), (C.c_int64 * 40)(), (C.c_int64 * 40)()
    _lib.check(L.turtle_cache_layout(h, 1, 256, 256, (C.c_int * 8)(*([0] * 8)), kind, ks, vs))
    assert tuple(ks[25:30]) == (1, 1, 1, 256, 4 * 4 * 256)    # dec3 k: D = ws*ws*c
    assert tuple(ks[35:40]) == tuple(vs[35:40]) == (1, 1, 1, 256, 16 * 16 * 64)
    L.turtle_destroy(h)
    cfg = _lib.config_from_arch(arch, True, 0)
    h2 = C.c_void_p()
    assert L.turtle_create(C.byref(cfg), C.byref(h2)) != 0
    from basicsr.models.archs import turtle_arch, turtle_t1_arch
    m0, m1 = turtle_arch.make_model(o), turtle_t1_arch.make_model(o)
    assert m0.arch.t0 and not m1.arch.t0          # the module decides, as in the reference
    assert list(m0.state_dict()) == list(m1.state_dict())


def test_graphed_runner_refuses_cpu_and_foreign_modules():
    """GraphedTurtle is a ROCm-only serving wrapper: no CPU path, TurtleHIP modules only."""
    import torch
    from turtlevsr_amd.graph import GraphedTurtle
    from turtlevsr_amd.model import TurtleHIP
    with open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "options",
                           "Turtle_Deblur_Gopro.yml")) as f:
        opt = yaml.safe_load(f)
    with pytest.raises(RuntimeError):
        GraphedTurtle(TurtleHIP(opt), 1, 64, 64)
    with pytest.raises(TypeError):
        GraphedTurtle(torch.nn.Linear(2, 2), 1, 64, 64)


def test_chm_on_encoder_level_is_refused():
    """A CHM on a level with Scale_patchsize 1 has SAB window 2: the reference's q/k token grid
    ((H+2-2)/2+1) no longer matches the v tokens (H/2) and attn @ v raises (turtle_t1_arch.py:
    573-599). The library refuses it when sizing the workspace (a dry run of the frame driver)."""
    o = dict(gopro(), encoder2_attn_type2="CHM")
    L, h = handle(o, False, 1)
    ws = C.c_size_t()
    rc = L.turtle_workspace_size(h, 1, 64, 64, C.byref(ws))
    assert rc != 0 and b"token grid" in L.turtle_last_error()
    L.turtle_destroy(h)
    L, h = handle(gopro(), False, 1)
    _lib.check(L.turtle_workspace_size(h, 1, 64, 64, C.byref(ws)))
    L.turtle_destroy(h)

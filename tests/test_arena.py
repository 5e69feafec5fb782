"""SAB history arenas of the drop-in module (model.py `_sab_out`), host logic only (CPU tensors
stand in for the device buffers; no library call): interleaved B = 1 streams - the tiled harness
runs one per tile position (basicsr/inference.py:172-246) - each keep their own arena, a stream
starts small and doubles its headroom at each refill up to the byte budget, and
`release_history` drops them (one arena per slot was re-allocated at full budget for
every tile)."""
import torch

from golden_io import load

T = 3                      # frames a slot keeps (tnew once full)
KS = (1, T, 1, 16, 8)      # [B, T, 1, N, d]


def _module():
    from turtlevsr_amd.model import TurtleHIP
    _, meta = load("clip_gopro_64")
    return TurtleHIP(meta["opt"], dtype="bf16")


def _step(m, cache, slot=5):
    """One frame of one stream: the incoming cache (None at frame 0) -> the returned views."""
    tin = 0 if cache is None else cache[0].shape[1]
    tnew = min(tin + 1, T)
    ks = (1, tnew) + KS[2:]
    kin = None if cache is None else cache[0].contiguous()
    vin = None if cache is None else cache[1].contiguous()
    return m._sab_out(slot, ks, ks, tin, kin, vin, torch.bfloat16, torch.device("cpu"))


def test_interleaved_streams_keep_their_own_arena():
    m = _module()
    caches = [None] * 5
    for frame in range(20):
        for s in range(5):
            prev = caches[s]
            caches[s] = _step(m, prev)
            if frame >= 1 and prev is not None and prev[0].shape[1] == T:
                # steady state: the new history starts one frame after the old one in the same
                # storage (no roll copy) unless this frame refilled the arena
                same = caches[s][0].untyped_storage().data_ptr() == prev[0].untyped_storage().data_ptr()
                if same:
                    fb = prev[0][0, 0].numel() * prev[0].element_size()
                    assert caches[s][0].data_ptr() == prev[0].data_ptr() + fb
    streams = m._arenas[5]
    assert len(streams) == 5
    # headroom doubled from 6 (byte budget ample here): refills at frames ~7, ~19 -> 24 frames max
    for a in streams:
        assert a["extra"] <= 24 and a["k"].shape[0] == T + a["extra"]
    # distinct storage per stream
    assert len({a["k"].data_ptr() for a in streams}) == 5


def test_refill_count_is_logarithmic_and_byte_capped():
    m = _module()
    m._ARENA_BYTES = 10 * 2 * (16 * 8) * 2       # ten frames of k + v
    cache, refills = None, 0
    for _ in range(100):
        prev = cache
        cache = _step(m, prev)
        if prev is not None and cache[0].untyped_storage().data_ptr() != prev[0].untyped_storage().data_ptr():
            refills += 1
    a = m._arenas[5][-1]
    assert a["extra"] == 10                        # 6 -> 10 (capped by bytes), never beyond
    assert refills <= 100 // 10 + 2


def test_branch_gets_small_arena_and_release():
    m = _module()
    cache = None
    for _ in range(4):
        cache = _step(m, cache)
    old = cache
    cache = _step(m, cache)
    # re-running from the older (no longer latest) history: a fresh small arena, not a hit
    branch = _step(m, old)
    assert branch[0].untyped_storage().data_ptr() != cache[0].untyped_storage().data_ptr()
    assert m._arenas[5][-1]["extra"] == m._ARENA_EXTRA
    m.release_history()
    assert m._arenas == {}
    # the caller's caches stay valid after the release
    assert cache[0].shape == (1, T, 1, 16, 8)


def test_lru_bound():
    m = _module()
    m._ARENA_STREAMS = 4
    for _ in range(10):
        _step(m, None)
    assert len(m._arenas[5]) == 4


def test_submodule_parameter_reassignment_changes_signature():
    """a Parameter assigned on a SUBmodule (not the top-level module) must invalidate
    the cached parameter list, so the next inference forward repacks the weights."""
    import torch.nn as nn
    m = _module()
    s0 = m._signature()
    assert m._signature() == s0                      # steady state: no change, cached list reused
    blk = m.encoder_level1.transformer_blocks[0]
    blk.norm1.body.weight = nn.Parameter(blk.norm1.body.weight.detach().clone())
    s1 = m._signature()
    assert s1 != s0
    assert any(p is blk.norm1.body.weight for p in m._plist)
    assert m._signature() == s1


def test_more_streams_than_default_after_reserve():
    """with more interleaved streams than arenas kept per slot (the harness at > 64 tiles),
    every call missed its arena; `reserve_history_streams` (called by the tiled harness with its tile
    count) keeps one per stream, so the second pass over 70 streams re-uses every arena."""
    m = _module()
    n = m._ARENA_STREAMS + 6
    m.reserve_history_streams(n)
    caches = [_step(m, None) for _ in range(n)]
    ptrs = [c[0].untyped_storage().data_ptr() for c in caches]
    caches = [_step(m, c) for c in caches]
    assert len(m._arenas[5]) == n
    assert [c[0].untyped_storage().data_ptr() for c in caches] == ptrs     # no stream re-allocated


def test_unrelated_registration_keeps_signature():
    """building another module (a loss, a second model) bumps the global registration epoch;
    the drop-in module's signature must not change (no repack of unchanged weights)."""
    import torch.nn as nn
    m = _module()
    s0 = m._signature()
    nn.Linear(3, 3)                                  # registers parameters on an unrelated module
    assert m._signature() == s0

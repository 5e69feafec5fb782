"""Turtle_t1 / TurtleSuper_t1 as drop-in ``nn.Module``s backed by libturtle_hip.so.

Interface of the reference plug-in (basicsr/models/archs/turtle_t1_arch.py):

* ``make_model(opt)`` reads the same option keys (10-53) and returns the module;
* ``state_dict()`` has the same 633 keys / shapes (module paths of 932-1043), so reference
  checkpoints load with ``strict=True``;
* ``forward(inp_img_[B,2,C,H,W], k_cached=None, v_cached=None) -> (out[B,C,H,W], k_list[8],
  v_list[8])`` (1045-1132): frame 0 passes None, later frames pass the previous return value.
  The returned caches are ordinary torch tensors with the reference's shapes; entries are None
  where the reference returns None.

Two execution modes, one parameter tree:

* inference (``eval()`` mode, or autograd off, or no parameter requiring grad): the forward runs
  on the HIP library; there is no PyTorch / CPU fallback: a module on a non-ROCm device or a
  missing library raises ``RuntimeError``;
* training (``train()`` mode - nn.Module's default, set by VideoRestorationModel.__init__ :42 -
  with autograd recording and a parameter requiring grad): the forward is the differentiable graph
  of ``train.TrainGraph`` over the same parameters (HIP kernels forward and backward, caches not
  detached), so the reference's ``optimize_parameters`` loop (video_restoration_model.py:78-107:
  fp16 autocast, BPTT over the clip, ``0 * sum(p)``, GradScaler, AdamW) trains this module.
  Validation (``eval()`` + ``no_grad``, :110-113) and inference.py (``eval()``, :253) take the HIP
  inference path.

Compute dtype: ``fp32`` (default, reference parity) or ``bf16`` (MFMA bf16, fp32 accumulation),
chosen by ``opt['hip_dtype']`` or ``set_compute_dtype``. Cache tensors are returned in the
compute dtype. The latent FrameHistoryRouter caches are strided views ([B, heads, rows, P] with
strides (P*heads*rows, rows, 1, heads*rows)); incoming caches of any layout are accepted.
"""
from __future__ import annotations

import ctypes as C
import math
import operator
from typing import List, Optional

import torch
import torch.nn as nn
from torch.nn.modules import module as _mod

from . import _lib
from .arch import resolve
from .params import TurtleParams
from .train import TrainGraph

_VERSION = operator.attrgetter("_version")

# bumped by every parameter / submodule registration on any nn.Module (global torch hooks): the
# drop-in module's cached parameter list is stale after one
_REG_EPOCH = [0]


def _bump_epoch(*_):
    _REG_EPOCH[0] += 1


_mod.register_module_parameter_registration_hook(_bump_epoch)
_mod.register_module_module_registration_hook(_bump_epoch)

_DT = {"fp32": (_lib.DTYPE_F32, torch.float32), "bf16": (_lib.DTYPE_BF16, torch.bfloat16)}


class _Handle:
    def __init__(self, cfg):
        L = _lib.lib()
        h = C.c_void_p()
        _lib.check(L.turtle_create(C.byref(cfg), C.byref(h)))
        self.h = h

    def __del__(self):
        try:
            if self.h:
                _lib.lib().turtle_destroy(self.h)
        except Exception:
            pass


class TurtleHIP(TrainGraph, TurtleParams):
    """Turtle_t1 (``sr=False``) / TurtleSuper_t1 (``sr=True``) / t0 Turtle (``t0=True``) on MI355X."""

    def __init__(self, opt: dict, sr: bool = False, dtype: str = "fp32", t0: Optional[bool] = None):
        arch = resolve(opt)
        if t0 is not None:          # the plug-in module decides (turtle_arch vs turtle_t1_arch)
            arch.t0 = bool(t0)
        if arch.t0 and sr:
            raise ValueError("the super-resolution network is t1 only (turtlesuper_t1_arch.py)")
        super().__init__(arch)
        self.sr = sr
        self.padder_size = 32
        self._dtype_name = dtype
        self._handle = None
        self._handle_dev = None
        self._sig = None
        self._ws = None
        self.set_compute_dtype(dtype)

    # ---------------------------------------------------------------------------------------
    def set_compute_dtype(self, dtype: str):
        if dtype not in _DT:
            raise ValueError(f"hip dtype must be one of {list(_DT)}")
        self._dtype_name = dtype
        self._handle = None
        self._sig = None
        return self

    @property
    def compute_dtype(self) -> torch.dtype:
        return _DT[self._dtype_name][1]

    def _signature(self):
        # parameter list cached (Parameter objects survive .to() and in-place loads); rebuilt after
        # load_state_dict (assign=True swaps the objects), refresh_weights, and whenever any module
        # anywhere registered a parameter or submodule since (_REG_EPOCH: a Parameter or module
        # assigned on a SUBmodule, e.g. blk.attn.temperature = nn.Parameter(...), counts too); the
        # version sum catches in-place updates, the leading data pointers catch device moves and
        # `.data` rebinding
        # a registration ANYWHERE bumps the epoch: the list is rebuilt then (cheap), but the signature
        # carries the identities of this module's parameter objects, not the epoch, so a loss or a
        # second model built next to this one does not trigger a repack
        ps = self.__dict__.get("_plist")
        if ps is None or self.__dict__.get("_plist_epoch") != _REG_EPOCH[0]:
            self.__dict__["_plist_epoch"] = _REG_EPOCH[0]
            ps = self.__dict__["_plist"] = list(self.parameters())
            self.__dict__["_plist_ids"] = hash(tuple(map(id, ps)))
        return (ps[0].device, self._dtype_name, self.__dict__["_plist_ids"], sum(map(_VERSION, ps)),
                tuple(p.data_ptr() for p in ps[:4]))

    def refresh_weights(self):
        """Pack the current parameters into the device layout (done automatically on change)."""
        L = _lib.lib()
        self.__dict__.pop("_plist", None)
        dev = next(self.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("TurtleHIP runs on a ROCm device only: call .to('cuda') first")
        if self._handle is None or self._handle_dev != dev:
            # a handle's lazily created device state (vendor GEMM workspace, events) lives on the
            # device it was first used on: a module moved to another device gets a fresh handle
            with torch.cuda.device(dev):
                self._handle = _Handle(_lib.config_from_arch(self.arch, self.sr, _DT[self._dtype_name][0]))
            self._handle_dev = dev
            self._ws = None
            self.__dict__["_layouts"] = {}
            self.__dict__["_arenas"] = {}
        h = self._handle.h
        with torch.cuda.device(dev):
            # one device->host transfer of all parameters (a per-tensor .cpu() is ~630 small copies)
            sd = [(name, t.detach()) for name, t in self.state_dict().items()]
            flat = torch.cat([t.reshape(-1).float() for _, t in sd]).cpu() if sd else torch.empty(0)
            off = 0
            for name, t in sd:
                n = t.numel()
                a = flat[off:off + n]
                off += n
                _lib.check(L.turtle_set_weight(h, name.encode(), C.c_void_p(a.data_ptr()), n))
            _lib.check(L.turtle_load_weights(h))
        self._sig = self._signature()

    def _load_from_state_dict(self, *args, **kw):
        super()._load_from_state_dict(*args, **kw)
        self._sig = None
        self.__dict__.pop("_plist", None)

    # ---------------------------------------------------------------------------------------
    def cache_layout(self, B: int, H: int, W: int, t_in: List[int]):
        key = (B, H, W, tuple(t_in))
        memo = self.__dict__.setdefault("_layouts", {})   # reset with the handle (refresh_weights)
        res = memo.get(key)
        if res is None:
            res = self._cache_layout(B, H, W, t_in)
            if len(memo) > 64:
                memo.clear()
            memo[key] = res
        return res

    def _cache_layout(self, B: int, H: int, W: int, t_in: List[int]):
        L = _lib.lib()
        kind = (C.c_int * 8)()
        ks = (C.c_int64 * 40)()
        vs = (C.c_int64 * 40)()
        _lib.check(L.turtle_cache_layout(self._handle.h, B, H, W, (C.c_int * 8)(*t_in), kind, ks, vs))
        return list(kind), [tuple(ks[5 * i:5 * i + 5]) for i in range(8)], [tuple(vs[5 * i:5 * i + 5]) for i in range(8)]

    @staticmethod
    def _fhr_strides(shape4):
        B, heads, rows, P = shape4
        return (P * heads * rows, rows, 1, heads * rows)

    def _workspace(self, B, H, W, dev):
        key = (B, H, W, dev, self._dtype_name)
        if self._ws is None or self._ws[0] != key:
            n = C.c_size_t()
            _lib.check(_lib.lib().turtle_workspace_size(self._handle.h, B, H, W, C.byref(n)))
            self._ws = (key, torch.empty(int(n.value), dtype=torch.uint8, device=dev))
        return self._ws[1]

    def _differentiable(self) -> bool:
        """Training mode with autograd recording and some parameter requiring grad."""
        return self.training and torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())

    def forward(self, inp_img_: torch.Tensor, k_cached: Optional[list] = None, v_cached: Optional[list] = None):
        if inp_img_.dim() != 5 or inp_img_.shape[1] != 2:
            raise ValueError("expected inp_img_ of shape [B, 2, C, H, W]")
        if self._differentiable():
            if inp_img_.device.type != "cuda" and self.graph_ops is None:
                raise RuntimeError("TurtleHIP trains on a ROCm device only (the HIP training kernels have no CPU path)")
            return self.graph_forward(inp_img_, k_cached, v_cached)
        if inp_img_.device.type != "cuda":
            raise RuntimeError("TurtleHIP.forward needs ROCm device tensors (no CPU path)")
        if self._sig is None or self._sig != self._signature():
            self.refresh_weights()
        B, _, Cc, H, W = inp_img_.shape
        dev = inp_img_.device
        inp = inp_img_.detach().to(torch.float32).contiguous()
        if k_cached is None:
            k_cached, v_cached = [None] * 8, [None] * 8
        kind0, _, _ = self.cache_layout(B, H, W, [0] * 8)
        cdt = self.compute_dtype
        t_in, k_in, v_in = [0] * 8, [None] * 8, [None] * 8
        for i in range(8):
            kc, vc = k_cached[i], v_cached[i]
            if kind0[i] == 0 or kc is None or vc is None:
                continue
            if kind0[i] == 1:            # FHR rows [B, heads, rows, P]
                t_in[i] = int(kc.shape[2])
                st = self._fhr_strides(tuple(kc.shape))
                k_in[i] = self._as_layout(kc, st, cdt, dev)
                v_in[i] = self._as_layout(vc, st, cdt, dev)
            else:                        # SAB frames [B, T, 1, N, d]
                t_in[i] = int(kc.shape[1])
                k_in[i] = kc.detach().to(device=dev, dtype=cdt).contiguous()
                v_in[i] = vc.detach().to(device=dev, dtype=cdt).contiguous()
        kind, kshape, vshape = self.cache_layout(B, H, W, t_in)
        self._check_caches(kind, kshape, vshape, t_in, k_cached, v_cached)
        k_out, v_out = [None] * 8, [None] * 8
        for i in range(8):
            if kind[i] == 1:
                s4 = kshape[i][:4]
                k_out[i] = torch.empty_strided(s4, self._fhr_strides(s4), dtype=cdt, device=dev)
                v_out[i] = torch.empty_strided(s4, self._fhr_strides(s4), dtype=cdt, device=dev)
            elif kind[i] == 2:
                k_out[i], v_out[i] = self._sab_out(i, kshape[i], vshape[i], t_in[i], k_in[i], v_in[i], cdt, dev)
        s = 4 if self.sr else 1
        out = torch.empty(B, Cc, H * s, W * s, dtype=torch.float32, device=dev)
        ws = self._workspace(B, H, W, dev)

        def ptrs(lst):
            return (C.c_void_p * 8)(*[C.c_void_p(t.data_ptr()) if t is not None else None for t in lst])

        with torch.cuda.device(dev):
            stream = torch.cuda.current_stream(dev).cuda_stream
            _lib.check(_lib.lib().turtle_forward(
                self._handle.h, C.c_void_p(inp.data_ptr()), B, H, W, C.c_void_p(out.data_ptr()),
                ptrs(k_in), ptrs(v_in), (C.c_int * 8)(*t_in), ptrs(k_out), ptrs(v_out),
                C.c_void_p(ws.data_ptr()), ws.numel(), C.c_void_p(stream)))
        # keep inputs alive until the stream has consumed them (caller-owned caches are freed lazily)
        self._keepalive = (inp, k_in, v_in)
        return out, k_out, v_out

    # SAB history slots (B = 1): the returned k / v are views of a frame arena, laid out so that
    # the new cache's kept frames ARE the incoming cache's last frames - the library then skips the
    # roll copy (turtle.cpp chm: source == destination) and only writes the current frame. Every
    # arena frame is written once and never again (the history stays immutable for callers holding
    # older caches). Arenas are kept per STREAM: each slot holds a short LRU list, and a call's
    # arena is the one whose latest frames its incoming cache is (interleaved B = 1 streams - the
    # tiled harness runs one per tile position - each keep their own). A stream starts with a small
    # arena (tnew + _ARENA_EXTRA frames) and doubles its headroom at each refill, up to the byte
    # budget, so only a long single stream ends up with a large one; an incoming cache that is no
    # arena's latest (a branched or moved history, B > 1) gets a fresh small arena filled by copying.
    _ARENA_EXTRA = 6                  # initial frames of headroom
    _ARENA_MAX_EXTRA = 64
    _ARENA_BYTES = 6 << 30            # per stream and slot, reached only by doubling
    _ARENA_STREAMS = 64               # arenas remembered per slot (least recently used dropped)

    def reserve_history_streams(self, n: int):
        """Keep at least n interleaved B = 1 streams' arenas per slot (the tiled harness calls this with
        its tile count: with more tiles than arenas kept, every call would miss and re-allocate)."""
        self.__dict__["_ARENA_STREAMS"] = max(type(self)._ARENA_STREAMS, int(n) + 1)

    def release_history(self):
        """Drop the SAB history arenas this module keeps for fast cache hand-over (caches the caller
        still holds stay valid: they own their storage)."""
        self.__dict__["_arenas"] = {}

    def _sab_out(self, i, ks, vs, tin, kin, vin, cdt, dev):
        if ks[0] != 1:
            return torch.empty(ks, dtype=cdt, device=dev), torch.empty(vs, dtype=cdt, device=dev)
        streams = self.__dict__.setdefault("_arenas", {}).setdefault(i, [])
        tnew = ks[1]
        first = tin - (tnew - 1)                  # first incoming frame kept in the new cache
        fbytes = (math.prod(ks[2:]) + math.prod(vs[2:])) * torch.empty(0, dtype=cdt).element_size()
        extra = self._ARENA_EXTRA
        if tin > 0:
            for j, a in enumerate(streams):
                if a["k"].dtype != cdt or a["k"].device != dev or tuple(a["k"].shape[1:]) != tuple(ks[2:]) or \
                        tuple(a["v"].shape[1:]) != tuple(vs[2:]):
                    continue
                s0 = a["next"] - tin              # arena index of the incoming cache's frame 0
                if s0 < 0 or kin.data_ptr() != a["k"][s0].data_ptr() or vin.data_ptr() != a["v"][s0].data_ptr():
                    continue
                del streams[j]
                b = s0 + first
                if b + tnew <= a["k"].shape[0]:
                    a["next"] = b + tnew
                    streams.append(a)             # most recently used last
                    return a["k"][b:b + tnew].unsqueeze(0), a["v"][b:b + tnew].unsqueeze(0)
                # this stream outgrew its arena: refill into one with twice the headroom (a refill
                # copies the kept frames; HBM is plentiful, a 1080p level-1 slot is ~0.27 GB a frame)
                cap_bytes = max(self._ARENA_EXTRA, min(self._ARENA_MAX_EXTRA, self._ARENA_BYTES // max(fbytes, 1)))
                extra = min(cap_bytes, 2 * a["extra"])
                break
        cap = tnew + extra
        a = dict(k=torch.empty((cap,) + tuple(ks[2:]), dtype=cdt, device=dev),
                 v=torch.empty((cap,) + tuple(vs[2:]), dtype=cdt, device=dev), next=tnew, extra=extra)
        streams.append(a)
        del streams[:-self._ARENA_STREAMS]
        return a["k"][:tnew].unsqueeze(0), a["v"][:tnew].unsqueeze(0)

    @staticmethod
    def _check_caches(kind, kshape, vshape, t_in, k_cached, v_cached):
        """Every incoming cache must have the layout this frame's size and batch imply, up to its
        temporal extent: the kernels index the caller's buffers with these dimensions (the
        reference fails in torch.cat on a mismatch, turtle_t1_arch.py:272, 581)."""
        for i in range(8):
            kc, vc = k_cached[i], v_cached[i]
            if kind[i] == 0 or (kc is None and vc is None):
                continue
            if kc is None or vc is None:
                raise ValueError(f"cache slot {i}: k and v must both be given or both be None")
            if kind[i] == 1:             # FHR [B, heads, rows, P]: rows = t_in
                want_k = want_v = (kshape[i][0], kshape[i][1], t_in[i], kshape[i][3])
            else:                        # SAB [B, T, 1, N, d]: T = t_in
                want_k = (kshape[i][0], t_in[i], kshape[i][2], kshape[i][3], kshape[i][4])
                want_v = (vshape[i][0], t_in[i], vshape[i][2], vshape[i][3], vshape[i][4])
            if tuple(kc.shape) != want_k or tuple(vc.shape) != want_v:
                raise ValueError(f"cache slot {i}: got k {tuple(kc.shape)} / v {tuple(vc.shape)}, expected "
                                 f"{want_k} / {want_v} for this batch and frame size")

    # ---------------------------------------------------------------------------------------
    def set_option(self, name: str, value: int):
        """Kernel-selection switch (turtle_set_option): 'fuse', 'panel_gemm', 'gemm_lds', 'sab_mfma', 'stem_mfma', 'dw_rows', 'gemm9', .... Same results."""
        if self._handle is None or self._sig is None:
            self.refresh_weights()
        _lib.check(_lib.lib().turtle_set_option(self._handle.h, name.encode(), int(value)))
        # a switch may change which kernels (and workspace buffers) a forward uses: size the workspace
        # again at the next forward (raising sk_max_px after a forward left it too small)
        self._ws = None
        return self

    def profile_begin(self, kernel_class: str = "all", tag: Optional[str] = None):
        """Bracket every launch of `kernel_class` (see _lib.K_CLASSES, or 'all') with HIP events;
        with `tag`, only the launches of that shape (the per-launch dump's tag column)."""
        cls = _lib.K_ALL if kernel_class == "all" else _lib.K_CLASSES.index(kernel_class)
        if self._handle is None or self._sig is None:
            self.refresh_weights()
        L = _lib.lib()
        _lib.check(L.turtle_profile_filter(self._handle.h, tag.encode() if tag else None))
        _lib.check(L.turtle_profile_begin(self._handle.h, cls))

    def profile_end(self) -> dict:
        """Per class: summed kernel ms, launches, algorithmic bytes and FLOPs."""
        out = (C.c_double * (4 * len(_lib.K_CLASSES)))()
        _lib.check(_lib.lib().turtle_profile_end(self._handle.h, out))
        return {k: dict(ms=out[4 * i], launches=int(out[4 * i + 1]), bytes=out[4 * i + 2], flops=out[4 * i + 3])
                for i, k in enumerate(_lib.K_CLASSES)}

    @staticmethod
    def _as_layout(t: torch.Tensor, strides, dtype, dev):
        t = t.detach().to(device=dev, dtype=dtype)
        if t.stride() == tuple(strides):
            return t
        o = torch.empty_strided(tuple(t.shape), strides, dtype=dtype, device=dev)
        o.copy_(t)
        return o


def make_model(opt: dict, sr: bool = False) -> TurtleHIP:
    """make_model(opt) of turtle_t1_arch.py:10-53 (``sr=True``: turtlesuper_t1_arch.py)."""
    return TurtleHIP(opt, sr=sr, dtype=opt.get("hip_dtype", "fp32"))

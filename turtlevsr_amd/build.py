"""Build libturtle_hip.so for gfx950 in-tree (hipcc, no JIT cache, no torch extension).

    python -m turtlevsr_amd.build [--force]

Objects go to ``turtlevsr_amd/build/``, the library to ``turtlevsr_amd/lib/libturtle_hip.so``
(git-ignored; it travels to the GPU box with the gpurun snapshot).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(PKG, "build")
LIB = os.path.join(PKG, "lib", "libturtle_hip.so")
SOURCES = ["gemm.hip", "gemm2.hip", "gemm3.hip", "gemm5.hip", "spatial.hip", "attn.hip", "sab.hip", "fused.hip", "fused2.hip", "dwgemm.hip", "tilepd.hip", "gemm8.hip", "gemm9.hip", "gemm_f32.hip", "gemm_sk.hip", "ffn.hip", "t0.hip", "train_ops.hip", "turtle.cpp"]
ARCH = os.environ.get("TURTLE_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm 7.x required)")


def _flags():
    return ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
            "-I", CSRC, "-I", os.path.join(REPO, "include")]


def _compile(src: str, force: bool) -> str:
    obj = os.path.join(OBJ, src + ".o")
    path = os.path.join(CSRC, src)
    deps = [path] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    deps.append(os.path.join(REPO, "include", "turtle_hip.h"))
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(d) for d in deps):
        return obj
    cmd = [hipcc()] + _flags() + ["-x", "hip", "-c", path, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-8000:]}")
    return obj


def build(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), SOURCES))
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-8000:]}")
    if verbose:
        print("built", LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)


def source_hash() -> str:
    """Hash of the HIP kernel sources + this build script: ties committed PMC counters
    (profiles/pmc_traffic.json) to the kernels they were measured on."""
    import hashlib
    hs = hashlib.sha256()
    for rel in sorted(os.listdir(CSRC)) + ["../build.py"]:
        path = os.path.join(CSRC, rel)
        if os.path.isfile(path):
            hs.update(rel.encode())
            with open(path, "rb") as f:
                hs.update(f.read())
    return hs.hexdigest()[:16]

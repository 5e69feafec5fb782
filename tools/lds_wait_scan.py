"""Scan the gfx950 code objects of the built library for an MFMA that reads a register an inline-asm
LDS read (ds_read_b64_tr_b16 / ds_read*) is still filling: a use with no `s_waitcnt lgkmcnt` between
the read and the use. The compiler does not see the asm reads as LDS loads, so it does not insert
that wait itself. Compiles each kernel source to gfx950 assembly with the library's flags.
    python tools/lds_wait_scan.py [source.hip ...]   (default: every turtlevsr_amd/csrc/*.hip)"""
import glob
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from turtlevsr_amd import build  # noqa: E402


def regs(spec):
    m = re.match(r"v\[(\d+):(\d+)\]", spec)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", spec)
    return {int(m.group(1))} if m else set()


def scan(asm_lines):
    """Per kernel, a forward dataflow over the basic blocks: the registers of LDS reads still in flight
    at each label are the union over every edge into it (fall-through and s_branch / s_cbranch_*,
    back-edges included: iterated to a fixpoint), so a use after a join or at a loop header is
    judged on every path into it, and code after an unconditional branch inherits nothing."""
    kernels, cur = [], None
    for ln in asm_lines:
        if re.match(r"^[A-Za-z_.$][\w.$]*:", ln) and not ln.startswith("."):
            cur = (ln.split(":")[0], [])
            kernels.append(cur)
            continue
        if cur is not None:
            cur[1].append(ln)
    bad = []
    for kernel, body in kernels:
        entry = {}                   # label -> registers in flight on some edge into it
        for _ in range(8):
            changed, found = False, []
            pending, live = set(), True
            for ln in body:
                t = ln.split("//")[0].split(";")[0].strip()
                m = re.match(r"^(\.LBB\w+):", t)
                if m:
                    pending = (pending if live else set()) | entry.get(m.group(1), set())
                    live = True
                    continue
                parts = t.split(None, 1)
                if not parts or not live:
                    continue
                op = parts[0]
                ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
                if op == "s_waitcnt" and "lgkmcnt" in t:
                    pending = set()          # conservative: any lgkm wait is taken to cover the reads
                elif op.startswith("ds_read") and ops:
                    pending = pending | regs(ops[0])
                elif op.startswith("v_mfma") and len(ops) >= 3:
                    used = regs(ops[1]) | regs(ops[2])
                    if used & pending:
                        found.append((kernel, t))
                elif op.startswith("s_cbranch") or op == "s_branch":
                    tgt = ops[0] if ops else ""
                    if pending - entry.get(tgt, set()):
                        entry[tgt] = entry.get(tgt, set()) | pending
                        changed = True
                    if op == "s_branch":
                        live = False
                elif op == "s_endpgm":
                    live = False
            if not changed:
                break
        bad += found
    return bad


def asm_of(src):
    from concurrent.futures import ThreadPoolExecutor  # noqa: F401
    out = "/tmp/_lds_scan_" + os.path.basename(src) + ".s"
    cmd = [build.hipcc()] + [f for f in build._flags() if f != "-fPIC"] + ["--cuda-device-only", "-S", "-x", "hip", src, "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(r.stderr[-2000:])
    return open(out).read().splitlines()


def main():
    from concurrent.futures import ThreadPoolExecutor
    srcs = sys.argv[1:] or sorted(glob.glob(os.path.join(REPO, "turtlevsr_amd", "csrc", "*.hip")))
    with ThreadPoolExecutor(max_workers=8) as ex:
        asms = list(ex.map(asm_of, srcs))
    total = 0
    for src, lines in zip(srcs, asms):
        bad = scan(lines)
        total += len(bad)
        for k, t in bad[:5]:
            print(f"{os.path.basename(src)}: {k[:60]} {t}")
    print(f"{len(srcs)} sources, {total} MFMA reads of registers with an LDS read in flight")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())

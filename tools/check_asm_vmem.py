"""Static check of the counted-vmcnt discipline of inline-asm vector-memory loads.

    python tools/check_asm_vmem.py                    every turtlevsr_amd/csrc/*.hip (gfx950 assembly)
    python tools/check_asm_vmem.py src.hip [...]      these sources
    python tools/check_asm_vmem.py --asm file.s [sub] an existing listing (kernels whose name has `sub`)

Several kernels (tilepd, gemm8, gemm_pn, gemm_kt, dwgemm ...) issue `global_load*` /
`global_load_lds*` from inline asm and wait for them with hand-counted `s_waitcnt vmcnt(N)`: the
compiler does not know those registers are still being filled, so it may read or copy them (a
register copy at a loop entry did exactly that in round 4's `sab_avt` bring-up: DESIGN.md §3.9).

For every kernel that contains an inline-asm VMEM load, the check builds the control-flow graph of
its listing (labels, `s_branch`, `s_cbranch_*`, fall-through) and runs a forward data-flow analysis
to a fixed point: the state at a program point is the queue of vector-memory operations in flight,
oldest first (every load, store and LDS-DMA counts; only the destination registers of inline-asm
loads are tracked, the compiler waits for its own); `s_waitcnt vmcnt(N)` keeps the newest N (the
hardware retires in issue order); at a join the queues are aligned at their newest end and merged
position by position (a register is in flight if it is on ANY path). Every instruction that reads or
writes a register still awaiting an asm load is reported - including uses reached only through a
loop back-edge or a branch, which a text-order scan misses.
Exit status 1 if anything is reported."""
import glob
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
BRANCH = re.compile(r"^s_(c?branch\w*)\s+(\S+)")
MAXQ = 64                      # the vmcnt counter is 6 bits: a longer queue cannot be in flight


def regs(text):
    out = set()
    for m in VREG.finditer(text):
        if m.group(1):
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def _instrs(body):
    """(line no, instruction text, inside inline asm) of a function body; labels kept as 'L:'."""
    out, in_asm = [], False
    for ln, raw in body:
        if ";;#ASMSTART" in raw:
            in_asm = True
            continue
        if ";;#ASMEND" in raw:
            in_asm = False
            continue
        t = raw.split(";")[0].split("//")[0].strip()
        if not t:
            continue
        if t.endswith(":"):
            if t.startswith(".L"):
                out.append((ln, t, None))
            continue
        if t.startswith("."):
            continue
        out.append((ln, t, in_asm))
    return out


def _blocks(ins, cfg=True):
    """Basic blocks: [label, [(ln, text, in_asm)], successors]; cfg=False: text order only (each
    block falls through to the next, branches ignored - the pre-round-5 scan, for comparison)."""
    blocks, cur = [], [None, [], None]
    for ln, t, a in ins:
        if a is None:                            # label: a new block
            if cur[1] or cur[0] is not None:
                blocks.append(cur)
            cur = [t[:-1], [], None]
            continue
        cur[1].append((ln, t, a))
        op = t.split()[0]
        if op.startswith("s_branch") or op.startswith("s_cbranch") or op == "s_endpgm" or op.startswith("s_setpc"):
            blocks.append(cur)
            cur = [None, [], None]
    if cur[1] or cur[0] is not None:
        blocks.append(cur)
    index = {b[0]: i for i, b in enumerate(blocks) if b[0] is not None}
    for i, b in enumerate(blocks):
        succ = []
        last = b[1][-1][1] if b[1] else ""
        op = last.split()[0] if last else ""
        m = BRANCH.match(last)
        if op == "s_endpgm" or op.startswith("s_setpc"):
            pass
        elif m and m.group(1) == "branch":
            succ.append(index.get(m.group(2)))
        else:
            if m:
                succ.append(index.get(m.group(2)))
            if i + 1 < len(blocks):
                succ.append(i + 1)
        if not cfg:
            succ = [i + 1] if i + 1 < len(blocks) else []
        b[2] = [s for s in succ if s is not None]
    return blocks


def _join(a, b):
    if a is None:
        return b
    n = max(len(a), len(b))
    out = []
    for k in range(n, 0, -1):
        x = a[-k] if k <= len(a) else frozenset()
        y = b[-k] if k <= len(b) else frozenset()
        out.append(x | y)
    return tuple(out)


def _step(state, t, in_asm, report):
    """Transfer of one instruction; calls report(hit regs) on a use of an in-flight asm load."""
    op = t.split()[0]
    m = re.match(r"s_waitcnt\s+.*vmcnt\((\d+)\)", t)
    if m:
        n = int(m.group(1))
        return state[-n:] if n else ()
    busy = set().union(*state) if state else set()
    used = regs(t)
    if op.startswith("global_load_lds") or ((op.startswith("buffer_load") or op.startswith("global_load")) and " lds" in t):
        new = frozenset()
        hit = used & busy
    elif op.startswith(("global_load", "buffer_load", "scratch_load", "flat_load")):
        parts = t.split(None, 1)[1].split(",", 1)
        dst = regs(parts[0])
        new = frozenset(dst) if in_asm else frozenset()
        hit = used & busy
    elif op.startswith(("global_store", "buffer_store", "scratch_store", "flat_store", "global_atomic", "buffer_atomic")):
        new = frozenset()
        hit = used & busy
    else:
        new = None
        hit = used & busy
    if hit:
        report(hit)
    if new is None:
        return state
    s = state + (new,)
    return s[-MAXQ:]


def check_function(name, body, out=print, cfg=True):
    """Data-flow check of one kernel; returns the number of hazardous instructions."""
    ins = _instrs(body)
    if not any(a and t.split()[0].startswith(("global_load", "buffer_load")) for _, t, a in ins):
        return 0
    blocks = _blocks(ins, cfg)
    if not blocks:
        return 0
    state_in = [None] * len(blocks)
    state_in[0] = ()
    work = [0]
    while work:
        i = work.pop()
        s = state_in[i]
        for _, t, a in blocks[i][1]:
            s = _step(s, t, a, lambda h: None)
        for j in blocks[i][2]:
            ns = _join(state_in[j], s)
            if ns != state_in[j]:
                state_in[j] = ns
                work.append(j)
    bad = {}
    for i, b in enumerate(blocks):
        s = state_in[i]
        if s is None:
            continue
        for ln, t, a in b[1]:
            s = _step(s, t, a, lambda h, ln=ln, t=t: bad.setdefault(ln, (sorted(h), t)))
    for ln in sorted(bad)[:20]:
        h, t = bad[ln]
        out(f"{name}: line {ln}: touches v{h} while an inline-asm load into it is in flight: {t}")
    return len(bad)


def functions(lines, sub=""):
    """(name, [(line no, text)]) of every function in a device listing whose name contains `sub`."""
    i = 0
    while i < len(lines):
        head = lines[i].split(";")[0].rstrip()
        if head.endswith(":") and not head.startswith((".", "\t", " ")) and sub in head:
            name, body, j = head[:-1], [], i + 1
            while j < len(lines) and not lines[j].startswith(".Lfunc_end"):
                body.append((j + 1, lines[j]))
                j += 1
            yield name, body
            i = j
        i += 1


def scan_lines(lines, sub="", out=print, cfg=True):
    total = nk = 0
    for name, body in functions(lines, sub):
        n = check_function(name, body, out, cfg)
        total += n
        nk += 1
    return total, nk


def asm_of(src):
    sys.path.insert(0, REPO)
    from turtlevsr_amd import build
    dst = "/tmp/_vmem_scan_" + os.path.basename(src) + ".s"
    cmd = [build.hipcc()] + [f for f in build._flags() if f != "-fPIC"] + ["--cuda-device-only", "-S", "-x", "hip", src, "-o", dst]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(r.stderr[-2000:])
    return open(dst).read().splitlines()


def main(argv):
    if argv and argv[0] == "--asm":
        lines = open(argv[1]).read().splitlines()
        total, nk = scan_lines(lines, argv[2] if len(argv) > 2 else "")
        print(f"{nk} functions, {total} hazards")
        return 1 if total else 0
    from concurrent.futures import ThreadPoolExecutor
    srcs = argv or sorted(glob.glob(os.path.join(REPO, "turtlevsr_amd", "csrc", "*.hip")))
    with ThreadPoolExecutor(max_workers=8) as ex:
        asms = list(ex.map(asm_of, srcs))
    total = 0
    for src, lines in zip(srcs, asms):
        n, nk = scan_lines(lines, "", lambda s, b=os.path.basename(src): print(f"{b}: {s}"))
        total += n
    print(f"{len(srcs)} sources, {total} uses of registers with an inline-asm load in flight")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))

"""Static check of the counted-vmcnt discipline in hand-scheduled kernels (gemm3.hip).

    python tools/check_asm_vmem.py <device .s file> [kernel-name-substring]

Walks each matching kernel's instruction stream in text order, keeping the queue of vector-memory
operations in flight (loads with their destination registers, stores, LDS-DMA); an
`s_waitcnt vmcnt(N)` retires the oldest until N remain (the hardware retires in issue order).
Reports every instruction that reads or writes a VGPR still awaiting a load. Text order ignores
branches, so a report is a lead to read in the listing, not proof; a clean run on straight-line
tiles is the property the kernel relies on."""
import re
import sys

VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in VREG.finditer(text):
        if m.group(1):
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def check(lines, name):
    q = []            # (kind, dest regs): every VMEM op counts; only asm loads are tracked for
    bad = 0           # register use (the compiler waits for its own loads itself)
    in_asm = False
    for ln, raw in lines:
        if ";;#ASMSTART" in raw:
            in_asm = True
            continue
        if ";;#ASMEND" in raw:
            in_asm = False
            continue
        t = raw.split(";")[0].strip()
        if not t or t.endswith(":") or t.startswith("."):
            continue
        op = t.split()[0]
        m = re.match(r"s_waitcnt\s+.*vmcnt\((\d+)\)", t)
        if m:
            n = int(m.group(1))
            while len(q) > n:
                q.pop(0)
            continue
        if op == "s_endpgm":
            break
        busy = set()
        for _, d in q:
            busy |= d
        used = regs(t)
        if op.startswith("global_load_lds") or op.startswith("buffer_load") and " lds" in t:
            q.append(("dma", set()))
            hit = used & busy
        elif op.startswith("global_load") or op.startswith("buffer_load") or op.startswith("scratch_load"):
            dst, rest = t.split(None, 1)[1].split(",", 1)
            q.append(("load", regs(dst) if in_asm else set()))
            hit = (regs(dst) | regs(rest)) & busy
        elif op.startswith("global_store") or op.startswith("buffer_store") or op.startswith("scratch_store"):
            q.append(("store", set()))
            hit = used & busy
        else:
            hit = used & busy
        if hit:
            bad += 1
            if bad <= 20:
                print(f"{name}: line {ln}: touches in-flight v{sorted(hit)}: {t}")
    return bad


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "gemm_pn_kernel"
    lines = open(path).read().split("\n")
    total = 0
    i = 0
    while i < len(lines):
        l = lines[i]
        head = l.split(";")[0].rstrip()
        if head.endswith(":") and sub in head and not head.startswith(".") and not head.startswith("\t"):
            name = head[:-1]
            body = []
            j = i + 1
            while j < len(lines) and "s_endpgm" not in lines[j]:
                body.append((j + 1, lines[j]))
                j += 1
            body.append((j + 1, lines[j] if j < len(lines) else ""))
            n = check(body, name)
            print(f"{name}: {n} hazards")
            total += n
            i = j
        i += 1
    sys.exit(1 if total else 0)


if __name__ == "__main__":
    main()

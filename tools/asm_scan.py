"""Per-kernel summary of a hipcc -S device assembly file: line count, scratch (spill) accesses,
MFMAs, DPP ops, vmcnt(0) waits and the line spans they sit in (quick register / pipeline check).
    python3 tools/asm_scan.py file.s [kernel-substring]"""
import re
import sys

s = open(sys.argv[1]).read()
want = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"\n(_Z\w+):[^\n]*\n(.*?)\.Lfunc_end", s, re.S):
    name, body = m.group(1), m.group(2)
    if want not in name:
        continue
    lines = body.split("\n")
    idx = lambda pat: [j for j, l in enumerate(lines) if re.search(pat, l)]
    sc, mf, dp, w0 = idx(r"scratch_"), idx(r"v_mfma"), idx(r"row_sh"), idx(r"s_waitcnt.*vmcnt\(0\)")
    print(name[:70], "lines", len(lines), "scratch", len(sc), "mfma", len(mf), "dpp", len(dp), "vmcnt0", len(w0))
    if sc:
        print("   scratch at", sc[:6], "...", sc[-6:])
    if mf:
        print("   mfma span", mf[0], mf[-1], " dpp span", (dp[0], dp[-1]) if dp else None, " vmcnt0 at", w0[:12])

"""Per (kernel, grid size) SQ counter report from rocprofv3 --pmc CSVs (tools/bench_pmc.sh,
tools/tp_pmc.sh): medians over dispatches, then per-wave and per-cycle ratios.
    python3 tools/sq_report.py gpurun_out/<tag> [kernel-substring]
Units (MI355X_MICROARCH.md): SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles,
SQ_VALU_MFMA_BUSY_CYCLES counts cycles; SQ_BUSY_CYCLES is per SE."""
import collections
import csv
import glob
import os
import statistics
import sys

d = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else ""
per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if want not in r["Kernel_Name"]:
            continue
        k = (r["Kernel_Name"].replace("void turtle::", "")[:60], int(r["Grid_Size"]), r.get("VGPR_Count"), r.get("LDS_Block_Size"))
        per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(per.items()):
    m = {c: statistics.median(v) for c, v in cs.items()}
    waves = m.get("SQ_WAVES", 0) or 0
    print(f"{k[0]}  grid={k[1]} vgpr={k[2]} lds={k[3]}  dispatches~{max(len(v) for v in cs.values())}")
    line = []
    if waves:
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM"):
            if c in m:
                line.append(f"{c[9:]}/w={m[c] / waves:.0f}")
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_MFMA",
                  "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS", "SQ_WAIT_INST_VMEM"):
            if c in m:
                line.append(f"{c[3:].lower()}={m[c] / wc:.2f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "SQ_BUSY_CYCLES" in m:
        line.append(f"mfma_busy/busy={m['SQ_VALU_MFMA_BUSY_CYCLES'] / max(m['SQ_BUSY_CYCLES'], 1):.2f}")
    if "SQ_LDS_BANK_CONFLICT" in m and "SQ_LDS_IDX_ACTIVE" in m:
        line.append(f"lds_conflict={m['SQ_LDS_BANK_CONFLICT'] / max(m['SQ_LDS_IDX_ACTIVE'], 1):.2f}")
    print("   " + "  ".join(line))

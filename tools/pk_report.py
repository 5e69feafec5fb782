"""Summarise tools/prof_kernel.sh output: per (kernel, grid, LDS) group, counters per wave.

    python tools/pk_report.py gpurun_out/pk_<tag>
"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(__file__))
from pmc_report import grid, short  # noqa: E402


def main():
    d = sys.argv[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        seen = set()
        for r in csv.DictReader(open(f)):
            key = (short(r["Kernel_Name"]).split("<")[0], grid(r), int(r["LDS_Block_Size"]), int(r["VGPR_Count"]))
            acc[key][r["Counter_Name"] + "@" + os.path.basename(os.path.dirname(f))] += float(r["Counter_Value"])
    for key, c in sorted(acc.items(), key=lambda kv: -max(v for k, v in kv[1].items() if k.startswith("SQ_WAVE_CYCLES") or True)):
        print(f"== {key[0]} grid={key[1]} lds={key[2]} vgpr={key[3]}")
        byp = collections.defaultdict(dict)
        for k, v in c.items():
            name, p = k.split("@")
            byp[p][name] = v
        for p in sorted(byp):
            w = byp[p].get("SQ_WAVES", 0) or 1
            items = ", ".join(f"{n}={v / w:.1f}" for n, v in sorted(byp[p].items()) if n != "SQ_WAVES")
            print(f"  [{p}] waves={w:.0f}: per wave {items}")


if __name__ == "__main__":
    main()

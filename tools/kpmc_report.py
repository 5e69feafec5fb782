"""Per-dispatch PMC summary of tools/kbench_pmc.sh output (first dispatch of each kernel+grid).

    python tools/kpmc_report.py gpurun_out/kpmc
Values are per dispatch; FETCH_SIZE is reported in KB by rocprofv3 and doubled here for the gfx950
wide-read undercount (MI355X_MICROARCH.md, HBM section); WRITE_SIZE in KB as is.
"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    per = collections.OrderedDict()
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("void turtle::", "").split("(")[0]
            key = (name, int(r["Grid_Size"]))
            did = int(r["Dispatch_Id"])
            ent = per.setdefault(key, {})
            ent.setdefault(r["Counter_Name"], {})
            ent[r["Counter_Name"]].setdefault(did, 0.0)
            ent[r["Counter_Name"]][did] += float(r["Counter_Value"])
            ent["_ns_%s" % did] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for (name, grid), ent in per.items():
        vals = {}
        for c, dv in ent.items():
            if c.startswith("_"):
                continue
            ks = sorted(dv)
            vals[c] = dv[ks[len(ks) // 2]] if ks else 0
        w = vals.get("SQ_WAVES", 0) or 1
        cyc = vals.get("SQ_WAVE_CYCLES", 0)
        out = [f"{name:34s} grid={grid:9d}"]
        if cyc:
            out.append(f"wait={vals.get('SQ_WAIT_ANY', 0) / cyc:.2f} inst={vals.get('SQ_WAIT_INST_ANY', 0) / cyc:.2f} "
                       f"act={vals.get('SQ_ACTIVE_INST_ANY', 0) / cyc:.2f} mfma={vals.get('SQ_ACTIVE_INST_MFMA', 0) / cyc:.2f} "
                       f"valu={vals.get('SQ_ACTIVE_INST_VALU', 0) / cyc:.2f}")
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                  "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS"):
            if c in vals:
                out.append(f"{c[8:] if c.startswith('SQ_INSTS') else c[3:]}/w={vals[c] / w:.0f}")
        for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CU_CYCLES", "SQ_WAIT_INST_LDS", "SQ_VMEM_WR_TA_DATA_FIFO_FULL",
                  "SQ_VMEM_TA_ADDR_FIFO_FULL", "SQ_INST_LEVEL_VMEM"):
            if c in vals and cyc:
                out.append(f"{c[3:]}/wcyc={vals[c] / cyc:.3f}")
        ns = [v for k, v in ent.items() if k.startswith("_ns_")]
        if ns:
            out.append(f"us={sorted(ns)[len(ns) // 2] / 1e3:.1f}")
        if "FETCH_SIZE" in vals:
            out.append(f"fetchMB={2 * vals['FETCH_SIZE'] / 1024:.1f}")
        if "WRITE_SIZE" in vals:
            out.append(f"writeMB={vals['WRITE_SIZE'] / 1024:.1f}")
        if "TCC_HIT_sum" in vals:
            h, m = vals["TCC_HIT_sum"], vals["TCC_MISS_sum"]
            out.append(f"L2hit={h / max(h + m, 1):.2f}")
        print(" ".join(out))


if __name__ == "__main__":
    main()

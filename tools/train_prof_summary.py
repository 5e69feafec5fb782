"""Summarise a rocprofv3 --stats kernel CSV of the training step by kernel family (in-tree HIP,
ATen, MIOpen, Tensile, other): python tools/train_prof_summary.py <run_kernel_stats.csv> [top]"""
import csv
import sys


def family(n: str) -> str:
    if "turtle" in n:
        return "turtle (in-tree HIP)"
    if "at::native" in n or n.startswith("void at::"):
        return "aten"
    if n.startswith("Cijk") or "Tensile" in n:
        return "tensile"
    if "naive_conv" in n or "Im2d" in n or n.startswith("igemm") or "miopen" in n.lower() or "conv" in n.lower() \
            or n.startswith("batched_transpose") or "TensorOp" in n:
        return "miopen"
    return "other"


rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
agg = {}
for r in rows:
    f = family(r["Name"])
    agg[f] = agg.get(f, 0.0) + float(r["TotalDurationNs"])
print(f"total GPU kernel time {tot / 1e6:.1f} ms")
for k, v in sorted(agg.items(), key=lambda x: -x[1]):
    print(f"  {k:24s} {v / 1e6:9.1f} ms  {100 * v / tot:5.1f} %")
print()
for r in rows[:top]:
    print(f"{float(r['TotalDurationNs']) / 1e6:8.1f} ms {r['Calls']:>6} x {float(r['AverageNs']) / 1e3:8.1f} us  {r['Name'][:110]}")

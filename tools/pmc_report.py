"""Join a tools/prof_round.sh profile: kernel-trace durations with the separate PMC passes.

    python tools/pmc_report.py gpurun_out/prof_<tag> [--top 30]

Launches are grouped by (kernel name, grid size, LDS bytes) -- the same key in every pass since
the bench replays an identical launch sequence. Per group: calls per pass, mean duration (us),
HBM read/write bytes per launch (FETCH_SIZE doubled: gfx950 reports half of a 16-B/lane
coalesced stream, MI355X_MICROARCH.md "HBM"; both counters are in KiB), achieved HBM GB/s, and
the SQ stall split (wait = parked on s_waitcnt/barrier, inst = issue stall, active).
"""
import argparse
import collections
import csv
import os
import re


def short(name):
    # trace files mix mangled and demangled names: key on the base identifier + template ints
    m = re.search(r"(\w+_kernel|sab_\w+|__amd_\w+)", name)
    base = re.sub(r"^_ZN\d+turtle\d+", "", m.group(1)) if m else name[:40]
    ints = re.findall(r"(?:Li|<|, )(\d+)", name)
    return base + ("<" + ",".join(ints) + ">" if ints else "")


def grid(r):
    if "Grid_Size" in r:
        return int(r["Grid_Size"])
    return int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])


def load_counters(path):
    g = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    if not os.path.exists(path):
        return g, n
    seen = set()
    for r in csv.DictReader(open(path)):
        key = (short(r["Kernel_Name"]).split("<")[0], grid(r), int(r["LDS_Block_Size"]))
        g[key][r["Counter_Name"]] += float(r["Counter_Value"])
        d = (key, r["Dispatch_Id"])
        if d not in seen:
            seen.add(d)
            n[key] += 1
    return g, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(a.dir, "trace", "run_kernel_trace.csv"))):
        key = (short(r["Kernel_Name"]).split("<")[0], grid(r), int(r["LDS_Block_Size"]))
        dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    fetch, nf = load_counters(os.path.join(a.dir, "fetch", "run_counter_collection.csv"))
    write, nw = load_counters(os.path.join(a.dir, "write", "run_counter_collection.csv"))
    sq, ns = load_counters(os.path.join(a.dir, "sq", "run_counter_collection.csv"))
    rows = sorted(dur.items(), key=lambda kv: -sum(kv[1]))
    tot = sum(sum(v) for v in dur.values())
    print(f"trace total {tot / 1e3:.2f} ms over {sum(len(v) for v in dur.values())} dispatches")
    print(f"{'ms':>7} {'n':>4} {'us':>8} {'rdMB':>7} {'wrMB':>7} {'GB/s':>6} {'wait%':>5} {'inst%':>5} {'act%':>5}  kernel [grid, lds]")
    for key, ds in rows[: a.top]:
        us = sum(ds) / len(ds)
        rd = 2 * 1024 * fetch[key].get("FETCH_SIZE", 0) / max(nf[key], 1)
        wr = 1024 * write[key].get("WRITE_SIZE", 0) / max(nw[key], 1)
        gbs = (rd + wr) / (us * 1e-6) / 1e9 if us > 0 else 0
        s = sq.get(key, {})
        wc = s.get("SQ_WAVE_CYCLES", 0)
        pct = lambda c: 100 * s.get(c, 0) / wc if wc else 0
        print(f"{sum(ds) / 1e3:7.2f} {len(ds):4d} {us:8.1f} {rd / 1e6:7.1f} {wr / 1e6:7.1f} {gbs:6.0f} "
              f"{pct('SQ_WAIT_ANY'):5.0f} {pct('SQ_WAIT_INST_ANY'):5.0f} {pct('SQ_ACTIVE_INST_ANY'):5.0f}  "
              f"{key[0]} [{key[1]}, {key[2]}]")


if __name__ == "__main__":
    main()

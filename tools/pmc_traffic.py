"""HBM traffic per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/prof_round.sh).

    python tools/pmc_traffic.py gpurun_out/prof_<tag> 'TAG@@KERNEL_REGEX[:GRID]' ... > profiles/pmc_traffic.json

Per (kernel symbol, grid size) group: median FETCH_SIZE x 2 (gfx950 counts a wide 16-B/lane read
at half its bytes: MI355X_MICROARCH.md, HBM section) + WRITE_SIZE, both reported in KB. A launch
tag (the library's per-launch description, bench.py roofline "kernel") is mapped to a group only
where that kernel symbol + grid is unique to the tag's shape; ambiguous shapes stay unprofiled."""
import collections
import csv
import glob
import json
import os
import re
import statistics
import sys


def load(d, counter):
    per = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            per[(r["Kernel_Name"], int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return per


def main():
    d = sys.argv[1]
    fetch, write = load(os.path.join(d, "fetch"), "FETCH_SIZE"), load(os.path.join(d, "write"), "WRITE_SIZE")
    groups = {}
    for key in sorted(set(fetch) | set(write)):
        f = 2 * 1024 * statistics.median(fetch[key]) if fetch.get(key) else None
        w = 1024 * statistics.median(write[key]) if write.get(key) else None
        groups[f"{key[0].split('(')[0]} grid={key[1]}"] = dict(fetch_bytes=f, write_bytes=w, dispatches=len(fetch.get(key, [])),
                                                               hbm_bytes=(f or 0) + (w or 0))
    per_tag = {}
    for spec in sys.argv[2:]:
        tag, rest = spec.split("@@", 1)
        rx, grid = rest.rsplit(":", 1) if re.search(r":\d+$", rest) else (rest, None)
        hits = [k for k in groups if re.search(rx, k) and (grid is None or k.endswith(f"grid={grid}"))]
        if len(hits) == 1:
            g = groups[hits[0]]
            per_tag[tag] = dict(kernel=hits[0], hbm_bytes_per_launch=g["hbm_bytes"], fetch_bytes=g["fetch_bytes"],
                                write_bytes=g["write_bytes"])
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from turtlevsr_amd.build import source_hash
    json.dump(dict(source=d, source_hash=source_hash(), note="FETCH_SIZE doubled (gfx950 wide-read undercount); KB -> bytes",
                   per_tag=per_tag, groups=groups), sys.stdout, indent=1)


if __name__ == "__main__":
    main()

"""Summarise a TURTLE_PROF_DUMP file (one line per profiled launch: class ms bytes flops tag).

    TURTLE_PROF_DUMP=gpurun_out/launches.tsv python bench.py --steps 2 ...
    python tools/launch_report.py gpurun_out/launches.tsv [--steps 2]

Groups launches by tag and prints, sorted by total time: count per step, mean microseconds,
achieved GB/s (algorithmic bytes) and TFLOP/s, and the fraction of the step each group takes.
"""
import argparse
import collections

CLASSES = ["gemm", "dwconv", "chan_attn", "sab_score", "sab_av", "sab_window", "other", "fused"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=1, help="timed steps the dump covers")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    g = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
    total = 0.0
    for line in open(a.path):
        parts = line.rstrip("\n").split("\t")
        if len(parts) < 4:
            continue
        cls, ms, by, fl = int(parts[0]), float(parts[1]), float(parts[2]), float(parts[3])
        tag = parts[4] if len(parts) > 4 and parts[4] else CLASSES[cls]
        r = g[tag]
        r[0] += 1; r[1] += ms; r[2] += by; r[3] += fl
        total += ms
    rows = sorted(g.items(), key=lambda kv: -kv[1][1])
    print(f"total {total / a.steps:.3f} ms/step over {sum(r[0] for r in g.values()) // a.steps} launches/step")
    print(f"{'ms/step':>8} {'%':>5} {'n':>4} {'us/launch':>9} {'GB/s':>7} {'TF/s':>6}  tag")
    for tag, (n, ms, by, fl) in rows[: a.top]:
        s = ms / 1e3
        print(f"{ms / a.steps:8.3f} {100 * ms / total:5.1f} {n // a.steps:4d} {1e3 * ms / n:9.1f} "
              f"{by / s / 1e9:7.0f} {fl / s / 1e12:6.1f}  {tag}")


if __name__ == "__main__":
    main()

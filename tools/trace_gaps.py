#!/usr/bin/env python3
"""Per-kernel in-graph duration and preceding gap from a rocprofv3 --kernel-trace CSV
(decode steps of bench.py): launches grouped by kernel name + grid."""
import collections
import csv
import glob
import os
import statistics
import sys


def main():
    d = sys.argv[1]
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[-1]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))

    def short(r):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("qie::", "")
        return f"{n} g{r.get('Grid_Size_X', r.get('Grid_Size', '?'))}"

    seq = [(short(r), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    # decode window: from a third of the way through the decode-attention launches to the last
    idx = [i for i, x in enumerate(seq) if "attn_decode" in x[0]]
    lo, hi = idx[len(idx) // 3], idx[-1]
    stats = collections.defaultdict(lambda: ([], []))
    for i in range(lo, hi + 1):
        n, s, e = seq[i]
        stats[n][0].append((e - s) / 1e3)
        stats[n][1].append((s - seq[i - 1][2]) / 1e3)
    tot = (seq[hi][2] - seq[lo][1]) / 1e3
    busy = sum(sum(v[0]) for v in stats.values())
    print(f"window {tot:.1f} us, busy {busy:.1f} us, gaps {tot - busy:.1f} us, launches {hi - lo + 1}")
    for n, (du, gp) in sorted(stats.items(), key=lambda kv: -sum(kv[1][0])):
        print(f"{n[:90]:90s} n={len(du):5d} dur med {statistics.median(du):8.2f} mean {statistics.mean(du):8.2f}"
              f"  gap med {statistics.median(gp):6.2f} mean {statistics.mean(gp):6.2f}")


if __name__ == "__main__":
    main()

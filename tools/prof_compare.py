#!/usr/bin/env python3
"""Side-by-side per-kernel durations of two rocprofv3 kernel traces (tools/prof_config2.sh):
calls, median and mean microseconds per kernel name (template arguments kept), and the
difference.  usage: tools/prof_compare.py DIR_A DIR_B [OUT.md]"""
import collections
import csv
import os
import statistics
import sys


def load(d):
    g = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("qie::", "")
        wg = int(r["Workgroup_Size_X"])
        name += f" [g {int(r['Grid_Size_X']) // wg} x {wg}]"
        g[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return g


def main(a, b, out=None):
    A, B = load(a), load(b)
    rows = []
    for k in sorted(set(A) | set(B), key=lambda k: -(sum(A.get(k, [])) + sum(B.get(k, [])))):
        va, vb = A.get(k, []), B.get(k, [])
        ma = statistics.median(va) if va else float("nan")
        mb = statistics.median(vb) if vb else float("nan")
        rows.append(f"| `{k}` | {len(va)} | {ma:.2f} | {len(vb)} | {mb:.2f} | {mb - ma:+.2f} |")
    lines = [f"| kernel | calls A | median us A | calls B | median us B | B - A |", "|---|---|---|---|---|---|"] + rows
    text = "\n".join(lines)
    print(f"A = {a}\nB = {b}\n{text}")
    if out:
        with open(out, "w") as f:
            f.write(f"A = `{a}`, B = `{b}`\n\n{text}\n")


if __name__ == "__main__":
    main(*sys.argv[1:])

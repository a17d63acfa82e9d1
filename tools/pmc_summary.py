#!/usr/bin/env python3
"""Per-launch HBM traffic of the decode kernels from the two rocprofv3 --pmc passes of
tools/pmc_probe.py (gpu_check.sh PMC=1).  FETCH_SIZE / WRITE_SIZE are kilobytes; on gfx950
FETCH_SIZE counts half the bytes of 16-B-per-lane streaming reads (MI355X_MICROARCH.md
'HBM'), so fetch bytes = 2 x FETCH_SIZE x 1024.  Writes profiles/<name>.json."""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(path, counter):
    rows = list(csv.DictReader(open(path)))
    rows = [r for r in rows if r["Counter_Name"] == counter and not r["Kernel_Name"].startswith("__amd_rocclr")]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def main(out_name="r01_pmc_traffic"):
    meta = json.load(open(os.path.join(ROOT, "gpurun_out", "pmc_probe_meta.json")))
    n = meta["order"][0]["launches"]
    total = n * len(meta["order"])
    fetch = per_dispatch(os.path.join(ROOT, "gpurun_out", "pmc_FETCH_SIZE", "pmc_counter_collection.csv"), "FETCH_SIZE")
    write = per_dispatch(os.path.join(ROOT, "gpurun_out", "pmc_WRITE_SIZE", "pmc_counter_collection.csv"), "WRITE_SIZE")
    fetch, write = fetch[-total:], write[-total:]
    res = []
    for i, m in enumerate(meta["order"]):
        wu = m.get("warmup", 1)
        f = fetch[i * n:(i + 1) * n][wu:]   # drop the warm-up launches
        w = write[i * n:(i + 1) * n][wu:]
        names = {r["Kernel_Name"].split("(")[0] for r in f}
        fb = statistics.median(2 * float(r["Counter_Value"]) * 1024 for r in f)
        wb = statistics.median(float(r["Counter_Value"]) * 1024 for r in w)
        res.append({"kernel": m["kernel"], "device_function": sorted(names), "algorithmic_bytes": m["algorithmic_bytes"],
                    "fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb,
                    "traffic_over_algorithmic": (fb + wb) / m["algorithmic_bytes"] if m["algorithmic_bytes"] else None,
                    "avg_us_eager": m["avg_us"]})
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) over tools/pmc_probe.py",
           "correction": "fetch_bytes = 2 x FETCH_SIZE[KB] x 1024 (gfx950 streaming-read tally); write_bytes = WRITE_SIZE[KB] x 1024",
           "launches_per_kernel": n - meta["order"][0].get("warmup", 1), "kernels": res}
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    path = os.path.join(ROOT, "profiles", out_name + ".json")
    with open(path, "w") as fh:
        json.dump(doc, fh, indent=1)
    for r in res:
        print(f"{r['kernel']:8s} alg {r['algorithmic_bytes']/1e6:9.2f} MB  hbm {r['hbm_bytes']/1e6:9.2f} MB "
              f"(fetch {r['fetch_bytes']/1e6:9.2f} write {r['write_bytes']/1e6:7.3f})  ratio {r['traffic_over_algorithmic']:.3f}  {r['device_function']}")


if __name__ == "__main__":
    main(*sys.argv[1:])

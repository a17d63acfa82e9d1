#!/usr/bin/env python3
"""MFMA evidence for the prefill kernels from tools/pmc_mfma.sh's passes.

Per role (QKV / O / gate-up / down GEMM, flash attention) over the last measured prefill:
  * duration (kernel trace, a separate run of the same launch sequence, matched by order),
  * algorithmic flops per launch and their rate against the 2.5 PFLOP/s dense bf16 peak,
  * MFMA busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
    (GRBM_GUI_ACTIVE is summed over the 8 XCDs; the busy counter counts issue cycles of
    every SIMD, 32 per 32x32x16 / 16x16x32 bf16 MFMA: MI355X_MICROARCH.md);
  * flops implied by the busy counter (1024 flops per busy SIMD cycle) over the
    algorithmic flops: > 1 means MFMA work the algorithm does not need (padding, the
    attention's three-part P.V);
  * SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 where listed, and LDS bank conflicts per LDS cycle.
Writes profiles/<name>.json."""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PEAK = 2.5e15


def short(n):
    return n.split("(")[0].replace("void ", "").replace("qie::", "")


def last_prefill(seq):
    """indices of the dispatches of the last prefill (after the last embedding_kernel)"""
    starts = [i for i, n in enumerate(seq) if n.startswith("embedding_kernel")]
    return list(range(starts[-1], len(seq))) if starts else []


def roles(names):
    """GEMM roles from the launch order of a prefill layer (QKV GEMM, qkv_post, attention,
    O GEMM, norm, gate/up GEMM, down GEMM), whatever kernel variant each one runs."""
    out, prev = [], None
    for n in names:
        r = None
        if n.startswith("attn_prefill"):
            r = "attention"
        elif n.startswith("gemm_big_kernel<2") or n.startswith("gemm8_kernel<2"):
            r = "gate_up"
        elif n.startswith("gemm_kernel") or n.startswith("gemm_big_kernel") or n.startswith("gemm8_kernel"):
            r = {"attention": "o", "gate_up": "down"}.get(prev, "qkv")
        out.append(r)
        if r:
            prev = r
    return out


def counters(d):
    path = os.path.join(OUT, d, "pmc_counter_collection.csv")
    if not os.path.exists(path):
        return None
    per = {}
    for r in csv.DictReader(open(path)):
        if r["Kernel_Name"].startswith("__amd_rocclr"):
            continue
        k = int(r["Dispatch_Id"])
        e = per.setdefault(k, {"name": short(r["Kernel_Name"])})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    seq = [per[k] for k in sorted(per)]
    idx = last_prefill([e["name"] for e in seq])
    return [seq[i] for i in idx]


def main(name="r02_pmc_mfma"):
    meta = json.load(open(os.path.join(OUT, "pmc_mfma_meta.json")))
    P = meta["prompt"]
    H, nq, nkv, hd, I = 3584, 28, 4, 128, 18944
    flops = {"qkv": 2.0 * P * (nq + 2 * nkv) * hd * H, "o": 2.0 * P * H * nq * hd,
             "gate_up": 2.0 * P * 2 * I * H, "down": 2.0 * P * I * H,
             "attention": 4.0 * nq * hd * P * (P + 1) / 2}
    tr = list(csv.DictReader(open(os.path.join(OUT, "pmc_mfma_trace", "tr_kernel_trace.csv"))))
    tr = [r for r in tr if not r["Kernel_Name"].startswith("__amd_rocclr")]
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    tnames = [short(r["Kernel_Name"]) for r in tr]
    tidx = last_prefill(tnames)
    trace = [(tnames[i], (int(tr[i]["End_Timestamp"]) - int(tr[i]["Start_Timestamp"])) * 1e-9) for i in tidx]
    passes = {d: counters(d) for d in ("pmc_mfma_busy", "pmc_mfma_mops", "pmc_mfma_lds")}
    troles = roles([n for n, _ in trace])
    res = {}
    for role in ("qkv", "attention", "o", "gate_up", "down"):
        ti = [i for i, r in enumerate(troles) if r == role]
        if not ti:
            continue
        dur = statistics.mean(trace[i][1] for i in ti)
        e = {"kernel": sorted({trace[i][0] for i in ti}), "launches": len(ti), "avg_us": round(dur * 1e6, 2),
             "algorithmic_flops": flops[role], "tflops": round(flops[role] / dur / 1e12, 1),
             "frac_of_bf16_peak": round(flops[role] / dur / PEAK, 4)}
        for d, seq in passes.items():
            if not seq:
                continue
            pr = roles([x["name"] for x in seq])
            rows = [seq[i] for i, r in enumerate(pr) if r == role]
            if len(rows) != len(ti):
                e[d + "_note"] = f"{len(rows)} counter dispatches vs {len(ti)} traced"
                if not rows:
                    continue
            avg = {c: statistics.mean(x[c] for x in rows) for c in rows[0] if c != "name"}
            if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
                cyc = avg["GRBM_GUI_ACTIVE"] / 8.0
                e["mfma_busy_frac"] = round(avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024), 4)
                e["clock_ghz"] = round(cyc / dur / 1e9, 3)
                e["busy_implied_over_algorithmic_flops"] = round(avg["SQ_VALU_MFMA_BUSY_CYCLES"] * 1024 / flops[role], 3)
            if "SQ_INSTS_VALU_MFMA_MOPS_BF16" in avg:
                e["mops_bf16_x512_over_algorithmic"] = round(avg["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512 / flops[role], 3)
                e["mfma_bf16_insts"] = avg.get("SQ_INSTS_VALU_MFMA_BF16")
            if "SQ_LDS_BANK_CONFLICT" in avg and avg.get("SQ_LDS_IDX_ACTIVE"):
                e["lds_bank_conflict_per_active"] = round(avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_LDS_IDX_ACTIVE"], 4)
        res[role] = e
    doc = {"source": "rocprofv3 --pmc passes over tools/pmc_mfma_probe.py (Qwen2-7B bf16 prefill, P = %d); "
                     "durations from a --kernel-trace run of the same sequence" % P,
           "formulas": {"mfma_busy_frac": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)",
                        "frac_of_bf16_peak": "algorithmic flops / avg duration / 2.5e15"},
           "meta": meta, "roles": res}
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", name + ".json"), "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])

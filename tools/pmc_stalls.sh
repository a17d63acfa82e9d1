#!/bin/bash
# Wave-state counters (where the wave-cycles go) of the kernels a probe program runs: two
# rocprofv3 --pmc passes (8 SQ counters each, never combined with trace domains), summed per
# kernel name over the dispatches and averaged.  PMC_PROBE (default tools/pmc_mfma_probe.py,
# the Qwen2-7B P = 2048 prefill), PMC_FILTER (substring of the kernel names to keep).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
probe=${PMC_PROBE:-tools/pmc_mfma_probe.py}
p1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
p2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA"
i=0
for p in "$p1" "$p2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $p --output-format csv -d "$R/gpurun_out/pmc_st$i" -o pmc \
      -- python3 "$R/$probe" > "$R/gpurun_out/pmc_st$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cd "$R" && PMC_FILTER=${PMC_FILTER:-} python3 - <<'PY'
import csv, glob, collections, os
flt = os.environ.get("PMC_FILTER", "")
tot = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for f in glob.glob("gpurun_out/pmc_st*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if flt and flt not in k:
            continue
        k = k.split("(")[0].replace("void ", "")[:60]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])] += 1
for k, d in tot.items():
    a = {c: v / max(1, cnt[(k, c)]) for c, v in d.items()}
    wc = a.get("SQ_WAVE_CYCLES", 0) or 1
    frac = {c: round(a[c] / wc, 3) for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                              "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS") if c in a}
    print(k, "per dispatch:", {c: round(v, 1) for c, v in sorted(a.items())}, "fraction of wave-cycles:", frac)
PY

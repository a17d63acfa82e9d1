#!/bin/bash
# Stall counters of the batch-8 decode projections (config 4, fp8: dec8 / skinny kernels): tools/ubench_b8.py under
# two rocprofv3 --pmc passes (one run each, never combined with trace domains).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
export UB8_FP8=${UB8_FP8:-1}
p1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD"
p2="SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_SCA SQ_WAVES"
i=0
for p in "$p1" "$p2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $p --output-format csv -d "$R/gpurun_out/pmc_sk$i" -o pmc \
      -- python3 "$R/tools/ubench_b8.py" > "$R/gpurun_out/pmc_sk$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cd "$R" && python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for f in glob.glob("gpurun_out/pmc_sk*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "skinny" not in k and "gemv_kernel" not in k and "dec8" not in k:
            continue
        k = k.split("(")[0][:70]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])] += 1
for k, d in tot.items():
    print(k, {c: round(v / max(1, cnt[(k, c)]), 1) for c, v in sorted(d.items())})
PY

#!/bin/bash
# rocprofv3 kernel stats of prefill (bench.py with 2 timed prefills, 1 decode step).
set -u
R=$GRAFT_REPO_ROOT; mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/pprof" -o pf \
   -- python3 "$R/bench.py" --steps 1 --warmup 0 --prefill-iters 2 --no-cpu-baseline ${PF_ARGS:-} > "$R/gpurun_out/pprof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$R" && python3 - <<'PY'
import csv, glob, collections
f = sorted(glob.glob("gpurun_out/pprof/**/*kernel_trace.csv", recursive=True))[-1]
agg = collections.defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("qie::", "")
    k = f"{n} g{r.get('Grid_Size_X','?')}x{r.get('Grid_Size_Y','?')}"
    agg[k][0] += 1; agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
    print(f"{k[:100]:100s} n={n:5d} total_us={t:10.1f} avg_us={t/n:9.2f}")
PY

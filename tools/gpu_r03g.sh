#!/bin/bash
# In-graph A/B of RoPE-in-projection (dev library): headline bench, alternating, 2 runs each.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export QIE_LIB=$GRAFT_REPO_ROOT/qwen_inference_engine_amd/lib/dev/libqie.so
for i in 1 2; do
  for rp in 0 1; do
    QIE_ROPE_IN_PROJ=$rp timeout -k 10 300 python -u bench.py --steps 200 --warmup 8 --no-cpu-baseline \
        > gpurun_out/r03g_rp${rp}_$i.log 2>&1
    rc=$?; echo "rp=$rp run $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python3 - "$rp" "$i" <<'PY'
import json, sys
for l in open(f"gpurun_out/r03g_rp{sys.argv[1]}_{sys.argv[2]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print("rp", sys.argv[1], d["value"], d["ms_per_step"], {k: v["avg_us"] for k, v in d["kernels"].items()})
PY
  done
done

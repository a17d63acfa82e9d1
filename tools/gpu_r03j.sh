#!/bin/bash
# config-4 A/B of the fp8 batched-decode kernel's fused norm (dev library), in-graph step time
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export QIE_LIB=$GRAFT_REPO_ROOT/qwen_inference_engine_amd/lib/dev/libqie.so
for v in "base:" "old:QIE_DEC8=0" "prenorm:QIE_DEC8_PRENORM=1" "nonw:QIE_DEC8_DBG=1" "nonorm:QIE_DEC8_DBG=2"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 300 python -u bench.py --fp8 --batch 8 --prompt 1024 --gen 256 --steps 128 --warmup 8 \
      --no-cpu-baseline > gpurun_out/r03j_$name.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -5 gpurun_out/r03j_$name.log; exit $rc; }
  python3 - "$name" <<'PY'
import json, sys
for l in open(f"gpurun_out/r03j_{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[1], d["value"], d["ms_per_step"], {k: v["avg_us"] for k, v in d["kernels"].items()})
PY
done

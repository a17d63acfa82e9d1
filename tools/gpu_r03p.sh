#!/bin/bash
# config-4 decode attention split-target A/B (dev library): 32 (default) / 8 / 4 / 32 again
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export QIE_LIB=$GRAFT_REPO_ROOT/qwen_inference_engine_amd/lib/dev/libqie.so
for v in "s32:" "s8:QIE_DEC_SPLITS=8" "s4:QIE_DEC_SPLITS=4" "s32b:"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 300 python -u bench.py --fp8 --batch 8 --prompt 1024 --gen 256 --steps 128 --warmup 8 \
      --no-cpu-baseline > gpurun_out/r03p_$name.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -5 gpurun_out/r03p_$name.log; exit $rc; }
  python3 - "$name" <<'PY'
import json, sys
for l in open(f"gpurun_out/r03p_{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[1], d["value"], d["ms_per_step"], {k: v["avg_us"] for k, v in d["kernels"].items()})
PY
done

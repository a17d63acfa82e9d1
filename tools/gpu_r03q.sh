#!/bin/bash
# config-4 attention split A/B (gpu_r03p.sh), then the other BASELINE configurations (one
# bench line each) and the config-4 kernel trace (gpu_r03i.sh)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_r03p.sh || exit $?
unset QIE_LIB
for cfg in "fp8b8:--fp8 --batch 8 --prompt 1024 --gen 256" "b8:--batch 8 --prompt 1024 --gen 256" \
           "c2:--model Qwen2-0.5B --prompt 128 --gen 128"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 400 python -u bench.py $args --no-cpu-baseline > gpurun_out/r03z_bench_$name.log 2>&1
  rc=$?; echo "bench $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
bash tools/gpu_r03i.sh

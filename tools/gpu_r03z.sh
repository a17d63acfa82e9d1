#!/bin/bash
# Round-3 final check (2/2): the other BASELINE configurations (one bench line each), then
# the config-4 kernel trace (gpu_r03i.sh), then the CPU baseline at BASELINE.md §3's sizes (P = 2048 prefill + 8 steps, median of 3).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "fp8b8:--fp8 --batch 8 --prompt 1024 --gen 256" "b8:--batch 8 --prompt 1024 --gen 256" \
           "c2:--model Qwen2-0.5B --prompt 128 --gen 128"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 400 python -u bench.py $args --no-cpu-baseline > gpurun_out/r03z_bench_$name.log 2>&1
  rc=$?; echo "bench $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
bash tools/gpu_r03i.sh || exit $?
timeout -k 10 700 python -u bench.py --steps 64 --cpu-full > gpurun_out/r03z_bench_cpufull.log 2>&1
rc=$?; echo "bench cpu-full rc=$rc"; exit $rc

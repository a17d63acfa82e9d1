#!/bin/bash
# CPU baseline at BASELINE.md §3's sizes (bench.py --cpu-full: P = 2048 prefill + 8 steps, median of 3)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u bench.py --steps 64 --cpu-full > gpurun_out/r03t_bench_cpufull.log
rc=$?; tail -1 gpurun_out/r03t_bench_cpufull.log | cut -c1-400; echo "bench cpu-full rc=$rc"; exit $rc

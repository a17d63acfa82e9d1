#!/bin/bash
# Round-3 final: the whole GPU suite, then the CPU baseline at BASELINE.md §3's sizes
# (bench.py --cpu-full: P = 2048 prefill + 8 decode steps, median of 3)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 600 \
    --timeout-method thread > gpurun_out/r03s_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03s_pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 560 python -u bench.py --steps 64 --cpu-full > gpurun_out/r03s_bench_cpufull.log 2>&1
rc=$?; tail -1 gpurun_out/r03s_bench_cpufull.log | cut -c1-600; echo "bench cpu-full rc=$rc"; exit $rc

#!/bin/bash
# qkv_post batched-load change: its GPU tests plus the prefill-bearing suites, then one
# rocprofv3 kernel trace of the headline bench for the kernel's duration.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; OUT=gpurun_out/qp; mkdir -p $OUT
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_ops.py tests/test_gpu_headline.py tests/test_gpu_paged.py tests/test_gpu_hf.py tests/test_gpu_engine.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof" -o run \
    -- python3 "$R/bench.py" --steps 16 --warmup 4 --prefill-iters 2 --no-cpu-baseline --no-configs > "$R/$OUT/prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc

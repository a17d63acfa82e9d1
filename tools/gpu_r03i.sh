#!/bin/bash
# rocprofv3 kernel trace of config 4 (fp8 weights, batch 8, prompt 1024) -> gpurun_out/prof_fp8
set -u
R=$GRAFT_REPO_ROOT
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_fp8" -o run \
    -- python3 "$R/bench.py" --fp8 --batch 8 --prompt 1024 --gen 256 --steps 32 --warmup 4 --prefill-iters 1 \
    --no-cpu-baseline > "$R/gpurun_out/prof_fp8.log" 2>&1
rc=$?; echo "rocprof fp8 rc=$rc"; tail -1 "$R/gpurun_out/prof_fp8.log" | cut -c1-400; exit $rc

#!/bin/bash
# Kernel-trace timeline of the headline decode (rocprofv3 --kernel-trace, no counters):
# per-kernel in-graph durations and the gaps between consecutive kernels.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/trace" -o tr \
   -- python3 "$R/bench.py" --steps 32 --warmup 2 --prefill-iters 1 --no-cpu-baseline ${TRACE_ARGS:-} > "$R/gpurun_out/trace.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$R" && python3 tools/trace_gaps.py gpurun_out/trace > gpurun_out/trace_gaps.txt && tail -40 gpurun_out/trace_gaps.txt

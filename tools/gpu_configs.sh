#!/bin/bash
# The BASELINE.md single-GPU configurations besides the headline (bench.py lines), then a
# kernel trace of config 4 (fp8 weights, batch 8) for its in-graph per-kernel durations.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline --fp8 --batch 8 --prompt 1024 --gen 256 --steps 255 > gpurun_out/cfg4_fp8.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --batch 8 --prompt 1024 --gen 256 --steps 255 > gpurun_out/cfg4_bf16.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --model Qwen2-0.5B --prompt 128 --gen 128 --steps 127 > gpurun_out/cfg2.log 2>&1 || exit $?
for f in cfg4_fp8 cfg4_bf16 cfg2; do tail -1 gpurun_out/$f.log | cut -c1-400; echo; done
if [ "${TRACE:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_cfg4" -o run \
     -- python3 "$R/bench.py" --no-cpu-baseline --fp8 --batch 8 --prompt 1024 --gen 256 --steps 64 --warmup 4 --prefill-iters 1 \
     > "$R/gpurun_out/prof_cfg4.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; exit $rc
fi

#!/bin/bash
# Config-2 regression, per kernel: rocprofv3 kernel traces of the round-3 tree (git worktree
# _ab/r03) and this tree on the same box, Qwen2-0.5B bf16, B = 1, P = 128, 127 timed steps
# (the driver's configs.config2 command).  tools/prof_compare.py reads the two traces.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for tree in ${TREES:-cur}; do   # the round-3 tree segfaults on the host under rocprofv3 (launch_step)
  src=$R; extra=--no-configs
  [ $tree = r03 ] && { src=$R/_ab/r03; extra=; }   # the round-3 bench has no config lines
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_c2_$tree" -o run \
      -- python3 "$src/bench.py" --model Qwen2-0.5B --prompt 128 --gen 128 --steps 127 --warmup 8 \
      --no-cpu-baseline $extra ${EXTRA:-} > "$R/gpurun_out/prof_c2_$tree.log" 2>&1
  rc=$?; echo "rocprof config2 $tree rc=$rc"; [ $rc -eq 0 ] || exit $rc
done

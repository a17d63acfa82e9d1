#!/bin/bash
# Config-2 graph-mode kernel traces at 64 timed steps (the length that completes under the
# profiler; 127 steps crash inside hipGraphLaunch's interception, r05 and r06): the round-3
# tree (git worktree _ab/r03, commit e468abd) then this tree, same box.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for tree in ${TREES:-r03 cur}; do
  src=$R; extra=--no-configs
  [ $tree = r03 ] && { src=$R/_ab/r03; extra=; }
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_c2g_$tree" -o run \
      -- python3 "$src/bench.py" --model Qwen2-0.5B --prompt 128 --gen 128 --steps 64 --warmup 4 \
      --prefill-iters 1 --no-cpu-baseline $extra > "$R/gpurun_out/prof_c2g_$tree.log" 2>&1
  rc=$?; echo "rocprof config2 graph $tree rc=$rc"; [ $rc -eq 0 ] || exit $rc
done

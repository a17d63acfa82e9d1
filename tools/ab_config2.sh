#!/bin/bash
# Config-2 regression A/B (verdict r04 item 7): the round-3 tree (git worktree _ab/r03, its own
# bench.py + libqie.so built from commit e468abd) against this tree, same box, same command,
# alternating three rounds: Qwen2-0.5B bf16, B = 1, P = 128, 127 timed steps after 8 warm-up
# (the driver's configs.config2 method) and 511 steps after 16 (the r03 profiles' method).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out
OUT=gpurun_out/r05_ab_config2.jsonl
: > $OUT
for round in 1 2 3; do
  for tree in _ab/r03 .; do
    for args in "--steps 127 --warmup 8" "--steps 511 --warmup 16"; do
      line=$(cd $tree && timeout -k 10 120 python bench.py --model Qwen2-0.5B --prompt 128 --gen 128 $args \
             --no-cpu-baseline 2>/dev/null | tail -1)
      rc=$?
      [ $rc -eq 0 ] || { echo "bench failed rc=$rc ($tree)"; exit $rc; }
      echo "{\"round\": $round, \"tree\": \"$tree\", \"args\": \"$args\", \"line\": $line}" >> $OUT
      python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['kernels']['attention']['avg_us'])" "$line" "$tree" "$args"
    done
  done
done

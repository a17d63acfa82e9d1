#!/bin/bash
# Round-6 final pass on one box; each GPU step under its own limit, stop at the first failure.
#   STEPS: 1 full -m gpu suite, 2 default bench line (N = 1), 3 rocprofv3 kernel traces
#   (headline, config 4), 4 config-2 graph-mode kernel trace (last: the profiler has crashed
#   on that graph before), 5 one-device TP2 rehearsal (peer backend)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; OUT=gpurun_out/r06f; mkdir -p $OUT
S=${STEPS:-1 2}
on() { case " $S " in *" $1 "*) return 0;; esac; return 1; }
if on 1; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?; tail -5 $OUT/tests.log; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if on 2; then
  timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
  rc=$?; tail -3 $OUT/bench.err; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if on 5; then
  QIE_BENCH_ONE_DEVICE=1 timeout -k 10 900 python -u bench.py --gpus 2 --comm peer --no-cpu-baseline \
    > $OUT/tp2.json 2> $OUT/tp2.err
  rc=$?; tail -3 $OUT/tp2.err; echo "tp2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if on 3; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof" -o run \
      -- python3 "$R/bench.py" --steps 64 --warmup 4 --prefill-iters 1 --no-cpu-baseline --no-configs \
      > "$R/$OUT/prof.log" 2>&1
  rc=$?; echo "rocprof headline rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_cfg4" -o run \
      -- python3 "$R/bench.py" --steps 64 --warmup 4 --prefill-iters 1 --no-cpu-baseline --no-configs \
      --batch 8 --fp8 --prompt 1024 --gen 256 --page-tokens 128 > "$R/$OUT/prof_cfg4.log" 2>&1
  rc=$?; echo "rocprof config4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
  cd "$R"
fi
if on 4; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/$OUT/prof_cfg2" -o run \
      -- python3 "$R/bench.py" --model Qwen2-0.5B --prompt 128 --gen 128 --steps 64 --warmup 4 --prefill-iters 1 \
      --no-cpu-baseline --no-configs > "$R/$OUT/prof_cfg2.log" 2>&1
  rc=$?; echo "rocprof config2 (graph) rc=$rc"; exit $rc
fi
exit 0

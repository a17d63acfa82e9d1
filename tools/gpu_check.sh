#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench.  Stops at the first fault/abort/timeout
# (exit codes other than 0/1 from pytest), never retries a GPU step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-} \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; echo "smoke rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ "${SKIP_BENCH:-0}" = "1" ] && exit 0
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; tail -3 gpurun_out/bench.log; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
if [ "${PROFILE:-0}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" \
      -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 64 --warmup 4 --prefill-iters 1 --no-cpu-baseline ${PROF_ARGS:-} \
      > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; cd "$GRAFT_REPO_ROOT"
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${PMC:-0}" = "1" ]; then
  # HBM traffic per launch: one counter per pass (FETCH_SIZE and WRITE_SIZE cannot share
  # a gfx950 TCC pass), --pmc alone (never with sys/runtime traces).
  cd /tmp && export TMPDIR=/tmp
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c" -o pmc \
        -- python3 "$GRAFT_REPO_ROOT/tools/pmc_probe.py" > "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c.log" 2>&1
    rc=$?; echo "pmc $c rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
  cd "$GRAFT_REPO_ROOT"
fi
exit $rc

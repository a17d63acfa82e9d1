#!/bin/bash
# Quick GPU pass: selected parity tests ($TESTS, default the decode/attention/engine files),
# then the headline bench without the CPU leg, then optional ubench ($UB_SET).  Stops at the
# first failure; never retries a GPU step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TESTS:-tests/test_gpu_ops.py tests/test_gpu_engine.py tests/test_gpu_headline.py tests/test_gpu_paged.py}
if [ "$T" != "none" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest $T -m gpu -x -q -p no:cacheprovider --timeout 300 \
      --timeout-method thread > gpurun_out/pytest_quick.log 2>&1
  rc=$?; tail -4 gpurun_out/pytest_quick.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 400 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_quick.log 2>&1
  rc=$?; tail -1 gpurun_out/bench_quick.log | cut -c1-600; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${UB_SET:-}" ]; then
  UB_SET=$UB_SET timeout -k 10 300 python tools/ubench.py > gpurun_out/ubench.log 2>&1
  rc=$?; cat gpurun_out/ubench.log | cut -c1-200; echo "ubench rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
exit 0

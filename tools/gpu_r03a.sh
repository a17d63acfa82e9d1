#!/bin/bash
# Round-3 check: the whole GPU suite (new parity / driver-tier / RCCL-in-graph tests included),
# then the default bench (CPU leg + full-depth forced-decision parity).  Stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider --timeout 600 \
    --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/r03a_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r03a_pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
[ "${SKIP_BENCH:-0}" = "1" ] && exit 0
timeout -k 10 900 python -u bench.py > gpurun_out/r03a_bench.log 2>&1
rc=$?; tail -1 gpurun_out/r03a_bench.log | cut -c1-3000; echo "bench rc=$rc"; exit $rc

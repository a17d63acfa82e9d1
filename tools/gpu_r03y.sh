#!/bin/bash
# Round-3 final check (1/2): the whole GPU suite, then the default headline bench (CPU leg +
# full-depth forced-decision parity).  Stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 600 \
    --timeout-method thread > gpurun_out/r03y_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r03y_pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r03y_bench.log 2>&1
rc=$?; tail -1 gpurun_out/r03y_bench.log | cut -c1-1500; echo "bench rc=$rc"; exit $rc

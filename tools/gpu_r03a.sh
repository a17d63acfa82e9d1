#!/bin/bash
# Round-3 check: the new parity / driver-tier tests, then the default bench (with the CPU leg
# and the full-depth forced-decision parity).  Stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_compat.py tests/test_gpu_headline.py -m gpu -x -v \
    -p no:cacheprovider --timeout 600 --timeout-method thread -s > gpurun_out/r03a_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r03a_pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/r03a_bench.log 2>&1
rc=$?; tail -1 gpurun_out/r03a_bench.log | cut -c1-3000; echo "bench rc=$rc"; exit $rc

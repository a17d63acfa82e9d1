#!/bin/bash
# GEMV/attention A/B on the dev library (ubench), quick parity tests, the headline bench.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
QIE_LIB=$GRAFT_REPO_ROOT/qwen_inference_engine_amd/lib/dev/libqie.so timeout -k 10 300 python -u tools/ubench.py \
    > gpurun_out/ubench.log 2>&1
rc=$?; cut -c1-200 gpurun_out/ubench.log; echo "ubench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_engine.py tests/test_gpu_headline.py -m gpu -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r03d_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03d_pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r03d_bench.log 2>&1
rc=$?; tail -1 gpurun_out/r03d_bench.log | cut -c1-1500; echo "bench rc=$rc"; exit $rc

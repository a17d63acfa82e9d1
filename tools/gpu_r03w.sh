#!/bin/bash
# final binary: smoke() + fp8 and engine GPU tests
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03w_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/r03w_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_engine.py "tests/test_gpu_headline.py::test_config4_fp8_batch8_prompt1024" \
    -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r03w_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r03w_pytest.log; echo "pytest rc=$rc"; exit $rc

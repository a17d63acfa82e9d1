#!/bin/bash
# r06 call A: mx probe (both lane maps), then the GPU tests touched this round.
set -u
OUT=gpurun_out/r06a; mkdir -p $OUT
timeout -k 10 120 ./tools/bin/mx_mfma_probe > $OUT/mx_probe.txt 2>&1; rc=$?
echo "probe_rc=$rc" >> $OUT/mx_probe.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_headline.py tests/test_gpu_fp8_mx.py tests/test_gpu_paged.py tests/test_gpu_tp.py > $OUT/tests.log 2>&1
echo "tests_rc=$?" >> $OUT/tests.log
tail -5 $OUT/tests.log

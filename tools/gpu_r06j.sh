#!/bin/bash
# r06 item 6: peer exchange forms (tagged / pushed) — parity, then the one-device TP2 rehearsal
set -u
OUT=gpurun_out/r06j; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_tp.py -k "peer" -x -v --timeout 300 --timeout-method thread \
  > $OUT/tp_tests.log 2>&1; rc=$?; tail -15 $OUT/tp_tests.log; echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
QIE_BENCH_ONE_DEVICE=1 timeout -k 10 900 python -u bench.py --gpus 2 --comm peer --no-cpu-baseline \
  > $OUT/tp2.json 2> $OUT/tp2.err; rc=$?; tail -3 $OUT/tp2.err; echo "bench rc=$rc"
exit $rc

#!/bin/bash
# r06 call B: the persistent decode step — bit-exact tests, then the in-process A/B.
set -u
OUT=gpurun_out/r06b; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_persist.py > $OUT/tests.log 2>&1
rc=$?; echo "tests_rc=$rc" >> $OUT/tests.log; tail -4 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=2 AB_STEPS=128 timeout -k 10 400 python -u tools/ab_persist.py > $OUT/ab.json 2> $OUT/ab.err
rc=$?; echo "ab_rc=$rc"; cat $OUT/ab.json; tail -3 $OUT/ab.err
exit $rc

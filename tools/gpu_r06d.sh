#!/bin/bash
# persistent step: bit-exact tests, phase trace, A/B
set -u
OUT=gpurun_out/r06d; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_persist.py > $OUT/tests.log 2>&1
rc=$?; echo "tests_rc=$rc" >> $OUT/tests.log; tail -4 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
PT_OUT=$OUT/stamps.npz timeout -k 10 300 python -u tools/pk_trace.py > $OUT/trace.json 2> $OUT/trace.err
rc=$?; echo "trace_rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('$OUT/trace.json'));print({k:v['cu_median'] for k,v in d['phases_since_layer_start'].items()}, d['kernel_span_us'])"
AB_ROUNDS=2 AB_STEPS=128 timeout -k 10 400 python -u tools/ab_persist.py > $OUT/ab.json 2> $OUT/ab.err
rc=$?; echo "ab_rc=$rc"; cat $OUT/ab.json
exit $rc

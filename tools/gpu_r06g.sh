#!/bin/bash
set -u
OUT=gpurun_out/r06g; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_persist.py > $OUT/tests.log 2>&1
rc=$?; echo "tests_rc=$rc" >> $OUT/tests.log; tail -4 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
AB_MODEL=Qwen2-0.5B AB_P=128 AB_ROUNDS=2 AB_STEPS=120 timeout -k 10 300 python -u tools/ab_persist.py > $OUT/ab05.json 2> $OUT/ab05.err
rc=$?; echo "ab05_rc=$rc"; cat $OUT/ab05.json; [ $rc -eq 0 ] || exit $rc
PT_MODEL=Qwen2-0.5B PT_P=128 PT_OUT=$OUT/stamps05.npz timeout -k 10 300 python -u tools/pk_trace.py > $OUT/trace05.json 2> $OUT/trace05.err
rc=$?; echo "trace05_rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('$OUT/trace05.json'));print({k:v['cu_median'] for k,v in d['phases_since_layer_start'].items()}, d['kernel_span_us'])"
OUT=$OUT/xw bash tools/pk_variants.sh QIE_PK_XW=100 QIE_PK_XW=92 QIE_PK_XW=85

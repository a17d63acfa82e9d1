#!/bin/bash
# r06: smoke() + persistent-mode tests + peer TP tests on the final build
set -u
OUT=gpurun_out/r06l; mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; tail -2 $OUT/smoke.log; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_tp.py tests/test_gpu_paged.py tests/test_gpu_headline.py -k "persist or peer or paged or config4" -x -v \
  --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
# config 4 (fp8, B = 8, paged 128): the first step's page loaded beside the position vs behind it
export AB_VARIANTS='[{"_PAGE": 128}, {"_PAGE": 128, "QIE_DEC_DBG": "256"}]'
QIE_LIB=qwen_inference_engine_amd/lib/dev/libqie.so AB_BATCH=8 AB_FP8=1 AB_P=1024 AB_STEPS=200 AB_ROUNDS=4 \
  timeout -k 10 600 python -u tools/ab_decode.py > $OUT/ab_pg.json 2> $OUT/ab_pg.err
rc=$?; tail -2 $OUT/ab_pg.err; cat $OUT/ab_pg.json; echo "ab rc=$rc"; exit $rc

#!/bin/bash
# r06: two-stream prefill A/B (dev build, same process, interleaved) + prefill parity tests
set -u
OUT=gpurun_out/r06m; mkdir -p $OUT
export AB_VARIANTS='[{}, {"QIE_PF_STREAMS": "0"}]'
QIE_LIB=qwen_inference_engine_amd/lib/dev/libqie.so AB_PREFILL=1 AB_STEPS=32 AB_ROUNDS=5 AB_KERNELS=0 \
  timeout -k 10 600 python -u tools/ab_decode.py > $OUT/ab_pf.json 2> $OUT/ab_pf.err
rc=$?; tail -2 $OUT/ab_pf.err; cat $OUT/ab_pf.json; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_engine.py tests/test_gpu_paged.py -x -q \
  --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; echo "tests rc=$rc"; exit $rc

#!/bin/bash
# r06: down-projection chunks-in-flight A/B (dev build, in-graph, interleaved variants)
set -u
OUT=gpurun_out/r06k; mkdir -p $OUT
DEFV='[{}, {"QIE_GEMV_XL2_U": "10"}, {"QIE_GEMV_XL2_U": "13"}]'
export AB_VARIANTS="${AB_VARIANTS:-$DEFV}"
QIE_LIB=qwen_inference_engine_amd/lib/dev/libqie.so AB_ROUNDS=4 AB_STEPS=256 \
  timeout -k 10 600 python -u tools/ab_decode.py > $OUT/ab_down.json 2> $OUT/ab_down.err
rc=$?; tail -3 $OUT/ab_down.err; cat $OUT/ab_down.json | tail -5; echo "ab rc=$rc"; exit $rc

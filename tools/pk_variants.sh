#!/bin/bash
# dev-build variants of the persistent step: phase trace + A/B per variant (QIE_LIB = dev build)
set -u
OUT=${OUT:-gpurun_out/pkv}; mkdir -p $OUT
export QIE_LIB=qwen_inference_engine_amd/lib/dev/libqie.so
i=0
for V in "$@"; do
  i=$((i+1))
  env $V PT_OUT=$OUT/stamps_$i.npz timeout -k 10 300 python -u tools/pk_trace.py > $OUT/trace_$i.json 2> $OUT/trace_$i.err
  rc=$?; [ $rc -eq 0 ] || { echo "variant $V trace rc=$rc"; tail -3 $OUT/trace_$i.err; exit $rc; }
  python3 -c "import json;d=json.load(open('$OUT/trace_$i.json'));print('$V', {k:v['cu_median'] for k,v in d['phases_since_layer_start'].items()}, d['kernel_span_us'])"
done

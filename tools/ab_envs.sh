#!/bin/bash
# bench.py (decode B=1 headline, no CPU baseline) once per environment string in $AB_LIST
# ("|"-separated, "-" = none); prints value / ms per step / prefill tok/s per variant.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
IFS='|' read -ra V <<< "${AB_LIST:--}"
i=0
for env in "${V[@]}"; do
  [ "$env" = "-" ] && env="QIE_NONE=1"
  timeout -k 10 300 env $env python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$i.log 2>&1 || { echo "FAIL $env"; exit 1; }
  python3 -c "
import json,sys
for l in open('gpurun_out/ab_$i.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$env', d['value'], d['ms_per_step'], 'prefill', d['prefill_tok_s'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
  i=$((i+1))
done

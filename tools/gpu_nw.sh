#!/bin/bash
# Prefill attention 4- vs 8-wave workgroups (dev build): bit-equality, timing, and the
# prefill-bearing GPU tests with the 8-wave form.  Each GPU step under its own limit.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; OUT=gpurun_out/nw; mkdir -p $OUT
export QIE_LIB=qwen_inference_engine_amd/lib/dev/libqie.so
timeout -k 10 180 python3 -u tools/attn_nw_check.py > $OUT/check.txt 2>&1
rc=$?; cat $OUT/check.txt; [ $rc -eq 0 ] || exit $rc
UB_ITERS=50 UB_ENVS="QIE_ATTN_PF_NW=8,QIE_ATTN_PF_NW=4,QIE_ATTN_PF_NW=8" timeout -k 10 300 python3 -u tools/ubench_prefill.py > $OUT/ub.jsonl 2>&1
rc=$?; cat $OUT/ub.jsonl; [ $rc -eq 0 ] || exit $rc
QIE_ATTN_PF_NW=8 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_headline.py tests/test_gpu_paged.py tests/test_gpu_hf.py tests/test_gpu_ops.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests_nw8.log 2>&1
rc=$?; tail -3 $OUT/tests_nw8.log; echo "tests rc=$rc"; exit $rc

#!/bin/bash
# prefill GEMM tile choice at 8,192 rows: GEMM + headline tests, config-4 and bf16 B=8 benches
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -k "big_gemm or linear" tests/test_gpu_fp8.py \
    -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r03r_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03r_pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for cfg in "fp8b8:--fp8 --batch 8 --prompt 1024 --gen 256" "b8:--batch 8 --prompt 1024 --gen 256"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 400 python -u bench.py $args --no-cpu-baseline > gpurun_out/r03r_bench_$name.log 2>&1
  rc=$?; echo "bench $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - "$name" <<'PY'
import json, sys
for l in open(f"gpurun_out/r03r_bench_{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[1], d["value"], d["ms_per_step"], "prefill", d["prefill_tok_s"], d["prefill_ms"])
PY
done

#!/bin/bash
# fp8 / ops parity, then config-4 (fp8 B=8), bf16 B=8 and the headline bench.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_ops.py -m gpu -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r03f_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03f_pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for cfg in "fp8b8:--fp8 --batch 8 --prompt 1024 --gen 256" "b8:--batch 8 --prompt 1024 --gen 256" "b1:"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 400 python -u bench.py $args --no-cpu-baseline > gpurun_out/r03f_bench_$name.log 2>&1
  rc=$?; echo "bench $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python - <<'PY'
import json
for f in ("fp8b8", "b8", "b1"):
    for l in open(f"gpurun_out/r03f_bench_{f}.log"):
        if l.startswith("{"):
            d = json.loads(l)
            print(f, d["value"], d["ms_per_step"], d["roofline"]["frac"], {k: v["avg_us"] for k, v in d["kernels"].items()})
PY

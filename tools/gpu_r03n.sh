#!/bin/bash
# fp8 tests + config-4 bench (release library)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp8.py -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r03n_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03n_pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --fp8 --batch 8 --prompt 1024 --gen 256 --no-cpu-baseline \
    > gpurun_out/r03n_bench_fp8b8.log 2>&1
rc=$?; echo "bench fp8b8 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import json
for l in open("gpurun_out/r03n_bench_fp8b8.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print("fp8b8", d["value"], d["ms_per_step"], d["roofline"]["frac"], d["step_roofline"]["frac"], {k: v["avg_us"] for k, v in d["kernels"].items()})
PY

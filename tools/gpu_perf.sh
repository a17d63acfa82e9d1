#!/bin/bash
# Parity tests, then the three decode benches (fp8 B=8, bf16 B=8, bf16 B=1 headline) with
# per-kernel timings; stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --fp8 --batch 8 --prompt 1024 --gen 256 --no-cpu-baseline > gpurun_out/bench_fp8.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --batch 8 --prompt 1024 --gen 256 --no-cpu-baseline > gpurun_out/bench_b8.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_b1.log 2>&1 || exit $?
python - <<'PY'
import json
for f in ("bench_fp8","bench_b8","bench_b1"):
    for l in open(f"gpurun_out/{f}.log"):
        if l.startswith("{"):
            d=json.loads(l); print(f, d["value"], d["ms_per_step"], {k:(v["avg_us"]) for k,v in d["kernels"].items()})
PY

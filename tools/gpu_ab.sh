#!/bin/bash
# Parity tests (optionally a subset), then bench.py with and without the A/B knobs in
# $AB_ENV (e.g. "QIE_GEMV_BALANCED=0 QIE_ATTN_PREFILL_V1=1"); stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_new.log 2>&1 || exit $?
timeout -k 10 300 env ${AB_ENV:-QIE_NOTHING=1} python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_old.log 2>&1 || exit $?
python - <<'PY'
import json
for f in ("bench_new", "bench_old"):
    for l in open(f"gpurun_out/{f}.log"):
        if l.startswith("{"):
            d = json.loads(l)
            print(f, d["value"], d["ms_per_step"], "prefill", d["prefill_tok_s"], d["prefill_ms"],
                  {k: v["avg_us"] for k, v in d["kernels"].items()})
PY

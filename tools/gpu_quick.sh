#!/bin/bash
# One GPU-box pass, every step optional, stops at the first failure (never retries a GPU step):
#   TESTS      pytest files/node ids for `-m gpu` ("all" = tests/, "none" = skip; default the
#              decode / attention / engine files); TEST_ENV="QIE_X=1 ..." runs them on the
#              development library with those knobs
#   BENCH=1    bench.py headline line without the CPU leg (BENCH_ARGS appended)
#   AB_VARIANTS='[{}, {"QIE_X": "1"}]'  tools/ab_decode.py on the development library
#              (AB_MODEL / AB_P / AB_STEPS / AB_ROUNDS / AB_BATCH / AB_FP8 / AB_PREFILL)
#   AB_GEMM_VARIANTS='[{}, {"QIE_GEMM8": "1"}]'  tools/ab_gemm.py (prefill GEMMs, bit-equality + time)
#   UB_SET     tools/ubench.py kernel variants (development library)
#   PROFILE=1  rocprofv3 kernel trace of a short bench (PROF_ARGS appended)
#   PMC=1      tools/pmc_traffic.sh (FETCH_SIZE / WRITE_SIZE per decode launch; PMC_CONFIG=fp8b8)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out
DEVLIB=$R/qwen_inference_engine_amd/lib/dev/libqie.so
T=${TESTS:-tests/test_gpu_ops.py tests/test_gpu_engine.py tests/test_gpu_headline.py tests/test_gpu_paged.py}
[ "$T" = "all" ] && T=tests
if [ "$T" != "none" ]; then
  # TEST_ENV="QIE_X=1 ...": run the tests on the development library with those knobs
  [ -n "${TEST_ENV:-}" ] && export QIE_LIB=$DEVLIB $TEST_ENV
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest $T -m gpu -x -q -p no:cacheprovider --timeout 300 \
      --timeout-method thread > gpurun_out/pytest_quick.log 2>&1
  rc=$?; tail -4 gpurun_out/pytest_quick.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
  if [ -n "${TEST_ENV:-}" ]; then unset QIE_LIB; for kv in $TEST_ENV; do unset "${kv%%=*}"; done; fi
fi
if [ -n "${AB_GEMM_VARIANTS:-}" ]; then
  QIE_LIB=$DEVLIB timeout -k 10 300 python -u tools/ab_gemm.py > gpurun_out/ab_gemm.log 2> gpurun_out/ab_gemm.err
  rc=$?; cat gpurun_out/ab_gemm.log | cut -c1-400; tail -3 gpurun_out/ab_gemm.err; echo "ab_gemm rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${AB_VARIANTS:-}" ]; then
  QIE_LIB=$DEVLIB timeout -k 10 ${AB_TIMEOUT:-600} python -u tools/ab_decode.py > gpurun_out/ab_decode.log 2> gpurun_out/ab_decode.err
  rc=$?; cat gpurun_out/ab_decode.log | cut -c1-700; tail -3 gpurun_out/ab_decode.err; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 400 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_quick.log 2>&1
  rc=$?; tail -1 gpurun_out/bench_quick.log | cut -c1-900; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${UB_SET:-}" ]; then
  QIE_LIB=$DEVLIB UB_SET=$UB_SET timeout -k 10 300 python tools/ubench.py > gpurun_out/ubench.log 2>&1
  rc=$?; cat gpurun_out/ubench.log | cut -c1-200; echo "ubench rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ "${PROFILE:-0}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run \
      -- python3 "$R/bench.py" --steps 64 --warmup 4 --prefill-iters 1 --no-cpu-baseline --no-configs ${PROF_ARGS:-} \
      > "$R/gpurun_out/prof.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; cd "$R"; [ $rc -eq 0 ] || exit $rc
fi
if [ "${PMC:-0}" = "1" ]; then   # HBM traffic per launch (FETCH_SIZE, WRITE_SIZE passes)
  PMC_CONFIG=${PMC_CONFIG:-} bash tools/pmc_traffic.sh
  rc=$?; [ $rc -eq 0 ] || exit $rc
fi
exit 0

#!/bin/bash
# fp8 tests (release), then config-4 A/B of the decode-kernel shapes (dev library)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp8.py -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r03o_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03o_pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
export QIE_LIB=$GRAFT_REPO_ROOT/qwen_inference_engine_amd/lib/dev/libqie.so
for v in "new:" "ks7:QIE_DEC8_KS14=0" "g8:QIE_DEC8G=1" "gold:QIE_DEC8G=0" "new2:"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 300 python -u bench.py --fp8 --batch 8 --prompt 1024 --gen 256 --steps 128 --warmup 8 \
      --no-cpu-baseline > gpurun_out/r03o_$name.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -5 gpurun_out/r03o_$name.log; exit $rc; }
  python3 - "$name" <<'PY'
import json, sys
for l in open(f"gpurun_out/r03o_{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[1], d["value"], d["ms_per_step"], {k: v["avg_us"] for k, v in d["kernels"].items()})
PY
done

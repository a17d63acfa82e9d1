#!/bin/bash
# RoPE-in-projection A/B (dev library), attention op tests, then rocprofv3 kernel traces of
# the headline decode and of the fp8 batch-8 configuration (BASELINE config 4).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
UB_VARIANTS='[["attn",5,{}],["attn",5,{"QIE_ROPE_IN_PROJ":"1"}],["qkv",2,{}],["qkv",2,{"QIE_ROPE_IN_PROJ":"1"}]]' \
QIE_LIB=$R/qwen_inference_engine_amd/lib/dev/libqie.so timeout -k 10 300 python -u tools/ubench.py \
    > gpurun_out/ubench.log 2>&1
rc=$?; cut -c1-200 gpurun_out/ubench.log; echo "ubench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k attention_decode -m gpu -x -q \
    -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03e_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03e_pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run \
    -- python3 "$R/bench.py" --steps 64 --warmup 4 --prefill-iters 1 --no-cpu-baseline > "$R/gpurun_out/prof.log" 2>&1
rc=$?; echo "rocprof headline rc=$rc"; tail -1 "$R/gpurun_out/prof.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_fp8" -o run \
    -- python3 "$R/bench.py" --fp8 --batch 8 --prompt 1024 --gen 256 --steps 32 --warmup 4 --prefill-iters 1 \
    --no-cpu-baseline > "$R/gpurun_out/prof_fp8.log" 2>&1
rc=$?; echo "rocprof fp8 rc=$rc"; tail -3 "$R/gpurun_out/prof_fp8.log" | cut -c1-300; exit $rc

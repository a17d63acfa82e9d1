#!/bin/bash
# ubench A/B ($UB_VARIANTS, dev library) first, then the GPU suite + default bench (tools/gpu_r03a.sh).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -n "${UB_VARIANTS:-}" ]; then
  QIE_LIB=$GRAFT_REPO_ROOT/qwen_inference_engine_amd/lib/dev/libqie.so timeout -k 10 300 python -u tools/ubench.py \
      > gpurun_out/ubench.log 2>&1
  rc=$?; cut -c1-200 gpurun_out/ubench.log; echo "ubench rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
[ "${SKIP_SUITE:-0}" = "1" ] && exit 0
exec_rc=0
bash tools/gpu_r03a.sh

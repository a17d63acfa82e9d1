#!/bin/bash
# stream probe (pure weight-stream floor per launch), then the suite + bench (gpu_r03a.sh)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 240 ./tools/bin/stream_probe > gpurun_out/stream_probe.log 2>&1
rc=$?; cat gpurun_out/stream_probe.log; echo "probe rc=$rc"; [ $rc -eq 0 ] || exit $rc
[ "${SKIP_SUITE:-0}" = "1" ] && exit 0
bash tools/gpu_r03a.sh

#!/bin/bash
# fp8 tests + config-4 bench + kernel trace (gpu_r03l.sh), then config-4 PMC HBM traffic
set -u
R=$GRAFT_REPO_ROOT
bash "$R/tools/gpu_r03l.sh" || exit $?
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  PMC_CONFIG=fp8b8 timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/pmc_$c" -o pmc \
      -- python3 "$R/tools/pmc_probe.py" > "$R/gpurun_out/pmc_$c.log" 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done

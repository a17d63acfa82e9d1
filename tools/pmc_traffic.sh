#!/bin/bash
# HBM traffic per launch of the decode kernels: one rocprofv3 --pmc pass per counter
# (FETCH_SIZE and WRITE_SIZE cannot share a gfx950 TCC pass), never with trace domains.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/pmc_$c" -o pmc \
      -- python3 "$R/tools/pmc_probe.py" > "$R/gpurun_out/pmc_$c.log" 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done

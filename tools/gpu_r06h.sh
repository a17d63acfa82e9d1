#!/bin/bash
# r06 call H: MX probe lane-map fit, PMC traffic (headline + config-4 paged), config-2 graph trace
set -u
R=$(pwd); OUT=$R/gpurun_out/r06h; mkdir -p $OUT
timeout -k 10 120 ./tools/bin/mx_mfma_probe > $OUT/mx_probe.txt 2>&1; rc=$?; echo "probe_rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for cfg in head c4; do
  if [ $cfg = c4 ]; then export PMC_CONFIG=fp8b8 PMC_PAGED=128; else unset PMC_CONFIG PMC_PAGED; fi
  bash tools/pmc_traffic.sh; rc=$?; [ $rc -eq 0 ] || exit $rc
  name=r06_pmc_traffic; [ $cfg = c4 ] && name=r06_fp8_b8_paged_pmc_traffic
  python3 tools/pmc_summary.py $name > $OUT/pmc_$cfg.txt 2>&1; cp profiles/$name.json $OUT/ 2>/dev/null
  mkdir -p $OUT/pmc_$cfg; cp -r gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE gpurun_out/pmc_probe_meta.json $OUT/pmc_$cfg/ 2>/dev/null
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run \
    -- python3 $R/bench.py --model Qwen2-0.5B --prompt 128 --gen 128 --steps 127 --warmup 8 --no-cpu-baseline --no-configs \
    > $OUT/prof_c2.log 2>&1
echo "rocprof_c2_rc=$?"

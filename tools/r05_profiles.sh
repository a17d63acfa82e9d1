#!/bin/bash
# Round-5 profile pass on one box (each step under its own limit, stop at the first failure):
#   1. config-2 kernel traces, round-3 tree vs this tree (tools/prof_config2.sh)
#   2. headline kernel trace (gpurun_out/prof) and config-4 kernel trace (gpurun_out/prof_cfg4)
#   3. HBM traffic passes, headline then config 4 (r05_pmc_traffic, r05_fp8_b8_pmc_traffic)
#   4. prefill MFMA counter passes (r05_pmc_mfma)
# STEPS="1 2 3 4" selects.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out
S=${STEPS:-1 2 3 4}
on() { case " $S " in *" $1 "*) return 0;; esac; return 1; }
if on 1; then bash tools/prof_config2.sh || exit $?; fi
if on 2; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run \
      -- python3 "$R/bench.py" --steps 64 --warmup 4 --prefill-iters 1 --no-cpu-baseline --no-configs \
      > "$R/gpurun_out/prof.log" 2>&1
  rc=$?; echo "rocprof headline rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_cfg4" -o run \
      -- python3 "$R/bench.py" --steps 64 --warmup 4 --prefill-iters 1 --no-cpu-baseline --no-configs \
      --batch 8 --fp8 --prompt 1024 --gen 256 --page-tokens 128 > "$R/gpurun_out/prof_cfg4.log" 2>&1
  rc=$?; echo "rocprof config4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
  cd "$R"
fi
if on 3; then
  PMC_CONFIG= bash tools/pmc_traffic.sh || exit $?
  python3 tools/pmc_summary.py r05_pmc_traffic && cp profiles/r05_pmc_traffic.json gpurun_out/ || exit $?
  PMC_CONFIG=fp8b8 bash tools/pmc_traffic.sh || exit $?
  python3 tools/pmc_summary.py r05_fp8_b8_pmc_traffic && cp profiles/r05_fp8_b8_pmc_traffic.json gpurun_out/ || exit $?
fi
if on 4; then PMC_TAG=r05 bash tools/pmc_mfma.sh || exit $?; fi
exit 0

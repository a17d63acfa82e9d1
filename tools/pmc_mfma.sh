#!/bin/bash
# MFMA counter passes over the Qwen2-7B P = 2048 prefill (tools/pmc_mfma_probe.py), one
# rocprofv3 --pmc run per pass (never combined with trace domains), then the summary.
# A pass whose counters the box does not list is skipped, not retried.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 -L > "$R/gpurun_out/pmc_avail.txt" 2>&1 || true
have() { for c in "$@"; do grep -q "\b$c\b" "$R/gpurun_out/pmc_avail.txt" || return 1; done; return 0; }
pass() {   # pass <dir> <counters...>
  local d=$1; shift
  if ! have "$@"; then echo "skip $d: $* not listed"; return 0; fi
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/$d" -o pmc \
      -- python3 "$R/tools/pmc_mfma_probe.py" > "$R/gpurun_out/$d.log" 2>&1
  local rc=$?; echo "pass $d ($*) rc=$rc"; return $rc
}
pass pmc_mfma_busy SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE || exit $?
pass pmc_mfma_mops SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_BF16 || exit $?
pass pmc_mfma_lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE || exit $?
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_mfma_trace" -o tr \
    -- python3 "$R/tools/pmc_mfma_probe.py" > "$R/gpurun_out/pmc_mfma_trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$R" && python3 tools/pmc_mfma_summary.py "${PMC_TAG:-r02}_pmc_mfma" && cp profiles/${PMC_TAG:-r02}_pmc_mfma.json gpurun_out/

#!/bin/bash
# Round-6 GPU passes on one box (gpurun), one named step or several: STEPS="persist pmc".
# Each GPU step runs under its own time limit; the script stops at the first failure.
#   mxprobe   tools/bin/mx_mfma_probe -> profiles/r06_mx_mfma_probe.txt (both lane maps)
#   persist   tests/test_gpu_persist.py, then tools/ab_persist.py and tools/pk_trace.py at
#             Qwen2-7B (profiles/r06_pk_evidence.json)
#   persist05 the same A/B and trace at Qwen2-0.5B, then the XCD row-share variants
#             (tools/pk_variants.sh QIE_PK_XW=100/92/85, dev build)
#   pmc       HBM traffic passes, headline and config 4 on the paged cache
#             (profiles/r06_pmc_traffic.json, profiles/r06_fp8_b8_paged_pmc_traffic.json)
#   graphdump every node of the 0.5B and 7B decode graphs (dev QIE_GRAPH_DUMP;
#             profiles/r06_graph_nodes_*.txt)
#   peer      the peer-backend tests, then the one-device TP2 rehearsal
#             (profiles/r06_bench_tp2_peer_onedevice.json)
# Final-build passes (full -m gpu suite, bench line, rocprof traces): tools/r06_final.sh.
# Measured and dropped this round, their dev knobs removed after the measurement (DESIGN.md
# §13): down-GEMV chunks in flight (profiles/r06_ab_down_chunks.json), the paged first-step
# page loaded beside the position (profiles/r06_ab_paged_page_prefetch.json), two-stream
# prefill (profiles/r06_ab_prefill_two_streams.json) — each an interleaved tools/ab_decode.py
# run over the variants named in its JSON.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; OUT=gpurun_out/r06; mkdir -p $OUT
S=${STEPS:-persist}
on() { case " $S " in *" $1 "*) return 0;; esac; return 1; }
DEV=qwen_inference_engine_amd/lib/dev/libqie.so
if on mxprobe; then
  timeout -k 10 120 ./tools/bin/mx_mfma_probe > $OUT/mx_probe.txt 2>&1; rc=$?; echo "probe rc=$rc"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
if on persist; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_persist.py \
    > $OUT/persist_tests.log 2>&1; rc=$?; tail -3 $OUT/persist_tests.log; [ $rc -eq 0 ] || exit $rc
  AB_ROUNDS=2 AB_STEPS=128 timeout -k 10 400 python -u tools/ab_persist.py > $OUT/ab7b.json 2> $OUT/ab7b.err
  rc=$?; cat $OUT/ab7b.json; [ $rc -eq 0 ] || exit $rc
  PT_OUT=$OUT/stamps7b.npz timeout -k 10 300 python -u tools/pk_trace.py > $OUT/trace7b.json 2> $OUT/trace7b.err
  rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if on persist05; then
  AB_MODEL=Qwen2-0.5B AB_P=128 AB_ROUNDS=2 AB_STEPS=120 timeout -k 10 300 python -u tools/ab_persist.py \
    > $OUT/ab05.json 2> $OUT/ab05.err; rc=$?; cat $OUT/ab05.json; [ $rc -eq 0 ] || exit $rc
  PT_MODEL=Qwen2-0.5B PT_P=128 PT_OUT=$OUT/stamps05.npz timeout -k 10 300 python -u tools/pk_trace.py \
    > $OUT/trace05.json 2> $OUT/trace05.err; rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
  OUT=$OUT/xw bash tools/pk_variants.sh QIE_PK_XW=100 QIE_PK_XW=92 QIE_PK_XW=85 || exit $?
fi
if on pmc; then
  for cfg in head c4; do
    if [ $cfg = c4 ]; then export PMC_CONFIG=fp8b8 PMC_PAGED=128; else unset PMC_CONFIG PMC_PAGED; fi
    bash tools/pmc_traffic.sh || exit $?
    name=r06_pmc_traffic; [ $cfg = c4 ] && name=r06_fp8_b8_paged_pmc_traffic
    python3 tools/pmc_summary.py $name > $OUT/pmc_$cfg.txt 2>&1 || exit $?
  done
fi
if on graphdump; then
  QIE_LIB=$DEV QIE_GRAPH_DUMP=1 GD_MODEL=Qwen2-0.5B timeout -k 10 120 python3 tools/graph_dump.py > $OUT/dump05.txt 2>&1 \
    || exit $?
  QIE_LIB=$DEV QIE_GRAPH_DUMP=1 GD_MODEL=Qwen2-7B GD_P=2048 timeout -k 10 200 python3 tools/graph_dump.py \
    > $OUT/dump7b.txt 2>&1 || exit $?
  grep "graph:" $OUT/dump05.txt $OUT/dump7b.txt
fi
if on peer; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_tp.py -k "peer" -x -v --timeout 300 --timeout-method thread \
    > $OUT/peer_tests.log 2>&1; rc=$?; tail -3 $OUT/peer_tests.log; [ $rc -eq 0 ] || exit $rc
  QIE_BENCH_ONE_DEVICE=1 timeout -k 10 900 python -u bench.py --gpus 2 --comm peer --no-cpu-baseline \
    > $OUT/tp2.json 2> $OUT/tp2.err; rc=$?; echo "tp2 rc=$rc"; exit $rc
fi
exit 0

#!/bin/bash
set -u
OUT=gpurun_out/r06c; mkdir -p $OUT
PT_OUT=$OUT/stamps.npz timeout -k 10 300 python -u tools/pk_trace.py > $OUT/trace.json 2> $OUT/trace.err
rc=$?; echo "trace_rc=$rc"; cat $OUT/trace.json; tail -3 $OUT/trace.err; exit $rc

#!/bin/bash
set -u
OUT=gpurun_out/r06i; mkdir -p $OUT
export QIE_LIB=qwen_inference_engine_amd/lib/dev/libqie.so QIE_GRAPH_DUMP=1
GD_MODEL=Qwen2-0.5B timeout -k 10 120 python3 tools/graph_dump.py > $OUT/dump05.txt 2>&1; echo "rc05=$?"
GD_MODEL=Qwen2-7B GD_P=2048 timeout -k 10 200 python3 tools/graph_dump.py > $OUT/dump7b.txt 2>&1; echo "rc7b=$?"
grep "graph:" $OUT/dump05.txt $OUT/dump7b.txt

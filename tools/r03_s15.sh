#!/bin/bash
# Wave-fill study: tile 16 time vs block count (n sweep) on deep-layer shapes
set -e
mkdir -p gpurun_out/r03
X=""
for n in 16 24 32 40 41 48 64 80 96; do X="$X;$n,20,20,512,512,3,1"; done
for n in 8 16 24 32 40 41 48; do X="$X;$n,40,40,256,256,3,1"; done
for n in 8 16 24 32 40 41; do X="$X;$n,40,40,512,256,1,1"; done
IDX=$(python3 -c "print(','.join(str(28+i) for i in range(9+7+6)))")
CONV_EXTRA="${X#;}" CONV_SHAPES=$IDX timeout -k 10 300 python3 tests/probes/conv_bench.py 16 18 > gpurun_out/r03/fill.log 2>&1
cat gpurun_out/r03/fill.log

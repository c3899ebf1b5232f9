#!/bin/bash
# Kernel-trace summaries of the side configurations (run through gpurun):
#   bash tools/side_profiles.sh r02  ->  gpurun_out/<round>/side_prof_{fp8_b64,c4_1280}/
set -e -o pipefail
R=${1:-r02}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$R
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/side_prof_fp8_b64" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --precision fp8 --batch 64 --cpu-seconds 0 --steps 40 > "$OUT/side_prof_fp8_b64.log" 2>&1
tail -n 1 "$OUT/side_prof_fp8_b64.log" | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/side_prof_c4_1280" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --size 1280 --batch 8 --cpu-seconds 0 --steps 40 > "$OUT/side_prof_c4_1280.log" 2>&1
tail -n 1 "$OUT/side_prof_c4_1280.log" | cut -c1-200

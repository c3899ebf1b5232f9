#!/bin/bash
# Side configurations of BASELINE.json outside the profiler (run through gpurun), one bench line
# each, comparable with the headline (tools/side_profiles.sh takes the same configs under rocprofv3):
#   bash tools/side_plain.sh r05  ->  gpurun_out/<round>/plain_<name>.json
set -e -o pipefail
R=${1:-r05}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$R
mkdir -p "$OUT"
cd "$ROOT"
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python3 bench.py --cpu-seconds 0 --fp16-steps 0 --pipelined-steps 0 "$@" > "$OUT/plain_$name.log" 2>&1
  grep '^{"metric' "$OUT/plain_$name.log" | tail -n 1 > "$OUT/plain_$name.json"
  cut -c1-160 "$OUT/plain_$name.json"
}
run fp16 --precision fp16
run fp8_b64 --precision fp8 --batch 64
run c4_1280 --size 1280 --batch 8
run b64 --batch 64

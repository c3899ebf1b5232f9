#!/bin/bash
# Side configurations of BASELINE.json under rocprofv3 --kernel-trace --stats, each with its bench
# line and per-op roofline gap table (run through gpurun):
#   bash tools/side_profiles.sh r04  ->  gpurun_out/<round>/side_<name>/ + side_<name>.json / _ops.json
# fp16 bs 32 (the north_star mode), fp8 bs 64 (C5), 1280^2 bs 8 (C4), bf16 bs 64 (C5's shape in bf16).
set -e -o pipefail
R=${1:-r04}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$R
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
run() {  # name, bench args...
  local name=$1; shift
  YCX_BENCH_KERNELS=$OUT/side_${name}_ops.json timeout -k 10 400 rocprofv3 --kernel-trace --stats \
    -d "$OUT/side_$name" -o run --output-format csv -- python3 "$ROOT/bench.py" --cpu-seconds 0 --steps 40 "$@" \
    > "$OUT/side_$name.log" 2>&1
  grep '^{"metric' "$OUT/side_$name.log" | tail -n 1 > "$OUT/side_$name.json"
  cut -c1-160 "$OUT/side_$name.json"
}
run fp16 --precision fp16
run fp8_b64 --precision fp8 --batch 64
run c4_1280 --size 1280 --batch 8
run b64 --batch 64

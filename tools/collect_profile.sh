#!/bin/bash
# Copy the summaries of a tools/profile_round.sh run (merged back into gpurun_out/<round>/) into
# profiles/<round>/ (tracked):  bash tools/collect_profile.sh r04
set -e
R=${1:-r04}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$R
P=$ROOT/profiles/$R
mkdir -p "$P"
grep "^{\"metric" "$OUT/bench_under_rocprof.log" | tail -n 1 > "$P/bench_under_rocprof.json"
cp "$(find "$OUT/trace" -name '*kernel_stats.csv' | head -n 1)" "$P/kernel_stats.csv"
[ -f "$OUT/kernel_stats_roofline_leg.csv" ] && cp "$OUT/kernel_stats_roofline_leg.csv" "$P/"
cp "$OUT/trace_legs.txt" "$OUT/ops.json" "$OUT/traffic.json" "$OUT/traffic_summary.json" "$P/"
python3 "$ROOT/tools/op_gap.py" "$OUT/ops.json" > "$P/op_gap.md"
tail -n 1 "$OUT/bench.log" > "$P/bench.json"
ls "$P"

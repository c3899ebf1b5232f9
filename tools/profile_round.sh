#!/bin/bash
# Profile this round's bench on the GPU box (run through gpurun), one coherent set from one build:
#   bash tools/profile_round.sh r04
# 1. rocprofv3 --kernel-trace --stats of the bench command (headline leg and its roofline leg; the
#    fp16 leg and the CPU baseline are left out so that the roofline leg is the trace's last conv work:
#    the f16 build's kernels carry the same symbol names); the same run writes the per-op roofline gap
#    table (YCX_BENCH_KERNELS, HIP events of the serial roofline leg)
# 2. tools/trace_leg_stats.py: the profiler's own per-kernel averages over that roofline leg
# 3. two PMC passes (FETCH_SIZE, WRITE_SIZE) over tools/pmc_workload.py
# 4. tools/pmc_traffic.py -> per-op HBM bytes (traffic.json)
# 5. the bench again, now reporting roofline.traffic from profiles/<round>/traffic.json
# Everything lands in gpurun_out/<round>/ (the box merges only gpurun_out/ back); then, locally,
#   bash tools/collect_profile.sh r04   copies the summaries into profiles/<round>/.
set -e -o pipefail
R=${1:-r04}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$R
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
YCX_BENCH_KERNELS=$OUT/ops.json timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run \
  --output-format csv -- python3 "$ROOT/bench.py" --fp16-steps 0 --pipelined-steps 0 --cpu-seconds 0 > "$OUT/bench_under_rocprof.log" 2>&1
TRACE=$(find "$OUT/trace" -name '*kernel_trace.csv' | head -n 1)
NOPS=$(python3 -c "import json; print(len(json.load(open('$OUT/ops.json'))['ops']))")
python3 "$ROOT/tools/trace_leg_stats.py" "$TRACE" "$NOPS" 3 "$OUT/kernel_stats_roofline_leg.csv" > "$OUT/trace_legs.txt"
python3 "$ROOT/tools/op_gap.py" "$OUT/ops.json" > "$OUT/op_gap.md"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
  python3 "$ROOT/tools/pmc_workload.py" > "$OUT/pmc_fetch.log" 2>&1
cp "$ROOT/gpurun_out/pmc_ops.json" "$OUT/pmc_ops_fetch.json"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
  python3 "$ROOT/tools/pmc_workload.py" > "$OUT/pmc_write.log" 2>&1
python3 "$ROOT/tools/pmc_traffic.py" --fetch "$OUT/pmc_fetch" --write "$OUT/pmc_write" \
  --ops "$ROOT/gpurun_out/pmc_ops.json" --out "$OUT/traffic.json" > "$OUT/traffic_summary.json"
mkdir -p "$ROOT/profiles/$R" && cp "$OUT/traffic.json" "$ROOT/profiles/$R/traffic.json"  # read by the bench below
cd "$ROOT"
timeout -k 10 300 python3 bench.py > "$OUT/bench.log" 2>&1
tail -n 1 "$OUT/bench.log" | cut -c1-600

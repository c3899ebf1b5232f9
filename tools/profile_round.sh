#!/bin/bash
# Profile this round's bench on the GPU box (run through gpurun):
#   bash tools/profile_round.sh r01
# 1. rocprofv3 --kernel-trace --stats of the default bench command
# 2. two PMC passes (FETCH_SIZE, WRITE_SIZE) over tools/pmc_workload.py
# 3. tools/pmc_traffic.py -> per-op HBM bytes (traffic.json)
# 4. the bench again, now reporting roofline.traffic from traffic.json
# Everything lands in gpurun_out/<round>/; copy the summaries into profiles/<round>/.
set -e -o pipefail
R=${1:-r01}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$R
mkdir -p "$OUT" "$ROOT/profiles/$R"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" > "$OUT/bench_under_rocprof.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
  python3 "$ROOT/tools/pmc_workload.py" > "$OUT/pmc_fetch.log" 2>&1
cp "$ROOT/gpurun_out/pmc_ops.json" "$OUT/pmc_ops_fetch.json"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
  python3 "$ROOT/tools/pmc_workload.py" > "$OUT/pmc_write.log" 2>&1
python3 "$ROOT/tools/pmc_traffic.py" --fetch "$OUT/pmc_fetch" --write "$OUT/pmc_write" \
  --ops "$ROOT/gpurun_out/pmc_ops.json" --out "$OUT/traffic.json" > "$OUT/traffic_summary.json"
cp "$OUT/traffic.json" "$ROOT/profiles/$R/traffic.json"
cd "$ROOT"
timeout -k 10 300 python3 bench.py > "$OUT/bench.log" 2>&1
tail -n 1 "$OUT/bench.log"

#!/bin/bash
# Same-box comparison of several arms of the concurrent bench (development tool), interleaved
# ROUNDS times (default 2). Each arm is NAME or NAME:VAR=value[;VAR=value...] on the in-tree
# library; BENCH_ARGS are passed to bench.py, and an arm's own ARM_ARGS after them. Run through gpurun:
#   BENCH_ARGS="--batch 64" bash tools/ab_arms.sh r06 base 'big:YCX_TILE_MAP=16<600:25/26'
R=${1:-r06}; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$ROOT/gpurun_out/$R/arms
mkdir -p "$O"
FAST="--cpu-seconds 0 --fp16-steps 0 --pipelined-steps 0 --image-in-steps 0 --latency-steps 0"
for r in $(seq 1 "${ROUNDS:-2}"); do
  for arm in "$@"; do
    name=${arm%%:*}
    envs=""
    [ "$name" != "$arm" ] && envs=${arm#*:}
    (
      IFS=';'
      for kv in $envs; do export "$kv"; done
      unset IFS
      YCX_BENCH_KERNELS=$O/ops_${name}_$r.json timeout -k 10 300 python "$ROOT/bench.py" $FAST $BENCH_ARGS $ARM_ARGS \
        > "$O/bench_${name}_$r.log" 2>&1
    ) || { echo "arm $name failed"; tail -5 "$O/bench_${name}_$r.log"; exit 1; }
    tail -1 "$O/bench_${name}_$r.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['value'], d['ms_per_step'], d['roofline']['forward_kernel_ms'])"
  done
done

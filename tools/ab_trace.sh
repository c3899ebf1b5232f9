#!/bin/bash
# Same-box A/B of the concurrent bench (development tool), with the kernels-in-flight split of
# each arm: A = yolo-continuous_amd/ycx/libycx_A.so (or A_ENV="VAR=value" on the in-tree library),
# B = the in-tree library. Run through gpurun:  bash tools/ab_trace.sh r06 [bench args]
# 1. the bench, A B A B (--cpu-seconds 0 --fp16-steps 0 --pipelined-steps 0 --image-in-steps 0), per-op tables of both arms
# 2. per arm (unless NO_TRACE=1): rocprofv3 --kernel-trace of the bench's timed loop -> tools/trace_busy.py
R=${1:-r06}; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$ROOT/gpurun_out/$R/ab
mkdir -p "$O"
A=$ROOT/yolo-continuous_amd/ycx/libycx_A.so
arm() {  # arm A|B: the environment of that arm
  unset YCX_LIB
  if [ "$1" = A ]; then
    if [ -n "$A_ENV" ]; then export "$A_ENV"; else export YCX_LIB=$A; fi
  else
    [ -n "$A_ENV" ] && unset "${A_ENV%%=*}"
  fi
}
FAST="--cpu-seconds 0 --fp16-steps 0 --pipelined-steps 0 --image-in-steps 0"
for v in A B A B; do
  arm $v
  YCX_BENCH_KERNELS=$O/ops_$v.json timeout -k 10 300 python "$ROOT/bench.py" $FAST "$@" > "$O/bench_$v.log" 2>&1 || { tail -5 "$O/bench_$v.log"; exit 1; }
  tail -1 "$O/bench_$v.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['p50_ms'], d['roofline']['forward_kernel_ms'])"
done
[ -n "$NO_TRACE" ] && exit 0
cd /tmp && export TMPDIR=/tmp
for v in A B; do
  arm $v
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/trace_$v" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" $FAST --latency-steps 0 --roofline-steps 1 "$@" > "$O/trace_$v.log" 2>&1 || { tail -5 "$O/trace_$v.log"; exit 1; }
  python3 "$ROOT/tools/trace_busy.py" "$(find "$O/trace_$v" -name '*kernel_trace.csv' | head -n 1)" > "$O/busy_$v.txt"
  echo "busy $v"; head -8 "$O/busy_$v.txt"
  rm -rf "$O/trace_$v"
done

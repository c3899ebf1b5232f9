#!/bin/bash
# GPU jobs (run through gpurun):  YCX_ROUND=r05 bash tools/job.sh JOB [args]
# Every GPU step has its own time limit and the steps are chained with &&.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
O=$R/gpurun_out/${YCX_ROUND:-r05}
mkdir -p "$O"
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
job=$1
shift
case "$job" in
  tests)  # a test selection: bash tools/job.sh tests 'tests/test_x.py::y' ...
    timeout -k 10 900 $PYT -s "$@" > "$O/tests.log" 2>&1; rc=$?
    tail -30 "$O/tests.log"; exit $rc ;;
  bench)  # the default bench + the per-op gap table
    YCX_BENCH_KERNELS=$O/ops.json timeout -k 10 600 python bench.py "$@" > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
    tail -1 "$O/bench.log" | cut -c1-3000
    python tools/op_gap.py "$O/ops.json" 25 > "$O/op_gap.md" && head -40 "$O/op_gap.md" ;;
  full)  # the round-end sequence: GPU suite, smoke, bench
    timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/gputests.log" 2>&1 || { tail -40 "$O/gputests.log"; exit 1; }
    tail -2 "$O/gputests.log"
    timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
    tail -1 "$O/smoke.log"
    YCX_BENCH_KERNELS=$O/ops.json timeout -k 10 600 python bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
    tail -1 "$O/bench.log" | cut -c1-1500
    python tools/op_gap.py "$O/ops.json" > "$O/op_gap.md" ;;
  probe)  # a probe script: bash tools/job.sh probe tests/probes/x.py args
    timeout -k 10 600 python -u "$@" > "$O/probe.log" 2>&1; rc=$?
    tail -60 "$O/probe.log"; exit $rc ;;
  *) echo "unknown job $job"; exit 2 ;;
esac

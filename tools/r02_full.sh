#!/bin/bash
# Round-2 checkpoint (run through gpurun): GPU suite, smoke, default bench, rocprof profile.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r02
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02/gputests.log 2>&1 || { tail -40 gpurun_out/r02/gputests.log; exit 1; }
tail -2 gpurun_out/r02/gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02/smoke.log 2>&1 || { tail -20 gpurun_out/r02/smoke.log; exit 1; }
tail -1 gpurun_out/r02/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r02/bench_default.log 2>&1 || { tail -20 gpurun_out/r02/bench_default.log; exit 1; }
tail -1 gpurun_out/r02/bench_default.log
bash tools/profile_round.sh r02

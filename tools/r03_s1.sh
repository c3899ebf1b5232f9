# round-3 checkpoint: full GPU suite (incl. fp16 plan), smoke, default bench, fp16 bench line
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r03/gputests.log 2>&1 || { tail -60 gpurun_out/r03/gputests.log; exit 1; }
tail -2 gpurun_out/r03/gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03/smoke.log 2>&1 || { tail -20 gpurun_out/r03/smoke.log; exit 1; }
tail -1 gpurun_out/r03/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r03/bench.log 2>&1 || { tail -20 gpurun_out/r03/bench.log; exit 1; }
tail -1 gpurun_out/r03/bench.log | cut -c1-600
timeout -k 10 300 python bench.py --precision fp16 --cpu-seconds 0 > gpurun_out/r03/bench_f16.log 2>&1 || { tail -20 gpurun_out/r03/bench_f16.log; exit 1; }
tail -1 gpurun_out/r03/bench_f16.log | cut -c1-600

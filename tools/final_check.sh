R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/final
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/gputests.log 2>&1 || { tail -40 gpurun_out/final/gputests.log; exit 1; }
tail -2 gpurun_out/final/gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/final/bench.log 2>&1 || { tail -20 gpurun_out/final/bench.log; exit 1; }
tail -1 gpurun_out/final/bench.log | cut -c1-400
timeout -k 10 300 python bench.py --dist --cpu-seconds 0 > gpurun_out/final/dist.log 2>&1 || { tail -20 gpurun_out/final/dist.log; exit 1; }
tail -1 gpurun_out/final/dist.log | cut -c1-300

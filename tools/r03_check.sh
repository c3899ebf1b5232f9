# GPU suite + the config parity cases with their printed reports (run through gpurun)
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/gputests.log 2>&1 || { tail -40 gpurun_out/r03/gputests.log; exit 1; }
tail -2 gpurun_out/r03/gputests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r03/configs.log 2>&1 || { tail -40 gpurun_out/r03/configs.log; exit 1; }
grep -E "image|rel err|passed|failed" gpurun_out/r03/configs.log

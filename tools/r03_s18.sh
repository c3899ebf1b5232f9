# predict chain tests (near-tie order rule)
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_image.py -x -q -k "predict_vs_oracle_chain" --timeout 200 --timeout-method thread > gpurun_out/r03/pred.log 2>&1 || grep -E "^E  " gpurun_out/r03/pred.log | head -4 | cut -c1-600
tail -1 gpurun_out/r03/pred.log

# side configs on the tile-50 build: fp16 (north_star 1e-3 mode) and bf16 bs 64
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 300 python bench.py --cpu-seconds 0 --precision fp16 > gpurun_out/r03/side_fp16_s44.log 2>&1 || { tail -20 gpurun_out/r03/side_fp16_s44.log; exit 1; }
tail -1 gpurun_out/r03/side_fp16_s44.log | cut -c1-160
timeout -k 10 300 python bench.py --cpu-seconds 0 --batch 64 > gpurun_out/r03/side_b64_s44.log 2>&1 || { tail -20 gpurun_out/r03/side_b64_s44.log; exit 1; }
tail -1 gpurun_out/r03/side_b64_s44.log | cut -c1-160

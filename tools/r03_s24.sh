# fp8 parity after the packed epilogue; C4 1280 bs 8 kernel stats (NMS share)
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03/c4prof
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_fp8.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/s24_fp8.log 2>&1 || { grep -E "^E  |FAILED" gpurun_out/r03/s24_fp8.log | head -10; exit 1; }
tail -1 gpurun_out/r03/s24_fp8.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03/c4prof -o run --output-format csv -- python3 $R/bench.py --size 1280 --batch 8 --cpu-seconds 0 --image-in-steps 0 > $R/gpurun_out/r03/c4prof/bench.log 2>&1 || { tail -5 $R/gpurun_out/r03/c4prof/bench.log; exit 1; }
tail -1 $R/gpurun_out/r03/c4prof/bench.log | cut -c1-200
find $R/gpurun_out/r03/c4prof -name "*kernel_stats.csv" | head -2

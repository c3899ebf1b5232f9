# band halo tiles 48 / 49 (40-wide maps): parity, then the yolov7 40^2 3x3 shapes vs tile 16
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "halo" --timeout 120 --timeout-method thread > gpurun_out/r03/s26_tests.log 2>&1 || { grep -E "^E  |FAILED" gpurun_out/r03/s26_tests.log | head -10; exit 1; }
tail -1 gpurun_out/r03/s26_tests.log
X="32,40,40,128,128,3,1;32,40,40,256,128,3,1;32,40,40,256,256,3,1;32,40,40,256,512,3,1"
CONV_EXTRA="$X" CONV_SHAPES=28,29,30,31 timeout -k 10 300 python3 tests/probes/conv_bench.py 16 48 49 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03/band.log

# tiles 41-43 parity + isolation table vs tile 16; nms per-wave search profile
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "big or bf16_tiles or fp16_tiles" --timeout 200 --timeout-method thread > gpurun_out/r03/tiles_tests.log 2>&1 || { tail -30 gpurun_out/r03/tiles_tests.log; exit 1; }
tail -1 gpurun_out/r03/tiles_tests.log
CONV_SHAPES=0,1,2,5,10,12,14,15,16,18,20,22,23,26,27 timeout -k 10 300 python tests/probes/conv_bench.py 16 41 42 43 > gpurun_out/r03/conv_bigt.log 2>&1 || { tail -20 gpurun_out/r03/conv_bigt.log; exit 1; }
cat gpurun_out/r03/conv_bigt.log
timeout -k 10 120 python tests/probes/nms_phases.py || exit 1

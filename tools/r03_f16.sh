# fp16 plan: kernel + model + C2 parity, then its bench line; tile 40 tests + isolation table
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "fp16 or big or bf16_tiles" --timeout 200 --timeout-method thread > gpurun_out/r03/f16_kernels.log 2>&1 || { tail -30 gpurun_out/r03/f16_kernels.log; exit 1; }
tail -1 gpurun_out/r03/f16_kernels.log
CONV_SHAPES=0,2,14,15,16,20,26,8,18,12 timeout -k 10 300 python tests/probes/conv_bench.py 16 40 > gpurun_out/r03/big40.log 2>&1 || { tail -20 gpurun_out/r03/big40.log; exit 1; }
cat gpurun_out/r03/big40.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py -x -q -s -k "fp16" --timeout 300 --timeout-method thread > gpurun_out/r03/f16_model.log 2>&1 || { grep -E "rel err|Error|assert" gpurun_out/r03/f16_model.log | tail -30; exit 1; }
grep -E "decoded|G2|passed|failed" gpurun_out/r03/f16_model.log | tail -20
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -q -s -k "fp16" --timeout 300 --timeout-method thread > gpurun_out/r03/f16_c2.log 2>&1 || { grep -E "rel err|Error|assert|image" gpurun_out/r03/f16_c2.log | tail -30; exit 1; }
grep -E "rel err|image|passed|failed" gpurun_out/r03/f16_c2.log
timeout -k 10 300 python bench.py --precision fp16 --cpu-seconds 0 > gpurun_out/r03/bench_f16.log 2>&1 || { tail -20 gpurun_out/r03/bench_f16.log; exit 1; }
tail -1 gpurun_out/r03/bench_f16.log | cut -c1-700

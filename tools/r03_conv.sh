# conv tile experiments: tile 16 (128x128x64, 2 blocks/CU) vs tile 40 (256x256x32, 4-stage, 1 block/CU)
# in isolation, then the XCD region map (YCX_GLDS_GC) on isolated layers and in the bench
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "big or bf16_tiles or fp16_tiles" --timeout 200 --timeout-method thread > gpurun_out/r03/tiles_tests.log 2>&1 || { tail -30 gpurun_out/r03/tiles_tests.log; exit 1; }
tail -1 gpurun_out/r03/tiles_tests.log
CONV_SHAPES=0,2,5,10,12,14,16,18,20,22,23,26,27 timeout -k 10 300 python tests/probes/conv_bench.py 16 40 41 42 43 > gpurun_out/r03/conv_16_40.log 2>&1 || { tail -20 gpurun_out/r03/conv_16_40.log; exit 1; }
cat gpurun_out/r03/conv_16_40.log
for gc in 0 2 4; do
  echo "gc=$gc"
  YCX_GLDS_GC=$gc CONV_SHAPES=5,14,20,22,26 timeout -k 10 120 python tests/probes/conv_bench.py 16 || exit 1
done > gpurun_out/r03/gc_layers.log 2>&1
cat gpurun_out/r03/gc_layers.log
for gc in 0 2 4 0 2 4; do
  YCX_GLDS_GC=$gc timeout -k 10 200 python bench.py --cpu-seconds 0 --latency-steps 0 > gpurun_out/r03/gc_b$gc.log 2>&1 || exit 1
  tail -1 gpurun_out/r03/gc_b$gc.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('gc=$gc', d['value'], d['ms_per_step'], d['roofline']['forward_kernel_ms'], d['roofline']['avg_launch_ms'])"
done

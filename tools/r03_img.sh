# image-in leg + batched letterbox test + big-tile isolation table
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_image.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03/img_tests.log 2>&1 || { tail -30 gpurun_out/r03/img_tests.log; exit 1; }
tail -1 gpurun_out/r03/img_tests.log
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/r03/bench_img.log 2>&1 || { tail -20 gpurun_out/r03/bench_img.log; exit 1; }
tail -1 gpurun_out/r03/bench_img.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: v for k, v in d.items() if k in ('value','ms_per_step','p50_ms_unloaded','value_image_in','ms_per_step_image_in','p50_ms_image_in_unloaded')})"
CONV_SHAPES=0,1,2,5,14,15,16,20,22,26,27,12 timeout -k 10 300 python tests/probes/conv_bench.py 0 16 24 25 26 > gpurun_out/r03/bigtiles.log 2>&1 || { tail -20 gpurun_out/r03/bigtiles.log; exit 1; }
cat gpurun_out/r03/bigtiles.log

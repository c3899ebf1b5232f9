# A/B: every big class through the three-launch wide path (split search) vs the LDS fast path; fp16 predict at 640
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_image.py -q -s -k "predict" --timeout 200 --timeout-method thread > gpurun_out/r03/predict.log 2>&1 || { tail -30 gpurun_out/r03/predict.log; }
grep -E "fp16 predict|passed|failed" gpurun_out/r03/predict.log
YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_nofast.so timeout -k 10 300 python -u -m pytest tests/test_gpu_post.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03/nofast_post.log 2>&1 || { tail -30 gpurun_out/r03/nofast_post.log; exit 1; }
tail -1 gpurun_out/r03/nofast_post.log
for v in fast nofast fast nofast; do
  lib=$R/yolo-continuous_amd/ycx/libycx_hip.so; [ $v = nofast ] && lib=$R/yolo-continuous_amd/ycx/libycx_nofast.so
  YCX_LIB=$lib timeout -k 10 200 python bench.py --cpu-seconds 0 --latency-steps 20 > gpurun_out/r03/ab.log 2>&1 || exit 1
  tail -1 gpurun_out/r03/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['p50_ms_unloaded'])"
done

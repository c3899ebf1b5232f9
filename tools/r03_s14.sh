# nms_prep with loads in flight: NMS parity, post time, bench
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_post.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03/nms_post.log 2>&1 || { tail -40 gpurun_out/r03/nms_post.log; exit 1; }
tail -1 gpurun_out/r03/nms_post.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -q -s --timeout 300 --timeout-method thread -k "keep" > gpurun_out/r03/nms_configs.log 2>&1 || { grep -E "image|Error|assert" gpurun_out/r03/nms_configs.log | tail -30; exit 1; }
grep -E "image [0-9]+:|passed|failed" gpurun_out/r03/nms_configs.log | cut -c1-200
YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_hip.so timeout -k 10 120 python tests/probes/nms_phases.py || exit 1
for i in 1 2; do
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/r03/b14.log 2>&1 || { tail -20 gpurun_out/r03/b14.log; exit 1; }
tail -1 gpurun_out/r03/b14.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_ms_unloaded'])"
done

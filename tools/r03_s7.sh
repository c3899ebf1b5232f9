# NMS radix rank sort (fast path) + nms_wide (large classes): parity, phase profile, C4 side bench
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_post.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03/nms_post.log 2>&1 || { tail -40 gpurun_out/r03/nms_post.log; exit 1; }
tail -1 gpurun_out/r03/nms_post.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r03/nms_configs.log 2>&1 || { grep -E "image|Error|assert" gpurun_out/r03/nms_configs.log | tail -30; exit 1; }
grep -E "image [0-9]+:|passed|failed" gpurun_out/r03/nms_configs.log | cut -c1-300
timeout -k 10 120 python tests/probes/nms_phases.py > gpurun_out/r03/nms_phases.log 2>&1 || { tail -5 gpurun_out/r03/nms_phases.log; exit 1; }
cat gpurun_out/r03/nms_phases.log
YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_hip.so timeout -k 10 120 python tests/probes/nms_phases.py || exit 1
timeout -k 10 300 python bench.py --size 1280 --batch 8 --cpu-seconds 0 > gpurun_out/r03/side_c4.log 2>&1 || { tail -20 gpurun_out/r03/side_c4.log; exit 1; }
tail -1 gpurun_out/r03/side_c4.log | cut -c1-300

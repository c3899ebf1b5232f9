# new LDS-resident nms_big fast path: post + config parity, phase profile (new vs old), bench
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_post.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03/nms_post.log 2>&1 || { tail -40 gpurun_out/r03/nms_post.log; exit 1; }
tail -1 gpurun_out/r03/nms_post.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r03/nms_configs.log 2>&1 || { grep -E "image|Error|assert" gpurun_out/r03/nms_configs.log | tail -30; exit 1; }
grep -E "image [0-9]+:|passed|failed" gpurun_out/r03/nms_configs.log | cut -c1-300
echo "--- new"; timeout -k 10 120 python tests/probes/nms_phases.py || exit 1
echo "--- old"; YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_hip_prof_old.so timeout -k 10 120 python tests/probes/nms_phases.py || exit 1
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/r03/bench_nms.log 2>&1 || { tail -20 gpurun_out/r03/bench_nms.log; exit 1; }
tail -1 gpurun_out/r03/bench_nms.log | cut -c1-400

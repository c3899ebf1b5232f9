# nms fast path v2 (32 u16 slots): post parity + configs, phase profile, bench; then the conv tile experiments
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_post.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03/nms_post.log 2>&1 || { tail -40 gpurun_out/r03/nms_post.log; exit 1; }
tail -1 gpurun_out/r03/nms_post.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r03/nms_configs.log 2>&1 || { grep -E "image|Error|assert" gpurun_out/r03/nms_configs.log | tail -30; exit 1; }
grep -E "image [0-9]+:|passed|failed" gpurun_out/r03/nms_configs.log | cut -c1-300
echo "--- new"; timeout -k 10 120 python tests/probes/nms_phases.py || exit 1
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/r03/bench_nms.log 2>&1 || { tail -20 gpurun_out/r03/bench_nms.log; exit 1; }
tail -1 gpurun_out/r03/bench_nms.log | cut -c1-300
bash tools/r03_conv.sh

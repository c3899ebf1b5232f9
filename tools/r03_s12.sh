# conv_bigt DMA-issue placement (tiles 44-47) vs 16 / 41 / 40: parity, isolation, stamps
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "big_tile" --timeout 200 --timeout-method thread > gpurun_out/r03/tiles_tests.log 2>&1 || { tail -30 gpurun_out/r03/tiles_tests.log; exit 1; }
tail -1 gpurun_out/r03/tiles_tests.log
CONV_SHAPES=0,2,5,12,14,16,18,20,26 timeout -k 10 300 python tests/probes/conv_bench.py 16 41 44 45 46 40 47 > gpurun_out/r03/conv_dpos.log 2>&1 || { tail -20 gpurun_out/r03/conv_dpos.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03/conv_dpos.log
for t in 44 46; do
  YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_stamp.so timeout -k 10 200 python tests/probes/glds_stamps.py $t 0 14 || exit 1
done 2>&1 | grep -v amdgpu.ids
# three-launch wide path (nms_wide_a / _s / _b): parity at C4 and the wide tests, C4 NMS timing
timeout -k 10 300 python -u -m pytest tests/test_gpu_post.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03/nms_post.log 2>&1 || { tail -40 gpurun_out/r03/nms_post.log; exit 1; }
tail -1 gpurun_out/r03/nms_post.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -q -s --timeout 300 --timeout-method thread -k "c4" > gpurun_out/r03/nms_configs.log 2>&1 || { grep -E "image|Error|assert" gpurun_out/r03/nms_configs.log | tail -30; exit 1; }
grep -E "image [0-9]+:|passed|failed" gpurun_out/r03/nms_configs.log | cut -c1-200
NMS_PROBE_ARGS="--size 1280 --batch 8" YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_hip.so timeout -k 10 200 python tests/probes/nms_phases.py 2>&1 | grep -E "post ms" || exit 1
timeout -k 10 300 python bench.py --size 1280 --batch 8 --cpu-seconds 0 > gpurun_out/r03/side_c4.log 2>&1 || { tail -20 gpurun_out/r03/side_c4.log; exit 1; }
tail -1 gpurun_out/r03/side_c4.log | cut -c1-200

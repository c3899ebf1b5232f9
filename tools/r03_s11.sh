# per-phase stamps: tile 16 vs conv_bigt tiles 41 / 42 / 43; then the wide-path radix (striped) parity + C4 NMS profile
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
for t in 16 41 42 43; do
  YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_stamp.so timeout -k 10 200 python tests/probes/glds_stamps.py $t 0 14 26 || exit 1
done > gpurun_out/r03/stamps_tiles.log 2>&1
grep -v amdgpu.ids gpurun_out/r03/stamps_tiles.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_post.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03/nms_post.log 2>&1 || { tail -40 gpurun_out/r03/nms_post.log; exit 1; }
tail -1 gpurun_out/r03/nms_post.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -q -s --timeout 300 --timeout-method thread -k "c4" > gpurun_out/r03/nms_configs.log 2>&1 || { grep -E "image|Error|assert" gpurun_out/r03/nms_configs.log | tail -30; exit 1; }
grep -E "image [0-9]+:|passed|failed" gpurun_out/r03/nms_configs.log | cut -c1-200
NMS_PROBE_ARGS="--size 1280 --batch 8" timeout -k 10 200 python tests/probes/nms_phases.py 2>&1 | grep -E "post ms|nms_wide" || exit 1

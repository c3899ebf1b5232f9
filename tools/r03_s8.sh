# single-launch fast path + split task lists: NMS parity; C4 side bench + kernel stats, nms_wide vs the r02 general path
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_post.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03/nms_post.log 2>&1 || { tail -40 gpurun_out/r03/nms_post.log; exit 1; }
tail -1 gpurun_out/r03/nms_post.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -q -s --timeout 300 --timeout-method thread -k "c4 or c2_bs32_forward or c2_bs32_keep" > gpurun_out/r03/nms_configs.log 2>&1 || { grep -E "image|Error|assert" gpurun_out/r03/nms_configs.log | tail -30; exit 1; }
grep -E "image [0-9]+:|passed|failed" gpurun_out/r03/nms_configs.log | cut -c1-200
YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_hip.so timeout -k 10 120 python tests/probes/nms_phases.py || exit 1
cd /tmp && export TMPDIR=/tmp
for v in new oldbig; do
  lib=$R/yolo-continuous_amd/ycx/libycx_hip.so; [ $v = oldbig ] && lib=$R/yolo-continuous_amd/ycx/libycx_hip_oldbig.so
  YCX_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03/c4_$v -o run --output-format csv -- python3 $R/bench.py --size 1280 --batch 8 --cpu-seconds 0 --steps 40 > $R/gpurun_out/r03/c4_$v.log 2>&1 || exit 1
  tail -1 $R/gpurun_out/r03/c4_$v.log | cut -c1-160
done
cd $R
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/r03/bench_s8.log 2>&1 || { tail -20 gpurun_out/r03/bench_s8.log; exit 1; }
tail -1 gpurun_out/r03/bench_s8.log | cut -c1-200

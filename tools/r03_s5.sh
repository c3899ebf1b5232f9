# NMS profile (fixed instrumentation) + release post time; chunked-prefix experiment
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 120 python tests/probes/nms_phases.py || exit 1
YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_hip.so timeout -k 10 120 python tests/probes/nms_phases.py || exit 1
YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_hip_prof_old.so timeout -k 10 120 python tests/probes/nms_phases.py | head -2 || exit 1
bash tools/r03_chunk.sh

# NMS phase counters at C4 (1280 bs 8) with the prof library
R=$GRAFT_REPO_ROOT
cd $R
NMS_PROBE_ARGS="--size 1280 --batch 8" YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_hip_prof.so timeout -k 10 200 python tests/probes/nms_phases.py 2>&1 | grep -v amdgpu.ids

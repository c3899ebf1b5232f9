# glds tile-16 per-phase stamps (where a K step's cycles go) on four yolov7 shapes
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_stamp.so timeout -k 10 200 python tests/probes/glds_stamps.py 16 0 14 2 26 12 > gpurun_out/r03/glds_stamps.log 2>&1 || { tail -20 gpurun_out/r03/glds_stamps.log; exit 1; }
cat gpurun_out/r03/glds_stamps.log

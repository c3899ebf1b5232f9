cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04
for v in hip w8 f4 w8f4 f10; do echo "== $v"; YCX_LIB=$PWD/yolo-continuous_amd/ycx/libycx_$v.so timeout -k 10 120 python tests/probes/stem2_bench.py fused fused_old || exit 1; done

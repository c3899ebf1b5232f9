# fp8 weight-resident 1x1 without its output stores (timing only): are the stores the bound?
R=$GRAFT_REPO_ROOT
cd $R
for v in hip f8nost; do
echo "== $v"; YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_$v.so OP_TOP=60 timeout -k 10 200 python tests/probes/op_times.py --precision fp8 --batch 64 2>&1 | grep -v amdgpu.ids | grep -E "wres|forward" | head -6
done

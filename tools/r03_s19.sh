# stem2_fused time split: act / conv / stem phases removed one at a time (timing-only variant libs)
R=$GRAFT_REPO_ROOT
cd $R
for v in hip s2na1 s2na2 s2nact s2nconv s2nstem; do
echo -n "$v: "; YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_$v.so timeout -k 10 120 python tests/probes/stem2_bench.py fused 2>&1 | grep -v amdgpu.ids | tail -1
done

# stem2_fused A/B on one box: HEAD (s2base), packed SiLU + column order without reuse (s2noreuse), with reuse (hip)
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2 3; do for v in s2base s2noreuse hip; do
echo -n "$v: "; YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_$v.so timeout -k 10 120 python tests/probes/stem2_bench.py fused 2>&1 | grep -v amdgpu.ids | tail -1
done; done

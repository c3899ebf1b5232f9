# fp8 weight-resident 1x1 ring depth / pixels per wave: per-op serial times (fp8 bs64), then C5 bench
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
for v in hip f8ns8 f8ns12 f8tpw128; do
echo "== $v"; YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_$v.so OP_TOP=60 timeout -k 10 200 python tests/probes/op_times.py --precision fp8 --batch 64 2>&1 | grep -v amdgpu.ids | grep -E "wres|forward" 
done
for v in hip f8ns12 hip f8ns12; do
YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_$v.so timeout -k 10 300 python bench.py --cpu-seconds 0 --image-in-steps 0 --precision fp8 --batch 64 > gpurun_out/r03/b39.log 2>&1 || { tail -20 gpurun_out/r03/b39.log; exit 1; }
echo -n "C5 $v "; tail -1 gpurun_out/r03/b39.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done

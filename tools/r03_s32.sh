# nms_prep class phase on 1 / 4 / 16 workgroups per image (count/bucket on 16) vs HEAD: C2 post ms and bench, C4 bench
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
for v in base pb1 pb4 hip; do echo -n "$v "; YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_$v.so timeout -k 10 120 python bench.py --post-micro --obj-shift 0 2>&1 | grep -v amdgpu | tail -1 | cut -c1-160; done
for v in base pb1 pb4; do
YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_$v.so timeout -k 10 300 python bench.py --cpu-seconds 0 --image-in-steps 0 > gpurun_out/r03/b32.log 2>&1 || { tail -20 gpurun_out/r03/b32.log; exit 1; }
echo -n "C2 $v "; tail -1 gpurun_out/r03/b32.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_ms_unloaded'])"
done
for v in base pb1 pb4; do
YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_$v.so timeout -k 10 300 python bench.py --cpu-seconds 0 --image-in-steps 0 --size 1280 --batch 8 > gpurun_out/r03/b32.log 2>&1 || { tail -20 gpurun_out/r03/b32.log; exit 1; }
echo -n "C4 $v "; tail -1 gpurun_out/r03/b32.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_ms_unloaded'])"
done

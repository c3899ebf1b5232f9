# tile 50 halo ring depth: parity at NB 4 (product build), isolated timing NB 2/3/4, bench A/B
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "conv3x3s2" --timeout 120 --timeout-method thread > gpurun_out/r03/s2wsr_kernels.log 2>&1 || { tail -40 gpurun_out/r03/s2wsr_kernels.log; exit 1; }
tail -1 gpurun_out/r03/s2wsr_kernels.log
L=yolo-continuous_amd/ycx
CONV_EXTRA="64,320,320,64,128,3,2" CONV_SHAPES=10,28 timeout -k 10 200 python3 tests/probes/conv_ab.py $L/libycx_hip.so $L/libycx_nb2.so $L/libycx_nb3.so --tile 50 --shapes 10,28 > gpurun_out/r03/s2wsr_ab.log 2>&1 || { tail -20 gpurun_out/r03/s2wsr_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03/s2wsr_ab.log
for v in hip nb2 hip nb2; do
YCX_LIB=$R/$L/libycx_$v.so timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/r03/b50.log 2>&1 || { tail -20 gpurun_out/r03/b50.log; exit 1; }
echo -n "$v "; tail -1 gpurun_out/r03/b50.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_ms_unloaded'], d['roofline'].get('forward_kernel_ms'))"
done
echo done

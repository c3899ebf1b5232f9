# tile 50 (3x3/s2 64->128, weights in registers): kernel parity, isolated timing vs tile 16, bench A/B
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "s2_wsr or conv3x3s2" --timeout 120 --timeout-method thread > gpurun_out/r03/s2wsr_kernels.log 2>&1 || { tail -40 gpurun_out/r03/s2wsr_kernels.log; exit 1; }
tail -1 gpurun_out/r03/s2wsr_kernels.log
CONV_EXTRA="64,320,320,64,128,3,2" CONV_SHAPES=10,28 timeout -k 10 200 python3 tests/probes/conv_bench.py 16 50 > gpurun_out/r03/s2wsr_bench.log 2>&1 || { tail -20 gpurun_out/r03/s2wsr_bench.log; exit 1; }
cat gpurun_out/r03/s2wsr_bench.log | grep -v amdgpu.ids
for v in 0 1 0 1; do
YCX_NO_S2WSR=$v timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/r03/b50.log 2>&1 || { tail -20 gpurun_out/r03/b50.log; exit 1; }
echo -n "NO_S2WSR=$v "; tail -1 gpurun_out/r03/b50.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_ms_unloaded'], d['roofline'].get('forward_kernel_ms'))"
done
echo done

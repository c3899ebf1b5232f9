# fp8 ws64 epilogue (permuted rows, 8-byte stores): fp8 parity, C5 configs, C5 bench A/B vs HEAD
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_configs.py -x -q -k "not c4" --timeout 400 --timeout-method thread > gpurun_out/r03/s37.log 2>&1 || { grep -E "^E  |FAILED" gpurun_out/r03/s37.log | head -10; exit 1; }
tail -1 gpurun_out/r03/s37.log
for v in base hip base hip; do
YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_$v.so timeout -k 10 300 python bench.py --cpu-seconds 0 --image-in-steps 0 --precision fp8 --batch 64 > gpurun_out/r03/b37.log 2>&1 || { tail -20 gpurun_out/r03/b37.log; exit 1; }
echo -n "C5 $v "; tail -1 gpurun_out/r03/b37.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done

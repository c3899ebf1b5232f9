# band tile 48 in the auto pick: C2 full-keep parity, bench A/B vs HEAD (libycx_base)
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -x -q -k "c2" --timeout 400 --timeout-method thread > gpurun_out/r03/s27_tests.log 2>&1 || { grep -E "^E  |FAILED" gpurun_out/r03/s27_tests.log | head -10; exit 1; }
tail -1 gpurun_out/r03/s27_tests.log
for v in base hip base hip; do
YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_$v.so timeout -k 10 300 python bench.py --cpu-seconds 0 --image-in-steps 0 > gpurun_out/r03/b27.log 2>&1 || { tail -20 gpurun_out/r03/b27.log; exit 1; }
echo -n "$v "; tail -1 gpurun_out/r03/b27.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_ms_unloaded'])"
done

# f32 predict chain failure details (x2 for determinism), then bench SK on/off
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
for i in 1 2; do
timeout -k 10 300 python -u -m pytest tests/test_gpu_image.py -x -q -k "predict_vs_oracle_chain and f32" --timeout 200 --timeout-method thread > gpurun_out/r03/pred.log 2>&1 || grep -E "^E  " gpurun_out/r03/pred.log | head -8
tail -1 gpurun_out/r03/pred.log
done
for sk in 1 0 1 0; do
YCX_SK=$sk timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/r03/b17.log 2>&1 || { tail -20 gpurun_out/r03/b17.log; exit 1; }
echo -n "SK=$sk "; tail -1 gpurun_out/r03/b17.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_ms_unloaded'])"
done

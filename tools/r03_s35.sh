# batches in flight (depth 2 / 3 / 4) on the current kernels, bf16 C2; forward-only diagnostic
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
for dp in 3 4 2 3 4; do
timeout -k 10 300 python bench.py --cpu-seconds 0 --image-in-steps 0 --depth $dp > gpurun_out/r03/b35.log 2>&1 || { tail -20 gpurun_out/r03/b35.log; exit 1; }
echo -n "depth $dp "; tail -1 gpurun_out/r03/b35.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_ms'], d['p50_ms_unloaded'])"
done
timeout -k 10 300 python bench.py --cpu-seconds 0 --image-in-steps 0 --diag-forward-only > gpurun_out/r03/b35.log 2>&1 || { tail -20 gpurun_out/r03/b35.log; exit 1; }
echo -n "forward only "; tail -1 gpurun_out/r03/b35.log | cut -c1-200

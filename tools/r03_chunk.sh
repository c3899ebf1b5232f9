# image-chunked prefix experiment (YCX_CHUNK): bit-identity test, then the bench A/B
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q -k "chunked" --timeout 200 --timeout-method thread > gpurun_out/r03/chunk_test.log 2>&1 || { tail -30 gpurun_out/r03/chunk_test.log; exit 1; }
tail -1 gpurun_out/r03/chunk_test.log
for c in none 4:@160 8:@160 4:@80 8:@80 none 4:@160 8:@160; do
  if [ $c = none ]; then unset YCX_CHUNK; else export YCX_CHUNK=$c; fi
  timeout -k 10 200 python bench.py --cpu-seconds 0 --latency-steps 0 > gpurun_out/r03/chunk_b.log 2>&1 || exit 1
  tail -1 gpurun_out/r03/chunk_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('chunk=$c', d['value'], d['ms_per_step'])"
done
unset YCX_CHUNK

# fused Detect-head decode: parity tests, then bench A/B (fused vs separate decode_filter)
mkdir -p gpurun_out/r02
timeout -k 10 400 python -u -m pytest tests/test_gpu_post.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r02/t_head.log 2>&1 || { tail -30 gpurun_out/r02/t_head.log; exit 1; }
tail -3 gpurun_out/r02/t_head.log
for v in "" "--no-fuse-heads" "" "--no-fuse-heads"; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 --latency-steps 0 --steps 30 $v > gpurun_out/r02/b_head.log 2>&1 || exit 1
  tail -1 gpurun_out/r02/b_head.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])"
done

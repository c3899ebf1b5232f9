mkdir -p gpurun_out/r02
timeout -k 10 200 python bench.py --cpu-seconds 0 --latency-steps 0 --steps 30 > gpurun_out/r02/b_full.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --cpu-seconds 0 --latency-steps 0 --steps 30 --diag-forward-only > gpurun_out/r02/b_fwd.log 2>&1 || exit 1
for f in gpurun_out/r02/b_full.log gpurun_out/r02/b_fwd.log; do tail -1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['forward_kernel_ms'])"; done

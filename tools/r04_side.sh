cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04
# side configurations with the per-op gap table: fp8 bs 64 (C5), bf16 bs 64, fp16 bs 32
YCX_BENCH_KERNELS=gpurun_out/r04/ops_fp8_b64.json timeout -k 10 300 python bench.py --precision fp8 --batch 64 --cpu-seconds 0 --image-in-steps 0 > gpurun_out/r04/side_fp8_b64.log 2>&1 || exit 1
YCX_BENCH_KERNELS=gpurun_out/r04/ops_bf16_b64.json timeout -k 10 300 python bench.py --batch 64 --cpu-seconds 0 --image-in-steps 0 > gpurun_out/r04/side_b64.log 2>&1 || exit 1
for f in side_fp8_b64 side_b64; do python -c "import json,sys; d=json.loads(open('gpurun_out/r04/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['roofline']['forward_kernel_ms'], d['roofline']['kernel'], d['roofline']['frac'])"; done
python tools/op_gap.py gpurun_out/r04/ops_fp8_b64.json 30 > gpurun_out/r04/op_gap_fp8_b64.md

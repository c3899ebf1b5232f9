cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04
bash tools/r04.sh tests tests/test_gpu_kernels.py -k "pair" tests/test_gpu_model.py -k "pair or plan_properties" tests/test_abi.py > gpurun_out/r04/kt.txt 2>&1; rc=$?; tail -5 gpurun_out/r04/kt.txt; [ $rc = 0 ] || exit $rc
YCX_BENCH_KERNELS=gpurun_out/r04/ops_pair.json timeout -k 10 300 python bench.py --cpu-seconds 0 --image-in-steps 0 > gpurun_out/r04/b1.log 2>&1 || exit 1
YCX_NO_CONV_PAIR=1 timeout -k 10 300 python bench.py --cpu-seconds 0 --image-in-steps 0 > gpurun_out/r04/b0.log 2>&1 || exit 1
YCX_BENCH_KERNELS=gpurun_out/r04/ops_pair2.json timeout -k 10 300 python bench.py --cpu-seconds 0 --image-in-steps 0 > gpurun_out/r04/b2.log 2>&1 || exit 1
for f in b1 b0 b2; do python -c "import json,sys; d=json.loads(open('gpurun_out/r04/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['roofline']['forward_kernel_ms'])"; done

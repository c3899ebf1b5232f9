cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04
# A/B: the current library vs libycx_old.so (the previous commit's conv unit)
bash tools/r04.sh tests tests/test_gpu_kernels.py -k "${AB_TESTS:-ws64 or special}" > gpurun_out/r04/kt.txt 2>&1; rc=$?; tail -2 gpurun_out/r04/kt.txt; [ $rc = 0 ] || exit $rc
for lib in hip old; do
  echo "== $lib"; CONV_SHAPES=${AB_SHAPES:-3,4,13} YCX_LIB=$PWD/yolo-continuous_amd/ycx/libycx_$lib.so timeout -k 10 200 python tests/probes/conv_bench.py ${AB_TILES:-23} || exit 1
done
for i in 1 2; do for lib in hip old; do
  YCX_LIB=$PWD/yolo-continuous_amd/ycx/libycx_$lib.so timeout -k 10 300 python bench.py --cpu-seconds 0 --image-in-steps 0 > gpurun_out/r04/ab_$lib.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/r04/ab_$lib.log').read().strip().splitlines()[-1]); print('$lib', d['value'], d['roofline']['forward_kernel_ms'])"
done; done

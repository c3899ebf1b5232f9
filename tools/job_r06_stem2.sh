# stem2_fused change A/B: A = yolo-continuous_amd/ycx/libycx_A.so (previous source), B = in-tree
mkdir -p gpurun_out/r06
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "stem" > gpurun_out/r06/stem_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r06/stem_tests.log
[ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then export YCX_LIB=$PWD/yolo-continuous_amd/ycx/libycx_A.so; else unset YCX_LIB; fi
    echo "$v $(timeout -k 10 100 python -u tests/probes/stem2_bench.py 2>/dev/null | grep fused)"
  done
done
unset YCX_LIB
bash tools/ab_bench.sh 2>&1 | tail -4

# A/B bench on one box (development tool): A = yolo-continuous_amd/ycx/libycx_A.so, B = the in-tree library.
A=$GRAFT_REPO_ROOT/yolo-continuous_amd/ycx/libycx_A.so
for v in A B A B; do
  if [ $v = A ]; then export YCX_LIB=$A; else unset YCX_LIB; fi
  timeout -k 10 200 python bench.py --cpu-seconds 0 > gpurun_out/ab_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/ab_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['p50_ms'], d['roofline']['forward_kernel_ms'])"
done

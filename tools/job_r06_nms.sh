# C4 wide-class sort: NMS parity tests, same-box bench A/B (A = one-workgroup sort), NMS share under rocprof
mkdir -p gpurun_out/r06/nms
O=$PWD/gpurun_out/r06/nms
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_post.py tests/test_gpu_configs.py -k "nms or c4 or post" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
for v in A B A B; do
  if [ $v = A ]; then export YCX_LIB=$PWD/yolo-continuous_amd/ycx/libycx_A.so; else unset YCX_LIB; fi
  timeout -k 10 300 python bench.py --size 1280 --batch 8 --cpu-seconds 0 --fp16-steps 0 --pipelined-steps 0 --image-in-steps 0 > $O/c4_$v.log 2>&1 || { tail -5 $O/c4_$v.log; exit 1; }
  tail -1 $O/c4_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['detections_last_step'])"
done
unset YCX_LIB
cd /tmp && export TMPDIR=/tmp
for v in A B; do
  if [ $v = A ]; then export YCX_LIB=$GRAFT_REPO_ROOT/yolo-continuous_amd/ycx/libycx_A.so; else unset YCX_LIB; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --size 1280 --batch 8 --cpu-seconds 0 --fp16-steps 0 --pipelined-steps 0 --image-in-steps 0 --steps 40 > $O/prof_$v.log 2>&1 || { tail -5 $O/prof_$v.log; exit 1; }
  echo "== $v"; python3 $GRAFT_REPO_ROOT/tools/nms_share.py $O/prof_$v | tee $O/nms_share_$v.txt
  cp $(find $O/prof_$v -name '*kernel_stats.csv' | head -1) $O/kernel_stats_$v.csv; rm -rf $O/prof_$v
done

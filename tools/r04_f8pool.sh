# fp8 MP-pool fusion (run through gpurun): parity tests, then C5 bench lines with / without the fusion.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04 && O=gpurun_out/r04
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fp8.py \
  tests/test_gpu_model.py -k "pool or fp8" > $O/f8pool_tests.log 2>&1; rc=$?
tail -3 $O/f8pool_tests.log; [ $rc = 0 ] || { grep -E "Error|assert" $O/f8pool_tests.log | head -20; exit $rc; }
for i in 1 2; do for f in 0 1; do
  if [ $f = 1 ]; then export YCX_NO_POOL_FUSE=1; else unset YCX_NO_POOL_FUSE; fi
  timeout -k 10 300 python bench.py --cpu-seconds 0 --image-in-steps 0 --precision fp8 --batch 64 > $O/f8pool_c5.log 2>&1 || exit 1
  python -c "
import json; d=json.loads(open('$O/f8pool_c5.log').read().strip().splitlines()[-1]); print('c5 nofuse=$f', d['value'], d['roofline'].get('forward_kernel_ms'))"
done; done

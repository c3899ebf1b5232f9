# A/B of two libraries (run through gpurun): AB_A / AB_B library names under ycx/, C2 and C4 bench lines.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04 && O=gpurun_out/r04
L=$PWD/yolo-continuous_amd/ycx
if [ -n "$AB_TESTS" ]; then
  YCX_LIB=$L/libycx_$AB_A.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread $AB_TESTS > $O/ab2_tests.log 2>&1; rc=$?
  tail -2 $O/ab2_tests.log; [ $rc = 0 ] || exit $rc
fi
for i in 1 2; do for lib in $AB_A $AB_B; do for c in ${AB_CONFIGS:-c2 c4}; do
  args=""; [ $c = c4 ] && args="--size 1280 --batch 8"; [ $c = c5 ] && args="--precision fp8 --batch 64"
  YCX_LIB=$L/libycx_$lib.so timeout -k 10 300 python bench.py --cpu-seconds 0 --image-in-steps 0 $args > $O/ab2_$c.log 2>&1 || exit 1
  python -c "
import json; d=json.loads(open('$O/ab2_$c.log').read().strip().splitlines()[-1]); print('$c', '$lib', d['value'], d['p50_ms'], d['p50_ms_unloaded'])"
done; done; done
if [ -n "$AB_MICRO" ]; then for lib in $AB_A $AB_B; do for sh in -3 0; do
  YCX_LIB=$L/libycx_$lib.so timeout -k 10 300 python bench.py --post-micro --obj-shift $sh > $O/ab2_micro.log 2>&1 || exit 1
  python -c "
import json; d=json.loads(open('$O/ab2_micro.log').read().strip().splitlines()[-1]); print('micro shift $sh', '$lib', d['value'], d.get('ms_per_step'))"
done; done; fi

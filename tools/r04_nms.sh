# NMS split A/B (run through gpurun): parity tests, then C4 / C2 bench lines and post timing
# with the current library vs libycx_old.so (the previous commit's build).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04 && O=gpurun_out/r04
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_post.py \
  tests/test_gpu_configs.py -k "nms or c4 or c2 or keep or post" > $O/nms_tests.log 2>&1; rc=$?
tail -3 $O/nms_tests.log; [ $rc = 0 ] || { tail -40 $O/nms_tests.log; exit $rc; }
for lib in hip old; do
  echo "== $lib"
  NMS_PROBE_ARGS="--size 1280 --batch 8" YCX_LIB=$PWD/yolo-continuous_amd/ycx/libycx_$lib.so timeout -k 10 200 python tests/probes/nms_phases.py 2>&1 | grep -E "post ms|release" || exit 1
  NMS_PROBE_ARGS="" YCX_LIB=$PWD/yolo-continuous_amd/ycx/libycx_$lib.so timeout -k 10 200 python tests/probes/nms_phases.py 2>&1 | grep -E "post ms|release" || exit 1
done
NMS_PROBE_ARGS="--size 1280 --batch 8" timeout -k 10 200 python tests/probes/nms_phases.py 2>&1 | tail -12
for i in ${AB_REPS:-1 2}; do for lib in hip old; do
  YCX_LIB=$PWD/yolo-continuous_amd/ycx/libycx_$lib.so timeout -k 10 300 python bench.py --cpu-seconds 0 --image-in-steps 0 --size 1280 --batch 8 > $O/nab_c4_$lib.log 2>&1 || exit 1
  YCX_LIB=$PWD/yolo-continuous_amd/ycx/libycx_$lib.so timeout -k 10 300 python bench.py --cpu-seconds 0 --image-in-steps 0 > $O/nab_c2_$lib.log 2>&1 || exit 1
  python -c "
import json
for c in ('c4','c2'):
    d=json.loads(open('$O/nab_'+c+'_$lib.log').read().strip().splitlines()[-1]); print(c, '$lib', d['value'], d['p50_ms'], d['p50_ms_unloaded'])"
done; done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/nms_c4 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-seconds 0 --image-in-steps 0 --size 1280 --batch 8 --steps 40 > $GRAFT_REPO_ROOT/$O/nms_c4.log 2>&1

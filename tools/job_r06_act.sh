# tile timings: previous conv source (act 1) vs this one (act 1, act 3 = YCX_ACT_SILU_PS), interleaved
mkdir -p gpurun_out/r06
O=gpurun_out/r06/act_ab.txt; : > $O
for r in 1 2; do
  for v in OLD:1 NEW:1 NEW:3; do
    lib=${v%%:*}; act=${v##*:}
    if [ $lib = OLD ]; then export YCX_LIB=$PWD/yolo-continuous_amd/ycx/libycx_OLD.so; else unset YCX_LIB; fi
    echo "== $lib act $act" >> $O
    CONV_ACT=$act CONV_SHAPES=0,2,14,15,3,1 timeout -k 10 120 python -u tests/probes/conv_bench.py 16 22 23 19 >> $O 2>&1 || exit 1
  done
done
unset YCX_LIB
grep -v amdgpu $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06/gputests2.log 2>&1; tail -3 gpurun_out/r06/gputests2.log

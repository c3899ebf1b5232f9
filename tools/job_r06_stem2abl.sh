# stem2_fused ablation timings (development builds: phases / activations switched off), isolated
mkdir -p gpurun_out/r06
for r in 1 2; do
  for v in hip nostem noconv noact1 noact2 noact; do
    export YCX_LIB=$PWD/yolo-continuous_amd/ycx/libycx_$v.so
    echo "$v $(timeout -k 10 100 python -u tests/probes/stem2_bench.py 2>/dev/null | grep fused)"
  done
done

# A/B of the XCD region map (YCX_GLDS_GC) on the LDS-DMA conv tiles: isolated layers, then the bench
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
for gc in 0 2 4 8; do
  echo "gc=$gc"
  YCX_GLDS_GC=$gc CONV_SHAPES=0,2,5,14,16,20,22,26,27,21 timeout -k 10 120 python tests/probes/conv_bench.py 0 || exit 1
done > gpurun_out/r03/gc_layers.log 2>&1
cat gpurun_out/r03/gc_layers.log
for gc in 0 2 4 0 2 4; do
  YCX_GLDS_GC=$gc timeout -k 10 200 python bench.py --cpu-seconds 0 --latency-steps 0 > gpurun_out/r03/gc_b$gc.log 2>&1 || exit 1
  tail -1 gpurun_out/r03/gc_b$gc.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('gc=$gc', d['value'], d['ms_per_step'], d['roofline']['forward_kernel_ms'], d['roofline']['avg_launch_ms'])"
done

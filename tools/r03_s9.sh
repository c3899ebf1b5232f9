# full GPU suite + smoke; NMS phase profiles at C2 and C4; bench lines (bf16 default, fp16, C4)
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r03/gputests2.log 2>&1 || { tail -60 gpurun_out/r03/gputests2.log; exit 1; }
tail -1 gpurun_out/r03/gputests2.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03/smoke2.log 2>&1 || { tail -20 gpurun_out/r03/smoke2.log; exit 1; }
tail -1 gpurun_out/r03/smoke2.log
timeout -k 10 120 python tests/probes/nms_phases.py > gpurun_out/r03/nms_phases_c2.log 2>&1 || exit 1
NMS_PROBE_ARGS="--size 1280 --batch 8" timeout -k 10 200 python tests/probes/nms_phases.py > gpurun_out/r03/nms_phases_c4.log 2>&1 || exit 1
cat gpurun_out/r03/nms_phases_c2.log gpurun_out/r03/nms_phases_c4.log
for a in "" "--precision fp16" "--size 1280 --batch 8" "--precision fp8 --batch 64" "--batch 64"; do
  timeout -k 10 300 python bench.py --cpu-seconds 0 $a > gpurun_out/r03/b.log 2>&1 || { tail -5 gpurun_out/r03/b.log; exit 1; }
  tail -1 gpurun_out/r03/b.log > "gpurun_out/r03/side_$(echo $a | tr -d ' -')x.json"
  tail -1 gpurun_out/r03/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a', d['value'], d['ms_per_step'], d['p50_ms_unloaded'], d['roofline']['frac'], d['roofline']['forward_kernel_ms'])"
done

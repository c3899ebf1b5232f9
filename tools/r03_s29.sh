# nms_wide_a's work inside the nms_fast launch: NMS parity (post + C2/C4/C5 keep), C2 post ms, C4 + C2 bench A/B vs HEAD
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_post.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03/s29_post.log 2>&1 || { grep -E "^E  |FAILED" gpurun_out/r03/s29_post.log | head -10; exit 1; }
tail -1 gpurun_out/r03/s29_post.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r03/s29_cfg.log 2>&1 || { grep -E "^E  |FAILED" gpurun_out/r03/s29_cfg.log | head -10; exit 1; }
tail -1 gpurun_out/r03/s29_cfg.log
for v in base hip; do echo -n "$v "; YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_$v.so timeout -k 10 120 python tests/probes/nms_phases.py 2>&1 | grep "post ms"; done
for v in base hip base hip; do
YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_$v.so timeout -k 10 300 python bench.py --cpu-seconds 0 --image-in-steps 0 --size 1280 --batch 8 > gpurun_out/r03/b29.log 2>&1 || { tail -20 gpurun_out/r03/b29.log; exit 1; }
echo -n "C4 $v "; tail -1 gpurun_out/r03/b29.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_ms_unloaded'])"
done
for v in base hip; do
YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_$v.so timeout -k 10 300 python bench.py --cpu-seconds 0 --image-in-steps 0 > gpurun_out/r03/b29.log 2>&1 || { tail -20 gpurun_out/r03/b29.log; exit 1; }
echo -n "C2 $v "; tail -1 gpurun_out/r03/b29.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_ms_unloaded'])"
done

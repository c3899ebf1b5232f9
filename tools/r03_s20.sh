# stem2_fused: packed SiLU + stem row reuse down tile columns: parity (bit-identical to the split pair), model, timing
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q -k "stem or yolov7 or g1 or G1 or tiny" --timeout 200 --timeout-method thread > gpurun_out/r03/s2_tests.log 2>&1 || { grep -E "^E  |FAILED" gpurun_out/r03/s2_tests.log | head -10; exit 1; }
tail -1 gpurun_out/r03/s2_tests.log
for i in 1 2; do timeout -k 10 120 python tests/probes/stem2_bench.py fused 2>&1 | grep -v amdgpu.ids | tail -1; done

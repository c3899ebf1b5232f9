# NMS parity with the split bucketing (class phase on 4 workgroups per image)
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_post.py tests/test_gpu_image.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03/s33_post.log 2>&1 || { grep -E "^E  |FAILED" gpurun_out/r03/s33_post.log | head -10; exit 1; }
tail -1 gpurun_out/r03/s33_post.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_fp8.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r03/s33_cfg.log 2>&1 || { grep -E "^E  |FAILED" gpurun_out/r03/s33_cfg.log | head -10; exit 1; }
tail -1 gpurun_out/r03/s33_cfg.log
timeout -k 10 120 python bench.py --post-micro --obj-shift 0 2>&1 | grep -v amdgpu | tail -1 > gpurun_out/r03/post_micro_dense.json
timeout -k 10 120 python bench.py --post-micro --obj-shift -3 2>&1 | grep -v amdgpu | tail -1 > gpurun_out/r03/post_micro_sparse.json
cut -c1-200 gpurun_out/r03/post_micro_dense.json gpurun_out/r03/post_micro_sparse.json

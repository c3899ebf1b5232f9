# r06: fp8 ws64 with the deferred epilogue — fp8 parity tests, C5 bench A/B against the previous code
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06ws8
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fp8.py > gpurun_out/r06ws8/tests.log 2>&1 || { tail -30 gpurun_out/r06ws8/tests.log; exit 1; }
tail -2 gpurun_out/r06ws8/tests.log
BENCH_ARGS="--precision fp8 --batch 64" bash tools/ab_arms.sh r06ws8 prev:YCX_LIB=/root/repo/yolo-continuous_amd/ycx/libycx_prev.so base

# r06: class-finish fast path — parity tests, isolated head timings, concurrent bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06head
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_post.py tests/test_gpu_configs.py > gpurun_out/r06head/tests.log 2>&1 || { tail -30 gpurun_out/r06head/tests.log; exit 1; }
tail -2 gpurun_out/r06head/tests.log
timeout -k 10 300 python -u tests/probes/head_bench.py /root/repo/yolo-continuous_amd/ycx/libycx_prev.so /root/repo/yolo-continuous_amd/ycx/libycx_hip.so --rounds 9 > gpurun_out/r06head/head_bench.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r06head/head_bench.txt
bash tools/ab_arms.sh r06head prev:YCX_LIB=/root/repo/yolo-continuous_amd/ycx/libycx_prev.so base

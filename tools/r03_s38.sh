# per-op serial times: bf16 bs32 (C2) and fp8 bs64 (C5)
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 200 python tests/probes/op_times.py 2>&1 | grep -v amdgpu.ids > gpurun_out/r03/ops_bf16.txt || { tail -5 gpurun_out/r03/ops_bf16.txt; exit 1; }
timeout -k 10 200 python tests/probes/op_times.py --precision fp8 --batch 64 2>&1 | grep -v amdgpu.ids > gpurun_out/r03/ops_fp8.txt || { tail -5 gpurun_out/r03/ops_fp8.txt; exit 1; }
tail -1 gpurun_out/r03/ops_bf16.txt; tail -1 gpurun_out/r03/ops_fp8.txt

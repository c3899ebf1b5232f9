# stream-K tile 48: kernel parity, fill study (t16 vs t48), model parity, bench SK on / off
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "stream_k" --timeout 120 --timeout-method thread > gpurun_out/r03/sk_kernels.log 2>&1 || { tail -40 gpurun_out/r03/sk_kernels.log; exit 1; }
tail -1 gpurun_out/r03/sk_kernels.log
X=""
for n in 16 24 32 40 64 80; do X="$X;$n,20,20,512,512,3,1"; done
for n in 16 32 40 48; do X="$X;$n,40,40,256,256,3,1"; done
for n in 16 32 40; do X="$X;$n,40,40,512,256,1,1"; done
X="$X;32,80,80,128,128,3,1;32,20,20,512,256,3,1;32,40,40,256,128,1,1;32,20,20,1024,512,1,1"
IDX=$(python3 -c "print(','.join(str(28+i) for i in range(6+4+3+4)))")
CONV_EXTRA="${X#;}" CONV_SHAPES=$IDX timeout -k 10 300 python3 tests/probes/conv_bench.py 16 48 > gpurun_out/r03/fill_sk.log 2>&1 || { tail -20 gpurun_out/r03/fill_sk.log; exit 1; }
cat gpurun_out/r03/fill_sk.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_image.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/sk_model.log 2>&1 || { tail -40 gpurun_out/r03/sk_model.log; exit 1; }
tail -1 gpurun_out/r03/sk_model.log
for sk in 1 0 1 0; do
YCX_SK=$sk timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/r03/b16.log 2>&1 || { tail -20 gpurun_out/r03/b16.log; exit 1; }
echo -n "SK=$sk "; tail -1 gpurun_out/r03/b16.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_ms_unloaded'])"
done
echo done

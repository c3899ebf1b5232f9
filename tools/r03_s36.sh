# fp8 bs64 (C5) kernel stats under rocprof
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03/fp8prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03/fp8prof -o run --output-format csv -- python3 $R/bench.py --precision fp8 --batch 64 --cpu-seconds 0 --image-in-steps 0 --steps 40 > $R/gpurun_out/r03/fp8prof/bench.log 2>&1 || { tail -5 $R/gpurun_out/r03/fp8prof/bench.log; exit 1; }
grep "^{" $R/gpurun_out/r03/fp8prof/bench.log | tail -1 | cut -c1-200

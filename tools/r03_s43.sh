# final check of the tile-50 build: GPU suite, smoke, bench, dist leg; rocprof kernel stats of a short bench
R=$GRAFT_REPO_ROOT
cd $R
[ -n "$SKIP_FINAL" ] || bash tools/final_check.sh || exit 1
mkdir -p $R/gpurun_out/r03 && cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03/prof_s43 -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 --steps 20 --warmup 5 > $R/gpurun_out/r03/prof_s43.log 2>&1 || { tail -20 $R/gpurun_out/r03/prof_s43.log; exit 1; }
tail -1 $R/gpurun_out/r03/prof_s43.log | cut -c1-200
find $R/gpurun_out/r03/prof_s43 -name "*kernel_stats.csv" | head -2
cd $R && OP_TOP=40 timeout -k 10 200 python tests/probes/op_times.py > gpurun_out/r03/ops_s43.txt 2>&1 || { tail -20 gpurun_out/r03/ops_s43.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r03/ops_s43.txt | head -5; tail -1 gpurun_out/r03/ops_s43.txt

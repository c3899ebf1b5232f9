# L2 / HBM counters of tile 16 on the stride-2 3x3 layers (ops 10, 19, 28 of the bs 32 plan) and two
# stride-1 3x3s for comparison (development probe), run through gpurun:  bash tests/probes/pmc_s2.sh
# Output: gpurun_out/pmc_s2/<shape>/p<i>/...; summaries gpurun_out/pmc_s2/<shape>.txt
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export CONV_EXTRA="32,160,160,128,128,3,2;32,80,80,256,256,3,2;32,40,40,512,512,3,2"
for S in ${PMC_SHAPES:-28 29 30 1 0}; do
  i=0
  for C in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" \
           "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TA_BUSY_avr"; do
    i=$((i+1))
    CONV_SHAPES=$S timeout -s KILL 90 rocprofv3 --pmc $C -d $R/gpurun_out/pmc_s2/$S/p$i -o run --output-format csv -- python3 $R/tests/probes/conv_bench.py 16 > $R/gpurun_out/pmc_s2/$S.p$i.log 2>&1 || { echo "pass $i shape $S failed"; exit 1; }
  done
  python3 $R/tests/probes/pmc_summary.py $R/gpurun_out/pmc_s2/$S > $R/gpurun_out/pmc_s2/$S.txt
done

# Cache / memory-pipeline PMC counters of one conv_bench tile on a few shapes (development probe),
# run through gpurun:   SHAPES="0 14 5" TILE=16 bash tests/probes/pmc_tile.sh
# Output: gpurun_out/pmc_tile/<tile>_<shape>/p<i>/...; summarise with tests/probes/pmc_summary.py
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${TILE:-16}
for S in ${SHAPES:-0 14 5}; do
  i=0
  for C in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE" \
           "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL"; do
    i=$((i+1))
    CONV_SHAPES=$S timeout -s KILL 90 rocprofv3 --pmc $C -d $R/gpurun_out/pmc_tile/${T}_$S/p$i -o run --output-format csv -- python3 $R/tests/probes/conv_bench.py $T > $R/gpurun_out/pmc_tile/${T}_$S.p$i.log 2>&1 || { echo "pass $i shape $S failed"; exit 1; }
  done
  python3 $R/tests/probes/pmc_summary.py $R/gpurun_out/pmc_tile/${T}_$S > $R/gpurun_out/pmc_tile/${T}_$S.txt
done

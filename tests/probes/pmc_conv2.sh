# PMC counters of conv_bench shapes/tiles (development probe), run through gpurun:
#   SHAPE=26 TILES="16 27" bash tests/probes/pmc_conv2.sh
# Output: gpurun_out/pmc2/<tile>/<pass>/...; summarise with tests/probes/pmc_summary.py
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for T in ${TILES:-16}; do
  i=0
  for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM" \
           "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    CONV_SHAPES=${SHAPE:-26} timeout -s KILL 90 rocprofv3 --pmc $C -d $R/gpurun_out/pmc2/$T/p$i -o run --output-format csv -- python3 $R/tests/probes/conv_bench.py $T > $R/gpurun_out/pmc2/$T.p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  done
done

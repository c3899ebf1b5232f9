# PMC counters of one conv_bench shape/tile (development probe), run through gpurun:
#   SHAPE=8 TILE=22 bash tests/probes/pmc_conv.sh
# Output: gpurun_out/pmc_conv/<tile>/<first counter>/...; summarise with tests/probes/pmc_summary.py
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${TILE:-15}
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_MFMA" \
         "SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD" \
         "SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_BANK_CONFLICT" \
         "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
         "TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum" \
         "TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  N=$(echo $C | cut -d' ' -f1)
  CONV_SHAPES=${SHAPE:-3} timeout -k 10 120 rocprofv3 --pmc $C -d $R/gpurun_out/pmc_conv/$T/$N -o run --output-format csv -- python3 $R/tests/probes/conv_bench.py $T > $R/gpurun_out/pmc_conv/$T.$N.log 2>&1 || echo "pass $N failed"
done

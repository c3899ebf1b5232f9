# PMC counters of the stem kernels (development probe), run through gpurun:
#   MODE=fused bash tests/probes/pmc_stem.sh ; python tests/probes/pmc_summary.py gpurun_out/pmc_stem stem2
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_MFMA" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD" \
         "SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LEVEL_WAVES" \
         "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_WRITE_REQ_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  N=$(echo $C | cut -d' ' -f1)
  timeout -k 10 120 rocprofv3 --pmc $C -d $R/gpurun_out/pmc_stem/$N -o run --output-format csv -- python3 $R/tests/probes/stem2_bench.py ${MODE:-fused} > $R/gpurun_out/pmc_stem.$N.log 2>&1 || echo "pass $N failed"
done

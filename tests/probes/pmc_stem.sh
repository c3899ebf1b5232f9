# PMC counters of the stem kernels (split path) — development probe, run through gpurun.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_MFMA" "SQ_WAVES SQ_INSTS_VALU_TRANS_F32 TA_BUSY_avr TA_TA_BUSY_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  N=$(echo $C | cut -d' ' -f1)
  timeout -k 10 120 rocprofv3 --pmc $C -d $R/gpurun_out/pmc_stem/$N -o run --output-format csv -- python3 $R/tests/probes/stem2_bench.py ${MODE:-split} || exit 1
done

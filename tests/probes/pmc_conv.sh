cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
  N=$(echo $C | cut -d' ' -f1)
  CONV_SHAPES=${SHAPE:-3} timeout -k 10 120 rocprofv3 --pmc $C -d $R/gpurun_out/pmc_conv/$N -o run --output-format csv -- python3 $R/tests/probes/conv_bench.py ${TILE:-15} || exit 1
done

#!/bin/bash
# Round-2 baseline probe (run through gpurun): default bench with per-op kernel
# times, then SQ counter passes on the dominant conv tile (16) for two shapes.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r02
cd $R
YCX_BENCH_KERNELS=$R/gpurun_out/r02/k_base.json timeout -k 10 300 python3 bench.py --cpu-seconds 0 > gpurun_out/r02/bench_base.log 2>&1 || { echo bench failed; exit 1; }
tail -1 gpurun_out/r02/bench_base.log
cd /tmp
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM" \
         "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  for S in 0 14; do
    CONV_SHAPES=$S timeout -s KILL 90 rocprofv3 --pmc $C -d $R/gpurun_out/r02/pmc16/s$S/p$i -o run --output-format csv -- python3 $R/tests/probes/conv_bench.py 16 > $R/gpurun_out/r02/pmc16_s$S.p$i.log 2>&1 || { echo "pass $i shape $S failed"; exit 1; }
  done
done
echo done

# PMC counters of nms_big on the bench workload (development probe), run through gpurun:
#   bash tests/probes/pmc_nms.sh ; python tests/probes/pmc_summary.py gpurun_out/pmc_nms nms_big
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_nms
export YCX_LIB=$R/yolo-continuous_amd/csrc/build/libycx_hip_prof.so  # the probe reads the phase counters
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH" \
         "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d $R/gpurun_out/pmc_nms/p$i -o run --output-format csv -- python3 $R/tests/probes/nms_phases.py > $R/gpurun_out/pmc_nms/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmc_nms/p$i.log; exit 1; }
done
cd $R && python3 tests/probes/pmc_summary.py gpurun_out/pmc_nms nms_big

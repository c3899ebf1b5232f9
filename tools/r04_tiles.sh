cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04
# the HBM-bound tile-16 1x1 shapes of the plan: tile 16 vs the weight-resident 1x1 (22)
export CONV_EXTRA="32,40,40,512,512,1,1;32,40,40,256,256,1,1;32,80,80,512,128,1,1;32,80,80,128,128,1,1;32,20,20,512,512,1,1;32,40,40,256,128,1,1;32,160,160,128,128,3,2;32,80,80,128,128,3,2"
CONV_SHAPES=28,29,30,31,32,33,34,35 timeout -k 10 300 python tests/probes/conv_bench.py 16 22 18 > gpurun_out/r04/tiles.txt 2>&1; rc=$?; cat gpurun_out/r04/tiles.txt; exit $rc

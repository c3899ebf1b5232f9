# isolated tile table: 3-stage one-block-per-CU tiles (9 co128xpx256, 11 co256xpx128, 12 co128xpx128) vs tile 16
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03
cd $R
CONV_SHAPES=0,2,5,14,15,16,20,22,26,8,18,12 timeout -k 10 300 python tests/probes/conv_bench.py 16 9 11 12 > gpurun_out/r03/tiles3.log 2>&1 || { tail -20 gpurun_out/r03/tiles3.log; exit 1; }
cat gpurun_out/r03/tiles3.log

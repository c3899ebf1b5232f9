cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04
bash tools/r04.sh tests tests/test_gpu_kernels.py -k "image20 or halo" > gpurun_out/r04/kt.txt 2>&1; rc=$?; tail -3 gpurun_out/r04/kt.txt; [ $rc = 0 ] || exit $rc
# the 20^2 3x3 layers of the plan: tile 16 / 18 vs the whole-image halo tiles
export CONV_EXTRA="32,20,20,256,256,3,1;32,20,20,512,256,3,1;32,20,20,512,512,3,1;32,20,20,512,1024,3,1;32,20,20,256,512,3,1"
CONV_SHAPES=28,29,30,31,32 timeout -k 10 300 python tests/probes/conv_bench.py 16 18 56 57 > gpurun_out/r04/tiles.txt 2>&1; rc=$?; cat gpurun_out/r04/tiles.txt; exit $rc

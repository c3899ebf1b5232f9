mkdir -p gpurun_out/r02
for T in 16 27 28 29 24; do echo "tile $T"; timeout -k 10 200 python tests/probes/conv_ab.py yolo-continuous_amd/csrc/build/libycx_exp.so --tile $T --shapes 0,14,16,20,26,2 --rounds 3; done > gpurun_out/r02/ab3.log 2>&1
cat gpurun_out/r02/ab3.log

#!/bin/bash
# Build an experiment variant of libycx_hip.so (development tool):
#   bash tools/build_variant.sh NAME -DFLAG ...  ->  yolo-continuous_amd/ycx/libycx_NAME.so
# (the conv unit rebuilt with the flags, in both element types; the other units as built by make)
set -e
cd "$(dirname "$0")/../yolo-continuous_amd/csrc"
make -s
NAME=$1; shift
mkdir -p build/var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -Wno-unused-function "$@" \
  -c ycx_conv.hip -o build/var/ycx_conv_$NAME.o 2>/dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -Wno-unused-function -DYCX_ELT_F16 "$@" \
  -c ycx_conv.hip -o build/var/ycx_conv_f16_$NAME.o 2>/dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC build/var/ycx_conv_$NAME.o build/var/ycx_conv_f16_$NAME.o \
  build/ycx_misc.o build/ycx_post.o build/ycx_nms.o build/ycx_image.o -ldl \
  -o ../ycx/libycx_$NAME.so
echo yolo-continuous_amd/ycx/libycx_$NAME.so

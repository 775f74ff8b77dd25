#!/bin/bash
# A/B library for the MWT non-temporal hints: batchnorm / hfsep / convwin compiled with
# -DEWVIT_MWT_NT=0, every other object from the in-tree build -> ab_lib/libewvit_old.so
set -e
cd "$(dirname "$0")/.."
make -C efficient-wavelet-vit_amd/csrc -j8 > /dev/null
mkdir -p ab_lib build/ab
for f in batchnorm hfsep convwin; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -DEWVIT_MWT_NT=0 \
    -c efficient-wavelet-vit_amd/csrc/$f.hip -o build/ab/$f.o &
done
wait
objs=$(ls build/obj/*.o | grep -v -e batchnorm.o -e hfsep.o -e convwin.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ab_lib/libewvit_old.so $objs build/ab/*.o
echo built ab_lib/libewvit_old.so

#!/bin/bash
# A/B library: the named csrc files compiled with extra defines, every other object from the
# in-tree build -> ab_lib/libewvit_old.so.  Usage: tools/build_ab.sh "-DNAME=V ..." file [file ...]
set -e
cd "$(dirname "$0")/.."
DEFS=$1; shift
make -C efficient-wavelet-vit_amd/csrc -j8 > /dev/null
mkdir -p ab_lib build/ab
rm -f build/ab/*.o
excl=()
for f in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function $DEFS \
    -c efficient-wavelet-vit_amd/csrc/$f.hip -o build/ab/$f.o &
  excl+=(-e "/$f.o")
done
wait
objs=$(ls build/obj/*.o | grep -v "${excl[@]}")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ab_lib/libewvit_old.so $objs build/ab/*.o
echo built ab_lib/libewvit_old.so

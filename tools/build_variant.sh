#!/bin/bash
# tools/build_variant.sh NAME "-DFOO=0 ..." -- an A/B build of libsmashgpu.so:
# csrc/mam.hip compiled with the given defines (the search kernel's
# compile-time switches, mam_sm.hpp), linked with the tree's other objects
# into smash-paper_amd/lib/libsmashgpu_NAME.so (run it with SMASH_LIB=...).
set -euo pipefail
NAME=${1:?name}
DEFS=${2:-}
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R/smash-paper_amd"
make -s -j8 lib/libsmashgpu.so
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -Wall -Wno-unused-result \
    $DEFS -c -o "build/mam_$NAME.o" csrc/mam.hip
OBJS=$(ls build/*.o | grep -v '/mam_' | grep -v '^build/mam.o$')
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "lib/libsmashgpu_$NAME.so" "build/mam_$NAME.o" $OBJS \
    -lz -lpthread -ldl
echo "lib/libsmashgpu_$NAME.so"

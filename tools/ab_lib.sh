#!/bin/bash
# Build an A/B variant of the library into abtmp/lib_<name>.so: crc_uniform.hip recompiled
# with extra flags (e.g. -DSUBSPACE_UNI_PROLOGUE=1), every other object from build/obj.
#   bash tools/ab_lib.sh <name> [hipcc flags...]
set -eu
NAME=$1; shift
make -s subspace_amd/libsubspace_crc.so
mkdir -p abtmp/obj_$NAME
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result "$@" \
  -c subspace_amd/csrc/crc_uniform.hip -o abtmp/obj_$NAME/crc_uniform.o
objs=$(ls build/obj/*.o | grep -v crc_uniform.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o abtmp/lib_$NAME.so abtmp/obj_$NAME/crc_uniform.o $objs
echo abtmp/lib_$NAME.so

#!/bin/bash
# Build an A/B variant of the library into abtmp/lib_<name>.so: one HIP source recompiled
# with extra flags (e.g. -DSUBSPACE_RAGGED_GLOBAL=1), every other object from build/obj.
#   [SRC=crc_ragged] bash tools/ab_lib.sh <name> [hipcc flags...]     (SRC default crc_uniform)
set -eu
NAME=$1; shift
SRC=${SRC:-crc_uniform}
make -s subspace_amd/libsubspace_crc.so
mkdir -p abtmp/obj_$NAME
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result "$@" \
  -c subspace_amd/csrc/$SRC.hip -o abtmp/obj_$NAME/$SRC.o
objs=$(ls build/obj/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o abtmp/lib_$NAME.so abtmp/obj_$NAME/$SRC.o $objs
echo abtmp/lib_$NAME.so

#!/bin/bash
# Build an A/B variant of the library into abtmp/lib_<name>.so: one HIP source recompiled
# with extra flags (e.g. -DSUBSPACE_SMALL_VARIANT=2), every other object from build/obj; and a
# matching development library abtmp/lib_<name>_dev.so (devtools.hip with the same flags: its
# PROBE instantiations of the uniform and small kernels). SUBSPACE_AB_BUILD is defined, so the
# timing-only variant knobs compile (they are a build error in the product library).
#   [SRC=crc_small] bash tools/ab_lib.sh <name> [hipcc flags...]     (SRC default crc_uniform)
# Load with SUBSPACE_CRC_PROBE_LIB=abtmp/lib_<name>.so SUBSPACE_CRC_PROBE_DEV_LIB=abtmp/lib_<name>_dev.so
set -eu
NAME=$1; shift
SRC=${SRC:-crc_uniform}
make -s subspace_amd/libsubspace_crc.so subspace_amd/libsubspace_crc_dev.so
mkdir -p abtmp/obj_$NAME
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -DSUBSPACE_AB_BUILD"
/opt/rocm/bin/hipcc $FLAGS "$@" -c subspace_amd/csrc/$SRC.hip -o abtmp/obj_$NAME/$SRC.o &
/opt/rocm/bin/hipcc $FLAGS "$@" -c subspace_amd/csrc/devtools.hip -o abtmp/obj_$NAME/devtools.o &
wait
objs=$(ls build/obj/*.o | grep -v "/$SRC.o" | grep -v "/devtools.o" | grep -v "/testutil.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--version-script=subspace_amd/csrc/exports.map \
  -o abtmp/lib_$NAME.so abtmp/obj_$NAME/$SRC.o $objs
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o abtmp/lib_${NAME}_dev.so abtmp/obj_$NAME/devtools.o \
  build/obj/testutil.o
echo abtmp/lib_$NAME.so abtmp/lib_${NAME}_dev.so

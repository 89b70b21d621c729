#!/bin/bash
# Investigation builds of libsubspace_crc.so with parts of the uniform kernel removed
# (SUBSPACE_CRC_PROBE bits, crc_uniform.hip): tools/ubench/probes/libprobe<N>.so.
# Use: SUBSPACE_CRC_PROBE_LIB=tools/ubench/probes/libprobe1.so python tools/sweep_uniform.py ...
set -e
cd "$(dirname "$0")/../.."
mkdir -p tools/ubench/probes/obj
for n in "$@"; do
  objs=""
  for f in crc_uniform crc_ragged crc_slots capi testutil; do
    o=tools/ubench/probes/obj/${f}_$n.o
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DSUBSPACE_CRC_PROBE=$n -c subspace_amd/csrc/$f.hip -o $o &
    objs="$objs $o"
  done
  g++ -O3 -std=c++17 -fPIC -c subspace_amd/csrc/host_crc.cpp -o tools/ubench/probes/obj/host_crc_$n.o
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/ubench/probes/libprobe$n.so $objs tools/ubench/probes/obj/host_crc_$n.o
done

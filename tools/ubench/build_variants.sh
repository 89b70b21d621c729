#!/bin/bash
# Timing-only builds of libsubspace_crc.so with the fused slot kernel's variants
# (crc_uniform.hip SUBSPACE_SLOT_VARIANT): tools/ubench/probes/libslot<N>.so.
# Use: SUBSPACE_CRC_PROBE_LIB=tools/ubench/probes/libslot1.so SLOT_GAP_NOCHECK=1 python tools/slot_gap.py
set -e
cd "$(dirname "$0")/../.."
mkdir -p tools/ubench/probes/obj
for n in "$@"; do
  objs=""
  for f in crc_uniform crc_small crc_ragged crc_long crc_combine crc_slots capi testutil; do
    o=tools/ubench/probes/obj/${f}_v$n.o
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DSUBSPACE_SLOT_VARIANT=$n -c subspace_amd/csrc/$f.hip -o $o &
    objs="$objs $o"
  done
  for f in host_crc split_alloc; do
    g++ -O3 -std=c++17 -fPIC -c subspace_amd/csrc/$f.cpp -o tools/ubench/probes/obj/${f}_v$n.o
    objs="$objs tools/ubench/probes/obj/${f}_v$n.o"
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/ubench/probes/libslot$n.so $objs
done

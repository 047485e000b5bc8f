#!/bin/bash
# Build compile-time variants of the HIP library for A/B timing on the GPU box:
#   tools/variants.sh NAME "-DFLAG=.. -DFLAG2=.." [NAME2 "FLAGS2" ...]
# Each lands in build/var/NAME/libapprox_counter_amd.so; run bench.py with
# APPROX_COUNTER_AMD_LIB=build/var/NAME/libapprox_counter_amd.so.
set -e
cd "$(dirname "$0")/.."
while [ $# -gt 1 ]; do
  name=$1; flags=$2; shift 2
  out=build/var/$name; mkdir -p $out
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Iinclude -Iapprox_counter_amd/csrc $flags \
    -mllvm -amdgpu-atomic-optimizer-strategy=None -c approx_counter_amd/csrc/wm_count.hip -o $out/wm_count.o
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Iinclude -Iapprox_counter_amd/csrc $flags \
    -c approx_counter_amd/csrc/exact_count.hip -o $out/exact_count.o
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Iinclude -Iapprox_counter_amd/csrc $flags \
    -x hip -c approx_counter_amd/csrc/capi.cpp -o $out/capi.o
  g++ -O3 -std=c++17 -fPIC -Wall $flags -c approx_counter_amd/csrc/host_pack.cpp -o $out/host_pack.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libapprox_counter_amd.so $out/wm_count.o $out/exact_count.o $out/capi.o $out/host_pack.o -pthread
  echo "built $out"
done

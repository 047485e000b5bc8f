#!/bin/bash
# Build the HIP library from a source tree (a copy of include/ + approx_counter_amd/csrc/ with an
# experiment undone or applied) for same-box A/B timing:
#   tools/variant_dir.sh DIR NAME ["-DFLAG ..."]  ->  build/var/NAME/libapprox_counter_amd.so
set -e
cd "$(dirname "$0")/.."
src=$1; name=$2; flags=${3:-}
out=build/var/$name; mkdir -p $out
C="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -I$src/include -I$src/approx_counter_amd/csrc $flags"
/opt/rocm/bin/hipcc $C -mllvm -amdgpu-atomic-optimizer-strategy=None -c $src/approx_counter_amd/csrc/wm_count.hip -o $out/wm_count.o
/opt/rocm/bin/hipcc $C -c $src/approx_counter_amd/csrc/exact_count.hip -o $out/exact_count.o
/opt/rocm/bin/hipcc $C -x hip -c $src/approx_counter_amd/csrc/capi.cpp -o $out/capi.o
g++ -O3 -std=c++17 -fPIC -Wall $flags -c $src/approx_counter_amd/csrc/host_pack.cpp -o $out/host_pack.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libapprox_counter_amd.so $out/*.o -pthread
echo "built $out from $src"

#!/bin/bash
# Build the HIP library of another git revision for same-box A/B timing:
#   tools/variant_rev.sh REV NAME ["-DFLAG ..."]  ->  build/var/NAME/libapprox_counter_amd.so
set -e
cd "$(dirname "$0")/.."
rev=$1; name=$2; flags=${3:-}
src=$(mktemp -d)
git archive "$rev" approx_counter_amd/csrc include | tar -x -C "$src"
out=build/var/$name; mkdir -p $out
C="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -I$src/include -I$src/approx_counter_amd/csrc $flags"
/opt/rocm/bin/hipcc $C -mllvm -amdgpu-atomic-optimizer-strategy=None -c $src/approx_counter_amd/csrc/wm_count.hip -o $out/wm_count.o
/opt/rocm/bin/hipcc $C -c $src/approx_counter_amd/csrc/exact_count.hip -o $out/exact_count.o
/opt/rocm/bin/hipcc $C -x hip -c $src/approx_counter_amd/csrc/capi.cpp -o $out/capi.o
g++ -O3 -std=c++17 -fPIC -Wall $flags -c $src/approx_counter_amd/csrc/host_pack.cpp -o $out/host_pack.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libapprox_counter_amd.so $out/*.o -pthread
rm -rf "$src"
echo "built $out from $rev"

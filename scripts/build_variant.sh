#!/bin/bash
# Build an experimental library variant: scripts/build_variant.sh NAME -DFLAG=1 ...
# -> rifraf.jl_amd/librifraf_NAME.so (same sources as the product library)
set -e
N=$1; shift
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-result "$@" \
  rifraf.jl_amd/csrc/rifraf_hip.hip rifraf.jl_amd/csrc/rifraf_batch.cpp -o rifraf.jl_amd/librifraf_$N.so.tmp
mv rifraf.jl_amd/librifraf_$N.so.tmp rifraf.jl_amd/librifraf_$N.so   # atomic: a snapshot never sees a partial file
echo "built librifraf_$N.so"

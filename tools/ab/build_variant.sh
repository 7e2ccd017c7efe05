#!/bin/bash
# Build the library with extra defines into tools/ab/librag_retrieval_<name>.so (A/B arms; build container).
#   bash tools/ab/build_variant.sh <name> "-DFOO=1 ..."
set -e
H=$(cd "$(dirname "$0")/../.." && pwd)
P=$H/rag-serving-system_amd
B=$H/tools/ab/build_$1
mkdir -p "$B"
F="-O3 -std=c++17 -Wno-unused-value -Wno-unused-result -fPIC -I$H/include -I$P/csrc $2"
/opt/rocm/bin/hipcc --offload-arch=gfx950 $F -c $P/csrc/rr_kernels.hip -o $B/rr_kernels.o &
/opt/rocm/bin/hipcc --offload-arch=gfx950 $F -c $P/csrc/rr_sk.hip -o $B/rr_sk.o &
/opt/rocm/bin/hipcc $F -pthread -c $P/csrc/rr_api.cpp -o $B/rr_api.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $B/*.o -L/opt/rocm/lib -lrccl -pthread -Wl,-rpath,/opt/rocm/lib \
  -o $H/tools/ab/librag_retrieval_$1.so
rm -rf "$B"

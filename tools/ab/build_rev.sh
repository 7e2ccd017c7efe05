#!/bin/bash
# Build the library from another git revision's sources into tools/ab/librag_retrieval_<name>.so (A/B arm).
#   bash tools/ab/build_rev.sh <name> <rev> ["-DFOO=1 ..."]      (<rev> = . : the working tree's sources)
set -e
H=$(cd "$(dirname "$0")/../.." && pwd)
T=$(mktemp -d)
if [ "$2" = . ]; then
  mkdir -p "$T/rag-serving-system_amd" && cp -r "$H/include" "$T/" && cp -r "$H/rag-serving-system_amd/csrc" "$T/rag-serving-system_amd/"
else
  git -C "$H" archive "$2" include rag-serving-system_amd/csrc | tar -x -C "$T"
fi
B=$T/build
mkdir -p "$B"
F="-O3 -std=c++17 -Wno-unused-value -Wno-unused-result -fPIC -I$T/include -I$T/rag-serving-system_amd/csrc $3"
P=$T/rag-serving-system_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 $F -c $P/rr_kernels.hip -o $B/rr_kernels.o &
/opt/rocm/bin/hipcc --offload-arch=gfx950 $F -c $P/rr_sk.hip -o $B/rr_sk.o &
[ -f $P/rr_topk.hip ] && /opt/rocm/bin/hipcc --offload-arch=gfx950 $F -c $P/rr_topk.hip -o $B/rr_topk.o &
/opt/rocm/bin/hipcc $F -pthread -c $P/rr_api.cpp -o $B/rr_api.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $B/*.o -L/opt/rocm/lib -lrccl -pthread -Wl,-rpath,/opt/rocm/lib \
  -o "$H/tools/ab/librag_retrieval_$1.so"
rm -rf "$T"

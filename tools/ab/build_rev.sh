#!/bin/bash
# Build the library from another git revision's sources into tools/ab/librag_retrieval_<name>.so (A/B arm).
#   bash tools/ab/build_rev.sh <name> <rev> ["-DFOO=1 ..."]      (<rev> = . : the working tree's sources)
# (every .hip unit of the revision's csrc/ — the split-K kernel's instantiation units too — compiled side by side;
# "-DRR_AB_ENV=1" gives an arm that reads its path options from RR_<NAME> environment variables)
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
for u in $P/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $F -c $u -o $B/$(basename $u .hip).o &
done
/opt/rocm/bin/hipcc $F -pthread -c $P/rr_api.cpp -o $B/rr_api.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $B/*.o -L/opt/rocm/lib -lrccl -pthread -Wl,-rpath,/opt/rocm/lib \
  -o "$H/tools/ab/librag_retrieval_$1.so"
rm -rf "$T"

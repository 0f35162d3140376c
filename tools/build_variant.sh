#!/bin/bash
# Build libmacroc_amd.so with extra compile definitions into abl/<name>.so for in-process A/B
# (tools/spmv_ab.py --lib abl/<name>.so).  Usage: tools/build_variant.sh NAME -DFOO=1 ...
set -e
name=$1; shift
mkdir -p abl/obj_$name
cd "$(dirname "$0")/.."
F="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -Wall -Wno-unused-function"
for f in api.cpp dmda.cpp comm.cpp vtu.cpp kernels.hip; do
  /opt/rocm/bin/hipcc $F "$@" -c macroc_amd/csrc/$f -o abl/obj_$name/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o abl/$name.so abl/obj_$name/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf abl/obj_$name

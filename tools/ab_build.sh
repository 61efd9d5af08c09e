#!/bin/bash
# Build A/B variants of libsstcodec.so with extra -D flags for some source files:
#   bash tools/ab_build.sh <name> <src.hip[,src2.hip]> <flags...>  -> lsm-kv-storage_amd/lib/ab/<name>/libsstcodec.so
# (the other objects are the in-tree build's; run build() first)
set -e
cd "$(dirname "$0")/.."
name=$1; srcs=$2; shift 2
L=lsm-kv-storage_amd/lib
out=$L/ab/$name; mkdir -p $out
bases=""
for src in ${srcs//,/ }; do
  base=$(basename $src); bases="$bases $base.o"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result "$@" -c lsm-kv-storage_amd/csrc/$src -o $out/$base.o
done
objs=""
for o in $L/obj/*.o; do b=$(basename $o); if [[ " $bases " == *" $b "* ]]; then objs="$objs $out/$b"; else objs="$objs $o"; fi; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libsstcodec.so $objs
echo "built $out/libsstcodec.so"

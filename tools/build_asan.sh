#!/bin/bash
# AddressSanitizer builds of the HOST code (device code as shipped; GPU ASan is
# not available on this pool): libsstcodec.so's host parts (the .hip files'
# host side with -Xarch_host, host/*.cpp) into lsm-kv-storage_amd/lib/asan/,
# and the drop-in harness (unmodified compact.cc + the drop-in iterators) linked against it, all with clang's ASan runtime:
#   bash tools/build_asan.sh   -> oracle/_ref/compact_dropin_asan_lib
# (oracle/Makefile's dropin-asan instruments the engine TUs only.)
set -e
cd "$(dirname "$0")/.."
ROOT=$PWD; REF=/root/reference
CL=/opt/rocm/lib/llvm/bin/clang++
HIPCC=/opt/rocm/bin/hipcc
OUT=lsm-kv-storage_amd/lib/asan; OBJ=$OUT/obj; mkdir -p $OBJ
ASAN="-fsanitize=address -fno-omit-frame-pointer -g -O1"
for s in sstc_kernels sstc_compact sstc_get sstc_api; do
  $HIPCC -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer \
    -c lsm-kv-storage_amd/csrc/$s.hip -o $OBJ/$s.o
done
for s in sst_table compact_files resident; do
  $CL $ASAN -std=c++17 -fPIC -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -c lsm-kv-storage_amd/csrc/host/$s.cpp -o $OBJ/$s.o
done
$HIPCC --offload-arch=gfx950 -shared -fPIC -Wl,--allow-shlib-undefined -o $OUT/libsstcodec.so $OBJ/*.o
D=oracle/_ref/dropin_asan_clang_obj; mkdir -p $D/sstc
INC="-Iinclude/dropin -Iinclude -I$REF"
# the drop-in build's engine TUs (oracle/Makefile DROPIN_SRCS)
srcs="sstable/block_builder.cc sstable/block_reader.cc sstable/block_reader_iterator.cc sstable/lru_block_item.cc
      sstable/block_reader_cache.cc sstable/table_reader.cc sstable/block_index.cc io/linux_file.cc io/buffer.cc
      db/config.cc sstable/lru_table_item.cc sstable/table_reader_cache.cc db/compact.cc
      db/version.cc db/version_edit.cc db/version_manager.cc"
objs=""
for s in $srcs; do
  o=$D/${s//\//_}.o
  fresh=1
  for h in $REF/$s include/dropin/sstable/*.h include/dropin/db/*.h include/sstc_table.h include/sstcodec.h; do
    [ $o -nt $h ] || fresh=0
  done
  [ $fresh = 1 ] || $CL -std=c++20 $ASAN $INC -c $REF/$s -o $o
  objs="$objs $o"
done
$CL -std=c++20 $ASAN -Wall $INC -c lsm-kv-storage_amd/csrc/dropin/table_reader_iterator.cc -o $D/sstc/tri.o
$CL -std=c++20 $ASAN -Wall $INC -c lsm-kv-storage_amd/csrc/dropin/merge_iterator.cc -o $D/sstc/mi.o
$CL -std=c++20 $ASAN -DSSTC_DROPIN $INC -o oracle/_ref/compact_dropin_asan_lib oracle/ref_pick_compact.cc $objs $D/sstc/tri.o $D/sstc/mi.o \
  -L$OUT -lsstcodec -Wl,-rpath,'$ORIGIN/../../lsm-kv-storage_amd/lib/asan' -lpthread
echo "built oracle/_ref/compact_dropin_asan_lib"

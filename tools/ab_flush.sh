#!/bin/bash
# A/B of library builds on the flush path (tools/bench_flush.py), alternating.
#   VARIANTS="base cur" ROUNDS=2 bash tools/ab_flush.sh   (cur = the in-tree build)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/abf
for r in $(seq ${ROUNDS:-2}); do
for v in ${VARIANTS:-base cur}; do
  if [ $v = cur ]; then unset SSTC_LIB_PATH; else export SSTC_LIB_PATH=$PWD/lsm-kv-storage_amd/lib/ab/$v/libsstcodec.so; fi
  timeout -k 10 300 python3 tools/bench_flush.py --reps ${REPS:-5} > gpurun_out/abf/f$v$r.log 2>&1 || { echo "flush $v failed"; tail -20 gpurun_out/abf/f$v$r.log; exit 4; }
  echo "round $r $v $(tail -1 gpurun_out/abf/f$v$r.log | cut -c1-400)"
done
done

#!/bin/bash
# Untraced A/B of library builds on the compaction job (tools/bench_compact.py
# device_s_median), configs and variants interleaved ROUNDS times.
#   VARIANTS="base cur" CONFIGS="3 4 5" bash tools/ab_jobs.sh   (cur = the in-tree build)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/abj
for r in $(seq ${ROUNDS:-2}); do
for c in ${CONFIGS:-3 4 5}; do
for v in ${VARIANTS:-base cur}; do
  if [ $v = cur ]; then unset SSTC_LIB_PATH; else export SSTC_LIB_PATH=$PWD/lsm-kv-storage_amd/lib/ab/$v/libsstcodec.so; fi
  timeout -k 10 300 python3 tools/bench_compact.py --config $c --steps ${STEPS:-20} --no-ref --no-files > gpurun_out/abj/b$c$v$r.log 2>&1 || { echo "bench $c $v failed"; tail -20 gpurun_out/abj/b$c$v$r.log; exit 4; }
  echo "round $r config $c $v $(grep -o '"device_s_median": [0-9.e-]*' gpurun_out/abj/b$c$v$r.log) $(grep -o '"matches_reference_fixture": [^]]*' gpurun_out/abj/b$c$v$r.log)"
done
done
done

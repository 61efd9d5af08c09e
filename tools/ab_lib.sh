#!/bin/bash
# A/B of library builds (tools/ab_build.sh) on the compaction job: configs 3 and 4,
# kernel trace per variant, outputs checked against the reference fixtures.
#   VARIANTS="base cur x y" bash tools/ab_lib.sh   (cur = the in-tree build)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/abl
for c in ${CONFIGS:-3 4}; do
for v in ${VARIANTS:-base cur}; do
  if [ $v = cur ]; then unset SSTC_LIB_PATH; else export SSTC_LIB_PATH=$PWD/lsm-kv-storage_amd/lib/ab/$v/libsstcodec.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/abl/t$c$v -o trace --output-format csv -- python3 tools/bench_compact.py --config $c --steps 5 --no-ref --no-files > gpurun_out/abl/b$c$v.log 2>&1 || { echo "bench $c $v failed"; tail -20 gpurun_out/abl/b$c$v.log; exit 4; }
  python3 tools/trace_compact.py $(find gpurun_out/abl/t$c$v -name "*kernel_trace.csv" | head -1) > gpurun_out/abl/k$c$v.txt
  echo "config $c $v $(grep -o '"matches_reference_fixture": [^]]*' gpurun_out/abl/b$c$v.log) $(grep -o '"device_s_median": [0-9.e-]*' gpurun_out/abl/b$c$v.log) | $(grep -E "${KERNELS:-filter}" gpurun_out/abl/k$c$v.txt | tr -s ' ' | tr '\n' ';')"
done
done

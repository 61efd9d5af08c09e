#!/bin/bash
# A/B of library builds on config 3-overlap (8 M in, 1 M kept): kernel trace per variant.
#   VARIANTS="prenf cur" bash tools/ab_overlap.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/abo
for v in ${VARIANTS:-prenf cur}; do
  if [ $v = cur ]; then unset SSTC_LIB_PATH; else export SSTC_LIB_PATH=$PWD/lsm-kv-storage_amd/lib/ab/$v/libsstcodec.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/abo/t$v -o trace --output-format csv -- python3 tools/bench_compact.py --config 3 --overlap --steps 5 --no-ref --no-files > gpurun_out/abo/b$v.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/abo/b$v.log; exit 4; }
  python3 tools/trace_compact.py $(find gpurun_out/abo/t$v -name "*kernel_trace.csv" | head -1) > gpurun_out/abo/k$v.txt
  echo "== $v $(grep -o '"device_s_median": [0-9.e-]*' gpurun_out/abo/b$v.log)"; head -30 gpurun_out/abo/k$v.txt
done

#!/bin/bash
# HIP API + kernel trace of one compaction job (host launch cost vs GPU gaps):
#   bash tools/hip_trace.sh <outdir> <config>
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
out=gpurun_out/${1:-hiptrace}; cfg=${2:-5}
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d $out/t -o trace --output-format csv -- python3 tools/bench_compact.py --config $cfg --steps 3 --no-ref --no-files > $out/b.log 2>&1 || { echo "trace failed"; tail -20 $out/b.log; exit 4; }
ls $out/t

#!/bin/bash
# rocprofv3 passes for the bench workload: kernel trace + stats, then one PMC
# pass per counter group (FETCH_SIZE and WRITE_SIZE do not fit one pass).
# Usage: bash tools/profile.sh <tag> [bench args...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
tag=${1:-run}; shift
args=${*:---steps 20 --no-cpu-baseline --no-e2e --no-hbm-variant}
out=gpurun_out/prof_$tag
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o trace --output-format csv -- python3 bench.py $args > $out/trace.log 2>&1 || { echo "trace failed"; tail -20 $out/trace.log; exit 3; }
echo "trace ok"; tail -2 $out/trace.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o fetch --output-format csv -- python3 bench.py $args > $out/fetch.log 2>&1 || { echo "fetch failed"; tail -20 $out/fetch.log; exit 4; }
echo "fetch ok"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $out/write -o write --output-format csv -- python3 bench.py $args > $out/write.log 2>&1 || { echo "write failed"; tail -20 $out/write.log; exit 5; }
echo "write ok"
find $out -name "*.csv" | head -20

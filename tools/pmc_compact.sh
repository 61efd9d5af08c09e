#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE; one counter group per run) over the
# config-3 compaction job.  Usage: bash tools/pmc_compact.sh <tag> [bench_compact args]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
tag=${1:-c3}; shift
args=${*:---config 3 --steps 1 --no-ref --no-files}
out=gpurun_out/pmc_$tag
mkdir -p $out
timeout -k 10 -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o fetch --output-format csv -- python3 tools/bench_compact.py $args > $out/fetch.log 2>&1 || { echo "fetch failed"; tail -5 $out/fetch.log; exit 4; }
timeout -k 10 -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $out/write -o write --output-format csv -- python3 tools/bench_compact.py $args > $out/write.log 2>&1 || { echo "write failed"; tail -5 $out/write.log; exit 5; }
echo ok; find $out -name "*counter_collection.csv"

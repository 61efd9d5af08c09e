# config 3: device SST open (sstc_open_tables) timed beside the compaction job,
# plus a rocprofv3 kernel trace of the ot_* kernels.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/open
timeout -k 10 400 python3 tools/bench_compact.py --config 3 --steps 3 > gpurun_out/open/c3.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/open/c3.log; exit 4; }
grep -o '"open_tables_ms": [0-9.]*, "host_index_py_ms": [0-9.]*' gpurun_out/open/c3.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/open/t3 -o trace --output-format csv -- python3 tools/bench_compact.py --config 3 --steps 1 --no-ref --no-files > gpurun_out/open/t3.log 2>&1 || { echo "trace failed"; tail -20 gpurun_out/open/t3.log; exit 5; }
f=$(find gpurun_out/open/t3 -name "*kernel_stats.csv" | head -1)
grep -E "Name|ot_" "$f"

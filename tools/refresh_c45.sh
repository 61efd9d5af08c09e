# configs 4 and 5: full bench_compact runs (device job, file pipeline, reference
# driver, bit-exact check) and a kernel trace of the device job.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/c45
for c in 4 5; do
  timeout -k 10 400 python3 tools/bench_compact.py --config $c --steps 3 > gpurun_out/c45/full$c.log 2>&1 || { echo "bench $c failed"; tail -20 gpurun_out/c45/full$c.log; exit 4; }
  grep -o '"device_s_median": [0-9.e-]*\|"bit_exact_vs_reference": [a-z]*\|"open_tables_ms": [0-9.]*' gpurun_out/c45/full$c.log
done
bash tools/trace_c45.sh

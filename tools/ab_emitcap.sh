cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/abc
for v in 512 1024 2048 4096; do
  SSTC_EMITCAP=$v timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/abc/t$v -o trace --output-format csv -- python3 tools/bench_compact.py --config 5 --steps 5 --no-ref --no-files > gpurun_out/abc/b$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/abc/b$v.log; exit 4; }
  echo "== cap $v $(grep -o '"device_s_median": [0-9.e-]*' gpurun_out/abc/b$v.log) $(grep -o '"matches_reference_fixture": [^]]*' gpurun_out/abc/b$v.log)"
  python3 tools/trace_compact.py $(find gpurun_out/abc/t$v -name "*kernel_trace.csv" | head -1) | grep -E "enc_emit|enc_lds"
done

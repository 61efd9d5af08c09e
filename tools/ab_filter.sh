#!/bin/bash
# A/B of the compaction filter layout: SSTC_FBLK=0 row-major rows (a scan per row), 1 blocked (8 consecutive records per thread, one scan).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/abf
timeout -k 10 600 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_files.py tests/test_gpu_configs.py tests/test_gpu_cpp_boundary.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abf/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/abf/pytest.log; exit 3; }
tail -1 gpurun_out/abf/pytest.log
for c in 3 4; do
for v in 0 1; do
  SSTC_FBLK=$v timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/abf/t$c$v -o trace --output-format csv -- python3 tools/bench_compact.py --config $c --steps 5 --no-ref --no-files > gpurun_out/abf/b$c$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/abf/b$c$v.log; exit 4; }
  echo "== config $c SSTC_FBLK=$v $(grep -o '"device_s_median": [0-9.e-]*' gpurun_out/abf/b$c$v.log) $(grep -o '"matches_reference_fixture": [^]]*' gpurun_out/abf/b$c$v.log)"
  python3 tools/trace_compact.py $(find gpurun_out/abf/t$c$v -name "*kernel_trace.csv" | head -1) > gpurun_out/abf/k$c$v.txt; grep -E "filter|span" gpurun_out/abf/k$c$v.txt
done
done

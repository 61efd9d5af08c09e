#!/bin/bash
# Compaction GPU tests (incl. full-size configs) + config 3 / 4 device legs with kernel traces.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/cc
timeout -k 10 600 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_files.py tests/test_gpu_configs.py tests/test_gpu_cpp_boundary.py tests/test_gpu_codec.py tests/test_gpu_table.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/cc/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/cc/pytest.log; exit 3; }
tail -1 gpurun_out/cc/pytest.log
for c in ${CONFIGS:-3 4}; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/cc/t$c -o trace --output-format csv -- python3 tools/bench_compact.py --config $c --steps 5 --no-ref --no-files > gpurun_out/cc/b$c.log 2>&1 || { echo "bench $c failed"; tail -20 gpurun_out/cc/b$c.log; exit 4; }
  echo "== config $c $(grep -o '"device_s_median": [0-9.e-]*' gpurun_out/cc/b$c.log) $(grep -o '"matches_reference_fixture": [^]]*' gpurun_out/cc/b$c.log)"
  python3 tools/trace_compact.py $(find gpurun_out/cc/t$c -name "*kernel_trace.csv" | head -1) > gpurun_out/cc/k$c.txt; grep -A8 "kernel sum" gpurun_out/cc/k$c.txt
done

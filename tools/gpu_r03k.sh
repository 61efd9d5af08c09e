#!/bin/bash
# compaction parity (meta entries from the encode waves), then configs 3 / 4 / 5 timings + traces
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r03k
timeout -k 10 600 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_files.py tests/test_gpu_configs.py tests/test_gpu_aswritten.py tests/test_gpu_dropin.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03k/pytest.log 2>&1 || { tail -30 gpurun_out/r03k/pytest.log; exit 3; }
tail -1 gpurun_out/r03k/pytest.log
for c in 3 4 5; do
  timeout -k 10 300 python tools/bench_compact.py --config $c --steps 7 --no-ref --no-files > gpurun_out/r03k/b$c.log 2>&1 || { tail -5 gpurun_out/r03k/b$c.log; exit 4; }
  echo "config $c: $(grep -o '"device_s_median": [0-9.e-]*' gpurun_out/r03k/b$c.log)"
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r03k/t$c -o trace --output-format csv -- python3 tools/bench_compact.py --config $c --steps 3 --no-ref --no-files > gpurun_out/r03k/tb$c.log 2>&1 || exit 5
  python3 tools/trace_compact.py $(find gpurun_out/r03k/t$c -name "*kernel_trace.csv" | head -1) > gpurun_out/r03k/k$c.txt
  head -8 gpurun_out/r03k/k$c.txt; grep "span us" gpurun_out/r03k/k$c.txt
done

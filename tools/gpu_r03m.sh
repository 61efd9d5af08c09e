#!/bin/bash
# every GPU test, smoke, bench, then configs 3 / 4 / 5 device-job medians and kernel traces
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_check.sh || exit $?
mkdir -p gpurun_out/r03m
for c in 3 4 5; do
  timeout -k 10 300 python tools/bench_compact.py --config $c --steps 7 --no-ref --no-files > gpurun_out/r03m/b$c.log 2>&1 || { tail -5 gpurun_out/r03m/b$c.log; exit 4; }
  echo "config $c: $(grep -o '"device_s_median": [0-9.e-]*' gpurun_out/r03m/b$c.log)"
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r03m/t$c -o trace --output-format csv -- python3 tools/bench_compact.py --config $c --steps 3 --no-ref --no-files > gpurun_out/r03m/tb$c.log 2>&1 || exit 5
  python3 tools/trace_compact.py $(find gpurun_out/r03m/t$c -name "*kernel_trace.csv" | head -1) > gpurun_out/r03m/k$c.txt
  head -4 gpurun_out/r03m/k$c.txt; grep "span us" gpurun_out/r03m/k$c.txt
done

#!/bin/bash
# Kernel traces of the device compaction job (tools/bench_compact.py) for configs 3, 4, 5.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/c345
for c in ${CONFIGS:-3 4 5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/c345/t$c -o trace --output-format csv -- python3 tools/bench_compact.py --config $c --steps 3 --no-ref --no-files > gpurun_out/c345/b$c.log 2>&1 || { echo "bench $c failed"; tail -20 gpurun_out/c345/b$c.log; exit 4; }
  echo "== config $c"; grep -o '"device_s_median": [0-9.e-]*' gpurun_out/c345/b$c.log
  python3 tools/trace_compact.py $(find gpurun_out/c345/t$c -name "*kernel_trace.csv" | head -1) > gpurun_out/c345/k$c.txt; cat gpurun_out/c345/k$c.txt
done

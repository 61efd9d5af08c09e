#!/bin/bash
# A/B of compaction-job variants selected by an env var: compaction parity
# tests, then config-3 device-leg timings + a kernel trace per variant.
# Usage: bash tools/ab_compact.sh VAR "v1 v2 ..." [bench_compact args]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
var=$1; vals=$2; shift 2
args=${*:---config 3 --steps 5 --no-ref --no-files}
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_files.py tests/test_gpu_codec.py tests/test_gpu_table.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/ab/pytest.log; exit 3; }
tail -1 gpurun_out/ab/pytest.log
for v in $vals; do
  export $var=$v
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ab/t$v -o trace --output-format csv -- python3 tools/bench_compact.py $args > gpurun_out/ab/b$v.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/ab/b$v.log; exit 4; }
  echo "== $var=$v"; grep -o '"device_s_median": [0-9.e-]*' gpurun_out/ab/b$v.log; grep -o '"bit_exact[^,]*' gpurun_out/ab/b$v.log
  python3 tools/trace_compact.py $(find gpurun_out/ab/t$v -name "*kernel_trace.csv" | head -1) > gpurun_out/ab/k$v.txt; head -12 gpurun_out/ab/k$v.txt
done

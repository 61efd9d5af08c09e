#!/bin/bash
# A/B of the compaction merge kernel (SSTC_MERGE=0: per-record co-rank
# searches, 1: pairwise merge tree in LDS): compaction parity tests under the
# new variant, then config 3 and 4 device legs with kernel traces per variant.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/abm
SSTC_MERGE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_files.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/abm/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/abm/pytest.log; exit 3; }
tail -1 gpurun_out/abm/pytest.log
for c in ${CONFIGS:-3 4}; do
for v in ${VARIANTS:-0 1}; do
  export SSTC_MERGE=$v
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/abm/t$c$v -o trace --output-format csv -- python3 tools/bench_compact.py --config $c --steps 5 --no-ref --no-files > gpurun_out/abm/b$c$v.log 2>&1 || { echo "bench $c $v failed"; tail -20 gpurun_out/abm/b$c$v.log; exit 4; }
  echo "== config $c SSTC_MERGE=$v"; grep -o '"device_s_median": [0-9.e-]*' gpurun_out/abm/b$c$v.log; grep -o '"matches_reference_fixture": [^]]*' gpurun_out/abm/b$c$v.log
  python3 tools/trace_compact.py $(find gpurun_out/abm/t$c$v -name "*kernel_trace.csv" | head -1) > gpurun_out/abm/k$c$v.txt; head -6 gpurun_out/abm/k$c$v.txt
done
done

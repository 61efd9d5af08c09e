#!/bin/bash
# merge A/B: rank merge (SSTC_MG_RANK=1) vs the pairwise tree; parity of the rank variant first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r03p
SSTC_MG_RANK=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "not lookup and not all_shards" > gpurun_out/r03p/pytest_rank.log 2>&1 || { tail -30 gpurun_out/r03p/pytest_rank.log; exit 3; }
tail -1 gpurun_out/r03p/pytest_rank.log
for round in 1 2; do
for v in 0 1; do
  for c in "3" "4" "3 --overlap"; do
    tag=$(echo $c | tr -d ' -')
    SSTC_MG_RANK=$v timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r03p/t$v$tag -o trace --output-format csv -- python3 tools/bench_compact.py --config $c --steps 5 --no-ref --no-files > gpurun_out/r03p/b$v$tag.log 2>&1 || { tail -5 gpurun_out/r03p/b$v$tag.log; exit 4; }
    python3 tools/trace_compact.py $(find gpurun_out/r03p/t$v$tag -name "*kernel_trace.csv" | head -1) > gpurun_out/r03p/k$v$tag.txt
    echo "round $round rank=$v config $c: $(grep -o '"matches_reference_fixture": [^]]*' gpurun_out/r03p/b$v$tag.log) $(grep -o '"device_s_median": [0-9.e-]*' gpurun_out/r03p/b$v$tag.log) | $(grep -E 'ck_mg_' gpurun_out/r03p/k$v$tag.txt | tr -s ' ')"
  done
done
done

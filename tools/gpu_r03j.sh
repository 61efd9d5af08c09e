#!/bin/bash
# merge A/B: prefix-plane tile (pf, 8 workgroups / CU) vs 32 B record tile; compaction parity on the pf build first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r03j
timeout -k 10 600 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_files.py tests/test_gpu_configs.py tests/test_gpu_aswritten.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03j/pytest.log 2>&1 || { tail -30 gpurun_out/r03j/pytest.log; exit 3; }
tail -1 gpurun_out/r03j/pytest.log
for round in 1 2; do
for v in tile pf; do
  for c in "3" "3 --overlap" "4"; do
    SSTC_MG_VARIANT=$v timeout -k 10 300 python tools/bench_compact.py --config $c --steps 7 --no-ref --no-files > gpurun_out/r03j/b_${v}_$(echo $c | tr -d ' -').log 2>&1 || { echo "bench $v $c failed"; tail -5 gpurun_out/r03j/b_${v}_$(echo $c | tr -d ' -').log; exit 4; }
    echo "round $round $v config $c: $(grep -o '"device_s_median": [0-9.e-]*' gpurun_out/r03j/b_${v}_$(echo $c | tr -d ' -').log)"
  done
done
done
for v in tile pf; do
  for c in 3 4; do
    SSTC_MG_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r03j/t${v}$c -o trace --output-format csv -- python3 tools/bench_compact.py --config $c --steps 3 --no-ref --no-files > gpurun_out/r03j/tb_${v}$c.log 2>&1 || exit 5
    python3 tools/trace_compact.py $(find gpurun_out/r03j/t${v}$c -name "*kernel_trace.csv" | head -1) > gpurun_out/r03j/k_${v}$c.txt
    echo "trace $v config $c: $(grep -E 'ck_mg_merge|span us' gpurun_out/r03j/k_${v}$c.txt | tr '\n' ' ')"
  done
done

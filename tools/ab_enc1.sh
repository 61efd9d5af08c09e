#!/bin/bash
# A/B of the compaction encode's dword emit: branches (default) vs sink stores (SSTC_ENC1_SINK=1)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/ab1
SSTC_ENC1_SINK=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_files.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab1/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/ab1/pytest.log; exit 3; }
tail -1 gpurun_out/ab1/pytest.log
for c in 3 4; do
for v in 0 1; do
  if [ $v = 1 ]; then export SSTC_ENC1_SINK=1; else unset SSTC_ENC1_SINK; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ab1/t$c$v -o trace --output-format csv -- python3 tools/bench_compact.py --config $c --steps 5 --no-ref --no-files > gpurun_out/ab1/b$c$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/ab1/b$c$v.log; exit 4; }
  python3 tools/trace_compact.py $(find gpurun_out/ab1/t$c$v -name "*kernel_trace.csv" | head -1) > gpurun_out/ab1/k$c$v.txt
  echo "config $c sink=$v $(grep -o '"matches_reference_fixture": [^]]*' gpurun_out/ab1/b$c$v.log) $(grep enc_lds gpurun_out/ab1/k$c$v.txt)"
done
done

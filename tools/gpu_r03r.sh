#!/bin/bash
# encode offsets kernel: 1024-thread workgroups (cur) vs 256 (head); encode parity first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r03r
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_table.py tests/test_gpu_streams.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03r/pytest.log 2>&1 || { tail -30 gpurun_out/r03r/pytest.log; exit 3; }
tail -1 gpurun_out/r03r/pytest.log
VARIANTS="head cur head cur head cur" ROUNDS=1 bash tools/ab_bench_legs.sh || exit 4

#!/bin/bash
# encode A/B: fused key/value span loads (cur) vs launch-bound variants vs the two-pass copy (nofuse)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r03h
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_table.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03h/pytest.log 2>&1 || { tail -30 gpurun_out/r03h/pytest.log; exit 3; }
tail -1 gpurun_out/r03h/pytest.log
VARIANTS="${VARIANTS:-nofuse cur lb6}" ROUNDS=3 bash tools/ab_bench_legs.sh || exit 4

#!/bin/bash
# DPP wave scans + fused key/value span loads: the GPU tests that exercise every scan, then bench legs A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r03i
timeout -k 10 900 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_table.py tests/test_gpu_compact.py tests/test_gpu_fuzz.py tests/test_gpu_host.py tests/test_gpu_streams.py \
  "tests/test_gpu_configs.py::test_config_full_size_vs_reference" -x -q --timeout 300 --timeout-method thread > gpurun_out/r03i/pytest.log 2>&1 || { tail -30 gpurun_out/r03i/pytest.log; exit 3; }
tail -1 gpurun_out/r03i/pytest.log
VARIANTS="${VARIANTS:-nofuse cur rtshfl w7}" ROUNDS=4 bash tools/ab_bench_legs.sh || exit 4

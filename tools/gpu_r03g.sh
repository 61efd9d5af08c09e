#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r03g
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_table.py tests/test_gpu_compact.py \
  "tests/test_gpu_configs.py::test_config_full_size_vs_reference" -x -q --timeout 300 --timeout-method thread > gpurun_out/r03g/pytest.log 2>&1 || { tail -30 gpurun_out/r03g/pytest.log; exit 3; }
tail -1 gpurun_out/r03g/pytest.log
VARIANTS="${VARIANTS:-head cur m1b nolb}" ROUNDS=3 bash tools/ab_bench_legs.sh || exit 4
VARIANTS="${VARIANTS:-head cur m1b nolb}" CONFIGS="3" KERNELS="enc_lds" bash tools/ab_lib.sh

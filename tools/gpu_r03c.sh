#!/bin/bash
# quick loop for the compaction kernels: compaction parity tests, then the
# previous build (lib/ab/base) against the tree's on configs 3 and 4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r03c
timeout -k 10 600 python -u -m pytest tests/test_gpu_compact.py "tests/test_gpu_configs.py::test_config_full_size_vs_reference" \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/r03c/pytest.log 2>&1 || { tail -30 gpurun_out/r03c/pytest.log; exit 3; }
tail -1 gpurun_out/r03c/pytest.log
VARIANTS="${VARIANTS:-base cur}" CONFIGS="${CONFIGS:-3 4}" KERNELS="${KERNELS:-merge|filter|split}" bash tools/ab_lib.sh 2>&1 | tee gpurun_out/r03c/ab.log

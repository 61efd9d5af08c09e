#!/bin/bash
# round 3: fused last merge pass + filter -- compaction parity tests, then A/B of
# the previous build (lib/ab/base) against the tree's on configs 3, 4, 5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r03b
timeout -k 10 900 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_files.py tests/test_gpu_configs.py \
  tests/test_gpu_aswritten.py tests/test_gpu_cpp_boundary.py tests/test_gpu_dropin.py -x -v --timeout 600 \
  --timeout-method thread > gpurun_out/r03b/pytest.log 2>&1 || { tail -30 gpurun_out/r03b/pytest.log; exit 3; }
tail -2 gpurun_out/r03b/pytest.log
VARIANTS="base cur base cur" CONFIGS="3 4 5" KERNELS="merge|filter|split" bash tools/ab_lib.sh 2>&1 | tee gpurun_out/r03b/ab.log

#!/bin/bash
# compaction job without the table / block count fetch: compaction-related GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r03l
timeout -k 10 600 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_files.py tests/test_gpu_cpp_boundary.py tests/test_gpu_dropin.py tests/test_gpu_lookup.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03l/pytest.log 2>&1 || { tail -40 gpurun_out/r03l/pytest.log; exit 3; }
tail -3 gpurun_out/r03l/pytest.log

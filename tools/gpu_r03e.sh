#!/bin/bash
# codec parity tests (round trip, decode, fuzz, host pipeline), then rt A/B at 256 MiB / 1 GiB
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r03e
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_fuzz.py tests/test_gpu_host.py tests/test_gpu_streams.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/r03e/pytest.log 2>&1 || { tail -30 gpurun_out/r03e/pytest.log; exit 3; }
tail -1 gpurun_out/r03e/pytest.log
timeout -k 10 600 python -u tools/ab_rt.py ${RT_VARIANTS:-rt0,cur} ${RT_ROUNDS:-3} 2>&1 | tee gpurun_out/r03e/ab_rt.log

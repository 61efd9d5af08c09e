#!/bin/bash
# round 2: full-size config parity tests, then the bench with the decode / encode legs
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_configs.py -v -s --timeout 300 --timeout-method thread > gpurun_out/configs.log 2>&1
rc=$?; echo "configs rc=$rc"; tail -12 gpurun_out/configs.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 30 --cpu-seconds 5 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
exit $rc

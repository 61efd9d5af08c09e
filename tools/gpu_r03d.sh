#!/bin/bash
# full GPU suite, bench, compaction-job PMC traffic
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r03d
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r03d/pytest.log 2>&1 || { tail -30 gpurun_out/r03d/pytest.log; exit 3; }
tail -1 gpurun_out/r03d/pytest.log
timeout -k 10 400 python -u bench.py --steps 20 > gpurun_out/r03d/bench.log 2>&1 || { tail -20 gpurun_out/r03d/bench.log; exit 4; }
bash tools/pmc_compact_job.sh 2>&1 | tail -3

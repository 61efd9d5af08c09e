#!/bin/bash
# Round-3 validation on one box: GPU tests, smoke, bench, rocprofv3 stats + PMC of
# the bench and of one config-3 compaction call, configs 3 / 3-overlap / 4 / 5
# (device job, file pipeline, reference driver).  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
out=gpurun_out/final
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 3; }
tail -1 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 4; }
tail -1 $out/smoke.log
timeout -k 10 400 python bench.py --steps 30 > $out/bench.log 2>&1 || { tail -5 $out/bench.log; exit 5; }
echo bench ok
bash tools/profile.sh final > $out/profile.log 2>&1 || { tail -5 $out/profile.log; exit 6; }
echo profile ok
bash tools/pmc_compact_job.sh > $out/pmc_compact.log 2>&1 || { tail -5 $out/pmc_compact.log; exit 7; }
tail -1 $out/pmc_compact.log
for c in "3" "3 --overlap" "4" "5"; do
  tag=$(echo $c | tr -d ' -')
  timeout -k 10 400 python tools/bench_compact.py --config $c --steps 7 > $out/c$tag.log 2>&1 || { echo "config $c failed"; tail -5 $out/c$tag.log; exit 8; }
  echo "== config $c"; tail -1 $out/c$tag.log | cut -c1-600
done

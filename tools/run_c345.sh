#!/bin/bash
# configs 3, 3-overlap, 4 (rank-0 shard), 5 through tools/bench_compact.py (device job,
# file pipeline, the reference driver on the box's host), one JSON line each
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
for c in "3" "3 --overlap" "4" "5"; do
  tag=$(echo $c | tr -d ' -')
  timeout -k 10 400 python tools/bench_compact.py --config $c --steps 5 > gpurun_out/c$tag.log 2>&1 || { echo "config $c failed"; tail -5 gpurun_out/c$tag.log; exit 3; }
  echo "== config $c"; tail -1 gpurun_out/c$tag.log | cut -c1-400
done

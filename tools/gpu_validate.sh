#!/bin/bash
# One GPU-box validation pass, by stages (default: all).  Stops at the first failure.
#   bash tools/gpu_validate.sh <outdir> [tests] [smoke] [bench] [trace] [pmc] [configs]
#   tests    pytest -m gpu (one process)
#   smoke    __graft_entry__.smoke()
#   bench    python bench.py --steps 30
#   profile  tools/profile.sh: rocprofv3 kernel trace + stats and FETCH / WRITE passes of the bench
#   trace    rocprofv3 kernel traces of the compaction job, configs 3 4 5 (tools/trace_compact.py tables)
#   pmc      FETCH_SIZE / WRITE_SIZE of one config-3, one config-4 and one config-5 compaction call
#   configs  tools/bench_compact.py configs 3, 3-overlap, 4, 5 with the reference driver beside them
# Env: PYTEST_K (pytest -k filter), CONFIGS (trace configs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
out=gpurun_out/${1:-val}; shift
stages=${*:-tests smoke bench profile trace pmc configs}
mkdir -p $out
has() { [[ " $stages " == *" $1 "* ]]; }
if has tests; then
  kf=(); [ -n "$PYTEST_K" ] && kf=(-k "$PYTEST_K")
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread "${kf[@]}" > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 3; }
  tail -1 $out/pytest_gpu.log
fi
if has smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 4; }
  tail -1 $out/smoke.log
fi
if has bench; then
  timeout -k 10 500 python bench.py --steps 30 > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 5; }
  tail -1 $out/bench.log | cut -c1-1500
fi
if has profile; then
  bash tools/profile.sh $(basename $out) > $out/profile.log 2>&1 || { tail -5 $out/profile.log; exit 9; }
  echo profile ok
fi
if has trace; then
  for c in ${CONFIGS:-3 4 5}; do
    timeout -k 10 300 rocprofv3 --kernel-trace -d $out/t$c -o trace --output-format csv -- python3 tools/bench_compact.py --config $c --steps 3 --no-ref --no-files > $out/b$c.log 2>&1 || { echo "trace $c failed"; tail -20 $out/b$c.log; exit 6; }
    python3 tools/trace_compact.py $(find $out/t$c -name "*kernel_trace.csv" | head -1) > $out/k$c.txt || exit 6
    echo "== config $c kernels"; head -14 $out/k$c.txt
  done
fi
if has pmc; then
  bash tools/pmc_compact_job.sh > $out/pmc_c3.log 2>&1 || { tail -5 $out/pmc_c3.log; exit 7; }
  cp gpurun_out/pmc_compact/summary.json $out/pmc_c3.json; tail -1 $out/pmc_c3.log
  bash tools/pmc_compact_job.sh --config 4 --steps 1 --no-ref --no-files > $out/pmc_c4.log 2>&1 || { tail -5 $out/pmc_c4.log; exit 7; }
  cp gpurun_out/pmc_compact/summary.json $out/pmc_c4.json; tail -1 $out/pmc_c4.log
  bash tools/pmc_compact_job.sh --config 5 --steps 1 --no-ref --no-files > $out/pmc_c5.log 2>&1 || { tail -5 $out/pmc_c5.log; exit 7; }
  cp gpurun_out/pmc_compact/summary.json $out/pmc_c5.json; tail -1 $out/pmc_c5.log
fi
if has configs; then
  for c in "3" "3 --overlap" "4" "5"; do
    tag=$(echo $c | tr -d ' -')
    timeout -k 10 400 python tools/bench_compact.py --config $c --steps 7 > $out/c$tag.log 2>&1 || { echo "config $c failed"; tail -5 $out/c$tag.log; exit 8; }
    echo "== config $c"; tail -1 $out/c$tag.log | cut -c1-600
  done
fi
exit 0

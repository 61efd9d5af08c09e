#!/bin/bash
# SQ + traffic counters of the compaction job's kernels (config 3 by default),
# one rocprofv3 pass per counter group.  Usage: bash tools/pmc_ck.sh <tag> [bench_compact args]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
tag=${1:-c3}; shift
args=${*:---config 3 --steps 1 --no-ref --no-files}
out=gpurun_out/pmcck_$tag
mkdir -p $out
run() { # pass-name counters...
  local p=$1; shift
  timeout -k 10 -s KILL 150 rocprofv3 --pmc "$@" -d $out/$p -o $p --output-format csv -- python3 tools/bench_compact.py $args > $out/$p.log 2>&1 || { echo "pass $p failed"; tail -5 $out/$p.log; exit 4; }
}
run a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
run b SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU
run f FETCH_SIZE
run w WRITE_SIZE
python3 - "$out" <<'PY'
import csv, glob, collections, sys
out = sys.argv[1]
agg = collections.defaultdict(float); cnt = collections.Counter()
for f in sorted(glob.glob(out + "/*/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"].split("(")[0][-40:], r["Counter_Name"]); agg[k] += float(r["Counter_Value"]); cnt[k] += 1
with open(out + "/summary.txt", "w") as fo:
    for k, v in sorted(agg.items()):
        line = f"{k[0]:40s} {k[1]:24s} {v / max(1, cnt[k]):16.0f} (launches {cnt[k]})"
        print(line); fo.write(line + "\n")
PY

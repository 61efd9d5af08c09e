#!/bin/bash
# SQ counters of the compaction merge kernel (config 3, SSTC_MERGE=1), two passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp SSTC_MERGE=${SSTC_MERGE:-1}
mkdir -p gpurun_out/pmcm
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/pmcm/a -o a --output-format csv -- python3 tools/bench_compact.py --config 3 --steps 1 --no-ref --no-files > gpurun_out/pmcm/a.log 2>&1 || { echo "pass a failed"; tail -5 gpurun_out/pmcm/a.log; exit 4; }
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU -d gpurun_out/pmcm/b -o b --output-format csv -- python3 tools/bench_compact.py --config 3 --steps 1 --no-ref --no-files > gpurun_out/pmcm/b.log 2>&1 || { echo "pass b failed"; tail -5 gpurun_out/pmcm/b.log; exit 5; }
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmcm/*/*counter_collection.csv")):
    agg = collections.defaultdict(float); cnt = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "merge" in r["Kernel_Name"] or "decode_kernel" in r["Kernel_Name"]:
            k = (r["Kernel_Name"][:40], r["Counter_Name"]); agg[k] += float(r["Counter_Value"]); cnt[k] += 1
    for k, v in sorted(agg.items()):
        print(k, v / max(1, cnt[k]))
PY

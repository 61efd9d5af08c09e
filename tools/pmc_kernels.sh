#!/bin/bash
# SQ + HBM counters of every kernel of one compaction job (tools/bench_compact.py
# --config C --steps 1), one rocprofv3 --pmc pass per counter group (the TCC
# and SQ slot limits of MI355X_MICROARCH.md), summarised per kernel (the job's
# last dispatch of each kernel; FETCH_SIZE x 2 for gfx950, KiB -> bytes).
#   bash tools/pmc_kernels.sh <outdir> [config]
# Env: KERNELS (regex of kernel names to keep in the summary, default all)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
out=gpurun_out/${1:-pmc_k}
cfg=${2:-3}
mkdir -p $out
args="--config $cfg --steps 1 --no-ref --no-files"
run() { local p=$1; shift
  timeout -k 10 -s KILL 150 rocprofv3 --pmc "$@" -d $out/$p -o $p --output-format csv -- python3 tools/bench_compact.py $args > $out/$p.log 2>&1 || { echo "pass $p failed"; tail -3 $out/$p.log; exit 4; }; }
run a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES
run b SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INSTS_FLAT
run f FETCH_SIZE
run w WRITE_SIZE
python3 - $out "${KERNELS:-.}" <<'PY'
import csv, glob, re, sys
out, keep = sys.argv[1], re.compile(sys.argv[2])
last = {}
def short(n):
    n = re.sub(r"\(.*", "", n.replace("void ", "").replace("(anonymous namespace)::", ""))
    return n.replace("sstc::", "")
for f in sorted(glob.glob(out + "/*/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        if "__amd_rocclr" in k or not keep.search(k):
            continue
        key = (k, r["Counter_Name"])
        d = int(r["Dispatch_Id"])
        v = float(r["Counter_Value"])
        if key not in last or d > last[key][0]:
            last[key] = (d, v)
        elif d == last[key][0]:
            last[key] = (d, last[key][1] + v)
with open(out + "/summary.txt", "w") as fo:
    for (k, c), (d, v) in sorted(last.items()):
        if c == "FETCH_SIZE":
            v *= 2 * 1024
        elif c == "WRITE_SIZE":
            v *= 1024
        line = f"{k:34s} {c:24s} {v:18.0f}"
        print(line)
        fo.write(line + "\n")
PY

#!/bin/bash
# kernel trace + SQ / HBM counters of the config-2 encode leg (tools/enc_leg.py), one pass per group
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
out=gpurun_out/pmc_enc
mkdir -p $out
timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --stats -d $out/trace -o trace --output-format csv -- python3 tools/enc_leg.py > $out/trace.log 2>&1 || { echo trace failed; tail -5 $out/trace.log; exit 4; }
run() { local p=$1; shift
  timeout -k 10 -s KILL 120 rocprofv3 --pmc "$@" -d $out/$p -o $p --output-format csv -- python3 tools/enc_leg.py > $out/$p.log 2>&1 || { echo "pass $p failed"; tail -3 $out/$p.log; exit 4; }; }
run a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES
run b SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU
run f FETCH_SIZE
run w WRITE_SIZE
python3 - $out <<'PY'
import csv, glob, collections, re, sys
out = sys.argv[1]
agg = collections.defaultdict(list)
def short(n):
    n = re.sub(r"\(.*", "", n.replace("void ", ""))
    return n.split("::")[-1]
for f in sorted(glob.glob(out + "/*/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "__amd_rocclr" in r["Kernel_Name"]:
            continue
        agg[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
with open(out + "/summary.txt", "w") as fo:
    for (k, c), v in sorted(agg.items()):
        v = sorted(v)[len(v) // 2]
        line = f"{k:28s} {c:24s} {v:16.0f}"
        print(line); fo.write(line + "\n")
PY

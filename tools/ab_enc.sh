#!/bin/bash
# enc_lds_kernel in the compaction job: interleaved (config 3) vs key-range
# inputs, kernel trace + FETCH_SIZE / WRITE_SIZE passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
for lay in "" "--ranges"; do
  tag=il; [ -n "$lay" ] && tag=rg
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/e_$tag -o t --output-format csv -- python3 $R/tools/bench_compact.py --no-ref --no-files --steps 1 $lay > $R/gpurun_out/e_$tag.log 2>&1 || exit 4
  echo "== $tag"; python3 $R/tools/trace_compact.py $(ls $R/gpurun_out/e_$tag/*kernel_trace.csv) | head -4
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/f_$tag -o f --output-format csv -- python3 $R/tools/bench_compact.py --no-ref --no-files --steps 1 $lay > $R/gpurun_out/f_$tag.log 2>&1 || exit 5
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/w_$tag -o w --output-format csv -- python3 $R/tools/bench_compact.py --no-ref --no-files --steps 1 $lay > $R/gpurun_out/w_$tag.log 2>&1 || exit 6
  python3 - $R/gpurun_out/f_$tag $R/gpurun_out/w_$tag <<'PY'
import csv, glob, sys
for d in sys.argv[1:]:
    f = glob.glob(d + "/*counter_collection.csv")[0]
    rows = [r for r in csv.DictReader(open(f)) if "enc_lds" in r["Kernel_Name"] or "decode_kernel" in r["Kernel_Name"] or "merge_tile" in r["Kernel_Name"] or "gather" in r["Kernel_Name"]]
    agg = {}
    for r in rows:
        k = (r["Kernel_Name"].split("(")[0][-24:], r["Counter_Name"])
        agg[k] = agg.get(k, 0) + float(r["Counter_Value"])
    for k, v in agg.items():
        print(k, f"{v / 1024:.1f} MiB(KiB units)")
PY
done

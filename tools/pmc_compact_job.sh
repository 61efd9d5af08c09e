#!/bin/bash
# HBM traffic of ONE sstc_compact call (config 3 by default) from two rocprofv3
# PMC passes (FETCH_SIZE, WRITE_SIZE: separate passes, MI355X_MICROARCH.md
# TCC slots), summed over the kernels of the job's last call (from its last
# count_scan_kernel / count_kernel dispatch on); FETCH_SIZE doubled (gfx950 wide-stream correction).
# Writes gpurun_out/pmc_compact/summary.json; copy it to profiles/pmc_compact.json.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
out=gpurun_out/pmc_compact
mkdir -p $out
args=${*:---config 3 --steps 1 --no-ref --no-files}
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $c -d $out/$c -o $c --output-format csv -- python3 tools/bench_compact.py $args > $out/$c.log 2>&1 || { echo "pass $c failed"; tail -5 $out/$c.log; exit 4; }
done
python3 - "$out" "$args" <<'PY'
import csv, glob, json, sys
out, args = sys.argv[1], sys.argv[2]
tag = next((f"config{c}" for c in "345" if f"--config {c}" in args), args)  # what bench.py's legs look up
res = {"workload": tag, "args": args, "note":
       "one sstc_compact call: every kernel from its last count_scan_kernel (count_kernel) dispatch on; FETCH_SIZE x 2 (gfx950), KiB"}
per = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    rows = []
    for f in glob.glob(f"{out}/{c}/**/*counter_collection.csv", recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == c]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    start = max(i for i, r in enumerate(rows) if "count_kernel" in r["Kernel_Name"] or "count_scan_kernel" in r["Kernel_Name"])
    tot = 0.0
    for r in rows[start:]:
        if r["Kernel_Name"].startswith("__amd_rocclr"):  # the caller's copies after the call, not the job
            continue
        v = float(r["Counter_Value"]) * 1024 * (2 if c == "FETCH_SIZE" else 1)
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("sstc::", "").split("(")[0]
        per.setdefault(k, {}).setdefault(c, 0.0)
        per[k][c] += v
        tot += v
    res[c + "_bytes"] = tot
res["hbm_bytes_per_call"] = res["FETCH_SIZE_bytes"] + res["WRITE_SIZE_bytes"]
res["per_kernel"] = {k: {c: round(v / 1e6, 1) for c, v in d.items()} for k, d in
                     sorted(per.items(), key=lambda kv: -sum(kv[1].values()))}
res["per_kernel_unit"] = "MB"
json.dump(res, open(out + "/summary.json", "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "per_kernel"}))
PY

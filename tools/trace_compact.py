"""Print the per-kernel timeline of the last sstc_compact call in a rocprofv3
kernel trace (tools/profile of tools/bench_compact.py)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "sstc::decode_kernel" in r["Kernel_Name"]]
# the job's first kernel: count_scan_kernel (count_kernel + scan + ck_start_kernel
# before round 5's end), the last one before the job's decode
start = max(i for i in range(idx[-1]) if "count_kernel" in rows[i]["Kernel_Name"]
            or "count_scan_kernel" in rows[i]["Kernel_Name"])
t0 = int(rows[start]["Start_Timestamp"])
last = t0
agg = {}
for r in rows[start:]:
    n = r["Kernel_Name"].replace("sstc::(anonymous namespace)::", "").replace("sstc::", "").split("(")[0]
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if n.startswith("__amd_rocclr_copyBuffer") and (en - st) > 100_000:
        break
    agg.setdefault(n, [0, 0.0])
    agg[n][0] += 1
    agg[n][1] += (en - st) / 1e3
    last = en
for n, (c, us) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{n[:32]:32s} calls={c:4d} total_us={us:9.1f}")
print(f"span us {(last - t0) / 1e3:.1f}  kernel sum us {sum(v[1] for v in agg.values()):.1f}")
# idle gaps between consecutive kernels of the job (host syncs, launch latency)
gaps = []
prev = None
for r in rows[start:]:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    n = r["Kernel_Name"].replace("sstc::(anonymous namespace)::", "").replace("sstc::", "").split("(")[0]
    if n.startswith("__amd_rocclr_copyBuffer") and (en - st) > 100_000:
        break
    if prev is not None:
        gaps.append(((st - prev[1]) / 1e3, prev[0][:28], n[:28]))
    prev = (n, en)
print(f"gaps total us {sum(g[0] for g in gaps):.1f} over {len(gaps)} boundaries; > 5 us:")
for g in gaps:
    if g[0] > 5:
        print(f"  {g[0]:7.1f} us  {g[1]} -> {g[2]}")

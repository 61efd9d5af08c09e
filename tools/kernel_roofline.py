"""Per-kernel HBM rate of one compaction call: PMC bytes (tools/pmc_compact_job.sh
summary, FETCH x 2 + WRITE, MB per kernel) over the kernel's time in a trace of
the same config (tools/trace_compact.py table), against 8 TB/s.

    python tools/kernel_roofline.py profiles/r05_final/pmc_c3.json profiles/r05_final/config3_kernels.txt
"""
import json
import re
import sys


def main():
    pmc = json.load(open(sys.argv[1]))["per_kernel"]
    times = {}
    for ln in open(sys.argv[2]):
        m = re.match(r"(.+?)\s+calls=\s*(\d+)\s+total_us=\s*([0-9.]+)", ln)
        if m:
            times[m.group(1).strip()] = (int(m.group(2)), float(m.group(3)))
    rows = []
    for name, v in pmc.items():
        key = next((k for k in times if name.startswith(k.rstrip(".").split("(")[0]) or k.startswith(name[:30])), None)
        if key is None:
            continue
        calls, us = times[key]
        mb = v["FETCH_SIZE"] + v["WRITE_SIZE"]
        rows.append((us, name, calls, mb, mb / us if us else 0.0))  # MB / us = TB/s
    rows.sort(reverse=True)
    print("| kernel | calls | µs | HBM MB (FETCH x 2 + WRITE) | TB/s | of 8 TB/s |")
    print("|---|---|---|---|---|---|")
    for us, name, calls, mb, tbs in rows:
        print(f"| `{name[:48]}` | {calls} | {us:.1f} | {mb:.0f} | {tbs:.2f} | {tbs / 8:.2f} |")


if __name__ == "__main__":
    main()

"""Host-side phase times of the drop-in compaction (oracle/_ref/compact_dropin:
the reference's unmodified db/compact.cc over the drop-in TableReaderIterator
and TableBuilder) on one BASELINE config, with SSTC_TRACE_HOST=1.

    python tools/dropin_trace.py --config 5

Inputs are written by the flush-path sstc::TableBuilder (GPU encode); prints the
PickCompact time and the summed [sstc] phase lines."""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lsm-kv-storage_amd"))


def key_range(rec):
    ko, kl = rec["key_off"], rec["key_len"]
    first = bytes(rec["key_src"][int(ko[0]):int(ko[0]) + int(kl[0])])
    last = bytes(rec["key_src"][int(ko[-1]):int(ko[-1]) + int(kl[-1])])
    return first, last


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=5)
    ap.add_argument("--repeat", type=int, default=1)
    ap.add_argument("--walk", type=int, nargs="*", default=[])
    ap.add_argument("--pf", nargs="*", default=["24"])
    args = ap.parse_args()
    import sstcodec
    from sstcodec import workload as W
    from sstcodec.table import build_table
    exe = os.path.join(ROOT, "oracle", "_ref", "compact_dropin")
    td = tempfile.mkdtemp(prefix="sstc_dropin_trace_", dir=os.environ.get("TMPDIR", "/tmp"))
    codec = sstcodec.Codec(0)
    cmd = [exe, os.path.join(td, "db"), "4096", str(32 << 20)]
    os.makedirs(os.path.join(td, "db"))
    for i, rec in enumerate(W.config_inputs(args.config)):
        p = os.path.join(td, f"in{i}.sst")
        fs, _ = build_table(codec, p, rec, 4096)
        lo, hi = key_range(rec)
        cmd += [p, str(fs), lo.hex() or "-", hi.hex() or "-"]
    codec.close()
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_pick_compact")
    files = cmd[4:]
    walk = [a for i, a in enumerate(files) if i % 4 < 2]
    for level in args.walk:  # the loop's parts (ref_pick_compact.cc --walk)
        for e, tag, pf in [(exe, "dropin", p) for p in args.pf] + [(ref, "reference", None)]:
            if level == 2 and tag == "reference":
                continue
            env = dict(os.environ, **({"SSTC_DROPIN_PF": pf} if pf is not None else {}))
            r = subprocess.run([e, "--walk", str(level)] + walk, capture_output=True, text=True, env=env)
            print(tag, "pf", pf, r.stdout.strip(), r.stderr[-500:] if r.returncode else "", flush=True)
    for rep in range(args.repeat - 1):  # untraced runs: PickCompact time only
        d = os.path.join(td, f"db{rep}")
        os.makedirs(d)
        r = subprocess.run([exe, d] + cmd[2:], capture_output=True, text=True)
        print("untraced", [ln for ln in r.stdout.splitlines() if ln.startswith("time")], flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True, env=dict(os.environ, SSTC_TRACE_HOST="1"))
    print("rc", r.returncode, [ln for ln in r.stdout.splitlines() if ln.startswith(("time", "init"))])
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    last = ""
    for ln in r.stderr.splitlines():
        m = re.match(r"\[sstc\] (.*?) ([0-9.]+) ms$", ln)
        if m:
            tot[m.group(1)] += float(m.group(2))
            cnt[m.group(1)] += 1
        elif ln.startswith("[sstc] Finish"):
            tot["Finish"] += float(ln.split(": ")[1].split(" ms")[0])
            cnt["Finish"] += 1
            for part, v in re.findall(r"(H2D \+ encode|D2H|meta|pwrite|fsync) ([0-9.]+)", ln):
                tot["Finish: " + part] += float(v)
                cnt["Finish: " + part] += 1
            last = ln
    for k, v in tot.items():
        print(f"{k}: {v:.1f} ms over {cnt[k]}")
    print(last)
    if r.returncode:
        print(r.stderr[-2000:])
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_pick_compact")
    if os.path.exists(ref):  # the reference as written on the same tables (heap kept mapped, as in the tests)
        os.makedirs(os.path.join(td, "db_ref"))
        rr = subprocess.run([ref, os.path.join(td, "db_ref")] + cmd[2:], capture_output=True, text=True,
                            env=dict(os.environ, GLIBC_TUNABLES="glibc.malloc.trim_threshold=17179869184"))
        print("reference rc", rr.returncode, [ln for ln in rr.stdout.splitlines() if ln.startswith("time")])


if __name__ == "__main__":
    main()

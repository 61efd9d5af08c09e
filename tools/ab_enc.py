"""A/B of encode variants, one process each, interleaved rounds: the config-2
encode leg (sstc_encode_blocks over 65 536 blocks' decoded records), median of
7 HIP-event spans of 30 calls, output checked.  A variant is a library build
lsm-kv-storage_amd/lib/ab/<name>/ or 'cur' (the tree's).
    python tools/ab_enc.py cur,nofuse [rounds]"""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, sys, ctypes, statistics, torch
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + "/lsm-kv-storage_amd")
import bench, sstcodec
dev = torch.device("cuda", 0)
codec = sstcodec.Codec(0)
nb = 65536
src, off, ln = bench.make_blocks(codec, dev, nb, 0)
P = lambda t: ctypes.c_void_p(t.data_ptr())
rec_base = codec.count(src, off, ln)
table, _, status = codec.decode(src, off, ln, rec_base=rec_base)
c = table.c()
first = torch.arange(0, table.n + 1, bench.PER_BLOCK, dtype=torch.int64, device=dev)
dst = torch.zeros_like(src)
oo = torch.empty(nb + 1, dtype=torch.int64, device=dev); ol = torch.empty(nb, dtype=torch.int64, device=dev)
call = lambda: codec.lib.sstc_encode_blocks(codec.h, P(src), P(src), c, table.n, P(first), nb, 0, P(dst), P(oo), P(ol))
codec._stream()
for _ in range(5): assert call() == 0
s = torch.cuda.current_stream(dev)
ms = []
for _ in range(7):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record(s)
    for _ in range(30): call()
    e1.record(s); torch.cuda.synchronize()
    ms.append(e0.elapsed_time(e1) / 30)
print(json.dumps({"ms": round(statistics.median(ms), 5), "min": round(min(ms), 5), "ok": bool(torch.equal(dst, src))}))
'''
res = {}
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
for v in sys.argv[1].split(",") * rounds:
    env = dict(os.environ)
    env.pop("SSTC_LIB_PATH", None)
    if v != "cur":
        env["SSTC_LIB_PATH"] = os.path.join(ROOT, "lsm-kv-storage_amd", "lib", "ab", v, "libsstcodec.so")
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=300)
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    d = json.loads(line[-1]) if line else {"error": r.stderr[-800:]}
    res.setdefault(v, []).append(d)
    print(v, d, flush=True)
alg = 65536 * 4188 + 1835008 * 149
for v, ds in res.items():
    m = [d["ms"] for d in ds if "ms" in d]
    if m:
        print(f"{v:10s} median {statistics.median(m):.4f} ms  frac {alg / (statistics.median(m) * 1e-3) / 8e12:.4f}  runs {m}")

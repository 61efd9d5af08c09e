"""A/B of rt_kernel variants, one process each: HIP-event time of
sstc_roundtrip_blocks at config 2 (65 536 blocks) and 4x (1 GiB), identity
checked.  A variant is a library build lsm-kv-storage_amd/lib/ab/<name>/
(tools/ab_build.sh) or 'cur' (the tree's).   python tools/ab_rt.py cur,p1,p2 [rounds]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, sys, ctypes, torch
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + "/lsm-kv-storage_amd")
import bench, sstcodec
dev = torch.device("cuda", 0)
codec = sstcodec.Codec(0)
out = {}
for nb in (65536, 262144):
    src, off, ln = bench.make_blocks(codec, dev, nb, 0)
    dst = torch.empty_like(src)
    ol = torch.empty(nb, dtype=torch.int64, device=dev); st = torch.empty(nb, dtype=torch.int32, device=dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    args = (P(src), P(dst), P(off), P(ln), nb, 0, P(ol), P(st))
    codec._stream()
    for _ in range(3): codec.roundtrip_raw(*args)
    s = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record(s)
    for _ in range(20): codec.roundtrip_raw(*args)
    e1.record(s); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    ok = bool(torch.equal(dst, src)) and bool((st == 0).all())
    out[nb] = {"ms": round(ms, 4), "TBps": round(2 * nb * 4188 / ms / 1e9, 3), "ok": ok}
    del src, dst, off, ln; torch.cuda.empty_cache()
print(json.dumps(out))
'''
res = {}
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 1
for v in sys.argv[1].split(",") * rounds:
    env = dict(os.environ)
    env.pop("SSTC_LIB_PATH", None)
    if v != "cur":
        env["SSTC_LIB_PATH"] = os.path.join(ROOT, "lsm-kv-storage_amd", "lib", "ab", v, "libsstcodec.so")
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=300)
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    res[v] = json.loads(line[-1]) if line else {"error": r.stderr[-800:]}
    print(v, res[v], flush=True)

"""A/B encode-kernel variants (SSTC_ENC_VARIANT, read once per process): one
process per variant, uniform config-2 records in order and with an
interleaved source order (what a k-way merge produces); HIP-event time of
sstc_encode_blocks, output checked against the in-order encode of variant 0.

    python tools/ab_encode.py 0,1,2,3
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, sys, numpy as np, torch
sys.path.insert(0, sys.argv[1] + "/lsm-kv-storage_amd")
import sstcodec
from sstcodec import workload as W
from sstcodec.codec import RecordTable
dev = torch.device("cuda", 0)
codec = sstcodec.Codec(0)
n = 65536 * 28
rec = W.uniform_records(n)
first = torch.arange(0, n + 1, 28, dtype=torch.int64, device=dev)
ks = torch.from_numpy(rec["key_src"]).to(dev)
vs = torch.from_numpy(rec["val_src"]).to(dev)
out = {}
ref = None
for name, perm in (("inorder", None), ("interleaved", np.arange(n).reshape(8, -1).T.reshape(-1))):
    r = dict(rec)
    if perm is not None:
        for k in ("key_off", "val_off"):
            r[k] = rec[k][perm]
    t = RecordTable.from_numpy(r, dev)
    dst, off, ln = codec.encode(t, ks, vs, first)
    torch.cuda.synchronize()
    h = int(dst.view(torch.int64).sum().item())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s = torch.cuda.current_stream(dev)
    e0.record(s)
    for _ in range(20):
        codec.encode(t, ks, vs, first, dst=dst)
    e1.record(s)
    torch.cuda.synchronize()
    out[name] = {"ms": e0.elapsed_time(e1) / 20, "sum": h}
print(json.dumps(out))
'''

res = {}
for v in sys.argv[1].split(","):
    env = dict(os.environ, SSTC_ENC_VARIANT=v)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=300)
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    res[v] = json.loads(line[-1]) if line else {"error": r.stderr[-500:]}
    print(v, res[v], flush=True)
print(json.dumps(res))

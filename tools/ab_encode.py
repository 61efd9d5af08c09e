"""A/B encode-kernel variants (SSTC_ENC_VARIANT) in one process: uniform
records in order (config 2 shape) and the same records with an interleaved
source order (what a k-way merge produces)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lsm-kv-storage_amd"))
import sstcodec  # noqa: E402
from sstcodec import workload as W  # noqa: E402
from sstcodec.codec import RecordTable  # noqa: E402

variants = sys.argv[1].split(",")
dev = torch.device("cuda", 0)
codec = sstcodec.Codec(0)
n = 65536 * 28
rec = W.uniform_records(n)
first = torch.arange(0, n + 1, 28, dtype=torch.int64, device=dev)
ks = torch.from_numpy(rec["key_src"]).to(dev)
vs = torch.from_numpy(rec["val_src"]).to(dev)
res = {}
for name, perm in (("inorder", None), ("interleaved", np.arange(n).reshape(8, -1).T.reshape(-1))):
    r = dict(rec)
    if perm is not None:
        for k in ("key_off", "val_off"):
            r[k] = rec[k][perm]
    t = RecordTable.from_numpy(r, dev)
    dst, off, ln = codec.encode(t, ks, vs, first)
    times = {v: [] for v in variants}
    for rnd in range(5):
        for v in variants:
            os.environ["SSTC_ENC_VARIANT"] = v
            codec.encode(t, ks, vs, first, dst=dst)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                codec.encode(t, ks, vs, first, dst=dst)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / 5)
    for v in variants:
        res[f"{name}/v{v}"] = round(float(np.median(times[v])), 4)
print(json.dumps(res, indent=1))

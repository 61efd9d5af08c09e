"""Encode timing of a config-5-shaped record set (Zipf values up to 64 KiB:
most blocks past an LDS slot) through sstc_encode_blocks; prints us per call.
Used to A/B the large-block paths (tools/ab_encoff.sh)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lsm-kv-storage_amd"))
import sstcodec  # noqa: E402
from sstcodec import workload as W  # noqa: E402
from sstcodec.codec import RecordTable  # noqa: E402

codec = sstcodec.Codec(0)
dev = codec.device
rec = W.compaction_inputs(1, 5000, 20000, seed=55, vmin=8, vmax=65536, zipf=1.1, p_delete=0.1)[0]
tab = RecordTable.from_numpy(rec, dev)
first = codec.segment(tab, 4096)
ks = torch.from_numpy(np.ascontiguousarray(rec["key_src"], np.uint8)).to(dev)
vs = torch.from_numpy(np.ascontiguousarray(rec["val_src"], np.uint8)).to(dev)
dst, off, ln = codec.encode(tab, ks, vs, first)
torch.cuda.synchronize()
ts = []
for _ in range(20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    codec.encode(tab, ks, vs, first, dst=dst)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
print({"blocks": int(first.numel() - 1), "bytes": int(dst.numel()), "us_median": round(float(np.median(ts)) * 1e6, 1),
       "sha_head": int(dst[:1 << 20].to(torch.int64).sum().item())})

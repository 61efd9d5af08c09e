"""A/B the round-trip kernel variants in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24).  SSTC_RT_VARIANT selects the variant
per call.  Prints median/min per-call ms for each variant and block count."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "lsm-kv-storage_amd"))
import bench  # noqa: E402
import sstcodec  # noqa: E402

variants = sys.argv[1].split(",") if len(sys.argv) > 1 else ["0", "1"]
sizes = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [65536, 262144]
rounds = 7
dev = torch.device("cuda", 0)
codec = sstcodec.Codec(0)
res = {}
for nb in sizes:
    src, off, ln = bench.make_blocks(codec, dev, nb, 0)
    dst = torch.empty_like(src)
    out_len = torch.empty(nb, dtype=torch.int64, device=dev)
    status = torch.empty(nb, dtype=torch.int32, device=dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    args = (P(src), P(dst), P(off), P(ln), nb, 0, P(out_len), P(status))
    codec._stream()
    times = {v: [] for v in variants}
    for r in range(rounds):
        for v in variants:
            os.environ["SSTC_RT_VARIANT"] = v
            for _ in range(3):
                codec.roundtrip_raw(*args)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                codec.roundtrip_raw(*args)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / 20)
            dst.zero_()
            codec.roundtrip_raw(*args)
            torch.cuda.synchronize()
            if v not in ("8", "9"):
                assert torch.equal(dst, src) and bool((status == 0).all()), f"variant {v} wrong"
    for v in variants:
        t = np.array(times[v])
        gbps = 2 * nb * 4188 / (np.median(t) * 1e-3) / 1e9
        res[f"{nb}/v{v}"] = {"median_ms": float(np.median(t)), "min_ms": float(t.min()), "GBps": round(gbps, 1)}
    del src, dst
print(json.dumps(res, indent=1))

"""PCIe probe for the e2e leg of bench.py: pinned H2D alone, D2H alone, both
at once, and the native chunked H2D -> rt_kernel -> D2H pipeline
(sstc_roundtrip_host) over chunk sizes (config-2 blocks).  Prints one JSON line per case."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "lsm-kv-storage_amd"))
import bench  # noqa: E402
import sstcodec  # noqa: E402

dev = torch.device("cuda", 0)
codec = sstcodec.Codec(0)
nb = 65536
src, off, ln = bench.make_blocks(codec, dev, nb, 0)
nbytes = src.numel()
h_src = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
h_dst = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
h_src.copy_(src.cpu())
d_a = torch.empty_like(src)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def h2d():
    d_a.copy_(h_src, non_blocking=True)


def d2h():
    h_dst.copy_(src, non_blocking=True)


def both():
    with torch.cuda.stream(s1):
        d_a.copy_(h_src, non_blocking=True)
    with torch.cuda.stream(s2):
        h_dst.copy_(src, non_blocking=True)


for name, fn in (("h2d", h2d), ("d2h", d2h), ("both", both)):
    el = timed(fn)
    print(json.dumps({"case": name, "GBps_each_dir": round(nbytes / el / 1e9, 2)}), flush=True)

# native pipeline (sstc_roundtrip_host): per-chunk enqueue cost is C++, not Python
o = off.cpu().numpy().view("u8")
n = ln.cpu().numpy().view("u8")
for chunk_mb in (2, 4, 8, 16, 32):
    cb = chunk_mb << 20
    codec.roundtrip_host(h_src, h_dst, o, n, chunk_bytes=cb)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        codec.roundtrip_host(h_src, h_dst, o, n, chunk_bytes=cb)
    el = (time.perf_counter() - t0) / 5
    ok = bool(torch.equal(h_dst, h_src))
    print(json.dumps({"case": "native", "chunk_MiB": chunk_mb, "GiBps": round(nbytes / el / 2 ** 30, 2),
                      "verified": ok}), flush=True)

"""A/B of the per-step launch overhead of the config-2 round trip: back-to-back
launches with an event between every launch (bench.py), with events only at
the ends, and the same K launches replayed from one HIP graph.  Prints
microseconds per step (wall and events)."""
import ctypes
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
nb, K = 65536, 50
src, off, ln = bench.make_blocks(codec, dev, nb, 0)
dst = torch.empty_like(src)
out_len = torch.empty(nb, dtype=torch.int64, device=dev)
status = torch.empty(nb, dtype=torch.int32, device=dev)
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
args = (P(src), P(dst), P(off), P(ln), nb, 0, P(out_len), P(status))


def plain(stream, per_launch_events):
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evs[0].record(stream)
    for i in range(K):
        codec.roundtrip_raw(*args)
        if per_launch_events:
            evs[i + 1].record(stream)
    if not per_launch_events:
        evs[K].record(stream)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / K * 1e6
    return wall, evs[0].elapsed_time(evs[K]) / K * 1e3


res = {}
for rnd in range(3):
    s = torch.cuda.current_stream(dev)
    codec._stream()
    for _ in range(5):
        codec.roundtrip_raw(*args)
    res.setdefault("events_each", []).append(plain(s, True))
    res.setdefault("events_ends", []).append(plain(s, False))
    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream(dev)
    with torch.cuda.stream(cs):
        codec._stream()
        with torch.cuda.graph(g, stream=cs):
            codec._stream()
            for _ in range(K):
                codec.roundtrip_raw(*args)
    codec._stream()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(s)
    g.replay()
    e1.record(s)
    torch.cuda.synchronize()
    res.setdefault("graph", []).append(((time.perf_counter() - t0) / K * 1e6, e0.elapsed_time(e1) / K * 1e3))
    ok = bool(torch.equal(dst, src))
for k, v in res.items():
    print(json.dumps({"case": k, "us_per_step_wall": [round(a, 1) for a, _ in v],
                      "us_per_step_events": [round(b, 1) for _, b in v], "identity": ok}), flush=True)

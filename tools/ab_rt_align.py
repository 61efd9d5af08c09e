"""rt_kernel at 1 GiB: back-to-back 4188 B blocks (shared 16 B edge chunks
written byte-wise by both neighbours) vs the same blocks at a 16 B-aligned
4192 B stride (no shared chunks).  Prints ms per launch and the fraction of
8 TB/s for each layout."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "lsm-kv-storage_amd"))
import bench  # noqa: E402
import sstcodec  # noqa: E402

codec = sstcodec.Codec(0)
dev = codec.device
nb = 4 * 65536
src, off, ln = bench.make_blocks(codec, dev, nb, 0)
L = int(ln[0].item())
stride = (L + 15) // 16 * 16
asrc = torch.zeros(nb * stride, dtype=torch.uint8, device=dev)
asrc.view(nb, stride)[:, :L] = src[: nb * L].view(nb, L)
aoff = torch.arange(0, nb * stride, stride, dtype=torch.int64, device=dev)


def run(s, o, label):
    d = torch.empty_like(s)
    out_len = torch.empty(nb, dtype=torch.int64, device=dev)
    st = torch.empty(nb, dtype=torch.int32, device=dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    args = (P(s), P(d), P(o), P(ln), nb, 0, P(out_len), P(st))
    codec._stream()
    stream = torch.cuda.current_stream(dev)
    for _ in range(3):
        assert codec.roundtrip_raw(*args) == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(20):
        codec.roundtrip_raw(*args)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    ok = bool((st == 0).all())
    print({"layout": label, "ms": round(ms, 4), "frac_8TBps": round(2 * nb * L / (ms * 1e-3) / 8e12, 4), "ok": ok},
          flush=True)


run(src, off, "packed 4188 B")
run(asrc, aoff, f"aligned {stride} B stride")
run(src, off, "packed 4188 B (again)")

"""rt_kernel and the plain copy probe over the 1 GiB config-2 variant (262 144
blocks), 5 launches each: the workload of the PMC passes behind
profiles/r03_ab/rt_1gib.md (tools/pmc_rt_1gib.sh)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "lsm-kv-storage_amd"))
import bench  # noqa: E402
import sstcodec  # noqa: E402
from sstcodec._lib import check  # noqa: E402

dev = torch.device("cuda", 0)
codec = sstcodec.Codec(0)
nb = 262144
src, off, ln = bench.make_blocks(codec, dev, nb, 0)
dst = torch.empty_like(src)
ol = torch.empty(nb, dtype=torch.int64, device=dev)
st = torch.empty(nb, dtype=torch.int32, device=dev)
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
codec._stream()
for _ in range(5):
    assert codec.roundtrip_raw(P(src), P(dst), P(off), P(ln), nb, 0, P(ol), P(st)) == 0
n16 = (src.numel() // 16) * 16
for _ in range(5):
    check(codec.lib.sstc_copy_probe(codec.h, P(src), P(dst), n16), "sstc_copy_probe")
torch.cuda.synchronize()
print("ok", nb)

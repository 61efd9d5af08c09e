"""The config-2 encode leg (bench.codec_legs: sstc_encode_blocks over 65 536
blocks' decoded records), 5 calls: the workload of the PMC passes behind
profiles/r03_ab/encode_pmc.md (tools/pmc_enc_leg.sh)."""
import ctypes
import os
import sys

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
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
rec_base = codec.count(src, off, ln)
table, _, status = codec.decode(src, off, ln, rec_base=rec_base)
c = table.c()
first = torch.arange(0, table.n + 1, bench.PER_BLOCK, dtype=torch.int64, device=dev)
dst = torch.zeros_like(src)
out_off = torch.empty(nb + 1, dtype=torch.int64, device=dev)
out_len = torch.empty(nb, dtype=torch.int64, device=dev)
codec._stream()
for _ in range(int(os.environ.get("ENC_CALLS", "5"))):
    assert codec.lib.sstc_encode_blocks(codec.h, P(src), P(src), c, table.n, P(first), nb, 0,
                                        P(dst), P(out_off), P(out_len)) == 0
torch.cuda.synchronize()
assert torch.equal(dst, src)
print("ok", nb, table.n)

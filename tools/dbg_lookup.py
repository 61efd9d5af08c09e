"""Debug: GPU lookups vs the oracle on one config-3-shaped table; prints the
first mismatches (query, GPU type/block, oracle type/block)."""
import os
import sys

R = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R + "/lsm-kv-storage_amd")
sys.path.insert(0, R + "/oracle")
import numpy as np  # noqa: E402
import torch  # noqa: E402
import sstcodec  # noqa: E402
from oracle import Oracle  # noqa: E402
from sstcodec import workload as W  # noqa: E402

orc = Oracle()
codec = sstcodec.Codec(0)
for nkeys in (1000, 100000):
    rec = W.uniform_records(nkeys, key_index=np.arange(nkeys, dtype=np.uint64) * np.uint64(8), seed=1)
    img = orc.table_build(rec, 4096)
    lk = sstcodec.Lookup(codec, [img])
    keys = [b"k%015d" % i for i in range(0, 8 * nkeys + 40, 3)]
    typ, vo, vl, blk = lk.get(np.zeros(len(keys), np.uint32), keys)
    torch.cuda.synchronize()
    ot, ovo, ovl, oblk = orc.table_get(img, keys)
    bad = np.nonzero((typ != ot) | (blk != oblk))[0]
    print("nkeys", nkeys, "blocks", int(lk.tfb[1].item()), "queries", len(keys), "mismatch", len(bad),
          "types gpu", np.bincount(typ, minlength=5).tolist(), "oracle", np.bincount(ot, minlength=5).tolist())
    for i in bad[:8]:
        print("  q", i, keys[i], "gpu", int(typ[i]), int(blk[i]), "orc", int(ot[i]), int(oblk[i]))

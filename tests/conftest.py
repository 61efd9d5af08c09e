import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "lsm-kv-storage_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
REC_KEYS = ("type", "key_len", "val_len", "txn", "key_off", "val_off")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C-ABI)")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def golden_records(g):
    return {k: g["rec_" + k] for k in REC_KEYS + ("key_src", "val_src")}


@pytest.fixture(scope="session")
def oracle():
    from oracle import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def reflib():
    from oracle import REF_SO, RefLib
    if not os.path.exists(REF_SO):
        pytest.skip("reference library not built (needs /root/reference)")
    return RefLib()


BLOCK_SETS = ["kat_basic.npz", "kat_edge.npz", "block_uniform.npz", "blocks_mixed.npz", "blocks_edge.npz"]


def sst_records(oracle, img):
    """Records of an SST image in file order: (key, txn, type, value or None),
    parsed with the oracle (table_reader.cc:52-156, block_reader.cc:59-114)."""
    idx = oracle.table_index(img)
    out = []
    for o, ln in zip(idx["blk_off"], idx["blk_len"]):
        st, d = oracle.decode_block(img[int(o):int(o + ln)], 1, int(o))  # correct txn mode
        assert st == 0
        for t, kl, vl, tx, ko, vo in zip(d["type"], d["key_len"], d["val_len"], d["txn"], d["key_off"], d["val_off"]):
            key = bytes(img[int(ko):int(ko) + int(kl)])
            val = None if vl == 0xFFFFFFFF else bytes(img[int(vo):int(vo) + int(vl)])
            out.append((key, int(tx), int(t), val))
    return out


def tie_case(g, name, base):
    ins = [g[f"{name}_in{i}"] for i in range(4)]
    outs = sorted((k for k in g if k.startswith(f"{name}_base{base}_out")), key=lambda x: int(x.rsplit("out", 1)[1]))
    return ins, [g[k] for k in outs]


def _runs(recs):
    out = []
    for r in recs:
        if out and out[-1][0] == r[:2]:
            out[-1][1].append(r)
        else:
            out.append((r[:2], [r]))
    return out


def same_up_to_tie_order(a, b, inputs):
    """Two compaction outputs (record streams) of the same inputs that may
    differ only in how runs of equal (key, txn) coming from several inputs
    were ordered: the same (key, txn) sequence, identical runs for pairs that
    occur in one input only, and for tied pairs only records of the inputs
    (which of them survive ShouldKeepEntry depends on the order, compact.cc:
    324-363)."""
    from collections import Counter
    seen = Counter()
    pool = {}
    for recs in inputs:
        for p in {r[:2] for r in recs}:
            seen[p] += 1
        for r in recs:
            pool.setdefault(r[:2], []).append(r)
    ra, rb = _runs(a), _runs(b)
    if [p for p, _ in ra] != [p for p, _ in rb]:
        return False
    for (p, x), (_, y) in zip(ra, rb):
        if seen[p] <= 1:
            if x != y:
                return False
        elif not all(r in pool[p] for r in x + y):
            return False
    return True


@pytest.fixture(autouse=True)
def _gpu_memlog(request):
    """SSTC_MEMLOG=1: free device memory after every GPU test (finds a test
    that leaves workspace behind)."""
    yield
    if os.environ.get("SSTC_MEMLOG") and request.node.get_closest_marker("gpu"):
        import torch
        free, total = torch.cuda.mem_get_info()
        print(f"\n[memlog] {request.node.name}: free {free / 2**30:.1f} of {total / 2**30:.1f} GiB", flush=True)

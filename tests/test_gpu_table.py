"""GPU: the host C++ TableBuilder / TableReader (over the codec kernels) write
and read the same SST bytes as the reference's TableBuilder / TableReader."""
import os
import tempfile

import numpy as np
import pytest
from conftest import REC_KEYS, golden_records, load_golden
from sstcodec import workload as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    import sstcodec
    return sstcodec.Codec(0)


def test_table_mini_matches_reference(codec):
    from sstcodec.table import build_table
    g = load_golden("table_mini.npz")
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "1.sst")
        fs, nb = build_table(codec, p, golden_records(g), 4096)
        assert fs == int(g["file_size"][0]) == 231 and nb == 1
        assert np.array_equal(np.fromfile(p, np.uint8), g["sst"])


@pytest.mark.parametrize("T", [4096, 32768])
def test_table_mixed_matches_reference(codec, T):
    from sstcodec.table import build_table, read_table
    g = load_golden(f"table_mixed_{T}.npz")
    rec = golden_records(load_golden("blocks_mixed.npz"))
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "t.sst")
        fs, nb = build_table(codec, p, rec, T)
        assert fs == int(g["file_size"][0])
        assert np.array_equal(np.fromfile(p, np.uint8), g["sst"])
        r = read_table(codec, p, fs, txn_mode=1)
        assert np.array_equal(r["blk_off"], g["idx_blk_off"]) and np.array_equal(r["blk_len"], g["idx_blk_len"])
        assert np.array_equal(r["txn"], rec["txn"]) and np.array_equal(r["type"], rec["type"])
        assert np.array_equal(r["key_len"], rec["key_len"]) and np.array_equal(r["val_len"], rec["val_len"])


def test_table_roundtrip_vs_oracle(codec, oracle):
    from sstcodec.table import build_table, read_table
    rec = W.mixed_records(20000, seed=123, max_val=700)
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "x.sst")
        fs, nb = build_table(codec, p, rec, 4096)
        f = np.fromfile(p, np.uint8)
        assert np.array_equal(f, oracle.table_build(rec, 4096)) and fs == f.size + 1
        r = read_table(codec, p, fs, txn_mode=0)
        idx = oracle.table_index(f)
        parts = {k: [] for k in REC_KEYS}
        for o, ln in zip(idx["blk_off"], idx["blk_len"]):
            st, d = oracle.decode_block(f[int(o):int(o + ln)], 0, int(o))
            assert st == 0
            for k in REC_KEYS:
                parts[k].append(d[k])
        for k in REC_KEYS:
            assert np.array_equal(r[k], np.concatenate(parts[k])), k


def test_table_empty(codec, oracle):
    from sstcodec.table import build_table
    rec = W.mixed_records(0)
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "e.sst")
        fs, nb = build_table(codec, p, rec, 4096)
        assert nb == 0 and fs == 41
        assert np.array_equal(np.fromfile(p, np.uint8), oracle.table_build(rec, 4096))

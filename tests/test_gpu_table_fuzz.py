"""sstc::TableBuilder (the flush path and the drop-in) over randomised record
sets against the oracle's restatement of the reference TableBuilder
(oracle/sst_oracle.c orc_table_build, pinned by the reference's own files in
test_gpu_table.py): ragged keys (0-200 B), empty values (the txn quirk),
DELETEs, values past a block, block thresholds from 1 B to 64 KiB, records
added in one batch or one AddEntry at a time, and several builders one after
another on the same thread (the builder's arrays come from a per-thread pool:
a builder must never see its predecessor's records)."""
import ctypes
import os

import numpy as np
import pytest
from sstcodec import workload as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    import sstcodec
    return sstcodec.Codec(0)


def build_per_record(codec, path, rec, threshold):
    """The drop-in's path: one AddEntry per record (sstc_tb_add)."""
    from sstcodec._lib import check, load
    from sstcodec.table import _sig
    lib = _sig(load())
    codec._stream()
    tb = ctypes.c_void_p()
    check(lib.sstc_tb_create(path.encode(), threshold, codec.h, ctypes.byref(tb)), "sstc_tb_create")
    try:
        check(lib.sstc_tb_open(tb), "sstc_tb_open")
        ks, vs = rec["key_src"], rec["val_src"]
        for i in range(len(rec["type"])):
            ko, kl = int(rec["key_off"][i]), int(rec["key_len"][i])
            vl = int(rec["val_len"][i])
            key = ks[ko:ko + kl].tobytes()
            if vl == W.NO_VALUE:
                val, vlen = None, 0
            else:
                vo = int(rec["val_off"][i])
                val, vlen = vs[vo:vo + vl].tobytes(), vl
            check(lib.sstc_tb_add(tb, key, kl, val if val is not None else None, vlen, int(rec["txn"][i]),
                                  int(rec["type"][i])), "sstc_tb_add")
        check(lib.sstc_tb_finish(tb), "sstc_tb_finish")
        return lib.sstc_tb_file_size(tb), lib.sstc_tb_num_blocks(tb)
    finally:
        lib.sstc_tb_destroy(tb)


CASES = [  # (seed, n, max_key, max_val, threshold)
    (0, 5000, 48, 300, 4096), (1, 3000, 200, 40, 1), (2, 800, 8, 70000, 65536), (3, 12000, 16, 100, 4096),
    (4, 2000, 1, 1, 64), (5, 400, 64, 9000, 512), (6, 1, 4, 4, 4096), (7, 20000, 30, 30, 16384),
]


@pytest.mark.timeout(240)
@pytest.mark.parametrize("seed,n,max_key,max_val,T", CASES)
def test_table_builder_fuzz_vs_oracle(codec, oracle, tmp_path, seed, n, max_key, max_val, T):
    from sstcodec.table import build_table
    rec = W.mixed_records(n, seed=300 + seed, max_key=max_key, max_val=max_val, p_delete=0.15, p_empty_val=0.1,
                          p_empty_key=0.03)
    want = oracle.table_build(rec, T)
    p = str(tmp_path / "b.sst")
    fs, nb = build_table(codec, p, rec, T)
    got = np.fromfile(p, np.uint8)
    assert fs == want.size + 1 and np.array_equal(got, want)
    if n <= 5000:  # one AddEntry at a time (the drop-in)
        q = str(tmp_path / "r.sst")
        fs2, nb2 = build_per_record(codec, q, rec, T)
        assert (fs2, nb2) == (fs, nb) and np.array_equal(np.fromfile(q, np.uint8), want)


def test_table_builders_in_sequence_share_nothing(codec, oracle, tmp_path):
    """Large, small, empty, large again on one thread: each file equals the
    oracle's (pooled arrays are cleared between builders)."""
    from sstcodec.table import build_table
    shapes = [(60000, 100), (3, 20), (0, 0), (25000, 900), (10, 5)]
    for k, (n, mv) in enumerate(shapes):
        rec = W.mixed_records(n, seed=900 + k, max_val=max(mv, 1))
        p = str(tmp_path / f"{k}.sst")
        fs, _ = build_table(codec, p, rec, 4096)
        want = oracle.table_build(rec, 4096)
        assert fs == want.size + 1 and np.array_equal(np.fromfile(p, np.uint8), want), k
        os.remove(p)

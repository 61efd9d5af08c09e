"""GPU batched point lookups (sstc_get_batch) against the reference's own
TableReader::GetValue results (tests/golden/lookup.npz) and the oracle
restatement on larger tables: repeated keys inside blocks (the probe order of
BlockReader::GetValue decides which version is returned), absent keys, keys
past the last block, empty tables, malformed blocks."""
import numpy as np
import pytest
import torch
from conftest import load_golden
from sstcodec import workload as W
from test_oracle_lookup import golden_queries, golden_values

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    import sstcodec
    return sstcodec.Codec(0)


def test_lookup_golden_two_tables(codec):
    import sstcodec
    g = load_golden("lookup.npz")
    tables = [g["sst0"], g["sst1"]]
    lk = sstcodec.Lookup(codec, tables)
    keys, qt, want_t, want_v = [], [], [], []
    for t in (0, 1):
        k = golden_queries(g, t)
        keys += k
        qt += [t] * len(k)
        want_t.append(g[f"q{t}_type"])
        want_v += golden_values(g, t)
    # interleave the two tables' queries
    perm = np.random.default_rng(0).permutation(len(keys))
    keys = [keys[i] for i in perm]
    qt = np.asarray(qt)[perm]
    want_t = np.concatenate(want_t)[perm]
    want_v = [want_v[i] for i in perm]
    typ, vo, vl, blk = lk.get(qt, keys)
    assert np.array_equal(typ, want_t)
    cat = np.concatenate(tables)
    for i in range(len(keys)):
        if typ[i] == 0:
            assert bytes(cat[int(vo[i]):int(vo[i]) + int(vl[i])]) == want_v[i]


@pytest.mark.parametrize("seed", range(3))
def test_lookup_vs_oracle(codec, oracle, seed):
    import sstcodec
    rec = W.compaction_inputs(1, [20000, 3000, 800][seed], 40000, seed=60 + seed, vmax=[120, 3000, 60000][seed],
                              p_delete=0.2, distinct=seed != 0)[0]
    img = oracle.table_build(rec, [4096, 32768, 4096][seed])
    rng = np.random.default_rng(seed)
    keys = [b"k%015d" % i for i in rng.integers(0, 41000, 30000)] + [b"", b"k", b"~"]
    typ, vo, vl, blk = sstcodec.Lookup(codec, [img]).get(np.zeros(len(keys), np.uint32), keys)
    ot, ovo, ovl, oblk = oracle.table_get(img, keys)
    assert np.array_equal(typ, ot) and np.array_equal(blk, oblk)
    put = typ == 0
    assert np.array_equal(vo[put], ovo[put]) and np.array_equal(vl[put], ovl[put])


def test_lookup_edges(codec, oracle):
    import sstcodec
    empty = oracle.table_build(W.compaction_inputs(1, 0, 10)[0], 4096)
    one = oracle.table_build(W.compaction_inputs(1, 50, 100, seed=2)[0], 4096)
    lk = sstcodec.Lookup(codec, [empty, one])
    keys = [b"k%015d" % i for i in range(100)]
    # empty table and an out-of-range table id: NOT_FOUND; table 1 vs the oracle
    typ, _, _, blk = lk.get([0] * 100 + [7] * 100 + [1] * 100, keys * 3)
    assert (typ[:200] == 2).all() and (blk[:200] == 2 ** 64 - 1).all()
    ot, _, _, _ = oracle.table_get(one, keys)
    assert np.array_equal(typ[200:], ot)
    assert lk.get([], [])[0].size == 0


def test_lookup_malformed_block(codec, oracle):
    import sstcodec
    rec = W.compaction_inputs(1, 400, 800, seed=9)[0]
    img = oracle.table_build(rec, 4096).copy()
    idx = oracle.table_index(img)
    b = 1
    end = int(idx["blk_off"][b] + idx["blk_len"][b])
    img[end - 8:end] = np.frombuffer((10 ** 9).to_bytes(8, "little"), np.uint8)  # offset section out of range
    lk = sstcodec.Lookup(codec, [img])
    codec.reset_errors()
    keys = [b"k%015d" % i for i in range(800)]
    typ, _, _, blk = lk.get(np.zeros(800, np.uint32), keys)
    ot, _, _, oblk = oracle.table_get(img, keys)
    assert np.array_equal(typ, ot) and (typ[blk == b] == 4).all() and (typ == 4).any()
    assert codec.error_count() == int((typ == 4).sum())


@pytest.mark.parametrize("seed", range(2))
def test_lookup_ragged_keys_vs_oracle(codec, oracle, seed):
    """Ragged 0-48 B keys (the empty key repeated with random txns, so a block
    holds several versions of it out of txn order), empty values, DELETEs:
    every probe -- present keys, their prefixes and extensions, the empty key
    -- answers as the reference's GetValue (oracle, pinned by lookup.npz)."""
    import sstcodec
    from test_gpu_compact_fuzz import ragged_sorted
    rec = ragged_sorted(6000, 800 + seed)
    img = oracle.table_build(rec, [4096, 512][seed])
    present = [rec["key_src"][int(o):int(o) + int(l)].tobytes() for o, l in zip(rec["key_off"], rec["key_len"])]
    rng = np.random.default_rng(seed)
    keys = present[::3] + [k[:-1] for k in present[1::7]] + [k + b"\x00" for k in present[2::11]] + [b"", b"~~~~"]
    keys = [keys[i] for i in rng.permutation(len(keys))]
    typ, vo, vl, blk = sstcodec.Lookup(codec, [img]).get(np.zeros(len(keys), np.uint32), keys)
    ot, ovo, ovl, oblk = oracle.table_get(img, keys)
    assert np.array_equal(typ, ot) and np.array_equal(blk, oblk)
    put = typ == 0
    assert np.array_equal(vo[put], ovo[put]) and np.array_equal(vl[put], ovl[put])

"""sstc_merge_records (include/sstcodec.h) straight through the C-ABI: the
order MergeIterator pops every record of many SSTs in (SeekToFirst + Next,
/root/reference/db/merge_iterator.cc:34-46,79-92; comparator key asc, txn desc,
merge_iterator.h:91-95; an input's own records leave in file order), with the
txn as the reference's iterator reads it (compat: block_reader.cc:109-111).
The expected order is built here from the oracle's block decode of every
input: each record's merge txn is the running minimum of the txns as read
over its key group in its input (the heap only ever sees an input's current
record), and ties between inputs are excluded by the data (the counters say
so).  Also: the capacity protocol, rejected inputs, the tie counters on the
reference-made tie fixtures.  The drop-in MergeIterator's walks over the same
call are compared with the reference's own iterator in test_gpu_dropin.py."""
import numpy as np
import pytest
from conftest import load_golden, tie_case
from sstcodec import workload as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    import sstcodec
    return sstcodec.Codec(0)


def _records(oracle, img, t):
    """(key, txn as read, table, index in the table, key offset in the image), file order"""
    idx = oracle.table_index(img)
    out = []
    for o, n in zip(idx["blk_off"], idx["blk_len"]):
        st, r = oracle.decode_block(img[int(o):int(o + n)], 0, int(o))
        assert st == 0
        for i in range(len(r["key_len"])):
            ko, kl = int(r["key_off"][i]), int(r["key_len"][i])
            out.append((bytes(img[ko:ko + kl]), int(r["txn"][i]), t, len(out), ko))
    return out


def _expected(oracle, files):
    rows = []
    for t, img in enumerate(files):
        recs = _records(oracle, img, t)
        m, prev = None, None
        for key, tx, tt, j, ko in recs:  # the merge txn: running minimum over the key's group in this input
            m = tx if key != prev else min(m, tx)
            prev = key
            rows.append((key, -m, tt, j, tx, ko))
    rows.sort()  # key asc, merge txn desc, lower input first, file order
    return rows


def _check(codec, oracle, files):
    recs, res = codec.merge_records(files)
    want = _expected(oracle, files)
    assert res.records == len(want) == len(recs)
    assert res.cross_ties == 0 and res.tie_diffs == 0  # (the expected order has no tie to break)
    base = np.concatenate([[0], np.cumsum([f.size for f in files])])
    cat = np.concatenate(files)
    got = []
    for ko, tx in recs.tolist():
        t = int(np.searchsorted(base, ko, side="right")) - 1
        kl = int(cat[ko - 4:ko].view(np.uint32)[0])
        got.append((bytes(cat[ko:ko + kl]), tx, t, ko - int(base[t])))
    assert got == [(k, tx, t, ko) for k, _, t, _, tx, ko in want]
    return res


@pytest.mark.parametrize("case", ["overlap", "versions", "many_inputs", "one_input", "empty_values"])
def test_merge_records_order_vs_oracle(codec, oracle, case):
    """overlap: 5 inputs over a shared key space (one merge pass); versions:
    keys repeated inside inputs, empty values among them (the compat txn
    quirk lowers their txns as read: out of txn order within a key group);
    many_inputs: 20 inputs (two merge passes); one_input; empty_values: every
    value empty."""
    sets = {
        "overlap": lambda: W.compaction_inputs(5, 2000, 3000, seed=11, vmin=1, vmax=300),
        "versions": lambda: W.compaction_inputs(3, 1500, 50, seed=70, p_delete=0.1, vmin=0, vmax=3, distinct=False),
        "many_inputs": lambda: W.compaction_inputs(20, 400, 5000, seed=12, vmin=1, vmax=120, distinct=False),
        "one_input": lambda: W.compaction_inputs(1, 3000, 9000, seed=9),
        "empty_values": lambda: W.compaction_inputs(4, 800, 900, seed=13, vmin=0, vmax=0, distinct=False),
    }[case]()
    files = [oracle.table_build(r, 4096) for r in sets]
    _check(codec, oracle, files)


def test_merge_records_capacity_and_rejections(codec, oracle):
    """max_records below the record count: SSTC_E_CAPACITY with the count in
    the result (the Python face then calls again with that much room); an
    input whose keys are not ascending (table_builder.h:77): SSTC_E_INVALID_ARG."""
    from sstcodec._lib import SSTC_E_CAPACITY, SSTC_E_INVALID_ARG, SstcError
    sets = W.compaction_inputs(3, 500, 2000, seed=14)
    files = [oracle.table_build(r, 4096) for r in sets]
    n = sum(len(r["type"]) for r in sets)
    with pytest.raises(SstcError) as e:
        codec.merge_records(files, max_records=n - 1)
    assert e.value.code == SSTC_E_CAPACITY
    recs, res = codec.merge_records(files, max_records=n)
    assert res.records == n and len(recs) == n
    bad = dict(sets[1])
    bad["key_off"] = bad["key_off"][::-1].copy()  # keys descending
    with pytest.raises(SstcError) as e:
        codec.merge_records([files[0], oracle.table_build(bad, 4096)])
    assert e.value.code == SSTC_E_INVALID_ARG


@pytest.mark.parametrize("name", ["same", "diff"])
def test_merge_records_tie_counters(codec, name):
    """The reference-made tie fixtures (compact_ties.npz): equal (key, txn)
    records in different inputs are counted (cross_ties); where their bytes
    differ too (tie_diffs) the reference's heap history decides their order,
    which is what makes the drop-in MergeIterator take the heaps."""
    ins, _ = tie_case(load_golden("compact_ties.npz"), name, 1)
    recs, res = codec.merge_records(ins)
    assert res.records == len(recs) > 0 and res.cross_ties > 0
    assert (res.tie_diffs > 0) == (name == "diff")


def fuzz_sets(seed):
    """random merge shapes: 1-40 inputs, 50-1500 records each, keys 4-40 B
    from a small or large space (versions inside inputs or not), values
    0 B-20 KiB with empty ones, 0-30 % DELETEs"""
    rng = np.random.default_rng(1000 + seed)
    k = int(rng.choice([1, 2, 5, 9, 17, 40]))
    n = int(rng.integers(50, 1500))
    space = int(rng.choice([40, 2000, 10 ** 6]))
    vmax = int(rng.choice([0, 16, 300, 20000]))
    width = int(rng.choice([4, 16, 40]))
    width = 16 if width == 4 and space > 999 else width  # "k" + 3 digits: keys in order only below 1000
    return W.compaction_inputs(k, n, space, seed=2000 + seed, p_delete=float(rng.choice([0.0, 0.1, 0.3])),
                               vmin=0, vmax=vmax, key_width=width, distinct=bool(rng.integers(0, 2)) and n <= space)


@pytest.mark.parametrize("seed", range(8))
def test_merge_records_fuzz_vs_oracle(codec, oracle, seed):
    """random shapes (fuzz_sets; the model is pinned to the reference's own
    MergeIterator on three of them in test_oracle_merge_order.py)"""
    files = [oracle.table_build(r, int(np.random.default_rng(seed).choice([256, 4096, 32768])))
             for r in fuzz_sets(seed)]
    _check(codec, oracle, files)

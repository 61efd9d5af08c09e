"""Compaction job (sstc_compact) over randomised shapes against the oracle
(oracle/ref_compact.cc restating Compact::DoCompactJob, compact.cc:232-363,
pinned by the reference's own outputs in test_oracle_compact.py): block
thresholds from 64 B to 64 KiB, table limits from one record per table to
one table, key widths 6-20 B (past the 16 B merge prefix, sharing it), values up to
96 KiB (blocks far past the encode's LDS slot), DELETE ratios, overlapping
and disjoint key sets, 1-13 inputs.  Bit-exact at base levels 1 and 0.

The job reads its kept count, table and block counts on the device only
(round 4), so every shape here also exercises the count bounds the layout
runs on (a table / block count past its bound would surface as
SSTC_E_INTERNAL)."""
import numpy as np
import pytest
from sstcodec import workload as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    import sstcodec
    return sstcodec.Codec(0)


def shapes():
    rng = np.random.default_rng(2024)
    out = []
    for seed in range(14):
        k = int(rng.integers(1, 14))
        n_per = int(rng.integers(50, 2500))
        vmax = int(rng.choice([16, 300, 4000, 98304]))
        if vmax >= 4000:  # keep the inputs within tens of MB
            k, n_per = min(k, 5), min(n_per, 200 if vmax > 4000 else 1200)
        out.append(dict(
            seed=seed, k=k, n_per=n_per,
            space=int(n_per * rng.choice([1.2, 2.0, 8.0])),
            key_width=int(rng.choice([6, 8, 16, 18, 20])),  # "k%0{w-1}d": distinct and sorted up to w = 20
            vmin=int(rng.choice([0, 1, 8])),
            vmax=vmax,
            zipf=float(rng.choice([0.0, 1.1, 1.5])),
            p_delete=float(rng.choice([0.0, 0.1, 0.5, 0.9])),
            distinct=bool(rng.random() < 0.8),
            threshold=int(rng.choice([64, 512, 4096, 16384, 65536])),
            limit_frac=float(rng.choice([0.0, 0.05, 0.3, 2.0])),
        ))
    return out


SHAPES = shapes()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("shape", SHAPES, ids=[f"s{s['seed']}" for s in SHAPES])
def test_compact_fuzz_vs_oracle(codec, oracle, shape):
    s = shape
    sets = W.compaction_inputs(s["k"], s["n_per"], s["space"], seed=1000 + s["seed"], p_delete=s["p_delete"],
                               vmin=max(s["vmin"], 1) if s["zipf"] else s["vmin"], vmax=s["vmax"],
                               key_width=s["key_width"], distinct=s["distinct"], zipf=s["zipf"] or None)
    ins = [oracle.table_build(r, s["threshold"]) for r in sets]
    total = sum(int(f.size) for f in ins)
    limit = max(1, int(total * s["limit_frac"]))  # 0.0 -> 1 B: every record its own table
    for base in (1, 0):
        want, kept = oracle.compact(ins, s["threshold"], limit, base)
        outs, res = codec.compact(ins, s["threshold"], limit, base)
        assert res.records_kept == kept
        assert res.tables_out == len(want) == len(outs)
        for t, (o, w) in enumerate(zip(outs, want)):
            assert np.array_equal(o, w), f"output table {t} of {len(want)} differs (base {base})"


@pytest.mark.parametrize("space", [50, 12])
@pytest.mark.parametrize("threshold", [256, 4096])
@pytest.mark.parametrize("seed", range(3))
def test_compact_versions_out_of_txn_order(codec, oracle, seed, threshold, space):
    """Several versions of a key in one input, some of them empty-value PUTs:
    the reference's reader returns (txn & 0xffffffff) << 32 for those
    (block_reader.cc:109-111), so a key's versions are out of txn order as
    read, and its MergeIterator heap pops each input in file order under the
    smallest txn so far.  The job merges on that running minimum (per block
    in the decode, carried across block boundaries: with 256 B blocks a key's
    ~30 versions span several blocks) and writes the txns as read.  The
    oracle is pinned for these inputs by the reference's own MergeIterator
    (tests/test_oracle_compact.py::test_live_ref_compact_versions_out_of_txn_order:
    seed 71, 4 KiB blocks)."""
    sets = W.compaction_inputs(3, 1500, space, seed=70 + seed, p_delete=0.1, vmin=0, vmax=3, key_width=16,
                               distinct=False)
    ins = [oracle.table_build(r, threshold) for r in sets]
    for base in (1, 0):
        want, kept = oracle.compact(ins, threshold, 1 << 20, base)
        outs, res = codec.compact(ins, threshold, 1 << 20, base)
        assert res.records_kept == kept and len(outs) == len(want)
        for o, w in zip(outs, want):
            assert np.array_equal(o, w)


def test_compact_long_version_groups(codec, oracle):
    """One key's versions over far more than kGroupCarryBlocks (64) blocks of
    an input (~200 blocks), in txn order and out of it as read (an
    empty-value version mid-group: its txn as read jumps): the running minimum
    is carried over every block (the check kernel's last workgroup repairs
    what its 64-block walks leave, long_carry_repair), bit-exact."""
    sets = W.compaction_inputs(1, 1200, 2, seed=5, p_delete=0.0, vmin=4, vmax=8, key_width=16, distinct=False)
    ins = [oracle.table_build(r, 128) for r in sets]  # ~3 records per block: ~200 blocks per key
    want, _ = oracle.compact(ins, 128, 1 << 20, 1)
    outs, _ = codec.compact(ins, 128, 1 << 20, 1)
    assert len(outs) == len(want) and all(np.array_equal(o, w) for o, w in zip(outs, want))
    rec = {key: v.copy() for key, v in sets[0].items()}
    rec["val_len"][len(rec["val_len"]) // 2] = 0  # one empty-value PUT mid-group: its txn as read jumps
    bad = [oracle.table_build(rec, 128)]
    for base in (1, 0):
        want, kept = oracle.compact(bad, 128, 1 << 20, base)
        outs, res = codec.compact(bad, 128, 1 << 20, base)
        assert res.records_kept == kept and len(outs) == len(want)
        assert all(np.array_equal(o, w) for o, w in zip(outs, want))


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("threshold", [128, 512])
def test_compact_long_groups_out_of_txn_order_fuzz(codec, oracle, seed, threshold):
    """Three inputs over three keys, hundreds of versions per key per input
    (each key's group spans 100-500 small blocks), empty-value PUTs among
    them (out of txn order as read), DELETEs: every group needs carries far
    past 64 blocks, several groups per input, groups ending and starting
    inside blocks; bit-exact vs the oracle at both base levels and with
    output splits."""
    sets = W.compaction_inputs(3, 1500, 3, seed=200 + seed, p_delete=0.1, vmin=0, vmax=3, key_width=16,
                               distinct=False)
    ins = [oracle.table_build(r, threshold) for r in sets]
    for base in (1, 0):
        for limit in (1 << 20, 200):
            want, kept = oracle.compact(ins, threshold, limit, base)
            outs, res = codec.compact(ins, threshold, limit, base)
            assert res.records_kept == kept and len(outs) == len(want)
            assert all(np.array_equal(o, w) for o, w in zip(outs, want))


def test_compact_long_in_order_group_beside_short_out_of_order_group(codec, oracle):
    """a long group in txn order (its walks give up at 64 blocks)
    and, in another input, a short group out of txn order: the job-wide notes
    send the job through the repair pass, which must leave the in-order group
    as it is and carry the short one; bit-exact."""
    long = W.compaction_inputs(1, 1200, 1, seed=5, p_delete=0.0, vmin=4, vmax=8, key_width=16, distinct=False)[0]
    short = W.compaction_inputs(1, 300, 40, seed=6, p_delete=0.0, vmin=0, vmax=3, key_width=16, distinct=False)[0]
    short["val_len"][::7] = 0
    ins = [oracle.table_build(long, 128), oracle.table_build(short, 128)]
    want, kept = oracle.compact(ins, 128, 1 << 20, 1)
    outs, res = codec.compact(ins, 128, 1 << 20, 1)
    assert res.records_kept == kept and all(np.array_equal(o, w) for o, w in zip(outs, want))


def long_hot_key_inputs():
    """a hot key with 2000 versions in one input (values 150-250 B:
    ~16 entries per 4 KiB block, so its group spans ~125 blocks) holding an
    older empty-value PUT, beside two ordinary inputs that hold the same key too."""
    hot = W.compaction_inputs(1, 2000, 1, seed=31, p_delete=0.0, vmin=150, vmax=250, key_width=16,
                              distinct=False)[0]
    hot["val_len"][1500] = 0  # an older version (txns descend in file order) with an empty value
    hot["val_off"][1500] = 0
    other = W.compaction_inputs(2, 3000, 5000, seed=32, p_delete=0.1, vmin=0, vmax=200, key_width=16)
    return [hot] + other


def test_compact_hot_key_2000_versions_vs_reference(codec, oracle, tmp_path):
    """The hot key of long_hot_key_inputs through sstc_compact: bit-exact vs the
    oracle (pinned for exactly these inputs by the reference's own
    MergeIterator + DoCompactJob loop, tests/test_oracle_compact.py::
    test_live_ref_compact_hot_key_2000_versions) and, where the reference
    driver travelled with the tree, vs a live run of it on this box."""
    import os
    from oracle import REF_COMPACT, ref_compact
    sets = long_hot_key_inputs()
    ins = [oracle.table_build(r, 4096) for r in sets]
    idx = oracle.table_index(ins[0])
    assert len(idx["blk_off"]) > 100  # the group spans > 70 blocks
    want, kept = oracle.compact(ins, 4096, 1 << 20, 1)
    outs, res = codec.compact(ins, 4096, 1 << 20, 1)
    assert res.records_kept == kept and len(outs) == len(want)
    assert all(np.array_equal(o, w) for o, w in zip(outs, want))
    if os.path.exists(REF_COMPACT):
        files = []
        for i, f in enumerate(ins):
            p = str(tmp_path / f"h{i}.sst")
            f.tofile(p)
            files.append((p, f.size + 1))
        od = tmp_path / "ref"
        od.mkdir()
        ref = ref_compact(files, str(od), 4096, 1 << 20, 1)
        assert len(ref) == len(outs)
        for (p, fs), o in zip(ref, outs):
            assert np.array_equal(np.fromfile(p, np.uint8), o) and fs == o.size + 1


@pytest.mark.timeout(240)
@pytest.mark.parametrize("per_table", [1, 7, 40])
def test_compact_many_output_tables(codec, oracle, per_table):
    """Thousands of output tables: equal-sized records with a table limit of
    per_table records' key + value bytes -- every hop of the table split
    starts where predicted (the parallel start hops cover the first 256
    tables, the wave hops on past them), more table slots than one workgroup
    holds (the table offsets by a separate scan), many table ends per
    1024-record tile of the block split (its LDS cache of ends overflows) --
    and per_table = 40 with 4 KiB blocks, tables of several blocks."""
    sets = W.compaction_inputs(3, 1500, 6000, seed=77, p_delete=0.0, vmin=24, vmax=24, key_width=16)
    ins = [oracle.table_build(r, 4096) for r in sets]
    limit = per_table * (16 + 24)
    want, _ = oracle.compact(ins, 4096 if per_table == 40 else 256, limit, 1)
    outs, res = codec.compact(ins, 4096 if per_table == 40 else 256, limit, 1)
    assert len(outs) == len(want) > (256 if per_table < 40 else 50)
    assert all(np.array_equal(o, w) for o, w in zip(outs, want))


@pytest.mark.parametrize("n_tables", [126, 127, 128, 129, 191, 300])
def test_compact_tiles_inside_the_last_of_many_tables(codec, oracle, n_tables):
    """n_tables equal output tables of 1100 records each (more than a 1024-record
    block-split tile), so tiles start inside the last table: the block split's
    64-ary search for a tile's first table end must reach the end list's last
    element (127 tables = 128 ends: two search rounds, its top lane at the
    range end)."""
    per = 1100
    total = n_tables * per
    # one input holding every key of the space once: exactly n_tables outputs
    sets = W.compaction_inputs(1, total, total, seed=91, p_delete=0.0, vmin=24, vmax=24, key_width=16)
    ins = [oracle.table_build(r, 4096) for r in sets]
    limit = per * (16 + 24)
    want, _ = oracle.compact(ins, 4096, limit, 1)
    outs, res = codec.compact(ins, 4096, limit, 1)
    assert len(want) == n_tables and len(outs) == len(want)
    assert all(np.array_equal(o, w) for o, w in zip(outs, want))


def wide_shapes():
    """Many inputs (multi-pass merges: 8 / 4-way splitter lanes, 2-3 passes),
    tiny key spaces (long version groups, 2 B keys)."""
    rng = np.random.default_rng(77)
    out = []
    for seed, k in enumerate([20, 64, 130, 9, 33]):
        tiny = seed >= 3
        out.append(dict(seed=100 + seed, k=k, n_per=int(rng.integers(30, 300)),
                        space=8 if tiny else int(rng.integers(200, 5000)),
                        key_width=2 if tiny else int(rng.choice([8, 16, 20])),
                        vmax=int(rng.choice([0, 40, 500])), p_delete=float(rng.choice([0.0, 0.3])),
                        threshold=int(rng.choice([128, 4096])), distinct=not tiny))
    return out


WIDE = wide_shapes()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("shape", WIDE, ids=[f"w{s['seed']}" for s in WIDE])
def test_compact_fuzz_wide_vs_oracle(codec, oracle, shape):
    s = shape
    sets = W.compaction_inputs(s["k"], s["n_per"], s["space"], seed=s["seed"], p_delete=s["p_delete"], vmin=0,
                               vmax=s["vmax"], key_width=s["key_width"], distinct=s["distinct"])
    ins = [oracle.table_build(r, s["threshold"]) for r in sets]
    for base in (1, 0):
        for limit in (1 << 30, 20_000):
            want, kept = oracle.compact(ins, s["threshold"], limit, base)
            outs, res = codec.compact(ins, s["threshold"], limit, base)
            assert res.records_kept == kept and len(outs) == len(want)
            for o, w in zip(outs, want):
                assert np.array_equal(o, w)


@pytest.mark.timeout(240)
@pytest.mark.parametrize("shape", SHAPES[:6] + WIDE[3:], ids=[f"s{s['seed']}" for s in SHAPES[:6] + WIDE[3:]])
def test_compact_files_fuzz_vs_oracle(codec, oracle, shape, tmp_path):
    """The same shapes through sstc_compact_files (footer / meta parse on the
    host, preads, the device job, pwrite + fsync): every output file equals
    the oracle's table, with the key range VersionEdit::AddNewFiles records."""
    import sstcodec
    s = shape
    zipf = s.get("zipf") or None
    sets = W.compaction_inputs(s["k"], s["n_per"], s["space"], seed=(1000 if "limit_frac" in s else 0) + s["seed"],
                               p_delete=s["p_delete"], vmin=(max(s["vmin"], 1) if zipf else s["vmin"]) if "vmin" in s else 0,
                               vmax=s["vmax"], key_width=s["key_width"], distinct=s["distinct"], zipf=zipf)
    ins = [oracle.table_build(r, s["threshold"]) for r in sets]
    limit = max(1, int(sum(int(f.size) for f in ins) * s.get("limit_frac", 0.3)))
    paths, sizes = [], []
    for i, img in enumerate(ins):
        p = tmp_path / f"in{i}.sst"
        img.tofile(p)
        paths.append(str(p))
        sizes.append(img.size + 1)  # GetFileSize
    want, _ = oracle.compact(ins, s["threshold"], limit, 1)
    (tmp_path / "out").mkdir()
    pipe = sstcodec.FilePipe(codec, io_threads=4)
    try:
        outs, _ = pipe.compact_files(paths, sizes, str(tmp_path / "out") + "/", 1, s["threshold"], limit, 1)
    finally:
        pipe.close()
    assert len(outs) == len(want)
    for (sid, fsize, lo, hi), w in zip(outs, want):
        got = np.fromfile(tmp_path / "out" / f"{sid}.sst", np.uint8)
        assert fsize == w.size + 1 and np.array_equal(got, w)
        ix = oracle.table_index(w)  # the table's first / last key from its own meta section
        if ix["nblocks"]:
            f0, l0 = int(ix["first_key_off"][0]), int(ix["first_key_len"][0])
            f1, l1 = int(ix["last_key_off"][-1]), int(ix["last_key_len"][-1])
            assert lo == bytes(w[f0:f0 + l0]) and hi == bytes(w[f1:f1 + l1])


@pytest.mark.parametrize("k", [3, 9, 20])
def test_compact_with_empty_inputs_among_others(codec, oracle, k):
    """Empty input SSTs (40 B: footer only) between non-empty ones: zero-length
    runs in every merge pass (9 and 20 inputs: multi-pass groups with empty
    runs), at both base levels."""
    sets = W.compaction_inputs(k, 400, 3000, seed=500 + k, p_delete=0.2, vmax=50)
    empty = W.compaction_inputs(1, 0, 10)[0]
    ins = []
    for i, r in enumerate(sets):
        if i % 3 == 1:
            ins.append(oracle.table_build(empty, 4096))
        ins.append(oracle.table_build(r, 4096))
    ins.append(oracle.table_build(empty, 4096))
    for base in (1, 0):
        want, kept = oracle.compact(ins, 4096, 30_000, base)
        outs, res = codec.compact(ins, 4096, 30_000, base)
        assert res.records_kept == kept and len(outs) == len(want)
        for o, w in zip(outs, want):
            assert np.array_equal(o, w)


def ragged_sorted(n, seed):
    """mixed_records sorted by key bytes (std::string_view order): ragged keys
    0-48 B (the empty key repeats, with random txns: out of txn order),
    empty values (the txn quirk), DELETEs."""
    r = W.mixed_records(n, seed=seed, max_key=48, max_val=120, p_delete=0.15, p_empty_val=0.1, p_empty_key=0.05)
    keys = [r["key_src"][int(o):int(o) + int(l)].tobytes() for o, l in zip(r["key_off"], r["key_len"])]
    order = sorted(range(n), key=lambda i: keys[i])
    return {k: (v[order] if k not in ("key_src", "val_src") else v) for k, v in r.items()}


@pytest.mark.parametrize("seed", range(3))
def test_compact_ragged_keys_vs_oracle(codec, oracle, seed):
    sets = [ragged_sorted(int(900 + 300 * t), 600 + 10 * seed + t) for t in range(2 + 2 * seed)]
    ins = [oracle.table_build(r, 4096) for r in sets]
    for base in (1, 0):
        want, kept = oracle.compact(ins, 4096, 50_000, base)
        outs, res = codec.compact(ins, 4096, 50_000, base)
        assert res.records_kept == kept and len(outs) == len(want)
        for o, w in zip(outs, want):
            assert np.array_equal(o, w)


def test_compact_inputs_of_mixed_block_sizes(codec, oracle):
    """Inputs written with different block thresholds (512 B .. 64 KiB, some
    blocks past the decode's LDS slot) compacted into 16 KiB blocks."""
    sets = W.compaction_inputs(5, 1500, 4000, seed=808, p_delete=0.2, vmin=0, vmax=900)
    ins = [oracle.table_build(r, t) for r, t in zip(sets, (512, 4096, 65536, 1024, 16384))]
    for base in (1, 0):
        want, kept = oracle.compact(ins, 16384, 200_000, base)
        outs, res = codec.compact(ins, 16384, 200_000, base)
        assert res.records_kept == kept and len(outs) == len(want)
        for o, w in zip(outs, want):
            assert np.array_equal(o, w)

"""CPU: the compaction restatement (orc_compact) against outputs of the
reference's own MergeIterator + TableBuilder (tests/golden/compaction.json,
compact_small_*.npz, made by oracle/_ref/ref_compact)."""
import hashlib
import json
import os
import sys
import tempfile

import numpy as np
import pytest
from conftest import GOLDEN, load_golden
from sstcodec import workload as W

CASES = json.load(open(os.path.join(GOLDEN, "compaction.json")))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.uint8).tobytes()).hexdigest()


def build_inputs(oracle, case):
    sets = W.compaction_inputs(case["k"], case["n_per"], case["key_space"], vmax=case["vmax"],
                               distinct=case["distinct"], **case.get("gen", {}))
    return [oracle.table_build(rec, case["block_threshold"]) for rec in sets]


@pytest.mark.parametrize("name", sorted(CASES))
def test_inputs_match_reference_tablebuilder(oracle, name):
    case = CASES[name]
    files = build_inputs(oracle, case)
    for f, want in zip(files, case["inputs"]):
        assert sha(f) == want["sha256"] and f.size + 1 == want["file_size"]


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("base", [1, 0])
def test_compact_matches_reference(oracle, name, base):
    case = CASES[name]
    files = build_inputs(oracle, case)
    outs, kept = oracle.compact(files, case["block_threshold"], case["table_limit"], base)
    want = case[f"outputs_base{base}"]
    assert len(outs) == len(want)
    for o, w in zip(outs, want):
        assert o.size + 1 == w["file_size"] and sha(o) == w["sha256"]


@pytest.mark.parametrize("base", [1, 0])
def test_compact_small_bytes(oracle, base):
    g = load_golden(f"compact_small_base{base}.npz")
    ins = [g[f"in{i}"] for i in range(4)]
    outs, _ = oracle.compact(ins, 4096, 32 << 20, base)
    assert len(outs) == len([k for k in g if k.startswith("out")])
    for j, o in enumerate(outs):
        assert np.array_equal(o, g[f"out{j}"])


def test_live_ref_compact(oracle):
    from oracle import REF_COMPACT, ref_compact
    if not os.path.exists(REF_COMPACT):
        pytest.skip("reference compaction driver not built")
    sets = W.compaction_inputs(6, 700, 900, seed=99, vmax=300, p_delete=0.3)
    with tempfile.TemporaryDirectory() as td:
        ins, files = [], []
        for i, rec in enumerate(sets):
            f = oracle.table_build(rec, 4096)
            p = os.path.join(td, f"i{i}.sst")
            f.tofile(p)
            ins.append((p, f.size + 1))
            files.append(f)
        od = os.path.join(td, "o")
        os.makedirs(od)
        outs = ref_compact(ins, od, 4096, 40_000, 1)
        mine, _ = oracle.compact(files, 4096, 40_000, 1)
        assert len(outs) == len(mine) > 2
        for (p, fs), m in zip(outs, mine):
            assert np.array_equal(np.fromfile(p, np.uint8), m) and fs == m.size + 1


CONFIGS = {k: v for k, v in json.load(open(os.path.join(GOLDEN, "compaction_configs.json"))).items() if "gen" in v}
# config 4's eight shards are alike: the CPU suite pins ranks 0 and 7 against
# the oracle (every shard runs through the HIP path in test_gpu_configs.py)
CONFIGS = {k: v for k, v in CONFIGS.items() if not k.startswith("config4_rank") or k in ("config4_rank0", "config4_rank7")}


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_config_full_size_matches_reference(oracle, name):
    """BASELINE configs 3 / 3-overlap / 4 (rank-0 shard) / 5 at full size: the
    oracle's inputs equal the reference TableBuilder's files and its compaction
    equals the reference's outputs (tests/golden/make_golden_configs.py)."""
    case = CONFIGS[name]
    files = [oracle.table_build(r, case["block_threshold"]) for r in W.config_inputs(**case["gen"])]
    for f, want in zip(files, case["inputs"]):
        assert f.size + 1 == want["file_size"] and sha(f) == want["sha256"]
    outs, _ = oracle.compact(files, case["block_threshold"], case["table_limit"], 1)
    want = case["outputs_base1"]
    assert len(outs) == len(want)
    for o, w in zip(outs, want):
        assert o.size + 1 == w["file_size"] and sha(o) == w["sha256"]


@pytest.mark.parametrize("base", [1, 0])
def test_ties_identical_copies_match_reference(oracle, base):
    """The same (key, txn) record in several inputs, identical copies (one
    write = one txn in the engine): output bytes equal the reference's."""
    from conftest import tie_case
    ins, want = tie_case(load_golden("compact_ties.npz"), "same", base)
    outs, _ = oracle.compact(ins, 4096, 6000, base)
    assert len(outs) == len(want) and all(np.array_equal(o, w) for o, w in zip(outs, want))


@pytest.mark.parametrize("base", [1, 0])
def test_ties_differing_copies_documented_divergence(oracle, base):
    """Same (key, txn), different type / value: the reference's
    std::priority_queue orders such ties by its heap history
    (db/merge_iterator.h:91-95); the build orders them by input index.  Every
    record, the (key, txn) sequence and each run's contents equal the
    reference's; inside equal-(key, txn) runs the order -- and at base level
    which of a run's records survive a DELETE at its head -- differs, and it
    does differ in this fixture (divergences)."""
    from conftest import same_up_to_tie_order, sst_records, tie_case
    ins, want = tie_case(load_golden("compact_ties.npz"), "diff", base)
    outs, _ = oracle.compact(ins, 4096, 6000, base)
    a = [r for o in outs for r in sst_records(oracle, o)]
    b = [r for w in want for r in sst_records(oracle, w)]
    assert same_up_to_tie_order(a, b, [sst_records(oracle, i) for i in ins])
    assert a != b  # the divergence is real (and documented), not vacuous


@pytest.mark.parametrize("name", sorted(CASES))
def test_fixture_exercises_base_level_tombstone_drop(oracle, name):
    """The reference-parity mode (base_level = 1) drops a DELETE that starts a
    key group (compact.cc:340-350): every fixture whose inputs hold such a
    group must show it gone in the reference's output -- so the drop path is
    pinned by the reference, not only by the restated loop."""
    from conftest import sst_records
    case = CASES[name]
    files = build_inputs(oracle, case)
    recs = [r for f in files for r in sst_records(oracle, f)]
    newest = {}
    for k, t, ty, v in recs:  # the record that heads each key group (max txn)
        if k not in newest or t > newest[k][0]:
            newest[k] = (t, ty)
    heads_deleted = {k for k, (t, ty) in newest.items() if ty == 1}
    if case.get("gen", {}).get("p_delete", 0.1) == 0:
        pytest.skip("no deletes")
    assert heads_deleted, "fixture has no DELETE at a key-group head"
    outs, _ = oracle.compact(files, case["block_threshold"], case["table_limit"], 1)
    want = case["outputs_base1"]
    assert [sha(o) for o in outs] == [w["sha256"] for w in want]  # the reference's bytes
    kept_keys = {k for o in outs for k, _, _, _ in sst_records(oracle, o)}
    first_key = min(newest)  # the merge's first record is always kept (compact.cc:335-338)
    assert not (heads_deleted - {first_key}) & kept_keys
    outs0, _ = oracle.compact(files, case["block_threshold"], case["table_limit"], 0)
    kept0 = {k for o in outs0 for k, _, _, _ in sst_records(oracle, o)}
    assert heads_deleted <= kept0  # base_level 0 keeps them (framework-defined mode)


@pytest.mark.parametrize("space", [50, 12])
def test_live_ref_compact_versions_out_of_txn_order(oracle, space):
    """Several versions of a key per input with empty-value PUTs among them:
    the reference's reader returns their txns as (t & 0xffffffff) << 32, so a
    key's versions are out of txn order as read.  The oracle's merge (each
    input in file order, best head first) and keep rule (`!(last_txn > txn)`)
    equal the reference's own MergeIterator + DoCompactJob loop here -- the
    pin for tests/test_gpu_compact_fuzz.py's out-of-order cases.  (4 KiB
    blocks: the reference driver aborts below its default block size; with
    12 keys a key's ~125 versions per input cross block boundaries.)"""
    threshold = 4096
    from oracle import REF_COMPACT, ref_compact
    if not os.path.exists(REF_COMPACT):
        pytest.skip("reference compaction driver not built")
    sets = W.compaction_inputs(3, 1500, space, seed=71, p_delete=0.1, vmin=0, vmax=3, key_width=16, distinct=False)
    with tempfile.TemporaryDirectory() as td:
        ins, files = [], []
        for i, rec in enumerate(sets):
            f = oracle.table_build(rec, threshold)
            p = os.path.join(td, f"i{i}.sst")
            f.tofile(p)
            ins.append((p, f.size + 1))
            files.append(f)
        od = os.path.join(td, "o")
        os.makedirs(od)
        outs = ref_compact(ins, od, threshold, 1 << 20, 1)
        mine, kept = oracle.compact(files, threshold, 1 << 20, 1)
        assert kept > 50  # versions above their group head survive (compact.cc:357-362)
        assert len(outs) == len(mine)
        for (p, fs), m in zip(outs, mine):
            assert np.array_equal(np.fromfile(p, np.uint8), m) and fs == m.size + 1


def test_live_ref_compact_hot_key_2000_versions(oracle):
    """a hot key with 2000 versions over ~125 blocks of one
    input, an older empty-value PUT among them (out of txn order as the
    reference reads it), beside two ordinary inputs: the oracle equals the
    reference's own MergeIterator + DoCompactJob loop (oracle/_ref/ref_compact)
    -- the pin for tests/test_gpu_compact_fuzz.py::
    test_compact_hot_key_2000_versions_vs_reference."""
    from oracle import REF_COMPACT, ref_compact
    if not os.path.exists(REF_COMPACT):
        pytest.skip("reference compaction driver not built")
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_gpu_compact_fuzz import long_hot_key_inputs
    sets = long_hot_key_inputs()
    with tempfile.TemporaryDirectory() as td:
        ins, files = [], []
        for i, rec in enumerate(sets):
            f = oracle.table_build(rec, 4096)
            p = os.path.join(td, f"h{i}.sst")
            f.tofile(p)
            ins.append((p, f.size + 1))
            files.append(f)
        assert len(oracle.table_index(files[0])["blk_off"]) > 100
        od = os.path.join(td, "o")
        os.makedirs(od)
        outs = ref_compact(ins, od, 4096, 1 << 20, 1)
        mine, kept = oracle.compact(files, 4096, 1 << 20, 1)
        assert len(outs) == len(mine)
        for (p, fs), m in zip(outs, mine):
            assert np.array_equal(np.fromfile(p, np.uint8), m) and fs == m.size + 1

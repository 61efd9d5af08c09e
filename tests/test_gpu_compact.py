"""GPU compaction job (sstc_compact) against the oracle and the outputs of the
reference's own MergeIterator + TableBuilder (tests/golden/compaction.json).

base_level = 1 is the reference's reachable state and the parity claim;
base_level = 0 (tombstones at a key-group head kept) is framework-defined
semantics, pinned by the restated driver oracle/ref_compact.cc (its fixtures
are labelled outputs_base0)."""
import hashlib
import json
import os

import numpy as np
import pytest
from conftest import GOLDEN, load_golden
from sstcodec import workload as W

pytestmark = pytest.mark.gpu
CASES = json.load(open(os.path.join(GOLDEN, "compaction.json")))


@pytest.fixture(scope="module")
def codec():
    import sstcodec
    return sstcodec.Codec(0)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.uint8).tobytes()).hexdigest()


@pytest.mark.parametrize("base", [1, 0])
def test_compact_small_reference_bytes(codec, base):
    g = load_golden(f"compact_small_base{base}.npz")
    ins = [g[f"in{i}"] for i in range(4)]
    outs, res = codec.compact(ins, 4096, 32 << 20, base)
    want = [g[k] for k in sorted((k for k in g if k.startswith("out")), key=lambda x: int(x[3:]))]
    assert len(outs) == len(want)
    for o, w in zip(outs, want):
        assert np.array_equal(o, w)


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("base", [1, 0])
def test_compact_reference_hashes(codec, oracle, name, base):
    case = CASES[name]
    sets = W.compaction_inputs(case["k"], case["n_per"], case["key_space"], vmax=case["vmax"],
                               distinct=case["distinct"], **case.get("gen", {}))
    ins = [oracle.table_build(r, case["block_threshold"]) for r in sets]
    outs, res = codec.compact(ins, case["block_threshold"], case["table_limit"], base)
    want = case[f"outputs_base{base}"]
    assert len(outs) == len(want)
    for o, w in zip(outs, want):
        assert o.size + 1 == w["file_size"] and sha(o) == w["sha256"]


@pytest.mark.parametrize("seed", range(4))
def test_compact_random_vs_oracle(codec, oracle, seed):
    k = [2, 5, 8, 13][seed]
    sets = W.compaction_inputs(k, 1500, 2500, seed=seed + 40, vmax=[50, 400, 900, 120][seed],
                               p_delete=[0.0, 0.1, 0.5, 0.2][seed], distinct=seed != 3)
    ins = [oracle.table_build(r, 4096) for r in sets]
    limit = [1 << 30, 60_000, 150_000, 9_000][seed]
    for base in (1, 0):
        want, kept = oracle.compact(ins, 4096, limit, base)
        outs, res = codec.compact(ins, 4096, limit, base)
        assert res.records_kept == kept
        assert len(outs) == len(want)
        for o, w in zip(outs, want):
            assert np.array_equal(o, w)


def test_compact_long_keys_and_quirk(codec, oracle):
    """Keys longer than the 16 B sort prefix sharing it, empty values (the
    compat txn quirk changes merge order input), and a single input table."""
    rng = np.random.default_rng(1)
    sets = []
    for t in range(3):
        n = 400
        idx = np.sort(rng.choice(600, n, replace=False))
        keys = [b"PREFIX-0123456789-" + b"%06d" % i for i in idx]  # 24 B, common 16 B prefix
        vals = [b"" if rng.random() < 0.2 else bytes(rng.integers(0, 256, int(rng.integers(1, 60)),
                                                                  dtype=np.uint8)) for _ in range(n)]
        ks = b"".join(keys)
        vs = b"".join(vals)
        rec = {"type": np.zeros(n, np.uint8), "key_len": np.array([len(k) for k in keys], np.uint32),
               "val_len": np.array([len(v) for v in vals], np.uint32),
               "txn": rng.permutation(np.arange(1, n + 1, dtype=np.uint64)) + np.uint64(t * 10000),
               "key_off": np.cumsum([0] + [len(k) for k in keys[:-1]]).astype(np.uint64),
               "val_off": np.cumsum([0] + [len(v) for v in vals[:-1]]).astype(np.uint64),
               "key_src": np.frombuffer(ks, np.uint8).copy(), "val_src": np.frombuffer(vs + b"\0", np.uint8).copy()}
        sets.append(rec)
    ins = [oracle.table_build(r, 4096) for r in sets]
    for tables in (ins, ins[:1]):
        want, _ = oracle.compact(tables, 4096, 20_000, 1)
        outs, _ = codec.compact(tables, 4096, 20_000, 1)
        assert len(outs) == len(want)
        for o, w in zip(outs, want):
            assert np.array_equal(o, w)


def test_compact_rejects_unsorted(codec, oracle):
    rec = W.mixed_records(300, seed=2)  # random keys: not sorted
    f = oracle.table_build(rec, 4096)
    with pytest.raises(Exception):
        codec.compact([f], 4096, 1 << 20, 1)


def test_compact_rejects_unsorted_multi_run(codec, oracle):
    """An unsorted run among sorted ones, large enough for many merge windows:
    the job is rejected (the merge kernels stand down on the device flag) and
    the context stays usable."""
    sets = W.compaction_inputs(3, 20_000, 50_000, seed=7, vmax=64, p_delete=0.1)
    good = [oracle.table_build(r, 4096) for r in sets]
    sets[1] = {key: v[::-1].copy() for key, v in sets[1].items()}  # keys descending
    bad = [oracle.table_build(r, 4096) for r in sets]
    with pytest.raises(Exception, match="not sorted"):
        codec.compact(bad, 4096, 1 << 20, 1)
    want, _ = oracle.compact(good, 4096, 1 << 20, 1)
    outs, _ = codec.compact(good, 4096, 1 << 20, 1)
    assert len(outs) == len(want) and all(np.array_equal(o, w) for o, w in zip(outs, want))


def test_compact_rejects_corrupt_block(codec, oracle):
    """A block whose extra is intact but whose entry lengths point outside it:
    its records are never written, so everything after the decode must stand
    down; the job reports the decode failure and the context stays usable."""
    sets = W.compaction_inputs(4, 6000, 15_000, seed=8, vmax=64, p_delete=0.1)
    ins = [oracle.table_build(r, 4096) for r in sets]
    broken = ins[2].copy()
    broken[1:5] = np.frombuffer(np.uint32(0xFFFF0000).tobytes(), np.uint8)  # entry 0 of block 0
    with pytest.raises(Exception, match="decode"):
        codec.compact([ins[0], ins[1], broken, ins[3]], 4096, 1 << 20, 1)
    want, _ = oracle.compact(ins, 4096, 1 << 20, 1)
    outs, _ = codec.compact(ins, 4096, 1 << 20, 1)
    assert len(outs) == len(want) and all(np.array_equal(o, w) for o, w in zip(outs, want))


def test_compact_no_records(codec, oracle):
    """No input records (no tables, or only empty 40 B SSTs): one empty output
    table, as DoCompactJob's first TableBuilder (compact.cc:234-243)."""
    empty = oracle.table_build(W.compaction_inputs(1, 0, 10)[0], 4096)
    assert empty.size == 40
    for tables in ([], [empty], [empty, empty]):
        want, kept = oracle.compact(tables, 4096, 1 << 20, 1)
        outs, res = codec.compact(tables, 4096, 1 << 20, 1)
        assert res.records_kept == kept == 0 and res.tables_out == 1
        assert len(outs) == len(want) == 1 and np.array_equal(outs[0], want[0])


@pytest.mark.parametrize("k,n_per,space,dup", [(20, 12_000, 150_000, False), (9, 30_000, 60_000, True)])
def test_compact_large_vs_oracle(codec, oracle, k, n_per, space, dup):
    """Larger jobs: k > 8 inputs (two k-way merge passes), many merge windows,
    filter and split tiles, overlapping keys (drops), duplicated (key, txn)
    records across inputs (equal-txn runs) and many output tables."""
    sets = W.compaction_inputs(k, n_per, space, seed=91 + k, vmax=160, p_delete=0.15, distinct=not dup)
    if dup:  # the same records in two inputs: equal (key, txn) runs in the merge
        sets[1] = {key: v.copy() for key, v in sets[0].items()}
    ins = [oracle.table_build(r, 4096) for r in sets]
    for base in (1, 0):
        want, kept = oracle.compact(ins, 4096, 300_000, base)
        outs, res = codec.compact(ins, 4096, 300_000, base)
        assert res.records_kept == kept
        assert len(outs) == len(want)
        for o, w in zip(outs, want):
            assert np.array_equal(o, w)


@pytest.mark.parametrize("base", [1, 0])
def test_ties_vs_reference(codec, oracle, base):
    """Equal (key, txn) records across inputs: identical
    copies give the reference's bytes; differing copies -- whose order the
    reference's heap decides by its history, merge_iterator.h:91-95 -- are
    refused with SSTC_E_TIE_ORDER and not one byte of the output buffer is
    written (the caller routes such a job to the drop-in MergeIterator, which
    takes the heap's order: tests/test_gpu_dropin.py ties cases)."""
    from sstcodec._lib import SSTC_E_TIE_ORDER, SstcError
    from conftest import tie_case
    g = load_golden("compact_ties.npz")
    ins, want = tie_case(g, "same", base)
    outs, _ = codec.compact(ins, 4096, 6000, base)
    assert len(outs) == len(want) and all(np.array_equal(o, w) for o, w in zip(outs, want))
    ins, want = tie_case(g, "diff", base)
    probe = []
    with pytest.raises(SstcError) as e:
        codec.compact(ins, 4096, 6000, base, probe=probe)
    assert e.value.code == SSTC_E_TIE_ORDER, str(e.value)
    assert bool((probe[0] == 0xA5).all()), "a refused job wrote output bytes"


@pytest.mark.parametrize("base", [1, 0])
def test_compact_many_entries_per_block(codec, oracle, base):
    """Tiny entries (8-byte values, half DELETEs: ~85 entries per 4 KiB block),
    so the encode copies blocks in several 64-entry rounds and the dwords at
    round boundaries overlap the neighbouring entries' bytes."""
    sets = W.compaction_inputs(5, 6000, 12000, seed=23, vmin=0, vmax=8, p_delete=0.5)
    ins = [oracle.table_build(r, 4096) for r in sets]
    want, kept = oracle.compact(ins, 4096, 90_000, base)
    outs, res = codec.compact(ins, 4096, 90_000, base)
    assert res.records_kept == kept and len(outs) == len(want)
    for o, w in zip(outs, want):
        assert np.array_equal(o, w)


def test_compact_capacity_exceeded_writes_nothing(codec):
    """sstc_compact with an output buffer one byte short: SSTC_E_CAPACITY, the
    exact output size in bytes_out (what sstc_compact_files retries with), and
    not one byte of the buffer written (the writers check the size on the
    device); the same call with the exact size gives the reference's bytes."""
    import ctypes
    import torch
    from sstcodec._lib import CompactParams, CompactResult
    g = load_golden("compact_small_base1.npz")
    ins = [g[f"in{i}"] for i in range(4)]
    want = [g[k] for k in sorted((k for k in g if k.startswith("out")), key=lambda x: int(x[3:]))]
    need = sum(w.size for w in want)
    src = torch.from_numpy(np.concatenate(ins)).to(codec.device)
    idx = codec.open_tables(src, [f.size for f in ins], strict=True)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    toff = torch.zeros(65, dtype=torch.int64, device=codec.device)
    tlen = torch.zeros(64, dtype=torch.int64, device=codec.device)
    prm = CompactParams(4096, 32 << 20, 1, 0)
    for cap, rc_want in ((need - 1, -5), (need, 0)):
        dst = torch.full((need + 64,), 0xA5, dtype=torch.uint8, device=codec.device)
        res = CompactResult()
        codec._stream()
        rc = codec.lib.sstc_compact(codec.h, P(src), P(idx["blk_off"]), P(idx["blk_len"]), int(idx["blk_off"].numel()),
                                    idx["table_first_block"].ctypes.data_as(ctypes.c_void_p), len(ins),
                                    ctypes.byref(prm), P(dst), cap, P(toff), P(tlen), 64, ctypes.byref(res))
        assert rc == rc_want
        assert res.bytes_out == need
        d = dst.cpu().numpy()
        assert (d[need:] == 0xA5).all()
        if rc:
            assert (d == 0xA5).all(), "a writer touched the output buffer past its capacity check"
        else:
            assert np.array_equal(d[:need], np.concatenate(want))


def test_compact_max_tables_exceeded_writes_nothing(codec):
    """More output tables than max_tables: SSTC_E_CAPACITY and not one byte of
    the output buffer written.  The table / block counts stay on the device
    (the layout runs on host-side bounds clamped to max_tables), so every
    layout, encode, meta and footer kernel must stand down on its own."""
    import ctypes
    import torch
    from sstcodec._lib import CompactParams, CompactResult
    g = load_golden("compact_small_base1.npz")
    ins = [g[f"in{i}"] for i in range(4)]
    src = torch.from_numpy(np.concatenate(ins)).to(codec.device)
    idx = codec.open_tables(src, [f.size for f in ins], strict=True)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    # a 4 KiB table limit splits the ~50 KB of surviving keys + values into many tables
    prm = CompactParams(4096, 4 << 10, 1, 0)
    need = int(src.numel()) * 2
    for max_tables, rc_want in ((0, -5), (3, -5), (4096, 0)):
        toff = torch.full((max_tables + 1,), -7, dtype=torch.int64, device=codec.device)
        tlen = torch.full((max(max_tables, 1),), -7, dtype=torch.int64, device=codec.device)
        dst = torch.full((need,), 0xA5, dtype=torch.uint8, device=codec.device)
        res = CompactResult()
        codec._stream()
        rc = codec.lib.sstc_compact(codec.h, P(src), P(idx["blk_off"]), P(idx["blk_len"]), int(idx["blk_off"].numel()),
                                    idx["table_first_block"].ctypes.data_as(ctypes.c_void_p), len(ins),
                                    ctypes.byref(prm), P(dst), need, P(toff), P(tlen), max_tables, ctypes.byref(res))
        assert rc == rc_want
        if rc:
            assert res.tables_out > max_tables or max_tables == 0
            assert (dst.cpu().numpy() == 0xA5).all(), "a writer ran although the tables exceed max_tables"
            if max_tables == 0:  # not even the table arrays
                assert int(toff[0]) == -7 and int(tlen[0]) == -7
        else:
            assert res.tables_out > 3


@pytest.mark.parametrize("bad", ["unsorted", "corrupt"])
def test_compact_rejected_job_writes_nothing(codec, oracle, bad):
    """The host reads the decode / sortedness verdicts only after the last
    kernel (the whole job is enqueued after the first fetch): a rejected job's
    filter reports no survivor, so the split finds no table and not one byte
    of the output buffer is written."""
    import ctypes
    import torch
    from sstcodec._lib import CompactParams, CompactResult
    sets = W.compaction_inputs(3, 20_000, 50_000, seed=9, vmax=64, p_delete=0.1)
    if bad == "unsorted":
        sets[1] = {key: v[::-1].copy() for key, v in sets[1].items()}  # keys descending
    block = 4096
    ins = [oracle.table_build(r, block) for r in sets]
    if bad == "corrupt":
        ins[2] = ins[2].copy()
        ins[2][1:5] = np.frombuffer(np.uint32(0xFFFF0000).tobytes(), np.uint8)  # entry 0 of block 0
    src = torch.from_numpy(np.concatenate(ins)).to(codec.device)
    idx = codec.open_tables(src, [f.size for f in ins], strict=True)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    need = int(src.numel()) * 2
    dst = torch.full((need,), 0xA5, dtype=torch.uint8, device=codec.device)
    toff = torch.zeros(4097, dtype=torch.int64, device=codec.device)
    tlen = torch.zeros(4096, dtype=torch.int64, device=codec.device)
    res = CompactResult()
    codec._stream()
    rc = codec.lib.sstc_compact(codec.h, P(src), P(idx["blk_off"]), P(idx["blk_len"]), int(idx["blk_off"].numel()),
                                idx["table_first_block"].ctypes.data_as(ctypes.c_void_p), len(ins),
                                ctypes.byref(CompactParams(4096, 32 << 20, 1, 0)), P(dst), need, P(toff), P(tlen),
                                4096, ctypes.byref(res))
    assert rc == -1  # SSTC_E_INVALID_ARG
    msg = codec.lib.sstc_last_error_string().decode()
    assert {"unsorted": "not sorted", "corrupt": "decode"}[bad] in msg
    assert (dst.cpu().numpy() == 0xA5).all(), "a writer ran for a rejected job"


def test_compact_all_deletes_base_level(codec, oracle):
    """Every input record a DELETE at the base level: ShouldKeepEntry drops
    them all but the first merged record (compact.cc:324-363 keeps the first
    record unconditionally), so the job emits one table of one entry."""
    sets = W.compaction_inputs(3, 2000, 5000, seed=3, vmax=64, p_delete=1.0)
    ins = [oracle.table_build(r, 4096) for r in sets]
    want, kept = oracle.compact(ins, 4096, 1 << 20, 1)
    outs, res = codec.compact(ins, 4096, 1 << 20, 1)
    assert res.records_kept == kept == 1 and len(outs) == len(want) == 1
    assert np.array_equal(outs[0], want[0])


def test_compact_long_keys_many_windows(codec, oracle):
    """Keys longer than the 16 B sort prefix, all sharing it (every merge
    comparison falls back to the source bytes), over 10 inputs (two merge
    passes, many merge windows and filter tiles), overlapping keys across
    inputs (drops) and one input duplicated (equal (key, txn) runs that the
    filter walks back through, across tile boundaries)."""
    rng = np.random.default_rng(5)
    sets = []
    txn = 1
    for t in range(10):
        n = 3000
        idx = np.sort(rng.choice(9000, n, replace=False))
        keys = [b"SHARED-PREFIX-16" + b"%08d" % i + (b"x" * int(i % 7)) for i in idx]  # 24..30 B
        vals = [bytes(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8)) for _ in range(n)]
        rec = {"type": (rng.random(n) < 0.1).astype(np.uint8),
               "key_len": np.array([len(k) for k in keys], np.uint32),
               "val_len": np.array([len(v) for v in vals], np.uint32),
               "txn": np.arange(txn, txn + n, dtype=np.uint64)[rng.permutation(n)],
               "key_off": np.cumsum([0] + [len(k) for k in keys[:-1]]).astype(np.uint64),
               "val_off": np.cumsum([0] + [len(v) for v in vals[:-1]]).astype(np.uint64),
               "key_src": np.frombuffer(b"".join(keys), np.uint8).copy(),
               "val_src": np.frombuffer(b"".join(vals) + b"\0", np.uint8).copy()}
        rec["val_len"][rec["type"] == 1] = 0xFFFFFFFF  # DELETE: no value fields
        txn += n
        sets.append(rec)
    sets[4] = {key: v.copy() for key, v in sets[3].items()}
    ins = [oracle.table_build(r, 4096) for r in sets]
    for base in (1, 0):
        want, kept = oracle.compact(ins, 4096, 150_000, base)
        outs, res = codec.compact(ins, 4096, 150_000, base)
        assert res.records_kept == kept
        assert len(outs) == len(want)
        for o, w in zip(outs, want):
            assert np.array_equal(o, w)


@pytest.mark.parametrize("fault", [1, 2, 3])
@pytest.mark.parametrize("case", ["mixed", "zipf"])
def test_compact_guard_rejects_corrupted_filter_output(codec, oracle, fault, case):
    """Downstream of the keep / drop filter, the encode, meta and footer
    kernels index with device-produced offsets (survivor key offsets, entry
    prefix sums).  With the filter output deliberately corrupted on the device
    (test hook sstc__ctx_set_fault: 1 = survivor key offsets 0xFF.., 2 = entry
    prefix sums garbage, 3 = the guard bit a decoupled look-back sets when it
    gives up waiting for a predecessor workgroup, kGuardLookback), the job's
    consistency guard must reject it (SSTC_E_INTERNAL) without an out-of-range
    access, and the context must stay usable.  'zipf' has blocks past the
    encode's LDS slot (the large-block path)."""
    import sstcodec
    if case == "zipf":
        sets = W.compaction_inputs(4, 600, 1200, seed=5, vmax=65536, vmin=8, zipf=1.1, p_delete=0.1)
    else:
        sets = W.compaction_inputs(4, 3000, 8000, seed=9, vmax=300, p_delete=0.1)
    ins = [oracle.table_build(r, 4096) for r in sets]
    want, _ = oracle.compact(ins, 4096, 4 << 20, 1)
    assert codec.lib.sstc__ctx_set_fault(codec.h, fault) == 0
    try:
        with pytest.raises(sstcodec.SstcError, match=r"\(-6\).*consistency" + (".*look-back" if fault == 3 else "")):
            codec.compact(ins, 4096, 4 << 20, 1)
    finally:
        codec.lib.sstc__ctx_set_fault(codec.h, 0)
    outs, _ = codec.compact(ins, 4096, 4 << 20, 1)
    assert len(outs) == len(want) and all(np.array_equal(o, w) for o, w in zip(outs, want))


@pytest.mark.timeout(120)
def test_compact_long_equal_runs(codec, oracle):
    """Runs of identical (key, txn) records far longer than the inputs count
    (ShouldKeepEntry keeps them all: last_txn == txn, compact.cc:357-362): the
    keep test finds a record's group head by galloping, O(log run) per record
    (a walk back over the run was O(run^2) in total); the tie check walks the
    run once.  With different values per input the job is refused
    (SSTC_E_TIE_ORDER: the reference's heap would order them by history)."""
    from sstcodec._lib import SSTC_E_TIE_ORDER, SstcError
    n = 60_000
    for same in (True, False):
        sets = []
        for t in range(3):
            # identical records (any heap order gives the same bytes), or
            # values that differ (SSTC_E_TIE_ORDER: the run spans inputs)
            rec = W.uniform_records(n, key_index=np.zeros(n, np.uint64), seed=1 if same else t + 1, value_len=20)
            rec["txn"][:] = 77  # one key, one txn, every record
            if same:
                rec["val_off"][:] = 0  # every record the same value: all copies alike
            sets.append(rec)
        extra = W.uniform_records(1000, key_index=np.arange(1, 1001, dtype=np.uint64), seed=9, value_len=20,
                                  txn_start=10)
        sets.append(extra)
        ins = [oracle.table_build(r, 4096) for r in sets]
        if not same:
            with pytest.raises(SstcError) as e:
                codec.compact(ins, 4096, 1 << 20, 1)
            assert e.value.code == SSTC_E_TIE_ORDER
            continue
        want, kept = oracle.compact(ins, 4096, 1 << 20, 1)
        outs, res = codec.compact(ins, 4096, 1 << 20, 1)
        assert res.records_kept == kept == 3 * n + 1000
        assert len(outs) == len(want) and all(np.array_equal(o, w) for o, w in zip(outs, want))


def _seg_stats(codec):
    import ctypes
    mode, redos = ctypes.c_uint32(), ctypes.c_uint64()
    assert codec.lib.sstc__ctx_seg_stats(codec.h, ctypes.byref(mode), ctypes.byref(redos)) == 0
    return mode.value, redos.value


def test_block_split_plan_follows_the_workload(oracle):
    """the block split's launch plan per context.  A job whose
    equal-size chain held makes the next job enqueue the chain alone (none of
    the general walk's launches); when that next job's records do not fit the
    chain (Zipf sizes) its writers stand down, the tail runs again with the
    general walk, and the outputs are still the oracle's; jobs after a failed
    chain take the walk alone, retrying both every kSegProbe jobs."""
    import sstcodec
    codec = sstcodec.Codec(0)  # a fresh context: plan "both"
    try:
        uni = [oracle.table_build(r, 4096) for r in W.config_inputs(3, ssts=4, keys=20_000)]
        zipf = [oracle.table_build(r, 4096) for r in
                W.compaction_inputs(4, 600, 1200, seed=5, vmin=8, vmax=65536, zipf=1.1, p_delete=0.1)]
        want_u, _ = oracle.compact(uni, 4096, 1 << 20, 1)
        want_z, _ = oracle.compact(zipf, 4096, 1 << 20, 1)
        plans = []
        for ins, want in [(uni, want_u), (uni, want_u), (zipf, want_z), (zipf, want_z), (uni, want_u)] + \
                [(uni, want_u)] * 8:
            outs, _ = codec.compact(ins, 4096, 1 << 20, 1)
            assert len(outs) == len(want) and all(np.array_equal(o, w) for o, w in zip(outs, want))
            plans.append(_seg_stats(codec))
        assert plans[0] == (1, 0) and plans[1] == (1, 0)  # the chain held: alone from then on
        assert plans[2] == (2, 1)  # chain alone failed on Zipf sizes: the tail ran twice, walk alone next
        assert plans[3] == (2, 1) and plans[4] == (2, 1)  # walk alone (a uniform job too, until the probe)
        assert (1, 1) in plans[5:]  # the probe ran both paths, the chain held again
    finally:
        codec.close()


def _table_blocks_vs_segment(oracle, tables, T):
    """Every output table's block split (record counts per block, decoded
    back) equals oracle.segment over that table's own records: the split is
    clamped at the table ends."""
    for t, img in enumerate(tables):
        idx = oracle.table_index(img)
        kl, vl, counts = [], [], []
        for o, n in zip(idx["blk_off"], idx["blk_len"]):
            st, r = oracle.decode_block(img[int(o):int(o + n)])
            assert st == 0
            kl.append(r["key_len"])
            vl.append(r["val_len"])
            counts.append(len(r["key_len"]))
        kl, vl = np.concatenate(kl), np.concatenate(vl)
        z = np.zeros(len(kl), np.uint64)
        rec = {"type": np.zeros(len(kl), np.uint8), "key_len": kl, "val_len": vl, "txn": z, "key_off": z,
               "val_off": z, "key_src": np.zeros(1, np.uint8), "val_src": np.zeros(1, np.uint8)}
        want = oracle.segment(rec, T)
        got = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
        assert np.array_equal(got, want), t


@pytest.mark.parametrize("case", ["ends_hold", "ends_one_fails", "over_1024_tables"])
def test_block_split_with_table_ends(oracle, case):
    """the block split's arithmetic chain with table ends (the
    compaction's multi-table split, seg_arith_kernel over ends = the table
    starts).  ends_hold: equal entries in ~30 output tables, every table's
    chain holds (the next job's plan: the chain alone); ends_one_fails: one
    record 3000 B heavier in one table, so that table's chain fails and the
    others would hold (the whole verdict falls back to the general walk, a
    note); over_1024_tables: more output tables than the chain takes (kArMax
    = 1024: the general walk).  Outputs bit-exact against the oracle and each
    table's blocks against oracle.segment."""
    import sstcodec
    sets = W.config_inputs(3, ssts=4, keys=5000)
    T, limit = 4096, 64 << 10
    if case == "ends_one_fails":
        r = dict(sets[2])
        j = 2500
        extra = W.random_bytes(77, 3100)
        r["val_off"] = r["val_off"].copy()
        r["val_len"] = r["val_len"].copy()
        r["val_off"][j] = r["val_src"].size
        r["val_len"][j] = 3100
        r["val_src"] = np.concatenate([r["val_src"], extra])
        sets[2] = r
    elif case == "over_1024_tables":
        T, limit = 512, 2048
    ins = [oracle.table_build(r, 4096) for r in sets]
    want, _ = oracle.compact(ins, T, limit, 1)
    if case == "over_1024_tables":
        assert len(want) > 1024
    else:
        assert 10 < len(want) <= 1024
    codec = sstcodec.Codec(0)  # a fresh context: plan "both"
    try:
        outs, _ = codec.compact(ins, T, limit, 1)
        assert len(outs) == len(want) and all(np.array_equal(o, w) for o, w in zip(outs, want))
        mode, redos = _seg_stats(codec)
        assert redos == 0
        assert mode == (1 if case == "ends_hold" else 2), mode  # the chain held / failed
    finally:
        codec.close()
    _table_blocks_vs_segment(oracle, want, T)
